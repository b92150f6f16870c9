#!/bin/bash
# engine A/B of refine.hip scheduler strategies (tools/build_variant.sh
# s_<strategy> -mllvm -amdgpu-sched-strategy=<strategy>): one 100k-column
# split at 164 and 214 rows, J = 1 and 256, interleaved, results checked
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for rows in 164 214; do
  for v in base s_max-ilp s_memclause; do
    if [ $v = base ]; then unset ALVRL_LIB; else export ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
    echo "== $v rows=$rows rep=$rep"
    timeout -k 10 120 python -u tools/refine_engine_bench.py --rows $rows --vrls 100000 --jobs 1 256 --reps 3 2>&1 | grep -v amdgpu | tail -1 || exit 1
  done
done
done
