#!/bin/bash
# engine A/B: base vs nochain at 164 and 214 rows, J=1 and 256, interleaved
cd $GRAFT_REPO_ROOT
export ALVRL_ENGINE_NOCHECK=1
for rep in 1 2; do
for rows in 164 214; do
  for v in base nochain; do
    if [ $v = base ]; then unset ALVRL_LIB; else export ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_nochain.so; fi
    echo "== $v rows=$rows rep=$rep"
    timeout -k 10 120 python -u tools/refine_engine_bench.py --rows $rows --vrls 100000 --jobs 1 256 --reps 3 2>&1 | grep -v amdgpu | tail -1 || exit 1
  done
done
done
