#!/bin/bash
# engine A/B: base vs coefficient-read variants (nocoef, noload: timing only; wnadd: valid)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export ALVRL_ENGINE_NOCHECK=1
for rep in 1 2; do
for rows in 164 214; do
  for v in base nocoef wnadd noload; do
    if [ $v = base ]; then unset ALVRL_LIB; else export ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
    echo "== $v rows=$rows rep=$rep"
    timeout -k 10 120 python -u tools/refine_engine_bench.py --rows $rows --vrls 100000 --jobs 1 256 --reps 3 --tag $v 2>&1 | grep -v amdgpu | tail -1 || exit 1
  done
done
done
unset ALVRL_ENGINE_NOCHECK
export ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_wnadd.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "refine" 2>&1 | tail -3
