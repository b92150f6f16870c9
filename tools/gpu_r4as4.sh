#!/bin/bash
# Round-4 session as4: J / Common through the constant address space (scalar loads) vs HEAD
mkdir -p gpurun_out
H=mitsuba-alvrl_amd/variants/libalvrl_head.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/as4_parity.log 2>&1 && \
for rep in 1 2; do
  echo "== rep $rep $(date +%T)" && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/as4_c4_new_$rep.json 2> gpurun_out/as4_c4_new_$rep.err && \
  ALVRL_LIB=$H ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/as4_c4_head_$rep.json 2> gpurun_out/as4_c4_head_$rep.err && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/as4_w8_new_$rep.log 2>&1 && \
  ALVRL_LIB=$H ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/as4_w8_head_$rep.log 2>&1 || exit 1
done
echo "== done $(date +%T)"
