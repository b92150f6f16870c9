#!/bin/bash
# Round-4 session cw: column weights' loads without a branch per load (a codegen regression of the
# constant-address-space change), vs the lds commit
mkdir -p gpurun_out
P=mitsuba-alvrl_amd/variants/libalvrl_lds.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/cw_parity.log 2>&1 && \
for rep in 1 2; do
  echo "== rep $rep" && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/cw_c4_new_$rep.json 2> gpurun_out/cw_c4_new_$rep.err && \
  ALVRL_LIB=$P ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/cw_c4_lds_$rep.json 2> gpurun_out/cw_c4_lds_$rep.err && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/cw_w8_new_$rep.log 2>&1 || exit 1
done && \
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/prof3_c4.json 2> gpurun_out/prof3_c4.err && \
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/prof3_w8_pop.log 2>&1
echo "== done"
