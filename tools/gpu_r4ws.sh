#!/bin/bash
# Round-4 session ws: weighted_sample_wave's stream by value, heap placement templates, part view
# copy; vs the lds commit; the leader's pop inlined (popinl); profiles of the new tree
mkdir -p gpurun_out
P=mitsuba-alvrl_amd/variants/libalvrl_lds.so
I=mitsuba-alvrl_amd/variants/libalvrl_popinl.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/ws_parity.log 2>&1 && \
ALVRL_LIB=$I timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "refine" > gpurun_out/ws_parity_inl.log 2>&1 && \
for rep in 1 2; do
  echo "== rep $rep" && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/ws_c4_new_$rep.json 2> gpurun_out/ws_c4_new_$rep.err && \
  ALVRL_LIB=$P ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/ws_c4_lds_$rep.json 2> gpurun_out/ws_c4_lds_$rep.err && \
  ALVRL_LIB=$I ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/ws_c4_inl_$rep.json 2> gpurun_out/ws_c4_inl_$rep.err && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/ws_w8_new_$rep.log 2>&1 && \
  ALVRL_LIB=$I ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/ws_w8_inl_$rep.log 2>&1 || exit 1
done && \
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/prof2_c4.json 2> gpurun_out/prof2_c4.err && \
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/prof2_w8_pop.log 2>&1 && \
ALVRL_LIB=$I ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/prof2_w8_pop_inl.log 2>&1
echo "== done"
