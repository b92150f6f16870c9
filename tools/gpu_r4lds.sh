#!/bin/bash
# Round-4 session lds: Prof and the part view in LDS, vs the as4 commit and the round-4 tree before it
mkdir -p gpurun_out
H=mitsuba-alvrl_amd/variants/libalvrl_head.so
A=mitsuba-alvrl_amd/variants/libalvrl_as4.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/lds_pytest.log 2>&1 && \
for rep in 1 2; do
  echo "== rep $rep" && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/lds_c4_new_$rep.json 2> gpurun_out/lds_c4_new_$rep.err && \
  ALVRL_LIB=$A ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/lds_c4_as4_$rep.json 2> gpurun_out/lds_c4_as4_$rep.err && \
  ALVRL_LIB=$H ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/lds_c4_head_$rep.json 2> gpurun_out/lds_c4_head_$rep.err && \
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/lds_w8_new_$rep.log 2>&1 && \
  ALVRL_LIB=$A ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/lds_w8_as4_$rep.log 2>&1 || exit 1
done
echo "== done"
