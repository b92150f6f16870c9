# Round-4 session q: the queue flags in the leader's heap nodes (variant qflag)
# -- refinement parity -- and C4 A/B against the session's start (r4start)
# and the current tree, then the C4 rank-0-of-8 share.
mkdir -p gpurun_out
Q=mitsuba-alvrl_amd/variants/libalvrl_qflag.so
ALVRL_LIB=$Q timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k refine > gpurun_out/r4q_parity.log 2>&1 && \
ALVRL_LIB=$Q timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py -k "c4_scale or team or refine" > gpurun_out/r4q_pipeline.log 2>&1 || exit 1
for v in cur r4start qflag cur r4start qflag; do
  if [ $v = cur ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
  ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4q_c4_$v.json 2>/dev/null || exit 1
  python -c "
import json
b=json.loads(open('gpurun_out/r4q_c4_$v.json').read().strip().splitlines()[-1])
print('$v', 'C4 refine', round(b['breakdown']['refine_kernel_ms'],2), 'value', round(b['value']/1e9,3))" >> gpurun_out/r4q_summary.txt
done
for v in cur qflag cur qflag; do
  if [ $v = cur ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
  ALVRL_LIB=$L ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4q_w8_$v.log 2>&1 || exit 1
  echo "$v $(grep 'job end' gpurun_out/r4q_w8_$v.log)" >> gpurun_out/r4q_summary.txt
done
