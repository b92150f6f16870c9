# Round-4 session v: queue flags + split()'s own projections -- refinement and
# pipeline parity, C4 N = 1 against the session's start, C4 rank 0 of 8, C5 rank 0.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/r4v_parity.log 2>&1 || exit 1
for v in cur r4start cur r4start; do
  if [ $v = cur ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
  ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4v_c4_$v.json 2>/dev/null || exit 1
  python -c "
import json
b=json.loads(open('gpurun_out/r4v_c4_$v.json').read().strip().splitlines()[-1])
print('$v', 'C4 refine', round(b['breakdown']['refine_kernel_ms'],2), 'value', round(b['value']/1e9,3))" >> gpurun_out/r4v_summary.txt
done
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4v_w8.log 2>&1 && echo "w8 $(grep 'job end' gpurun_out/r4v_w8.log)" >> gpurun_out/r4v_summary.txt && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4v_c5.log 2>&1 && echo "c5 $(grep 'job end' gpurun_out/r4v_c5.log)" >> gpurun_out/r4v_summary.txt
