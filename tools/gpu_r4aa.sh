# Round-4 session aa: weighted samples with 8 blocks of weights in flight.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/r4aa_parity.log 2>&1 || exit 1
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4aa_c5_b4.log 2>&1 || exit 1
ALVRL_PART_BLK=2 ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4aa_c5_b2.log 2>&1 || exit 1
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4aa_w8.log 2>&1 || exit 1
for v in cur r4start cur r4start; do
  if [ $v = cur ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
  ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4aa_c4_$v.json 2>/dev/null || exit 1
  python -c "
import json
b=json.loads(open('gpurun_out/r4aa_c4_$v.json').read().strip().splitlines()[-1])
print('$v', 'C4 refine', round(b['breakdown']['refine_kernel_ms'],2), 'value', round(b['value']/1e9,3))" >> gpurun_out/r4aa_summary.txt
done
