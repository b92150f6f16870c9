# Round-4 session o: render gathers with the two samples side by side (packed
# FP32) against the one-sample code, and at 4 waves per SIMD; gather parity.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r4o_parity.log 2>&1 && \
for v in scalar packed minb4 scalar packed minb4; do
  if [ $v = packed ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
  ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4o_c2_$v.json 2>/dev/null || exit 1
  ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4o_c4_$v.json 2>/dev/null || exit 1
  python -c "
import json
a=json.loads(open('gpurun_out/r4o_c2_$v.json').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/r4o_c4_$v.json').read().strip().splitlines()[-1])
print('$v', 'C2', round(a['value']/1e10,3), 'e10', round(a['breakdown']['render_kernel_ms'],2), 'ms | C4 render', round(b['breakdown']['render_kernel_ms'],2), 'rbuild', round(b['breakdown']['rbuild_ms'],2))" >> gpurun_out/r4o_summary.txt
done
