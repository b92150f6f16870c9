# Round-4 session p: the R build with the two samples side by side (packed) at
# 3 and 2 waves per SIMD, against the one-sample code.
mkdir -p gpurun_out
for v in base rbp3 rbp2 rb2 base rbp3 rbp2 rb2; do
  if [ $v = base ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
  ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4p_c4_$v.json 2>/dev/null || exit 1
  python -c "
import json
b=json.loads(open('gpurun_out/r4p_c4_$v.json').read().strip().splitlines()[-1])
print('$v', 'C4 rbuild', round(b['breakdown']['rbuild_ms'],2), 'render', round(b['breakdown']['render_kernel_ms'],2), 'value', round(b['value']/1e9,3))" >> gpurun_out/r4p_summary.txt
done
