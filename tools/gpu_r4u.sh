# Round-4 session u: which change slowed C4 N = 1 -- part polling in the
# helper loops (nohp) or the projection refactor (oldproj)?  Same box, interleaved.
mkdir -p gpurun_out
for v in r4start qflag nohp oldproj r4start qflag nohp oldproj; do
  L=mitsuba-alvrl_amd/variants/libalvrl_$v.so
  ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4u_$v.json 2>/dev/null || exit 1
  python -c "
import json
b=json.loads(open('gpurun_out/r4u_$v.json').read().strip().splitlines()[-1])
print('$v', 'C4 refine', round(b['breakdown']['refine_kernel_ms'],2), 'value', round(b['value']/1e9,3))" >> gpurun_out/r4u_summary.txt
done
