# Round-4 session t: is the C4 N = 1 slowdown the part board (idle counter,
# polling) or code generation?  Same box, interleaved.
mkdir -p gpurun_out
for v in r4start tmpl tmploff qflag qflagoff r4start tmpl tmploff qflag qflagoff; do
  case $v in
    tmploff) L=mitsuba-alvrl_amd/variants/libalvrl_tmpl.so; E="ALVRL_PART_MIN=0";;
    qflagoff) L=mitsuba-alvrl_amd/variants/libalvrl_qflag.so; E="ALVRL_PART_MIN=0";;
    *) L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; E="ALVRL_DUMMY=0";;
  esac
  env $E ALVRL_LIB=$L timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4t_$v.json 2>/dev/null || exit 1
  python -c "
import json
b=json.loads(open('gpurun_out/r4t_$v.json').read().strip().splitlines()[-1])
print('$v', 'C4 refine', round(b['breakdown']['refine_kernel_ms'],2), 'value', round(b['value']/1e9,3))" >> gpurun_out/r4t_summary.txt
done
