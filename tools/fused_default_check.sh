#!/bin/bash
# Fused render with the 20 ms roamer idle default: the opt-in parity tests,
# then four C4 benches in fused mode and one plain, each under its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-fdc}
cd "$R" && mkdir -p gpurun_out
echo "== $(date +%T) tests" >> gpurun_out/steps_$T.log
ALVRL_TEST_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fused_render or team_mode" > gpurun_out/tests_$T.log 2>&1 || exit 1
for i in plain 1 2 3 4; do
  f=1; [ $i = plain ] && f=0
  echo "== $(date +%T) bench $i" >> gpurun_out/steps_$T.log
  ALVRL_FUSED_RENDER=$f timeout -k 10 90 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err || exit 2
  python3 -c "
import json;d=json.load(open('gpurun_out/${T}_$i.json'));b=d['breakdown']
print('$i', round(d['value']/1e9,4), round(d['ms_per_step'],1), 'render %.2f refine %.2f' % (b['render_kernel_ms'], b['refine_kernel_ms']))" >> gpurun_out/$T.txt
done
