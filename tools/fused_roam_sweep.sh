#!/bin/bash
# Fused render at C4 against the roamers' idle bound (ALVRL_ROAM_IDLE_US),
# then repeated runs of the chosen bound to look for outliers.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-frs}
cd "$R" && mkdir -p gpurun_out
run() {
  local name=$1; shift
  echo "== $(date +%T) $name" >> gpurun_out/steps_$T.log
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/${T}_$name.json'));b=d['breakdown']
print('$name', round(d['value']/1e9,4), round(d['ms_per_step'],1), 'render %.2f refine %.2f' % (b['render_kernel_ms'], b['refine_kernel_ms']))" >> gpurun_out/$T.txt
}
for us in 1000 5000 20000 100000 60000000; do run idle$us ALVRL_FUSED_RENDER=1 ALVRL_ROAM_IDLE_US=$us; done
run plain ALVRL_FUSED_RENDER=0
for i in 1 2 3 4 5 6 7 8; do run rep$i ALVRL_FUSED_RENDER=1 ALVRL_ROAM_IDLE_US=${CHOSEN:-60000000}; done
