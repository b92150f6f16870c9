#!/bin/bash
# Where the fused render's time goes at C4: plain path, k_refine in fused mode
# without the gather, fused, fused with roamers that never leave early.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-fp}
cd "$R" && mkdir -p gpurun_out
run() {
  local name=$1; shift
  echo "== $(date +%T) $name" >> gpurun_out/steps_$T.log
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/${T}_$name.json'));b=d['breakdown']
print('$name', round(d['value']/1e9,4), round(d['ms_per_step'],1), 'render %.2f refine %.2f' % (b['render_kernel_ms'], b['refine_kernel_ms']), 'fused', b.get('render_fused'))" >> gpurun_out/$T.txt
}
run plain ALVRL_FUSED_RENDER=0
run nogather ALVRL_FUSED_RENDER=1 ALVRL_FUSED_NOGATHER=1
run fused ALVRL_FUSED_RENDER=1
run fused_roam ALVRL_FUSED_RENDER=1 ALVRL_ROAM_IDLE_US=60000000
run fused_team_stats ALVRL_FUSED_RENDER=1 ALVRL_REFINE_TEAM_STATS=1
