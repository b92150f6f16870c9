#!/bin/bash
# C4 refinement time per environment setting, each run twice, interleaved
# with the defaults:  tools/env_sweep2.sh "A=1 B=2" "A=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
B="python bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline --no-unconditional --no-records-mode"
run() {   # tag, settings
  env $2 timeout -k 10 200 $B > gpurun_out/sw2_$1.json 2> /dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sw2_$1.json').read().strip().splitlines()[-1]);print('[$2]', round(d['breakdown']['refine_kernel_ms'],2), round(d['ms_per_step'],1))"
}
for rep in ${SWEEP_REPS:-1 2}; do
  run base_$rep "ALVRL_DUMMY=1"
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    run s${i}_$rep "$cfg"
  done
done
