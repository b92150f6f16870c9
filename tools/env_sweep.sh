#!/bin/bash
# C4 refine time per environment setting: tools/env_sweep.sh "A=1 B=2" "A=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sweep_$i.json'));print('[$cfg]', round(d['breakdown']['refine_ms'],1), '%.3e' % d['value'])"
done
