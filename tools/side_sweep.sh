#!/bin/bash
# Leader side-task gate sweep on C4 (refine ms per setting).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for k in "$@"; do
  ALVRL_LEADER_SIDE=$k timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/side_$k.json 2> gpurun_out/side_$k.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/side_$k.json'));print('side_k=$k', d['breakdown']['refine_ms'], d['value'])"
done
