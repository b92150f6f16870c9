#!/bin/bash
# Developer sweep of the speculation width (ALVRL_SPEC_WIDTH): C4's rank-0-of-8
# share (tools/c5_share.py) and the C4 refinement at N = 1, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
C="python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 2"
B="python bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline --no-unconditional --no-records-mode"
for i in 1 2; do
  for w in ${WIDTHS:-56 64 96 128}; do
    ALVRL_SPEC_WIDTH=$w timeout -k 10 300 $C > gpurun_out/w8w_${w}_$i.log 2>&1 || exit 1
    ALVRL_SPEC_WIDTH=$w timeout -k 10 200 $B > gpurun_out/w1w_${w}_$i.json 2>/dev/null || exit 1
    echo "width $w run $i: N=8 $(grep -o 'refine [0-9]* ms' gpurun_out/w8w_${w}_$i.log | tr '\n' ' ') N=1 $(python -c "import json;d=json.loads(open('gpurun_out/w1w_${w}_$i.json').read().strip().splitlines()[-1]);print(round(d['breakdown']['refine_kernel_ms'],2))")"
  done
done
