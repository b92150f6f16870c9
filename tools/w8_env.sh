#!/bin/bash
# Developer sweep at N = 8: C4's rank-0-of-8 share (tools/c5_share.py) per
# environment setting, twice each, interleaved with the defaults:
#   tools/w8_env.sh "A=1 B=2" "A=0" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
C="python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 2"
for i in 1 2; do
  k=0
  for cfg in "ALVRL_DUMMY=1" "$@"; do
    k=$((k+1))
    env $cfg timeout -k 10 300 $C > gpurun_out/w8e_${k}_$i.log 2>&1 || exit 1
    echo "[$cfg] run $i: $(grep -o 'refine [0-9]* ms' gpurun_out/w8e_${k}_$i.log | tr '\n' ' ')"
  done
done
