#!/bin/bash
# Round-6 session: C4's slice-sharded shares at N = 2, 4, 8 on one GPU, every rank in turn (LPT
# assignment, strict R build, steady-state second pass), with the tile render checked against N = 1
set -o pipefail
T=${1:-r6n}
mkdir -p gpurun_out
for W in 8 4 2; do
  timeout -k 10 300 python3 -u tools/c5_share.py --full --res 1024 --vrls 100000 --world $W --props "targetNumSlices=100;localUndersampling=-1" \
      --json gpurun_out/c4_w${W}_$T.json > gpurun_out/c4_w${W}_$T.log 2>&1 || exit $?
done
