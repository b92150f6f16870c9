#!/bin/bash
# Developer A/B of the projection part size: C4 rank 0 of 8 (tools/w8_env.sh)
# and C5 rank 0, adaptive parts (default) against 16,384-column parts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
bash tools/w8_env.sh "ALVRL_PROJ_CPP_MIN=16384" || exit 1
for i in 1 2; do
  timeout -k 10 400 python tools/c5_share.py > gpurun_out/pcpp_c5_$i.log 2>&1 || exit 1
  ALVRL_PROJ_CPP_MIN=16384 timeout -k 10 400 python tools/c5_share.py > gpurun_out/pcpp_c5old_$i.log 2>&1 || exit 1
  echo "C5 rank 0 run $i: adaptive $(grep -o 'refine [0-9]* ms' gpurun_out/pcpp_c5_$i.log | tr '\n' ' ') 16384 $(grep -o 'refine [0-9]* ms' gpurun_out/pcpp_c5old_$i.log | tr '\n' ' ')"
done
