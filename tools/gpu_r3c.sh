#!/bin/bash
# round 3: where the C5 share's refinement time goes, and C4's rank-0 share at N = 2, 4, 8
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python tools/c5_share.py > gpurun_out/r3c_c5_stats.log 2>&1 || exit $?
ALVRL_REFINE_PROFILE=1 timeout -k 10 300 python tools/c5_share.py > gpurun_out/r3c_c5_prof.log 2>&1 || exit $?
for n in 2 4 8; do
  ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python tools/c5_share.py --res 1024 --vrls 100000 --world $n --passes 3 > gpurun_out/r3c_c4_w$n.log 2>&1 || exit $?
done
tail -n 3 gpurun_out/r3c_*.log
