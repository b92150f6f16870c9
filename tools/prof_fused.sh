#!/bin/bash
# Developer profile of the refinement (ALVRL_REFINE_PROFILE=1 phase cycles
# and split-size histogram, ALVRL_REFINE_TEAM_STATS=1 team counters), C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
P="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-unconditional --no-records-mode"
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 $P > gpurun_out/pf_cur.json 2> gpurun_out/pf_cur.err || exit 1
