#!/bin/bash
# Refinement team-mode A/B: the GPU parity suite with teams forced on, then
# the bench without teams (ALVRL_REFINE_TEAM=1), with teams of 2, and two
# speculation thresholds.  Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-ab}
CFG=${2:-C4}
cd "$R" && mkdir -p gpurun_out
export ALVRL_REFINE_SPIN_MS=5000 ALVRL_REFINE_TEAM_STATS=1
b() { timeout -k 10 240 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline; }
ALVRL_REFINE_TEAM=8 timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$T.log 2>&1 \
 && ALVRL_REFINE_TEAM=1 b > gpurun_out/${T}_solo.json 2> gpurun_out/${T}_solo.err \
 && ALVRL_REFINE_TEAM=2 b > gpurun_out/${T}_team.json 2> gpurun_out/${T}_team.err \
 && ALVRL_REFINE_TEAM=2 ALVRL_SPEC_MIN=16 b > gpurun_out/${T}_min16.json 2> gpurun_out/${T}_min16.err \
 && ALVRL_REFINE_TEAM=2 ALVRL_SPEC_MIN=512 b > gpurun_out/${T}_min512.json 2> gpurun_out/${T}_min512.err
echo "exit=$?"
