#!/bin/bash
# Team mode with roaming helpers: parity suite (teams + roamers on), then the
# bench solo / teams only / teams + roamers at the given config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-ab}
CFG=${2:-C4}
cd "$R" && mkdir -p gpurun_out
export ALVRL_REFINE_SPIN_MS=5000 ALVRL_REFINE_TEAM_STATS=1
b() { timeout -k 10 240 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$T.log 2>&1 \
 && ALVRL_REFINE_TEAM=1 b > gpurun_out/${T}_solo.json 2> gpurun_out/${T}_solo.err \
 && ALVRL_REFINE_ROAM=0 b > gpurun_out/${T}_team.json 2> gpurun_out/${T}_team.err \
 && b > gpurun_out/${T}_roam.json 2> gpurun_out/${T}_roam.err
echo "exit=$?"
