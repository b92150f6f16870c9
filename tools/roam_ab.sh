#!/bin/bash
# Parity suite, then C4 with and without roaming (ALVRL_REFINE_ROAM=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-ra}
CFG=${2:-C4}
cd "$R" && mkdir -p gpurun_out
export ALVRL_REFINE_SPIN_MS=5000 ALVRL_REFINE_TEAM_STATS=1
b() { timeout -k 10 240 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$T.log 2>&1 \
 && b > gpurun_out/${T}_roam.json 2> gpurun_out/${T}_roam.err \
 && ALVRL_REFINE_ROAM=0 b > gpurun_out/${T}_noroam.json 2> gpurun_out/${T}_noroam.err
echo "exit=$?"
