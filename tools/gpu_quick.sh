#!/bin/bash
# Parity suite, then a solo-mode refine profile and the default C4 bench.
#   tools/gpu_quick.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-q}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 \
 && ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM=1 timeout -k 10 200 python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/hist_$T.json 2> gpurun_out/hist_$T.err \
 && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
echo "exit=$?"
