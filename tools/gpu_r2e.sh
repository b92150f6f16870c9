#!/bin/bash
# Round-2 re-entry check: GPU parity suite, the default bench, then the
# experimental fused render test (with the team knob sweep in the same
# process, the sequence that once faulted).  Each GPU step has its own limit;
# the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r2e}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps_$T.log; }
step pytest && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 \
 && step bench && timeout -k 10 400 python bench.py --pmc-json profiles/r02_pmc_traffic.json > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err \
 && step fused && ALVRL_TEST_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fused_render or team_mode_settings" > gpurun_out/fused_$T.log 2>&1 \
 && step done
echo "exit=$?"
