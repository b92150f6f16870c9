#!/bin/bash
# End-of-round evidence for the current tree: GPU parity suite, the default
# bench (C4 + CPU baseline), rocprofv3 kernel statistics of the same bench
# command, smoke().  Each GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-final}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps_$T.log; }
step pytest && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 \
 && step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 \
 && step bench && timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err \
 && step rocprof && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$T" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_$T.log" 2>&1) \
 && step done
echo "exit=$?"
