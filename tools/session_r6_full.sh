#!/bin/bash
# Round-6 session: the GPU suite, smoke and a default bench on the current tree
set -o pipefail
T=${1:-r6b}
mkdir -p gpurun_out
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
