#!/bin/bash
# Round-6 session: the GPU suite (plugin run and C5 first), smoke and a default bench on the current tree
set -o pipefail
T=${1:-r6b}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_plugin_run.py tests/test_gpu_scale.py -x -q -s --timeout 600 --timeout-method thread > gpurun_out/pytest_first_$T.log 2>&1 &&
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_scale.py::test_c5_end_to_end > gpurun_out/pytest_$T.log 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
