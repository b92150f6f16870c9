#!/bin/bash
# Round-6 session: the strict-build tests (exhaustive fast-math checks incl. sqrt / rcp) and the R build timing
set -o pipefail
T=${1:-r6l}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_strict.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_strict_$T.log 2>&1 &&
timeout -k 10 120 python3 -u tools/rbuild_only.py --mode strict > gpurun_out/rbonly_$T.log 2>&1
