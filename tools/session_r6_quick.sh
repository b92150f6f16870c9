#!/bin/bash
# Round-6 session: the strict-build, area-scene and C5 GPU tests, then the R build timing
set -o pipefail
T=${1:-r6c}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_strict.py tests/test_gpu_area_scene.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 &&
timeout -k 10 120 python3 -u tools/rbuild_only.py --mode strict > gpurun_out/rbonly_$T.log 2>&1 &&
timeout -k 10 300 python3 -u tools/rbuild_bench.py --passes 3 --mode strict > gpurun_out/rbuild_$T.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py -x -q -s --timeout 500 --timeout-method thread > gpurun_out/pytest_c5_$T.log 2>&1
