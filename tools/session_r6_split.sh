#!/bin/bash
# Round-6 session: the host-gather split form (tests + records-mode timing)
set -o pipefail
T=${1:-r6d}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_ext_scene.py tests/test_gpu_area_scene.py tests/test_gpu_local_exchange.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 &&
timeout -k 10 300 python3 -u tools/records_mode_bench.py > gpurun_out/records_$T.json 2> gpurun_out/records_$T.err &&
ALVRL_HOST_SPLIT=0 timeout -k 10 300 python3 -u tools/records_mode_bench.py --blocks 32 > gpurun_out/records_nosplit_$T.json 2>> gpurun_out/records_$T.err &&
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick_$T.json 2> gpurun_out/bench_quick_$T.err
