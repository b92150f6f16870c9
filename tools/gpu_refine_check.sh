#!/bin/bash
# After a change to the refinement kernels: the bit-exact refinement tests
# and the pipeline parity tests, then a C4 bench (no CPU baseline) and the
# k_refine HBM traffic (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes).
#   tools/gpu_refine_check.sh TAG
cd "$(dirname "$0")/.."
tag=${1:-run}
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/refine_tests_$tag.log 2>&1 || { tail -5 gpurun_out/refine_tests_$tag.log; exit 1; }
tail -1 gpurun_out/refine_tests_$tag.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
python - "$tag" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
b = d["breakdown"]
print("bench", f'{d["value"]:.4g}', f'{d["ms_per_step"]:.1f} ms/step', "refine", f'{b["refine_kernel_ms"]:.1f}',
      "rbuild", f'{b["rbuild_ms"]:.1f}', "render", f'{b["render_kernel_ms"]:.1f}')
PY
bash tools/pmc_traffic.sh C4 || exit $?
python tools/pmc_summary.py C4 gpurun_out gpurun_out/pmc_traffic_$tag.json | grep -E "kernel_key|FETCH_SIZE_bytes|WRITE_SIZE_bytes|hbm_bytes"
