#!/bin/bash
# One iteration on the GPU box: the GPU parity suite, then a short C4 bench.
#   tools/gpu_iter.sh TAG [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-iter}
cd "$R" && mkdir -p gpurun_out
K=${2:+-k "$2"}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > gpurun_out/pytest_$T.log 2>&1 \
 && tail -2 gpurun_out/pytest_$T.log \
 && timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err \
 && python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));b=d['breakdown'];print('C4', '%.3e' % d['value'], 'ms/step %.1f refine %.1f rbuild %.1f render %.1f' % (d['ms_per_step'], b['refine_kernel_ms'], b['rbuild_ms'], b['render_kernel_ms']))"
rc=$?
echo "exit=$rc"
exit $rc
