#!/bin/bash
# The full GPU suite as the driver runs it (one process, per-test time bound),
# then smoke() and a short C4 bench.  Usage: tools/gpu_suite.sh TAG
cd "$(dirname "$0")/.."
tag=${1:-run}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
python - "$tag" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
b = d["breakdown"]
print("bench", f'{d["value"]:.4g}', f'{d["ms_per_step"]:.1f} ms/step', "refine", f'{b["refine_kernel_ms"]:.1f}',
      "rbuild", f'{b["rbuild_ms"]:.1f}', "render", f'{b["render_kernel_ms"]:.1f}',
      "cpu", d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None)
PY
exit $rc
