#!/bin/bash
# Developer A/B: C4 bench runs interleaved, this tree's library against
# variants/libalvrl_$1.so (built from another tree), after the refinement's
# parity tests on this tree.  Run on the GPU box (gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=$1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_strict.py > gpurun_out/ab_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/ab_pytest.log
[ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-unconditional --no-records-mode"
for i in 1 2 3; do
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_$V.so timeout -k 10 240 $B > gpurun_out/ab_${V}_$i.json 2>/dev/null || exit 1
  timeout -k 10 240 $B > gpurun_out/ab_tree_$i.json 2>/dev/null || exit 1
  echo "round $i"
done
python3 - "$V" <<'PY'
import json, sys
V = sys.argv[1]
for i in (1, 2, 3):
    for n in (V, "tree"):
        d = json.loads(open(f"gpurun_out/ab_{n}_{i}.json").read().strip().splitlines()[-1]); b = d["breakdown"]
        print(n, i, round(d["ms_per_step"], 1), "refine", round(b["refine_kernel_ms"], 2), "rbuild", round(b["rbuild_ms"], 2),
              "render", round(b["render_kernel_ms"], 2))
PY
