#!/bin/bash
# Developer A/B of the fused small-split path (split_fused): the refinement's
# bit-exact parity tests, then C4 bench runs interleaved -- the previous
# library (variants/libalvrl_base5.so), this tree with ALVRL_SPLIT_FUSED=1
# (float2 staging only) and with the default (2: means-only staging too).
# Run on the GPU box (gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_strict.py > gpurun_out/fused_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/fused_pytest.log
[ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-unconditional --no-records-mode"
for i in 1 2; do
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_base5.so timeout -k 10 240 $B > gpurun_out/fab_base_$i.json 2> gpurun_out/fab_base_$i.err || exit 1
  ALVRL_SPLIT_FUSED=1 timeout -k 10 240 $B > gpurun_out/fab_off_$i.json 2> gpurun_out/fab_off_$i.err || exit 1
  ALVRL_SPLIT_FUSED=2 timeout -k 10 240 $B > gpurun_out/fab_on_$i.json 2> gpurun_out/fab_on_$i.err || exit 1
  echo "round $i done"
done
python3 - <<'PY'
import json
for n in ("base_1", "off_1", "on_1", "base_2", "off_2", "on_2"):
    d = json.loads(open(f"gpurun_out/fab_{n}.json").read().strip().splitlines()[-1]); b = d["breakdown"]
    print(n, round(d["ms_per_step"], 1), "refine", round(b["refine_kernel_ms"], 2), "rbuild", round(b["rbuild_ms"], 2),
          "render", round(b["render_kernel_ms"], 2), "frac", round(d["roofline"]["frac"], 3))
PY
