#!/bin/bash
# Developer profile of the fused small-split modes (ALVRL_REFINE_PROFILE=1
# phase cycles and split-size histogram), C4, plus a bench A/B of a staging
# variant (variants/libalvrl_kb32.so: 32 loads in flight per thread).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
P="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-unconditional --no-records-mode"
for f in 1 2; do
  ALVRL_REFINE_PROFILE=1 ALVRL_SPLIT_FUSED=$f timeout -k 10 300 $P > gpurun_out/pf_f$f.json 2> gpurun_out/pf_f$f.err || exit 1
done
ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_kb32.so ALVRL_REFINE_PROFILE=1 ALVRL_SPLIT_FUSED=2 timeout -k 10 300 $P > gpurun_out/pf_kb32.json 2> gpurun_out/pf_kb32.err || exit 1
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-unconditional --no-records-mode"
for i in 1 2; do
  ALVRL_SPLIT_FUSED=1 timeout -k 10 240 $B > gpurun_out/fab_f1_$i.json 2>/dev/null || exit 1
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_kb32.so ALVRL_SPLIT_FUSED=1 timeout -k 10 240 $B > gpurun_out/fab_k1_$i.json 2>/dev/null || exit 1
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_kb32.so ALVRL_SPLIT_FUSED=2 timeout -k 10 240 $B > gpurun_out/fab_k2_$i.json 2>/dev/null || exit 1
  echo "round $i"
done
python3 - <<'PY'
import json
for n in ("f1_1", "k1_1", "k2_1", "f1_2", "k1_2", "k2_2"):
    d = json.loads(open(f"gpurun_out/fab_{n}.json").read().strip().splitlines()[-1]); b = d["breakdown"]
    print(n, round(d["ms_per_step"], 1), "refine", round(b["refine_kernel_ms"], 2))
PY
