#!/bin/bash
# round 3: MFMA column-weight microbenchmark, VALU PMC passes (C4, C2), leader profiles of C4 at N = 1 / 8
cd "$(dirname "$0")/.."
R=$(pwd)
export PYTHONUNBUFFERED=1
timeout -k 10 120 tools/ubench_colw_mfma > gpurun_out/ubench_colw_mfma.jsonl 2>&1 || exit $?
cat gpurun_out/ubench_colw_mfma.jsonl
for cfg in C4 C2; do
  bash tools/pmc_valu.sh $cfg || exit $?
  python3 - $cfg <<'PY' || exit $?
import json, sys
cfg = sys.argv[1]
line = [l for l in open(f"gpurun_out/pmc_{cfg}_VALU.log") if l.startswith("{")][-1]
b = json.loads(line)["breakdown"]
json.dump({"render": b["render_pairs"], "rbuild": b["prepass_pairs"]}, open(f"gpurun_out/pairs_{cfg}.json", "w"))
PY
  python3 tools/pmc_valu.py $cfg gpurun_out gpurun_out/pmc_valu_$cfg.json gpurun_out/pairs_$cfg.json || exit $?
done
ALVRL_REFINE_PROFILE=1 timeout -k 10 120 python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 2 > gpurun_out/r3d_c4_w8_prof.log 2>&1 || exit $?
ALVRL_REFINE_PROFILE=1 timeout -k 10 120 python tools/c5_share.py --res 1024 --vrls 100000 --world 1 --passes 2 > gpurun_out/r3d_c4_w1_prof.log 2>&1 || exit $?
grep -E "ctrl|job end|rank 0" gpurun_out/r3d_c4_w*_prof.log
