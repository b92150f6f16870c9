#!/bin/bash
# Developer check of the split sort's radix path (radix8_sort): the radix-vs-
# bitonic cluster-list test, the oracle parity tests with the radix sort on
# every split (ALVRL_SORT_RADIX_MIN=2), then C4 rank 0 of 8 and C4 N = 1
# against variants/libalvrl_head.so, and N = 1 with lower radix thresholds.
# Run on the GPU box (gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_sort.py > gpurun_out/sort_pytest1.log 2>&1 || { tail -30 gpurun_out/sort_pytest1.log; exit 1; }
tail -2 gpurun_out/sort_pytest1.log
ALVRL_SORT_RADIX_MIN=2 ALVRL_WS_WG_MIN=2 timeout -k 10 900 $P tests/test_gpu_parity.py tests/test_gpu_pipeline.py > gpurun_out/sort_pytest2.log 2>&1 || { tail -30 gpurun_out/sort_pytest2.log; exit 1; }
tail -2 gpurun_out/sort_pytest2.log
C="python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 2"
for i in 1 2; do
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_head.so timeout -k 10 300 $C > gpurun_out/sw8_head_$i.log 2>&1 || exit 1
  timeout -k 10 300 $C > gpurun_out/sw8_tree_$i.log 2>&1 || exit 1
  echo "head $i: $(grep -o 'refine [0-9]* ms' gpurun_out/sw8_head_$i.log | tr '\n' ' ')  tree $i: $(grep -o 'refine [0-9]* ms' gpurun_out/sw8_tree_$i.log | tr '\n' ' ')"
done
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-unconditional --no-records-mode"
for i in 1 2; do
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_head.so timeout -k 10 240 $B > gpurun_out/sb_head_$i.json 2> gpurun_out/sb_head_$i.err || exit 1
  timeout -k 10 240 $B > gpurun_out/sb_tree_$i.json 2> gpurun_out/sb_tree_$i.err || exit 1
  ALVRL_SORT_RADIX_MIN=4096 timeout -k 10 240 $B > gpurun_out/sb_r4k_$i.json 2> gpurun_out/sb_r4k_$i.err || exit 1
  ALVRL_SORT_RADIX_MIN=1024 timeout -k 10 240 $B > gpurun_out/sb_r1k_$i.json 2> gpurun_out/sb_r1k_$i.err || exit 1
  echo "bench round $i done"
done
python3 - <<'PY'
import json
for n in ("head_1", "tree_1", "r4k_1", "r1k_1", "head_2", "tree_2", "r4k_2", "r1k_2"):
    d = json.loads(open(f"gpurun_out/sb_{n}.json").read().strip().splitlines()[-1]); b = d["breakdown"]
    print(n, round(d["ms_per_step"], 1), "refine", round(b["refine_kernel_ms"], 2), "frac", round(d["roofline"]["frac"], 3))
PY
