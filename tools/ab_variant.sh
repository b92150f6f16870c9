#!/bin/bash
# Developer A/B of a refine.hip variant (variants/libalvrl_NAME.so, tools/build_variant.sh):
# the refinement parity tests on the variant, then C4 rank 0 of 8 and the C4 refinement at
# N = 1 interleaved with this tree.  Usage: tools/ab_variant.sh NAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
N=$1
V=$PWD/mitsuba-alvrl_amd/variants
ALVRL_LIB=$V/libalvrl_$N.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_sort.py > gpurun_out/${N}_pytest.log 2>&1 || { tail -20 gpurun_out/${N}_pytest.log; exit 1; }
tail -1 gpurun_out/${N}_pytest.log
C="python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 2"
for i in 1 2; do
  ALVRL_LIB=$V/libalvrl_$N.so timeout -k 10 300 $C > gpurun_out/${N}w8_v_$i.log 2>&1 || exit 1
  timeout -k 10 300 $C > gpurun_out/${N}w8_t_$i.log 2>&1 || exit 1
  echo "$N $i: $(grep -o 'refine [0-9]* ms' gpurun_out/${N}w8_v_$i.log | tr '\n' ' ')  tree $i: $(grep -o 'refine [0-9]* ms' gpurun_out/${N}w8_t_$i.log | tr '\n' ' ')"
done
B="python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-unconditional --no-records-mode"
for i in 1 2; do
  ALVRL_LIB=$V/libalvrl_$N.so timeout -k 10 240 $B > gpurun_out/${N}b_v_$i.json 2>/dev/null || exit 1
  timeout -k 10 240 $B > gpurun_out/${N}b_t_$i.json 2>/dev/null || exit 1
done
N=$N python3 - <<'PY'
import json, os
for n in ("v_1", "t_1", "v_2", "t_2"):
    d = json.loads(open(f"gpurun_out/{os.environ['N']}b_{n}.json").read().strip().splitlines()[-1])
    print(n, round(d["ms_per_step"], 1), "refine", round(d["breakdown"]["refine_kernel_ms"], 2))
PY
