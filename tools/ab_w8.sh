#!/bin/bash
# Developer A/B at N = 8: the refinement's parity tests on this tree, then C4's
# rank-0-of-8 share (tools/c5_share.py) interleaved, this tree against
# variants/libalvrl_$1.so.  Run on the GPU box (gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
V=$1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_fused_split.py > gpurun_out/ab_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/ab_pytest.log
[ $rc -eq 0 ] || exit $rc
C="python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 2"
for i in ${AB_RUNS:-1 2 3}; do
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_$V.so timeout -k 10 300 $C > gpurun_out/w8_${V}_$i.log 2>&1 || exit 1
  timeout -k 10 300 $C > gpurun_out/w8_tree_$i.log 2>&1 || exit 1
  echo "$V $i: $(grep -o 'refine [0-9]* ms' gpurun_out/w8_${V}_$i.log | tr '\n' ' ')  tree $i: $(grep -o 'refine [0-9]* ms' gpurun_out/w8_tree_$i.log | tr '\n' ' ')"
done
