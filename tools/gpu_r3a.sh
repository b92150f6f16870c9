#!/bin/bash
# round 3: the new parity tests, then the C5 rank-0 share timing
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_refine_bit_exact_c5_rows tests/test_gpu_parity.py::test_refine_depth_correction \
  tests/test_gpu_pipeline.py::test_pipeline_variants tests/test_gpu_pipeline.py::test_refine_c4_scale \
  > gpurun_out/r3a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/c5_share.py --json gpurun_out/c5_share_a.json > gpurun_out/r3a_c5.log 2>&1
rc2=$?
echo "c5 rc=$rc2"
tail -5 gpurun_out/r3a_c5.log
exit $rc2
