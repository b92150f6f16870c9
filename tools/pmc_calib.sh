#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/pmc_calib.hip) and the C4 k_refine
# traffic with and without the refinement team (ALVRL_REFINE_TEAM=1: one
# workgroup per slice job, no helpers, no polling).  Separate passes per
# counter, --kernel-trace only.
#   tools/pmc_calib.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-calib}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -d "$R/gpurun_out/calib_${T}_$c" -o run --output-format csv -- "$R/tools/pmc_calib" > "$R/gpurun_out/calib_${T}_$c.log" 2>&1 || exit $?
done
[ -n "$CALIB_ONLY" ] && { echo "exit=0"; exit 0; }
for team in 8 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    ALVRL_REFINE_TEAM=$team timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$R/gpurun_out/pmcref_${T}_t${team}_$c" -o run --output-format csv -- python3 "$R/bench.py" --config C4 --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmcref_${T}_t${team}_$c.log" 2>&1 || exit $?
  done
done
echo "exit=0"
