#!/bin/bash
# One GPU session: parity tests, the HBM-traffic PMC passes of C4 (summarised
# into gpurun_out/pmc_traffic_TAG.json), the default bench (C4 + CPU
# baseline) reading that summary, rocprofv3 kernel statistics of the same
# command and the tracer timing (the counter calibration: tools/pmc_calib.sh).  Each step
# has its own time limit; the first failure ends it.
#   tools/gpu_full.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-run}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps_$T.log; }
step pytest && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 \
 && step pmc && "$R/tools/pmc_traffic.sh" C4 \
 && step pmcsum && python3 tools/pmc_summary.py C4 gpurun_out gpurun_out/pmc_traffic_$T.json > /dev/null \
 && step bench && timeout -k 10 600 python bench.py --pmc-json gpurun_out/pmc_traffic_$T.json > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err \
 && step rocprof && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$T" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_$T.log" 2>&1) \
 \
 && step tracer && timeout -k 10 120 python tools/tracer_bench.py > gpurun_out/tracer_$T.log 2>&1 \
 && step done
echo "exit=$?"
