#!/bin/bash
# HBM traffic of every kernel of one bench step: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes (--kernel-trace only, MI355X_MICROARCH.md HBM and
# rocprofv3 sections).  Summarise with tools/pmc_summary.py.
#   tools/pmc_traffic.sh C4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cfg=${1:-C4}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$R/gpurun_out/pmc_${cfg}_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_${cfg}_$c.log" 2>&1 || exit $?
done
