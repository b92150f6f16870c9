#!/bin/bash
# Instruction-cache and issue counters of one C4 bench step (separate
# rocprofv3 passes, --kernel-trace only).
#   tools/pmc_icache.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-ic}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d "$R/gpurun_out/pmc_${T}_$i" -o run --output-format csv -- python3 "$R/bench.py" --config C4 --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_${T}_$i.log" 2>&1 || exit $?
done
echo "exit=0"
