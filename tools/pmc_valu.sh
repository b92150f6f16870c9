#!/bin/bash
# VALU counters of every kernel of one bench step (one rocprofv3 --pmc pass,
# --kernel-trace only; 8 SQ + 1 GRBM counters, within one pass's limits).
# Summarise with tools/pmc_valu.py.   tools/pmc_valu.sh C4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cfg=${1:-C4}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/pmc_${cfg}_VALU" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 1 --warmup 0 --no-cpu-baseline \
  > "$R/gpurun_out/pmc_${cfg}_VALU.log" 2>&1
