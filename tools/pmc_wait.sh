#!/bin/bash
# Where k_refine's waves spend their cycles (one rocprofv3 --pmc pass, --kernel-trace only;
# 8 SQ + 1 GRBM counters): wave cycles, waiting on anything / on instruction dependencies,
# issuing any / VALU / LDS / scalar-memory / vector-memory instructions.   tools/pmc_wait.sh C4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cfg=${1:-C4}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/pmc_${cfg}_WAIT" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 1 --warmup 0 --no-cpu-baseline \
  > "$R/gpurun_out/pmc_${cfg}_WAIT.log" 2>&1
