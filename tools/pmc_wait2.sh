#!/bin/bash
# Where k_refine's waves wait, two rocprofv3 --pmc passes (--kernel-trace only), C4:
#   pass 1 (8 SQ): wave cycles, waiting on anything / instruction dependencies / LDS issue,
#                  issuing any / VALU / LDS
#   pass 2 (5 SQ): instructions issued by type, LDS bank-conflict cycles
#   tools/pmc_wait2.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-w2}
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-unconditional --no-records-mode"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
  -d "$R/gpurun_out/pmc_${tag}_1" -o run --output-format csv -- python3 $B > "$R/gpurun_out/pmc_${tag}_1.log" 2>&1 \
&& timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT \
  -d "$R/gpurun_out/pmc_${tag}_2" -o run --output-format csv -- python3 $B > "$R/gpurun_out/pmc_${tag}_2.log" 2>&1
