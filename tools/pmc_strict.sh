#!/bin/bash
# Counters of the strict R build (k_build_R_strict), one C4 prepass, two
# rocprofv3 --pmc passes (--kernel-trace only):
#   tools/pmc_strict.sh TAG      -> gpurun_out/pmc_strict_TAG_{1,2}/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-s}
cd /tmp && export TMPDIR=/tmp
B="$R/tools/rbuild_bench.py --passes 1 --mode strict"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU \
  -d "$R/gpurun_out/pmc_strict_${tag}_1" -o run --output-format csv -- python3 $B > "$R/gpurun_out/pmc_strict_${tag}_1.log" 2>&1 \
&& timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_IFETCH SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/pmc_strict_${tag}_2" -o run --output-format csv -- python3 $B > "$R/gpurun_out/pmc_strict_${tag}_2.log" 2>&1
# pass 3: instruction cache
[ $? -eq 0 ] && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_LDS \
  -d "$R/gpurun_out/pmc_strict_${tag}_3" -o run --output-format csv -- python3 $B > "$R/gpurun_out/pmc_strict_${tag}_3.log" 2>&1
