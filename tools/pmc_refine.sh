#!/bin/bash
# rocprofv3 PMC passes for the refinement kernel (C3), each counter group in
# its own run with --kernel-trace only (MI355X_MICROARCH.md rocprofv3 rules).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/pmc_list.txt" 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc_refine_$i" -o run --output-format csv -- python3 "$R/bench.py" --config C3 --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_refine_$i.log" 2>&1 || exit $?
done
