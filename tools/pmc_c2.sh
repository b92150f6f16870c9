#!/bin/bash
# rocprofv3 PMC passes for the C2 gather (each counter group in its own run,
# --kernel-trace only, as MI355X_MICROARCH.md's rocprofv3 section prescribes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cfg=${1:-C2}
cd /tmp && export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc_${cfg}_$tag" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_${cfg}_$tag.log" 2>&1 || exit $?
done
