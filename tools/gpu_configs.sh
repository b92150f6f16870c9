#!/bin/bash
# The other BASELINE configurations on the current tree: C2 (brute force,
# 10k VRLs) and C3 (fixed-depth LightSlice), plus C2's rocprofv3 kernel
# statistics.  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-cfg}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps_$T.log; }
step c2 && timeout -k 10 400 python bench.py --config C2 > gpurun_out/bench_c2_$T.json 2> gpurun_out/bench_c2_$T.err \
 && step c3 && timeout -k 10 400 python bench.py --config C3 > gpurun_out/bench_c3_$T.json 2> gpurun_out/bench_c3_$T.err \
 && step rocprof_c2 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c2_$T" -o run --output-format csv -- python3 "$R/bench.py" --config C2 --no-cpu-baseline > "$R/gpurun_out/prof_c2_$T.log" 2>&1) \
 && step done
echo "exit=$?"
