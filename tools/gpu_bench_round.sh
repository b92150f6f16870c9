#!/bin/bash
# Benches + rocprofv3 kernel statistics for the round's profiles/ directory.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step bench_c2 && timeout -k 10 400 python bench.py --config C2 --steps 3 --warmup 1 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err \
 && step bench_c4 && timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err \
 && step rocprof_c4 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c4" -o run --output-format csv -- python3 "$R/bench.py" --config C4 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_c4.log" 2>&1) \
 && step rocprof_c2 && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --config C2 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_c2.log" 2>&1) \
 && step done
echo "exit=$?"
