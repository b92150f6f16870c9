#!/bin/bash
# GPU-box validation run: parity tests, benches, rocprofv3 kernel trace.
# Every GPU step has its own time limit; steps are chained so the first
# failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step pytest && timeout -k 10 600 python -m pytest tests -m gpu -q -s > gpurun_out/pytest_gpu.log 2>&1 \
 && step bench_c2 && timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err \
 && step bench_c1 && timeout -k 10 300 python bench.py --config C1 --steps 3 --warmup 1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err \
 && step rocprof_c2 && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --config C2 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_c2.log" 2>&1) \
 && step done
echo "exit=$?"
