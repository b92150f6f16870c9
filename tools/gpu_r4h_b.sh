# Round-4 measurement session h, part B: HBM traffic (FETCH/WRITE PMC
# passes) and VALU counters of C4 and C2, the default bench line (C4 + CPU
# baseline) reading them, rocprofv3 kernel statistics of the same command,
# C2 and C3 bench lines.  Each step has its own time limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps_r4h.log; }
step pmc && "$R/tools/pmc_traffic.sh" C4 \
 && step pmcsum && python3 tools/pmc_summary.py C4 gpurun_out gpurun_out/pmc_traffic_r4h.json > /dev/null \
 && step valu4 && "$R/tools/pmc_valu.sh" C4 && python3 tools/pmc_valu.py C4 gpurun_out gpurun_out/pmc_valu_C4.json tools/pairs_C4.json > /dev/null \
 && step valu2 && "$R/tools/pmc_valu.sh" C2 && python3 tools/pmc_valu.py C2 gpurun_out gpurun_out/pmc_valu_C2.json tools/pairs_C2.json > /dev/null \
 && step bench && timeout -k 10 600 python bench.py --pmc-json gpurun_out/pmc_traffic_r4h.json --valu-json "gpurun_out/pmc_valu_{cfg}.json" > gpurun_out/bench_r4h.json 2> gpurun_out/bench_r4h.err \
 && step rocprof && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r4h" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_r4h.log" 2>&1) \
 && step c2 && timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --valu-json "gpurun_out/pmc_valu_{cfg}.json" > gpurun_out/bench_c2_r4h.json 2> gpurun_out/bench_c2_r4h.err \
 && step c3 && timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > gpurun_out/bench_c3_r4h.json 2> gpurun_out/bench_c3_r4h.err \
 && step done
echo "exit=$?"
