#!/bin/bash
# One measurement session on the current tree (run through gpurun from the
# repository root).  Usage: tools/gpu_session.sh TAG a|b
#   a  the whole GPU suite and smoke()
#   b  HBM traffic (FETCH / WRITE PMC passes) and VALU counters of C4 and C2,
#      the default bench line (C4, CPU baseline, records mode, the oracle's own
#      pipeline) reading them, rocprofv3 kernel statistics of the same
#      command, C2 and C3 bench lines
# Each step has its own time limit; the first failure ends the session.
# Results land in gpurun_out/ (copy what is judged to profiles/<round>/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> "gpurun_out/steps_$tag.log"; }
if [ "$2" = a ]; then
  step suite && timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
      > "gpurun_out/pytest_$tag.log" 2>&1 \
  && step smoke && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$tag.log" 2>&1 \
  && step done
else
  step pmc && "$R/tools/pmc_traffic.sh" C4 \
  && step pmcsum && python3 tools/pmc_summary.py C4 gpurun_out "gpurun_out/pmc_traffic_$tag.json" > /dev/null \
  && step valu4 && "$R/tools/pmc_valu.sh" C4 \
  && python3 tools/pmc_valu.py C4 gpurun_out gpurun_out/pmc_valu_C4.json tools/pairs_C4.json > /dev/null \
  && step valu2 && "$R/tools/pmc_valu.sh" C2 \
  && python3 tools/pmc_valu.py C2 gpurun_out gpurun_out/pmc_valu_C2.json tools/pairs_C2.json > /dev/null \
  && step bench && timeout -k 10 700 python bench.py --steps 10 --warmup 3 --pmc-json "gpurun_out/pmc_traffic_$tag.json" \
      --valu-json "gpurun_out/pmc_valu_{cfg}.json" > "gpurun_out/bench_$tag.json" 2> "gpurun_out/bench_$tag.err" \
  && step rocprof && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$tag" -o run \
      --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_$tag.log" 2>&1) \
  && step c2 && timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --valu-json "gpurun_out/pmc_valu_{cfg}.json" \
      > "gpurun_out/bench_c2_$tag.json" 2> "gpurun_out/bench_c2_$tag.err" \
  && step c3 && timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > "gpurun_out/bench_c3_$tag.json" \
      2> "gpurun_out/bench_c3_$tag.err" \
  && step done
fi
rc=$?
echo "exit=$rc"
exit $rc
