#!/bin/bash
# Fused render after the list-walk fix: the parity test with the gather after
# k_refine and beside it, the team knob test, then C4 benches with and
# without fused render and the base/cur refine builds, interleaved.
# A failure or fault ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-fc}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps_$T.log; }
step fused
ALVRL_TEST_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -v --timeout 120 --timeout-method thread -k "fused_render" > gpurun_out/fused_$T.log 2>&1
echo "fused rc=$?" >> gpurun_out/steps_$T.log
if grep -q "encountered\|Aborted\|core dumped" gpurun_out/fused_$T.log; then exit 2; fi
for rep in 1 2; do
  for v in base cur; do
    for f in 0 1; do
      step "bench $v fused=$f"
      ALVRL_LIB="$R/variants/$v/libalvrl.so" ALVRL_FUSED_RENDER=$f timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${T}_${v}_$f.json 2> gpurun_out/ab_${T}_${v}_$f.err || exit 3
      python3 -c "
import json;d=json.load(open('gpurun_out/ab_${T}_${v}_$f.json'));b=d['breakdown']
print('$v fused=$f', round(d['value']/1e9,4), round(d['ms_per_step'],1), 'refine', round(b['refine_kernel_ms'],2), 'clusters', b['clusters_total'])" >> gpurun_out/ab_$T.txt
    done
  done
done
step done
