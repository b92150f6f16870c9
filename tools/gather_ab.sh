#!/bin/bash
# A/B of library builds under variants/<name>/libalvrl.so on the C4 bench
# (render gather, R build and refinement kernel times), interleaved twice.
#   tools/gather_ab.sh TAG name1 name2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-gab}; shift
cd "$R" && mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    ALVRL_LIB="$R/variants/$v/libalvrl.so" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/${T}_${v}_$rep.json'));b=d['breakdown']
print('$v', round(d['value']/1e9,4), 'render %.2f rbuild %.2f refine %.2f' % (b['render_kernel_ms'], b['rbuild_ms'], b['refine_kernel_ms']), 'clusters', b['clusters_total'])" >> gpurun_out/$T.txt || exit 1
  done
done
