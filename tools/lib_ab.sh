#!/bin/bash
# A/B of library builds under variants/<name>/libalvrl.so on the C4 bench,
# interleaved, each run with its own time limit; prints refine kernel ms.
#   tools/lib_ab.sh TAG name1 name2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-ab}; shift
cd "$R" && mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    ALVRL_LIB="$R/variants/$v/libalvrl.so" timeout -k 10 200 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${v}_$rep.json 2> gpurun_out/${T}_${v}_$rep.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/${T}_${v}_$rep.json'));b=d['breakdown'];print('$v', '%.3e' % d['value'], 'refine %.1f' % b['refine_kernel_ms'], 'clusters', b['clusters_total'])" || exit $?
  done
done
echo "exit=0"
