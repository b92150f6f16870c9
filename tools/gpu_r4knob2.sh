#!/bin/bash
# Round-4 session knob2: 8192-column projection parts at N = 1 (C4) and at C5 rank 0 (env knob only)
mkdir -p gpurun_out
for rep in 1 2; do
  for k in base cpp8k; do
    case $k in base) E="";; cpp8k) E="ALVRL_PROJ_CPP=8192";; esac
    env $E timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/knob2_c4_${k}_$rep.json 2> gpurun_out/knob2_c4_${k}_$rep.err || exit 1
  done
done
for k in base cpp8k; do
  case $k in base) E="";; cpp8k) E="ALVRL_PROJ_CPP=8192";; esac
  env $E ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/knob2_c5_$k.log 2>&1 || exit 1
done
echo "== done"
