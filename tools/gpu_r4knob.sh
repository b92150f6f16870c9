#!/bin/bash
# Round-4 session knob: part sizes for short jobs at rank 0 of 8 and N = 1 (env knobs only)
mkdir -p gpurun_out
for rep in 1 2; do
  for k in base blk1 cpp8k blk1cpp8k; do
    case $k in
      base) E="";; blk1) E="ALVRL_PART_BLK_SHORT=1";; cpp8k) E="ALVRL_PROJ_CPP=8192";; blk1cpp8k) E="ALVRL_PART_BLK_SHORT=1 ALVRL_PROJ_CPP=8192";;
    esac
    env $E ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/knob_w8_${k}_$rep.log 2>&1 || exit 1
  done
done
for k in base blk1; do
  case $k in base) E="";; blk1) E="ALVRL_PART_BLK_SHORT=1";; esac
  env $E timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/knob_c4_$k.json 2> gpurun_out/knob_c4_$k.err || exit 1
done
echo "== done"
