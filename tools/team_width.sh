#!/bin/bash
# Speculation width / threshold sweep at a config (teams + roamers).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-w}
CFG=${2:-C4}
cd "$R" && mkdir -p gpurun_out
export ALVRL_REFINE_SPIN_MS=5000 ALVRL_REFINE_TEAM_STATS=1
b() { timeout -k 10 240 python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline; }
for cfgv in "W=4" "W=8" "W=16" "W=8 M=8" "W=8 M=32"; do
  W=$(echo $cfgv | sed -n 's/.*W=\([0-9]*\).*/\1/p'); M=$(echo $cfgv | sed -n 's/.*M=\([0-9]*\).*/\1/p'); M=${M:-16}
  ALVRL_SPEC_WIDTH=$W ALVRL_SPEC_MIN=$M b > gpurun_out/${T}_w${W}_m${M}.json 2> gpurun_out/${T}_w${W}_m${M}.err || exit $?
done
echo "exit=0"
