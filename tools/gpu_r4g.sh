#!/bin/bash
# Round-4 measurement session g on the tree after the constant-address-space change: the whole GPU
# suite and smoke (A), PMC traffic / VALU / bench / rocprof / C2 / C3 (B), then the rank-0-of-8
# pop trace and the C4 refinement profile
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_r4g_a.sh && bash tools/gpu_r4g_b.sh > gpurun_out/r4g_b.log 2>&1 && grep -q "exit=0" gpurun_out/r4g_b.log && \
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4g_w8_pop.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4g_w8.log 2>&1 && \
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4g_prof_c4.json 2> gpurun_out/r4g_prof_c4.err
rc=$?
# part_min for short jobs (env knob): 2048 and 1024 columns at rank 0 of 8
[ $rc -eq 0 ] && ALVRL_PART_MIN=2048 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4g_w8_pm2048.log 2>&1 && \
ALVRL_PART_MIN=1024 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4g_w8_pm1024.log 2>&1
echo "== r4g exit=$rc $?"
