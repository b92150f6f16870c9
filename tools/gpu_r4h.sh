#!/bin/bash
# Round-4 measurement session h on the tree after the constant-address-space change: the whole GPU
# suite and smoke (A), PMC traffic / VALU / bench / rocprof / C2 / C3 (B), then the rank-0-of-8
# pop trace and the C4 refinement profile
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_r4h_a.sh && bash tools/gpu_r4h_b.sh > gpurun_out/r4h_b.log 2>&1 && grep -q "exit=0" gpurun_out/r4h_b.log && \
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4h_w8_pop.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4h_w8.log 2>&1 && \
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4h_prof_c4.json 2> gpurun_out/r4h_prof_c4.err
rc=$?
echo "== r4h exit=$rc"
