# Round-4 session c: the C5 rank-0 share's refinement profile (per-phase
# cycles, team counters, job end times, split cost by size).
mkdir -p gpurun_out
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 400 python -u tools/c5_share.py --json gpurun_out/c5_prof.json > gpurun_out/c5_prof.log 2>&1
