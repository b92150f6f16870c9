# Round-4 session w: C5 rank-0 share on the final tree -- phase profile and pop trace.
mkdir -p gpurun_out
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4w_c5_prof.log 2>&1 && \
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4w_c5_pop.log 2>&1
