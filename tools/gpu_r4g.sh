# Round-4 session g: C5 rank-0 share pop trace of the largest slice's leader.
mkdir -p gpurun_out
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4g_c5_pop.log 2>&1
