# Round-4 session k: C4 rank-0-of-8 share -- pop trace and phase profile.
mkdir -p gpurun_out
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4k_c4w8_pop.log 2>&1 && \
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4k_c4w8_prof.log 2>&1
