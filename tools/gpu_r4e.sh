# Round-4 session e: C5 rank-0 share with split parts -- phase profile, and
# more / smaller parts.
mkdir -p gpurun_out
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4e_c5_prof.log 2>&1 && \
ALVRL_PART_BLK=2 ALVRL_PART_MB=40000 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4e_c5_blk2.log 2>&1 && \
ALVRL_PART_BLK=4 ALVRL_PART_MB=40000 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4e_c5_blk4s.log 2>&1
