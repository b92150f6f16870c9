# Round-4 session l: initial-cluster parts for short jobs, part size for short jobs.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "refine" > gpurun_out/r4l_parity.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4l_c4w8_b2.log 2>&1 && \
ALVRL_PART_BLK_SHORT=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4l_c4w8_b1.log 2>&1 && \
ALVRL_PART_BLK_SHORT=4 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4l_c4w8_b4.log 2>&1 && \
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4l_c4w8_pop.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4l_c5.log 2>&1
