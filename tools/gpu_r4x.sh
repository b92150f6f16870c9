# Round-4 session x: the leader takes all column weights when it divides them,
# one-block parts for the initial clusters' variances; tall-job part size.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k refine > gpurun_out/r4x_parity.log 2>&1 || exit 1
ALVRL_POP_TRACE=1 ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4x_c5_b4.log 2>&1 || exit 1
ALVRL_PART_BLK=2 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4x_c5_b2.log 2>&1 || exit 1
ALVRL_PART_BLK=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4x_c5_b1.log 2>&1 || exit 1
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4x_w8.log 2>&1
