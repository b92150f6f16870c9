# Round-4 session j: short-job parts off in busy launches.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "refine" > gpurun_out/r4j_parity.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4j_c4.json 2> gpurun_out/r4j_c4.err && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4j_c4w8.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4j_c5.log 2>&1
