# Round-4 session g: parts for the column weights and the initial clusters'
# variances -- refinement parity first, then the C5 rank-0 share's pop trace.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "refine" > gpurun_out/r4g_parity.log 2>&1 && \
ALVRL_POP_TRACE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py > gpurun_out/r4g_c5_pop.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4g_c4.json 2> gpurun_out/r4g_c4.err
