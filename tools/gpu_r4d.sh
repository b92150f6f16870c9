# Round-4 session d: split parts -- refinement parity (bit-exact suites, parts
# forced on small splits), C4 bench with and without parts, C5 rank-0 share.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "refine" > gpurun_out/r4d_parity.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4d_c4_parts.json 2> gpurun_out/r4d_c4_parts.err && \
ALVRL_PART_MIN=0 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4d_c4_noparts.json 2> gpurun_out/r4d_c4_noparts.err && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u tools/c5_share.py --json gpurun_out/r4d_c5.json > gpurun_out/r4d_c5.log 2>&1
