# Round-4 session b: the C4 refinement's per-phase profile and team counters,
# then the C5 end-to-end test (tests/test_gpu_scale.py).
mkdir -p gpurun_out
ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 300 python -u bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/prof_c4.json 2> gpurun_out/prof_c4.err && \
ALVRL_C5_REPORT=gpurun_out/c5_report.json timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 1000 --timeout-method thread tests/test_gpu_scale.py > gpurun_out/c5full.log 2>&1
