# Round-4 session m: short-job parts in a busy launch gated on idle workgroups.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "refine" > gpurun_out/r4m_parity.log 2>&1 && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4m_c4_16.json 2> gpurun_out/r4m_c4_16.err && \
ALVRL_PART_IDLE_SHORT=8 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4m_c4_8.json 2> gpurun_out/r4m_c4_8.err && \
ALVRL_PART_IDLE_SHORT=32 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4m_c4_32.json 2> gpurun_out/r4m_c4_32.err && \
ALVRL_PART_MIN=0 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4m_c4_off.json 2> gpurun_out/r4m_c4_off.err && \
ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u tools/c5_share.py --res 1024 --vrls 100000 --world 8 > gpurun_out/r4m_c4w8.log 2>&1
