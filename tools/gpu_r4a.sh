mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c5_share.py --full --res 512 --vrls 20000 > gpurun_out/c5small.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ext_scene.py > gpurun_out/ext.log 2>&1 && \
for v in base rng7 rng0 base; do if [ $v = base ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi; ALVRL_LIB=$L timeout -k 10 120 python -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rng_$v.json 2> gpurun_out/rng_$v.err || exit 1; done && \
ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_ldscheck.so timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_chains.py > gpurun_out/ldscheck.log 2>&1
