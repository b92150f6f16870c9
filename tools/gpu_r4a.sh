# Round-4 session a: gather RNG-cost A/B (timing-only variants) and the
# refinement parity suites on the LDS-bounds-checking build.
mkdir -p gpurun_out
for v in base rng7 rng0 base; do
  if [ $v = base ]; then L=mitsuba-alvrl_amd/libalvrl.so; else L=mitsuba-alvrl_amd/variants/libalvrl_$v.so; fi
  ALVRL_LIB=$L timeout -k 10 120 python -u bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rng_$v.json 2> gpurun_out/rng_$v.err || exit 1
done && \
ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_ldscheck.so timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_chains.py tests/test_gpu_dielectric.py > gpurun_out/ldscheck.log 2>&1
