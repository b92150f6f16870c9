#!/bin/bash
# Round-4 session inl2: the small-split variance engine inlined into split() (variant) vs the tree
mkdir -p gpurun_out
V=mitsuba-alvrl_amd/variants
for rep in 1 2 3; do
  for v in base inlsmall; do
    if [ $v = base ]; then unset ALVRL_LIB; else export ALVRL_LIB=$V/libalvrl_$v.so; fi
    timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/inl2_c4_${v}_$rep.json 2> gpurun_out/inl2_c4_${v}_$rep.err || exit 1
  done
done
ALVRL_LIB=$V/libalvrl_inlsmall.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k refine > gpurun_out/inl2_parity.log 2>&1
echo "== done"
