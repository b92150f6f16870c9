#!/bin/bash
# Round-4 session inl: split()'s helpers inlined (projections + sort: inlproj; weighted picks: inlws) vs the tree
mkdir -p gpurun_out
V=mitsuba-alvrl_amd/variants
for rep in 1 2; do
  for v in base inlproj inlws; do
    if [ $v = base ]; then unset ALVRL_LIB; else export ALVRL_LIB=$V/libalvrl_$v.so; fi
    timeout -k 10 200 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/inl_c4_${v}_$rep.json 2> gpurun_out/inl_c4_${v}_$rep.err || exit 1
  done
done
unset ALVRL_LIB
for v in inlproj inlws; do
  ALVRL_LIB=$V/libalvrl_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k refine > gpurun_out/inl_parity_$v.log 2>&1 || exit 1
done
echo "== done"
