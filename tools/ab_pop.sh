set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_fused_split.py > gpurun_out/pop_pytest.log 2>&1 || { tail -20 gpurun_out/pop_pytest.log; exit 1; }
tail -1 gpurun_out/pop_pytest.log
C="python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 2"
for i in 1 2; do
  ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_head.so timeout -k 10 300 $C > gpurun_out/pab_head_$i.log 2>&1 || exit 1
  timeout -k 10 300 $C > gpurun_out/pab_tree_$i.log 2>&1 || exit 1
  ALVRL_PROJ_CPP=8192 timeout -k 10 300 $C > gpurun_out/pab_cpp_$i.log 2>&1 || exit 1
  echo "run $i: head $(grep -o 'refine [0-9]* ms' gpurun_out/pab_head_$i.log | tr '\n' ' ') tree $(grep -o 'refine [0-9]* ms' gpurun_out/pab_tree_$i.log | tr '\n' ' ') cpp8192 $(grep -o 'refine [0-9]* ms' gpurun_out/pab_cpp_$i.log | tr '\n' ' ')"
done
timeout -k 10 400 python tools/c5_share.py > gpurun_out/pab_c5.log 2>&1 || exit 1
ALVRL_PROJ_CPP=8192 timeout -k 10 400 python tools/c5_share.py > gpurun_out/pab_c5_cpp.log 2>&1 || exit 1
echo "C5 rank 0: $(grep -o 'refine [0-9]* ms' gpurun_out/pab_c5.log | tr '\n' ' ') cpp8192 $(grep -o 'refine [0-9]* ms' gpurun_out/pab_c5_cpp.log | tr '\n' ' ')"
