set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
C="python tools/c5_share.py --res 1024 --vrls 100000 --world 8 --passes 1"
for v in evlog evx_NOBAR evx_NOLOAD evx_NOCOEF; do
  ALVRL_EVLOG=$PWD/gpurun_out/evx_$v.log ALVRL_LIB=$PWD/mitsuba-alvrl_amd/variants/libalvrl_$v.so timeout -k 10 200 $C > gpurun_out/evx_$v.out 2>&1
  echo "$v rc=$?"
done
