#!/bin/bash
# Build libalvrl.so with extra flags for gather.hip only (developer A/B of the
# gather kernels; timing experiments such as -DALVRL_EXP_RNG_ROUNDS=N):
#   tools/build_variant_gather.sh NAME -DSOME_FLAG ...  -> mitsuba-alvrl_amd/variants/libalvrl_NAME.so
# The other objects come from the regular build (make first).
set -e
cd "$(dirname "$0")/../mitsuba-alvrl_amd"
name=$1; shift
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value \
  -I../include -fno-hip-fp32-correctly-rounded-divide-sqrt -fgpu-flush-denormals-to-zero -ffp-contract=on "$@" -c csrc/gather.hip -o /tmp/gather_$name.o
objs=$(ls build/*.o | grep -v '/gather.o$' | grep -v '/asan_')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libalvrl_$name.so /tmp/gather_$name.o $objs -lpthread -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl
echo "variants/libalvrl_$name.so"
