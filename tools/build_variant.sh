#!/bin/bash
# Build libalvrl.so with extra flags for refine.hip only (developer A/B):
#   tools/build_variant.sh NAME -DSOME_FLAG ...  -> mitsuba-alvrl_amd/variants/libalvrl_NAME.so
# The other objects come from the regular build (make first).
set -e
cd "$(dirname "$0")/../mitsuba-alvrl_amd"
name=$1; shift
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value \
  -I../include -ffp-contract=off "$@" -c csrc/refine.hip -o /tmp/refine_$name.o
objs=$(ls build/*.o | grep -v '/refine.o$' | grep -v '/asan_')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libalvrl_$name.so /tmp/refine_$name.o $objs -lpthread -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl
echo "variants/libalvrl_$name.so"
