#!/bin/bash
# Build libalvrl.so with extra flags for rbuild_strict.hip only (developer A/B):
#   tools/build_variant_strict.sh NAME -DSOME_FLAG ...  -> mitsuba-alvrl_amd/variants/libalvrl_NAME.so
# The other objects come from the regular build (make first).  Load with ALVRL_LIB=...
set -e
cd "$(dirname "$0")/../mitsuba-alvrl_amd"
name=$1; shift
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value \
  -I../include -Icsrc -ffp-contract=off -mllvm -disable-machine-licm "$@" -c csrc/rbuild_strict.hip -o /tmp/rbs_$name.o
objs=$(ls build/*.o | grep -v '/rbuild_strict.o$' | grep -v '/asan_')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libalvrl_$name.so /tmp/rbs_$name.o $objs -lpthread -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl
echo "variants/libalvrl_$name.so"
