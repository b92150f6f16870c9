#!/bin/bash
# The CPU suite (pytest -m "not gpu") on AddressSanitizer + UBSan builds of the
# host C++ (mitsuba-alvrl_amd/libalvrl_asan.so) and of the oracle
# (oracle/liboracle_asan.so).  Host code only: GPU sanitizers are not
# available on this pool.  Usage: tools/sanitize_cpu.sh [pytest args]
set -e
rc=0
cd "$(dirname "$0")/.."
make -s -C oracle asan
make -s -C mitsuba-alvrl_amd -j8 asan
export ALVRL_LIB=$PWD/mitsuba-alvrl_amd/libalvrl_asan.so
export ALVRL_ORACLE_LIB=$PWD/oracle/liboracle_asan.so
# the sanitizer runtimes are appended to whatever the environment preloads
# already (nothing of it is removed or reordered), so ASan's link-order check is off
export LD_PRELOAD="${LD_PRELOAD:+$LD_PRELOAD:}$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
# Python itself is not instrumented: no leak report at exit; stop at the first error
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@" || rc=$?

# the sanitizer builds are not loaded by any GPU run: keep them out of the tree gpurun ships
rm -f mitsuba-alvrl_amd/libalvrl_asan.so oracle/liboracle_asan.so
exit $rc
