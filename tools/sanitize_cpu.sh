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
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
# Python itself is not instrumented: no leak report at exit; stop at the first error
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@" || rc=$?

# the sanitizer builds are not loaded by any GPU run: keep them out of the tree gpurun ships
rm -f mitsuba-alvrl_amd/libalvrl_asan.so oracle/liboracle_asan.so
exit $rc
