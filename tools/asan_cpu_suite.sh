#!/bin/bash
# The CPU test suite (pytest -m "not gpu") under AddressSanitizer +
# UndefinedBehaviorSanitizer: the oracle (make -C oracle asan) and the host
# code of libccrdt (make -C antidote_ccrdt_amd/csrc asan; device code is not
# instrumented) are loaded instrumented, with clang's shared ASan runtime
# preloaded into the Python process.  CPU only -- run in the build container.
set -e -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
make -s -C antidote_ccrdt_amd/csrc asan -j8
RT=$(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
# detect_leaks=0: CPython's own allocations at exit are not ours to report
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" \
CCRDT_LIB="$PWD/antidote_ccrdt_amd/lib/libccrdt_asan.so" \
CCRDT_ORACLE_LIB="$PWD/oracle/build/liboracle_asan.so" \
  python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
