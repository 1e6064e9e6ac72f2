#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against ASan + UBSan builds of the
# host code: libfugu's host half (fugu.cpp, host.cpp; the device kernels are
# not instrumented) and the CPU oracle.
# Python is not instrumented, so the ASan runtime is preloaded; leak checking
# is off (the interpreter's own allocations are not ours to fix).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$R/fugu_amd/csrc" asan
make -s -C "$R/oracle" asan OUT="$R/oracle"
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
cd "$R"
LD_PRELOAD="$ASAN_RT $UBSAN_RT" \
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
FUGU_LIB="$R/fugu_amd/libfugu_asan.so" FUGU_ORACLE_LIB="$R/oracle/libfugu_oracle_asan.so" \
  python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
