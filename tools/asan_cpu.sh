#!/bin/bash
# AddressSanitizer + UBSan over the host code, on the CPU:
# builds oracle/_asan/liboracle.so (the restatement) and build-asan/libcyclone*.so
# (the C ABI's host side: argument checks, no-device paths, dataset staging,
# the libsvm parser; device code unsanitised) and runs the CPU test suite
# against them, the ASan runtime preloaded into python.  GPU ASan is not
# available on the pool (and not needed: the kernels are checked by parity).
# Usage: tools/asan_cpu.sh [pytest args]   (default: the whole -m "not gpu" suite)
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
make -s -j8 -C cycloneml_amd/csrc asan
RT=$(/opt/rocm/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export CYC_LIB_DIR="$PWD/build-asan"
export CYC_ORACLE_LIB="$PWD/oracle/_asan/liboracle.so"
# leaks: python and torch hold allocations to exit; container overflow and
# the allocator's mismatch checks would flag torch's own code, not ours
export ASAN_OPTIONS="detect_leaks=0:detect_container_overflow=0:alloc_dealloc_mismatch=0:halt_on_error=1:abort_on_error=1:print_summary=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
if [ $# -eq 0 ]; then set -- tests -m "not gpu" -q -p no:cacheprovider; fi
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" python -m pytest "$@"
