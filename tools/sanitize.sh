#!/bin/bash
# AddressSanitizer + UBSan over the CPU-side C / C++: the C oracle, the host builds
# of the product headers (deflate_len.hpp via tests/native/zlen_host.cpp, format_kernels.hpp via
# tests/native/fmt_host.cpp) and the engine library's host code (make -C taxi2_amd/csrc san: the
# C ABI entry points, taxi2_subset_aggregate, taxi2_dereplicate_walk), driven by the CPU tests that
# exercise them.  Runs here (no GPU); the log goes to profiles/r3/sanitize.log.
set -o pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r3/sanitize.log}
mkdir -p "$(dirname "$LOG")"
make -s -C oracle san || exit 1
make -s -C taxi2_amd/csrc san 2>&1 | grep -v "warning" || true
test -f taxi2_amd/_lib/libtaxi2_mi355x_san.so || exit 1
# clang's runtime (its ASan library carries the UBSan handlers): the engine library is built by
# hipcc (clang), so the oracle and the header harnesses are built by the same clang
LLVM=/opt/rocm/lib/llvm
ASAN_LIB=$(ls $LLVM/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
{
  echo "# tools/sanitize.sh $(date -u +%Y-%m-%dT%H:%MZ): -fsanitize=address,undefined ($($LLVM/bin/clang --version | head -1); hipcc -Xarch_host)"
  LD_PRELOAD="$ASAN_LIB" TAXI2_HOST_CXX=$LLVM/bin/clang++ ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  TAXI2_ORACLE_LIB=libtaxi2_oracle_san.so TAXI2_LIB=libtaxi2_mi355x_san.so \
  TAXI2_HOST_CFLAGS="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g" \
  timeout -k 10 1800 python -m pytest tests/test_oracle.py tests/test_ncd.py tests/test_writers_native.py \
      tests/test_subsets.py tests/test_dereplicate.py tests/test_group_minima.py tests/test_native_abi.py -m "not gpu" -q -p no:cacheprovider 2>&1
  echo "exit status: $?"
} | tee "$LOG" | tail -5
