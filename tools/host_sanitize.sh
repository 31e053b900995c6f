#!/bin/bash
# Host-code sanitizers (CPU container, no GPU): builds a copy of libghx whose HOST code is
# instrumented with AddressSanitizer + UndefinedBehaviorSanitizer (each -fsanitize= after
# -Xarch_host, so no device code is touched) in a scratch copy of the tree, and runs the CPU
# suite against it with the ASan runtime preloaded. Exercises the pattern producers, the halo
# generator, the oracle comparisons and the ABI's argument checks; the planner's device-table
# uploads need a GPU and are not covered here. The link-only tests (C++ headers compiled against
# libghx) are skipped: the instrumented library needs the sanitizer runtime at link time.
# Usage: bash tools/host_sanitize.sh [scratch dir, default /tmp/ghx_san]
set -e
S=${1:-/tmp/ghx_san}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$S" && mkdir -p "$S"
(cd "$ROOT" && git ls-files | tar -cf - -T -) | tar -xf - -C "$S"
for d in oracle/build oracle/_ref tools/bin tools/lib tests/cpp/bin; do
  mkdir -p "$S/$d"
  cp -r "$ROOT/$d/." "$S/$d/" 2>/dev/null || true
done
make -C "$S/ghex_amd/csrc" -j8 CXXFLAGS="-std=c++17 -O1 -g -fPIC -Wall -Wno-unused-parameter \
  -I../../include -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -Xarch_host -fno-omit-frame-pointer -shared-libsan" > "$S/build.log" 2>&1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$S"
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  LD_PRELOAD="$RT" python -m pytest tests -q -m "not gpu" -p no:cacheprovider -k "not compiles"
