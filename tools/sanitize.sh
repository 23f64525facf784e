#!/bin/bash
# Host ASan + UBSan run of the CPU test suite: the C-ABI layer (libshockidx_san.so: write_idx,
# argument checks, the Part/Range parsers, ...) and the C oracle (liboracle_san.so), loaded
# into one Python process with clang's sanitizer runtime preloaded.  CPU only (no GPU
# sanitizers on this pool); leaks are not checked (the interpreter's own allocations).
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C shock_amd/csrc all
make -s -C oracle && make -s -f tools/sanitize.mk
ASAN=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LD_PRELOAD="$ASAN" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0 \
  UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 SHOCKIDX_VARIANT=san ORACLE_VARIANT=san \
  python -m pytest -q -m "not gpu" -p no:cacheprovider --ignore=tests/test_dist_cpu.py \
  --ignore=tests/test_sanitize_host.py "${@:-tests}"
