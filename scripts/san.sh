#!/bin/bash
# Host sanitizer runs (SURVEY §5 "race detection / sanitizers"), CPU only:
#   1. ASan + UBSan builds of the oracle, the host harnesses of the product's
#      device code (loader, BVH builder, sample path) and the product library's
#      host side, then the whole CPU test suite on them (clang's shared ASan
#      runtime preloaded into python, leak checks off: python's own allocations);
#      tests/test_json_corpus.py feeds the JSON reader its malformed corpus there;
#   2. TSan: the oracle's threaded renderer (tests/native/tsan_driver.c) and the
#      product's loader / BVH builder / image writer from 8 threads
#      (tests/native/tsan_host.cpp).
# Logs go to $OUT (default gpurun_out/san); exit status non-zero on any report.
#   bash scripts/san.sh [out_dir]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$R/gpurun_out/san}
mkdir -p "$OUT"
cd "$R"
J=${MAKE_JOBS:-8}
make -s -C oracle san tsan
make -s -j"$J" -C tests/native san tsan
make -s -j"$J" -C rs-pathtracing_amd san
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
echo "== ASan+UBSan: CPU suite on the sanitizer builds ($RT)" | tee "$OUT/asan_suite.log"
LD_PRELOAD="$RT" \
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:detect_odr_violation=0:log_path="$OUT/asan" \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path="$OUT/ubsan" \
PT_ORACLE_LIB="$R/oracle/_build_san/liboracle.so" \
PT_NATIVE_BUILD=_build_san \
PT_AMD_LIB="$R/rs-pathtracing_amd/build_san/librs_pathtracing_amd.so" \
PT_SAN_RUN=1 \
    timeout -k 10 3000 python -m pytest tests -q -m "not gpu" -p no:xdist -p no:cacheprovider >> "$OUT/asan_suite.log" 2>&1
tail -3 "$OUT/asan_suite.log"
if ls "$OUT"/asan.* "$OUT"/ubsan.* > /dev/null 2>&1; then
    echo "sanitizer reports:"; ls "$OUT"/asan.* "$OUT"/ubsan.* 2>/dev/null; exit 1
fi
echo "== TSan" > "$OUT/tsan.log"
TSAN_OPTIONS=halt_on_error=1 ./oracle/_build_san/oracle_tsan >> "$OUT/tsan.log" 2>&1
mkdir -p /tmp/pt_tsan_host
TSAN_OPTIONS=halt_on_error=1 ./tests/native/_build_san/tsan_host scenes/cornell_box.json /tmp/pt_tsan_host >> "$OUT/tsan.log" 2>&1
cat "$OUT/tsan.log"
echo "sanitizer runs clean"
