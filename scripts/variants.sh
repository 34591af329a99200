#!/bin/bash
# Build alternate libraries for A/B runs (pt_wave.hip compile-time knobs):
#   bash scripts/variants.sh name "-DKNOB=1 -DOTHER=2" [name2 "flags2" ...]
# -> variants/<name>.so; the other objects are reused from the default build.
set -e
cd "$(dirname "$0")/../rs-pathtracing_amd"
make -s -j8 >/dev/null
mkdir -p ../variants
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    mkdir -p build_$name
    for o in build/*.o; do [ "$(basename $o)" = pt_wave.o ] || cp -p $o build_$name/; done
    rm -f build_$name/pt_wave.o
    make -s LIB=../variants/$name.so BUILD=build_$name EXTRA="$flags" >/dev/null &
done
wait
ls -la ../variants/
