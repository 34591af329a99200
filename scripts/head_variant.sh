#!/bin/bash
# A/B baseline: variants/<name>.so = the in-tree library with pt_wave.o rebuilt
# from the sources of git revision <rev> (default HEAD):
#   bash scripts/head_variant.sh [name] [rev]
set -e
name=${1:-head}; rev=${2:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive "$rev" rs-pathtracing_amd/csrc include | tar -x -C "$T"
mkdir -p "$R/variants" "$T/obj"
cd "$R/rs-pathtracing_amd" && make -s -j8 >/dev/null
for o in build/*.o; do [ "$(basename $o)" = pt_wave.o ] || cp -p $o "$T/obj/"; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 \
    -c "$T/rs-pathtracing_amd/csrc/pt_wave.hip" -o "$T/obj/pt_wave.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/variants/$name.so" "$T"/obj/*.o
rm -rf "$T"
ls -la "$R/variants/$name.so"
