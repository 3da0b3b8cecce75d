#!/bin/bash
# build/variants/<name>.so: libgcs.so compiled with extra -D flags (for tools/bench_variants.sh A/B runs on one box)
#   tools/build_variant.sh <name> -DGCS_X=1 ...
set -eu
name=$1; shift
src=$(cd "$(dirname "$0")/../3d-genome-cycle_amd/csrc" && pwd)
out=$(pwd)/build/variants; tmp=$(mktemp -d)
mkdir -p "$out"
for f in engine kernels contacts domain; do
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -Wno-unused-result "$@" -c -o "$tmp/$f.o" "$src/$f.hip" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out/$name.so" "$tmp"/*.o
rm -rf "$tmp"
