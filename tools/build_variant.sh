#!/bin/bash
# A kernel variant of the product library for same-box A/Bs (tools/ab.py, NB_LIB):
#   tools/build_variant.sh <name> -DKNOB=1 ...   -> build_ab/libnasp_bloom_<name>.so
# Reuses the host objects of the in-tree build (make -C nasp-key-value-engine_amd first).
set -eu
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/nasp-key-value-engine_amd/build
mkdir -p "$R/build_ab"
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" \
    -c "$R/nasp-key-value-engine_amd/csrc/bloom_kernels.hip" -o "$R/build_ab/bloom_kernels_$NAME.o"
hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/build_ab/libnasp_bloom_$NAME.so" \
    "$R/build_ab/bloom_kernels_$NAME.o" "$B/bloom_host.o" "$B/bloom_stream.o" "$B/merkle_kernels.o" "$B/nb_knobs.o"
echo "built build_ab/libnasp_bloom_$NAME.so"
