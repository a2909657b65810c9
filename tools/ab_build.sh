#!/bin/bash
# A/B library: the in-tree objects with ONE source recompiled under extra flags, linked to ab/<name>.so
# (load it with TMAE_LIB=ab/<name>.so).   usage: tools/ab_build.sh <name> <source.hip> <flags...>
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
O=textmae-image-compression_amd/lib/obj
mkdir -p ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Wno-unused-result "$@" \
  -c textmae-image-compression_amd/csrc/$src -o ab/$name.o
objs=$(ls $O/*.o | grep -v "/$src.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/$name.so $objs ab/$name.o
echo ab/$name.so
