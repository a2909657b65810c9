#!/bin/bash
# A/B library variant: recompile ONE source with extra flags and link it with the in-tree objects of every
# other source into ab/libtmae_<name>.so (use with TMAE_LIB=ab/libtmae_<name>.so).
#   usage: tools/build_variant.sh <name> <source.hip> [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
OBJ=textmae-image-compression_amd/lib/obj
mkdir -p ab
extra=""
[ "$src" = attention.hip ] || [ "$src" = qkv_attn.hip ] && extra="-fno-honor-nans"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Wno-unused-result $extra "$@" \
  -c "textmae-image-compression_amd/csrc/$src" -o "/tmp/variant_$name.o"
objs=$(ls $OBJ/*.o | grep -v "/$src.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "ab/libtmae_$name.so" $objs "/tmp/variant_$name.o"
echo "ab/libtmae_$name.so"
