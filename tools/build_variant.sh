#!/bin/bash
# A/B library variant: recompile ONE source with extra flags (or an older copy of it, given by path) and link it
# with the in-tree objects of every other source into ab/libtmae_<name>.so (use with TMAE_LIB=...).
#   usage: tools/build_variant.sh <name> <source.hip | path/to/source.hip> [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
CSRC=textmae-image-compression_amd/csrc
OBJ=textmae-image-compression_amd/lib/obj
base=$(basename "$src")
[ -f "$src" ] && path="$src" || path="$CSRC/$src"
mkdir -p ab
extra=""
{ [ "$base" = attention.hip ] || [ "$base" = qkv_attn.hip ]; } && extra="-fno-honor-nans"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$CSRC -Wno-unused-result $extra "$@" \
  -c "$path" -o "/tmp/variant_$name.o"
objs=$(ls $OBJ/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "ab/libtmae_$name.so" $objs "/tmp/variant_$name.o"
echo "ab/libtmae_$name.so"
