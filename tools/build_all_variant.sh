#!/bin/bash
# A/B library with extra flags on EVERY HIP source (a header-level knob such as common.h's TMAE_GELU_POLY):
# ab/libtmae_<name>.so.   usage: tools/build_all_variant.sh <name> [hipcc flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
CSRC=textmae-image-compression_amd/csrc
OBJ=textmae-image-compression_amd/lib/obj
out=/tmp/allvar_$name
mkdir -p "$out" ab
for f in $CSRC/*.hip; do
  extra=""
  case $(basename "$f") in attention.hip|qkv_attn.hip) extra="-fno-honor-nans";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$CSRC -Wno-unused-result $extra "$@" \
    -c "$f" -o "$out/$(basename "$f").o" || touch "$out/FAILED" &
done
wait
[ -e "$out/FAILED" ] && { echo "a source failed to compile"; rm -f "$out/FAILED"; exit 1; }
objs=$(ls $OBJ/*.cpp.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "ab/libtmae_$name.so" $out/*.hip.o $objs
echo "ab/libtmae_$name.so"
