#!/bin/bash
# phase-isolation builds of lic_stack.hip: lib/libtmae_d<N>.so with -DLSTK_DIAG=N (4 = no MFMA, 8 = no B
# LDS reads, 16 = no A loads; sums combine), every other object from the normal build (run build() first)
cd "$(dirname "$0")/.."
L=textmae-image-compression_amd/lib
for N in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Wno-unused-result -DLSTK_DIAG=$N \
    -c textmae-image-compression_amd/csrc/lic_stack.hip -o /tmp/lstk_d$N.o &
done
wait
for N in "$@"; do
  objs=$(ls $L/obj/*.o | grep -v lic_stack)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $L/libtmae_d$N.so $objs /tmp/lstk_d$N.o
done
