#!/bin/bash
# Build the library of a git revision (default HEAD) into ab/<name>.so for same-box A/B runs against the
# working tree (load it with TMAE_LIB=ab/<name>.so).   usage: tools/build_head_lib.sh [rev] [name]
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}; name=${2:-base}
tmp=$(mktemp -d /tmp/tmae_rev.XXXXXX)
git archive "$rev" textmae-image-compression_amd include | tar -x -C "$tmp"
(cd "$tmp" && python3 -c "import sys; sys.path.insert(0, 'textmae-image-compression_amd'); import build; build.build()")
mkdir -p ab
cp "$tmp/textmae-image-compression_amd/lib/libtmae.so" "ab/$name.so"
rm -rf "$tmp"
echo "ab/$name.so"
