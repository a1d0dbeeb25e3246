#!/usr/bin/env bash
# oracle/build_ref.sh -- TEST INFRASTRUCTURE recipe.  Compiles the reference's
# own sources, where they lie under /root/reference (the two vendored
# tarballs are unpacked into a scratch directory OUTSIDE the repo, which is
# deleted afterwards), with gcc/g++ directly -- the reference's makefile is not
# run.  Outputs go only to oracle/_ref/ (git-ignored; the built binaries travel
# to the GPU box, no reference source does):
#   oracle/_ref/libbz2ref.so  patched libbz2 1.0.6 + oracle/bz2_ref_harness.c
#   oracle/_ref/starch3       the reference CLI (src/starch3.cpp, -DDEBUG as mk:18)
#   oracle/_ref/zrealloc.so   LD_PRELOAD shim for exact Content capture
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
mkdir -p "$OUT"
if [ ! -d "$REF/third-party" ]; then
  echo "build_ref: $REF not present; skipping (prebuilt oracle/_ref is used as-is)" >&2
  exit 0
fi
TMP=$(mktemp -d /tmp/starch_ref_build.XXXXXX)
trap 'rm -rf "$TMP"' EXIT
tar xzf "$REF/third-party/bzip2-1.0.6.tar.gz" -C "$TMP" --exclude='bzip2-1.0.6/bzip2-1.0.6'
tar xzf "$REF/third-party/jansson-2.9.tar.gz" -C "$TMP" jansson-2.9/src/jansson.h jansson-2.9/android/jansson_config.h
BZ="$TMP/bzip2-1.0.6"
BZSRC="$BZ/blocksort.c $BZ/huffman.c $BZ/crctable.c $BZ/randtable.c $BZ/compress.c $BZ/decompress.c $BZ/bzlib.c"
# libbz2 exactly as its Makefile compiles it (-O2 -D_FILE_OFFSET_BITS=64), as a .so for ctypes
gcc -O2 -fPIC -D_FILE_OFFSET_BITS=64 -w -I"$BZ" -shared -Wl,-Bsymbolic \
    -o "$OUT/libbz2ref.so" $BZSRC "$HERE/bz2_ref_harness.c"
# the reference CLI: g++ -std=c++11 -O3 -DDEBUG (mk:2,18), statically including the patched libbz2
for f in $BZSRC; do gcc -O2 -D_FILE_OFFSET_BITS=64 -w -I"$BZ" -c "$f" -o "$TMP/$(basename "$f" .c).o"; done
g++ -std=c++11 -O3 -D_LARGEFILE64_SOURCE -D_FILE_OFFSET_BITS=64 -DDEBUG -w \
    -I"$REF/include" -I"$BZ" -I"$TMP/jansson-2.9/src" -I"$TMP/jansson-2.9/android" \
    "$REF/src/starch3.cpp" "$TMP"/*.o -lpthread -o "$OUT/starch3"
gcc -O2 -fPIC -shared -o "$OUT/zrealloc.so" "$HERE/zrealloc.c" -ldl
echo "build_ref: ok -> $OUT" >&2
