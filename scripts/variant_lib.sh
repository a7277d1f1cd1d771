#!/bin/bash
# A measurement variant of the library, built beside the product:
#   scripts/variant_lib.sh NAME PATCH.py
# copies bess_amd/{csrc,host} and include/ into build/var_NAME/, runs
# `python PATCH.py` there (it edits the copied sources in place), and builds
# scripts/bin/libbessgpu_NAME.so (+ its bg_rtc helper in scripts/bin/).
# bench.py --lib scripts/bin/libbessgpu_NAME.so times it on the same box;
# the product sources never carry the variant.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; PATCH=$(cd "$(dirname "$2")" && pwd)/$(basename "$2")
V="$ROOT/build/var_$NAME"
rm -rf "$V"; mkdir -p "$V/bess_amd"
cp -r "$ROOT/bess_amd/csrc" "$ROOT/bess_amd/host" "$V/bess_amd/"
cp -r "$ROOT/include" "$V/"
(cd "$V" && python3 "$PATCH")
mkdir -p "$ROOT/scripts/bin"
make -C "$V/bess_amd/csrc" -j8 OUT="$ROOT/scripts/bin/libbessgpu_$NAME.so" OBJDIR="$V/obj" \
  SONAME="libbessgpu_$NAME.so" > "$V/build.log" 2>&1 || { tail -20 "$V/build.log"; exit 1; }
echo "$ROOT/scripts/bin/libbessgpu_$NAME.so"
