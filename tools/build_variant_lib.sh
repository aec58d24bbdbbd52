#!/bin/bash
# Build the working tree's library with extra preprocessor definitions into ab/libadipose_<name>.so (same-box A/B of a
# compile-time variant against the tree's own library: tools/ab_libs.sh; timing only).
# usage: bash tools/build_variant_lib.sh <name> -DFOO=1 [-DBAR=2 ...]
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/adp_var.XXXXXX)
mkdir -p "$TMP/adipose_tissue-unet_amd" "$ROOT/ab"
cp -r "$ROOT/adipose_tissue-unet_amd/csrc" "$TMP/adipose_tissue-unet_amd/"
cp -r "$ROOT/include" "$TMP/"
rm -rf "$TMP/adipose_tissue-unet_amd/csrc/build"
make -C "$TMP/adipose_tissue-unet_amd/csrc" -j8 EXTRA_DEFS="$*" OUT="$ROOT/ab/libadipose_$NAME.so" \
  "$ROOT/ab/libadipose_$NAME.so" > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
rm -rf "$TMP"
echo "$ROOT/ab/libadipose_$NAME.so"
