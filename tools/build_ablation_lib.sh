#!/bin/bash
# Build the working tree's library with the timing-only ablation switches compiled in (make ABLATION=1: the kernels
# read options fwd_debug / wgrad_debug; common.h ADP_DBG) into ab/libadipose_ablation.so. Run an ablation tool with
# ADP_LIB_PATH=ab/libadipose_ablation.so (timing only; the product library ignores those options).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/adp_abl.XXXXXX)
mkdir -p "$TMP/adipose_tissue-unet_amd" "$ROOT/ab"
cp -r "$ROOT/adipose_tissue-unet_amd/csrc" "$TMP/adipose_tissue-unet_amd/"
cp -r "$ROOT/include" "$TMP/"
rm -rf "$TMP/adipose_tissue-unet_amd/csrc/build"
make -C "$TMP/adipose_tissue-unet_amd/csrc" -j8 ABLATION=1 OUT="$ROOT/ab/libadipose_ablation.so" \
  "$ROOT/ab/libadipose_ablation.so" > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
rm -rf "$TMP"
echo "$ROOT/ab/libadipose_ablation.so"
