#!/bin/bash
# Build libadipose_hip.so from a git revision (default HEAD) into ab/libadipose_<rev>.so, for same-box A/B
# timing against the working tree (ADP_LIB_PATH selects the library a process loads; timing only).
# usage: bash tools/build_ref_lib.sh [rev]
set -euo pipefail
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/adp_ref.XXXXXX)
git -C "$ROOT" archive "$REV" adipose_tissue-unet_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/ab"
TAG=$(git -C "$ROOT" rev-parse --short "$REV")
make -C "$TMP/adipose_tissue-unet_amd/csrc" -j8 OUT="$ROOT/ab/libadipose_$TAG.so" "$ROOT/ab/libadipose_$TAG.so" > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
rm -rf "$TMP"
echo "$ROOT/ab/libadipose_$TAG.so"
