#!/bin/bash
# HBM bytes per launch of the dominant forward kernel, layer by layer (unet_bn L5 shapes, tools/bench_kernels.py):
# kernel trace, then FETCH_SIZE and WRITE_SIZE in passes of their own (MI355X_MICROARCH.md, HBM section).
# usage (GPU box, repo root): bash tools/pmc_dom.sh [layers] [kinds] [variants]; results under gpurun_out/pmc_dom/
set -uo pipefail
export TMPDIR=/tmp
D=gpurun_out/pmc_dom
mkdir -p $D
LAYERS=${1:-L2 256->256,L3 512->512,L4 1024->1024}
KINDS=${2:-fwd,fwd_stats}
VARIANTS=${3:-tap64p_halo=1}
run() {  # tag, rocprof args...
  local tag=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" -f csv -d $D -o $tag -- python tools/bench_kernels.py --rounds 1 --reps 3 \
    --kinds "$KINDS" --variants "$VARIANTS" --layers "$LAYERS" > $D/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc"
  return $rc
}
run kt --kernel-trace --stats && run fetch --pmc FETCH_SIZE && run write --pmc WRITE_SIZE
