#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the forward tap64 launches of the unet_bn L5
# layer shapes (tools/bench_kernels.py), for the dominant-kernel analysis in DESIGN.md §3.
# usage (GPU box, repo root): bash tools/pmc_fwd.sh [layers] ; results under gpurun_out/pmc_fwd/
set -uo pipefail
export TMPDIR=/tmp
D=gpurun_out/pmc_fwd
mkdir -p $D
LAYERS=${1:-L2,L3 512->512,L4 1024->1024}
run() {  # tag, rocprof args...
  local tag=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" -f csv -d $D -o $tag -- python tools/bench_kernels.py --rounds 1 --reps 3 \
    --kinds fwd --variants "fwd_tap64=1" --layers "$LAYERS" > $D/$tag.log 2>&1
  echo "$tag rc=$?"
}
run kt --kernel-trace --stats
run sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE
run sq2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
run fetch --pmc FETCH_SIZE
