#!/bin/bash
# Round 6: split policy of the ConvTranspose weight gradients (igemm_wgrad_tap64_kernel, HBM-bound at 3.7-4.5 TB/s)
set -uo pipefail
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 300 python tools/bench_convt.py --kinds wgrad \
  --variants "wgrad_min_chunk=2048;wgrad_min_chunk=4096;wgrad_min_chunk=8192;wgrad_blocks=256;wgrad_blocks=512" \
  > $O/convt_wgrad.log 2>&1 || exit 3
grep -v amdgpu $O/convt_wgrad.log | tail -12
