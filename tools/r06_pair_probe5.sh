#!/bin/bash
# Round 6: LDS-DMA schedules of the tap-pair weight gradient (spread 6: 3-4-3-0 groups at row starts; 9: one group per
# MFMA-cluster boundary) and the cost of the wait for the next patch's DMA (ablation bit 4)
set -uo pipefail
mkdir -p gpurun_out/r06t
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "wgrad or dp_sliding" \
  > gpurun_out/r06t/tests.log 2>&1 || { echo tests_failed; exit 1; }
L="L0 64->64,L0 128,L1 128,L2,L3 512,L4 1024->1024,L3 1024,L1 256"
timeout -k 10 300 python -u tools/bench_kernels.py --kinds wgrad --rounds 4 --reps 5 \
  --variants "wgrad_halop_pair=0;wgrad_pair_spread=6;wgrad_pair_spread=9" --layers "$L" > gpurun_out/r06t/variants.log 2>&1 || exit 2
V="wgrad_pair_spread=6;wgrad_pair_spread=6,wgrad_debug=16;wgrad_pair_spread=6,wgrad_debug=2;wgrad_pair_spread=9,wgrad_debug=16"
V="$V;wgrad_pair_spread=6,wgrad_debug=1;wgrad_pair_spread=6,wgrad_debug=15"
ADP_LIB_PATH=ab/libadipose_ablation.so timeout -k 10 300 python -u tools/bench_kernels.py --kinds wgrad --rounds 3 --reps 5 \
  --variants "$V" --layers "L0 64->64,L2,L3 512,L4 1024->1024" > gpurun_out/r06t/ablation.log 2>&1 || exit 3
