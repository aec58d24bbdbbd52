#!/bin/bash
# Round 6: the tap-pair weight gradient's fragment-read schedules (wgrad_pair_pipe 0 / 1 / 2) and LDS-DMA schedules
set -uo pipefail
mkdir -p gpurun_out/r06r
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "wgrad" \
  > gpurun_out/r06r/tests.log 2>&1 || { echo tests_failed; exit 1; }
L="L0 64->64,L0 128,L1 128,L2,L3 512,L4 1024->1024,L3 1024,L1 256"
V="wgrad_halop_pair=0;wgrad_pair_pipe=0;wgrad_pair_pipe=1;wgrad_pair_pipe=2;wgrad_pair_spread=4,wgrad_pair_pipe=2"
timeout -k 10 400 python -u tools/bench_kernels.py --kinds wgrad --rounds 4 --reps 5 --variants "$V" --layers "$L" \
  > gpurun_out/r06r/variants.log 2>&1 || exit 2
V="wgrad_pair_pipe=2;wgrad_pair_pipe=2,wgrad_debug=1;wgrad_pair_pipe=2,wgrad_debug=2;wgrad_pair_pipe=2,wgrad_debug=4"
V="$V;wgrad_pair_pipe=2,wgrad_debug=8;wgrad_pair_pipe=2,wgrad_debug=15"
ADP_LIB_PATH=ab/libadipose_ablation.so timeout -k 10 300 python -u tools/bench_kernels.py --kinds wgrad --rounds 3 --reps 5 \
  --variants "$V" --layers "L0 64->64,L2,L3 512,L4 1024->1024" > gpurun_out/r06r/ablation.log 2>&1 || exit 3
