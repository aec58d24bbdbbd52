#!/bin/bash
# Round 6: staggered LDS-DMA (wgrad_pair_spread 8) vs 6 on the tap-pair weight gradient, and the whole bench step with
# the tap-pair form against the 8-wave form (same process, alternating blocks)
set -uo pipefail
mkdir -p gpurun_out/r06s
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "wgrad" \
  > gpurun_out/r06s/tests.log 2>&1 || { echo tests_failed; exit 1; }
L="L0 64->64,L0 128,L1 128,L2,L3 512,L4 1024->1024,L3 1024,L1 256"
V="wgrad_halop_pair=0;wgrad_pair_spread=6;wgrad_pair_spread=8"
timeout -k 10 300 python -u tools/bench_kernels.py --kinds wgrad --rounds 4 --reps 5 --variants "$V" --layers "$L" \
  > gpurun_out/r06s/variants.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/ab_step.py --variant opt --opts "wgrad_halop_pair=0;wgrad_halop_pair=1" --rounds 4 \
  > gpurun_out/r06s/step_ab.log 2>&1 || exit 3
