#!/bin/bash
# Round 6: weight-gradient block target of the 256x256 tap64 configuration (1024 -> 256) on both presets' steps
set -uo pipefail
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py \
  -k "wgrad and (tap64 or convt or transpose)" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/ab_step.py --variant opt --opts "wgrad_blocks_1tile=100000;wgrad_blocks_1tile=256" --rounds 4 \
  > $O/unet_bn_ab.log 2>&1 || exit 4
tail -2 $O/unet_bn_ab.log
timeout -k 10 400 python -u tools/ab_step.py --preset adipose_v3 --variant opt --opts "wgrad_blocks_1tile=100000;wgrad_blocks_1tile=256" \
  --rounds 4 > $O/v3_bf16_ab.log 2>&1 || exit 5
tail -2 $O/v3_bf16_ab.log
