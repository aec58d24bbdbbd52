#!/bin/bash
# Round 6: tap64 split-K threshold (tap64_ksplit_max: tiles x occupancy) on the f32 configs[0] step, the f32 1024^2 step
# and the bf16 bench step
set -uo pipefail
mkdir -p gpurun_out/r06k2
for o in 0 96 192 320; do
  timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 20 --no-cpu-baseline \
    --no-dice --opt tap64_ksplit_max=$o > gpurun_out/r06k2/cfg1_max$o.log 2>&1 || exit 3
  echo "cfg1 max=$o $(tail -1 gpurun_out/r06k2/cfg1_max$o.log | cut -c1-140)"
done
for o in 0 96 320; do
  timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 \
    --no-cpu-baseline --no-dice --opt tap64_ksplit_max=$o > gpurun_out/r06k2/f32_1024_max$o.log 2>&1 || exit 4
  echo "f32_1024 max=$o $(tail -1 gpurun_out/r06k2/f32_1024_max$o.log | cut -c1-140)"
done
timeout -k 10 300 python -u tools/ab_step.py --variant opt --opts "tap64_ksplit_max=96;tap64_ksplit_max=320" --rounds 3 \
  > gpurun_out/r06k2/bf16_step_ab.log 2>&1 || exit 5
tail -2 gpurun_out/r06k2/bf16_step_ab.log
