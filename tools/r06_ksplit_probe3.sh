#!/bin/bash
# Round 6: split-K threshold once tiles past 64 can split (claim slots of 512 counters): configs[0] f32, the f32 1024^2
# step, the bf16 bench step, plus the split-K parity tests
set -uo pipefail
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "split_k" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for o in 192 384 512 768; do
  timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 20 --no-cpu-baseline \
    --no-dice --opt tap64_ksplit_max=$o > $O/cfg1_max$o.log 2>&1 || exit 4
  echo "cfg1 max=$o $(grep -o '"ms_per_step": [0-9.]*' $O/cfg1_max$o.log)"
done
for o in 192 512; do
  timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 \
    --no-cpu-baseline --no-dice --opt tap64_ksplit_max=$o > $O/f32_1024_max$o.log 2>&1 || exit 5
  echo "f32_1024 max=$o $(grep -o '"ms_per_step": [0-9.]*' $O/f32_1024_max$o.log)"
done
timeout -k 10 400 python -u tools/ab_step.py --variant opt --opts "tap64_ksplit_max=192;tap64_ksplit_max=512" --rounds 3 \
  > $O/bf16_step_ab.log 2>&1 || exit 6
tail -3 $O/bf16_step_ab.log
