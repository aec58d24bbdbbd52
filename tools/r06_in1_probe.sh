#!/bin/bash
# Round 6: the f32 input-layer weight gradient (wgrad_in1_f32_kernel) -- tests, then the adipose_v3 f32 steps with it
# on and off (same process order alternating)
set -uo pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py \
  -k "input_layer or wgrad_f32" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for r in 1 2; do
  for o in 1 0; do
    timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 \
      --no-cpu-baseline --no-dice --opt wgrad_f32_in1=$o > $O/f32_1024_in1_${o}_$r.log 2>&1 || exit 4
    echo "f32_1024 in1=$o $(grep -o '"ms_per_step": [0-9.]*' $O/f32_1024_in1_${o}_$r.log)"
  done
done
for o in 1 0; do
  timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 20 --no-cpu-baseline \
    --no-dice --opt wgrad_f32_in1=$o > $O/cfg1_in1_$o.log 2>&1 || exit 5
  echo "cfg1 in1=$o $(grep -o '"ms_per_step": [0-9.]*' $O/cfg1_in1_$o.log)"
done
