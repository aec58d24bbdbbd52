#!/bin/bash
# Round 6: the Z3 tap split of 3-row-block chunk tails -- tests, per-layer probe, f32 step with it on and off
set -uo pipefail
O=gpurun_out/r06ad
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_network.py \
  -k "wgrad_f32 or f32_halo_wgrad or zero_tail or zt or input_layer" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/probes/f32_wgrad_probe.py "wgrad_f32_z3=0;wgrad_f32_z3=1;wgrad_f32_z3_w=40;wgrad_f32_z3_w=55" \
  > $O/probe.log 2>&1 || exit 4
sed -e "s/igemm_wgrad_halo_f32_kernel//g" -e "s/TF-real//g" $O/probe.log | grep -v amdgpu | cut -c1-230 | head -3
for r in 1 2; do
  for o in 1 0; do
    timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 \
      --no-cpu-baseline --no-dice --opt wgrad_f32_z3=$o > $O/f32_z3_${o}_$r.log 2>&1 || exit 5
    echo "f32_1024 z3=$o $(grep -o '"ms_per_step": [0-9.]*' $O/f32_z3_${o}_$r.log)"
  done
done
