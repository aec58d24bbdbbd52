#!/bin/bash
# Round 6: f32 halo weight-gradient row tails and the 40-combination zero-tail table -- tests, then the adipose_v3 f32
# steps (1024^2 B=2 and configs[0]) against the round-5 table (8 combinations, chunk tails only, weight 50 %)
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_network.py \
  -k "wgrad_f32 or f32_halo_wgrad or zero_tail or zt" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
OLD="--opt wgrad_f32_rt=0 --opt wgrad_f32_zt_max=8 --opt wgrad_f32_zt_w=50"
for r in 1 2; do
  for v in new old; do
    o=""; [ $v = old ] && o="$OLD"
    timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 \
      --no-cpu-baseline --no-dice $o > $O/f32_1024_${v}_$r.log 2>&1 || exit 4
    echo "f32_1024 $v $r $(tail -1 $O/f32_1024_${v}_$r.log | cut -c1-130)"
  done
done
for v in new old; do
  o=""; [ $v = old ] && o="$OLD"
  timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 20 --no-cpu-baseline \
    --no-dice $o > $O/cfg1_$v.log 2>&1 || exit 5
  echo "cfg1 $v $(tail -1 $O/cfg1_$v.log | cut -c1-130)"
done
