#!/bin/bash
# Same-box A/B of one native option on the f32 adipose_v3 1024^2 B=2 training step (bench.py --opt), ABAB x 3.
# usage: bash tools/f32_opt_ab.sh <option> <value A> <value B>
set -uo pipefail
O=$1; A=$2; B=$3
for r in 1 2 3; do
  for v in $A $B; do
    timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --batch 2 --steps 10 --warmup 3 --no-cpu-baseline \
      --no-dice --opt $O=$v 2>/dev/null | sed "s/^/$O=$v r$r /" || exit 1
  done
done
