#!/bin/bash
# Whole-step A/B of the conv kernels' run-time switches (GPU box): bench ms/step per option, 2 interleaved rounds.
# usage: bash tools/opt_sweep.sh > gpurun_out/opt_sweep.txt
mkdir -p gpurun_out
for r in 1 2; do
for o in "" "--opt wgrad_halop_grid=512" "--opt halo_persist_grid=512"; do
  v=$(timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 $o 2>/dev/null | grep '^{"metric"' | python -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])') || exit 1
  echo "r$r [$o] $v"
done; done
