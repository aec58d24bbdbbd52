#!/bin/bash
# sample GFX clock / power while the bench step runs (1 GPU)
( timeout -k 10 120 python bench.py --no-cpu-baseline --no-dice --steps 60 --warmup 3 > gpurun_out/clk_bench.log 2>&1 ) &
BP=$!
for i in $(seq 1 24); do
  sleep 0.5
  timeout 10 amd-smi metric -c -p 2>/dev/null | grep -E "SOCKET_POWER|^        GFX_0:|CLK: " | head -3 | tr '\n' ' ' >> gpurun_out/clk.log
  echo >> gpurun_out/clk.log
done
wait $BP
