#!/bin/bash
# Round 6: tap64 split-K -- its tests, the full GPU suite, and the f32 BASELINE configs[0] step with and without it
set -uo pipefail
mkdir -p gpurun_out/r06k
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "split_k" \
  > gpurun_out/r06k/ksplit_tests.log 2>&1 || { echo ksplit_tests_failed; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread \
  > gpurun_out/r06k/gpu_tests.log 2>&1 || { echo gpu_tests_failed; exit 2; }
for o in 0 1 0 1; do
  timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 20 --no-cpu-baseline \
    --no-dice --opt tap64_ksplit=$o > gpurun_out/r06k/cfg1_ksplit$o.log 2>&1 || exit 3
  tail -1 gpurun_out/r06k/cfg1_ksplit$o.log | cut -c1-160
done
