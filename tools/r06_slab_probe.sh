#!/bin/bash
# Round 6: slab reduction with 32 thread groups (option slab_groups) -- weight-gradient tests, then the step A/B
set -uo pipefail
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_network.py \
  tests/test_engine.py -k "wgrad or defer or deterministic or fallback_paths or slab" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 500 python -u tools/opt_sweep_step.py --rounds 4 --arms "slab_groups=8;slab_groups=32;slab_groups=8;slab_groups=32" \
  > $O/sweep.log 2>&1 || exit 4
grep -v amdgpu $O/sweep.log
