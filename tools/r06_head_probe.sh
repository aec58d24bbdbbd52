#!/bin/bash
# Round 6: the unrolled head forward (head_fwd_unroll) and the compile-time BNR head backward (head_bwd_fast) --
# head / network tests, then the kernels' rocprofv3 averages with both on and both off
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_network.py \
  -k "head or fallback_paths or deterministic or unet_bn" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for v in new old; do
  o=""; [ $v = old ] && o="--opt head_fwd_unroll=1 --opt head_bwd_fast=0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O -o kt_$v -- python3 bench.py --no-cpu-baseline --no-dice $o \
    > $O/kt_$v.log 2>&1 || exit 4
  python3 - "$O/kt_${v}_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'head_' in r['Name']:
        print(sys.argv[2], r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
done
