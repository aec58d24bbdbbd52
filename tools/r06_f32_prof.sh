#!/bin/bash
# f32 1024^2 B=2 kernel breakdown under rocprofv3 (kernel trace only)
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06k_f32}
mkdir -p $O
B="bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 --no-cpu-baseline --no-dice"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O -o kt -- python3 $B > $O/kt.log 2>&1 || exit 4
grep '^{"metric"' $O/kt.log | tail -1 > $O/bench.json
python3 tools/kstats.py $O/kt_kernel_trace.csv $O/bench.json > $O/kernel_breakdown.txt || exit 5
head -32 $O/kernel_breakdown.txt
