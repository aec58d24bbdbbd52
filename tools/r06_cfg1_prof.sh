#!/bin/bash
# Round 6: kernel breakdown of BASELINE configs[0] (adipose_v3 f32 256^2 B=2)
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
B="bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 20 --warmup 3 --no-cpu-baseline --no-dice"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O -o kt -- python3 $B > $O/kt.log 2>&1 || exit 4
grep '^{"metric"' $O/kt.log | tail -1 > $O/bench.json
python3 tools/kstats.py $O/kt_kernel_trace.csv $O/bench.json > $O/kernel_breakdown.txt || exit 5
head -40 $O/kernel_breakdown.txt
