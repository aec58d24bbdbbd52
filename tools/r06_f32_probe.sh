#!/bin/bash
# Round 6: (1) the 2-rank bench path rehearsed with gloo on one GPU, (2) kernel breakdown of the f32 1024^2 B=2 step
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --dist-backend gloo --no-dice > $O/bench_gloo2.log 2>&1 || exit 3
tail -1 $O/bench_gloo2.log | cut -c1-300
B="bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 --no-cpu-baseline --no-dice"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O -o f32kt -- python3 $B > $O/f32kt.log 2>&1 || exit 4
grep '^{"metric"' $O/f32kt.log | tail -1 > $O/f32_bench.json
python3 tools/kstats.py $O/f32kt_kernel_trace.csv $O/f32_bench.json > $O/f32_kernel_breakdown.txt || exit 5
head -30 $O/f32_kernel_breakdown.txt
