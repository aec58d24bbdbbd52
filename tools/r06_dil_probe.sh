#!/bin/bash
# Round 6: the dilated f32 halo weight gradient -- parity tests, then the f32 1024^2 and configs[0] steps with the
# kernel on and off, then the f32 kernel breakdown under rocprofv3, then the 2-rank bench path rehearsed with gloo
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py \
  -k "wgrad_f32_halo" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -3 $O/tests.log
for o in 1 0; do
  timeout -k 10 300 python bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 \
    --no-cpu-baseline --no-dice --opt wgrad_f32_dil=$o > $O/f32_1024_dil$o.log 2>&1 || exit 4
  echo "f32_1024 dil=$o $(tail -1 $O/f32_1024_dil$o.log | cut -c1-140)"
  timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --size 256 --batch 2 --steps 20 --no-cpu-baseline \
    --no-dice --opt wgrad_f32_dil=$o > $O/cfg1_dil$o.log 2>&1 || exit 5
  echo "cfg1 dil=$o $(tail -1 $O/cfg1_dil$o.log | cut -c1-140)"
done
B="bench.py --preset adipose_v3 --dtype f32 --size 1024 --batch 2 --steps 5 --warmup 2 --no-cpu-baseline --no-dice"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O -o f32kt -- python3 $B > $O/f32kt.log 2>&1 || exit 6
grep '^{"metric"' $O/f32kt.log | tail -1 > $O/f32_bench.json
python3 tools/kstats.py $O/f32kt_kernel_trace.csv $O/f32_bench.json > $O/f32_kernel_breakdown.txt || exit 7
head -24 $O/f32_kernel_breakdown.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --dist-backend gloo --no-dice > $O/bench_gloo2.log 2>&1 || exit 8
tail -1 $O/bench_gloo2.log | cut -c1-300
