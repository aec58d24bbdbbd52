#!/bin/bash
# Round profile of the default bench command (run on the GPU box, from the repo root):
#   1. rocprofv3 --kernel-trace --stats   -> profiles/<tag>_kernel_stats.csv (+ bench line)
#   2. rocprofv3 --pmc FETCH_SIZE          (own pass: TCC counter slots, MI355X_MICROARCH.md)
#   3. rocprofv3 --pmc WRITE_SIZE          (own pass)
#   -> gpurun_out/prof_<tag>/{kernel_stats.csv, traffic.json, kernel_breakdown.txt, bench.json}
#      (only gpurun_out/ travels back from the GPU box; copy them to profiles/<tag>_* afterwards:
#       bash tools/profile_round.sh --collect <tag>)
# usage: bash tools/profile_round.sh r01 [extra bench args]
set -euo pipefail
if [ "${1:-}" = "--collect" ]; then
  T=$2; D=gpurun_out/prof_$T
  cp "$D/kernel_stats.csv" "profiles/${T}_kernel_stats.csv"
  cp "$D/traffic.json" "profiles/${T}_traffic.json"
  cp "$D/kernel_breakdown.txt" "profiles/${T}_kernel_breakdown.txt"
  cp "$D/bench.json" "profiles/${T}_bench_under_rocprof.json"
  exit 0
fi
TAG=${1:-r01}
shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
BENCH="bench.py --no-cpu-baseline --no-dice $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o kt -- python3 $BENCH > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT" -o fetch -- python3 $BENCH > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT" -o write -- python3 $BENCH > "$OUT/write.log" 2>&1
cp "$OUT/kt_kernel_stats.csv" "$OUT/kernel_stats.csv"
grep '^{"metric"' "$OUT/kt.log" | tail -1 > "$OUT/bench.json" || true
python3 tools/traffic_summary.py "$OUT/fetch_counter_collection.csv" "$OUT/write_counter_collection.csv" "$OUT/traffic.json" \
  "$OUT/bench.json"
# per-step figures over the timed steps only (warm-up / first-step allocations excluded; steps from the bench line)
python3 tools/kstats.py "$OUT/kt_kernel_trace.csv" "$OUT/bench.json" > "$OUT/kernel_breakdown.txt"
echo done
