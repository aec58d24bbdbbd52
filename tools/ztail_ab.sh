set -uo pipefail
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --preset adipose_v3 --dtype f32 --batch 2 --steps 10 --warmup 3 --no-cpu-baseline --no-dice --opt f32_ztail=$v 2>/dev/null | sed "s/^/ztail=$v r$r /" || exit 1
  done
done
