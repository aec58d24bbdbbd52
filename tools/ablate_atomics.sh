# Timing-only ablations of the atomic epilogues (results are numerically wrong): bench step time with
# the BN-statistics / BN-backward-reduction atomics skipped (fwd_debug=2) and the weight-gradient dW
# atomics skipped (wgrad_debug=1); plus the weight-gradient split-partial slabs off (wgrad_partials=0).
# GPU box, repo root.
set -o pipefail
for o in "" "--opt wgrad_partials=0" "--opt wgrad_debug=1" ${EXTRA:-}; do
  echo "== $o" >> gpurun_out/ablate.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-dice --steps 8 $o 2>&1 | grep metric | cut -c1-160 >> gpurun_out/ablate.log || exit 1
done
