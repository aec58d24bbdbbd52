# A/B sweep of the BatchNorm elementwise launch shape (bn_unroll x bn_cap), GPU box
set -o pipefail
for u in ${UNROLLS:-1 2}; do for cap in ${CAPS:-65536 262144}; do
 timeout -k 10 100 python tools/bench_ew.py --ops bn_apply,bn_bwd_apply --opt bn_unroll=$u --opt bn_cap=$cap >> gpurun_out/ew_ab.log 2>&1 || exit 1
done; done
