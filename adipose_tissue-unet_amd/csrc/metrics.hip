// Pixel-level ROC AUC and average precision on the GPU (full_evaluation_enhanced.py:847-888, which calls
// scikit-learn's roc_auc_score / average_precision_score on the flattened probability map).
//
// Exact in the pixel counts, ties grouped by identical score as scikit-learn does:
//   1. key = order-preserving bits of the score, label = truth > 0.5; stable radix sort by key (rocPRIM
//      through hipCUB), inclusive sum of the sorted labels (positives at or below each rank) and an
//      inclusive max-scan of group-start ranks;
//   2. at the last rank e of each score group [s, e]: pos_g, neg_g from the positive prefix sums;
//        ROC AUC = sum_g pos_g * (negatives below s + neg_g / 2) / (P * N)   (Mann-Whitney with ties =
//                  the trapezoid area of the ROC curve over distinct thresholds);
//        AP      = sum_g (pos_g / P) * precision at threshold t_g, precision = positives / pixels >= t_g
//                  (the step-wise sum of average_precision_score over distinct thresholds);
//      terms are f64, reduced per block and added with f64 atomics;
//   3. NaN when only one class is present (the reference's early return).
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "../../include/adipose_hip.h"

namespace {

constexpr int TPB = 256;

__global__ void auc_prep_kernel(size_t n, const float* __restrict__ pred, const float* __restrict__ truth,
                                uint32_t* __restrict__ key, uint32_t* __restrict__ lab) {
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    uint32_t u = __float_as_uint(pred[i]);
    if (u == 0x80000000u) u = 0u;                       // -0 scores tie with +0
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);   // IEEE order -> unsigned order
    key[i] = u;
    lab[i] = truth[i] > 0.5f ? 1u : 0u;
  }
}

__global__ void auc_start_kernel(size_t n, const uint32_t* __restrict__ key, uint32_t* __restrict__ start) {
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
    start[i] = (i == 0 || key[i] != key[i - 1]) ? (uint32_t)i : 0u;
}

__global__ void auc_group_kernel(size_t n, const uint32_t* __restrict__ key, const uint32_t* __restrict__ cpos,
                                 const uint32_t* __restrict__ start, double* __restrict__ acc) {
  const double P = (double)cpos[n - 1];
  double roc = 0.0, ap = 0.0;
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    if (i + 1 < n && key[i] == key[i + 1]) continue;   // not the last rank of its score group
    const size_t s = start[i];
    const double before = s ? (double)cpos[s - 1] : 0.0;
    const double pos = (double)cpos[i] - before, cnt = (double)(i - s + 1), neg = cnt - pos;
    roc += pos * ((double)s - before + 0.5 * neg);
    ap += pos * ((P - before) / (double)(n - s));
  }
  __shared__ double r0[TPB / 64], r1[TPB / 64];
  for (int o = 32; o > 0; o >>= 1) {
    roc += __shfl_xor(roc, o, 64);
    ap += __shfl_xor(ap, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    r0[threadIdx.x >> 6] = roc;
    r1[threadIdx.x >> 6] = ap;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < TPB / 64; ++w) { a += r0[w]; b += r1[w]; }
    atomicAdd(acc, a);
    atomicAdd(acc + 1, b);
  }
}

__global__ void auc_final_kernel(size_t n, const uint32_t* __restrict__ cpos, const double* __restrict__ acc,
                                 double* __restrict__ out) {
  const double P = (double)cpos[n - 1], N = (double)n - P;
  const bool ok = P > 0.0 && N > 0.0;
  out[0] = ok ? acc[0] / (P * N) : __builtin_nan("");
  out[1] = ok ? acc[1] / P : __builtin_nan("");
}

}  // namespace

extern "C" int adp_auc_metrics(size_t n, const float* pred, const float* truth, double* out, adp_stream_t st) {
  ADP_REQUIRE(pred && truth && out && n > 0 && n < (size_t)UINT32_MAX, "adp_auc_metrics: 0 < n < 2^32 pixels");
  hipStream_t s = (hipStream_t)st;
  size_t sort_b = 0, sum_b = 0, max_b = 0;
  uint32_t* nul = nullptr;
  ADP_REQUIRE(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, nul, nul, nul, nul, (int)n, 0, 32, s) == hipSuccess &&
                  hipcub::DeviceScan::InclusiveSum(nullptr, sum_b, nul, nul, (int)n, s) == hipSuccess &&
                  hipcub::DeviceScan::InclusiveScan(nullptr, max_b, nul, nul, hipcub::Max(), (int)n, s) == hipSuccess,
              "adp_auc_metrics: temporary-storage query failed");
  const size_t tmp_b = (std::max(sort_b, std::max(sum_b, max_b)) + 255) / 256 * 256;
  const size_t arr = (n * 4 + 255) / 256 * 256;
  char* w = static_cast<char*>(adp::scratch(2, 6 * arr + tmp_b + 256));
  if (!w) return -2;
  uint32_t* key_in = reinterpret_cast<uint32_t*>(w);
  uint32_t* key_out = reinterpret_cast<uint32_t*>(w + arr);
  uint32_t* lab_in = reinterpret_cast<uint32_t*>(w + 2 * arr);
  uint32_t* lab_out = reinterpret_cast<uint32_t*>(w + 3 * arr);
  uint32_t* cpos = reinterpret_cast<uint32_t*>(w + 4 * arr);
  uint32_t* start = reinterpret_cast<uint32_t*>(w + 5 * arr);
  double* acc = reinterpret_cast<double*>(w + 6 * arr);
  void* tmp = w + 6 * arr + 256;
  const int grid = (int)std::min<size_t>((n + TPB - 1) / TPB, 4096);
  hipLaunchKernelGGL(auc_prep_kernel, dim3(grid), dim3(TPB), 0, s, n, pred, truth, key_in, lab_in);
  ADP_REQUIRE(hipcub::DeviceRadixSort::SortPairs(tmp, sort_b, key_in, key_out, lab_in, lab_out, (int)n, 0, 32, s) ==
                  hipSuccess, "adp_auc_metrics: radix sort failed");
  ADP_REQUIRE(hipcub::DeviceScan::InclusiveSum(tmp, sum_b, lab_out, cpos, (int)n, s) == hipSuccess,
              "adp_auc_metrics: scan failed");
  hipLaunchKernelGGL(auc_start_kernel, dim3(grid), dim3(TPB), 0, s, n, key_out, lab_in);   // sort inputs are free
  ADP_REQUIRE(hipcub::DeviceScan::InclusiveScan(tmp, max_b, lab_in, start, hipcub::Max(), (int)n, s) == hipSuccess,
              "adp_auc_metrics: max-scan failed");
  ADP_REQUIRE(hipMemsetAsync(acc, 0, 2 * sizeof(double), s) == hipSuccess, "adp_auc_metrics: memset failed");
  hipLaunchKernelGGL(auc_group_kernel, dim3(grid), dim3(TPB), 0, s, n, key_out, cpos, start, acc);
  hipLaunchKernelGGL(auc_final_kernel, dim3(1), dim3(1), 0, s, n, cpos, acc, out);
  return adp::check_launch("adp_auc_metrics");
}
