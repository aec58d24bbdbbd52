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

#define CL_OK(x)              \
  do {                        \
    const int r_ = (x);       \
    if (r_ != 0) return r_;   \
  } while (0)

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

// ---------------------------------------------------------------------------------------------------
// Boundary metrics (full_evaluation_enhanced.py:788-844): exact Euclidean distance transforms of ~pred_bin
// and ~true_bin (scipy.ndimage.distance_transform_edt with sampling (sy, sx)) by the separable
// Felzenszwalb-Huttenlocher algorithm -- per column the distance to the nearest set pixel (two sweeps),
// per row the lower envelope of the sampled parabolas, f64 throughout -- the surfaces
// bin & ~binary_erosion(bin) (skimage: cross footprint, pixels outside the image count as set), the
// distances of each map sampled at its own surface (the reference's pairing), then np.percentile(95)
// (linear, numpy's lerp) and the mean of the concatenated samples.
namespace {

constexpr double EDT_INF = __builtin_huge_val();

// g[y][x] = (sy * distance along the column to the nearest pixel with src > thr)^2, or inf
__global__ void edt_cols_kernel(int H, int W, const float* __restrict__ src, float thr, double sy,
                                double* __restrict__ g) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= W) return;
  int last = -1;
  for (int y = 0; y < H; ++y) {
    if (src[(size_t)y * W + x] > thr) last = y;
    g[(size_t)y * W + x] = last >= 0 ? (double)(y - last) : EDT_INF;
  }
  int next = -1;
  for (int y = H - 1; y >= 0; --y) {
    const size_t i = (size_t)y * W + x;
    if (src[i] > thr) next = y;
    double d = g[i];
    if (next >= 0) d = fmin(d, (double)(next - y));
    g[i] = d == EDT_INF ? EDT_INF : (sy * d) * (sy * d);
  }
}

// dist[y][x] = sqrt(min_q sx^2 (x - q)^2 + g[y][q]) (lower envelope of parabolas, one thread per row)
__global__ void edt_rows_kernel(int H, int W, const double* __restrict__ g, double sx, int* __restrict__ v,
                                double* __restrict__ z, double* __restrict__ dist) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= H) return;
  const double* f = g + (size_t)y * W;
  int* vv = v + (size_t)y * W;
  double* zz = z + (size_t)y * (W + 1);
  double* out = dist + (size_t)y * W;
  const double s2 = sx * sx;
  int k = -1;
  for (int q = 0; q < W; ++q) {
    const double fq = f[q];
    if (fq == EDT_INF) continue;
    if (k < 0) {
      k = 0;
      vv[0] = q;
      zz[0] = -EDT_INF;
      zz[1] = EDT_INF;
      continue;
    }
    double s;
    while (true) {
      const int p = vv[k];
      s = ((fq + s2 * (double)q * q) - (f[p] + s2 * (double)p * p)) / (2.0 * s2 * (double)(q - p));
      if (s <= zz[k]) --k;
      else break;
    }
    ++k;
    vv[k] = q;
    zz[k] = s;
    zz[k + 1] = EDT_INF;
  }
  if (k < 0) {
    for (int x = 0; x < W; ++x) out[x] = EDT_INF;
    return;
  }
  int j = 0;
  for (int x = 0; x < W; ++x) {
    while (zz[j + 1] < (double)x) ++j;
    const double dx = (double)(x - vv[j]);
    out[x] = sqrt(s2 * dx * dx + f[vv[j]]);
  }
}

ADP_DEV bool bin_at(const float* m, int H, int W, int y, int x, float thr) {
  return (y < 0 || y >= H || x < 0 || x >= W) ? true : m[(size_t)y * W + x] > thr;   // border counts as set
}

// counts: [0] pred pixels, [1] true pixels, [2] samples appended (pred surface then true surface)
__global__ void surface_kernel(int H, int W, const float* __restrict__ pred, const float* __restrict__ truth,
                               float thr, const double* __restrict__ dtp, const double* __restrict__ dtt,
                               double* __restrict__ vals, unsigned* __restrict__ cnt) {
  const size_t n = (size_t)H * W;
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int y = (int)(i / W), x = (int)(i - (size_t)y * W);
    const bool pb = pred[i] > thr, tb = truth[i] > 0.5f;
    if (pb) atomicAdd(cnt, 1u);
    if (tb) atomicAdd(cnt + 1, 1u);
    if (pb && !(bin_at(pred, H, W, y - 1, x, thr) && bin_at(pred, H, W, y + 1, x, thr) &&
                bin_at(pred, H, W, y, x - 1, thr) && bin_at(pred, H, W, y, x + 1, thr))) {
      vals[atomicAdd(cnt + 2, 1u)] = dtp[i];
      atomicAdd(cnt + 3, 1u);
    }
    if (tb && !(bin_at(truth, H, W, y - 1, x, 0.5f) && bin_at(truth, H, W, y + 1, x, 0.5f) &&
                bin_at(truth, H, W, y, x - 1, 0.5f) && bin_at(truth, H, W, y, x + 1, 0.5f))) {
      vals[atomicAdd(cnt + 2, 1u)] = dtt[i];
      atomicAdd(cnt + 4, 1u);
    }
  }
}

__global__ void sum_kernel(size_t n, const double* __restrict__ v, double* __restrict__ acc) {
  double s = 0.0;
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) s += v[i];
  __shared__ double r[TPB / 64];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int w = 0; w < TPB / 64; ++w) a += r[w];
    atomicAdd(acc, a);
  }
}

}  // namespace

extern "C" int adp_distance_transform(int H, int W, const float* src, float thr, double sy, double sx, double* dist,
                                      adp_stream_t st) {
  ADP_REQUIRE(H > 0 && W > 0 && src && dist && sy > 0 && sx > 0, "adp_distance_transform: bad arguments");
  hipStream_t s = (hipStream_t)st;
  const size_t n = (size_t)H * W;
  char* w = static_cast<char*>(adp::scratch(3, n * 8 + n * 4 + (size_t)H * (W + 1) * 8 + 512));
  if (!w) return -2;
  double* g = reinterpret_cast<double*>(w);
  double* z = reinterpret_cast<double*>(w + n * 8);
  int* v = reinterpret_cast<int*>(w + n * 8 + (size_t)H * (W + 1) * 8);
  hipLaunchKernelGGL(edt_cols_kernel, dim3((W + 63) / 64), dim3(64), 0, s, H, W, src, thr, sy, g);
  hipLaunchKernelGGL(edt_rows_kernel, dim3((H + 63) / 64), dim3(64), 0, s, H, W, g, sx, v, z, dist);
  return adp::check_launch("adp_distance_transform");
}

extern "C" int adp_boundary_metrics(int H, int W, const float* pred, const float* truth, float thr, double sy,
                                    double sx, double* out, adp_stream_t st) {
  ADP_REQUIRE(H > 0 && W > 0 && pred && truth && out && sy > 0 && sx > 0, "adp_boundary_metrics: bad arguments");
  hipStream_t s = (hipStream_t)st;
  const size_t n = (size_t)H * W;
  // own workspace (slot 4): dt_pred, dt_true, samples (<= 2n), counters; the EDTs use slot 3
  char* w = static_cast<char*>(adp::scratch(4, 4 * n * 8 + 512));
  if (!w) return -2;
  double* dtp = reinterpret_cast<double*>(w);
  double* dtt = dtp + n;
  double* vals = dtt + n;
  unsigned* cnt = reinterpret_cast<unsigned*>(w + 4 * n * 8);
  double* acc = reinterpret_cast<double*>(w + 4 * n * 8 + 256);
  CL_OK(adp_distance_transform(H, W, pred, thr, sy, sx, dtp, st));
  CL_OK(adp_distance_transform(H, W, truth, 0.5f, sy, sx, dtt, st));
  ADP_REQUIRE(hipMemsetAsync(cnt, 0, 256 + 8, s) == hipSuccess, "adp_boundary_metrics: memset failed");
  const int grid = (int)std::min<size_t>((n + TPB - 1) / TPB, 4096);
  hipLaunchKernelGGL(surface_kernel, dim3(grid), dim3(TPB), 0, s, H, W, pred, truth, thr, dtp, dtt, vals, cnt);
  unsigned hc[5];
  ADP_REQUIRE(hipMemcpyAsync(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess, "adp_boundary_metrics: count read-back failed");
  if (hc[0] == 0 && hc[1] == 0) { out[0] = out[1] = 0.0; return 0; }
  if (hc[0] == 0 || hc[1] == 0 || hc[3] == 0 || hc[4] == 0) { out[0] = out[1] = EDT_INF; return 0; }
  const size_t m = hc[2];
  // sort the samples (np.percentile) and sum them (np.mean)
  size_t sort_b = 0;
  ADP_REQUIRE(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_b, (double*)nullptr, (double*)nullptr, (int)m, 0, 64, s) ==
                  hipSuccess, "adp_boundary_metrics: sort query failed");
  char* w2 = static_cast<char*>(adp::scratch(5, m * 8 + sort_b + 512));
  if (!w2) return -2;
  double* sorted = reinterpret_cast<double*>(w2);
  void* tmp = w2 + (m * 8 + 255) / 256 * 256;
  ADP_REQUIRE(hipcub::DeviceRadixSort::SortKeys(tmp, sort_b, vals, sorted, (int)m, 0, 64, s) == hipSuccess,
              "adp_boundary_metrics: sort failed");
  ADP_REQUIRE(hipMemsetAsync(acc, 0, 8, s) == hipSuccess, "adp_boundary_metrics: memset failed");
  hipLaunchKernelGGL(sum_kernel, dim3((int)std::min<size_t>((m + TPB - 1) / TPB, 1024)), dim3(TPB), 0, s, m, sorted, acc);
  const double idx = 0.95 * (double)(m - 1);
  const size_t lo = (size_t)idx, hi = std::min(lo + 1, m - 1);
  const double t = idx - (double)lo;
  double a = 0.0, b = 0.0, sum = 0.0;
  ADP_REQUIRE(hipMemcpyAsync(&a, sorted + lo, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipMemcpyAsync(&b, sorted + hi, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipMemcpyAsync(&sum, acc, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess, "adp_boundary_metrics: read-back failed");
  const double d = b - a;   // numpy's _lerp
  out[0] = t >= 0.5 ? b - d * (1.0 - t) : a + d * t;
  out[1] = sum / (double)m;
  return adp::check_launch("adp_boundary_metrics");
}
