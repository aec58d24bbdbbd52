// The rest of the src/utils/model.py loss / metric surface on the GPU (weighted losses :103-153, metric
// helpers :21-91). None of these is on the reference's training step (compile_model :780-879 never selects
// them); they are part of the loss surface the drop-in must expose.
//
//   adp_border_weight       weighted_dice_loss / weighted_bce_dice_loss's weight map (model.py:104-116,
//                           :140-151): y -> expand_dims(y, 0) -> K.pool2d(21x21, stride 1, 'same', 'avg')
//                           -> border = (0.005 < avg < 0.995) -> weight = 1 + 2*border, sum(weight) for the
//                           renormalisation. The expanded (1, B, H, W) tensor is channels_last, so the pool
//                           window runs over (B, H) with W as the channel axis (the reference's quirk), and
//                           TF's 'SAME' average excludes the padding from the count.
//   adp_weighted_loss_stats the five sums of weighted_dice_coeff (:120-125) and weighted_bce_loss (:127-136)
//                           with w = weight * (w0 / w1) (the renormalisation, f32 as Keras does it)
//   adp_weighted_loss_grad  d/dp of  wbce * weighted_bce_loss + wdice * (1 - weighted_dice_coeff)
//   adp_value_stats         K.mean / K.min / K.max / K.std (population) of a tensor: act_* / mean_diff
//   adp_onehot_counts       argmax / argmin over the last axis of y_true and y_pred (first occurrence) and the
//                           counts tru_pos / fls_pos / tru_neg / fls_neg / precision_onehot / recall_onehot use
//
// HBM-bound grid-stride passes; sums in f64.
#include <climits>

#include "common.h"
#include "../../include/adipose_hip.h"

namespace {

constexpr int TPB = 256;
constexpr float KEPS = 1e-7f;   // keras.backend.epsilon()

ADP_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sums of NV doubles, thread 0 adds them into out[0..NV) (f64 atomics)
template <int NV>
ADP_DEV void block_add(double (&v)[NV], double* out) {
  __shared__ double red[TPB / 64][NV];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum_d(v[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wv][k] = v[k];
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < TPB / 64; ++w) s += red[w][threadIdx.x];
    atomicAdd(out + threadIdx.x, s);
  }
}

int grid_for(size_t n) { return (int)std::max<size_t>(1, std::min<size_t>((n + TPB - 1) / TPB, 4096)); }

// pass 1: column sums over the H window (per b, w): tmp[b][h][w] = sum_{|h'-h| <= r, 0 <= h' < H} y[b][h'][w]
__global__ void border_hsum_kernel(int B, int H, int W, int r, const float* __restrict__ y, float* __restrict__ tmp) {
  const size_t n = (size_t)B * H * W;
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int w = (int)(i % W);
    const size_t bh = i / W;
    const int h = (int)(bh % H), b = (int)(bh / H);
    const int h0 = max(h - r, 0), h1 = min(h + r, H - 1);
    const float* col = y + (size_t)b * H * W + w;
    float s = 0.f;
    for (int hh = h0; hh <= h1; ++hh) s += col[(size_t)hh * W];
    tmp[i] = s;
  }
}

// pass 2: sum over the B window, average over the valid window (TF 'SAME' avg-pool excludes the padding),
// border band -> weight = 1 + 2 * border; wsum[0] += sum(weight)
__global__ void border_weight_kernel(int B, int H, int W, int r, const float* __restrict__ tmp,
                                     float* __restrict__ weight, double* __restrict__ wsum) {
  const size_t n = (size_t)B * H * W, plane = (size_t)H * W;
  double acc[1] = {0.0};
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const size_t hw = i % plane;
    const int b = (int)(i / plane), h = (int)(hw / W);
    const int b0 = max(b - r, 0), b1 = min(b + r, B - 1);
    const int h0 = max(h - r, 0), h1 = min(h + r, H - 1);
    float s = 0.f;
    for (int bb = b0; bb <= b1; ++bb) s += tmp[(size_t)bb * plane + hw];
    const float avg = s / (float)((b1 - b0 + 1) * (h1 - h0 + 1));
    const float border = (avg > 0.005f && avg < 0.995f) ? 1.f : 0.f;
    const float wt = 1.f + border * 2.f;
    weight[i] = wt;
    acc[0] += (double)wt;
  }
  block_add<1>(acc, wsum);
}

// w0 / w1 of the renormalisation, in f32 (w0 = K.sum(ones) = n, w1 = K.sum(weight))
ADP_DEV float renorm(size_t n, const double* wsum) { return (float)n / (float)wsum[0]; }

struct WTerms {
  float w, y, pc, l;   // renormalised weight, label, clipped p, logit of the clipped p
};
ADP_DEV WTerms wterms(float wt, float ratio, float yv, float pv) {
  WTerms t;
  t.w = wt * ratio;
  t.y = yv;
  t.pc = fminf(fmaxf(pv, KEPS), 1.f - KEPS);
  t.l = logf(t.pc / (1.f - t.pc));
  return t;
}
// weighted_bce_loss's per-element term (tf.nn.weighted_cross_entropy_with_logits form, model.py:134-135)
ADP_DEV float wbce_term(const WTerms& t) {
  return (1.f - t.y) * t.l + (1.f + (t.w - 1.f) * t.y) * (logf(1.f + expf(-fabsf(t.l))) + fmaxf(-t.l, 0.f));
}

// stats: {sum w^2 y p, sum w^2 y, sum w^2 p, sum bce_term, sum w}
__global__ void wloss_stats_kernel(size_t n, const float* __restrict__ y, const float* __restrict__ p,
                                   const float* __restrict__ weight, const double* __restrict__ wsum,
                                   double* __restrict__ stats) {
  const float ratio = renorm(n, wsum);
  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const float pv = p[i];
    const WTerms t = wterms(weight[i], ratio, y[i], pv);
    const float w2 = t.w * t.w;
    acc[0] += (double)(w2 * (t.y * pv));
    acc[1] += (double)(w2 * t.y);
    acc[2] += (double)(w2 * pv);
    acc[3] += (double)wbce_term(t);
    acc[4] += (double)t.w;
  }
  block_add<5>(acc, stats);
}

// dp = wbce * d(sum bce / sum w)/dp + wdice * d(1 - (2 S_wyp + 1) / (S_wy + S_wp + 1))/dp, TF's subgradients:
// clip passes the gradient for KEPS <= p <= 1 - KEPS, d|l|/dl = sign(l) (0 at 0), d max(-l, 0)/dl = -1 for l <= 0
__global__ void wloss_grad_kernel(size_t n, const float* __restrict__ y, const float* __restrict__ p,
                                  const float* __restrict__ weight, const double* __restrict__ wsum,
                                  const double* __restrict__ stats, float wbce, float wdice, float* __restrict__ dp) {
  const float ratio = renorm(n, wsum);
  const double num = 2.0 * stats[0] + 1.0, den = stats[1] + stats[2] + 1.0;
  const float ddice_a = (float)(num / (den * den)), ddice_b = (float)(2.0 / den);
  const float inv_sw = (float)(1.0 / stats[4]);
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const float pv = p[i];
    const WTerms t = wterms(weight[i], ratio, y[i], pv);
    const float w2 = t.w * t.w;
    float g = wdice * w2 * (ddice_a - ddice_b * t.y);
    if (wbce != 0.f && pv >= KEPS && pv <= 1.f - KEPS) {
      const float e = expf(-fabsf(t.l));
      const float sgn = t.l > 0.f ? 1.f : (t.l < 0.f ? -1.f : 0.f);
      const float dsp = -sgn * e / (1.f + e) - (t.l <= 0.f ? 1.f : 0.f);   // d/dl of log(1+e^-|l|) + max(-l,0)
      const float dl = (1.f - t.y) + (1.f + (t.w - 1.f) * t.y) * dsp;
      g += wbce * inv_sw * dl / (t.pc * (1.f - t.pc));
    }
    dp[i] = g;
  }
}

// Chan-merge statistics: count, mean, M2 (sum of squared deviations), min, max (f64)
struct Moments {
  double n, mean, m2, mn, mx;
};
ADP_DEV Moments merge(const Moments& a, const Moments& b) {
  if (a.n == 0.0) return b;
  if (b.n == 0.0) return a;
  Moments r;
  r.n = a.n + b.n;
  const double d = b.mean - a.mean;
  r.mean = a.mean + d * (b.n / r.n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / r.n);
  r.mn = fmin(a.mn, b.mn);
  r.mx = fmax(a.mx, b.mx);
  return r;
}
ADP_DEV Moments shfl_moments(const Moments& m, int o) {
  return Moments{__shfl_xor(m.n, o, 64), __shfl_xor(m.mean, o, 64), __shfl_xor(m.m2, o, 64),
                 __shfl_xor(m.mn, o, 64), __shfl_xor(m.mx, o, 64)};
}
ADP_DEV Moments block_moments(Moments m) {
  __shared__ Moments red[TPB / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = merge(m, shfl_moments(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  Moments r = red[0];
  for (int w = 1; w < TPB / 64; ++w) r = merge(r, red[w]);
  return r;
}

__global__ void moments_kernel(size_t n, const float* __restrict__ x, Moments* __restrict__ part) {
  Moments m{0.0, 0.0, 0.0, INFINITY, -INFINITY};
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const double v = (double)x[i];
    m.n += 1.0;
    const double d = v - m.mean;
    m.mean += d / m.n;
    m.m2 += d * (v - m.mean);
    m.mn = fmin(m.mn, v);
    m.mx = fmax(m.mx, v);
  }
  const Moments r = block_moments(m);
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

__global__ void moments_final_kernel(int nparts, const Moments* __restrict__ part, double* __restrict__ out) {
  Moments m{0.0, 0.0, 0.0, INFINITY, -INFINITY};
  for (int i = threadIdx.x; i < nparts; i += TPB) m = merge(m, part[i]);
  const Moments r = block_moments(m);
  if (threadIdx.x == 0) {
    out[0] = r.mean;
    out[1] = r.mn;
    out[2] = r.mx;
    out[3] = r.n > 0.0 ? sqrt(r.m2 / r.n) : 0.0;   // K.std: population standard deviation
  }
}

// one wave per row of W values: first-occurrence argmax / argmin of y and p, then the per-row terms;
// out (int64): {sum at*ap, sum clip(ap-at,0,1), sum it*ip, sum clip(ip-it,0,1), #(at*ap >= 1), #(ap >= 1), #(at >= 1)}
ADP_DEV void wave_arg(float v, int i, float& bv, int& bi, bool want_max) {
  bv = v;
  bi = i;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    const bool take = want_max ? (ov > bv || (ov == bv && oi < bi)) : (ov < bv || (ov == bv && oi < bi));
    if (take) { bv = ov; bi = oi; }
  }
}

__global__ void onehot_counts_kernel(int rows, int W, const float* __restrict__ y, const float* __restrict__ p,
                                     unsigned long long* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wid = (blockIdx.x * TPB + threadIdx.x) >> 6, nw = (gridDim.x * TPB) >> 6;
  unsigned long long c[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int r = wid; r < rows; r += nw) {
    const float* yr = y + (size_t)r * W;
    const float* pr = p + (size_t)r * W;
    float ymx = -INFINITY, ymn = INFINITY, pmx = -INFINITY, pmn = INFINITY;
    int yai = INT_MAX, yii = INT_MAX, pai = INT_MAX, pii = INT_MAX;
    for (int j = lane; j < W; j += 64) {   // per lane: first occurrence (strictly better replaces)
      const float yv = yr[j], pv = pr[j];
      if (yv > ymx) { ymx = yv; yai = j; }
      if (yv < ymn) { ymn = yv; yii = j; }
      if (pv > pmx) { pmx = pv; pai = j; }
      if (pv < pmn) { pmn = pv; pii = j; }
    }
    float bv;
    int at, it, ap, ip;
    wave_arg(ymx, yai, bv, at, true);
    wave_arg(ymn, yii, bv, it, false);
    wave_arg(pmx, pai, bv, ap, true);
    wave_arg(pmn, pii, bv, ip, false);
    if (lane == 0) {
      c[0] += (unsigned long long)((long long)at * ap);
      c[1] += ap - at > 0 ? 1ull : 0ull;
      c[2] += (unsigned long long)((long long)it * ip);
      c[3] += ip - it > 0 ? 1ull : 0ull;
      c[4] += (long long)at * ap >= 1 ? 1ull : 0ull;
      c[5] += ap >= 1 ? 1ull : 0ull;
      c[6] += at >= 1 ? 1ull : 0ull;
    }
  }
  if (lane == 0)
    for (int k = 0; k < 7; ++k)
      if (c[k]) atomicAdd(out + k, c[k]);
}

}  // namespace

extern "C" int adp_border_weight(int B, int H, int W, int ksize, const float* y, float* tmp, float* weight,
                                 double* wsum, adp_stream_t st) {
  ADP_REQUIRE(B > 0 && H > 0 && W > 0 && ksize > 0 && ksize % 2 == 1 && y && tmp && weight && wsum,
              "adp_border_weight: positive B, H, W, odd ksize and every buffer");
  hipStream_t s = (hipStream_t)st;
  const size_t n = (size_t)B * H * W;
  const int r = ksize / 2;
  hipLaunchKernelGGL(border_hsum_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, B, H, W, r, y, tmp);
  hipLaunchKernelGGL(border_weight_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, B, H, W, r, tmp, weight, wsum);
  return adp::check_launch("adp_border_weight");
}

extern "C" int adp_weighted_loss_stats(size_t n, const float* y, const float* p, const float* weight,
                                       const double* wsum, double* stats, adp_stream_t st) {
  ADP_REQUIRE(n > 0 && y && p && weight && wsum && stats, "adp_weighted_loss_stats: null argument");
  hipLaunchKernelGGL(wloss_stats_kernel, dim3(grid_for(n)), dim3(TPB), 0, (hipStream_t)st, n, y, p, weight, wsum,
                     stats);
  return adp::check_launch("adp_weighted_loss_stats");
}

extern "C" int adp_weighted_loss_grad(size_t n, const float* y, const float* p, const float* weight,
                                      const double* wsum, const double* stats, float wbce, float wdice, float* dp,
                                      adp_stream_t st) {
  ADP_REQUIRE(n > 0 && y && p && weight && wsum && stats && dp, "adp_weighted_loss_grad: null argument");
  hipLaunchKernelGGL(wloss_grad_kernel, dim3(grid_for(n)), dim3(TPB), 0, (hipStream_t)st, n, y, p, weight, wsum,
                     stats, wbce, wdice, dp);
  return adp::check_launch("adp_weighted_loss_grad");
}

extern "C" int adp_value_stats(size_t n, const float* x, void* work, double* out, adp_stream_t st) {
  ADP_REQUIRE(n > 0 && x && work && out, "adp_value_stats: null argument");
  hipStream_t s = (hipStream_t)st;
  const int parts = std::min(grid_for(n), 1024);
  hipLaunchKernelGGL(moments_kernel, dim3(parts), dim3(TPB), 0, s, n, x, static_cast<Moments*>(work));
  hipLaunchKernelGGL(moments_final_kernel, dim3(1), dim3(TPB), 0, s, parts, static_cast<const Moments*>(work), out);
  return adp::check_launch("adp_value_stats");
}

extern "C" int adp_onehot_counts(int rows, int W, const float* y, const float* p, unsigned long long* out,
                                 adp_stream_t st) {
  ADP_REQUIRE(rows > 0 && W > 0 && y && p && out, "adp_onehot_counts: positive rows, W and every buffer");
  const int blocks = std::max(1, std::min((rows + TPB / 64 - 1) / (TPB / 64), 2048));
  hipLaunchKernelGGL(onehot_counts_kernel, dim3(blocks), dim3(TPB), 0, (hipStream_t)st, rows, W, y, p, out);
  return adp::check_launch("adp_onehot_counts");
}
