// Bandwidth-bound kernels of the U-Net step: weight repacking, 2x2 max-pool (+grad), nearest
// upsample grad, residual-add + ReLU-mask, BatchNorm statistics/backward, Adam, EMA.
// Every activation kernel moves 8-channel groups (16 B bf16 / 32 B f32 per lane).
//   MaxPooling2D((2,2),strides=(2,2))      Segmentation/train_adipose_unet_v3.py:670,674,678
//   UpSampling2D((2,2)) gradient            :691,698,705
//   Adam / AdamW (Keras defaults)           :800-806
//   EMACallback update (ema = d*ema+(1-d)w) :455-459
#include "common.h"
#include "../../include/adipose_hip.h"
#include <map>
#include <mutex>

namespace {

constexpr int TPB = 256;
inline int nblk(size_t n, int cap = 8192) {
  size_t b = (n + TPB - 1) / TPB;
  return (int)(b < (size_t)cap ? (b ? b : 1) : cap);
}

// replica of this block in the BatchNorm accumulator scratch (see adp::stat_scratch)
ADP_DEV double* stat_replica(double* scratch, unsigned block) {
  return scratch + (size_t)(block & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
}

// ------------------------------------------------------------------------------ repacking
// mode 0: dst[r][k] = src[r][k]; mode 1/2: dst[ci][t*Nout + co] = src[co][(taps-1-t)*Cin_s + ci]
template <typename To>
__global__ void pack_kernel(int mode, int taps, int Cin_s, int Nout, const float* src, int skp,
                            To* dst, int rows, int dkp) {
  size_t total = (size_t)rows * dkp;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    int r = (int)(i / dkp), k = (int)(i - (size_t)r * dkp);
    float v = 0.f;
    if (mode == 0) {
      v = k < skp ? src[(size_t)r * skp + k] : 0.f;
    } else if (r < Cin_s && k < taps * Nout) {
      int t = k / Nout, co = k - t * Nout;
      v = src[(size_t)co * skp + (size_t)(taps - 1 - t) * Cin_s + r];
    }
    dst[i] = from_f<To>(v);
  }
}

// Batched data-gradient repack (modes 1/2 of pack_kernel for many layers in one launch): dst tiles of
// 64 rows (ci) x 64 columns (k = t * Nout + co) are gathered through LDS so that both the source reads
// (along ci) and the destination writes (along k) are coalesced; pad rows / columns are written as 0.
struct PackJobs {
  adp_pack_job j[ADP_PACK_MAX_JOBS];
  int tile0[ADP_PACK_MAX_JOBS + 1];   // prefix sums of 64x64 destination tiles
  int n;
};

template <typename To>
__global__ __launch_bounds__(256) void pack_t_kernel(PackJobs P) {
  __shared__ float tile[64][65];
  int jb = 0;
  while (jb + 1 < P.n && (int)blockIdx.x >= P.tile0[jb + 1]) ++jb;
  const adp_pack_job& J = P.j[jb];
  const int t_local = blockIdx.x - P.tile0[jb];
  const int ktiles = (J.dst_kpad + 63) / 64;
  const int r0 = (t_local / ktiles) * 64, k0 = (t_local % ktiles) * 64;
  const float* src = J.src;
  const int tid = threadIdx.x, KN = J.taps * J.Nout;
  // load: thread column = ci (coalesced along the source row), 4 k rows per pass
  for (int kk = tid >> 6; kk < 64; kk += 4) {
    const int k = k0 + kk, ci = r0 + (tid & 63);
    float v = 0.f;
    if (k < KN && ci < J.Cin_s) {
      const int t = k / J.Nout, co = k - t * J.Nout;
      v = src[(size_t)co * J.src_kpad + (size_t)(J.taps - 1 - t) * J.Cin_s + ci];
    }
    tile[kk][tid & 63] = v;
  }
  __syncthreads();
  To* dst = reinterpret_cast<To*>(J.dst);
  for (int rr = tid >> 6; rr < 64; rr += 4) {
    const int r = r0 + rr, k = k0 + (tid & 63);
    if (r < J.dst_rows && k < J.dst_kpad) dst[(size_t)r * J.dst_kpad + k] = from_f<To>(tile[tid & 63][rr]);
  }
}

// ------------------------------------------------------------------------------ max-pool
template <typename T>
ADP_DEV void load_bn(Grp<T>& g, const T* p, const float* sc, const float* sh, int c, float* f) {
  grp_load(g, p);
  grp_to_f(g, f);
  if (sc) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[c + j], sh[c + j]), 0.f);
  }
}

// act = relu(z * sc + sh) (bn_apply) and its 2x2 max-pool in one pass: each thread owns a 2x2 pixel
// block x 8 channels (the pool of the stored bf16 values equals the rounded pool of the f32 values:
// rounding is monotone)
template <typename T>
__global__ void bn_apply_pool_kernel(int N, int H, int W, int C, const T* z, const float* sc, const float* sh,
                                     T* act, T* pool) {
  const int Ho = H >> 1, Wo = W >> 1, G = C >> 3;
  size_t total = (size_t)N * Ho * Wo * G;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    const int g = (int)(i % G);
    const size_t pix = i / G;
    const int xo = (int)(pix % Wo);
    const size_t t = pix / Wo;
    const int yo = (int)(t % Ho), n = (int)(t / Ho);
    const size_t b0 = (((size_t)n * H + 2 * yo) * W + 2 * xo) * C + g * 8;
    const size_t off[4] = {0, (size_t)C, (size_t)W * C, (size_t)W * C + C};
    float best[8], f[8];
    Grp<T> gr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      load_bn(gr, z + b0 + off[q], sc, sh, g * 8, f);
      grp_from_f(gr, f);
      grp_store(gr, act + b0 + off[q]);
#pragma unroll
      for (int j = 0; j < 8; ++j) best[j] = (q == 0 || f[j] > best[j]) ? f[j] : best[j];
    }
    grp_from_f(gr, best);
    grp_store(gr, pool + pix * C + g * 8);
  }
}

template <typename T>
__global__ void maxpool_fwd_kernel(int N, int H, int W, int C, const T* src, const float* sc,
                                   const float* sh, T* dst) {
  const int Ho = H >> 1, Wo = W >> 1, G = C >> 3;
  size_t total = (size_t)N * Ho * Wo * G;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    int g = (int)(i % G);
    size_t pix = i / G;
    int xo = (int)(pix % Wo);
    size_t t = pix / Wo;
    int yo = (int)(t % Ho);
    int n = (int)(t / Ho);
    float best[8], f[8];
    Grp<T> gr;
    const T* base = src + (((size_t)n * H + 2 * yo) * W + 2 * xo) * C + g * 8;
    load_bn(gr, base, sc, sh, g * 8, best);
    const size_t off[3] = {(size_t)C, (size_t)W * C, (size_t)W * C + C};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      load_bn(gr, base + off[q], sc, sh, g * 8, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) best[j] = f[j] > best[j] ? f[j] : best[j];
    }
    grp_from_f(gr, best);
    grp_store(gr, dst + pix * C + g * 8);
  }
}

// gradient routed to the first maximum in (0,0),(0,1),(1,0),(1,1) order (TF/cuDNN NHWC argmax)
template <typename T>
__global__ void maxpool_bwd_kernel(int N, int H, int W, int C, const T* src, const float* sc,
                                   const float* sh, const T* dpool, const T* addend, const T* mask,
                                   float mscale, T* dsrc) {
  const int Ho = H >> 1, Wo = W >> 1, G = C >> 3;
  size_t total = (size_t)N * Ho * Wo * G;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    int g = (int)(i % G);
    size_t pix = i / G;
    int xo = (int)(pix % Wo);
    size_t t = pix / Wo;
    int yo = (int)(t % Ho);
    int n = (int)(t / Ho);
    const size_t off[4] = {0, (size_t)C, (size_t)W * C, (size_t)W * C + C};
    const size_t base = (((size_t)n * H + 2 * yo) * W + 2 * xo) * C + g * 8;
    float v[4][8], best[8];
    int arg[8];
    Grp<T> gr;
#pragma unroll
    for (int q = 0; q < 4; ++q) load_bn(gr, src + base + off[q], sc, sh, g * 8, v[q]);
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = v[0][j]; arg[j] = 0; }
#pragma unroll
    for (int q = 1; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[q][j] > best[j]) { best[j] = v[q][j]; arg[j] = q; }
    float dp[8];
    grp_load(gr, dpool + pix * C + g * 8);
    grp_to_f(gr, dp);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float o[8], a[8], mk[8];
      if (addend) { grp_load(gr, addend + base + off[q]); grp_to_f(gr, a); }
      if (mask) { grp_load(gr, mask + base + off[q]); grp_to_f(gr, mk); }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = (arg[j] == q ? dp[j] : 0.f) + (addend ? a[j] : 0.f);
        if (mask) x = mk[j] > 0.f ? x * mscale : 0.f;
        o[j] = x;
      }
      grp_from_f(gr, o);
      grp_store(gr, dsrc + base + off[q]);
    }
  }
}

// unet_bn encoder form of the pool backward, channel-group-stationary (thread -> channel group
// t % G, pooled-pixel lane t / G): dsrc = route(dpool) + addend, with the BatchNorm-backward
// reduction of the layer whose activation relu(z*scale+shift) src is fused in (dbeta += sum db,
// dgamma += sum db*xhat over the STORED dsrc values, db = dsrc * (z*scale+shift > 0)), replacing the
// separate bn_bwd_reduce pass over (dsrc, z). src == nullptr: the argmax is taken over the activation
// recomputed from z exactly as bn_apply / bn_apply_pool stored it (fmaf, fmaxf, round to T: bit-identical
// values, so the same first maximum), which drops one of the four full-resolution streams (src, addend,
// z, dsrc) from the pass.
template <typename T, bool SRC>
__global__ __launch_bounds__(TPB) void maxpool_bwd_bnr_kernel(int N, int H, int W, int C, const T* src, const T* dpool, const T* addend,
                                       T* dsrc, const T* z, const float* sc, const float* sh, const float* mean,
                                       const float* invstd, double* stat) {
  const int G = C >> 3, lanes = TPB / G;
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  const unsigned Ho = H >> 1, Wo = W >> 1, P = (unsigned)N * Ho * Wo;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (pl < lanes) {
    float cs[8], ch[8], mu[8], is[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = g * 8 + j;
      cs[j] = sc[c]; ch[j] = sh[c]; mu[j] = mean[c]; is[j] = invstd[c];
    }
    const size_t off[4] = {0, (size_t)C, (size_t)W * C, (size_t)W * C + C};
    for (unsigned pix = blockIdx.x * lanes + pl; pix < P; pix += gridDim.x * lanes) {
      const unsigned xo = pix % Wo, t = pix / Wo, yo = t % Ho, n = t / Ho;
      const size_t base = (((size_t)n * H + 2 * yo) * W + 2 * xo) * C + g * 8;
      Grp<T> gv[SRC ? 4 : 1], ga[4], gz[4], gp;
      if constexpr (SRC) {
#pragma unroll
        for (int q = 0; q < 4; ++q) grp_load(gv[q], src + base + off[q]);
      }
      grp_load(gp, dpool + (size_t)pix * C + g * 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) grp_load(ga[q], addend + base + off[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) grp_load(gz[q], z + base + off[q]);
      float v[4][8], best[8], dp[8];
      int arg[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (SRC) {
          grp_to_f(gv[q], v[q]);
        } else {   // the stored activation, recomputed
          float f[8];
          grp_to_f(gz[q], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], cs[j], ch[j]), 0.f);
          Grp<T> r;
          grp_from_f(r, f);
          grp_to_f(r, v[q]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[j] = v[0][j]; arg[j] = 0; }
#pragma unroll
      for (int q = 1; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[q][j] > best[j]) { best[j] = v[q][j]; arg[j] = q; }
      grp_to_f(gp, dp);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float o[8], ad[8], zz[8];
        grp_to_f(ga[q], ad);
        grp_to_f(gz[q], zz);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (arg[j] == q ? dp[j] : 0.f) + ad[j];
        Grp<T> go;
        grp_from_f(go, o);
        grp_store(go, dsrc + base + off[q]);
        grp_to_f(go, o);   // the reduction sees the stored (rounded) gradient, as bn_bwd_reduce would
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float db = fmaf(zz[j], cs[j], ch[j]) > 0.f ? o[j] : 0.f;
          s1[j] += db;
          s2[j] += db * (zz[j] - mu[j]) * is[j];
        }
      }
    }
  }
  __shared__ float red[2][TPB * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x * 8 + j] = s1[j];
    red[1][threadIdx.x * 8 + j] = s2[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += TPB) {
    const int gg = c >> 3, j = c & 7;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < lanes; ++l) {
      a += red[0][(l * G + gg) * 8 + j];
      b += red[1][(l * G + gg) * 8 + j];
    }
    double* rep = stat_replica(stat, blockIdx.x);
    atomicAdd(rep + c, (double)a);           // folded into dbeta / dgamma by stat_fold_kernel
    atomicAdd(rep + adp::STAT_CMAX + c, (double)b);
  }
}

template <typename T>
__global__ void upsample_bwd_kernel(int N, int Hs, int Ws, int C, const T* dup, const T* addend,
                                    const T* mask, float mscale, T* dsrc) {
  const int G = C >> 3, Wu = Ws * 2;
  size_t total = (size_t)N * Hs * Ws * G;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    int g = (int)(i % G);
    size_t pix = i / G;
    int xs = (int)(pix % Ws);
    size_t t = pix / Ws;
    int ys = (int)(t % Hs);
    int n = (int)(t / Hs);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, f[8];
    Grp<T> gr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      size_t up = (((size_t)n * 2 * Hs + 2 * ys + (q >> 1)) * Wu + 2 * xs + (q & 1)) * C + g * 8;
      grp_load(gr, dup + up);
      grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    size_t o = pix * C + g * 8;
    if (addend) {
      grp_load(gr, addend + o); grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    if (mask) {
      grp_load(gr, mask + o); grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = f[j] > 0.f ? acc[j] * mscale : 0.f;
    }
    grp_from_f(gr, acc);
    grp_store(gr, dsrc + o);
  }
}

template <typename T>
__global__ void ew_add_mask_kernel(size_t ngrp, const T* a, const T* b, const T* mask, float ms, T* out) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < ngrp; i += (size_t)gridDim.x * TPB) {
    Grp<T> gr;
    float x[8], f[8];
    grp_load(gr, a + i * 8); grp_to_f(gr, x);
    if (b) {
      grp_load(gr, b + i * 8); grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += f[j];
    }
    if (mask) {
      grp_load(gr, mask + i * 8); grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = f[j] > 0.f ? x[j] * ms : 0.f;
    }
    grp_from_f(gr, x);
    grp_store(gr, out + i * 8);
  }
}

template <typename Ti, typename To>
__global__ void cast_kernel(size_t n, const Ti* src, To* dst) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
    dst[i] = from_f<To>(to_f(src[i]));
}

// out = bf16(sum_k src_k) over 8-element groups, the f32 sum taken in source order from 0: the value
// an f32 accumulator zeroed and then accumulated by each producer's epilogue (the bf16-rounded value
// it stored) holds, rounded once (the dilated bottleneck's Add, train_adipose_unet_v3.py:688)
struct SumSrcs { const bf16* p[8]; };
__global__ void sum_bf16_kernel(size_t g, int nsrc, SumSrcs S, bf16* out) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < g; i += (size_t)gridDim.x * TPB) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, f[8];
    for (int k = 0; k < nsrc; ++k) {
      Grp<bf16> gr;
      grp_load(gr, S.p[k] + i * 8);
      grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    Grp<bf16> go;
    grp_from_f(go, acc);
    grp_store(go, out + i * 8);
  }
}

__global__ void fill_kernel(size_t n, float v, float* dst) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) dst[i] = v;
}

// ------------------------------------------------------------------------------ BatchNorm
__global__ void bn_finalize_kernel(int C, float count, const float* sum, const float* sq,
                                   const float* gamma, const float* beta, float eps, float momentum,
                                   float* scale, float* shift, float* mean, float* invstd,
                                   float* rmean, float* rvar) {
  int c = blockIdx.x * TPB + threadIdx.x;
  if (c >= C) return;
  // count < 0: eval mode, (sum, sq) hold the running (mean, var)
  float mu = count > 0.f ? sum[c] / count : sum[c];
  float var = count > 0.f ? fmaxf(sq[c] / count - mu * mu, 0.f) : sq[c];
  float is = rsqrtf(var + eps);
  float sc = gamma[c] * is;
  scale[c] = sc;
  shift[c] = beta[c] - mu * sc;
  mean[c] = mu;
  invstd[c] = is;
  if (rmean && count > 0.f) {
    float unb = count > 1.f ? var * count / (count - 1.f) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
  }
}

// dst{0,1}[c] += sum over the replicas of scratch[r][{0,1}][c]; the replicas are re-zeroed
// block = 64 channels x 4 replica groups of STAT_REPL / 4: a thread sums 16 replicas (and zeroes them),
// the four partial sums meet in LDS (a launch-latency-bound fold: 4x shorter dependent chain). The replicas
// are f64 and every producer adds an f32 partial whose own order is fixed (one wave's or one block's pixels
// in a fixed sequence): f64 addition of those partials in any order agrees to ~1e-16 relative, far below
// the f32 rounding of the result, so the folded sums -- and the BatchNorm scale / shift / mean / invstd and
// dgamma / dbeta made from them -- are the same bits from run to run (f32 atomics in run-dependent order made
// bf16 runs of one network differ by rounding flips: profiles/r03_bf16_bn_nondeterminism.txt)
ADP_DEV void fold_replicas(int C, int c, int rg, double* scratch, double& s0, double& s1) {
  constexpr int RPER = adp::STAT_REPL / 4;
  s0 = 0.0;
  s1 = 0.0;
  if (c >= C) return;
#pragma unroll 4
  for (int r = rg * RPER; r < (rg + 1) * RPER; ++r) {
    double* p = scratch + (size_t)r * 2 * adp::STAT_CMAX + c;
    s0 += p[0];
    s1 += p[adp::STAT_CMAX];
    p[0] = 0.0;
    p[adp::STAT_CMAX] = 0.0;
  }
}
__global__ void stat_fold_kernel(int C, double* scratch, float* dst0, float* dst1) {
  __shared__ double part[2][4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s0, s1;
  fold_replicas(C, c, rg, scratch, s0, s1);
  part[0][rg][cl] = s0;
  part[1][rg][cl] = s1;
  __syncthreads();
  if (rg == 0 && c < C) {
    dst0[c] += (float)((part[0][0][cl] + part[0][1][cl]) + (part[0][2][cl] + part[0][3][cl]));
    if (dst1) dst1[c] += (float)((part[1][0][cl] + part[1][1][cl]) + (part[1][2][cl] + part[1][3][cl]));
  }
}

// stat_fold_kernel + bn_finalize_kernel in one launch: the replica sums are added into sum / sq (and
// re-zeroed), then the BatchNorm scale / shift / mean / invstd (and running statistics) of those sums
__global__ void bn_fold_finalize_kernel(int C, double* scratch, float* sum, float* sq, float count,
                                        const float* gamma, const float* beta, float eps, float momentum,
                                        float* scale, float* shift, float* mean, float* invstd, float* rmean,
                                        float* rvar) {
  __shared__ double part[2][4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s0, s1;
  fold_replicas(C, c, rg, scratch, s0, s1);
  part[0][rg][cl] = s0;
  part[1][rg][cl] = s1;
  __syncthreads();
  if (rg != 0 || c >= C) return;
  const float ts = sum[c] + (float)((part[0][0][cl] + part[0][1][cl]) + (part[0][2][cl] + part[0][3][cl]));
  const float tq = sq[c] + (float)((part[1][0][cl] + part[1][1][cl]) + (part[1][2][cl] + part[1][3][cl]));
  sum[c] = ts;
  sq[c] = tq;
  // = bn_finalize_kernel (training statistics, count > 0)
  const float mu = ts / count;
  const float var = fmaxf(tq / count - mu * mu, 0.f);
  const float is = rsqrtf(var + eps);
  const float g = gamma[c] * is;
  scale[c] = g;
  shift[c] = beta[c] - mu * g;
  mean[c] = mu;
  invstd[c] = is;
  if (rmean) {
    const float unb = count > 1.f ? var * count / (count - 1.f) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
  }
}

// per-channel sums of dBN and dBN*xhat; block = 256 threads as (pixel lane) x (channel group)
template <typename T>
__global__ void bn_bwd_reduce_kernel(size_t M, int C, const T* dA, const T* z, const float* sc,
                                     const float* sh, const float* mean, const float* invstd,
                                     float* dgamma, float* dbeta, double* stat) {
  const int G = C >> 3;
  const int lanes = TPB / G;           // pixels processed per block iteration
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (pl < lanes) {
    for (size_t m = (size_t)blockIdx.x * lanes + pl; m < M; m += (size_t)gridDim.x * lanes) {
      Grp<T> gr;
      float d[8], zz[8];
      grp_load(gr, dA + m * C + g * 8); grp_to_f(gr, d);
      grp_load(gr, z + m * C + g * 8); grp_to_f(gr, zz);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int c = g * 8 + j;
        float a = fmaf(zz[j], sc[c], sh[c]);
        float db = a > 0.f ? d[j] : 0.f;
        s1[j] += db;
        s2[j] += db * (zz[j] - mean[c]) * invstd[c];
      }
    }
  }
  __shared__ float red[2][TPB * 8 / 8 * 8];
  // reduce over pixel lanes with the same channel group through LDS
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x * 8 + j] = s1[j];
    red[1][threadIdx.x * 8 + j] = s2[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += TPB) {
    int gg = c >> 3, j = c & 7;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < lanes; ++l) {
      a += red[0][(l * G + gg) * 8 + j];
      b += red[1][(l * G + gg) * 8 + j];
    }
    double* rep = stat_replica(stat, blockIdx.x);
    atomicAdd(rep + c, (double)a);
    atomicAdd(rep + adp::STAT_CMAX + c, (double)b);
  }
}

// Channel-group-stationary BatchNorm elementwise passes: thread t of a block owns channel group
// g = t % G for its whole life and pixel lane t / G (TPB / G pixels per block row; G | TPB for every
// C <= 2048 that is a power-of-two multiple of 8, otherwise the remainder threads idle), so its
// per-channel coefficients sit in registers and the loop does no integer division. Two pixels per
// iteration (all loads before any store: safe in place); U pixels per thread per iteration.
//   dz = k*db + Q*(z - mean) + R,  k = gamma*invstd, Q = -k*invstd*dgamma/count, R = -k*dbeta/count,
//   db = dA * (z*scale + shift > 0)            (= gamma*invstd*(db - dbeta/n - xhat*dgamma/n))
template <typename T, int U>
__global__ void bn_bwd_apply_kernel(size_t M, int C, const T* dA, const T* z, const float* sc,
                                    const float* sh, const float* mean, const float* invstd,
                                    const float* gamma, const float* dgamma, const float* dbeta,
                                    float inv_count, T* dz) {
  const int G = C >> 3, lanes = TPB / G;
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  if (pl >= lanes) return;
  float s[8], h[8], mu[8], P[8], Q[8], R[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = g * 8 + j;
    const float k = gamma[c] * invstd[c];
    s[j] = sc[c]; h[j] = sh[c]; mu[j] = mean[c];
    P[j] = k;
    Q[j] = -k * invstd[c] * dgamma[c] * inv_count;
    R[j] = -k * dbeta[c] * inv_count;
  }
  auto one = [&](const Grp<T>& gd, const Grp<T>& gz, Grp<T>& go) {
    float d[8], zz[8], o[8];
    grp_to_f(gd, d);
    grp_to_f(gz, zz);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float db = fmaf(zz[j], s[j], h[j]) > 0.f ? d[j] : 0.f;
      o[j] = fmaf(P[j], db, fmaf(Q[j], zz[j] - mu[j], R[j]));
    }
    grp_from_f(go, o);
  };
  const size_t step = (size_t)gridDim.x * lanes;
  size_t m = (size_t)blockIdx.x * lanes + pl;
  for (; m + (U - 1) * step < M; m += U * step) {
    Grp<T> d[U], zz[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      grp_load(d[u], dA + (m + u * step) * C + g * 8);
      grp_load(zz[u], z + (m + u * step) * C + g * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(d[u], zz[u], r[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) grp_store(r[u], dz + (m + u * step) * C + g * 8);
  }
  for (; m < M; m += step) {
    const size_t o0 = m * C + g * 8;
    Grp<T> d0, z0, r0;
    grp_load(d0, dA + o0); grp_load(z0, z + o0);
    one(d0, z0, r0);
    grp_store(r0, dz + o0);
  }
}

// an empty asm that uses the loaded values: every load before it is issued before any math after it
__device__ __forceinline__ void ew_pin(float a, float b, const Grp<bf16>& g) {
  asm volatile("" ::"v"(a), "v"(b), "v"(g.v.x), "v"(g.v.y), "v"(g.v.z), "v"(g.v.w));
}
__device__ __forceinline__ void ew_pin(float a, float b, const Grp<float>& g) {
  asm volatile("" ::"v"(a), "v"(b), "v"(g.v[0].x), "v"(g.v[0].y), "v"(g.v[0].z), "v"(g.v[0].w));
  asm volatile("" ::"v"(g.v[1].x), "v"(g.v[1].y), "v"(g.v[1].z), "v"(g.v[1].w));
}

// adp_bn_bwd_apply of the layer under the sigmoid head with dA recomputed instead of read:
// dA = T(dp * p * (1 - p) * W[c]) (0 for c >= Cin), rounded exactly as adp_head_sigmoid_bwd_bnr stores
// it, so that launch need not store dA (one map write and one read fewer). Same thread layout and
// arithmetic as bn_bwd_apply_kernel; every load of a pass is issued before its arithmetic.
template <typename T, int U>
__global__ void bn_bwd_apply_head_kernel(size_t M, int C, int Cin, const T* z, const float* W, const float* p,
                                         const float* dp, const float* sc, const float* sh, const float* mean,
                                         const float* invstd, const float* gamma, const float* dgamma,
                                         const float* dbeta, float inv_count, T* dz) {
  const int G = C >> 3, lanes = TPB / G;
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  if (pl >= lanes) return;
  float s[8], h[8], mu[8], P[8], Q[8], R[8], wd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = g * 8 + j;
    const float k = gamma[c] * invstd[c];
    s[j] = sc[c]; h[j] = sh[c]; mu[j] = mean[c];
    P[j] = k;
    Q[j] = -k * invstd[c] * dgamma[c] * inv_count;
    R[j] = -k * dbeta[c] * inv_count;
  }
  // head weights as two 16-B loads (Cin % 8 == 0): a per-channel conditional load here made the
  // compiler split the whole coefficient prologue into 64 single-dword loads behind branches (6x slower)
  if (g * 8 < Cin) {
    const float4 w0 = reinterpret_cast<const float4*>(W)[2 * g], w1 = reinterpret_cast<const float4*>(W)[2 * g + 1];
    wd[0] = w0.x; wd[1] = w0.y; wd[2] = w0.z; wd[3] = w0.w;
    wd[4] = w1.x; wd[5] = w1.y; wd[6] = w1.z; wd[7] = w1.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) wd[j] = 0.f;
  }
  auto one = [&](float pm, float dpm, const Grp<T>& gz, Grp<T>& go) {
    const float dl = dpm * pm * (1.f - pm);
    float dv[8], d[8], zz[8], o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dv[j] = dl * wd[j] + 0.f;   // the head backward's expression (no addend)
    Grp<T> gd;
    grp_from_f(gd, dv);
    grp_to_f(gd, d);
    grp_to_f(gz, zz);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float db = fmaf(zz[j], s[j], h[j]) > 0.f ? d[j] : 0.f;
      o[j] = fmaf(P[j], db, fmaf(Q[j], zz[j] - mu[j], R[j]));
    }
    grp_from_f(go, o);
  };
  const size_t step = (size_t)gridDim.x * lanes;
  size_t m = (size_t)blockIdx.x * lanes + pl;
  for (; m + (U - 1) * step < M; m += U * step) {
    Grp<T> zz[U], r[U];
    float pm[U], dpm[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      grp_load(zz[u], z + (m + u * step) * C + g * 8);
      pm[u] = p[m + u * step];
      dpm[u] = dp[m + u * step];
    }
    // pin every load of the pass ahead of the arithmetic (left alone, the compiler sinks the later
    // pixels' loads below the earlier pixels' math: one pixel in flight per wave, 2.2 TB/s)
#pragma unroll
    for (int u = 0; u < U; ++u)
      ew_pin(pm[u], dpm[u], zz[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) one(pm[u], dpm[u], zz[u], r[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) grp_store(r[u], dz + (m + u * step) * C + g * 8);
  }
  for (; m < M; m += step) {
    const size_t o0 = m * C + g * 8;
    Grp<T> z0, r0;
    grp_load(z0, z + o0);
    one(p[m], dp[m], z0, r0);
    grp_store(r0, dz + o0);
  }
}

// a = relu(z*scale + shift): materialised post-BN activation (lets every consumer use LDS-DMA loads)
template <typename T, int U>
__global__ void bn_apply_kernel(size_t M, int C, const T* z, const float* sc, const float* sh, T* out) {
  const int G = C >> 3, lanes = TPB / G;
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  if (pl >= lanes) return;
  float s[8], h[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = sc[g * 8 + j]; h[j] = sh[g * 8 + j]; }
  auto one = [&](Grp<T>& gr) {
    float f[8];
    grp_to_f(gr, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], s[j], h[j]), 0.f);
    grp_from_f(gr, f);
  };
  const size_t step = (size_t)gridDim.x * lanes;
  size_t m = (size_t)blockIdx.x * lanes + pl;
  for (; m + (U - 1) * step < M; m += U * step) {
    Grp<T> a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) grp_load(a[u], z + (m + u * step) * C + g * 8);
#pragma unroll
    for (int u = 0; u < U; ++u) one(a[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) grp_store(a[u], out + (m + u * step) * C + g * 8);
  }
  for (; m < M; m += step) {
    const size_t o0 = m * C + g * 8;
    Grp<T> a0;
    grp_load(a0, z + o0);
    one(a0);
    grp_store(a0, out + o0);
  }
}

// blocks for a channel-group-stationary launch over M pixels, U pixels per thread per iteration
// (grid caps and unrolls measured with tools/bench_ew.py at the unet_bn level shapes: bn_apply
// U = 1 / 64K blocks 5.8-6.0 TB/s at 1024^2x64, bn_bwd_apply U = 2 / 32K blocks 5.6 TB/s)
inline int bn_blocks(size_t M, int C, int U, int cap) {
  const int lanes = TPB / (C / 8);
  const size_t b = (M + (size_t)U * lanes - 1) / ((size_t)U * lanes);
  return (int)std::max<size_t>(1, std::min<size_t>(b, (size_t)adp::option("bn_cap", cap)));
}
// (round 6: default 4 pixels a thread for the BatchNorm apply / backward-apply passes, -0.10 and -0.37 % on the
//  unet_bn step in two round-robin sweeps, profiles/r06x_bn_sweep.log, r06af_option_sweep.log; elementwise, so the
//  values are the same bits at any unroll)
#define BN_UNROLL_SWITCH(U, dflt, ...)                \
  do {                                                \
    const int u_ = adp::option("bn_unroll", dflt);    \
    if (u_ == 4) { constexpr int U = 4; __VA_ARGS__; } \
    else if (u_ == 1) { constexpr int U = 1; __VA_ARGS__; } \
    else { constexpr int U = 2; __VA_ARGS__; }        \
  } while (0)

// ---------------------------------------------------------------------------- fp8 inference path
// per-row (output channel) e4m3 quantisation of the forward weight layout: one block per row
__global__ void pack_fp8_kernel(const float* src, int skp, unsigned char* dst, int dkp, float* scale) {
  const int r = blockIdx.x;
  const float* row = src + (size_t)r * skp;
  float m = 0.f;
  for (int k = threadIdx.x; k < skp; k += TPB) m = fmaxf(m, fabsf(row[k]));
  __shared__ float red[TPB / 64];
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 8, 64));
  m = fmaxf(m, __shfl_xor(m, 4, 64));
  m = fmaxf(m, __shfl_xor(m, 2, 64));
  m = fmaxf(m, __shfl_xor(m, 1, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float amax = 0.f;
#pragma unroll
  for (int w = 0; w < TPB / 64; ++w) amax = fmaxf(amax, red[w]);
  const float sc = amax > 0.f ? amax / FP8_MAX : 1.f;
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) scale[r] = sc;
  for (int k8 = threadIdx.x * 8; k8 < dkp; k8 += TPB * 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = k8 + j < skp ? row[k8 + j] * inv : 0.f;
    *reinterpret_cast<uint2*>(dst + (size_t)r * dkp + k8) = f8x8_from_f(v);
  }
}

template <typename T>
ADP_DEV void load8f(const T* p, float* f) {
  Grp<T> gr;
  grp_load(gr, p);
  grp_to_f(gr, f);
}
ADP_DEV void load8f(const unsigned char* p, float* f) { f8x8_to_f(*reinterpret_cast<const uint2*>(p), f); }

template <typename T>
__global__ void bn_apply_fp8_kernel(size_t M, int C, const T* z, const float* sc, const float* sh,
                                    unsigned char* out) {
  const int G = C >> 3;
  size_t total = M * G;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    const int g = (int)(i % G);
    float f[8];
    load8f(z + i * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[g * 8 + j], sh[g * 8 + j]), 0.f);
    *reinterpret_cast<uint2*>(out + i * 8) = f8x8_from_f(f);
  }
}

template <typename T>
__global__ void maxpool_fwd_fp8_kernel(int N, int H, int W, int C, const T* src, unsigned char* dst) {
  const int Ho = H >> 1, Wo = W >> 1, G = C >> 3;
  size_t total = (size_t)N * Ho * Wo * G;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    int g = (int)(i % G);
    size_t pix = i / G;
    int xo = (int)(pix % Wo);
    size_t t = pix / Wo;
    int yo = (int)(t % Ho);
    int n = (int)(t / Ho);
    float best[8], f[8];
    const size_t base = (((size_t)n * H + 2 * yo) * W + 2 * xo) * C + g * 8;
    load8f(src + base, best);
    const size_t off[3] = {(size_t)C, (size_t)W * C, (size_t)W * C + C};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      load8f(src + base + off[q], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) best[j] = f[j] > best[j] ? f[j] : best[j];
    }
    *reinterpret_cast<uint2*>(dst + pix * C + g * 8) = f8x8_from_f(best);
  }
}

// ------------------------------------------------------------------------------ optimizer
// Keras 2.13 Adam.update_step: alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1);
// v += (g^2-v)(1-b2); w -= m*alpha/(sqrt(v)+eps). AdamW first applies w -= w*wd*lr.
__global__ void adam_kernel(size_t n, float* w, const float* g, float* m, float* v, float lr,
                            float b1, float b2, float eps, float alpha, float wd, float gs) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    float gi = g[i] * gs;
    float wi = w[i];
    if (wd != 0.f) wi -= wi * wd * lr;
    float mi = m[i] + (gi - m[i]) * (1.f - b1);
    float vi = v[i] + (gi * gi - v[i]) * (1.f - b2);
    m[i] = mi;
    v[i] = vi;
    w[i] = wi - (mi * alpha) / (sqrtf(vi) + eps);
  }
}

__global__ void ema_kernel(size_t n, float* ema, const float* p, float d) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
    ema[i] = d * ema[i] + (1.f - d) * p[i];
}

}  // namespace

namespace adp {
// a conv launch with bn_defer_fold leaves its BatchNorm sums in the replicas; until the matching
// adp_bn_finalize_fold (same channel count, sum vector and stream) runs, no other launch may use them
struct PendingFold { bool on = false; int C = 0; const float* sum = nullptr; hipStream_t s = nullptr; };
static std::mutex g_fold_mu;
static std::map<int, PendingFold>& pending_folds() {
  static std::map<int, PendingFold> m;
  return m;
}
int defer_fold_begin(int C, const float* sum, hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { set_error("defer_fold: hipGetDevice failed"); return -2; }
  std::lock_guard<std::mutex> lk(g_fold_mu);
  pending_folds()[dev] = PendingFold{true, C, sum, s};
  return 0;
}
static double* stat_scratch_impl(bool fold, int C, const float* sum, hipStream_t s) {
  static std::mutex mu;
  static std::map<int, double*> per_dev;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { set_error("stat_scratch: hipGetDevice failed"); return nullptr; }
  {
    std::lock_guard<std::mutex> lk(g_fold_mu);
    PendingFold& pf = pending_folds()[dev];
    if (fold) {
      if (!pf.on || pf.C != C || pf.sum != sum || pf.s != s) {
        set_error(pf.on ? "adp_bn_finalize_fold: does not match the pending deferred fold (channel count, sum "
                          "vector or stream differ)"
                        : "adp_bn_finalize_fold: no conv launch with bn_defer_fold is pending");
        return nullptr;
      }
      pf.on = false;
    } else if (pf.on) {
      set_error("BatchNorm accumulator replicas hold the sums of a bn_defer_fold launch: adp_bn_finalize_fold "
                "must run first");
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> lk(mu);
  auto it = per_dev.find(dev);
  if (it != per_dev.end()) return it->second;
  const size_t bytes = sizeof(double) * STAT_REPL * 2 * STAT_CMAX;
  double* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMemset(p, 0, bytes) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    set_error("stat_scratch: allocation of the BatchNorm accumulator replicas failed");
    return nullptr;
  }
  per_dev[dev] = p;
  return p;
}
double* stat_scratch() { return stat_scratch_impl(false, 0, nullptr, nullptr); }
// drop a deferred fold that never reached its adp_bn_finalize_fold (an error or exception between the two) and
// re-zero the replicas it left its sums in, stream-ordered on s; a no-op when nothing is pending -- and when the
// pending fold was left on another stream: that one belongs to another caller (engine handle, thread) whose launch
// may still be in flight, and a memset on s would neither be ordered after it nor be ours to make (round-4 ADVICE)
int bn_fold_reset(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { set_error("adp_bn_fold_reset: hipGetDevice failed"); return -2; }
  {
    std::lock_guard<std::mutex> lk(g_fold_mu);
    PendingFold& pf = pending_folds()[dev];
    if (!pf.on || pf.s != s) return 0;
    pf.on = false;
  }
  double* p = stat_scratch();
  if (!p) return -2;
  if (hipMemsetAsync(p, 0, sizeof(double) * STAT_REPL * 2 * STAT_CMAX, s) != hipSuccess) {
    set_error("adp_bn_fold_reset: clearing the accumulator replicas failed");
    return -2;
  }
  return 0;
}
double* stat_scratch_fold(int C, const float* sum, hipStream_t s) { return stat_scratch_impl(true, C, sum, s); }
int* claim_slot() {
  static std::mutex mu;
  static std::map<int, std::pair<int*, unsigned>> per_dev;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { set_error("claim_slot: hipGetDevice failed"); return nullptr; }
  std::lock_guard<std::mutex> lk(mu);
  auto& e = per_dev[dev];
  if (!e.first) {
    const size_t bytes = sizeof(int) * CLAIM_SLOTS * CLAIM_INTS;
    if (hipMalloc(&e.first, bytes) != hipSuccess || hipMemset(e.first, 0, bytes) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      e.first = nullptr;
      set_error("claim_slot: allocation of the tile-claiming counters failed");
      return nullptr;
    }
  }
  return e.first + (size_t)(e.second++ % CLAIM_SLOTS) * CLAIM_INTS;
}
void* scratch(int slot, size_t bytes) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, std::pair<void*, size_t>> bufs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) { set_error("scratch: hipGetDevice failed"); return nullptr; }
  std::lock_guard<std::mutex> lk(mu);
  auto& e = bufs[{dev, slot}];
  if (e.second >= bytes) return e.first;
  if (e.first) {   // kernels queued on any stream may still use the old buffer
    if (hipDeviceSynchronize() != hipSuccess || hipFree(e.first) != hipSuccess) {
      set_error("scratch: releasing the old buffer failed");
      return nullptr;
    }
    e = {nullptr, 0};
  }
  const size_t want = bytes + bytes / 4;   // grow with headroom
  if (hipMalloc(&e.first, want) != hipSuccess) {
    e = {nullptr, 0};
    set_error("scratch: hipMalloc failed");
    return nullptr;
  }
  e.second = want;
  return e.first;
}
int stat_fold(int C, float* dst0, float* dst1, hipStream_t s) { return stat_fold_at(0, C, dst0, dst1, s); }
int stat_fold_at(int c0, int C, float* dst0, float* dst1, hipStream_t s) {
  double* sc = stat_scratch();
  if (!sc) return -1;
  hipLaunchKernelGGL(stat_fold_kernel, dim3((C + 63) / 64), dim3(256), 0, s, C, sc + c0, dst0, dst1);
  return check_launch("stat_fold");
}
}  // namespace adp

#define DTYPE_SWITCH(dtype, T, ...)                                   \
  do {                                                                \
    if ((dtype) == ADP_F32) { using T = float; __VA_ARGS__; }         \
    else if ((dtype) == ADP_BF16) { using T = bf16; __VA_ARGS__; }    \
    else { adp::set_error("unknown dtype"); return -1; }              \
  } while (0)

extern "C" int adp_pack_weights(int dtype_out, int mode, int taps, int Cin_s, int Nout,
                                const float* src, int src_kpad, void* dst, int dst_rows, int dst_kpad,
                                adp_stream_t st) {
  ADP_REQUIRE(src && dst && dst_rows > 0 && dst_kpad > 0, "adp_pack_weights: bad arguments");
  ADP_REQUIRE(mode >= 0 && mode <= 2, "adp_pack_weights: bad mode");
  size_t n = (size_t)dst_rows * dst_kpad;
  DTYPE_SWITCH(dtype_out, T,
               hipLaunchKernelGGL(pack_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, mode, taps,
                                  Cin_s, Nout, src, src_kpad, (T*)dst, dst_rows, dst_kpad));
  return adp::check_launch("adp_pack_weights");
}

extern "C" int adp_pack_weights_batch(int dtype_out, int n, const adp_pack_job* jobs, adp_stream_t st) {
  ADP_REQUIRE(n >= 1 && n <= ADP_PACK_MAX_JOBS && jobs, "adp_pack_weights_batch: 1..ADP_PACK_MAX_JOBS jobs");
  PackJobs P{};
  P.n = n;
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const adp_pack_job& J = jobs[i];
    ADP_REQUIRE(J.src && J.dst && J.taps >= 1 && J.Cin_s > 0 && J.Nout > 0 && J.dst_rows >= J.Cin_s &&
                    J.dst_kpad >= J.taps * J.Nout && J.src_kpad >= J.taps * J.Cin_s,
                "adp_pack_weights_batch: job shape mismatch");
    P.j[i] = J;
    P.tile0[i] = tiles;
    tiles += ((J.dst_rows + 63) / 64) * ((J.dst_kpad + 63) / 64);
  }
  P.tile0[n] = tiles;
  DTYPE_SWITCH(dtype_out, T,
               hipLaunchKernelGGL(pack_t_kernel<T>, dim3(tiles), dim3(256), 0, (hipStream_t)st, P));
  return adp::check_launch("adp_pack_weights_batch");
}

extern "C" int adp_bn_apply_maxpool2(int dtype, int N, int H, int W, int C, const void* z, const float* sc,
                                     const float* sh, void* act, void* pool, adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && H % 2 == 0 && W % 2 == 0 && sc && sh, "adp_bn_apply_maxpool2: need C%8==0, even H,W");
  size_t n = (size_t)N * (H / 2) * (W / 2) * (C / 8);
  DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL(bn_apply_pool_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, H, W,
                                  C, (const T*)z, sc, sh, (T*)act, (T*)pool));
  return adp::check_launch("adp_bn_apply_maxpool2");
}

extern "C" int adp_maxpool2_fwd(int dtype, int N, int H, int W, int C, const void* src,
                                const float* sc, const float* sh, void* dst, adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && H % 2 == 0 && W % 2 == 0, "adp_maxpool2_fwd: need C%8==0 and even H,W");
  size_t n = (size_t)N * (H / 2) * (W / 2) * (C / 8);
  DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, H, W,
                                  C, (const T*)src, sc, sh, (T*)dst));
  return adp::check_launch("adp_maxpool2_fwd");
}

extern "C" int adp_maxpool2_bwd(int dtype, int N, int H, int W, int C, const void* src,
                                const float* sc, const float* sh, const void* dpool, const void* addend,
                                const void* mask, float ms, void* dsrc, adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && H % 2 == 0 && W % 2 == 0, "adp_maxpool2_bwd: need C%8==0 and even H,W");
  size_t n = (size_t)N * (H / 2) * (W / 2) * (C / 8);
  DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, H, W,
                                  C, (const T*)src, sc, sh, (const T*)dpool, (const T*)addend,
                                  (const T*)mask, ms, (T*)dsrc));
  return adp::check_launch("adp_maxpool2_bwd");
}

extern "C" int adp_maxpool2_bwd_bnr(int dtype, int N, int H, int W, int C, const void* src, const void* dpool,
                                    const void* addend, void* dsrc, const void* z, const float* sc, const float* sh,
                                    const float* mean, const float* invstd, float* dgamma, float* dbeta,
                                    adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && C / 8 <= TPB && H % 2 == 0 && W % 2 == 0 && dpool && addend && dsrc && z && sc &&
                  sh && mean && invstd && dgamma && dbeta,
              "adp_maxpool2_bwd_bnr: need C%8==0, C<=2048, even H,W and every operand");
  ADP_REQUIRE((size_t)N * (H / 2) * (W / 2) < (1ull << 31), "adp_maxpool2_bwd_bnr: too many pooled pixels");
  const int lanes = TPB / (C / 8);
  const size_t P = (size_t)N * (H / 2) * (W / 2);
  const int blocks = (int)std::max<size_t>(1, std::min<size_t>((P + lanes - 1) / lanes,
                                                               (size_t)adp::option("pool_bnr_blocks", 2048)));
  double* stat = adp::stat_scratch();
  if (!stat) return -1;
  DTYPE_SWITCH(dtype, T,
               if (src) hipLaunchKernelGGL((maxpool_bwd_bnr_kernel<T, true>), dim3(blocks), dim3(TPB), 0, (hipStream_t)st,
                                           N, H, W, C, (const T*)src, (const T*)dpool, (const T*)addend, (T*)dsrc,
                                           (const T*)z, sc, sh, mean, invstd, stat);
               else hipLaunchKernelGGL((maxpool_bwd_bnr_kernel<T, false>), dim3(blocks), dim3(TPB), 0, (hipStream_t)st,
                                       N, H, W, C, (const T*)src, (const T*)dpool, (const T*)addend, (T*)dsrc,
                                       (const T*)z, sc, sh, mean, invstd, stat));
  if (adp::check_launch("adp_maxpool2_bwd_bnr")) return -2;
  return adp::stat_fold(C, dbeta, dgamma, (hipStream_t)st);
}

extern "C" int adp_upsample2_bwd(int dtype, int N, int Hs, int Ws, int C, const void* dup,
                                 const void* addend, const void* mask, float ms, void* dsrc,
                                 adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0, "adp_upsample2_bwd: need C%8==0");
  size_t n = (size_t)N * Hs * Ws * (C / 8);
  DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL(upsample_bwd_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, Hs,
                                  Ws, C, (const T*)dup, (const T*)addend, (const T*)mask, ms, (T*)dsrc));
  return adp::check_launch("adp_upsample2_bwd");
}

extern "C" int adp_ew_add_mask(int dtype, size_t n, const void* a, const void* b, const void* mask,
                               float ms, void* out, adp_stream_t st) {
  ADP_REQUIRE(n % 8 == 0, "adp_ew_add_mask: n must be a multiple of 8");
  size_t g = n / 8;
  DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL(ew_add_mask_kernel<T>, dim3(nblk(g)), dim3(TPB), 0, (hipStream_t)st, g,
                                  (const T*)a, (const T*)b, (const T*)mask, ms, (T*)out));
  return adp::check_launch("adp_ew_add_mask");
}

extern "C" int adp_cast(int di, int dout, size_t n, const void* src, void* dst, adp_stream_t st) {
  hipStream_t s = (hipStream_t)st;
  if (di == ADP_F32 && dout == ADP_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(nblk(n)), dim3(TPB), 0, s, n, (const float*)src, (bf16*)dst);
  else if (di == ADP_BF16 && dout == ADP_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(nblk(n)), dim3(TPB), 0, s, n, (const bf16*)src, (float*)dst);
  else if (di == ADP_F32 && dout == ADP_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(nblk(n)), dim3(TPB), 0, s, n, (const float*)src, (float*)dst);
  else if (di == ADP_BF16 && dout == ADP_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(nblk(n)), dim3(TPB), 0, s, n, (const bf16*)src, (bf16*)dst);
  else { adp::set_error("adp_cast: bad dtype"); return -1; }
  return adp::check_launch("adp_cast");
}

extern "C" int adp_sum_bf16(int nsrc, const void* const* srcs, size_t n, void* out, adp_stream_t st) {
  if (nsrc < 1 || nsrc > 8 || n % 8 != 0 || !srcs || !out) {
    adp::set_error("adp_sum_bf16: 1..8 sources, n a multiple of 8");
    return -1;
  }
  SumSrcs S{};
  for (int k = 0; k < nsrc; ++k) {
    if (!srcs[k] || (reinterpret_cast<uintptr_t>(srcs[k]) & 15)) { adp::set_error("adp_sum_bf16: source not 16-B aligned"); return -1; }
    S.p[k] = (const bf16*)srcs[k];
  }
  const size_t g = n / 8;
  hipLaunchKernelGGL(sum_bf16_kernel, dim3(nblk(g)), dim3(TPB), 0, (hipStream_t)st, g, nsrc, S, (bf16*)out);
  return adp::check_launch("adp_sum_bf16");
}

extern "C" int adp_fill_f32(size_t n, float v, float* dst, adp_stream_t st) {
  hipLaunchKernelGGL(fill_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, n, v, dst);
  return adp::check_launch("adp_fill_f32");
}

extern "C" int adp_bn_finalize(int C, float count, const float* sum, const float* sq, const float* gamma,
                               const float* beta, float eps, float momentum, float* scale, float* shift,
                               float* mean, float* invstd, float* rmean, float* rvar, adp_stream_t st) {
  ADP_REQUIRE(C > 0 && count != 0, "adp_bn_finalize: bad arguments");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + TPB - 1) / TPB), dim3(TPB), 0, (hipStream_t)st, C, count,
                     sum, sq, gamma, beta, eps, momentum, scale, shift, mean, invstd, rmean, rvar);
  return adp::check_launch("adp_bn_finalize");
}

extern "C" int adp_bn_fold_reset(adp_stream_t st) { return adp::bn_fold_reset((hipStream_t)st) ? -2 : 0; }
extern "C" int adp_wgrad_defer(int on, adp_stream_t st) { return adp::wgrad_defer((hipStream_t)st, on) ? -1 : 0; }
extern "C" int adp_wgrad_flush(adp_stream_t st) {
  adp::wgrad_flush((hipStream_t)st);
  return adp::check_launch("adp_wgrad_flush");
}
extern "C" int adp_wgrad_release(adp_stream_t st) { return adp::wgrad_release((hipStream_t)st) ? -1 : 0; }
extern "C" int adp_wgrad_arena_chunks(adp_stream_t st) { return adp::wgrad_arena_chunks((hipStream_t)st); }

extern "C" int adp_bn_finalize_fold(int C, float count, float* sum, float* sq, const float* gamma, const float* beta,
                                    float eps, float momentum, float* scale, float* shift, float* mean, float* invstd,
                                    float* rmean, float* rvar, adp_stream_t st) {
  ADP_REQUIRE(C > 0 && C <= adp::STAT_CMAX && count > 0 && sum && sq && gamma && beta && scale && shift && mean &&
                  invstd,
              "adp_bn_finalize_fold: bad arguments (training statistics, C <= 2048)");
  double* sc = adp::stat_scratch_fold(C, sum, (hipStream_t)st);
  if (!sc) return -1;
  hipLaunchKernelGGL(bn_fold_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, (hipStream_t)st, C, sc, sum, sq,
                     count, gamma, beta, eps, momentum, scale, shift, mean, invstd, rmean, rvar);
  return adp::check_launch("adp_bn_finalize_fold");
}

extern "C" int adp_bn_bwd_reduce(int dtype, size_t M, int C, const void* dA, const void* z, const float* sc,
                                 const float* sh, const float* mean, const float* invstd, float* dgamma,
                                 float* dbeta, adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && C / 8 <= TPB, "adp_bn_bwd_reduce: C must be a multiple of 8 and <= 2048");
  int lanes = TPB / (C / 8);
  int blocks = (int)std::min<size_t>((M + lanes - 1) / lanes, 2048);
  double* stat = adp::stat_scratch();
  if (!stat) return -1;
  DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3(blocks), dim3(TPB), 0, (hipStream_t)st, M, C,
                                  (const T*)dA, (const T*)z, sc, sh, mean, invstd, dgamma, dbeta, stat));
  if (adp::check_launch("adp_bn_bwd_reduce")) return -2;
  return adp::stat_fold(C, dbeta, dgamma, (hipStream_t)st);
}

extern "C" int adp_bn_bwd_apply(int dtype, size_t M, int C, const void* dA, const void* z, const float* sc,
                                const float* sh, const float* mean, const float* invstd, const float* gamma,
                                const float* dgamma, const float* dbeta, float count, void* dz,
                                adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && C / 8 <= TPB && count > 0, "adp_bn_bwd_apply: bad arguments (C % 8 == 0, C <= 2048)");
  BN_UNROLL_SWITCH(U, 4, DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL((bn_bwd_apply_kernel<T, U>), dim3(bn_blocks(M, C, U, 32768)), dim3(TPB), 0, (hipStream_t)st,
                                  M, C, (const T*)dA, (const T*)z, sc, sh, mean, invstd, gamma, dgamma, dbeta,
                                  1.f / count, (T*)dz)));
  return adp::check_launch("adp_bn_bwd_apply");
}

extern "C" int adp_bn_bwd_apply_head(int dtype, size_t M, int C, int Cin, const float* W, const float* p,
                                     const float* dp, const void* z, const float* sc, const float* sh,
                                     const float* mean, const float* invstd, const float* gamma,
                                     const float* dgamma, const float* dbeta, float count, void* dz,
                                     adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && C / 8 <= TPB && Cin <= C && Cin % 8 == 0 && count > 0 && W && p && dp &&
                  ((uintptr_t)W & 15) == 0,
              "adp_bn_bwd_apply_head: bad arguments (C % 8 == 0, C <= 2048, Cin <= C, Cin % 8 == 0, W 16-B aligned)");
  BN_UNROLL_SWITCH(U, 4, DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL((bn_bwd_apply_head_kernel<T, U>), dim3(bn_blocks(M, C, U, 32768)), dim3(TPB), 0,
                                  (hipStream_t)st, M, C, Cin, (const T*)z, W, p, dp, sc, sh, mean, invstd, gamma,
                                  dgamma, dbeta, 1.f / count, (T*)dz)));
  return adp::check_launch("adp_bn_bwd_apply_head");
}

extern "C" int adp_bn_apply(int dtype, size_t M, int C, const void* z, const float* sc, const float* sh, void* out,
                            adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && C / 8 <= TPB && sc && sh, "adp_bn_apply: bad arguments (C % 8 == 0, C <= 2048)");
  BN_UNROLL_SWITCH(U, 4, DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL((bn_apply_kernel<T, U>), dim3(bn_blocks(M, C, U, 65536)), dim3(TPB), 0, (hipStream_t)st, M,
                                  C, (const T*)z, sc, sh, (T*)out)));
  return adp::check_launch("adp_bn_apply");
}

extern "C" int adp_adam(size_t n, float* w, const float* g, float* m, float* v, float lr, float b1,
                        float b2, float eps, int step, float wd, float gs, adp_stream_t st) {
  ADP_REQUIRE(step >= 1, "adp_adam: step counts from 1");
  double alpha = (double)lr * sqrt(1.0 - pow((double)b2, step)) / (1.0 - pow((double)b1, step));
  hipLaunchKernelGGL(adam_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, n, w, g, m, v, lr, b1, b2,
                     eps, (float)alpha, wd, gs);
  return adp::check_launch("adp_adam");
}

extern "C" int adp_ema(size_t n, float* ema, const float* p, float d, adp_stream_t st) {
  hipLaunchKernelGGL(ema_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, n, ema, p, d);
  return adp::check_launch("adp_ema");
}

extern "C" int adp_pack_weights_fp8(int rows, const float* src, int src_kpad, void* dst, int dst_kpad, float* scale,
                                    adp_stream_t st) {
  ADP_REQUIRE(rows > 0 && src && dst && scale && dst_kpad % 8 == 0 && dst_kpad >= src_kpad,
              "adp_pack_weights_fp8: bad arguments (dst_kpad % 8 == 0 and >= src_kpad)");
  hipLaunchKernelGGL(pack_fp8_kernel, dim3(rows), dim3(TPB), 0, (hipStream_t)st, src, src_kpad, (unsigned char*)dst,
                     dst_kpad, scale);
  return adp::check_launch("adp_pack_weights_fp8");
}

namespace {
__global__ void vec_mul_kernel(size_t n, const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ o) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) o[i] = a[i] * b[i];
}
}  // namespace

namespace {
template <typename T>
__global__ void scale_rows_kernel(int rows, int cols, const float* __restrict__ src, int src_ld,
                                  const float* __restrict__ scale, int nscale, T* __restrict__ dst, int dst_ld) {
  const size_t n = (size_t)rows * cols;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int r = (int)(i / cols), c = (int)(i - (size_t)r * cols);
    const float sc = r < nscale ? scale[r] : 0.f;
    dst[(size_t)r * dst_ld + c] = from_f<T>(src[(size_t)r * src_ld + c] * sc);
  }
}
}  // namespace

extern "C" int adp_scale_rows(int dtype_out, int rows, int cols, const float* src, int src_ld, const float* scale,
                              int nscale, void* dst, int dst_ld, adp_stream_t st) {
  ADP_REQUIRE(src && scale && dst && rows > 0 && cols > 0 && src_ld >= cols && dst_ld >= cols && nscale >= 0,
              "adp_scale_rows: bad arguments");
  const size_t n = (size_t)rows * cols;
  DTYPE_SWITCH(dtype_out, T,
               hipLaunchKernelGGL(scale_rows_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, rows, cols, src,
                                  src_ld, scale, nscale, (T*)dst, dst_ld));
  return adp::check_launch("adp_scale_rows");
}

extern "C" int adp_vec_mul(size_t n, const float* a, const float* b, float* out, adp_stream_t st) {
  ADP_REQUIRE(a && b && out, "adp_vec_mul: null vector");
  if (n == 0) return 0;
  hipLaunchKernelGGL(vec_mul_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, n, a, b, out);
  return adp::check_launch("adp_vec_mul");
}

extern "C" int adp_bn_apply_fp8(int dtype, size_t M, int C, const void* z, const float* sc, const float* sh,
                                void* out, adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && sc && sh, "adp_bn_apply_fp8: bad arguments");
  size_t n = M * (C / 8);
  DTYPE_SWITCH(dtype, T,
               hipLaunchKernelGGL(bn_apply_fp8_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, M, C,
                                  (const T*)z, sc, sh, (unsigned char*)out));
  return adp::check_launch("adp_bn_apply_fp8");
}

extern "C" int adp_maxpool2_fwd_fp8(int dtype, int N, int H, int W, int C, const void* src, void* dst,
                                    adp_stream_t st) {
  ADP_REQUIRE(C % 8 == 0 && H % 2 == 0 && W % 2 == 0, "adp_maxpool2_fwd_fp8: need C%8==0 and even H,W");
  size_t n = (size_t)N * (H / 2) * (W / 2) * (C / 8);
  hipStream_t s = (hipStream_t)st;
  if (dtype == ADP_FP8)
    hipLaunchKernelGGL(maxpool_fwd_fp8_kernel<unsigned char>, dim3(nblk(n)), dim3(TPB), 0, s, N, H, W, C,
                       (const unsigned char*)src, (unsigned char*)dst);
  else
    DTYPE_SWITCH(dtype, T,
                 hipLaunchKernelGGL(maxpool_fwd_fp8_kernel<T>, dim3(nblk(n)), dim3(TPB), 0, s, N, H, W, C,
                                    (const T*)src, (unsigned char*)dst));
  return adp::check_launch("adp_maxpool2_fwd_fp8");
}
