// Per-pixel heads, bilinear aux resize, BCE+Dice / OHEM loss and metric reductions.
//   main head  Conv2D(2,1,activation='softmax') -> [...,1:2] -> squeeze
//              Segmentation/train_adipose_unet_v3.py:729-731
//   aux heads  Conv2D(1,1,activation='sigmoid') + tf.image.resize(bilinear)      :715-726
//   losses     dice_loss :217-225, combined_loss_standard :228-241, label smoothing :244-279,
//              online_hard_example_mining_loss(+smoothing) :282-363; Keras 2.13 binary_crossentropy
//              (clip to [1e-7, 1-1e-7], log(p+1e-7), mean over the last axis)
//   metrics    dice_coef src/utils/model.py:93-98, Keras binary_accuracy (threshold 0.5),
//              calculate_pixel_metrics counts Segmentation/full_evaluation_enhanced.py:721-785
#include "common.h"
#include <algorithm>
#include "../../include/adipose_hip.h"

namespace {
constexpr int TPB = 256;
constexpr float KEPS = 1e-7f;

inline int nblk(size_t n, int cap = 8192) {
  size_t b = (n + TPB - 1) / TPB;
  return (int)(b < (size_t)cap ? (b ? b : 1) : cap);
}

// ---------------------------------------------------------------------------------- heads
// forward: thread per pixel, dot over Cin channels (8-channel groups), NOUT = 1 or 2
template <typename T, int NOUT>
__global__ void head_fwd_kernel(size_t M, int Cs, int Cin, const T* x, const float* W, const float* b,
                                const float* sc, const float* sh, float* p) {
  __shared__ float ws[NOUT * 1024];
  for (int i = threadIdx.x; i < NOUT * Cs; i += TPB) {
    int o = i / Cs, c = i - o * Cs;
    ws[i] = c < Cin ? W[o * Cin + c] : 0.f;
  }
  __syncthreads();
  const float b0 = b[0], b1 = NOUT == 2 ? b[1] : 0.f;
  for (size_t m = blockIdx.x * (size_t)TPB + threadIdx.x; m < M; m += (size_t)gridDim.x * TPB) {
    float z0 = b0, z1 = b1;
    for (int g = 0; g < Cs; g += 8) {
      Grp<T> gr;
      float f[8];
      grp_load(gr, x + m * Cs + g);
      grp_to_f(gr, f);
      if (sc) {   // BatchNorm+ReLU on load, rounded to T as adp_bn_apply would materialize it
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[g + j], sh[g + j]), 0.f);
        grp_from_f(gr, f);
        grp_to_f(gr, f);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        z0 = fmaf(f[j], ws[g + j], z0);
        if (NOUT == 2) z1 = fmaf(f[j], ws[Cs + g + j], z1);
      }
    }
    // softmax over 2 logits, channel 1 kept == 1/(1+exp(z0-z1)); sigmoid otherwise
    p[m] = NOUT == 2 ? 1.f / (1.f + expf(z0 - z1)) : 1.f / (1.f + expf(-z0));
  }
}

// forward, coalesced form for G = Cs/8 a power of two <= 64: the G lanes of one pixel each own one
// 8-channel group (adjacent 16-B loads), partial dot products are summed with lane shuffles.
template <typename T, int NOUT, int G>
__global__ void head_fwd_grp_kernel(size_t M, int Cs, int Cin, const T* x, const float* W, const float* b,
                                    const float* sc, const float* sh, float* p) {
  const int g = threadIdx.x % G;
  float w0[8], w1[8], s_[8], h_[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = g * 8 + j;
    w0[j] = c < Cin ? W[c] : 0.f;
    w1[j] = (NOUT == 2 && c < Cin) ? W[Cin + c] : 0.f;
    s_[j] = sc ? sc[c] : 1.f;
    h_[j] = sc ? sh[c] : 0.f;
  }
  const float b0 = b[0], b1 = NOUT == 2 ? b[1] : 0.f;
  const size_t lanes = TPB / G;
  for (size_t m = blockIdx.x * lanes + threadIdx.x / G; m < M; m += (size_t)gridDim.x * lanes) {
    Grp<T> gr;
    float f[8];
    grp_load(gr, x + m * Cs + g * 8);
    grp_to_f(gr, f);
    float z0 = 0.f, z1 = 0.f;
    if (sc) {   // BatchNorm+ReLU on load, rounded to T as adp_bn_apply would materialize it
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], s_[j], h_[j]), 0.f);
      grp_from_f(gr, f);
      grp_to_f(gr, f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      z0 = fmaf(f[j], w0[j], z0);
      if (NOUT == 2) z1 = fmaf(f[j], w1[j], z1);
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      z0 += __shfl_xor(z0, o, 64);
      if (NOUT == 2) z1 += __shfl_xor(z1, o, 64);
    }
    if (g == 0) {
      z0 += b0; z1 += b1;
      p[m] = NOUT == 2 ? 1.f / (1.f + expf(z0 - z1)) : 1.f / (1.f + expf(-z0));
    }
  }
}

template <typename T, int NOUT>
void launch_head_fwd(size_t M, int Cs, int Cin, const T* x, const float* W, const float* b, const float* sc,
                     const float* sh, float* p, hipStream_t s) {
  const int G = Cs / 8;
  const int blk = (int)std::min<size_t>((M * G + TPB - 1) / TPB, 8192);
  switch (G) {
#define ADP_HG(GG) case GG: hipLaunchKernelGGL((head_fwd_grp_kernel<T, NOUT, GG>), dim3(blk), dim3(TPB), 0, s, M, Cs, Cin, x, W, b, sc, sh, p); return;
    ADP_HG(1) ADP_HG(2) ADP_HG(4) ADP_HG(8) ADP_HG(16) ADP_HG(32) ADP_HG(64)
#undef ADP_HG
    default:
      hipLaunchKernelGGL((head_fwd_kernel<T, NOUT>), dim3(nblk(M)), dim3(TPB), 0, s, M, Cs, Cin, x, W, b, sc, sh, p);
  }
}

// backward: block = 32 pixel lanes x 8 channel groups (Cs <= 64*8); dW reduced in LDS then atomics.
// BNR (x = the pre-BN map z, sc/sh its BatchNorm): also the BatchNorm-backward reduction of that layer
// over the stored dx (adp_bn_bwd_reduce fused): dbeta += sum db, dgamma += sum db*(z-mean)*invstd,
// db = dx*(z*sc+sh > 0)
template <typename T, int NOUT, bool BNR = false, bool FAST = false>
__global__ __launch_bounds__(TPB) void head_bwd_kernel(size_t M, int Cs, int Cin, const T* x, const float* W, const float* sc,
                                const float* sh, const float* p, const float* dp, const T* addend,
                                const T* mask, float ms, T* dx, float* dW, float* db, const float* bmean = nullptr,
                                const float* binv = nullptr, double* stat = nullptr) {
  const int G = Cs >> 3;                 // groups per pixel
  const int lanes = TPB / G;
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  float wd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int c = g * 8 + j;
    float w1 = c < Cin ? W[(NOUT - 1) * Cin + c] : 0.f;
    float w0 = (NOUT == 2 && c < Cin) ? W[c] : 0.f;
    wd[j] = NOUT == 2 ? w1 - w0 : w1;
  }
  // per-channel BatchNorm coefficients of this thread's group in registers (the loop's stores through dx
  // could alias them, so they would be re-read every pixel)
  float s_[8], h_[8], mu[8], iv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = g * 8 + j;
    s_[j] = sc ? sc[c] : 1.f;
    h_[j] = sc ? sh[c] : 0.f;
    mu[j] = BNR ? bmean[c] : 0.f;
    iv[j] = BNR ? binv[c] : 0.f;
  }
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float r1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, r2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float dbacc = 0.f;
  // U pixels per thread per pass, their x / p / dp loads issued before the first use (one 16-B load per
  // thread in flight left the kernel at ~3 TB/s); addend / mask (softmax2 heads only) load per pixel
  constexpr int U = 4;
  auto one = [&](size_t m, float pm, float dpm, const Grp<T>& gx) {
    const float dz = dpm * pm * (1.f - pm);   // d p/d(z1-z0) for softmax2, d p/dz for sigmoid
    float f[8], o[8], a[8], mk[8];
    grp_to_f(gx, f);
    Grp<T> gt;
    // FAST (round 6, the unet_bn BNR head: BatchNorm coefficients present, no addend or mask -- compile-time, so the
    // loop has no per-element selects)
    const bool has_add = !FAST && addend, has_mask = !FAST && mask;
    if (has_add) { grp_load(gt, addend + m * Cs + g * 8); grp_to_f(gt, a); }
    if (has_mask) { grp_load(gt, mask + m * Cs + g * 8); grp_to_f(gt, mk); }
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (FAST || sc) ? fmaxf(fmaf(f[j], s_[j], h_[j]), 0.f) : f[j];
    if constexpr (BNR) {   // the activation as adp_bn_apply materializes it (rounded to T)
      Grp<T> gv;
      grp_from_f(gv, v);
      grp_to_f(gv, v);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[j] = fmaf(dz, v[j], acc[j]);
      float d = dz * wd[j] + (has_add ? a[j] : 0.f);
      if (has_mask) d = mk[j] > 0.f ? d * ms : 0.f;
      o[j] = d;
    }
    Grp<T> gr;
    grp_from_f(gr, o);
    if (dx) grp_store(gr, dx + m * Cs + g * 8);
    if constexpr (BNR) {   // over the stored (rounded) gradient, as adp_bn_bwd_reduce reads it
      float os[8];
      grp_to_f(gr, os);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = fmaf(f[j], s_[j], h_[j]) > 0.f ? os[j] : 0.f;
        r1[j] += d;
        r2[j] += d * (f[j] - mu[j]) * iv[j];
      }
    }
    if (g == 0) dbacc += dz;
  };
  if (pl < lanes) {
    const size_t step = (size_t)gridDim.x * lanes;
    size_t m = (size_t)blockIdx.x * lanes + pl;
    for (; m + (U - 1) * step < M; m += U * step) {
      float pm[U], dpm[U];
      Grp<T> gx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t mu_ = m + u * step;
        pm[u] = p[mu_];
        dpm[u] = dp[mu_];
        grp_load(gx[u], x + mu_ * Cs + g * 8);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) one(m + u * step, pm[u], dpm[u], gx[u]);
    }
    for (; m < M; m += step) {
      Grp<T> gx;
      grp_load(gx, x + m * Cs + g * 8);
      one(m, p[m], dp[m], gx);
    }
  }
  __shared__ float red[TPB * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = acc[j];
  __shared__ float redb[TPB];
  redb[threadIdx.x] = dbacc;
  __syncthreads();
  // BNR: every sum goes to this block's replica of the accumulator scratch (adp::stat_scratch; same-address
  // f32 atomics from thousands of blocks serialise), folded by the host wrapper: row 0 [0, Cs) dbeta,
  // row 1 [0, Cs) dgamma, row 0 [Cs, Cs + Cin) dW, row 0 Cs + Cin db
  double* rep = BNR ? stat + (size_t)(blockIdx.x & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX : nullptr;
  for (int c = threadIdx.x; c < Cin; c += TPB) {
    int gg = c >> 3, j = c & 7;
    float s = 0.f;
    for (int l = 0; l < lanes; ++l) s += red[(l * G + gg) * 8 + j];
    if (BNR) atomicAdd(rep + Cs + c, (double)s);
    else if (NOUT == 2) { atomicAdd(dW + c, -s); atomicAdd(dW + Cin + c, s); }
    else atomicAdd(dW + c, s);
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int l = 0; l < lanes; ++l) s += redb[l * G];
    if (BNR) atomicAdd(rep + Cs + Cin, (double)s);
    else if (NOUT == 2) { atomicAdd(db, -s); atomicAdd(db + 1, s); }
    else atomicAdd(db, s);
  }
  if constexpr (BNR) {
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = pass ? r2[j] : r1[j];
      __syncthreads();
      for (int c = threadIdx.x; c < Cs; c += TPB) {
        const int gg = c >> 3, j = c & 7;
        float t = 0.f;
        for (int l = 0; l < lanes; ++l) t += red[(l * G + gg) * 8 + j];
        atomicAdd(rep + (pass ? adp::STAT_CMAX : 0) + c, (double)t);
      }
    }
  }
}

// ------------------------------------------------------------------- bilinear (half-pixel)
// TF ResizeBilinear(half_pixel_centers=True): in = (out+0.5)*scale-0.5, lo = max(floor,0),
// hi = min(ceil, n-1), lerp = in - floor(in); value = top + (bottom-top)*ylerp.
ADP_DEV void bil_coord(int o, float scale, int n, int& lo, int& hi, float& t) {
  float in = ((float)o + 0.5f) * scale - 0.5f;
  float fl = floorf(in);
  lo = in > 0.f ? (int)fl : 0;
  hi = (in < (float)(n - 1)) ? (int)ceilf(in) : n - 1;
  t = in - fl;
}

__global__ void resize_fwd_kernel(int N, int Hs, int Ws, int Ho, int Wo, const float* src, float* dst) {
  const float sy = (float)Hs / Ho, sx = (float)Ws / Wo;
  size_t total = (size_t)N * Ho * Wo;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    int xo = (int)(i % Wo);
    size_t t = i / Wo;
    int yo = (int)(t % Ho), n = (int)(t / Ho);
    int y0, y1, x0, x1;
    float ty, tx;
    bil_coord(yo, sy, Hs, y0, y1, ty);
    bil_coord(xo, sx, Ws, x0, x1, tx);
    const float* s = src + (size_t)n * Hs * Ws;
    float tl = s[y0 * Ws + x0], tr = s[y0 * Ws + x1], bl = s[y1 * Ws + x0], br = s[y1 * Ws + x1];
    float top = tl + (tr - tl) * tx, bot = bl + (br - bl) * tx;
    dst[i] = top + (bot - top) * ty;
  }
}

// adjoint as a gather: dsrc[ys][xs] = sum_{yo,xo} wy(yo,ys) wx(xo,xs) dout[yo][xo]
ADP_DEV float bil_w(int o, float scale, int n, int s) {
  int lo, hi;
  float t;
  bil_coord(o, scale, n, lo, hi, t);
  return (lo == s ? 1.f - t : 0.f) + (hi == s ? t : 0.f);
}

__global__ void resize_bwd_kernel(int N, int Hs, int Ws, int Ho, int Wo, const float* dout, float* dsrc) {
  const float sy = (float)Hs / Ho, sx = (float)Ws / Wo;
  const int fy = (Ho + Hs - 1) / Hs, fx = (Wo + Ws - 1) / Ws;
  size_t total = (size_t)N * Hs * Ws;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    int xs = (int)(i % Ws);
    size_t t = i / Ws;
    int ys = (int)(t % Hs), n = (int)(t / Hs);
    int ya = max(0, (ys - 1) * fy - fy), yb = min(Ho - 1, (ys + 2) * fy + fy);
    int xa = max(0, (xs - 1) * fx - fx), xb = min(Wo - 1, (xs + 2) * fx + fx);
    const float* d = dout + (size_t)n * Ho * Wo;
    float acc = 0.f;
    for (int yo = ya; yo <= yb; ++yo) {
      float wy = bil_w(yo, sy, Hs, ys);
      if (wy == 0.f) continue;
      float rs = 0.f;
      for (int xo = xa; xo <= xb; ++xo) {
        float wx = bil_w(xo, sx, Ws, xs);
        if (wx != 0.f) rs = fmaf(wx, d[(size_t)yo * Wo + xo], rs);
      }
      acc = fmaf(wy, rs, acc);
    }
    dsrc[i] = acc;
  }
}

// ---------------------------------------------------------------------------------- losses
ADP_DEV float smooth_y(float y, int smooth, float ep, float en) {
  return smooth ? y * (1.f - ep - en) + en : y;
}
ADP_DEV float clipp(float p) { return fminf(fmaxf(p, KEPS), 1.f - KEPS); }

ADP_DEV double block_sum_d(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += sh[i];
  return r;   // valid in thread 0
}

// one block per image row
ADP_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one wave per image row (row BCE by lane shuffles); the 8 global statistics are accumulated per
// lane across the wave's rows and reduced once per block (one f64 atomic per statistic and block)
__global__ void loss_rows_kernel(int N, int H, int W, const float* p, const float* y, int smooth,
                                 float ep, float en, float* row_bce, double* stats) {
  constexpr int WPB = TPB / 64;
  __shared__ double sh[8][WPB];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int row = blockIdx.x * WPB + wave; row < N * H; row += gridDim.x * WPB) {
    const float* pr = p + (size_t)row * W;
    const float* yr = y + (size_t)row * W;
    float bce = 0.f, s_yp = 0.f, s_y = 0.f, s_p = 0.f, r_yp = 0.f, r_y = 0.f, r_p = 0.f, acc = 0.f, r_yi = 0.f;
    for (int x = lane; x < W; x += 64) {
      float pv = pr[x], yv = yr[x];
      float ys = smooth_y(yv, smooth, ep, en);
      float pc = clipp(pv);
      bce -= ys * logf(pc + KEPS) + (1.f - ys) * logf(1.f - pc + KEPS);
      s_yp += ys * pc; s_y += ys; s_p += pc;
      r_yp += yv * pv; r_y += yv; r_p += pv;
      const float pb = pv > 0.5f ? 1.f : 0.f;   // == round(clip(p,0,1)) (round half to even)
      acc += (yv == pb) ? 1.f : 0.f;
      r_yi += yv * pb;
    }
    const double rb = wave_sum_d((double)bce);
    if (lane == 0) row_bce[row] = (float)(rb / W);
    st[0] += s_yp; st[1] += s_y; st[2] += s_p; st[3] += r_yp;
    st[4] += r_y; st[5] += r_p; st[6] += acc; st[7] += r_yi;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const double v = wave_sum_d(st[i]);
    if (lane == 0) sh[i][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < WPB; ++w) t += sh[threadIdx.x][w];
    atomicAdd(stats + threadIdx.x, t);
  }
}

// one block (1024 threads) per image: bitonic sort of (bce desc, row asc) keys, first k selected
__global__ void loss_select_kernel(int N, int H, int W, const float* row_bce, int ohem, float keep,
                                   float weight, float norm_rows, float* row_coef, double* out) {
  __shared__ float kv[2048];
  __shared__ int ki[2048];
  __shared__ double sh[16];
  const int b = blockIdx.x;
  const float* rb = row_bce + (size_t)b * H;
  float* rc = row_coef + (size_t)b * H;
  const float coef = weight / (norm_rows * (float)W);
  if (!ohem) {
    double s = 0.0;
    for (int r = threadIdx.x; r < H; r += blockDim.x) { rc[r] = coef; s += rb[r]; }
    s = block_sum_d(s, sh);
    if (threadIdx.x == 0) atomicAdd(out, (double)weight * s / norm_rows);
    return;
  }
  int P = 1;
  while (P < H) P <<= 1;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    kv[i] = i < H ? rb[i] : -INFINITY;
    ki[i] = i < H ? i : 0x7fffffff;
  }
  __syncthreads();
  // sort descending by value, ascending by index on ties
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        int l = i ^ j;
        if (l > i) {
          bool desc = (i & k) == 0;
          float a = kv[i], c = kv[l];
          int ia = ki[i], ic = ki[l];
          bool a_first = (a > c) || (a == c && ia < ic);
          if (desc != a_first) { kv[i] = c; kv[l] = a; ki[i] = ic; ki[l] = ia; }
        }
      }
      __syncthreads();
    }
  }
  const int kk = (int)((float)H * keep);
  double s = 0.0;
  for (int i = threadIdx.x; i < H; i += blockDim.x) {
    bool sel = i < kk;
    rc[ki[i]] = sel ? coef : 0.f;
    if (sel) s += kv[i];
  }
  s = block_sum_d(s, sh);
  if (threadIdx.x == 0) atomicAdd(out, (double)weight * s / norm_rows);
}

__global__ void loss_grad_kernel(int N, int H, int W, const float* p, const float* y, int smooth,
                                 float ep, float en, const float* row_coef, const double* stats,
                                 float weight, int accumulate, float* dp) {
  const double I = stats[0], Sy = stats[1], Sp = stats[2];
  const double den = Sy + Sp + 1.0;
  const float g_i = (float)(-(weight * 2.0) / den);                  // coefficient of y_i
  const float g_c = (float)(weight * (2.0 * I + 1.0) / (den * den));  // constant term
  size_t total = (size_t)N * H * W;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < total; i += (size_t)gridDim.x * TPB) {
    float pv = p[i];
    float ys = smooth_y(y[i], smooth, ep, en);
    float d = 0.f;
    if (pv >= KEPS && pv <= 1.f - KEPS) {
      float pc = pv;
      float dbce = -ys / (pc + KEPS) + (1.f - ys) / (1.f - pc + KEPS);
      d = row_coef[i / W] * dbce + (g_i * ys + g_c);
    }
    dp[i] = accumulate ? dp[i] + d : d;
  }
}

__global__ void pixel_counts_kernel(size_t n, const float* pred, const float* truth, float thr,
                                    unsigned long long* counts) {
  unsigned long long c[4] = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    bool pb = pred[i] > thr, tb = truth[i] > 0.5f;
    c[pb ? (tb ? 0 : 1) : (tb ? 2 : 3)]++;
  }
  __shared__ unsigned long long sh[4][TPB / 64];
  for (int k = 0; k < 4; ++k) {
    unsigned long long v = c[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) sh[k][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long v = 0;
    for (int w = 0; w < TPB / 64; ++w) v += sh[threadIdx.x][w];
    atomicAdd(counts + threadIdx.x, v);
  }
}
// threshold sweep: per pixel j = #{t : pred > thr[t]} over ascending thresholds (compared in double, as
// numpy compares a float32 map with float64 thresholds), histogram of j split by the truth bit in LDS,
// one atomic per bin and block. tp(t) = sum_{j > t} hist[1][j], fp(t) = sum_{j > t} hist[0][j].
struct ThrList { double t[64]; };
__global__ void threshold_hist_kernel(size_t n, const float* pred, const float* truth, int nt, ThrList thr,
                                      unsigned long long* hist) {
  __shared__ unsigned int h[2][65];
  for (int i = threadIdx.x; i < 2 * 65; i += TPB) (&h[0][0])[i] = 0;
  __syncthreads();
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const double p = pred[i];
    int lo = 0, hi = nt;            // first t with !(p > thr[t]) (thresholds ascending)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (p > thr.t[mid]) lo = mid + 1; else hi = mid;
    }
    atomicAdd(&h[truth[i] > 0.5f ? 1 : 0][lo], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * (nt + 1); i += TPB) {
    const unsigned int v = h[i / (nt + 1)][i % (nt + 1)];
    if (v) atomicAdd(hist + i, (unsigned long long)v);
  }
}
}  // namespace

#define DTYPE_SWITCH(dtype, T, ...)                                   \
  do {                                                                \
    if ((dtype) == ADP_F32) { using T = float; __VA_ARGS__; }         \
    else if ((dtype) == ADP_BF16) { using T = bf16; __VA_ARGS__; }    \
    else { adp::set_error("unknown dtype"); return -1; }              \
  } while (0)

extern "C" int adp_head_softmax2_fwd(int dtype, size_t M, int Cs, int Cin, const void* x, const float* W,
                                     const float* b, const float* sc, const float* sh, float* p,
                                     adp_stream_t st) {
  ADP_REQUIRE(Cs % 8 == 0 && Cs <= 1024 && Cin <= Cs, "adp_head_softmax2_fwd: bad channels");
  DTYPE_SWITCH(dtype, T,
               launch_head_fwd<T, 2>(M, Cs, Cin, (const T*)x, W, b, sc, sh, p, (hipStream_t)st));
  return adp::check_launch("adp_head_softmax2_fwd");
}

extern "C" int adp_head_sigmoid_fwd(int dtype, size_t M, int Cs, int Cin, const void* x, const float* W,
                                    const float* b, const float* sc, const float* sh, float* p,
                                    adp_stream_t st) {
  ADP_REQUIRE(Cs % 8 == 0 && Cs <= 1024 && Cin <= Cs, "adp_head_sigmoid_fwd: bad channels");
  DTYPE_SWITCH(dtype, T,
               launch_head_fwd<T, 1>(M, Cs, Cin, (const T*)x, W, b, sc, sh, p, (hipStream_t)st));
  return adp::check_launch("adp_head_sigmoid_fwd");
}

template <int NOUT>
static int head_bwd(int dtype, size_t M, int Cs, int Cin, const void* x, const float* W, const float* sc,
                    const float* sh, const float* p, const float* dp, const void* addend, const void* mask,
                    float ms, void* dx, float* dW, float* db, hipStream_t s) {
  ADP_REQUIRE(Cs % 8 == 0 && Cs / 8 <= TPB, "head backward: Cs must be a multiple of 8 and <= 2048");
  int lanes = TPB / (Cs / 8);
  DTYPE_SWITCH(dtype, T, {
    const int cap = adp::option("head_bwd_blocks",
                                adp::resident_grid(reinterpret_cast<const void*>(&head_bwd_kernel<T, NOUT>), TPB));
    const int blocks = (int)std::min<size_t>((M + lanes - 1) / lanes, (size_t)cap);
    hipLaunchKernelGGL((head_bwd_kernel<T, NOUT>), dim3(blocks), dim3(TPB), 0, s, M, Cs, Cin, (const T*)x, W, sc, sh,
                       p, dp, (const T*)addend, (const T*)mask, ms, (T*)dx, dW, db);
  });
  return adp::check_launch("adp_head_bwd");
}

extern "C" int adp_head_softmax2_bwd(int dtype, size_t M, int Cs, int Cin, const void* x, const float* W,
                                     const float* sc, const float* sh, const float* p, const float* dp,
                                     const void* addend, const void* mask, float ms, void* dx, float* dW,
                                     float* db, adp_stream_t st) {
  return head_bwd<2>(dtype, M, Cs, Cin, x, W, sc, sh, p, dp, addend, mask, ms, dx, dW, db, (hipStream_t)st);
}

extern "C" int adp_head_sigmoid_bwd_bnr(int dtype, size_t M, int Cs, int Cin, const void* z, const float* W,
                                        const float* sc, const float* sh, const float* mean, const float* invstd,
                                        const float* p, const float* dp, void* dx, float* dW, float* db,
                                        float* dgamma, float* dbeta, adp_stream_t st) {
  ADP_REQUIRE(Cs % 8 == 0 && Cs / 8 <= TPB && Cin <= Cs && z && sc && sh && mean && invstd && dgamma && dbeta,
              "adp_head_sigmoid_bwd_bnr: Cs % 8 == 0, Cin <= Cs, all BatchNorm pointers");
  ADP_REQUIRE(Cs + Cin + 1 <= adp::STAT_CMAX, "adp_head_sigmoid_bwd_bnr: Cs + Cin too large");
  double* stat = adp::stat_scratch();
  if (!stat) return -1;
  const int lanes = TPB / (Cs / 8);
  // every block resident at once (measured at level 0: 233 us with 2 blocks per CU, 286 us with 4096)
  DTYPE_SWITCH(dtype, T, {
    const bool fast = adp::option("head_bwd_fast", 1) != 0;   // (sc / sh are required above)
    const void* kf = fast ? reinterpret_cast<const void*>(&head_bwd_kernel<T, 1, true, true>)
                          : reinterpret_cast<const void*>(&head_bwd_kernel<T, 1, true>);
    const int cap = adp::option("head_bwd_blocks", adp::resident_grid(kf, TPB));
    const int blocks = (int)std::min<size_t>((M + lanes - 1) / lanes, (size_t)cap);
    if (fast)
      hipLaunchKernelGGL((head_bwd_kernel<T, 1, true, true>), dim3(blocks), dim3(TPB), 0, (hipStream_t)st, M, Cs, Cin,
                         (const T*)z, W, sc, sh, p, dp, (const T*)nullptr, (const T*)nullptr, 1.f, (T*)dx, dW, db, mean,
                         invstd, stat);
    else
      hipLaunchKernelGGL((head_bwd_kernel<T, 1, true>), dim3(blocks), dim3(TPB), 0, (hipStream_t)st, M, Cs, Cin,
                         (const T*)z, W, sc, sh, p, dp, (const T*)nullptr, (const T*)nullptr, 1.f, (T*)dx, dW, db, mean,
                         invstd, stat);
  });
  if (adp::check_launch("adp_head_sigmoid_bwd_bnr")) return -2;
  if (adp::stat_fold_at(0, Cs, dbeta, dgamma, (hipStream_t)st)) return -2;
  if (adp::stat_fold_at(Cs, Cin, dW, nullptr, (hipStream_t)st)) return -2;
  return adp::stat_fold_at(Cs + Cin, 1, db, nullptr, (hipStream_t)st);
}

extern "C" int adp_head_sigmoid_bwd(int dtype, size_t M, int Cs, int Cin, const void* x, const float* W,
                                    const float* sc, const float* sh, const float* p, const float* dp,
                                    const void* addend, const void* mask, float ms, void* dx, float* dW,
                                    float* db, adp_stream_t st) {
  return head_bwd<1>(dtype, M, Cs, Cin, x, W, sc, sh, p, dp, addend, mask, ms, dx, dW, db, (hipStream_t)st);
}

extern "C" int adp_resize_bilinear_fwd(int N, int Hs, int Ws, int Ho, int Wo, const float* src, float* dst,
                                       adp_stream_t st) {
  ADP_REQUIRE(N > 0 && Hs > 0 && Ws > 0 && Ho > 0 && Wo > 0, "adp_resize_bilinear_fwd: bad dims");
  size_t n = (size_t)N * Ho * Wo;
  hipLaunchKernelGGL(resize_fwd_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, Hs, Ws, Ho, Wo, src, dst);
  return adp::check_launch("adp_resize_bilinear_fwd");
}

extern "C" int adp_resize_bilinear_bwd(int N, int Hs, int Ws, int Ho, int Wo, const float* dout, float* dsrc,
                                       adp_stream_t st) {
  ADP_REQUIRE(N > 0 && Hs > 0 && Ws > 0 && Ho >= Hs && Wo >= Ws, "adp_resize_bilinear_bwd: upsampling only");
  size_t n = (size_t)N * Hs * Ws;
  hipLaunchKernelGGL(resize_bwd_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, Hs, Ws, Ho, Wo, dout, dsrc);
  return adp::check_launch("adp_resize_bilinear_bwd");
}

extern "C" int adp_loss_rows(int N, int H, int W, const float* p, const float* y, int smooth, float ep,
                             float en, float* row_bce, double* stats, adp_stream_t st) {
  ADP_REQUIRE(N > 0 && H > 0 && W > 0, "adp_loss_rows: bad dims");
  const int lrb = std::min((N * H + TPB / 64 - 1) / (TPB / 64), 512);
  hipLaunchKernelGGL(loss_rows_kernel, dim3(lrb), dim3(TPB), 0, (hipStream_t)st, N, H, W, p, y, smooth, ep, en,
                     row_bce, stats);
  return adp::check_launch("adp_loss_rows");
}

extern "C" int adp_loss_select(int N, int H, int W, const float* row_bce, int ohem, float keep, float weight,
                               float norm_rows, float* row_coef, double* out, adp_stream_t st) {
  ADP_REQUIRE(H <= 2048, "adp_loss_select: H must be <= 2048");
  ADP_REQUIRE(norm_rows > 0, "adp_loss_select: norm_rows must be > 0");
  hipLaunchKernelGGL(loss_select_kernel, dim3(N), dim3(1024), 0, (hipStream_t)st, N, H, W, row_bce, ohem, keep,
                     weight, norm_rows, row_coef, out);
  return adp::check_launch("adp_loss_select");
}

extern "C" int adp_loss_grad(int N, int H, int W, const float* p, const float* y, int smooth, float ep,
                             float en, const float* row_coef, const double* stats, float weight, int accumulate,
                             float* dp, adp_stream_t st) {
  size_t n = (size_t)N * H * W;
  hipLaunchKernelGGL(loss_grad_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, H, W, p, y, smooth, ep,
                     en, row_coef, stats, weight, accumulate, dp);
  return adp::check_launch("adp_loss_grad");
}

extern "C" int adp_pixel_counts(size_t n, const float* pred, const float* truth, float thr,
                                unsigned long long* counts, adp_stream_t st) {
  hipLaunchKernelGGL(pixel_counts_kernel, dim3(nblk(n, 2048)), dim3(TPB), 0, (hipStream_t)st, n, pred, truth, thr,
                     counts);
  return adp::check_launch("adp_pixel_counts");
}

extern "C" int adp_threshold_hist(size_t n, const float* pred, const float* truth, int nthr, const double* thr,
                                  unsigned long long* hist, adp_stream_t st) {
  ADP_REQUIRE(nthr >= 1 && nthr <= 64 && thr && pred && truth && hist, "adp_threshold_hist: 1..64 thresholds");
  ThrList tl;
  for (int i = 0; i < nthr; ++i) {
    ADP_REQUIRE(i == 0 || thr[i] >= thr[i - 1], "adp_threshold_hist: thresholds must be ascending");
    tl.t[i] = thr[i];
  }
  hipLaunchKernelGGL(threshold_hist_kernel, dim3(nblk(n, 2048)), dim3(TPB), 0, (hipStream_t)st, n, pred, truth, nthr,
                     tl, hist);
  return adp::check_launch("adp_threshold_hist");
}
