// Implicit-GEMM convolution kernels on CDNA4 MFMA (gfx950).
//
// One forward-shaped kernel (adp_igemm_fwd) covers every dense layer of both presets:
//   * 3x3 'same' conv, any dilation           -> Keras Conv2D(...,3,padding='same',dilation_rate=d)
//                                                 (Segmentation/train_adipose_unet_v3.py:668-709)
//   * its data-gradient (same gather, pre-flipped/transposed weights)
//   * nearest-x2 upsample folded into the gather -> UpSampling2D((2,2)) + Conv2D (:691-692, :698-699, :705-706)
//   * two-source channel concat folded into K   -> Concatenate(axis=-1) + Conv2D (:693-694, :700-701, :707-708)
//   * ConvTranspose 2x2/s2 forward (pixel-shuffle store) and data-gradient (stride-2 4-tap gather)
//     for the north-star `unet_bn` preset (no reference code; BASELINE.json configs 2/3/5)
// Epilogue fusions: bias, ReLU, dropout (stateless hash mask), running-sum accumulate (dilated
// bottleneck Add, :688), residual addend + ReLU mask (backward), channel-split store (concat
// backward), per-channel sum / sum-of-squares (BatchNorm statistics).
//
// A second kernel (adp_igemm_wgrad) computes weight (+bias) gradients with a split-M reduction.
//
// Tiling: 256 threads = 4 waves (2x2), block tile 128(M pixels) x 64(N channels) x 32(K), register-
// staged double-buffered LDS, v_mfma_f32_16x16x32_bf16 (bf16) or v_mfma_f32_16x16x4_f32 (f32, exact).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 64, BK = 32, NT = 256;

template <typename T> struct LdsTr;
template <> struct LdsTr<bf16> { static constexpr int LDK = BK + 8; };   // 80 B rows
template <> struct LdsTr<float> { static constexpr int LDK = BK + 4; };  // 144 B rows

struct FwdArgs {
  const void* srcA; const void* srcB;
  const float* scA; const float* shA;   // BN-apply(+ReLU) on load of source A (nullable)
  const float* scB; const float* shB;
  int CAs, CBs;          // channel strides of the sources (%8 == 0); CBs == 0 -> single source
  int Nimg, Hs, Ws;      // source spatial dims
  int up;                // 1 or 2: nearest upsample folded into the gather
  int Ho, Wo, stride;    // output spatial, input stride
  int kh, kw, dil, pad;  // tap grid; input coord = o*stride + tap*dil - pad (virtual grid)
  const void* W; int Kpad; int K;
  const float* bias;
  int Nout;              // logical GEMM N
  int relu;
  uint32_t drop_seed; float drop_rate;   // drop_rate > 0 -> inverted dropout after ReLU
  void* out; int out_stride; int out_mode; int Cps;   // out_mode 0 plain, 1 pixel-shuffle, 2 split
  void* out2; int out2_stride; int split_c;
  const void* addend; int addend_stride;
  const void* mask; int mask_stride; float mask_scale;
  const void* mask2; int mask2_stride; float mask2_scale;
  float* accum; int accum_stride;
  float* bn_sum; float* bn_sq;
  int M;
  int ntile_n;           // gridDim decomposition helper
  int nblocks;
};

template <typename T>
ADP_DEV void load_a_group(const FwdArgs& a, Grp<T>& g, bool rowvalid, int n, int ybase, int xbase,
                          int tap, int ci, int k) {
  grp_zero(g);
  if (!rowvalid || k >= a.K) return;
  int ty = tap / a.kw, tx = tap - ty * a.kw;
  int yi = ybase + ty * a.dil - a.pad;
  int xi = xbase + tx * a.dil - a.pad;
  int Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  if (yi < 0 || xi < 0 || yi >= Hv || xi >= Wv) return;
  if (a.up == 2) { yi >>= 1; xi >>= 1; }
  size_t pix = ((size_t)n * a.Hs + yi) * a.Ws + xi;
  const float* sc; const float* sh;
  if (ci < a.CAs) {
    grp_load(g, reinterpret_cast<const T*>(a.srcA) + pix * a.CAs + ci);
    sc = a.scA; sh = a.shA;
  } else {
    ci -= a.CAs;
    grp_load(g, reinterpret_cast<const T*>(a.srcB) + pix * a.CBs + ci);
    sc = a.scB; sh = a.shB;
  }
  if (sc) {
    float f[8];
    grp_to_f(g, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[ci + j], sh[ci + j]), 0.f);
    grp_from_f(g, f);
  }
}

template <typename T>
ADP_DEV void mma_tile(const T* As, const T* Bs, int wr, int wc, int lane, f32x4 (&acc)[4][2]);

template <>
ADP_DEV void mma_tile<bf16>(const bf16* As, const bf16* Bs, int wr, int wc, int lane,
                            f32x4 (&acc)[4][2]) {
  constexpr int LDK = LdsTr<bf16>::LDK;
  const int r = lane & 15, kq = (lane >> 4) * 8;
  bf16x8 b[2];
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
    b[ni] = *reinterpret_cast<const bf16x8*>(Bs + (wc * 32 + ni * 16 + r) * LDK + kq);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    bf16x8 av = *reinterpret_cast<const bf16x8*>(As + (wr * 64 + mi * 16 + r) * LDK + kq);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
      acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b[ni], acc[mi][ni], 0, 0, 0);
  }
}

template <>
ADP_DEV void mma_tile<float>(const float* As, const float* Bs, int wr, int wc, int lane,
                             f32x4 (&acc)[4][2]) {
  constexpr int LDK = LdsTr<float>::LDK;
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < BK; ks += 4) {
    float b0 = Bs[(wc * 32 + r) * LDK + ks + kq];
    float b1 = Bs[(wc * 32 + 16 + r) * LDK + ks + kq];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      float av = As[(wr * 64 + mi * 16 + r) * LDK + ks + kq];
      acc[mi][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc[mi][0], 0, 0, 0);
      acc[mi][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc[mi][1], 0, 0, 0);
    }
  }
}

// XCD-aware bijective remap of the linear block id: each XCD (blocks b, b+8, ...) receives a
// contiguous run of tiles, N-tile fastest, so the A (activation) panel of one M-tile is shared
// through one XCD's L2 by all its N-tiles.
ADP_DEV int xcd_remap(int bid, int nwg) {
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <typename T>
__global__ __launch_bounds__(NT) void igemm_fwd_kernel(FwdArgs a) {
  constexpr int LDK = LdsTr<T>::LDK;
  __shared__ __attribute__((aligned(16))) T As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * LDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int lin = xcd_remap(blockIdx.x, a.nblocks);
  const int tn = lin % a.ntile_n, tm = lin / a.ntile_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // A staging: thread owns rows (tid>>2) and (tid>>2)+64, k-group tid&3.
  const int kg = tid & 3;
  int an[2], ay[2], ax[2];
  bool av[2];
  const int HWo = a.Ho * a.Wo;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int m = m0 + (tid >> 2) + i * 64;
    av[i] = m < a.M;
    int mm = av[i] ? m : 0;
    an[i] = mm / HWo;
    int rem = mm - an[i] * HWo;
    int yo = rem / a.Wo;
    ay[i] = yo * a.stride;
    ax[i] = (rem - yo * a.Wo) * a.stride;
  }
  const int Cin_s = a.CAs + a.CBs;
  int k = kg * 8;
  int tap = k / Cin_s, ci = k - tap * Cin_s;
  // B staging: thread owns weight row n0 + (tid>>2), k-group tid&3.
  const T* Wp = reinterpret_cast<const T*>(a.W) + (size_t)(n0 + (tid >> 2)) * a.Kpad + kg * 8;

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Grp<T> ga[2], gb;
  const int nk = a.Kpad / BK;
  // prologue
#pragma unroll
  for (int i = 0; i < 2; ++i) load_a_group<T>(a, ga[i], av[i], an[i], ay[i], ax[i], tap, ci, k);
  grp_load(gb, Wp);
#pragma unroll
  for (int i = 0; i < 2; ++i) grp_store(ga[i], &As[0][((tid >> 2) + i * 64) * LDK + kg * 8]);
  grp_store(gb, &Bs[0][(tid >> 2) * LDK + kg * 8]);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      k += BK; ci += BK;
      while (ci >= Cin_s) { ci -= Cin_s; ++tap; }
#pragma unroll
      for (int i = 0; i < 2; ++i) load_a_group<T>(a, ga[i], av[i], an[i], ay[i], ax[i], tap, ci, k);
      grp_load(gb, Wp + (size_t)(kt + 1) * BK);
    }
    mma_tile<T>(As[cur], Bs[cur], wr, wc, lane, acc);
    if (more) {
#pragma unroll
      for (int i = 0; i < 2; ++i) grp_store(ga[i], &As[cur ^ 1][((tid >> 2) + i * 64) * LDK + kg * 8]);
      grp_store(gb, &Bs[cur ^ 1][(tid >> 2) * LDK + kg * 8]);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const int col = lane & 15, rq = (lane >> 4) * 4;
  float bsum[2] = {0.f, 0.f}, bsq[2] = {0.f, 0.f};
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int n = n0 + wc * 32 + ni * 16 + col;
    const bool nvalid = n < a.Nout;
    const float bias = (nvalid && a.bias) ? a.bias[a.out_mode == 1 ? n % a.Cps : n] : 0.f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 64 + mi * 16 + rq + r;
        if (!nvalid || m >= a.M) continue;
        float v = acc[mi][ni][r] + bias;
        if (a.relu) v = fmaxf(v, 0.f);
        if (a.drop_rate > 0.f) {
          float u = adp_uniform(a.drop_seed, (uint64_t)m * (uint64_t)a.Nout + n);
          v = (u >= a.drop_rate) ? v * (1.f / (1.f - a.drop_rate)) : 0.f;
        }
        if (a.out_mode == 1) {
          // ConvTranspose 2x2/s2: n = sub*Cps + c, sub = 2*dy + dx
          int sub = n / a.Cps, c = n - sub * a.Cps;
          int nimg = m / HWo, rem = m - nimg * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
          size_t pix = ((size_t)nimg * (2 * a.Ho) + 2 * yo + (sub >> 1)) * (2 * a.Wo) + 2 * xo + (sub & 1);
          reinterpret_cast<T*>(a.out)[pix * a.out_stride + c] = from_f<T>(v);
          if (a.bn_sum) { bsum[ni] += v; bsq[ni] += v * v; }
          continue;
        }
        if (a.out_mode == 2 && n >= a.split_c) {
          const int c = n - a.split_c;
          if (a.mask2) {
            float mv = to_f(reinterpret_cast<const T*>(a.mask2)[(size_t)m * a.mask2_stride + c]);
            v = mv > 0.f ? v * a.mask2_scale : 0.f;
          }
          reinterpret_cast<T*>(a.out2)[(size_t)m * a.out2_stride + c] = from_f<T>(v);
          continue;
        }
        if (!a.out) continue;
        if (a.addend) v += to_f(reinterpret_cast<const T*>(a.addend)[(size_t)m * a.addend_stride + n]);
        if (a.mask) {
          float mv = to_f(reinterpret_cast<const T*>(a.mask)[(size_t)m * a.mask_stride + n]);
          v = mv > 0.f ? v * a.mask_scale : 0.f;
        }
        const T vs = from_f<T>(v);
        reinterpret_cast<T*>(a.out)[(size_t)m * a.out_stride + n] = vs;
        if (a.accum) a.accum[(size_t)m * a.accum_stride + n] += to_f(vs);
        if (a.bn_sum) { bsum[ni] += v; bsq[ni] += v * v; }
      }
    }
  }
  if (a.bn_sum) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      float s = bsum[ni], q = bsq[ni];
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      const int n = n0 + wc * 32 + ni * 16 + col;
      if (lane < 16 && n < a.Nout) {
        int c = a.out_mode == 1 ? n % a.Cps : n;
        atomicAdd(a.bn_sum + c, s);
        atomicAdd(a.bn_sq + c, q);
      }
    }
  }
}

// ------------------------------------------------------------------------------------ wgrad
struct WgradArgs {
  const void* srcA; const void* srcB;
  const float* scA; const float* shA; const float* scB; const float* shB;
  int CAs, CBs, Nimg, Hs, Ws, up, Ho, Wo, stride, kh, kw, dil, pad;
  int K, Kpad;
  const void* dY; int dy_stride; int dy_mode; int Cps;   // dy_mode 0 plain [M][N], 1 pixel-shuffle gather
  int Nout;
  float* dW;            // [Npad][Kpad] f32, accumulated with atomics
  float* dB;            // [Nout] f32 or null
  int M, mchunk, ntile_k, ntile_n;
};

template <typename T> struct WTr;
template <> struct WTr<bf16> { static constexpr int LDM = 32 + 8; };
template <> struct WTr<float> { static constexpr int LDM = 32 + 1; };

template <typename T>
ADP_DEV void wg_mma(const T* Ds, const T* Xs, int wr, int wc, int lane, f32x4 (&acc)[2][2]);

template <>
ADP_DEV void wg_mma<bf16>(const bf16* Ds, const bf16* Xs, int wr, int wc, int lane, f32x4 (&acc)[2][2]) {
  constexpr int L = WTr<bf16>::LDM;
  const int r = lane & 15, kq = (lane >> 4) * 8;
  bf16x8 b[2];
  // Xs/Ds are [row][m] with 80-B rows: 8 consecutive m of one row are one aligned 16-B read.
#pragma unroll
  for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Xs + (wc * 32 + j * 16 + r) * L + kq);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    bf16x8 av = *reinterpret_cast<const bf16x8*>(Ds + (wr * 32 + i * 16 + r) * L + kq);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b[j], acc[i][j], 0, 0, 0);
  }
}

template <>
ADP_DEV void wg_mma<float>(const float* Ds, const float* Xs, int wr, int wc, int lane, f32x4 (&acc)[2][2]) {
  constexpr int L = WTr<float>::LDM;
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < 32; ks += 4) {
    float b0 = Xs[(wc * 32 + r) * L + ks + kq];
    float b1 = Xs[(wc * 32 + 16 + r) * L + ks + kq];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float av = Ds[(wr * 32 + i * 16 + r) * L + ks + kq];
      acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc[i][0], 0, 0, 0);
      acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc[i][1], 0, 0, 0);
    }
  }
}

// dW[n][k] += sum_m dY[m][n] * X_tap(k)[m]; output tile 64(n) x 64(k), M split over blockIdx.y.
template <typename T>
__global__ __launch_bounds__(NT) void igemm_wgrad_kernel(WgradArgs a) {
  constexpr int L = WTr<T>::LDM;
  __shared__ __attribute__((aligned(16))) T Ds[64 * L];
  __shared__ __attribute__((aligned(16))) T Xs[64 * L];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int tk = blockIdx.x % a.ntile_k, tn = blockIdx.x / a.ntile_k;
  const int k0 = tk * 64, n0 = tn * 64;
  const int mbeg = blockIdx.y * a.mchunk;
  const int mend = min(a.M, mbeg + a.mchunk);
  if (mbeg >= mend) return;

  const int row = tid >> 3, g = tid & 7;   // staging: pixel row 0..31, 8-wide group 0..7
  const int Cin_s = a.CAs + a.CBs;
  const int k = k0 + g * 8;
  const int tap = k < a.K ? k / Cin_s : 0;
  int ci = k - tap * Cin_s;
  const int ty = tap / a.kw, tx = tap - ty * a.kw;
  const int n = n0 + g * 8;
  const int HWo = a.Ho * a.Wo;
  const int Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  const bool useB = ci >= a.CAs;
  const int cl = useB ? ci - a.CAs : ci;
  const T* src = reinterpret_cast<const T*>(useB ? a.srcB : a.srcA);
  const int cs = useB ? a.CBs : a.CAs;
  const float* sc = useB ? a.scB : a.scA;
  const float* sh = useB ? a.shB : a.shA;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;

  for (int mb = mbeg; mb < mend; mb += 32) {
    const int m = mb + row;
    Grp<T> gx, gd;
    grp_zero(gx); grp_zero(gd);
    if (m < mend) {
      int nimg = m / HWo, rem = m - nimg * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
      if (k < a.K) {
        int yi = yo * a.stride + ty * a.dil - a.pad, xi = xo * a.stride + tx * a.dil - a.pad;
        if (yi >= 0 && xi >= 0 && yi < Hv && xi < Wv) {
          if (a.up == 2) { yi >>= 1; xi >>= 1; }
          grp_load(gx, src + (((size_t)nimg * a.Hs + yi) * a.Ws + xi) * cs + cl);
          if (sc) {
            float f[8];
            grp_to_f(gx, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[cl + j], sh[cl + j]), 0.f);
            grp_from_f(gx, f);
          }
        }
      }
      if (n < a.Nout) {
        const T* dy = reinterpret_cast<const T*>(a.dY);
        if (a.dy_mode == 0) {
          grp_load(gd, dy + (size_t)m * a.dy_stride + n);
        } else {
          int sub = n / a.Cps, c = n - sub * a.Cps;
          size_t pix = ((size_t)nimg * (2 * a.Ho) + 2 * yo + (sub >> 1)) * (2 * a.Wo) + 2 * xo + (sub & 1);
          grp_load(gd, dy + pix * a.dy_stride + c);
        }
      }
    }
    __syncthreads();
    {
      const T* ex = reinterpret_cast<const T*>(&gx);
      const T* ed = reinterpret_cast<const T*>(&gd);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Xs[(g * 8 + j) * L + row] = ex[j];
        Ds[(g * 8 + j) * L + row] = ed[j];
      }
    }
    __syncthreads();
    wg_mma<T>(Ds, Xs, wr, wc, lane, acc);
    if (a.dB && tk == 0 && tid < 64) {
#pragma unroll 8
      for (int j = 0; j < 32; ++j) dbacc += to_f(Ds[tid * L + j]);
    }
  }

  const int col = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nn = n0 + wr * 32 + i * 16 + rq + r;
        const int kk = k0 + wc * 32 + j * 16 + col;
        if (nn < a.Nout && kk < a.K) atomicAdd(a.dW + (size_t)nn * a.Kpad + kk, acc[i][j][r]);
      }
  if (a.dB && tk == 0 && tid < 64 && n0 + tid < a.Nout)
    atomicAdd(a.dB + (a.dy_mode == 1 ? (n0 + tid) % a.Cps : n0 + tid), dbacc);
}

}  // namespace

// ============================================================================ C ABI
#include "../../include/adipose_hip.h"

namespace {
template <typename T>
int launch_fwd(const adp_conv_desc* d, const adp_conv_io* io, hipStream_t s) {
  FwdArgs a{};
  a.srcA = io->srcA; a.srcB = io->srcB;
  a.scA = io->bn_scaleA; a.shA = io->bn_shiftA; a.scB = io->bn_scaleB; a.shB = io->bn_shiftB;
  a.CAs = d->CA_stride; a.CBs = d->CB_stride;
  a.Nimg = d->N; a.Hs = d->Hs; a.Ws = d->Ws; a.up = d->upsample ? 2 : 1;
  a.Ho = d->Ho; a.Wo = d->Wo; a.stride = d->stride;
  a.kh = d->kh; a.kw = d->kw; a.dil = d->dil; a.pad = d->pad;
  a.W = io->W; a.K = d->kh * d->kw * (d->CA_stride + d->CB_stride); a.Kpad = (a.K + 31) / 32 * 32;
  a.bias = io->bias; a.Nout = d->Nout; a.relu = d->relu;
  a.drop_seed = d->dropout_seed; a.drop_rate = d->dropout_rate;
  a.out = io->out; a.out_stride = d->out_stride; a.out_mode = d->out_mode; a.Cps = d->shuffle_c;
  a.out2 = io->out2; a.out2_stride = d->out2_stride; a.split_c = d->split_c;
  a.addend = io->addend; a.addend_stride = d->out_stride;
  a.mask = io->mask; a.mask_stride = d->mask_stride; a.mask_scale = d->mask_scale;
  a.mask2 = io->mask2; a.mask2_stride = d->mask2_stride; a.mask2_scale = d->mask2_scale;
  a.accum = io->accum; a.accum_stride = d->accum_stride;
  a.bn_sum = io->bn_sum; a.bn_sq = io->bn_sqsum;
  a.M = d->N * d->Ho * d->Wo;
  ADP_REQUIRE(a.CAs % 8 == 0 && a.CBs % 8 == 0, "adp_conv_fwd: channel strides must be multiples of 8");
  ADP_REQUIRE(a.M > 0 && a.Nout > 0, "adp_conv_fwd: empty problem");
  ADP_REQUIRE(d->out_mode != 1 || (d->shuffle_c > 0 && d->Nout % d->shuffle_c == 0), "adp_conv_fwd: bad shuffle_c");
  ADP_REQUIRE(d->out_mode != 2 || (io->out2 && d->split_c > 0), "adp_conv_fwd: split store needs out2/split_c");
  a.ntile_n = (a.Nout + BN - 1) / BN;
  const int ntm = (a.M + BM - 1) / BM;
  a.nblocks = ntm * a.ntile_n;
  hipLaunchKernelGGL(igemm_fwd_kernel<T>, dim3(a.nblocks), dim3(NT), 0, s, a);
  return adp::check_launch("adp_conv_fwd");
}

template <typename T>
int launch_wgrad(const adp_conv_desc* d, const adp_conv_io* io, const void* dY, int dy_stride,
                 float* dW, float* dB, hipStream_t s) {
  WgradArgs a{};
  a.srcA = io->srcA; a.srcB = io->srcB;
  a.scA = io->bn_scaleA; a.shA = io->bn_shiftA; a.scB = io->bn_scaleB; a.shB = io->bn_shiftB;
  a.CAs = d->CA_stride; a.CBs = d->CB_stride; a.Nimg = d->N; a.Hs = d->Hs; a.Ws = d->Ws;
  a.up = d->upsample ? 2 : 1; a.Ho = d->Ho; a.Wo = d->Wo; a.stride = d->stride;
  a.kh = d->kh; a.kw = d->kw; a.dil = d->dil; a.pad = d->pad;
  a.K = d->kh * d->kw * (d->CA_stride + d->CB_stride); a.Kpad = (a.K + 31) / 32 * 32;
  a.dY = dY; a.dy_stride = dy_stride; a.dy_mode = d->out_mode == 1 ? 1 : 0; a.Cps = d->shuffle_c;
  a.Nout = d->Nout; a.dW = dW; a.dB = dB;
  a.M = d->N * d->Ho * d->Wo;
  ADP_REQUIRE(a.CAs % 8 == 0 && a.CBs % 8 == 0 && a.Nout % 8 == 0,
              "adp_conv_wgrad: channel strides and Nout must be multiples of 8");
  ADP_REQUIRE(d->out_mode != 2, "adp_conv_wgrad: split-store descriptors are dgrad-only");
  a.ntile_k = (a.K + 63) / 64;
  a.ntile_n = (a.Nout + 63) / 64;
  const int tiles = a.ntile_k * a.ntile_n;
  int splits = (2048 + tiles - 1) / tiles;
  int maxsplit = (a.M + 255) / 256;
  if (splits > maxsplit) splits = maxsplit;
  if (splits < 1) splits = 1;
  a.mchunk = ((a.M + splits - 1) / splits + 31) / 32 * 32;
  splits = (a.M + a.mchunk - 1) / a.mchunk;
  hipLaunchKernelGGL(igemm_wgrad_kernel<T>, dim3(tiles, splits), dim3(NT), 0, s, a);
  return adp::check_launch("adp_conv_wgrad");
}
}  // namespace

extern "C" int adp_conv_fwd(int dtype, const adp_conv_desc* d, const adp_conv_io* io, adp_stream_t st) {
  hipStream_t s = (hipStream_t)st;
  ADP_REQUIRE(d && io, "adp_conv_fwd: null descriptor");
  if (dtype == ADP_F32) return launch_fwd<float>(d, io, s);
  if (dtype == ADP_BF16) return launch_fwd<bf16>(d, io, s);
  adp::set_error("adp_conv_fwd: unknown dtype");
  return -1;
}

extern "C" int adp_conv_wgrad(int dtype, const adp_conv_desc* d, const adp_conv_io* io, const void* dY,
                              int dy_stride, float* dW, float* dB, adp_stream_t st) {
  hipStream_t s = (hipStream_t)st;
  ADP_REQUIRE(d && io && dY && dW, "adp_conv_wgrad: null argument");
  if (dtype == ADP_F32) return launch_wgrad<float>(d, io, dY, dy_stride, dW, dB, s);
  if (dtype == ADP_BF16) return launch_wgrad<bf16>(d, io, dY, dy_stride, dW, dB, s);
  adp::set_error("adp_conv_wgrad: unknown dtype");
  return -1;
}
