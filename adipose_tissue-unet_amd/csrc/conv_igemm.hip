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
#include "conv_common.h"
#include <type_traits>

namespace {

constexpr int BM = 128, BN = 64, BK = 32, NT = 256;

template <typename T> struct LdsTr;
template <> struct LdsTr<bf16> { static constexpr int LDK = BK + 8; };   // 80 B rows
template <> struct LdsTr<float> { static constexpr int LDK = BK + 4; };  // 144 B rows


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


// Shared epilogue of the forward-shaped kernels: acc[mi][ni] holds the 16x16 MFMA tile whose
// rows are mbase + mi*16 + 4*(lane>>4) + r and columns nbase + ni*16 + (lane&15).
template <typename T, int MI, int NI>
ADP_DEV void fwd_epilogue(const FwdArgs& a, f32x4 (&acc)[MI][NI], int mbase, int nbase, int lane) {
  const int col = lane & 15, rq = (lane >> 4) * 4;
  const int HWo = a.Ho * a.Wo;
  float bsum[NI], bsq[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) { bsum[ni] = 0.f; bsq[ni] = 0.f; }
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int n = nbase + ni * 16 + col;
    const bool nvalid = n < a.Nout;
    const float bias = (nvalid && a.bias) ? a.bias[a.out_mode == 1 ? n % a.Cps : n] : 0.f;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mbase + mi * 16 + rq + r;
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
          if (a.bn_sum) { bsum[ni] += v; bsq[ni] += v * v; }
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
    for (int ni = 0; ni < NI; ++ni) {
      float s = bsum[ni], q = bsq[ni];
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      const int n = nbase + ni * 16 + col;
      if (lane < 16 && n < a.Nout) {
        int c = a.out_mode == 1 ? n % a.Cps : n;
        if (a.stat) {   // the block's f64 replica (folded in a fixed order by the launcher: deterministic sums)
          double* rep = a.stat + (size_t)((blockIdx.x + blockIdx.y * gridDim.x) & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
          atomicAdd(rep + c, (double)s);
          atomicAdd(rep + adp::STAT_CMAX + c, (double)q);
        } else {
          atomicAdd(a.bn_sum + c, s);
          atomicAdd(a.bn_sq + c, q);
        }
      }
    }
  }
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

  fwd_epilogue<T, 4, 2>(a, acc, m0 + wr * 64, n0 + wc * 32, lane);
}

// LDS-staged epilogue of the bf16 throughput kernel: every wave dumps its f32 accumulators into a
// [BM][BN+4] LDS tile, then each thread finishes whole 8-channel groups (16-B loads of addend/mask,
// 16-B stores), keeping per-thread BN partial sums for a fixed channel group.
template <int BM, int BN>
ADP_DEV void fwd_epilogue_lds(const FwdArgs& a, f32x4 (&acc)[4][4], float* tile, int m0, int n0, int wr,
                              int wc, int tid) {
  constexpr int LT = BN + 4;
  const int lane = tid & 63, col = lane & 15, rq = (lane >> 4) * 4;
  __syncthreads();  // main loop LDS reads done before the tile overwrites the staging buffers
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        tile[(wr * 64 + mi * 16 + rq + r) * LT + wc * 64 + ni * 16 + col] = acc[mi][ni][r];
  __syncthreads();
  float bs[8], bq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bs[j] = 0.f; bq[j] = 0.f; }
  epi_rows<NT, BN>(a, tile, BM, m0, n0, tid, bs, bq);
  if (a.bn_sum) epi_bn_flush<NT, BN>(a, tile, n0, tid, bs, bq);
}

// --------------------------------------------------------------- bf16 throughput forward kernel
// 4 waves, each owning a 64x64 output tile (16 accumulators of 16x16), block tile BM x BN with
// BM*BN = 4*64*64, BK = 64 per LDS stage (two MFMA k-substeps per barrier, 32 MFMAs per wave per
// barrier), register-staged double buffer, 2 blocks per CU. Same gather/epilogue semantics as
// igemm_fwd_kernel.
template <int BM, int BN>
__global__ __launch_bounds__(NT, 2) void igemm_fwd_bf16_kernel(FwdArgs a) {
  constexpr int WN = BN / 64;
  constexpr int LDK = 64 + 8;            // 144-B rows
  constexpr int AG = BM / 32, BG = BN / 32;  // 16-B groups per thread per stage
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (BM + BN) * LDK];
  // stage b: A tile at smem + b*(BM+BN)*LDK, B tile right after it
#define ADP_AS(b) (smem + (b) * (BM + BN) * LDK)
#define ADP_BS(b) (smem + (b) * (BM + BN) * LDK + BM * LDK)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int lin = xcd_remap(blockIdx.x, a.nblocks);
  const int tn = lin % a.ntile_n, tm = lin / a.ntile_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kg = tid & 7, prow = tid >> 3;   // group column (8 per 64-wide k row), base row

  int an[AG], ay[AG], ax[AG];
  bool av[AG];
  const int HWo = a.Ho * a.Wo;
#pragma unroll
  for (int i = 0; i < AG; ++i) {
    int m = m0 + prow + 32 * i;
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
  const bf16* Wp = reinterpret_cast<const bf16*>(a.W) + (size_t)(n0 + prow) * a.Kpad + kg * 8;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Grp<bf16> ga[AG], gb[BG];
  const int nk = (a.Kpad + 63) / 64;
  auto load_stage = [&](int kt) {
#pragma unroll
    for (int i = 0; i < AG; ++i) load_a_group<bf16>(a, ga[i], av[i], an[i], ay[i], ax[i], tap, ci, k);
    const bool kin = kt * 64 + kg * 8 < a.Kpad;
#pragma unroll
    for (int j = 0; j < BG; ++j) {
      if (kin) grp_load(gb[j], Wp + (size_t)(32 * j) * a.Kpad + (size_t)kt * 64);
      else grp_zero(gb[j]);
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AG; ++i) grp_store(ga[i], ADP_AS(buf) + (prow + 32 * i) * LDK + kg * 8);
#pragma unroll
    for (int j = 0; j < BG; ++j) grp_store(gb[j], ADP_BS(buf) + (prow + 32 * j) * LDK + kg * 8);
  };

  load_stage(0);
  store_stage(0);
  __syncthreads();
  const int r = lane & 15, kq = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      k += 64; ci += 64;
      while (ci >= Cin_s) { ci -= Cin_s; ++tap; }
      load_stage(kt + 1);
    }
    const bf16* A = ADP_AS(cur) + (wr * 64 + r) * LDK + kq;
    const bf16* Bq = ADP_BS(cur) + (wc * 64 + r) * LDK + kq;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 b[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) b[ni] = *reinterpret_cast<const bf16x8*>(Bq + ni * 16 * LDK + s * 32);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        bf16x8 av8 = *reinterpret_cast<const bf16x8*>(A + mi * 16 * LDK + s * 32);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av8, b[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    if (more) store_stage(cur ^ 1);
    __syncthreads();
  }
  fwd_epilogue_lds<BM, BN>(a, acc, reinterpret_cast<float*>(smem), m0, n0, wr, wc, tid);
#undef ADP_AS
#undef ADP_BS
}

// ------------------------------------------------------ bf16 forward kernel, LDS-DMA staged ("glds")
// Same GEMM decomposition as igemm_fwd_bf16_kernel (4 waves x 64x64, BK = 64) but both operands are
// moved HBM/L2 -> LDS by global_load_lds_dwordx4 (no VGPR staging, so a whole stage is in flight per
// wave while the previous stage computes). The implicit-GEMM gather is the per-lane SOURCE address;
// padding taps read a zero page. The LDS image is linear (128-B rows, 8 x 16-B chunks); chunk c of
// tile row r is stored at position c ^ ((r >> 1) & 7), a swizzle that makes the ds_read_b128 fragment
// reads of the 16x16x32 MFMA bank-conflict free. No BN-on-load (the BN preset materialises its
// activations for this path).
__device__ __attribute__((aligned(256))) uint4 adp_zero_page[64];

template <int BM, int BN>
__global__ __launch_bounds__(NT, 2) void igemm_fwd_glds_kernel(FwdArgs a) {
  constexpr int WN = BN / 64;
  constexpr int ROWB = 128;                         // bytes per LDS row (64 bf16)
  constexpr int STAGE = (BM + BN) * ROWB;           // bytes per stage
  constexpr int AI = BM / 32, BI = BN / 32;         // glds instructions per wave per stage
  constexpr int EPI = BM * (BN + 4) * 4;            // epilogue tile bytes
  constexpr int SMEM = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WN, wc = wave % WN;
  const int lin = xcd_remap(blockIdx.x, a.nblocks);
  const int tn = lin % a.ntile_n, tm = lin / a.ntile_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lrow = lane >> 3, pos = lane & 7;
  const int HWo = a.Ho * a.Wo, Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  const int Cin_s = a.CAs + a.CBs;
  const int Wrows = (a.Nout + 63) / 64 * 64;

  // A: this wave loads tile rows [wave*BM/4, (wave+1)*BM/4), 8 rows per instruction
  int a_n[AI], a_y[AI], a_x[AI], a_tap[AI], a_ci[AI], a_ty[AI], a_tx[AI], a_k[AI];
  bool a_v[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = wave * (BM / 4) + 8 * i + lrow;
    const int m = m0 + r;
    a_v[i] = m < a.M;
    const int mm = a_v[i] ? m : 0;
    a_n[i] = mm / HWo;
    const int rem = mm - a_n[i] * HWo, yo = rem / a.Wo;
    a_y[i] = yo * a.stride - a.pad;
    a_x[i] = (rem - yo * a.Wo) * a.stride - a.pad;
    const int c = pos ^ swz(r);
    a_k[i] = 8 * c;
    a_tap[i] = a_k[i] / Cin_s;
    a_ci[i] = a_k[i] - a_tap[i] * Cin_s;
    a_ty[i] = a_tap[i] / a.kw;
    a_tx[i] = a_tap[i] - a_ty[i] * a.kw;
  }
  // B: tile rows [wave*BN/4, ...)
  const bf16* b_src[BI];
  int b_c[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int r = wave * (BN / 4) + 8 * i + lrow;
    b_c[i] = pos ^ swz(r);
    b_src[i] = (n0 + r < Wrows) ? reinterpret_cast<const bf16*>(a.W) + (size_t)(n0 + r) * a.Kpad + 8 * b_c[i] : nullptr;
  }
  const bf16* srcA = reinterpret_cast<const bf16*>(a.srcA);
  const bf16* srcB = reinterpret_cast<const bf16*>(a.srcB);

  auto issue = [&](int kt, int buf) {
    unsigned char* sb = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const void* p = adp_zero_page;
      if (a_v[i] && a_k[i] < a.K) {
        int yi = a_y[i] + a_ty[i] * a.dil, xi = a_x[i] + a_tx[i] * a.dil;
        if (yi >= 0 && xi >= 0 && yi < Hv && xi < Wv) {
          if (a.up == 2) { yi >>= 1; xi >>= 1; }
          const size_t pix = ((size_t)a_n[i] * a.Hs + yi) * a.Ws + xi;
          p = a_ci[i] < a.CAs ? (const void*)(srcA + pix * a.CAs + a_ci[i])
                              : (const void*)(srcB + pix * a.CBs + (a_ci[i] - a.CAs));
        }
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(sb + (wave * (BM / 4) + 8 * i) * ROWB), 16, 0, 0);
      // advance this slot's K position by one stage (64)
      a_k[i] += 64;
      a_ci[i] += 64;
      while (a_ci[i] >= Cin_s) {
        a_ci[i] -= Cin_s;
        if (++a_tx[i] == a.kw) { a_tx[i] = 0; ++a_ty[i]; }
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const void* p = adp_zero_page;
      if (b_src[i] && kt * 64 + 8 * b_c[i] < a.Kpad) p = b_src[i] + (size_t)kt * 64;
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(sb + BM * ROWB + (wave * (BN / 4) + 8 * i) * ROWB), 16, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.Kpad + 63) / 64;
  const int r16 = lane & 15, h = lane >> 4;
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      issue(kt + 1, cur ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AI + BI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const unsigned char* sA = smem + cur * STAGE;
    const unsigned char* sB = sA + BM * ROWB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + h;
      bf16x8 b[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = wc * 64 + ni * 16 + r16;
        b[ni] = *reinterpret_cast<const bf16x8*>(sB + row * ROWB + ((c ^ swz(row)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = wr * 64 + mi * 16 + r16;
        const bf16x8 av8 = *reinterpret_cast<const bf16x8*>(sA + row * ROWB + ((c ^ swz(row)) << 4));
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av8, b[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  fwd_epilogue_lds<BM, BN>(a, acc, reinterpret_cast<float*>(smem), m0, n0, wr, wc, tid);
}

// ------------------------------------------------------------------------------------ wgrad

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

// ------------------------------------------------------------------- bf16 throughput wgrad kernel
// dW[n][k] += sum_m dY[m][n] X(k)[m]. Block tile TN (n) x TK (k); 4 waves, each a 64x64 output tile;
// 64 pixels per LDS stage (2 MFMA k-substeps, 32 MFMAs per wave per barrier).
// Both operands are staged in their natural [pixel][channel] layout (coalesced 16-B loads, one
// ds_write_b128 per group) and fed to v_mfma_f32_16x16x32_bf16 with ds_read_b64_tr_b16, which
// transposes on the read (MFMA k = pixel). The pixel (reduction) order inside a 32-pixel substep is
// permuted, rho(8g+e) = 16(g>>1) + 8(e>>2) + 4(g&1) + (e&3), so that the 8 rows one 32-lane half reads
// are 8 consecutive LDS rows; with row strides of 32*odd bytes that read is bank-conflict free.

ADP_DEV bf16x8 tr_frag(const bf16* lds_base, int row0, int rowstride_el, int col0, int lane) {
  // lane (g = lane>>4, i = lane&15 = 4q+p) -> 8 consecutive k (pixels) of column col0 + i
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int rlo = 16 * (g >> 1) + 4 * (g & 1) + q;   // e = q      (rho(8g+q))
  const bf16* a0 = lds_base + (row0 + rlo) * rowstride_el + col0 + 4 * p;
  const bf16* a1 = a0 + 8 * rowstride_el;             // e = 4 + q  (rho(8g+4+q))
  v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(a0));
  v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(a1));
  bf16x8 r;
  const bf16* l = reinterpret_cast<const bf16*>(&lo);
  const bf16* h = reinterpret_cast<const bf16*>(&hi);
#pragma unroll
  for (int e = 0; e < 4; ++e) { r[e] = l[e]; r[4 + e] = h[e]; }
  return r;
}

template <int TN, int TK>
__global__ __launch_bounds__(NT, 2) void igemm_wgrad_bf16_kernel(WgradArgs a) {
  constexpr int MS = 64;                        // pixels per stage
  constexpr int LX = TK + 16, LD = TN + 16;     // row strides (elements): 2*T + 32 bytes
  constexpr int WK = TK / 64;                   // waves along k
  constexpr int GXR = TK / 8, GDR = TN / 8;     // 16-B groups per staged row
  constexpr int GX = MS * GXR / NT, GD = MS * GDR / NT;  // groups per thread
  constexpr int RX = NT / GXR, RD = NT / GDR;   // row step between a thread's groups
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * MS * (LX + LD)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WK, wk = wave % WK;
  const int tk = blockIdx.x % a.ntile_k, tn = blockIdx.x / a.ntile_k;
  const int k0 = tk * TK, n0 = tn * TN;
  const int mbeg = blockIdx.y * a.mchunk;
  const int mend = min(a.M, mbeg + a.mchunk);
  if (mbeg >= mend) return;

  // X staging: fixed k-group per thread -> fixed tap / channel / source
  const int kgx = tid % GXR, rowx = tid / GXR;
  const int Cin_s = a.CAs + a.CBs;
  const int k = k0 + kgx * 8;
  const bool kvalid = k < a.K;
  const int tap = kvalid ? k / Cin_s : 0;
  const int ci = k - tap * Cin_s;
  const int ty = tap / a.kw, tx = tap - ty * a.kw;
  const bool useB = ci >= a.CAs;
  const int cl = useB ? ci - a.CAs : ci;
  const bf16* src = reinterpret_cast<const bf16*>(useB ? a.srcB : a.srcA);
  const int cs = useB ? a.CBs : a.CAs;
  const float* sc = useB ? a.scB : a.scA;
  const float* sh = useB ? a.shB : a.shA;
  // dY staging
  const int cgd = tid % GDR, rowd = tid / GDR;
  const int nn = n0 + cgd * 8;
  const bool nvalid = nn < a.Nout;
  const int HWo = a.Ho * a.Wo, Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  const bf16* dy = reinterpret_cast<const bf16*>(a.dY);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool do_bias = a.dB && tk == 0 && nvalid;

  Grp<bf16> gx[GX], gd[GD];
  auto load_stage = [&](int mb) {
#pragma unroll
    for (int i = 0; i < GX; ++i) {
      grp_zero(gx[i]);
      const int m = mb + rowx + RX * i;
      if (m < mend && kvalid) {
        int nimg = m / HWo, rem = m - nimg * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
        int yi = yo * a.stride + ty * a.dil - a.pad, xi = xo * a.stride + tx * a.dil - a.pad;
        if (yi >= 0 && xi >= 0 && yi < Hv && xi < Wv) {
          if (a.up == 2) { yi >>= 1; xi >>= 1; }
          grp_load(gx[i], src + (((size_t)nimg * a.Hs + yi) * a.Ws + xi) * cs + cl);
          if (sc) {
            float f[8];
            grp_to_f(gx[i], f);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[cl + j], sh[cl + j]), 0.f);
            grp_from_f(gx[i], f);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GD; ++i) {
      grp_zero(gd[i]);
      const int m = mb + rowd + RD * i;
      if (m < mend && nvalid) {
        if (a.dy_mode == 0) {
          grp_load(gd[i], dy + (size_t)m * a.dy_stride + nn);
        } else {
          int nimg = m / HWo, rem = m - nimg * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
          int sub = nn / a.Cps, c = nn - sub * a.Cps;
          size_t pix = ((size_t)nimg * (2 * a.Ho) + 2 * yo + (sub >> 1)) * (2 * a.Wo) + 2 * xo + (sub & 1);
          grp_load(gd[i], dy + pix * a.dy_stride + c);
        }
        if (do_bias) {
          float f[8];
          grp_to_f(gd[i], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) bacc[j] += f[j];
        }
      }
    }
  };
  auto store_stage = [&](int buf) {
    bf16* Xs = smem + buf * MS * (LX + LD);
    bf16* Ds = Xs + MS * LX;
#pragma unroll
    for (int i = 0; i < GX; ++i) grp_store(gx[i], Xs + (rowx + RX * i) * LX + kgx * 8);
#pragma unroll
    for (int i = 0; i < GD; ++i) grp_store(gd[i], Ds + (rowd + RD * i) * LD + cgd * 8);
  };

  load_stage(mbeg);
  store_stage(0);
  __syncthreads();
  int buf = 0;
  for (int mb = mbeg; mb < mend; mb += MS) {
    const bool more = mb + MS < mend;
    if (more) load_stage(mb + MS);
    const bf16* Xs = smem + buf * MS * (LX + LD);
    const bf16* Ds = Xs + MS * LX;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bx[4];
#pragma unroll
      for (int ki = 0; ki < 4; ++ki) bx[ki] = tr_frag(Xs, 32 * s, LX, wk * 64 + ki * 16, lane);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        bf16x8 ad = tr_frag(Ds, 32 * s, LD, wn * 64 + ni * 16, lane);
#pragma unroll
        for (int ki = 0; ki < 4; ++ki)
          acc[ni][ki] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad, bx[ki], acc[ni][ki], 0, 0, 0);
      }
    }
    if (more) store_stage(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  const int col = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int ki = 0; ki < 4; ++ki)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 64 + ni * 16 + rq + r;
        const int kk = k0 + wk * 64 + ki * 16 + col;
        if (n < a.Nout && kk < a.K) atomicAdd(a.dW + (size_t)n * a.Kpad + kk, acc[ni][ki][r]);
      }
  if (a.dB && tk == 0) {
    // reduce the per-thread 8-channel partial sums of threads sharing a channel group
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bacc[j];
    __syncthreads();
    if (tid < TN) {
      const int g = tid >> 3, j = tid & 7;
      float s = 0.f;
      for (int t = g; t < NT; t += GDR) s += red[t * 8 + j];
      const int n = n0 + tid;
      if (n < a.Nout) atomicAdd(a.dB + (a.dy_mode == 1 ? n % a.Cps : n), s);
    }
  }
}

// ---------------------------------------------------------- bf16 wgrad kernel, LDS-DMA staged
// Operands X[pixel][k] and dY[pixel][n] are moved by global_load_lds into linear rows of RB bytes
// (RB = 2*TK or 2*TN); 16-B chunk c of row r sits at chunk position c ^ g(r), g(r) = 2*(r & 7) for
// RB >= 256 and 2*((r >> 1) & 3) for RB = 128, which spreads the 8 rows read by one 32-lane half of a
// ds_read_b64_tr_b16 over 8 distinct 32-B bank slots. Pixel order inside a 32-pixel substep is the
// rho permutation of igemm_wgrad_bf16_kernel. The bias gradient is a separate channel-sum launch.
template <int TN, int TK>
__global__ __launch_bounds__(NT, 2) void igemm_wgrad_glds_kernel(WgradArgs a) {
  constexpr int MS = 64;
  constexpr int RX = 2 * TK, RD = 2 * TN;              // row bytes
  constexpr int SX = MS * RX, SD = MS * RD, STAGE = SX + SD;
  constexpr int XI = SX / 1024 / 4, DI = SD / 1024 / 4; // glds per wave per stage
  constexpr int XRPI = 1024 / RX, DRPI = 1024 / RD;     // rows per instruction
  constexpr int WK = TK / 64;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WK, wk = wave % WK;
  const int tk = blockIdx.x % a.ntile_k, tn = blockIdx.x / a.ntile_k;
  const int k0 = tk * TK, n0 = tn * TN;
  const int mbeg = blockIdx.y * a.mchunk;
  const int mend = min(a.M, mbeg + a.mchunk);
  if (mbeg >= mend) return;
  const int HWo = a.Ho * a.Wo, Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  const int Cin_s = a.CAs + a.CBs;

  // X slots: instruction i of this wave covers rows wave*(MS/4) + XRPI*i + lane / (RX/16)
  int xr[XI], xdy[XI], xdx[XI], xcl[XI];
  const bf16* xsrc[XI];
  int xcs[XI];
  bool xk[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int r = wave * (MS / 4) + XRPI * i + lane / (RX / 16);
    const int pos = lane % (RX / 16);
    const int c = pos ^ gsw<RX>(r);
    const int k = k0 + 8 * c;
    xr[i] = r;
    xk[i] = k < a.K;
    const int tap = xk[i] ? k / Cin_s : 0;
    const int ci = k - tap * Cin_s;
    const int ty = tap / a.kw, tx = tap - ty * a.kw;
    xdy[i] = ty * a.dil - a.pad;
    xdx[i] = tx * a.dil - a.pad;
    const bool useB = ci >= a.CAs;
    xcl[i] = useB ? ci - a.CAs : ci;
    xsrc[i] = reinterpret_cast<const bf16*>(useB ? a.srcB : a.srcA);
    xcs[i] = useB ? a.CBs : a.CAs;
  }
  int dr[DI], dn[DI];
#pragma unroll
  for (int i = 0; i < DI; ++i) {
    const int r = wave * (MS / 4) + DRPI * i + lane / (RD / 16);
    const int pos = lane % (RD / 16);
    dr[i] = r;
    dn[i] = n0 + 8 * (pos ^ gsw<RD>(r));
  }
  const bf16* dy = reinterpret_cast<const bf16*>(a.dY);

  auto issue = [&](int mb, int buf) {
    unsigned char* sb = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const void* p = adp_zero_page;
      const int m = mb + xr[i];
      if (m < mend && xk[i]) {
        const int nimg = m / HWo, rem = m - nimg * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
        int yi = yo * a.stride + xdy[i], xi = xo * a.stride + xdx[i];
        if (yi >= 0 && xi >= 0 && yi < Hv && xi < Wv) {
          if (a.up == 2) { yi >>= 1; xi >>= 1; }
          p = xsrc[i] + (((size_t)nimg * a.Hs + yi) * a.Ws + xi) * xcs[i] + xcl[i];
        }
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(sb + (wave * (MS / 4) + XRPI * i) * RX), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const void* p = adp_zero_page;
      const int m = mb + dr[i];
      if (m < mend && dn[i] < a.Nout) {
        if (a.dy_mode == 0) {
          p = dy + (size_t)m * a.dy_stride + dn[i];
        } else {
          const int nimg = m / HWo, rem = m - nimg * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
          const int sub = dn[i] / a.Cps, c = dn[i] - sub * a.Cps;
          const size_t pix = ((size_t)nimg * (2 * a.Ho) + 2 * yo + (sub >> 1)) * (2 * a.Wo) + 2 * xo + (sub & 1);
          p = dy + pix * a.dy_stride + c;
        }
      }
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(sb + SX + (wave * (MS / 4) + DRPI * i) * RD), 16, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(mbeg, 0);
  int buf = 0;
  for (int mb = mbeg; mb < mend; mb += MS) {
    if (mb + MS < mend) {
      issue(mb + MS, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(XI + DI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const unsigned char* Xs = smem + buf * STAGE;
    const unsigned char* Ds = Xs + SX;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 bx[4];
#pragma unroll
      for (int ki = 0; ki < 4; ++ki) bx[ki] = tr_frag_sw<RX>(Xs, 32 * s, wk * 64 + ki * 16, lane);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const bf16x8 ad = tr_frag_sw<RD>(Ds, 32 * s, wn * 64 + ni * 16, lane);
#pragma unroll
        for (int ki = 0; ki < 4; ++ki)
          acc[ni][ki] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad, bx[ki], acc[ni][ki], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    buf ^= 1;
  }

  const int col = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int ki = 0; ki < 4; ++ki)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 64 + ni * 16 + rq + r;
        const int kk = k0 + wk * 64 + ki * 16 + col;
        if (n < a.Nout && kk < a.K) atomicAdd(a.dW + (size_t)n * a.Kpad + kk, acc[ni][ki][r]);
      }
}

// per-channel sum over pixels (bias gradient); plain [M][C] or pixel-shuffled ConvT gradient
// (channel n of the GEMM = sub*Cps + c -> bias c)
// part != 0: out is this launch's slab [gridDim.x][C] and block b stores its sums in row b (plain stores, summed in a
// fixed order by adp::slab_reduce: deterministic), else f32 atomics into out
template <typename T>
__global__ void channel_sum_kernel(size_t M, int C, int stride, const T* x, float* out, int fold, int part = 0) {
  const int G = C >> 3;
  const int lanes = NT / G;
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (pl < lanes) {
    for (size_t m = (size_t)blockIdx.x * lanes + pl; m < M; m += (size_t)gridDim.x * lanes) {
      Grp<T> gr;
      float f[8];
      grp_load(gr, x + m * stride + g * 8);
      grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
  __shared__ float red[NT * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = s[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    float t = 0.f;
    for (int l = 0; l < lanes; ++l) t += red[(l * G + (c >> 3)) * 8 + (c & 7)];
    if (part) out[(size_t)blockIdx.x * C + c] = t;
    else atomicAdd(out + (fold ? c % fold : c), t);
  }
}

// bias gradient of a weight-gradient launch: per-channel sums of dY (ConvT: of its 2x-resolution pixel-shuffled
// gradient); option wgrad_det (default on): per-block rows + the fixed-order slab reduce instead of f32 atomics
template <typename T>
void launch_bias_grad(const WgradArgs& a, hipStream_t s) {
  const size_t Mp = a.dy_mode == 0 ? (size_t)a.M : (size_t)a.M * 4;
  const int C = a.dy_mode == 0 ? a.Nout : a.Cps;
  const int G = C / 8, lanes = NT / G;
  const int blocks = (int)std::min<size_t>((Mp + lanes - 1) / lanes, 1024);
  float* part = adp::option("wgrad_det", 1) && C % 4 == 0 ? adp::reduce_part(3, (size_t)blocks * C * sizeof(float), s)
                                                           : nullptr;
  hipLaunchKernelGGL(channel_sum_kernel<T>, dim3(blocks), dim3(NT), 0, s, Mp, C, a.dy_stride,
                     reinterpret_cast<const T*>(a.dY), part ? part : a.dB, 0, part ? 1 : 0);
  if (part) adp::slab_reduce(blocks, (size_t)C / 4, part, a.dB, s);
}

}  // namespace

// ============================================================================ C ABI
#include "../../include/adipose_hip.h"

namespace {
template <typename T>
int launch_fwd_plain(FwdArgs& a, hipStream_t s, int fast);

void fill_fwd_args(const adp_conv_desc* d, const adp_conv_io* io, FwdArgs& a) {
  a = FwdArgs{};
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
  a.defer_fold = d->bn_defer_fold && io->bn_sum && !io->bnr_z;
  a.bnr_z = io->bnr_z; a.bnr_zs = d->bnr_stride;
  a.bnr_sc = io->bnr_scale; a.bnr_sh = io->bnr_shift; a.bnr_mean = io->bnr_mean; a.bnr_invstd = io->bnr_invstd;
  a.bnr_dgamma = io->bnr_dgamma; a.bnr_dbeta = io->bnr_dbeta;
  a.M = d->N * d->Ho * d->Wo;
  a.debug_flags = adp::option("fwd_debug", 0);
  a.f32 = 0;
  a.stat = (a.bn_sum || a.bnr_z) ? adp::stat_scratch() : nullptr;
  a.act_out = io->act_outA;
  // zero tails of the weights (the caller's real channel counts, adp_conv_desc v19): products with zero weight
  // columns / rows that a kernel may skip exactly
  a.ca_real = d->CA_real;
  auto tail48 = [](int stride, int real) { return stride == 64 && real > 0 && real <= 48; };
  a.ztail = (tail48(d->CA_stride, d->CA_real) && (d->CB_stride == 0 || tail48(d->CB_stride, d->CB_real)) ? 1 : 0) |
            (tail48(d->Nout, d->Nout_real) && d->out_mode == 0 ? 2 : 0);
}

// after a launch whose epilogue added BatchNorm sums into the replicas: fold them into the caller's
// accumulators (statistics: bn_sum / bn_sq; BN-backward reduction: bnr_dbeta / bnr_dgamma)
int fold_stats(const FwdArgs& a, hipStream_t s) {
  if (!a.stat) return 0;
  if (a.defer_fold)   // (deferred: adp_bn_finalize_fold folds them)
    return adp::defer_fold_begin(a.out_mode == 1 ? a.Cps : a.Nout, a.bn_sum, s);
  const int C = a.out_mode == 1 ? a.Cps : a.Nout;
  if (a.bnr_z) return adp::stat_fold(C, a.bnr_dbeta, a.bnr_dgamma, s);
  return adp::stat_fold(C, a.bn_sum, a.bn_sq, s);
}

// fp8 e4m3 forward launch (BASELINE configs[4]): tap64 kernel only, no fallback
int launch_fwd_f8(const adp_conv_desc* d, const adp_conv_io* io, hipStream_t s) {
  FwdArgs a;
  fill_fwd_args(d, io, a);
  a.f8 = 1;
  a.wscale = io->w_scale;
  a.out_f8 = d->out_fp8;
  ADP_REQUIRE(a.wscale && a.M > 0 && a.Nout > 0 && a.Nout % 8 == 0, "adp_conv_fwd(fp8): needs w_scale and Nout % 8 == 0");
  ADP_REQUIRE(!a.scA && !a.scB && !a.addend && !a.mask && !a.accum && !a.bn_sum && !a.bnr_z && a.drop_rate == 0.f &&
                  (d->out_mode == 0 || d->out_mode == 1) && a.out,
              "adp_conv_fwd(fp8): plain or pixel-shuffle store only (no BN / addend / mask / accum / dropout)");
  ADP_REQUIRE(d->out_mode != 1 || (d->shuffle_c > 0 && d->Nout % d->shuffle_c == 0), "adp_conv_fwd: bad shuffle_c");
  // 64-channel sources (unet_bn level 0): the fp8 halo kernel (tap pairs / two concatenated sources per K step)
  if (a.CAs == 64 && a.CBs % 64 == 0 && adp::launch_fwd_halop_f8(a, s)) {
    adp::kernel_end();
    return adp::check_launch("adp_conv_fwd");
  }
  ADP_REQUIRE(a.CAs % 128 == 0 && a.CBs % 128 == 0,
              "adp_conv_fwd(fp8): source channel strides must be multiples of 128 (one 128-channel K step per tap)");
  if (!adp::launch_fwd_tap64(a, s)) {
    adp::set_error("adp_conv_fwd(fp8): no fp8 kernel for this geometry (needs K == taps * Cin_s, K % 128 == 0)");
    return -1;
  }
  adp::kernel_end();
  return adp::check_launch("adp_conv_fwd");
}

template <typename T>
int launch_fwd(const adp_conv_desc* d, const adp_conv_io* io, hipStream_t s) {
  FwdArgs a;
  fill_fwd_args(d, io, a);
  ADP_REQUIRE(a.CAs % 8 == 0 && a.CBs % 8 == 0, "adp_conv_fwd: channel strides must be multiples of 8");
  if (d->out_fp8) {   // a bf16 launch storing fp8: the input layer of the fp8 forward (UNetBN.forward_fp8) only
    ADP_REQUIRE((std::is_same<T, bf16>::value), "adp_conv_fwd: out_fp8 needs a bf16 or fp8 launch");
    a.out_f8 = 1;
    if (!adp::launch_fwd_cin8(a, s)) {
      adp::set_error("adp_conv_fwd: out_fp8 on a bf16 launch: input layers only (one 8-channel source, Nout == 64, "
                     "no statistics)");
      return -1;
    }
    adp::kernel_end();
    return adp::check_launch("adp_conv_fwd");
  }
  ADP_REQUIRE(a.M > 0 && a.Nout > 0, "adp_conv_fwd: empty problem");
  ADP_REQUIRE(d->out_mode != 1 || (d->shuffle_c > 0 && d->Nout % d->shuffle_c == 0), "adp_conv_fwd: bad shuffle_c");
  ADP_REQUIRE(d->out_mode != 2 || (io->out2 && d->split_c > 0), "adp_conv_fwd: split store needs out2/split_c");
  ADP_REQUIRE(!a.bnr_z || (d->out_mode == 0 && !a.bn_sum && a.bnr_sc && a.bnr_sh && a.bnr_mean && a.bnr_invstd &&
                           a.bnr_dgamma && a.bnr_dbeta && a.bnr_zs == a.out_stride && a.bnr_zs % 8 == 0 &&
                           a.Nout % 8 == 0),
              "adp_conv_fwd: fused BN-backward reduction needs out_mode 0, all bnr_* pointers, z stride == out stride");
  ADP_REQUIRE(!(a.bn_sum || a.bnr_z) || a.stat,
              std::string("adp_conv_fwd: BatchNorm accumulator replicas unavailable: ") + adp_last_error());
  ADP_REQUIRE(!a.stat || (d->out_mode == 1 ? d->shuffle_c : d->Nout) <= adp::STAT_CMAX,
              "adp_conv_fwd: BatchNorm sums need <= 2048 channels");
  const int fast = adp::option("conv_fast", 2);
  if (a.act_out) {
    // BN-on-load with the applied source stored too: one launch of the persistent halo forward where it takes the
    // shape, else adp_bn_apply into act_outA and the launch on it (the same bits either way)
    ADP_REQUIRE(a.scA && a.shA && !a.scB && a.CBs == 0 && io->srcA != io->act_outA,
                "adp_conv_fwd: act_outA needs bn_scaleA / bn_shiftA, one source and its own buffer");
    if (std::is_same<T, bf16>::value && fast == 2 && adp::launch_fwd_halo(a, s)) {
      adp::kernel_end();
      if (adp::check_launch("adp_conv_fwd")) return -2;
      return fold_stats(a, s);
    }
    const int rc = adp_bn_apply(std::is_same<T, bf16>::value ? ADP_BF16 : ADP_F32, (size_t)a.Nimg * a.Hs * a.Ws, a.CAs,
                                a.srcA, a.scA, a.shA, a.act_out, (adp_stream_t)s);
    if (rc) return rc;
    a.srcA = a.act_out;
    a.scA = a.shA = nullptr;
    a.act_out = nullptr;
  }
  if (std::is_same<T, bf16>::value && fast == 2 && !a.scA && !a.scB &&
      (adp::launch_fwd_cin8(a, s) || adp::launch_fwd_halo(a, s) || adp::launch_fwd_tap64(a, s))) {
    adp::kernel_end();
    if (adp::check_launch("adp_conv_fwd")) return -2;
    return fold_stats(a, s);
  }
  // f32: the LDS-DMA tap kernel with 32-channel K steps where every K step lies in one tap and one source
  if (std::is_same<T, float>::value && fast == 2 && !a.scA && !a.scB) {
    a.f32 = 1;
    if (adp::launch_fwd_cin8_f32(a, s) || adp::launch_fwd_tap64(a, s)) {
      adp::kernel_end();
      if (adp::check_launch("adp_conv_fwd")) return -2;
      return fold_stats(a, s);
    }
    a.f32 = 0;
  }
  // every other kernel: plain launch, then the standalone BN-backward reduction on the stored output
  const FwdArgs bnr = a;
  a.bnr_z = nullptr;
  if (!a.bn_sum) a.stat = nullptr;
  const int rc = launch_fwd_plain<T>(a, s, fast);
  if (rc != 0) return rc;
  // every kernel added its statistics into the f64 replicas (since round 4 the register-staged generic kernels
  // too: their f32 atomics into bn_sum made the f32 input layer's statistics run-dependent)
  if (a.stat && fold_stats(a, s) != 0) return -2;
  if (!bnr.bnr_z) return 0;
  return adp_bn_bwd_reduce(std::is_same<T, bf16>::value ? ADP_BF16 : ADP_F32, (size_t)bnr.M, bnr.out_stride, bnr.out,
                           bnr.bnr_z, bnr.bnr_sc, bnr.bnr_sh, bnr.bnr_mean, bnr.bnr_invstd, bnr.bnr_dgamma,
                           bnr.bnr_dbeta, (adp_stream_t)s);
}

template <typename T>
int launch_fwd_plain(FwdArgs& a, hipStream_t s, int fast) {
  if (std::is_same<T, bf16>::value && fast == 2 && !a.scA && !a.scB) {
    const int w64 = (a.Nout + 63) / 64 * 64 - a.Nout, w128 = (a.Nout + 127) / 128 * 128 - a.Nout;
    if (a.Nout > 64 && w128 <= w64) {
      a.ntile_n = (a.Nout + 127) / 128;
      a.nblocks = ((a.M + 127) / 128) * a.ntile_n;
      adp::set_kernel("igemm_fwd_glds_kernel<128, 128>");
      hipLaunchKernelGGL((igemm_fwd_glds_kernel<128, 128>), dim3(a.nblocks), dim3(NT), 0, s, a);
    } else {
      a.ntile_n = (a.Nout + 63) / 64;
      a.nblocks = ((a.M + 255) / 256) * a.ntile_n;
      adp::set_kernel("igemm_fwd_glds_kernel<256, 64>");
      hipLaunchKernelGGL((igemm_fwd_glds_kernel<256, 64>), dim3(a.nblocks), dim3(NT), 0, s, a);
    }
    adp::kernel_end();
    return adp::check_launch("adp_conv_fwd");
  }
  if (std::is_same<T, bf16>::value && fast >= 1) {
    // tile choice: least padded-N waste, ties -> 128x128 (more A reuse per block)
    const int w64 = (a.Nout + 63) / 64 * 64 - a.Nout, w128 = (a.Nout + 127) / 128 * 128 - a.Nout;
    if (a.Nout > 64 && w128 <= w64) {
      a.ntile_n = (a.Nout + 127) / 128;
      a.nblocks = ((a.M + 127) / 128) * a.ntile_n;
      adp::set_kernel("igemm_fwd_bf16_kernel<128, 128>");
      hipLaunchKernelGGL((igemm_fwd_bf16_kernel<128, 128>), dim3(a.nblocks), dim3(NT), 0, s, a);
    } else {
      a.ntile_n = (a.Nout + 63) / 64;
      a.nblocks = ((a.M + 255) / 256) * a.ntile_n;
      adp::set_kernel("igemm_fwd_bf16_kernel<256, 64>");
      hipLaunchKernelGGL((igemm_fwd_bf16_kernel<256, 64>), dim3(a.nblocks), dim3(NT), 0, s, a);
    }
    adp::kernel_end();
    return adp::check_launch("adp_conv_fwd");
  }
  a.ntile_n = (a.Nout + BN - 1) / BN;
  const int ntm = (a.M + BM - 1) / BM;
  a.nblocks = ntm * a.ntile_n;
  adp::set_kernel(std::is_same<T, bf16>::value ? "igemm_fwd_kernel<bf16>" : "igemm_fwd_kernel<float>");
  hipLaunchKernelGGL(igemm_fwd_kernel<T>, dim3(a.nblocks), dim3(NT), 0, s, a);
  adp::kernel_end();
  return adp::check_launch("adp_conv_fwd");
}

template <typename T>
int launch_wgrad(const adp_conv_desc* d, const adp_conv_io* io, const void* dY, int dy_stride,
                 float* dW, float* dB, hipStream_t s, const adp_bn_bwd_args* bn = nullptr) {
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
  a.ca_real = d->CA_real; a.cb_real = d->CB_real; a.nout_real = d->Nout_real;
  ADP_REQUIRE(a.CAs % 8 == 0 && a.CBs % 8 == 0 && a.Nout % 8 == 0,
              "adp_conv_wgrad: channel strides and Nout must be multiples of 8");
  ADP_REQUIRE(d->out_mode != 2, "adp_conv_wgrad: split-store descriptors are dgrad-only");
  if (bn) {   // adp_conv_wgrad_bn: fused into the halo kernel, else the apply launch first
    a.bna_dA = bn->dA; a.bna_z = bn->z;
    a.bna_sc = bn->scale; a.bna_sh = bn->shift; a.bna_mean = bn->mean; a.bna_invstd = bn->invstd;
    a.bna_gamma = bn->gamma; a.bna_dgamma = bn->dgamma; a.bna_dbeta = bn->dbeta;
    a.bna_inv_count = 1.f / bn->count;
    if (!(std::is_same<T, bf16>::value && adp::option("conv_fast", 2) == 2 && adp::wgrad_bna_fusable(a))) {
      a.bna_dA = nullptr;
      if (!dY) {   // dz not wanted by the caller: the two-launch form computes it in library scratch
        dY = adp::scratch(1, (size_t)a.M * dy_stride * (std::is_same<T, bf16>::value ? 2 : 4));
        if (!dY) return -2;
        a.dY = dY;
      }
      if (adp_bn_bwd_apply(std::is_same<T, bf16>::value ? ADP_BF16 : ADP_F32, (size_t)a.M, dy_stride, bn->dA, bn->z,
                           bn->scale, bn->shift, bn->mean, bn->invstd, bn->gamma, bn->dgamma, bn->dbeta, bn->count,
                           const_cast<void*>(dY), s))
        return -2;
    }
  }
  if (std::is_same<T, bf16>::value && adp::option("conv_fast", 2) == 2 && !a.scA && !a.scB) {
    if (!adp::launch_wgrad_tap64(a, s)) {
      if (a.bna_dA) {   // no kernel took the fused form: dY = bn_bwd_apply(dA, z) first, then the fallback
        a.bna_dA = nullptr;
        if (!dY) {
          dY = adp::scratch(1, (size_t)a.M * dy_stride * 2);
          if (!dY) return -2;
          a.dY = dY;
        }
        if (adp_bn_bwd_apply(ADP_BF16, (size_t)a.M, dy_stride, bn->dA, bn->z, bn->scale, bn->shift, bn->mean,
                             bn->invstd, bn->gamma, bn->dgamma, bn->dbeta, bn->count, const_cast<void*>(dY), s))
          return -2;
      }
      const int TN = (a.Nout <= 64 && adp::option("wgrad_glds_tn64", 1)) ? 64 : 128, TK = TN == 64 ? 256 : 128;
      a.ntile_k = (a.K + TK - 1) / TK;
      a.ntile_n = (a.Nout + TN - 1) / TN;
      const int tiles = a.ntile_k * a.ntile_n;
      int splits = (2048 + tiles - 1) / tiles;
      const int maxsplit = (a.M + 511) / 512;
      splits = std::max(1, std::min(splits, maxsplit));
      a.mchunk = ((a.M + splits - 1) / splits + 63) / 64 * 64;
      splits = (a.M + a.mchunk - 1) / a.mchunk;
      if (TN == 64)
        { adp::set_kernel("igemm_wgrad_glds_kernel<64, 256>");
          hipLaunchKernelGGL((igemm_wgrad_glds_kernel<64, 256>), dim3(tiles, splits), dim3(NT), 0, s, a); }
      else
        { adp::set_kernel("igemm_wgrad_glds_kernel<128, 128>");
          hipLaunchKernelGGL((igemm_wgrad_glds_kernel<128, 128>), dim3(tiles, splits), dim3(NT), 0, s, a); }
    }
    adp::kernel_end();   // (no-op when launch_wgrad_tap64 marked it before its split reduce)
    if (a.dB) launch_bias_grad<bf16>(a, s);
    return adp::check_launch("adp_conv_wgrad");
  }
  if (std::is_same<T, bf16>::value && adp::option("conv_fast", 2) >= 1) {
    // 64x256 only when explicitly asked ("wgrad_tn64"): measured slower than 128x128 at N=64
    const int TN = (a.Nout <= 64 && adp::option("wgrad_tn64", 0)) ? 64 : 128, TK = TN == 64 ? 256 : 128;
    a.ntile_k = (a.K + TK - 1) / TK;
    a.ntile_n = (a.Nout + TN - 1) / TN;
    const int tiles = a.ntile_k * a.ntile_n;
    int splits = (1536 + tiles - 1) / tiles;
    const int maxsplit = (a.M + 511) / 512;
    splits = std::max(1, std::min(splits, maxsplit));
    a.mchunk = ((a.M + splits - 1) / splits + 63) / 64 * 64;
    splits = (a.M + a.mchunk - 1) / a.mchunk;
    if (TN == 64)
      { adp::set_kernel("igemm_wgrad_bf16_kernel<64, 256>");
        hipLaunchKernelGGL((igemm_wgrad_bf16_kernel<64, 256>), dim3(tiles, splits), dim3(NT), 0, s, a); }
    else
      { adp::set_kernel("igemm_wgrad_bf16_kernel<128, 128>");
        hipLaunchKernelGGL((igemm_wgrad_bf16_kernel<128, 128>), dim3(tiles, splits), dim3(NT), 0, s, a); }
    adp::kernel_end();
    return adp::check_launch("adp_conv_wgrad");
  }
  // f32: the LDS-DMA weight-gradient kernel (conv_wgrad_f32.hip), bias gradient as a channel-sum launch
  if (std::is_same<T, float>::value && adp::launch_wgrad_f32(a, s)) {
    if (a.dB) launch_bias_grad<float>(a, s);
    return adp::check_launch("adp_conv_wgrad");
  }
  a.ntile_k = (a.K + 63) / 64;
  a.ntile_n = (a.Nout + 63) / 64;
  const int tiles = a.ntile_k * a.ntile_n;
  int splits = (2048 + tiles - 1) / tiles;
  int maxsplit = (a.M + 255) / 256;
  if (splits > maxsplit) splits = maxsplit;
  if (splits < 1) splits = 1;
  a.mchunk = ((a.M + splits - 1) / splits + 31) / 32 * 32;
  splits = (a.M + a.mchunk - 1) / a.mchunk;
  adp::set_kernel(std::is_same<T, bf16>::value ? "igemm_wgrad_kernel<bf16>" : "igemm_wgrad_kernel<float>");
  hipLaunchKernelGGL(igemm_wgrad_kernel<T>, dim3(tiles, splits), dim3(NT), 0, s, a);
  adp::kernel_end();
  return adp::check_launch("adp_conv_wgrad");
}
}  // namespace

extern "C" int adp_conv_fwd(int dtype, const adp_conv_desc* d, const adp_conv_io* io, adp_stream_t st) {
  hipStream_t s = (hipStream_t)st;
  ADP_REQUIRE(d && io, "adp_conv_fwd: null descriptor");
  adp::set_launch_stream(s);
  if (dtype == ADP_F32) return launch_fwd<float>(d, io, s);
  if (dtype == ADP_BF16) return launch_fwd<bf16>(d, io, s);
  if (dtype == ADP_FP8) return launch_fwd_f8(d, io, s);
  adp::set_error("adp_conv_fwd: unknown dtype");
  return -1;
}

extern "C" int adp_conv_wgrad_bn(int dtype, const adp_conv_desc* d, const adp_conv_io* io, const adp_bn_bwd_args* bn,
                                 void* dY, int dy_stride, float* dW, float* dB, adp_stream_t st) {
  hipStream_t s = (hipStream_t)st;
  ADP_REQUIRE(d && io && bn && bn->dA && bn->z && dW, "adp_conv_wgrad_bn: null argument");
  ADP_REQUIRE(dY || !dB, "adp_conv_wgrad_bn: dY may be NULL only without dB (nothing then reads dz)");
  adp::set_launch_stream(s);
  ADP_REQUIRE(bn->scale && bn->shift && bn->mean && bn->invstd && bn->gamma && bn->dgamma && bn->dbeta && bn->count > 0,
              "adp_conv_wgrad_bn: BatchNorm vectors and count");
  ADP_REQUIRE(d->out_mode == 0 && dy_stride == d->Nout && dy_stride % 8 == 0,
              "adp_conv_wgrad_bn: plain [M][Nout] gradient (dA, z, dY share the channel stride)");
  if (dtype == ADP_F32) return launch_wgrad<float>(d, io, dY, dy_stride, dW, dB, s, bn);
  if (dtype == ADP_BF16) return launch_wgrad<bf16>(d, io, dY, dy_stride, dW, dB, s, bn);
  adp::set_error("adp_conv_wgrad_bn: unknown dtype");
  return -1;
}

extern "C" int adp_conv_wgrad(int dtype, const adp_conv_desc* d, const adp_conv_io* io, const void* dY,
                              int dy_stride, float* dW, float* dB, adp_stream_t st) {
  hipStream_t s = (hipStream_t)st;
  ADP_REQUIRE(d && io && dY && dW, "adp_conv_wgrad: null argument");
  adp::set_launch_stream(s);
  if (dtype == ADP_F32) return launch_wgrad<float>(d, io, dY, dy_stride, dW, dB, s);
  if (dtype == ADP_BF16) return launch_wgrad<bf16>(d, io, dY, dy_stride, dW, dB, s);
  adp::set_error("adp_conv_wgrad: unknown dtype");
  return -1;
}
