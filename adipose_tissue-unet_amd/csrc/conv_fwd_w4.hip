// Four-wave persistent halo forward for the wide 3x3 layers (unet_bn levels 1-4, >= 256 output channels):
// one 256-thread block per CU, ONE wave per SIMD, each wave owning a 128-pixel x 128-channel quarter of the
// block's 256 x 256 output tile (8 x 32 patch x 256 channels) in 256 accumulator registers.
//
// Against the 8-wave LDS-DMA kernel (conv_fwd_tap64p.hip, two waves per SIMD, 128 x 64 per wave):
//   * the weights (B operand) never touch the LDS: each lane loads its MFMA fragments straight from global
//     memory (16-B buffer loads, L2-resident: a layer's weights are <= 18 MiB and every CU of an XCD walks
//     the same K rows) one K step ahead into a second register set. That removes the weight LDS-DMA, whose
//     issue cost (60-185 cycles per 1-KiB wave piece) was what the K loop waited on, and a third of the LDS
//     reads;
//   * the wave tile doubles (128 x 128): LDS reads per MAC halve again (16 KiB of activation fragments per
//     wave per 64-deep K step for 2M MACs);
//   * the only LDS data is the 10 x 34 input halo of the patch per 64-channel chunk (read by all 9 taps), so
//     the block synchronises once per chunk (every 9 K steps) instead of once per K step. The next chunk's
//     halo goes through registers (2 x 16-B loads per thread at taps 0-5, written to the free slot one step
//     later) -- plain vector memory ops, no LDS-DMA issue stalls on the one wave of the SIMD.
// K stream of a tile: chunk-major, taps 0..8 inside a chunk (weight row kt = tap * nch + chunk). The tiles of
// a block form one stream: the next tile's first weights and halo are in flight during the epilogue.
// Epilogue: from registers (a lane holds 4 consecutive channels of one pixel per 16 x 16 block), bias,
// ReLU, bf16 8-B stores, BatchNorm statistics of the stored values into the block's LDS sums -> one
// replica of the accumulators per block (folded by the launcher, as for every bn_sum launch).
#include "conv_common.h"

namespace {

constexpr unsigned W4_OOB = 0x80000000u;
constexpr int W4_RSRC3 = 0x00020000;
constexpr int W4_HROWS = 340, W4_HBUF = W4_HROWS * 128;   // halo pixels of an 8 x 32 patch, bytes per slot
constexpr int W4_GH = (W4_HROWS * 8 + 255) / 256;          // 16-B halo groups per thread per chunk (11)
typedef unsigned int v2u32_4 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32_4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4u32_4 w4_ld16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

// DBG (timing-only ablations, option fwd_w4_dbg; results invalid): bit 0 no weight reloads in the K loop,
// bit 1 no halo refills, bit 2 no epilogue stores
// LB: the weight tile of a K step goes global -> registers (8 x 16 B per thread, whole 128-B rows) -> LDS
// (two-stage ring, written once per step, one barrier per step), and every wave reads its fragments from
// there: half the L2 / TA traffic of the direct form (the two waves of a channel half no longer fetch the
// same fragments) at 32 KiB of LDS writes and 64 KiB of reads per step.
template <bool STATS, int DBG = 0, bool LB = false>
__global__ __launch_bounds__(256, 1) void igemm_fwd_w4_kernel(FwdArgs a) {
  constexpr int NTH = 256, ROWB = 128;
  constexpr int OBS = 2 * W4_HBUF, BSTAGE = 256 * ROWB;            // weight stages (LB)
  constexpr int OCST = OBS + (LB ? 2 * BSTAGE : 0);
  constexpr int ODUM = OCST + 256 * 4 + 2 * 256 * 8;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[ODUM + 256 * 16];
  float* cst = reinterpret_cast<float*>(smem + OCST);   // bias [256]
  // block's BN sums [2][256] in f64: the waves' f32 row partials added in any order give the same f64 sum up to
  // ~1e-16 relative (deterministic after the fold's single rounding to f32, as the other producers' sums)
  double* sacc = reinterpret_cast<double*>(cst + 256);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;   // pixel half (patch rows 4 wr .. 4 wr + 3), channel half
  const int r16 = lane & 15, h4 = lane >> 4;
  const int G = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, G);
  const int ntiles = a.nblocks;
  const int mine = lin < ntiles ? (ntiles - lin + G - 1) / G : 0;
  if (mine == 0) return;
  const int n0 = (lin % a.ntile_n) * 256;
  const int Cin_s = a.CAs + a.CBs, nch = Cin_s / 64;
  const int us = a.up >> 1;
  const int ptx = a.Wo / 32, pty = a.Ho / 8;

  if (tid < 256) {
    const int n = n0 + tid;
    cst[tid] = (a.bias && n < a.Nout) ? a.bias[n] : 0.f;
    sacc[tid] = 0.0;
    sacc[256 + tid] = 0.0;
  }

  const int npix = a.Nimg * a.Hs * a.Ws;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.srcA, 0, npix * a.CAs * 2, W4_RSRC3);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.CBs ? a.srcB : a.srcA), 0, npix * (a.CBs ? a.CBs : a.CAs) * 2, W4_RSRC3);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, a.Nout * a.Kpad * 2, W4_RSRC3);
  const int out_bytes = a.M * a.out_stride * 2;
  const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, out_bytes, W4_RSRC3);

  // weight fragment offsets: row n0 + wc*128 + ni*16 + r16, bytes 16*h4 (+64 for the second 32-deep half)
  unsigned bo[8];
#pragma unroll
  for (int ni = 0; ni < 8; ++ni) bo[ni] = (unsigned)((n0 + wc * 128 + ni * 16 + r16) * a.Kpad * 2 + 16 * h4);

  struct PatchO { int img, y0, x0; };
  auto patch_of = [&](int k) {
    const int t = (lin + k * G) / a.ntile_n;
    PatchO P;
    P.x0 = (t % ptx) * 32;
    const int r = t / ptx;
    P.y0 = (r % pty) * 8;
    P.img = r / pty;
    return P;
  };
  // one 16-B group g of the halo of chunk c of tile k (registers): out-of-image pixels read zeros, and so
  // does a group that is not to be loaded (ok = false: the K loop issues its two loads every step)
  auto halo_load = [&](int k, int c, int g, bool ok) -> v4u32_4 {
    const int idx = g * NTH + tid;
    const PatchO P = patch_of(k);
    const int hr = idx >> 3, hp = idx & 7;
    const int yi = P.y0 - 1 + hr / 34, xi = P.x0 - 1 + hr % 34;
    const int ci = c * 64;
    const bool srcb = ci >= a.CAs;
    const int cs = (srcb ? a.CBs : a.CAs) * 2, cb = (srcb ? ci - a.CAs : ci) * 2;
    const int sy = yi >> us, sx = xi >> us;
    const bool v = ok && idx < W4_HROWS * 8 && (unsigned)sy < (unsigned)a.Hs && (unsigned)sx < (unsigned)a.Ws;
    const unsigned off = v ? (unsigned)(((P.img * a.Hs + sy) * a.Ws + sx) * cs + cb + 16 * hp) : W4_OOB;
    return w4_ld16(srcb ? rsB : rsA, off);
  };
  // ... and its LDS store (ok = false, or past the 340 halo rows: into this thread's slot of a scratch row)
  auto halo_store = [&](int g, int slot, v4u32_4 v, bool ok) {
    const int idx = g * NTH + tid;
    const int hr = idx >> 3, hp = idx & 7;
    const unsigned off = ok && idx < W4_HROWS * 8 ? (unsigned)(slot * W4_HBUF + hr * ROWB + ((hp ^ (hr & 7)) << 4))
                                                  : (unsigned)(ODUM + tid * 16);
    *reinterpret_cast<v4u32_4*>(smem + off) = v;
  };

  const int nk = 9 * nch;
  const int total = mine * nk;
  // weight fragments (32-deep half s) of stream step g into B[.][s]: row kt = tap * nch + chunk
  auto load_B = [&](int g, int s, bf16x8 (&B)[8][2]) {
    const int t = g % nk, c = t / 9, tp = t - 9 * c;
    const unsigned kb = (unsigned)(tp * nch + c) * ROWB + 64 * s;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) B[ni][s] = __builtin_bit_cast(bf16x8, w4_ld16(rsW, bo[ni] + kb));
  };

  // LB: thread t stages rows (t >> 3) + 32 i (i < 8), 16-B chunk t & 7, of the step's 256 x 64 weight tile;
  // the LDS image uses the MFMA-fragment swizzle of conv_common.h (chunk c of row r at c ^ swz(r))
  unsigned wo[LB ? 8 : 1];
  if constexpr (LB) {
#pragma unroll
    for (int i = 0; i < 8; ++i) wo[i] = (unsigned)((n0 + (tid >> 3) + 32 * i) * a.Kpad * 2 + 16 * (tid & 7));
  }
  auto stage_load = [&](int g, v4u32_4 (&st)[8]) {
    const int t = g % nk, c = t / 9, tp = t - 9 * c;
    const unsigned kb = (unsigned)(tp * nch + c) * ROWB;
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = w4_ld16(rsW, wo[LB ? i : 0] + kb);
  };
  auto stage_store = [&](int buf, const v4u32_4 (&st)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = (tid >> 3) + 32 * i, cp = tid & 7;
      *reinterpret_cast<v4u32_4*>(smem + OBS + buf * BSTAGE + r * ROWB + ((cp ^ swz(r)) << 4)) = st[i];
    }
  };
  auto frag_B = [&](int buf, int s_, bf16x8 (&Bf)[8]) {
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int r = wc * 128 + ni * 16 + r16, cc = 4 * s_ + h4;
      Bf[ni] = *reinterpret_cast<const bf16x8*>(smem + OBS + buf * BSTAGE + r * ROWB + ((cc ^ swz(r)) << 4));
    }
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- epilogue of tile k from registers
  auto epilogue = [&](int k) {
    const PatchO P = patch_of(k);
    const int m0 = (P.img * a.Ho + P.y0) * a.Wo + P.x0;
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int cl = wc * 128 + ni * 16 + 4 * h4;
      const float4 b4 = *reinterpret_cast<const float4*>(cst + cl);
      const float bias[4] = {b4.x, b4.y, b4.z, b4.w};
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const int p = wr * 128 + mi * 16 + r16;
        const int m = m0 + (p >> 5) * a.Wo + (p & 31);
        float x[4];
        bf16x4_4 o;
        f32x4 v = acc[mi][ni];
        asm volatile("" : "+v"(v));   // one accumulator block at a time out of the AGPRs
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[r] = v[r] + bias[r];
          if (a.relu) x[r] = fmaxf(x[r], 0.f);
          o[r] = (__bf16)x[r];
          if constexpr (STATS) { s1[r] += x[r]; s2[r] += x[r] * x[r]; }
        }
        if constexpr (!(DBG & 4))
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_4, o), rsO,
                                                (unsigned)((m * a.out_stride + n0 + cl) * 2), 0, 0);
        else
          asm volatile("" ::"v"(o));
        acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (STATS) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[r] = row16_sum(s1[r]);
          s2[r] = row16_sum(s2[r]);
        }
        if (r16 == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            atomicAdd(&sacc[cl + r], (double)s1[r]);
            atomicAdd(&sacc[256 + cl + r], (double)s2[r]);
          }
        }
      }
    }
  };

  // ---- prologue: the first chunk's halo and the first weights
  const int hbase = (4 * wr) * 34 + r16;   // halo row of fragment mi = 0 at tap 0: patch row 4 wr, column r16
#pragma unroll
  for (int g = 0; g < W4_GH; ++g) halo_store(g, 0, halo_load(0, 0, g, true), true);
  v4u32_4 hs[2];
  hs[0] = hs[1] = v4u32_4{0u, 0u, 0u, 0u};
  if constexpr (LB) {
    v4u32_4 st[8];
    bf16x8 Bf0[8], Bf1[8];
    stage_load(0, st);
    stage_store(0, st);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    frag_B(0, 0, Bf0);
    int g = 0;
    for (int k = 0; k < mine; ++k) {
#pragma unroll 1
      for (int c = 0; c < nch; ++c) {
        const int slot = (k * nch + c) & 1;
        const bool has_next = c + 1 < nch || k + 1 < mine;
        const int k2 = c + 1 < nch ? k : k + 1, c2 = c + 1 < nch ? c + 1 : 0;
        const unsigned char* hb = smem + slot * W4_HBUF;
#pragma unroll 1
        for (int tp = 0; tp < 9; ++tp, ++g) {
          // (the step barrier below orders the halo slots: a chunk's halo is stored at its predecessor's taps
          // 1-6, and the slot it overwrites was last read at tap 8 of the chunk before, behind two barriers)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int gs_ = 2 * (tp - 1) + j;
            halo_store(gs_ < 0 ? 0 : gs_, slot ^ 1, hs[j], has_next && tp >= 1 && gs_ < W4_GH);
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int gl = 2 * tp + j;
            hs[j] = halo_load(k2, c2, gl, has_next && gl < W4_GH);
          }
          __builtin_amdgcn_sched_barrier(0);
          stage_load(g + 1 < total ? g + 1 : g, st);   // next step's weight tile, stored mid-step
          __builtin_amdgcn_sched_barrier(0);
          frag_B(g & 1, 1, Bf1);                          // this step's second half
          const int dy = tp / 3, dx = tp - 3 * dy;
          auto readA = [&](int q) {
            const int s_ = q >> 3, mi = q & 7;
            const int hr = hbase + ((mi >> 1) + dy) * 34 + (mi & 1) * 16 + dx, cc = 4 * s_ + h4;
            return *reinterpret_cast<const bf16x8*>(hb + hr * ROWB + ((cc ^ (hr & 7)) << 4));
          };
          bf16x8 Ar[3];
          Ar[0] = readA(0);
          Ar[1] = readA(1);
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            if (q + 2 < 16) Ar[(q + 2) % 3] = readA(q + 2);
            const int mi = q & 7;
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(q < 8 ? Bf0[ni] : Bf1[ni], Ar[q % 3], acc[mi][ni],
                                                                    0, 0, 0);
            if (q == 11) {   // next step's tile into the other stage; barrier; its first-half fragments
              __builtin_amdgcn_sched_barrier(0);
              stage_store((g + 1) & 1, st);
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
              __builtin_amdgcn_s_barrier();
              frag_B((g + 1) & 1, 0, Bf0);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
      }
      epilogue(k);
    }
  } else {
  // one register set of weight fragments: the half s is refilled with the next step's fragments as soon as
  // its 64 MFMAs are issued (half a K step of load cover)
  bf16x8 B[8][2];
  load_B(0, 0, B);
  load_B(0, 1, B);
  int g = 0;   // stream step
  for (int k = 0; k < mine; ++k) {
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      const int slot = (k * nch + c) & 1;
      // chunk start: its halo written by every wave, the other slot free for the next chunk
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();
      const bool has_next = c + 1 < nch || k + 1 < mine;
      const int k2 = c + 1 < nch ? k : k + 1, c2 = c + 1 < nch ? c + 1 : 0;
      const unsigned char* hb = smem + slot * W4_HBUF;
#pragma unroll 1
      for (int tp = 0; tp < 9; ++tp, ++g) {
        // next chunk of the stream: groups 2 tp, 2 tp + 1 loaded at tap tp, stored at tap tp + 1
        // (branch-free: every step stores two groups and issues two loads, the ones not needed aimed at the
        // scratch row / out of range, so the compiler's vmcnt bookkeeping stays exact across the loop)
        if constexpr (!(DBG & 2)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int gs_ = 2 * (tp - 1) + j;
          halo_store(gs_ < 0 ? 0 : gs_, slot ^ 1, hs[j], has_next && tp >= 1 && gs_ < W4_GH);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int gl = 2 * tp + j;
          hs[j] = halo_load(k2, c2, gl, has_next && gl < W4_GH);
        }
        }
        const int dy = tp / 3, dx = tp - 3 * dy;
        // activation fragment q = 8 s + mi, read two groups ahead of its 8 MFMAs (the LDS latency hides
        // behind the 16 MFMAs of the two groups before it)
        auto readA = [&](int q) {
          const int s_ = q >> 3, mi = q & 7;
          const int hr = hbase + ((mi >> 1) + dy) * 34 + (mi & 1) * 16 + dx, cc = 4 * s_ + h4;
          return *reinterpret_cast<const bf16x8*>(hb + hr * ROWB + ((cc ^ (hr & 7)) << 4));
        };
        bf16x8 Ar[3];
        Ar[0] = readA(0);
        Ar[1] = readA(1);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          if (q + 2 < 16) Ar[(q + 2) % 3] = readA(q + 2);
          const int s_ = q >> 3, mi = q & 7;
#pragma unroll
          for (int ni = 0; ni < 8; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(B[ni][s_], Ar[q % 3], acc[mi][ni], 0, 0, 0);
          if (mi == 7) {   // (pinned here: the scheduler would otherwise sink the loads to the end of the step)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!(DBG & 1)) load_B(g + 1 < total ? g + 1 : g, s_, B);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
    epilogue(k);
  }
  }

  // ---- BatchNorm sums of the block -> its replica of the accumulators (folded by the launcher)
  if constexpr (STATS) {
    if (ADP_DBG(a) & 2) return;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    double* rep = a.stat + (size_t)(blockIdx.x & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
    const int n = n0 + tid;
    if (n < a.Nout) {
      atomicAdd(rep + n, sacc[tid]);
      atomicAdd(rep + adp::STAT_CMAX + n, sacc[256 + tid]);
    }
  }
}

}  // namespace

namespace adp {
// 3x3 stride-1 'same' bf16 layers (optional nearest x2 upsample folded into the halo gather, one or two
// sources of 64-channel multiples) with Nout % 256 == 0 and a plain / bias / ReLU / BatchNorm-statistics
// epilogue. 0 = not eligible (the caller falls back).
int launch_fwd_w4(FwdArgs& a, hipStream_t s) {
  if (!option("fwd_w4", 0)) return 0;   // opt-in: slower than the 8-wave kernel (profiles/r03_w4_ab.txt)
  if (a.f8 || a.f32 || a.bnr_z || a.out_mode != 0 || a.addend || a.mask || a.mask2 || a.accum ||
      a.drop_rate > 0.f || a.scA || a.scB || !a.out)
    return 0;
  const int Cin_s = a.CAs + a.CBs;
  if (a.kh != 3 || a.kw != 3 || a.dil != 1 || a.pad != 1 || a.stride != 1 || (a.up != 1 && a.up != 2) ||
      a.Ho != a.Hs * a.up || a.Wo != a.Ws * a.up || a.Ho % 8 != 0 || a.Wo % 32 != 0 || a.CAs % 64 != 0 ||
      a.CBs % 64 != 0 || Cin_s == 0 || a.K != 9 * Cin_s || a.Kpad != a.K || a.Nout % 256 != 0 ||
      a.out_stride % 4 != 0 || a.out_stride < a.Nout)
    return 0;
  const size_t lim = (size_t)1 << 31, pix = (size_t)a.Nimg * a.Hs * a.Ws;
  if (pix * a.CAs * 2 >= lim || pix * a.CBs * 2 >= lim || (size_t)a.M * a.out_stride * 2 >= lim ||
      (size_t)a.Nout * a.Kpad * 2 >= lim)
    return 0;
  a.ntile_n = a.Nout / 256;
  a.nblocks = (a.M / 256) * a.ntile_n;   // 8 x 32 patches x N tiles
  int grid = std::min(a.nblocks, option("fwd_w4_grid", 256));
  grid -= grid % a.ntile_n;
  if (grid <= 0) grid = a.ntile_n;
  const int dbg = option("fwd_w4_dbg", 0);
  if (option("fwd_w4_lb", 1)) {
    if (a.bn_sum) {
      adp::set_kernel("igemm_fwd_w4_kernel<true, 0, true>");
      hipLaunchKernelGGL((igemm_fwd_w4_kernel<true, 0, true>), dim3(grid), dim3(256), 0, s, a);
    } else {
      adp::set_kernel("igemm_fwd_w4_kernel<false, 0, true>");
      hipLaunchKernelGGL((igemm_fwd_w4_kernel<false, 0, true>), dim3(grid), dim3(256), 0, s, a);
    }
    return 1;
  }
  if (a.bn_sum && dbg > 0 && dbg < 8) {
    adp::set_kernel("igemm_fwd_w4_kernel<true, %d, false>", dbg);
#define W4_DBG(D) if (dbg == D) hipLaunchKernelGGL((igemm_fwd_w4_kernel<true, D>), dim3(grid), dim3(256), 0, s, a)
    W4_DBG(1); W4_DBG(2); W4_DBG(3); W4_DBG(4); W4_DBG(5); W4_DBG(6); W4_DBG(7);
#undef W4_DBG
  } else if (a.bn_sum) {
    adp::set_kernel("igemm_fwd_w4_kernel<true, 0, false>");
    hipLaunchKernelGGL(igemm_fwd_w4_kernel<true>, dim3(grid), dim3(256), 0, s, a);
  } else {
    adp::set_kernel("igemm_fwd_w4_kernel<false, 0, false>");
    hipLaunchKernelGGL(igemm_fwd_w4_kernel<false>, dim3(grid), dim3(256), 0, s, a);
  }
  return 1;
}
}  // namespace adp
