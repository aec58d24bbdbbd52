// Halo-reuse 3x3 convolution ("halo") for the narrow, full-resolution layers: 3x3, stride 1, dilation
// 1, 'same' padding, Cin_s % 64 == 0 and at most 128 output channels (unet_bn levels 0-1 forward and
// data-gradient launches). Semantics are those of igemm_fwd_kernel (conv_igemm.hip).
//
// Why: with 64-128 output columns the implicit GEMM re-gathers every input pixel once per tap (9x) and
// the LDS-DMA gather rate, not the MFMA rate, bounds the tap64 kernel. Here a block owns an 8 x 32
// output patch; per 64-channel input chunk it moves the 10 x 34 input halo into LDS once and all nine
// taps read shifted 16-pixel windows of it (340 instead of 2304 pixel rows per chunk, 6.8x less A
// traffic). The weights stream per tap through a 3-deep LDS ring.
//
// Block: 4 (M) x WN (N) x KS waves, each 64 output pixels (two patch rows of 32) x 64 channels = 4 x 4
// v_mfma_f32_16x16x32_bf16 accumulators; with KS = 2 (the 64-channel layers) the two wave groups take
// the two 32-deep halves of every step and their accumulators are summed through LDS at the end, so
// that two waves share each SIMD. LDS: 2 halo buffers (double-buffered over chunks) + 3 weight
// slots, all filled by global_load_lds_dwordx4 with the XOR chunk swizzle on the source address.
// K loop: step s = chunk * ceil(9/TPS) + j covers taps j*TPS ..; at step s the block issues the weights
// of step s+2 (and, at a chunk's first step, the next chunk's halo) and retires step s+1 with one
// counted vmcnt before the step's barrier. The 64-channel layers take two taps per step.
#include <type_traits>

#include "conv_common.h"

namespace {

__device__ __attribute__((aligned(256))) uint4 halo_zero_page[64];

constexpr int PH = 8, PW = 32;                  // output patch
constexpr int HH = PH + 2, HW = PW + 2;         // input halo
constexpr int HROWS = HH * HW;                  // 340 halo pixels
constexpr int ROWB = 128;                       // 64 bf16 channels per LDS row

// 16-B chunk swizzle of the halo rows: c ^ (r & 7). The taps read 16 consecutive halo rows from ANY
// base row ((wave + dy) * HW + mf * 16 + dx), and with swz(r) = (r >> 1) & 7 three bases in four put two
// lanes of a ds_read_b128 lane group on one bank quad (8 LDS cycles instead of 4); r & 7 is conflict-free
// for every base (the weight rows keep swz: their bases are multiples of 16).
__device__ __forceinline__ int hswz(int r) { return r & 7; }

// LDS-only barrier: this wave's LDS traffic done, then the hardware barrier. Unlike __syncthreads() it does
// not wait for outstanding global stores / LDS-DMA prefetches (its workgroup fence drains vmcnt).
#define LDS_BAR()                                             \
  do {                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
    __builtin_amdgcn_s_barrier();                             \
    asm volatile("" ::: "memory");                            \
  } while (0)

#define HALO_BAR()                         \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_s_barrier();          \
    asm volatile("" ::: "memory");         \
  } while (0)

// TPS taps per K step (a weight slot holds TPS taps; steps per chunk = ceil(9 / TPS)). NHB halo
// buffers: 2 double-buffers the halo over input chunks; 1 (single-chunk layers, Cin_s == 64) halves the
// LDS footprint so that two blocks share a CU and one block's halo load overlaps the other's MFMAs.
template <int WN, int KS, int TPS, int NHB>
constexpr int halo_lds() {
  constexpr int NTH = 4 * WN * KS * 64;
  constexpr int GH = (HROWS * 8 + NTH - 1) / NTH;
  return NHB * (GH * NTH / 8) * ROWB + 3 * TPS * WN * 64 * ROWB;
}

template <int WN, int KS, int TPS, int NHB, bool BNR>
__global__ __launch_bounds__(4 * WN * KS * 64, (halo_lds<WN, KS, TPS, NHB>() <= 81920 ? 2 : 1))
void igemm_fwd_halo_kernel(FwdArgs a) {
  constexpr int NTH = 4 * WN * KS * 64;
  constexpr int BN = WN * 64;
  constexpr int SPC = (9 + TPS - 1) / TPS;
  constexpr int GH = (HROWS * 8 + NTH - 1) / NTH;          // halo glds per thread per chunk
  constexpr int HROWS_PAD = GH * NTH / 8;                  // rows the last instruction may touch
  constexpr int HBUF = HROWS_PAD * ROWB;
  constexpr int GB1 = BN * 8 / NTH;                        // weight glds per thread per tap
  static_assert(GB1 * NTH == BN * 8, "weight slot must split evenly");
  constexpr int GB = GB1 * TPS;                            // ... per step
  constexpr int WTAP = BN * ROWB;
  constexpr int WSLOT = TPS * WTAP;
  constexpr int OFF_W = NHB * HBUF;
  constexpr int LT = BN + 4;
  constexpr int EPI = PH * PW * LT * 4;
  constexpr int SMEM = (OFF_W + 3 * WSLOT > EPI) ? OFF_W + 3 * WSLOT : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % 4, wn = (wave / 4) % WN, kh = wave / (4 * WN);
  // block -> (n-tile, image, patch row, patch col), n-tile fastest, XCD-grouped
  const int tx_n = a.Wo / PW, ty_n = a.Ho / PH;
  const int lin = xcd_remap(blockIdx.x, a.nblocks);
  const int tn = lin % a.ntile_n;
  int rest = lin / a.ntile_n;
  const int px = rest % tx_n; rest /= tx_n;
  const int py = rest % ty_n;
  const int img = rest / ty_n;
  const int y0 = py * PH, x0 = px * PW, n0 = tn * BN;
  const int Cin_s = a.CAs + a.CBs;
  const int nchunk = Cin_s / 64, nsteps = nchunk * SPC;
  const int Wrows = (a.Nout + 63) / 64 * 64;
  const bf16* srcA = reinterpret_cast<const bf16*>(a.srcA);
  const bf16* srcB = reinterpret_cast<const bf16*>(a.srcB);

  // ---- halo slots of this thread: pixel offset (image-relative) or -1 (padding / beyond the halo)
  int hoff[GH], hcol[GH];
#pragma unroll
  for (int i = 0; i < GH; ++i) {
    const int idx = i * NTH + tid;
    const int hr = idx >> 3, pos = idx & 7;
    hcol[i] = 8 * (pos ^ hswz(hr));
    const int gy = y0 - 1 + hr / HW, gx = x0 - 1 + hr % HW;
    hoff[i] = (hr < HROWS && gy >= 0 && gy < a.Hs && gx >= 0 && gx < a.Ws) ? (img * a.Hs + gy) * a.Ws + gx : -1;
  }
  // ---- weight slots: row q of the slot = output channel n0 + q
  const bf16* wp[GB1];
#pragma unroll
  for (int i = 0; i < GB1; ++i) {
    const int idx = i * NTH + tid;
    const int q = idx >> 3, pos = idx & 7;
    wp[i] = (n0 + q < Wrows) ? reinterpret_cast<const bf16*>(a.W) + (size_t)(n0 + q) * a.Kpad + 8 * (pos ^ swz(q))
                             : nullptr;
  }

  auto issue_halo = [&](int c, int buf) {
    const int ci = c * 64;
    const bf16* base = ci < a.CAs ? srcA + ci : srcB + (ci - a.CAs);
    const int cs = ci < a.CAs ? a.CAs : a.CBs;
    unsigned char* dst = smem + buf * HBUF + wave * 8 * ROWB;
#pragma unroll
    for (int i = 0; i < GH; ++i) {
      const void* p = hoff[i] >= 0 ? (const void*)(base + (size_t)hoff[i] * cs + hcol[i]) : (const void*)halo_zero_page;
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(dst + i * (NTH / 8) * ROWB), 16, 0, 0);
    }
  };
  auto issue_w = [&](int s) {
    const int c = s / SPC, j = s - SPC * c;
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      const int t = j * TPS + u;                 // t == 9 only in a chunk's short last step: a zero load
      const int k = t * Cin_s + c * 64;          // keeps the per-step glds count uniform
      unsigned char* dst = smem + OFF_W + (s % 3) * WSLOT + u * WTAP + wave * 8 * ROWB;
#pragma unroll
      for (int i = 0; i < GB1; ++i) {
        const void* p = (wp[i] && t < 9) ? (const void*)(wp[i] + k) : (const void*)halo_zero_page;
        __builtin_amdgcn_global_load_lds(p, (lds_void*)(dst + i * (NTH / 8) * ROWB), 16, 0, 0);
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, h4 = lane >> 4;
  // ---- prologue: halo(0), weights(0), weights(1); retire halo(0) + weights(0)
  issue_halo(0, 0);
  issue_w(0);
  if (nsteps > 1) {
    issue_w(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GB) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  HALO_BAR();

  for (int s = 0; s < nsteps; ++s) {
    const int c = s / SPC, j = s - SPC * c;
    const bool nh = NHB == 2 && j == 0 && c + 1 < nchunk;   // prefetch the next chunk's halo
    if (nh) issue_halo(c + 1, (c + 1) & 1);
    const bool nw = s + 2 < nsteps;
    if (nw) issue_w(s + 2);
    const unsigned char* H = smem + (NHB == 2 ? (c & 1) : 0) * HBUF;
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
    const int t = j * TPS + u;
    if (t >= 9) break;
    // ---- 64 pixels x 64 channels x 64 deep of tap t for this wave
    const int dy = t / 3, dx = t - 3 * dy;
    const unsigned char* Wt = smem + OFF_W + (s % 3) * WSLOT + u * WTAP;
#pragma unroll
    for (int kq = 0; kq < 2 / KS; ++kq) {
      const int ck = 4 * (KS == 2 ? kh : kq) + h4;
      bf16x8 fb[4], fa[4];
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) {
        const int q = wn * 64 + nf * 16 + r16;
        fb[nf] = *reinterpret_cast<const bf16x8*>(Wt + q * ROWB + ((ck ^ swz(q)) << 4));
      }
#pragma unroll
      for (int mf = 0; mf < 4; ++mf) {
        const int prow = 2 * wm + (mf >> 1), pcol = (mf & 1) * 16 + r16;
        const int hr = (prow + dy) * HW + pcol + dx;
        fa[mf] = *reinterpret_cast<const bf16x8*>(H + hr * ROWB + ((ck ^ hswz(hr)) << 4));
      }
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mf], fb[nf], acc[mf][nf], 0, 0, 0);
    }
    }
    // retire step s+1 (weights of s+1 and, at a chunk boundary, the halo of chunk c+1, both issued
    // before this step's issues) before the barrier that precedes its reads
    if (nw) {
      if (nh) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GB + GH) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    HALO_BAR();
  }

  // ---- epilogue: accumulators -> LDS tile [patch pixel][channel] -> one patch row at a time
  float* tile = reinterpret_cast<float*>(smem);
  const int col = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int part = 0; part < KS; ++part) {   // KS = 2: k-half 0 stores, k-half 1 adds
    if (kh == part) {
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = (2 * wm + (mf >> 1)) * PW + (mf & 1) * 16 + rq + r;
            float* e = tile + p * LT + wn * 64 + nf * 16 + col;
            *e = part == 0 ? acc[mf][nf][r] : *e + acc[mf][nf][r];
          }
    }
    ADP_LDS_BARRIER();
  }
  float bs[8], bq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bs[j] = 0.f; bq[j] = 0.f; }
  for (int pr = 0; pr < PH; ++pr) {
    const int m0 = (img * a.Ho + y0 + pr) * a.Wo + x0;
    if constexpr (BNR) epi_rows_bnr<NTH, BN>(a, tile + pr * PW * LT, PW, m0, n0, tid, bs, bq);
    else epi_rows<NTH, BN>(a, tile + pr * PW * LT, PW, m0, n0, tid, bs, bq);
  }
  if (a.bn_sum || a.bnr_z) epi_bn_flush<NTH, BN>(a, tile, n0, tid, bs, bq);
}

// Persistent form for the single-chunk layers (Cin_s == 64) with <= 64 output channels or 128 in two
// 64-channel halves (unet_bn level-0 64->64 convs and their data gradients, enc1_conv1 64->128, the
// split data gradient of dec0_conv1). One block (8 waves, one patch row of 32
// pixels each, full K) per CU walks tiles lin, lin + G, ... All nine weight taps stay resident in LDS
// for the whole launch (the one-tile kernel's per-tap weight ring waits ~1 us per LDS-DMA fill); the
// product is computed transposed (C^T = W X^T: a lane holds 4 consecutive output channels of one
// pixel), so each wave stores its outputs straight from the accumulators (8-B vectors) with no LDS
// staging and no barrier; the next tile's halo is prefetched into registers at the first tap and
// written to the single LDS halo buffer between two barriers; BatchNorm sums stay in registers until
// the block's last tile and go to the accumulator replicas once per wave.
#ifndef HALOP_VALU_PER_MFMA
#define HALOP_VALU_PER_MFMA 8
#endif
// EPI (non-BNR launches): 0 plain store, 1 + BatchNorm statistics, 2 + ReLU, 3 + ReLU + statistics of the
// stored values, 4 + addend and / or ReLU-backward mask (the data gradients of the adipose_v3 convs:
// out = (acc + addend) * (mask > 0 ? mask_scale : 0), mask2 / mask2_scale on a split store's second part,
// the arithmetic of epi_rows), 5 + ReLU + inverted dropout (adipose_v3's Dropout after up*_conv3: the
// stateless hash of epi_rows, so the mask matches every other kernel's) -- compile-time, so the epilogue
// carries no per-element selects for the launch-uniform flags
// WIDE: the epilogue handles the channel quads of 16-channel groups nf and nf + 1 together and joins them
// with v_permlane16_swap into 8-channel runs (lane row h4 then holds channels 16 (nf + (h4 & 1)) + 8 (h4 >> 1)
// .. + 7 of its pixel): one 16-B store per pair of units instead of two 8-B ones (the persistent forward's
// tap64p_wide); needs the store limit (Nout, or split_c for the first part) on an 8-channel boundary
// DYN: tiles claimed from a counter (a.claim) instead of the static list -- a compile-time form, since the
// claimed tile id and the pending claim cost registers the tightest forms do not have
// SWP (round 5): software-pipelined fragment reads -- the LDS reads of K step s + 1 are issued before the MFMAs of step
// s (two fragment sets in registers), so a wave no longer waits for its own step's reads before every MFMA cluster.
// Without it each step is "6 reads, wait, 8 MFMAs" and the waves, which leave each tile's barriers together, read
// and multiply in phase: with the halo loads removed (timing ablation, profiles/r05g_halop_ablation.log) the L0
// 64 -> 64 forward still ran at only 1.16 PF.
template <int I, int N, typename F>
__device__ __forceinline__ void halop_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    halop_static_for<I + 1, N>(f);
  }
}
// EPI_ 6 (round 5, BNL): EPI 1 (statistics) on a source A read pre-BatchNorm: every halo chunk goes through
// relu(z * scale + shift) (a.scA / a.shA: adp_bn_apply's arithmetic, bit-identical; out-of-image chunks stay 0) on its
// way from the registers into LDS, and the blocks of output block 0 store the interior chunks of each patch -- every
// pixel of the activation exactly once over the launch -- to a.act_out (which the weight gradient reads later). It
// replaces the adp_bn_apply pass between the two convs of a unet_bn level (read z + write act, then the conv reads
// act) by the conv's own read of z plus the act stores. The next patch's chunks are applied in the registers they were
// loaded into, chunk j between the MFMAs of tap 3 + j (kq 1), so that only the LDS stores remain at the tile's end (applied
// there, after the barrier, the one-chunk forward ran 20 % and the two-chunk one 44 % longer; profiles/r05u_*).
template <bool BNR, int NCH, int BN, bool PIPE, int EPI_, bool WIDE = false, bool DYN = false, bool SWP = false>
__global__ __launch_bounds__(512, 1) void igemm_fwd_halop_kernel(FwdArgs a) {
  constexpr bool BNL = EPI_ == 6;
  constexpr int EPI = BNL ? 1 : EPI_;
  static_assert(!BNL || (!BNR && !DYN && !SWP && NCH == 1), "BN-on-load: one-chunk static-list forward launches");
  static_assert(!BNR || EPI == 0, "the BN-backward reduction launch stores the plain product");
  static_assert(EPI < 4 || !PIPE, "mask / addend quads, the dropout hash and two accumulator sets: registers");
  // NCH 64-channel input chunks (1: Cin_s 64; 2: Cin_s 128 from one or two sources), BN output channels
  // per block (64, or 32 for two chunks: 2 x 340 halo rows + 9 x 2 x 32 weight rows = 157 KiB of LDS)
  constexpr int NTH = 512, NF = BN / 16;
  constexpr int HCH = NCH * HROWS * 8;                      // 16-B halo chunks (all input chunks)
  constexpr int GH = (HCH + NTH - 1) / NTH;                 // halo chunks per thread
  // (BNL applies the next patch's chunk j between the MFMAs of tap 3 + j, taps 3..8: six chunks at most, or later
  //  chunks would reach LDS without the BatchNorm-ReLU -- round-5 ADVICE)
  static_assert(!BNL || GH <= 6, "BN-on-load: at most six halo chunks per thread");
  constexpr int HBUF = HCH * 16;
  constexpr int GW = 9 * NCH * BN * 8 / NTH;                // resident weight chunks per thread
  constexpr int WTAP = NCH * BN * ROWB;
  constexpr int OFF_W = HBUF, OFF_C = OFF_W + 9 * WTAP;
  constexpr int OFF_S = OFF_C + 5 * BN * 4 + 16;            // + per-channel epilogue constants, claimed-tile ring
  constexpr int SMEM = OFF_S + (BNL ? 2 * NCH * 64 * 4 : 0); // + BNL: scale | shift of the input channels
  static_assert(GW * NTH == 9 * NCH * BN * 8, "weights must split evenly");
  static_assert(SMEM <= 160 * 1024, "LDS");
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  typedef unsigned int v2u32_h __attribute__((ext_vector_type(2)));
  typedef unsigned int v4u32_h __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // = patch row
  prio_static<ADP_PRIO_FWD>(wave);
  const int tx_n = a.Wo / PW, ty_n = a.Ho / PH;
  const int T = a.nblocks, G = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, G);
  // tiles: the static list lin, lin + G, ... (nt of them), or (dyn, conv_common.h) super-tiles of CH consecutive
  // patches claimed from the counter of the block's output block: super-tiles 0 and 1 are the block's static
  // ones (nothing to wait for at the start), claim value c is super-tile 2 G / NT + c; super-tile s + 2 is
  // claimed at the start of super-tile s and published at the end of its first tile (the halo prefetch needs a
  // tile's successor at the start of the tile)
  constexpr bool dyn = DYN;
  const bool full = dyn && a.claim_full;   // every super-tile claimed (0 and 1 by one claim at the start)
  const int nt = dyn ? 0 : (lin < T ? (T - lin + G - 1) / G : 0);
  if (!dyn && nt == 0) return;
  const int Wrows = (a.Nout + 63) / 64 * 64;
  // ntile_n = NT output blocks of BN channels: tile t = NT * patch + block, the grid is a multiple of
  // NT, so a block keeps one output block (its resident weights) and the blocks of a patch run side by
  // side on one XCD (halo shared through L2). A split store (out_mode 2) sends channels >= split_c to
  // out2 (split_c a multiple of BN).
  const int NT = a.ntile_n;
  const int nh = lin % NT, n0 = BN * nh;
  const bool second = a.out_mode == 2 && n0 >= a.split_c;
  bf16* obase = reinterpret_cast<bf16*>(second ? a.out2 : a.out);
  const int ostride = second ? a.out2_stride : a.out_stride;
  const int ocol0 = second ? n0 - a.split_c : n0;
  const int nlim = a.out_mode == 2 && !second ? a.split_c : a.Nout;
  const int Cin_s = a.CAs + a.CBs;

  int* ring = reinterpret_cast<int*>(smem + OFF_C + 5 * BN * 4);
  const int npatch = T / NT;
  const int CH = dyn ? a.claim_chunk : 1, nsup = (npatch + CH - 1) / CH;
  auto sup_id = [&](int sidx) -> int {   // dyn: super-tile index of the block's local super-tile sidx, -1 past the end
    const int v = full ? claim_ring_read(ring + (sidx & 3))
                       : sidx < 2 ? lin / NT + sidx * (G / NT) : 2 * (G / NT) + claim_ring_read(ring + (sidx & 3));
    return v < nsup ? v : -1;
  };
  // patch index of the block's local tile k, -1 past its end
  auto tile_id = [&](int k) -> int {
    if (!dyn) return k < nt ? lin / NT + k * (G / NT) : -1;
    const int v = sup_id(k / CH);
    const int t = v * CH + k % CH;
    return v >= 0 && t < npatch ? t : -1;
  };
  if (full) {
    if (tid == 0) {
      const int r = claim_next2(a.claim + nh);
      ring[0] = r;
      ring[1] = r + 1;
    }
    __syncthreads();
  }
  if (dyn && tile_id(0) < 0) {   // (uniform) more blocks than super-tiles (full: the work is taken already)
    if (tid == 0) claim_block_done(a.claim, NT, G);
    return;
  }
  auto tile_origin = [&](int t, int& img, int& y0, int& x0) {   // (t: the patch index from tile_id)
    const int px = t % tx_n, r = t / tx_n;
    y0 = (r % ty_n) * PH;
    img = r / ty_n;
    x0 = px * PW;
  };
  // halo gather of group i: chunk idx = i * NTH + tid -> (input chunk cc, halo row hr, 16-B position pos);
  // derived per call (a few VALU per group and tile) instead of held in 5 x GH registers per thread, which
  // the pipelined epilogue needs. pos = tid & 7 for every group (NTH and HROWS * 8 are multiples of 8).
  auto halo_src = [&](int img, int y0, int x0, int i) -> const uint4* {
    const int idx = i * NTH + tid;
    const int cc = NCH == 1 ? 0 : (idx >= HROWS * 8 ? 1 : 0), hr = (idx - cc * HROWS * 8) >> 3;
    const int hy = hr / HW, hx = hr - hy * HW;
    // (gy, gx) in the conv's input grid = the source upsampled x a.up (nearest: source (gy >> 1, gx >> 1))
    const int gy = y0 + hy - 1, gx = x0 + hx - 1, us = a.up >> 1;
    const bool ok = (i < GH - 1 || idx < HCH) && (unsigned)gy < (unsigned)(a.Hs << us) && (unsigned)gx < (unsigned)(a.Ws << us);
    if (!ok) return nullptr;
    const bool inA = cc * 64 < a.CAs;
    const bf16* src = reinterpret_cast<const bf16*>(inA ? a.srcA : a.srcB);
    const int cs = inA ? a.CAs : a.CBs;
    return reinterpret_cast<const uint4*>(src + (size_t)((img * a.Hs + (gy >> us)) * a.Ws + (gx >> us)) * cs +
                                          (inA ? cc * 64 : cc * 64 - a.CAs) + 8 * ((tid & 7) ^ hswz(hr)));
  };

  // BNL: the applied halo chunk i of patch (img, y0, x0) (returned; v as loaded, zeros outside the image). Branch-free:
  // the act store goes through a buffer resource, lanes with nothing to store aim past its end
  const float* sS = reinterpret_cast<const float*>(smem + OFF_S);
  const bool act_w = BNL && n0 == 0 && a.act_out != nullptr && !(ADP_DBG(a) & 4096);   // (fwd_debug bit 12: timing)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      a.act_out, 0, act_w ? a.Nimg * a.Hs * a.Ws * a.CAs * 2 : 0, 0x00020000);
  auto bnl = [&](uint4 v, int img, int y0, int x0, int i) -> uint4 {
    const int idx = i * NTH + tid;
    const int cc = NCH == 1 ? 0 : (idx >= HROWS * 8 ? 1 : 0), hr = (idx - cc * HROWS * 8) >> 3;
    const int hy = hr / HW, hx = hr - hy * HW;
    const int gy = y0 + hy - 1, gx = x0 + hx - 1;   // (up == 1)
    const bool inimg = (unsigned)gy < (unsigned)a.Hs && (unsigned)gx < (unsigned)a.Ws;
    const int c0 = cc * 64 + 8 * ((tid & 7) ^ hswz(hr));
    Grp<bf16> g;
    g.v = v;
    // (two halves of four channels: fewer registers live at once in the K loop the apply sits in)
    bf16* e = reinterpret_cast<bf16*>(&g.v);
#pragma unroll
    for (int hv = 0; hv < 2; ++hv) {
      const float4 q = *reinterpret_cast<const float4*>(sS + c0 + 4 * hv);
      const float4 r = *reinterpret_cast<const float4*>(sS + NCH * 64 + c0 + 4 * hv);
      e[4 * hv + 0] = (bf16)fmaxf(fmaf((float)e[4 * hv + 0], q.x, r.x), 0.f);
      e[4 * hv + 1] = (bf16)fmaxf(fmaf((float)e[4 * hv + 1], q.y, r.y), 0.f);
      e[4 * hv + 2] = (bf16)fmaxf(fmaf((float)e[4 * hv + 2], q.z, r.z), 0.f);
      e[4 * hv + 3] = (bf16)fmaxf(fmaf((float)e[4 * hv + 3], q.w, r.w), 0.f);
    }
    const bool wr = inimg && hy >= 1 && hy <= PH && hx >= 1 && hx <= PW;
    const unsigned off = wr ? (unsigned)((((img * a.Hs + gy) * a.Ws + gx) * a.CAs + c0) * 2) : 0x80000000u;
    if (act_w) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_h, g.v), rsA, off, 0, 0);
    return inimg ? g.v : v;
  };

  // ---- prologue: nine weight taps (resident), first halo, per-channel constants
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int idx = i * NTH + tid;             // chunk idx of the [tap][input chunk][row q][8 chunks] image
    const int tc = idx / (BN * 8), rem = idx - tc * BN * 8;
    const int t = tc / NCH, cc = tc - t * NCH;
    const int q = rem >> 3, pos = rem & 7;
    const void* p = n0 + q < Wrows
                        ? (const void*)(reinterpret_cast<const bf16*>(a.W) + (size_t)(n0 + q) * a.Kpad + t * Cin_s + cc * 64 +
                                        8 * (pos ^ swz(q)))
                        : (const void*)halo_zero_page;
    __builtin_amdgcn_global_load_lds(p, (lds_void*)(smem + OFF_W + (size_t)(i * NTH + wave * 64) * 16), 16, 0, 0);
  }
  int img0, y00, x00;
  tile_origin(tile_id(0), img0, y00, x00);
#pragma unroll
  for (int i = 0; i < GH; ++i) {
    if (i * NTH + tid < HCH) {
      const uint4* p = halo_src(img0, y00, x00, i);
      __builtin_amdgcn_global_load_lds(p ? (const void*)p : (const void*)halo_zero_page,
                                       (lds_void*)(smem + (size_t)(i * NTH + wave * 64) * 16), 16, 0, 0);
    }
  }
  float* cst = reinterpret_cast<float*>(smem + OFF_C);      // [5][BN]: bias | scale shift mean invstd
  if (tid < BN) {
    const int c = n0 + tid;
    const bool v = c < a.Nout;
    cst[tid] = (!BNR && a.bias && v) ? a.bias[c] : 0.f;
    cst[BN + tid] = (BNR && v) ? a.bnr_sc[c] : 0.f;
    cst[2 * BN + tid] = (BNR && v) ? a.bnr_sh[c] : 0.f;
    cst[3 * BN + tid] = (BNR && v) ? -a.bnr_mean[c] * a.bnr_invstd[c] : 0.f;   // xhat = z * invstd + this
    cst[4 * BN + tid] = (BNR && v) ? a.bnr_invstd[c] : 0.f;
  }
  if constexpr (BNL) {
    float* sw = reinterpret_cast<float*>(smem + OFF_S);
    if (tid < NCH * 64) {
      sw[tid] = a.scA[tid];
      sw[NCH * 64 + tid] = a.shA[tid];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (BNL) {   // the first patch's halo came in by LDS-DMA: each thread applies its own chunks in place
#pragma unroll
    for (int i = 0; i < GH; ++i)
      if (i * NTH + tid < HCH) {
        uint4* q = reinterpret_cast<uint4*>(smem + (size_t)(i * NTH + tid) * 16);
        *q = bnl(*q, img0, y00, x00, i);
      }
    __syncthreads();
  }

  const int r16 = lane & 15, h4 = lane >> 4;
  constexpr bool stats = BNR || EPI == 1 || EPI == 3;
  float s1[NF][4], s2[NF][4];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf)
#pragma unroll
    for (int i = 0; i < 4; ++i) { s1[nf][i] = 0.f; s2[nf][i] = 0.f; }

  // the store target as a buffer resource: a lane whose channel quad lies past nlim stores to an
  // out-of-range offset (dropped) instead of branching around the store, so the epilogue has no divergent
  // control flow and its units can sit between the MFMAs of the next tile (PIPE)
  const __amdgpu_buffer_rsrc_t rsO =
      __builtin_amdgcn_make_buffer_rsrc((void*)obase, 0, a.M * ostride * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsZ = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BNR ? a.bnr_z : a.out), 0, BNR ? a.M * a.bnr_zs * 2 : 0, 0x00020000);
  // EPI 4: the mask (mask2 on a split store's second part) and the addend (first part only) of the block
  const void* mptr = second ? a.mask2 : a.mask;
  const int mstr = second ? a.mask2_stride : a.mask_stride;
  const float mscale = second ? a.mask2_scale : a.mask_scale;
  const bool has_mask = EPI == 4 && mptr != nullptr, has_add = EPI == 4 && !second && a.addend != nullptr;
  const __amdgpu_buffer_rsrc_t rsM =
      __builtin_amdgcn_make_buffer_rsrc((void*)mptr, 0, has_mask ? a.M * mstr * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsD =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.addend, 0, has_add ? a.M * a.addend_stride * 2 : 0, 0x00020000);
  // BNR: the z quads of one accumulator tile; EPI 4: its mask and addend quads (at the store's column)
  auto load_q = [&](__amdgpu_buffer_rsrc_t rs, int str, int col0, int mrow_, uint2 (&zr)[2][NF]) {
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
        const int c0 = nf * 16 + 4 * h4;
        const unsigned off = n0 + c0 < nlim ? (unsigned)(((mrow_ + mf * 16 + r16) * str + col0 + c0) * 2) : 0x80000000u;
        zr[mf][nf] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
      }
  };
  auto load_z = [&](int mrow_, uint2 (&zr)[2][NF]) {
    if (ADP_DBG(a) & 8192) {   // (timing-only ablation, fwd_debug bit 13: no z loads)
#pragma unroll
      for (int mf = 0; mf < 2; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) zr[mf][nf] = uint2{0u, 0u};
      return;
    }
    load_q(rsZ, a.bnr_zs, n0, mrow_, zr);
  };
  // epilogue of accumulator tile (mf, nf): lane = pixel mrow_ + mf*16 + r16, channels nf*16 + 4*h4 .. +3;
  // returns the stored quad (the BatchNorm sums are taken here), epi_unit / epi_pair store it
  auto epi_vals = [&](int mf, int nf, const f32x4& av, uint2 zv, int mrow_, uint2 dv = uint2{0u, 0u}) -> bf16x4 {
    const int c0 = nf * 16 + 4 * h4;
    const float4 cb = *reinterpret_cast<const float4*>(cst + c0);
    const int m = mrow_ + mf * 16 + r16;
    float v[4] = {av[0] + cb.x, av[1] + cb.y, av[2] + cb.z, av[3] + cb.w};
    if constexpr (EPI == 4) {   // epi_rows: + addend, then the mask
      const bf16x4 dd = __builtin_bit_cast(bf16x4, dv), mm = __builtin_bit_cast(bf16x4, zv);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (has_add) v[i] += (float)dd[i];
        if (has_mask) v[i] = (float)mm[i] > 0.f ? v[i] * mscale : 0.f;
      }
    }
    if constexpr (EPI == 5) {   // epi_rows: ReLU, then the dropout of element (m, channel)
      const float ks = 1.f / (1.f - a.drop_rate);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float u = adp_uniform(a.drop_seed, (uint64_t)m * (uint64_t)a.Nout + (n0 + c0 + i));
        v[i] = u >= a.drop_rate ? fmaxf(v[i], 0.f) * ks : 0.f;
      }
    }
    bf16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (EPI == 2 || EPI == 3) v[i] = fmaxf(v[i], 0.f);
      o[i] = (bf16)v[i];
    }
    if constexpr (BNR) {
      if (ADP_DBG(a) & 16384) return o;   // (timing-only ablation, fwd_debug bit 14: no BN-backward sums)
      const float4 sc = *reinterpret_cast<const float4*>(cst + BN + c0);
      const float4 sh = *reinterpret_cast<const float4*>(cst + 2 * BN + c0);
      const float4 nm = *reinterpret_cast<const float4*>(cst + 3 * BN + c0);
      const float4 is = *reinterpret_cast<const float4*>(cst + 4 * BN + c0);
      const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
      const float nmv[4] = {nm.x, nm.y, nm.z, nm.w}, isv[4] = {is.x, is.y, is.z, is.w};
      bf16x4 zz = __builtin_bit_cast(bf16x4, zv);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float g = (float)o[i], zf = (float)zz[i];   // the stored (rounded) gradient
        const float db = fmaf(zf, scv[i], shv[i]) > 0.f ? g : 0.f;   // (z = 0 past nlim: sc = sh = 0 there)
        s1[nf][i] += db;
        s2[nf][i] = fmaf(db, fmaf(zf, isv[i], nmv[i]), s2[nf][i]);   // db * (z - mean) * invstd
      }
    } else if constexpr (EPI == 1 || EPI == 3) {
      // (no channel mask: channels past nlim accumulate zero products and the final flush skips them)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s1[nf][i] += v[i];
        s2[nf][i] = fmaf(v[i], v[i], s2[nf][i]);
      }
    }
    return o;
  };
  auto epi_unit = [&](int mf, int nf, const f32x4& av, uint2 zv, int mrow_, uint2 dv = uint2{0u, 0u}) {
    const bf16x4 o = epi_vals(mf, nf, av, zv, mrow_, dv);
    const int c0 = nf * 16 + 4 * h4, m = mrow_ + mf * 16 + r16;
    const unsigned off = n0 + c0 < nlim ? (unsigned)((m * ostride + ocol0 + c0) * 2) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_h, o), rsO, off, 0, 0);
  };
  // WIDE: the stored quads o0 / o1 of units (mf, nf) and (mf, nf + 1), nf even, as one 16-B store per lane
  auto epi_join = [&](int mf, int nf, v2u32_h o0, v2u32_h o1, int mrow_) {
    const auto e0 = __builtin_amdgcn_permlane16_swap(o0.x, o1.x, false, false);
    const auto e1 = __builtin_amdgcn_permlane16_swap(o0.y, o1.y, false, false);
    const v4u32_h st = {e0[0], e1[0], e0[1], e1[1]};
    const int cw = 16 * (nf + (h4 & 1)) + 8 * (h4 >> 1), m = mrow_ + mf * 16 + r16;
    const unsigned off = n0 + cw < nlim ? (unsigned)((m * ostride + ocol0 + cw) * 2) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b128(st, rsO, off, 0, 0);
  };
  auto epi_pair = [&](int mf, int nf, const f32x4& av0, const f32x4& av1, uint2 zv0, uint2 zv1, int mrow_,
                      uint2 dv0 = uint2{0u, 0u}, uint2 dv1 = uint2{0u, 0u}) {
    const v2u32_h o0 = __builtin_bit_cast(v2u32_h, epi_vals(mf, nf, av0, zv0, mrow_, dv0));
    const v2u32_h o1 = __builtin_bit_cast(v2u32_h, epi_vals(mf, nf + 1, av1, zv1, mrow_, dv1));
    epi_join(mf, nf, o0, o1, mrow_);
  };
  v2u32_h pend = {0u, 0u};   // WIDE, pipelined: the first unit of a pair, stored at the next tap
  // every unit of an accumulator set, in the store form of the launch
  auto epi_all = [&](const f32x4 (&av)[2][NF], const uint2 (&zv)[2][NF], int mrow_, const uint2 (&dv)[EPI == 4 ? 2 : 1][NF]) {
    if constexpr (WIDE) {
#pragma unroll
      for (int nf = 0; nf < NF; nf += 2)
#pragma unroll
        for (int mf = 0; mf < 2; ++mf)
          epi_pair(mf, nf, av[mf][nf], av[mf][nf + 1], zv[mf][nf], zv[mf][nf + 1], mrow_, dv[EPI == 4 ? mf : 0][nf],
                   dv[EPI == 4 ? mf : 0][nf + 1]);
    } else {
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
#pragma unroll
        for (int mf = 0; mf < 2; ++mf) epi_unit(mf, nf, av[mf][nf], zv[mf][nf], mrow_, dv[EPI == 4 ? mf : 0][nf]);
    }
  };

  f32x4 acc[2][NF], accp[2][NF];   // this tile's / the previous tile's accumulators (PIPE)
  uint2 zreg[2][NF], dreg[EPI == 4 ? 2 : 1][NF];
  int mrowp = 0;
  // one tile: prefetch the next tile's halo into registers, nine taps, then (PIPE) nothing -- the
  // previous tile's epilogue units run between this tile's taps -- or (!PIPE) this tile's epilogue.
  // tk = tile_id(k); returns tile_id(k + 1) (dyn: each is an LDS read of the claim ring with its own lgkmcnt
  // wait, so the ids are read once per tile and carried)
  auto load_halo = [&](int t, uint4 (&hr)[GH]) {   // registers <- the halo of patch t
    int img1, y01, x01;
    tile_origin(t, img1, y01, x01);
    const bool nohalo = (ADP_DBG(a) & 1024) != 0;   // timing-only ablation (fwd_debug bit 10): no halo loads
#pragma unroll
    for (int i = 0; i < GH; ++i) {
      const uint4* p = nohalo ? nullptr : halo_src(img1, y01, x01, i);
      hr[i] = p ? *p : make_uint4(0, 0, 0, 0);
    }
  };
  // hreg: the next tile's halo, loaded at the start of this tile and written to LDS at its end
  auto run_tile = [&](int k, int tk, auto with_prev, uint4 (&hreg)[GH]) -> int {
    constexpr bool EPI_PREV = decltype(with_prev)::value;
    if constexpr (!DYN) tk = tile_id(k);   // (static lists: arithmetic -- nothing carried across the taps)
    const int tn = tile_id(k + 1);
    const bool more = tn >= 0;
    // dyn: claim tile k + 2 now (a compiler-visible atomic in a file built without the atomic optimizer, whose
    // wave form would wait for the result at once: the wait lands before its use at the end of this tile)
    // (a claim is published at the end of this tile, inside `if (more)`: claim_now implies more)
    const bool claim_now = dyn && k % CH == 0 && more && sup_id(k / CH + 1) >= 0;
    int claimed = 0;
    if (claim_now && tid == 0) claimed = __hip_atomic_fetch_add(a.claim + nh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int img, y0, x0;
    tile_origin(tk, img, y0, x0);
    const int mrow = (img * a.Ho + y0 + wave) * a.Wo + x0;   // first output pixel of this wave's row
    if constexpr (BNR) load_z(EPI_PREV ? mrowp : mrow, zreg);
    if constexpr (EPI == 4) {
      if (has_mask) load_q(rsM, mstr, ocol0, mrow, zreg);
      if (has_add) load_q(rsD, a.addend_stride, ocol0, mrow, dreg);
    }
    if (more) load_halo(DYN ? tn : tile_id(k + 1), hreg);
    int img1 = 0, y01 = 0, x01 = 0;   // BNL: the next patch (uniform)
    if constexpr (BNL) {
      if (more) tile_origin(tn, img1, y01, x01);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (SWP) {
      constexpr int NS = 18 * NCH;   // K steps of a tile: (tap, input chunk, 32-deep half)
      bf16x8 FB[2][NF], FA[2][2];
      auto ldf = [&](auto sc, bf16x8 (&fb)[NF], bf16x8 (&fa)[2]) {
        constexpr int st = decltype(sc)::value, t = st / (2 * NCH), cc = (st >> 1) % NCH, kq = st & 1;
        constexpr int dy = t / 3, dx = t - 3 * dy;
        const unsigned char* Wt = smem + OFF_W + t * WTAP + cc * BN * ROWB;
        const unsigned char* Hc = smem + cc * HROWS * ROWB;
        const int ck = 4 * kq + h4;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const int q = nf * 16 + r16;
          fb[nf] = *reinterpret_cast<const bf16x8*>(Wt + q * ROWB + ((ck ^ swz(q)) << 4));
        }
#pragma unroll
        for (int mf = 0; mf < 2; ++mf) {
          const int hr = (wave + dy) * HW + mf * 16 + r16 + dx;
          fa[mf] = *reinterpret_cast<const bf16x8*>(Hc + hr * ROWB + ((ck ^ hswz(hr)) << 4));
        }
      };
      ldf(std::integral_constant<int, 0>{}, FB[0], FA[0]);
      halop_static_for<0, NS>([&](auto sc) {
        constexpr int st = decltype(sc)::value, t = st / (2 * NCH), cc = (st >> 1) % NCH, kq = st & 1;
        if constexpr (st + 1 < NS) ldf(std::integral_constant<int, st + 1>{}, FB[(st + 1) & 1], FA[(st + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);   // (the next step's reads stay ahead of this step's MFMAs)
        const bf16x8(&fb)[NF] = FB[st & 1];
        const bf16x8(&fa)[2] = FA[st & 1];
        constexpr bool with_unit = EPI_PREV && cc == 0 && kq == 0 && t >= 1 && t - 1 < 2 * NF;
        if constexpr (with_unit) {
          constexpr int u = t - 1;
          if constexpr (WIDE) {
            constexpr int p = u >> 1, mf = p & 1, nf = 2 * (p >> 1);
            if constexpr ((u & 1) == 0) {
              pend = __builtin_bit_cast(v2u32_h, epi_vals(mf, nf, accp[mf][nf], zreg[mf][nf], mrowp));
            } else {
              epi_join(mf, nf, pend, __builtin_bit_cast(v2u32_h, epi_vals(mf, nf + 1, accp[mf][nf + 1],
                                                                          zreg[mf][nf + 1], mrowp)), mrowp);
            }
          } else {
            epi_unit(u & 1, u >> 1, accp[u & 1][u >> 1], zreg[u & 1][u >> 1], mrowp);
          }
        }
        if constexpr (!with_unit) prio_hi<ADP_PRIO_FWD>();
#pragma unroll
        for (int mf = 0; mf < 2; ++mf)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf)
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nf], fa[mf], acc[mf][nf], 0, 0, 0);
        if constexpr (!with_unit) prio_lo<ADP_PRIO_FWD>();
        if constexpr (with_unit) {
#pragma unroll
          for (int i = 0; i < 2 * NF; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, HALOP_VALU_PER_MFMA, 0);
          }
        }
      });
    }
#pragma unroll
    for (int t = 0; t < (SWP ? 0 : 9); ++t) {
      const int dy = t / 3, dx = t - 3 * dy;
#pragma unroll
      for (int cc = 0; cc < NCH; ++cc) {
        const unsigned char* Wt = smem + OFF_W + t * WTAP + cc * BN * ROWB;
        const unsigned char* Hc = smem + cc * HROWS * ROWB;
#pragma unroll
        for (int kq = 0; kq < 2; ++kq) {
          const int ck = 4 * kq + h4;
          bf16x8 fb[NF], fa[2];
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) {
            const int q = nf * 16 + r16;
            fb[nf] = *reinterpret_cast<const bf16x8*>(Wt + q * ROWB + ((ck ^ swz(q)) << 4));
          }
#pragma unroll
          for (int mf = 0; mf < 2; ++mf) {
            const int hr = (wave + dy) * HW + mf * 16 + r16 + dx;
            fa[mf] = *reinterpret_cast<const bf16x8*>(Hc + hr * ROWB + ((ck ^ hswz(hr)) << 4));
          }
          // previous tile's epilogue unit u in tap u + 1 (the z loads had a tap's time to land), its VALU
          // spread between this step's MFMAs
          constexpr bool unit_here = EPI_PREV;
          const bool with_unit = unit_here && cc == 0 && kq == 0 && t >= 1 && t - 1 < 2 * NF;
          if (with_unit) {
            const int u = t - 1;
            if constexpr (WIDE) {
              // pair p = u >> 1 = units (p & 1, 2 (p >> 1)) and (p & 1, 2 (p >> 1) + 1), its two halves in
              // consecutive taps (the per-tap VALU of the narrow form): the first unit's quad is held in
              // registers, the second tap joins it with its own and stores 16 B
              const int p = u >> 1, mf = p & 1, nf = 2 * (p >> 1);
              if ((u & 1) == 0) {
                pend = __builtin_bit_cast(v2u32_h, epi_vals(mf, nf, accp[mf][nf], zreg[mf][nf], mrowp));
              } else {
                epi_join(mf, nf, pend, __builtin_bit_cast(v2u32_h, epi_vals(mf, nf + 1, accp[mf][nf + 1],
                                                                            zreg[mf][nf + 1], mrowp)), mrowp);
              }
            } else {
              const int mf = u & 1, nf = u >> 1;
              epi_unit(mf, nf, accp[mf][nf], zreg[mf][nf], mrowp);
            }
          }
          // BNL: chunk t - 3 of the next patch's halo through the BatchNorm-ReLU, its VALU between this step's MFMAs
          const bool with_apply = BNL && kq == 1 && t >= 3 && t - 3 < GH;
          if constexpr (BNL) {
            if (with_apply && more) hreg[t - 3] = bnl(hreg[t - 3], img1, y01, x01, t - 3);
          }
          if (!with_unit && !with_apply) prio_hi<ADP_PRIO_FWD>();   // (setprio would split the interleave region)
#pragma unroll
          for (int mf = 0; mf < 2; ++mf)
#pragma unroll
            for (int nf = 0; nf < NF; ++nf)   // transposed: rows = output channels, columns = pixels
              acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nf], fa[mf], acc[mf][nf], 0, 0, 0);
          if (!with_unit && !with_apply) prio_lo<ADP_PRIO_FWD>();
          if (with_unit || with_apply) {
#pragma unroll
            for (int i = 0; i < 2 * NF; ++i) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
              __builtin_amdgcn_sched_group_barrier(0x002, HALOP_VALU_PER_MFMA, 0);   // then VALU
            }
          }
        }
      }
    }
    if constexpr (PIPE) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) accp[i][j] = acc[i][j];
      mrowp = mrow;
    } else {
      epi_all(acc, zreg, mrow, dreg);
    }
    if (more) {
      LDS_BAR();   // every wave is done with this tile's halo
#pragma unroll
      for (int i = 0; i < GH; ++i)   // (BNL: applied in the K loop)
        if (i * NTH + tid < HCH) *reinterpret_cast<uint4*>(smem + (size_t)(i * NTH + tid) * 16) = hreg[i];
      if (claim_now && tid == 0) ring[(k / CH + 2) & 3] = claimed;   // (slot of super-tile s - 2: long done)
      LDS_BAR();
    }
    return DYN ? tn : tile_id(k + 1);
  };
  uint4 hA[GH];
  int tnext = run_tile(0, tile_id(0), std::false_type{}, hA);
  for (int k = 1; tnext >= 0; ++k) tnext = run_tile(k, tnext, std::integral_constant<bool, PIPE>{}, hA);
  if constexpr (PIPE) {   // the last tile's epilogue
    if constexpr (BNR) load_z(mrowp, zreg);
    epi_all(accp, zreg, mrowp, dreg);
  }
  if (dyn && tid == 0) claim_block_done(a.claim, NT, G);   // (every claim of the block has returned)
  if (!stats || (ADP_DBG(a) & 2)) return;   // (uniform)
  double* d0 = a.stat + (size_t)((blockIdx.x * 8 + wave) & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
#pragma unroll
  for (int nf = 0; nf < NF; ++nf)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = row16_sum(s1[nf][i]), y = row16_sum(s2[nf][i]);
      const int c = n0 + nf * 16 + 4 * h4 + i;
      if (r16 == 0 && c < a.Nout) {
        atomicAdd(d0 + c, (double)x);
        atomicAdd(d0 + adp::STAT_CMAX + c, (double)y);
      }
    }
}

#undef HALO_BAR
#undef LDS_BAR

template <int WN, int KS, int TPS, int NHB>
void launch_halo(FwdArgs& a, hipStream_t s) {
  constexpr int BN = WN * 64;
  a.ntile_n = (a.Nout + BN - 1) / BN;
  a.nblocks = a.Nimg * (a.Ho / PH) * (a.Wo / PW) * a.ntile_n;
  adp::set_kernel("igemm_fwd_halo_kernel<%d, %d, %d, %d, %s>", WN, KS, TPS, NHB, a.bnr_z ? "true" : "false");
  const dim3 g(a.nblocks), b(4 * WN * KS * 64);
  if (a.bnr_z) hipLaunchKernelGGL((igemm_fwd_halo_kernel<WN, KS, TPS, NHB, true>), g, b, 0, s, a);
  else hipLaunchKernelGGL((igemm_fwd_halo_kernel<WN, KS, TPS, NHB, false>), g, b, 0, s, a);
}

}  // namespace

namespace adp {
int launch_fwd_halo(FwdArgs& a, hipStream_t s) {
  const int mode = option("fwd_halo", 1);   // 0 off, 1 auto, 2 = no single-buffer form (A/B)
  if (mode == 0) return 0;
  const int Cin_s = a.CAs + a.CBs;
  // BN-on-load of source A (a.scA with a.act_out: EPI 6 of the persistent kernel) only where that form exists; every
  // other BN-on-load launch goes to the register-staged kernels (adp_conv_fwd materialises act_out first)
  const bool bnl = a.scA != nullptr;
  if (bnl && !(a.act_out && a.CBs == 0 && a.up == 1 && a.CAs == 64 && a.bn_sum && !a.bnr_z &&
               !a.relu && !a.bias && option("halop_bnl", 1)))
    return 0;
  // up = 2 (nearest upsample folded into the gather): the persistent forms only
  if (a.scB || a.kh != 3 || a.kw != 3 || a.dil != 1 || a.pad != 1 || a.stride != 1 || (a.up != 1 && a.up != 2) ||
      a.Ho != a.Hs * a.up || a.Wo != a.Ws * a.up || a.Ho % PH != 0 || a.Wo % PW != 0 || a.CAs % 64 != 0 || a.CBs % 64 != 0 ||
      a.K != 9 * Cin_s || a.Kpad != a.K || a.Nout > 128)
    return 0;
  if (a.bnr_z && (a.out_mode != 0 || a.bias || a.relu || a.drop_rate > 0.f || a.accum || a.bn_sum)) return 0;
  const bool one_chunk = Cin_s == 64;
  const bool plain = !a.addend && !a.mask && !a.mask2 && !a.accum && a.drop_rate == 0.f && a.out_stride % 8 == 0;
  // EPI 5 (option halop_dropout): ReLU + dropout on a plain store (adipose_v3 up*_conv3 in training)
  const bool dropepi = a.drop_rate > 0.f && a.relu && !a.addend && !a.mask && !a.mask2 && !a.accum && !a.bn_sum &&
                       !a.bnr_z && a.out_mode == 0 && a.out_stride % 8 == 0 && option("halop_dropout", 1);
  // EPI 4 (option halop_mask): an addend and / or ReLU-backward masks, no bias / ReLU / statistics (the
  // adipose_v3 data gradients); operands read as 8-B quads
  const bool maskepi = (a.addend || a.mask || a.mask2) && !a.accum && a.drop_rate == 0.f && !a.bnr_z && !a.bn_sum && !a.relu && !a.bias &&
                       a.out_stride % 8 == 0 && (!a.mask || a.mask_stride % 4 == 0) &&
                       (!a.mask2 || a.mask2_stride % 4 == 0) && (!a.addend || a.addend_stride % 4 == 0) &&
                       (size_t)a.M * std::max(std::max(a.mask ? a.mask_stride : 0, a.mask2 ? a.mask2_stride : 0),
                                              a.addend ? a.addend_stride : 0) * 2 < ((size_t)1 << 31) &&
                       option("halop_mask", 1);
  // persistent forms: one chunk with <= 64 outputs (one block) or 128 (two 64-wide blocks); two chunks
  // with 64 / 128 outputs in 32-wide blocks
  int bn = 0;
  if (one_chunk && (a.Nout <= 64 || a.Nout == 128)) bn = 64;
  else if (Cin_s == 128 && (a.Nout == 64 || a.Nout == 128) && option("halo_persist2", 1)) bn = 32;
  const int nt_n = bn ? (a.Nout + bn - 1) / bn : 1;
  const bool split_ok = a.out_mode == 2 && bn && a.split_c > 0 && a.split_c % bn == 0 && a.split_c < a.Nout &&
                        (!a.mask2 || maskepi) && a.out2_stride % 8 == 0 && (a.Nout - a.split_c) % bn == 0;
  const size_t lim = (size_t)1 << 31;   // the persistent form stores / reads z through buffer resources
  const bool fits = (size_t)a.M * a.out_stride * 2 < lim && (!a.out2 || (size_t)a.M * a.out2_stride * 2 < lim) &&
                    (!a.bnr_z || (size_t)a.M * a.bnr_zs * 2 < lim);
  if (bn && (plain || maskepi || dropepi) && fits && (a.out_mode == 0 || split_ok) && option("halo_persist", 1) &&
      (a.up == 1 || !a.bnr_z)) {
    const int tiles = a.Nimg * (a.Ho / PH) * (a.Wo / PW) * nt_n;
    a.ntile_n = nt_n;
    a.nblocks = tiles;   // the persistent kernel reads the tile count from nblocks
    int grid = std::max(1, std::min(tiles, option("halo_persist_grid", 256)));
    grid -= grid % nt_n;   // a block keeps one output block
    if (grid == 0) grid = nt_n;
    const bool bnr = a.bnr_z != nullptr;
    // PIPE (option halop_pipe): the epilogue of tile k runs between the MFMAs of tile k+1 (not for the
    // BN-backward reduction launches: their z quads and sums do not fit the registers next to two
    // accumulator sets)
    // (one-chunk launches only by default: +8 % on the 64 -> 64 forward; the two-chunk form has twice the
    // MFMA work per epilogue and lost 2-5 % to the extra registers -- profiles/r02_halop_pipe_ab.txt)
    const int pm = option("halop_pipe", 1);
    // SWP (option halop_swp: 0 off, 1 every non-BNR form, 2 the two-chunk ones -- default) replaces the pipelined
    // epilogue (with both the forms spill). Measured (profiles/r05i_swp_ab.log): two-chunk forward +4-6 % (L0 128->64,
    // L1 128->128), the one-chunk forward 1 % behind its pipelined epilogue, L1 256->128 (tap64p) untouched
    const int swm = option("halop_swp", 2);
    const bool swp_req = !bnr && !dropepi && (swm == 1 || (swm == 2 && !one_chunk));   // (the dropout form spills)
    const bool pipe = !swp_req && !bnr && !maskepi && !dropepi && (pm == 2 || (pm == 1 && one_chunk));
    const int epi = bnr ? 0 : dropepi ? 5 : maskepi ? 4 : (a.bn_sum ? 1 : 0) + (a.relu ? 2 : 0);
    // WIDE (option halop_wide: 0 off, 1 the tile-serial forms, 2 every form, 3 every form but the pipelined
    // ones with statistics): 16-B stores of channel-quad pairs when every 8-channel run of the store is wholly
    // inside or outside its limit. Not the BN-backward reduction forms (two units' z quads and constants at
    // once spill). Measured (profiles/r03_halop_wide_ab.txt): two-chunk forward with statistics +4 %, one-chunk
    // pipelined forward +6 %, one-chunk pipelined forward with statistics -2..-5 % (kept narrow)
    const int wm = option("halop_wide", 3);
    const bool wide = !bnr && (wm == 2 || (wm == 1 && !pipe) || (wm == 3 && !(pipe && (epi == 1 || epi == 3)))) &&
                      a.Nout % 8 == 0 && (a.out_mode != 2 || a.split_c % 8 == 0);
    // dynamic tile claiming (option halop_claim; nullptr from claim_slot: static lists). Not the one-chunk
    // BN-backward-reduction form nor the pipelined forms with statistics: their claimed forms spill (the
    // latter run in the forward pass only, where no all-reduce holds CUs)
    a.claim = option("halop_claim", option("dp_claim", 0)) && nt_n + 1 <= CLAIM_INTS && !(bnr && one_chunk) && !(pipe && (epi == 1 || epi == 3))
                  ? claim_slot() : nullptr;
    a.claim_chunk = std::max(1, option("halop_claim_chunk", 4));   // patches per claim
    a.claim_full = 0;
    if (a.claim) {   // (no more blocks per output block than super-tiles)
      const int nsup = (tiles / nt_n + a.claim_chunk - 1) / a.claim_chunk;
      grid = std::max(nt_n, std::min(grid, nsup * nt_n));
      // claim_full only with at least 4 super-tiles per block (its first claim takes two at once)
      a.claim_full = option("claim_full", 0) && nsup >= 4 * (grid / nt_n);
    }
    if (bnl) a.claim = nullptr;   // (static lists only)
    const bool dyn = a.claim != nullptr;
    // SWP (option halop_swp, static lists only): the software-pipelined K loop of the kernel comment
    const bool swp = !dyn && swp_req;
    if (bnl) {   // the two forms of the unet_bn convs after a BatchNorm-ReLU: levels 0 and 1
      if (one_chunk && a.Nout <= 64 && pipe && !wide && !swp && epi == 1) {
        adp::set_kernel("igemm_fwd_halop_kernel<false, 1, 64, true, 6, false, false, false>");
        hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, 1, 64, true, 6, false, false, false>), dim3(grid), dim3(512), 0,
                           s, a);
        return 1;
      }
      // (the two-chunk forms: 4 output blocks apply each halo again, and with the software-pipelined K loop the
      //  apply spills 37 VGPRs; without it, applied at the tile's end, L1's conv2 ran 44 % longer -- 143 us against
      //  the 89 us of the apply pass it saves: profiles/r05u_*. Such launches take the two-launch form.)
      return 0;
    }
    adp::set_kernel("igemm_fwd_halop_kernel<%s, %d, %d, %s, %d, %s, %s, %s>", bnr ? "true" : "false", one_chunk ? 1 : 2, bn,
                    pipe ? "true" : "false", epi, wide ? "true" : "false", dyn ? "true" : "false", swp ? "true" : "false");
#define HALOP_LAUNCH_WD(NCH_, BN_, W_, D_, P_)                                                                   \
  do {                                                                                                      \
    if (bnr) hipLaunchKernelGGL((igemm_fwd_halop_kernel<true, NCH_, BN_, false, 0, false, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
    else if (epi == 4) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 4, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
    else if (epi == 5) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 5, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
    else if (pipe) {                                                                                        \
      if (epi == 1) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, true, 1, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
      else if (epi == 2) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, true, 2, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
      else if (epi == 3) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, true, 3, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
      else hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, true, 0, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
    } else {                                                                                                \
      if (epi == 1) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 1, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
      else if (epi == 2) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 2, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
      else if (epi == 3) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 3, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
      else hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 0, W_, D_, P_>), dim3(grid), dim3(512), 0, s, a); \
    }                                                                                                       \
  } while (0)
#define HALOP_LAUNCH_SWP(NCH_, BN_, W_)                                                                         \
  do {                                                                                                      \
    if (epi == 4) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 4, W_, false, true>), dim3(grid), dim3(512), 0, s, a); \
    else if (epi == 1) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 1, W_, false, true>), dim3(grid), dim3(512), 0, s, a); \
    else if (epi == 2) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 2, W_, false, true>), dim3(grid), dim3(512), 0, s, a); \
    else if (epi == 3) hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 3, W_, false, true>), dim3(grid), dim3(512), 0, s, a); \
    else hipLaunchKernelGGL((igemm_fwd_halop_kernel<false, NCH_, BN_, false, 0, W_, false, true>), dim3(grid), dim3(512), 0, s, a); \
  } while (0)
#define HALOP_LAUNCH_W(NCH_, BN_, W_)                          \
  do {                                                         \
    if (dyn) HALOP_LAUNCH_WD(NCH_, BN_, W_, true, false);      \
    else if (swp) HALOP_LAUNCH_SWP(NCH_, BN_, W_);              \
    else HALOP_LAUNCH_WD(NCH_, BN_, W_, false, false);         \
  } while (0)
#define HALOP_LAUNCH(NCH_, BN_)                  \
  do {                                           \
    if (wide) HALOP_LAUNCH_W(NCH_, BN_, true);   \
    else HALOP_LAUNCH_W(NCH_, BN_, false);       \
  } while (0)
    if (one_chunk) HALOP_LAUNCH(1, 64);
    else HALOP_LAUNCH(2, 32);
#undef HALOP_LAUNCH_W
#undef HALOP_LAUNCH_WD
#undef HALOP_LAUNCH_SWP
#undef HALOP_LAUNCH
    return 1;
  }
  // 128 outputs from more than two input chunks (unet_bn dec1_conv1, 256 -> 128): the 256x128 halo form of
  // the persistent tap64 kernel takes plain launches (917 vs 852 TF with statistics,
  // profiles/r02_tap64p_halo_ab.txt)
  if (bnl) return 0;
  if (a.Nout == 128 && Cin_s > 128 && !a.bnr_z && plain && a.out_mode != 1 && option("halo_defer_tap64p", 1))
    return 0;
  if (a.up != 1) return 0;   // (the non-persistent halo kernels gather at the source resolution)
  if (a.Nout <= 64) {
    if (one_chunk && mode != 2) launch_halo<1, 2, 1, 1>(a, s);   // two blocks per CU
    else launch_halo<1, 2, 2, 2>(a, s);
  } else {
    if (one_chunk && mode != 2) launch_halo<2, 1, 1, 1>(a, s);
    else launch_halo<2, 1, 1, 2>(a, s);
  }
  return 1;
}
}  // namespace adp
