// Persistent form of the tap64 forward-shaped kernel (conv_fwd_tap64.hip) for the 256x256 tile: one
// 512-thread block per CU walks output tiles lin, lin + G, ... (G = grid, a multiple of the N-tile count,
// so a block keeps one N tile), and the tile boundary is pipelined:
//   * the first K step of tile k+1 is issued by LDS-DMA at the LAST K step of tile k (its stage is free),
//   * the epilogue of tile k runs from registers -- the product is accumulated transposed (C^T = W X^T:
//     a lane holds 4 consecutive output channels of one pixel) and stored as 8-B buffer stores, no LDS
//     staging, no barrier -- while those loads land,
//   * the next K loop waits only for the loads: every thread issues exactly EPI_OPS vector-memory
//     instructions in an epilogue (out-of-range lanes store to an out-of-range buffer offset, which the
//     hardware drops), so `s_waitcnt vmcnt(EPI_OPS)` retires everything older than the epilogue.
// Per block, the non-persistent kernel paid the prologue load latency and an LDS-staged epilogue
// (accumulators -> LDS -> 16-B stores, two row groups, four barriers) with the MFMA pipe idle: 5-17 % of
// a 3x3 layer at K = 9216..2304 and 40-75 % of a ConvTranspose forward (K = 128..1024).
// Epilogue forms: plain / pixel-shuffle (ConvTranspose) / channel-split store, bias, ReLU, BatchNorm
// statistics of the stored values (bn_sum), fused BatchNorm-backward reduction (BNR); every other epilogue
// term (addend, mask, accumulate, dropout, fp8) stays on the non-persistent kernel.
#include "conv_common.h"

namespace {

constexpr unsigned P_OOB = 0x80000000u;   // buffer offset beyond every resource: loads read 0, stores drop
constexpr int P_RSRC3 = 0x00020000;       // raw buffer descriptor word 3 (gfx9: 32-bit data format)
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef int v8i32 __attribute__((ext_vector_type(8)));
typedef unsigned int v4u32_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void p_lds16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
}
__device__ __forceinline__ void p_st8(__amdgpu_buffer_rsrc_t r, unsigned off, v2u32 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 0);
}
__device__ __forceinline__ v2u32 p_ld8(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
}

// epilogue constant read (ds_read_b128 + its own lgkmcnt wait) as inline asm: the compiler's form of an
// LDS read after the LDS-DMA prefetch of the next stages gets a vmcnt(0) in front -- it cannot tell the
// constants from the stages being written -- which drained the whole prefetch at every tile's epilogue
__device__ __forceinline__ float4 p_lds_f4(const float* p) {
  float4 r;
  const unsigned addr = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
  return r;
}

// the block's BatchNorm sums: LDS f64 add as inline asm for the same reason (no lgkmcnt wait: nothing
// reads sacc before the final barrier, which is preceded by an explicit lgkmcnt(0)). f64: the waves of one
// channel set add their per-tile f32 partials in a run-dependent order, which f64 sums absorb (common.h)
__device__ __forceinline__ void p_lds_add(double* p, float v) {
  const unsigned addr = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)p;
  const double d = (double)v;
  asm volatile("ds_add_f64 %0, %1" ::"v"(addr), "v"(d) : "memory");
}
#define P_BAR()                            \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_s_barrier();          \
    asm volatile("" ::: "memory");         \
  } while (0)

// BM x BN tile, NST-stage LDS ring. 8 waves: WN = BN / 64 along N, WM = 8 / WN along M, a wave owns TM
// pixels x 64 channels. The K steps of ALL the block's tiles form one stream: the loader runs NST - 1 steps
// ahead of the multiply, across tile boundaries, so with NST = 3 two stages are in flight while a third
// multiplies (the small-K ConvTranspose / N = 128 shapes, whose tiles are only 2..18 steps long).
// HALO (3x3 stride-1 'same' layers, 8 x 32 output patches, BM = BN = 256, NST = 2): the A operand is not
// gathered per tap but read from the 10 x 34 input halo of the patch, moved into LDS once per 64-channel
// chunk (a two-slot ring beside the weight stages). The K stream of a tile is chunk-major (chunk c: taps
// 0..8 over the same halo), each step stages only the weight rows of its (tap, chunk), and the halo of the
// NEXT chunk of the stream -- the next tile's first chunk at a tile's last one -- goes out one 16-B group
// per step at the steps of taps 1..6 (its slot was freed by the previous chunk's last step). LDS-DMA
// pieces per thread per step: 4 weight + <= 1 halo, against 4 + 4 gathered A pieces (their issue is what
// the K loop waits on: profiles/r02_stagger_ab.txt).
constexpr int P_HROWS = 340;   // 10 x 34 halo pixels of an 8 x 32 patch
template <int BM, int BN, int NST, bool BNR, bool HALO = false>
constexpr int tap64p_lds() {
  // (+16 B: the ring of claimed tile ids, dynamic claiming)
  // (constants: 5 f32 rows; the block's BatchNorm sums: 2 f64 rows)
  return (HALO ? NST * BN * 128 + 2 * P_HROWS * 128 + 9 * BN * 4 : NST * (BM + BN) * 128 + 9 * BN * 4) + 16;
}
__device__ __forceinline__ int p_hswz(int r) { return r & 7; }   // (conv_fwd_halo.hip: conflict-free)

// F8 (halo form, fp8 e4m3 operands, BASELINE configs[4]): the same byte schedule with 128-channel K steps
// (a 128-B row is 128 fp8 channels); the two 16-B fragments a lane reads per row are one 32-B operand of
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales; A and B share the permutation of K), and the
// epilogue multiplies by the per-column weight scale; bf16 output, plain store, no BatchNorm sums.
// WREG (halo form, 2 stages, bf16): the weight rows of a K step are not moved by LDS-DMA but loaded into
// registers one step ahead (4 x 16-B buffer loads per thread) and written into the free stage with ds_write
// when the step is issued: the LDS-DMA issue (60-185 cycles per 1-KiB wave piece, what the K loop waited on:
// profiles/r02_tap64p_halo_ablation.txt) is left to the <= 1 halo group per step.
// F32 (halo form, 256x128 / 3 stages; the f32 path of adipose_v3, every drop-in CLI's default dtype): the same
// byte schedule with 32-channel K steps (a 128-B row is 32 f32 channels). The two 16-B fragments a lane reads per
// row are 8 f32 of k = 16 s + 4 h4 + e (s = 0, 1; e = 0..3): eight exact v_mfma_f32_16x16x4_f32 per 16x16 block,
// the e-th of half s taking element e -- lane group h4 then supplies k = 16 s + 4 h4 + e to it, and A and B share
// that permutation, so every k of the step enters the dot product once. f32 epilogue: 16-B stores of a lane's
// channel quad.
// EPIC (bf16 forms): -1 = the epilogue chosen at run time from a.wide_st (narrow / pair-major 16-B / line-ordered
// 16-B); 2 = only the line-ordered one compiled in -- the launcher's default store form, without the register
// allocation of two epilogues it never runs (measured on the fp8 forms, whose ConvTranspose launch went from 0.215 to
// 0.120 ms when the unused 16-B bf16 epilogues left it); 3 = the same with static tile lists only (no claiming code:
// the launches without a claim counter, i.e. every default launch; option tap64p_epic3); 4 = 3 with plain stores only
// (out_mode 0: no pixel-shuffle or split store paths; option tap64p_epic4)
template <int BM, int BN, int NST, bool BNR, bool HALO = false, bool F8 = false, bool WREG = false, bool F32 = false,
          int EPIC = -1>
__global__ __launch_bounds__(512, 1) void igemm_fwd_tap64p_kernel(FwdArgs a) {
  static_assert(EPIC < 0 || ((EPIC == 2 || EPIC == 3 || EPIC == 4) && !BNR && !F8 && !F32),
                "compile-time epilogue: the bf16 line-ordered form");
  static_assert(!F8 || !BNR, "fp8: no BN-backward reduction");
  static_assert(!WREG || (HALO && NST == 2 && !F8), "register-staged weights: the bf16 2-stage halo form");
  static_assert(!F32 || (HALO && !BNR && !F8 && !WREG), "f32: the halo form");
  constexpr int NTH = 512, ROWB = 128, ES = F8 ? 1 : (F32 ? 4 : 2), KSTEP = F8 ? 128 : (F32 ? 32 : 64);
  constexpr int OES = F32 ? 4 : 2;   // output / z element bytes (bf16; f32)
  constexpr int WN = BN / 64, WM = 8 / WN, TM = BM / WM;
  static_assert(WN * WM == 8 && TM % 32 == 0 && TM >= 64, "wave layout");
  static_assert(!HALO || (!BNR && BM == 256 && ((BN == 256 && NST == 2) || (BN == 128 && NST == 3))),
                "halo form: 256x256 / 2 stages or 256x128 / 3 stages, no BN-backward reduction");
  constexpr int QA = BM / 2, QB = BN / 2, GA = QA * 8 / NTH, GB = QB * 8 / NTH;
  static_assert(GA >= 1 && GB >= 1, "staging split");
  constexpr int HM = TM / 2, MIQ = TM / 32;
  constexpr int STAGE = (HALO ? BN : BM + BN) * ROWB;
  constexpr int OA1 = QA * ROWB, OB0 = HALO ? 0 : BM * ROWB, OB1 = (HALO ? QB : BM + QB) * ROWB;
  constexpr int HBUF = P_HROWS * ROWB, OH = NST * STAGE;   // halo slots (HALO)
  constexpr int GH = (P_HROWS * 8 + NTH - 1) / NTH;        // halo groups per chunk (the last one partial)
  // HALO: group g of the next chunk's halo rides on the loader step of tap g + NST - 1 (the compute is then
  // past the barrier of the chunk's first step, so the slot's previous chunk is no longer read)
  static_assert(!HALO || GH + NST - 1 <= 9, "halo groups ride on taps NST-1 .. 8");
  constexpr int LOPS = HALO ? 2 * GB : 2 * GA + 2 * GB;   // LDS-DMA pieces per thread per stage (HALO: + halo)
  constexpr bool ZALL = BNR && MIQ == 2;                     // (see load_zall)
  constexpr int EPI_OPS = 2 * MIQ * 4 * (BNR && !ZALL ? 2 : 1);   // vector-memory ops per thread per epilogue
  constexpr int EPI_OPS_W = 2 * MIQ * 2;                          // ... with 16-B stores (wide_st)
  constexpr int EPI_OPS_Q = 2 * MIQ;                              // ... fp8 output, 16-B line stores (wide_st 3)
  // (vmcnt holds 0..63: a larger count is clamped, which only waits for more)
  constexpr int VM_EPI = (NST - 2) * LOPS + EPI_OPS < 63 ? (NST - 2) * LOPS + EPI_OPS : 63;
  constexpr int VM_EPI_W = (NST - 2) * LOPS + EPI_OPS_W < 63 ? (NST - 2) * LOPS + EPI_OPS_W : 63;
  constexpr int VM_EPI_Q = (NST - 2) * LOPS + EPI_OPS_Q < 63 ? (NST - 2) * LOPS + EPI_OPS_Q : 63;
  constexpr int VM_Z = (NST - 2) * LOPS + 4 * 2 * MIQ < 63 ? (NST - 2) * LOPS + 4 * 2 * MIQ : 63;
  // ONE LDS object: with several, the compiler tags every LDS access with per-object alias scopes, and the
  // waitcnt pass then drains vmcnt(0) between the LDS-DMA prefetch of stage t+1 and the fragment reads of
  // stage t (one object: no such wait -- measured 12 % of the K loop)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[tap64p_lds<BM, BN, NST, BNR, HALO>()];
  constexpr int OC = NST * STAGE + (HALO ? 2 * HBUF : 0);
  float (*cst)[BN] = reinterpret_cast<float (*)[BN]>(smem + OC);   // epilogue constants:
                                                                  // bias | scale shift mean invstd (BNR)
  double (*sacc)[BN] = reinterpret_cast<double (*)[BN]>(smem + OC + 5 * BN * 4);   // block's BN sums (f64)
  int* ring = reinterpret_cast<int*>(smem + OC + 9 * BN * 4);   // dynamic claiming: tile ids of local tiles k & 3

  // f32 (WN = 2): waves w and w + 4 share a SIMD and take the two column halves of the tile (wc = w >> 2), and a
  // wave skips the MFMAs of a 32-column group that lies wholly past Nout (the 96- and 192-channel levels of
  // adipose_v3's f32 path leave a quarter of a 128-wide tile column empty): the SIMD of such a pair then runs
  // 3/4 of the MFMAs instead of idling through zero columns (option f32_skip)
  const bool SPLIT = F32 && WN == 2 && a.f32_skip;   // (f32_skip = 0: the bf16 forms' wave layout)
  auto w_row = [&](int w) { return SPLIT ? (w & 3) : w / WN; };
  auto w_col = [&](int w) { return SPLIT ? (w >> 2) : w % WN; };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = w_row(wave), wc = w_col(wave);
  const int G = gridDim.x;
  prio_static<ADP_PRIO_FWD>(wave);
  const int lin = xcd_remap(blockIdx.x, G);
  const int ntiles = a.nblocks;
  // tiles: static lists (lin, lin + G, ...: `mine` of them) or claimed one tile ahead from the counter of the
  // block's N column (dyn, conv_common.h); either way a block keeps one N column
  // (the fp8 eval forms and the opt-in register-staged form keep static lists: no spare registers there)
  const bool dyn = EPIC < 3 && !F8 && !WREG && a.claim != nullptr;
  const bool full = dyn && a.claim_full;   // every tile claimed (tiles 0 and 1 by one claim at the start)
  int r2 = 0;
  if (full && tid == 0) r2 = claim_next2(a.claim + lin % a.ntile_n);   // (its wait lands at the cst stores)
  const int ntn = a.ntile_n, ntm = ntiles / ntn, col = lin % ntn;
  const int mine = dyn ? 0 : (lin < ntiles ? (ntiles - lin + G - 1) / G : 0);
  if (!dyn && mine == 0) return;   // uniform per block
  const int n0 = col * BN;
  const int wcu = w_col(__builtin_amdgcn_readfirstlane(wave));
  const bool skip0 = SPLIT && n0 + wcu * 64 >= a.Nout;        // (block- and wave-uniform)
  const bool skip1 = SPLIT && n0 + wcu * 64 + 32 >= a.Nout;
  const int pos = lane & 7;
  const int HWo = a.Ho * a.Wo, Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  const int Cin_s = a.CAs + a.CBs;
  const int Wrows = (a.Nout + 63) / 64 * 64;
  const int nk = a.K / KSTEP;
  if (tid < BN) {   // (read in the epilogue through LDS: no vector-memory wait there)
    const int n = n0 + tid;
    const bool v = n < a.Nout;
    cst[0][tid] = (!BNR && a.bias && v) ? a.bias[a.out_mode == 1 ? n % a.Cps : n] : 0.f;
    cst[1][tid] = (BNR && v) ? a.bnr_sc[n] : (F8 && v) ? a.wscale[n] : 0.f;
    cst[2][tid] = (BNR && v) ? a.bnr_sh[n] : 0.f;
    cst[3][tid] = (BNR && v) ? a.bnr_mean[n] : 0.f;
    cst[4][tid] = (BNR && v) ? a.bnr_invstd[n] : 0.f;
    sacc[0][tid] = 0.0;
    sacc[1][tid] = 0.0;
  }
  // (ordered before the epilogue by the first K step's barrier)
  // dyn: a block's first tile is its static one (lin / ntn: no claim to wait for at the start); claim value c is
  // tile G / ntn + c

  const int npix = a.Nimg * a.Hs * a.Ws;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.srcA, 0, npix * a.CAs * ES, P_RSRC3);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.CBs ? a.srcB : a.srcA), 0, npix * (a.CBs ? a.CBs : a.CAs) * ES, P_RSRC3);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, Wrows * a.Kpad * ES, P_RSRC3);

  // ---- B staging (weights): fixed for the block's N tile
  unsigned bo[2][GB];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int q = i * (NTH / 8) + (tid >> 3);
      const int col = (q / 32) * 64 + h * 32 + (q % 32);
      bo[h][i] = n0 + col < Wrows ? (unsigned)((n0 + col) * a.Kpad * ES + 16 * (pos ^ swz(q))) : P_OOB;
    }
  // ---- A staging rows of the tile being LOADED: quarter h, instruction i -> quarter row q
  int ry[2][GA], rx[2][GA], pb[2][GA];   // (up == 1 only: an invalid row has ry far out of range)
  const int rc = 16 * (pos ^ ((tid >> 4) & 7));   // = 16 * (pos ^ swz(q)) for every staging row q of this thread
  auto setup_rows = [&](int m0) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int q = i * (NTH / 8) + (tid >> 3);
        const int m = m0 + (q / HM) * TM + h * HM + (q % HM);
        const bool v = m < a.M;
        const int mm = v ? m : 0;
        const int n = mm / HWo, rem = mm - n * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
        ry[h][i] = v ? yo * a.stride - a.pad : -(1 << 20);
        rx[h][i] = xo * a.stride - a.pad;
        pb[h][i] = (n * a.Hs + yo * a.stride - a.pad) * a.Ws + rx[h][i];
      }
  };
  // ---- K-step iterator of the tile being loaded (channel-chunk fastest inside a tap)
  struct Kt { int oy, ox, cs, cb, srcb, dpix, kt; };
  int it_ci = 0, it_ty = 0, it_tx = 0, it_kt = 0;
  auto kinfo = [&]() {
    Kt r;
    r.oy = it_ty * a.dil; r.ox = it_tx * a.dil; r.kt = it_kt;
    r.dpix = r.oy * a.Ws + r.ox;
    if (it_ci < a.CAs) { r.cb = it_ci * ES; r.cs = a.CAs * ES; r.srcb = 0; }
    else { r.cb = (it_ci - a.CAs) * ES; r.cs = a.CBs * ES; r.srcb = 1; }
    ++it_kt;
    it_ci += KSTEP;
    if (it_ci >= Cin_s) {
      it_ci = 0;
      if (++it_tx == a.kw) { it_tx = 0; ++it_ty; }
    }
    return r;
  };
  const bool l2_only = (ADP_DBG(a) & 256) != 0;   // (fwd_debug bit 8)
  auto issue = [&](const Kt& k, int buf) {
    // A0 B0 B1 A1
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      unsigned char* dst = smem + buf * STAGE + h * OA1 + wave * 8 * ROWB;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int yi = ry[h][i] + k.oy, xi = rx[h][i] + k.ox;
        const bool v = (unsigned)yi < (unsigned)Hv && (unsigned)xi < (unsigned)Wv;
        unsigned off = v ? (unsigned)((pb[h][i] + k.dpix) * k.cs + k.cb + rc) : P_OOB;
        if (l2_only && v) off &= 0x3FFF0u;   // timing-only ablation: the A gather from a 256-KiB window
        p_lds16(k.srcb ? rsB : rsA, dst + i * (NTH / 8) * ROWB, off);
      }
      unsigned char* dsb = smem + buf * STAGE + (h ? OB1 : OB0) + wave * 8 * ROWB;
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const unsigned off = bo[h][i] == P_OOB ? P_OOB : bo[h][i] + (unsigned)k.kt * ROWB;
        p_lds16(rsW, dsb + i * (NTH / 8) * ROWB, off);
      }
    }
  };
  // the loader: the next K step of the block's stream (tile lk, step lt) into stage ls
  int lk = 0, lt = 0, ls = 0;
  // HALO: tile -> 8 x 32 patch (image, y0, x0); its first output pixel is the tile's "m0" and pixel p of the
  // tile (p = 32 * patch row + column) is output pixel m0 + (p >> 5) * Wo + (p & 31)
  const int ptx = HALO ? a.Wo / 32 : 1, pty = HALO ? a.Ho / 8 : 1;
  struct PatchO { int img, y0, x0; };
  // tile id (M-tile / patch index) of the block's local tile k, -1 past the end of its work. dyn: the ring slot
  // was written at the top of the compute step whose stage is the loader's first step of tile k - 1, before
  // that step's barrier -- ahead of every reader (the loader needs tile k from step NST - 1 of tile k - 1 on)
  auto tile_id = [&](int k) -> int {
    if (!dyn) return k < mine ? lin / ntn + k * (G / ntn) : -1;
    if (k == 0 && !full) return lin / ntn;
    const int t = (full ? 0 : G / ntn) + claim_ring_read(ring + (k & 3));   // (uniform: scalar registers)
    return t < ntm ? t : -1;   // (a claim past the last tile: the work is taken)
  };
  auto patch_t = [&](int t) {
    PatchO P;
    P.x0 = (t % ptx) * 32;
    const int r = t / ptx;
    P.y0 = (r % pty) * 8;
    P.img = r / pty;
    return P;
  };
  auto m0_of = [&](int t) {   // first output pixel of tile t
    if constexpr (HALO) {
      const PatchO P = patch_t(t);
      return (P.img * a.Ho + P.y0) * a.Wo + P.x0;
    }
    return t * BM;
  };
  auto pix = [&](int m0, int p) { return HALO ? m0 + (p >> 5) * a.Wo + (p & 31) : m0 + p; };
  const bool no_dma = (ADP_DBG(a) & 32) != 0;   // timing-only ablation (fwd_debug bit 5): the K loop
                                                    // multiplies whatever the prologue loaded
  int nissued = 0;
  // HALO: one 16-B group g of the halo of chunk c of tile k into slot `slot`; returns whether this wave
  // issued an instruction (the last group covers 160 of 512 threads: waves 3-7 skip it)
  const int nch = Cin_s / KSTEP;
  auto issue_halo = [&](int t, int c, int g, int slot) {
    const int idx = g * NTH + tid;
    if (g == GH - 1 && __builtin_amdgcn_readfirstlane(g * NTH + wave * 64) >= P_HROWS * 8) return false;
    if (idx < P_HROWS * 8) {
      const PatchO P = patch_t(t);
      const int hr = idx >> 3, hp = idx & 7;
      // (yi, xi) in the conv's input grid, which is the source upsampled x up (nearest: source pixel
      // (yi >> 1, xi >> 1) for up = 2, the UpSampling2D of train_adipose_unet_v3.py:691 folded in)
      const int yi = P.y0 - 1 + hr / 34, xi = P.x0 - 1 + hr % 34;
      const int ci = c * KSTEP;
      const bool srcb = ci >= a.CAs;
      const int cs = (srcb ? a.CBs : a.CAs) * ES, cb = (srcb ? ci - a.CAs : ci) * ES;
      // (bounds on the source coordinates: an arithmetic shift keeps -1 negative)
      const int sy = yi >> (a.up >> 1), sx = xi >> (a.up >> 1);
      const bool v = (unsigned)sy < (unsigned)a.Hs && (unsigned)sx < (unsigned)a.Ws;
      const unsigned off = v ? (unsigned)(((P.img * a.Hs + sy) * a.Ws + sx) * cs + cb + 16 * (hp ^ p_hswz(hr))) : P_OOB;
      p_lds16(srcb ? rsB : rsA, smem + OH + slot * HBUF + (size_t)(g * NTH + wave * 64) * 16, off);
    }
    return true;
  };
  // WREG: the halo group g of chunk c of tile k through a register (ok = false: an out-of-range load, 0)
  auto load_halo_reg = [&](int t, int c, int g, bool ok) -> v4u32_t {
    const int idx = g * NTH + tid;
    const PatchO P = patch_t(t);
    const int hr = idx >> 3, hp = idx & 7;
    const int yi = P.y0 - 1 + hr / 34, xi = P.x0 - 1 + hr % 34;
    const int ci = c * KSTEP;
    const bool srcb = ci >= a.CAs;
    const int cs = (srcb ? a.CBs : a.CAs) * ES, cb = (srcb ? ci - a.CAs : ci) * ES;
    const int sy = yi >> (a.up >> 1), sx = xi >> (a.up >> 1);
    const bool v = ok && idx < P_HROWS * 8 && (unsigned)sy < (unsigned)a.Hs && (unsigned)sx < (unsigned)a.Ws;
    const unsigned off = v ? (unsigned)(((P.img * a.Hs + sy) * a.Ws + sx) * cs + cb + 16 * (hp ^ p_hswz(hr))) : P_OOB;
    return __builtin_amdgcn_raw_buffer_load_b128(srcb ? rsB : rsA, off, 0, 0);
  };
  // ... and its LDS store; a store not wanted goes to `spare` (a slot the caller overwrites right after)
  auto store_halo_reg = [&](int g, int slot, v4u32_t v, bool ok, unsigned spare) {
    const int idx = g * NTH + tid;
    const unsigned off = ok && idx < P_HROWS * 8 ? (unsigned)(OH + slot * HBUF + idx * 16) : spare;
    *reinterpret_cast<v4u32_t*>(smem + off) = v;
  };
  v4u32_t hreg = {0u, 0u, 0u, 0u};   // WREG: halo group loaded at the previous step, stored at this one
  int hpend_g = 0, hpend_slot = 0;
  bool hpend = false;
  bool hg_last = false;   // HALO: the latest load_next issued a halo group after its weights (wave-uniform)
  // WREG: the weights of the next step to be issued, in registers (same per-lane source offsets and LDS
  // positions as the LDS-DMA pieces)
  v4u32_t wst[WREG ? 2 : 1][WREG ? GB : 1];
  auto load_w = [&](int lt_) {
    if constexpr (WREG) {
      const int c_ = lt_ / 9, tp_ = lt_ - 9 * c_;
      const unsigned kt = (unsigned)(tp_ * nch + c_);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < GB; ++i)
          wst[h][i] = __builtin_amdgcn_raw_buffer_load_b128(rsW, bo[h][i] == P_OOB ? P_OOB : bo[h][i] + kt * ROWB, 0, 0);
    }
  };
  auto store_w = [&](int buf) {
    if constexpr (WREG) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < GB; ++i)
          *reinterpret_cast<v4u32_t*>(smem + buf * STAGE + (h ? OB1 : OB0) + wave * 8 * ROWB + i * (NTH / 8) * ROWB +
                                      lane * 16) = wst[h][i];
    }
  };
  // the loader's bookkeeping after issuing stream step lsteps = (tile lk, step lt)
  int lsteps = 0, lk_tile = -1;
  auto advance = [&]() {
    ++lsteps;
    ls = ls == NST - 1 ? 0 : ls + 1;
    if (++lt == nk) { lt = 0; ++lk; }
  };
  auto load_next_halo = [&]() {
    hg_last = false;
    if (lt == 0) lk_tile = tile_id(lk);
    if (lk_tile < 0) return;   // stream exhausted (uniform)
    if (no_dma && nissued >= NST - 1) {   // (timing-only ablation, fwd_debug bit 5: bookkeeping only)
      advance();
      return;
    }
    ++nissued;
    const int c = lt / 9, tp = lt - 9 * c;
    // one group of the next chunk of the stream rides on taps NST-1 .. NST-1+GH-1: its tile (the next tile's
    // at the last chunk; -1 past the end of the block's work) and its slot (e + 1) & 1, e = this chunk's index
    const bool hwin = tp >= NST - 1 && tp < NST - 1 + GH;
    const int t2 = !hwin ? -1 : c + 1 < nch ? lk_tile : tile_id(lk + 1);
    const int nc2 = c + 1 < nch ? c + 1 : 0, e = lk * nch + c;
    if constexpr (WREG) {
      // the halo group loaded at the previous step into its slot (or, if none, into this thread's first
      // weight slot of stage ls, which store_w overwrites next), this step's staged weights into stage ls,
      // then the next halo group (taps NST-1 .. NST-1+GH-1 of a chunk) and the next step's weights into
      // registers (the next tile's first step after a tile's last: the same rows for every tile). No LDS-DMA:
      // every wait is the compiler's, on registers.
      store_halo_reg(hpend_g, hpend_slot, hreg, hpend, (unsigned)(ls * STAGE + OB0 + wave * 8 * ROWB + lane * 16));
      store_w(ls);
      hpend = hwin && t2 >= 0;
      hpend_g = hpend ? tp - (NST - 1) : 0;
      hpend_slot = (e + 1) & 1;
      hreg = load_halo_reg(hpend ? t2 : lk_tile, nc2, hpend_g, hpend);
      load_w(lt + 1 < nk ? lt + 1 : 0);
      advance();
      return;
    }
    {   // weights of (tap tp, chunk c): GEMM K rows kt = tp * nch + c
      const unsigned kt = (unsigned)(tp * nch + c);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        unsigned char* dsb = smem + ls * STAGE + (h ? OB1 : OB0) + wave * 8 * ROWB;
#pragma unroll
        for (int i = 0; i < GB; ++i) {
          const unsigned off = bo[h][i] == P_OOB ? P_OOB : bo[h][i] + kt * ROWB;
          p_lds16(rsW, dsb + i * (NTH / 8) * ROWB, off);
        }
      }
    }
    if (t2 >= 0) hg_last = issue_halo(t2, nc2, tp - (NST - 1), (e + 1) & 1);
    advance();
  };
  auto load_next = [&]() {
    if constexpr (HALO) { load_next_halo(); return; }
    if (lt == 0) lk_tile = tile_id(lk);
    if (lk_tile < 0) return;   // stream exhausted (uniform)
    if (no_dma && nissued >= NST - 1) {   // (keep the loader's bookkeeping, issue nothing)
      advance();
      return;
    }
    ++nissued;
    if (lt == 0) {
      setup_rows(m0_of(lk_tile));
      it_ci = it_ty = it_tx = it_kt = 0;
    }
    issue(kinfo(), ls);
    advance();
  };

  const int r16 = lane & 15, h4 = lane >> 4;
  auto readA = [&](int buf, int h, bf16x8 (&fa)[MIQ][2]) {
    const unsigned char* base = smem + buf * STAGE + h * OA1;
#pragma unroll
    for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int q = wr * HM + mi * 16 + r16, c = 4 * s + h4;
        fa[mi][s] = *reinterpret_cast<const bf16x8*>(base + q * ROWB + ((c ^ swz(q)) << 4));
      }
  };
  auto readA_halo = [&](int slot, int dy, int dx, int h, bf16x8 (&fa)[MIQ][2]) {
    const unsigned char* base = smem + OH + slot * HBUF;
#pragma unroll
    for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int p = wr * TM + h * HM + mi * 16 + r16;   // tile pixel: patch row p >> 5, column p & 31
        const int hr = ((p >> 5) + dy) * 34 + (p & 31) + dx, c = 4 * s + h4;
        fa[mi][s] = *reinterpret_cast<const bf16x8*>(base + hr * ROWB + ((c ^ p_hswz(hr)) << 4));
      }
  };
  auto readB = [&](int buf, int h, bf16x8 (&fb)[2][2]) {
    const unsigned char* base = smem + buf * STAGE + (h ? OB1 : OB0);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int q = wc * 32 + ni * 16 + r16, c = 4 * s + h4;
        fb[ni][s] = *reinterpret_cast<const bf16x8*>(base + q * ROWB + ((c ^ swz(q)) << 4));
      }
  };
  // acc[ha*MIQ + mi][hb*2 + ni]: transposed tile, rows = channels n0 + wc*64 + (hb*2+ni)*16 + 4*h4 + reg,
  // column = pixel m0 + wr*TM + ha*HM + mi*16 + r16
  f32x4 acc[2 * MIQ][4];
  auto mma = [&](const bf16x8 (&fa)[MIQ][2], const bf16x8 (&fb)[2][2], int ha, int hb) {
    if constexpr (F32)
      if (hb ? skip1 : skip0) return;
    prio_hi<ADP_PRIO_FWD>();
    if constexpr (F8) {
#pragma unroll
      for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[ha * MIQ + mi][hb * 2 + ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              __builtin_bit_cast(v8i32, fb[ni]), __builtin_bit_cast(v8i32, fa[mi]), acc[ha * MIQ + mi][hb * 2 + ni],
              0, 0, 0, 127, 0, 127);
      prio_lo<ADP_PRIO_FWD>();
      return;
    }
    if constexpr (F32) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[ha * MIQ + mi][hb * 2 + ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                  __builtin_bit_cast(f32x4, fb[ni][s])[e], __builtin_bit_cast(f32x4, fa[mi][s])[e],
                  acc[ha * MIQ + mi][hb * 2 + ni], 0, 0, 0);
      prio_lo<ADP_PRIO_FWD>();
      return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[ha * MIQ + mi][hb * 2 + ni] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ni][s], fa[mi][s], acc[ha * MIQ + mi][hb * 2 + ni], 0, 0, 0);
    prio_lo<ADP_PRIO_FWD>();
  };

  // ---- epilogue resources
  const bool shuffle = EPIC != 4 && a.out_mode == 1, split = EPIC != 4 && a.out_mode == 2;   // (EPIC 4: plain stores)
  const int Hq = 2 * a.Ho, Wq = 2 * a.Wo;
  const bool o8 = F8 && a.out_f8;   // fp8 output (the ConvTranspose forwards of UNetBN.forward_fp8)
  const int oes = o8 ? 1 : OES;
  const unsigned out_bytes = shuffle ? (unsigned)(a.Nimg * Hq * Wq) * a.out_stride * oes : (unsigned)a.M * a.out_stride * oes;
  const int out2_bytes = split ? a.M * a.out2_stride * OES : 0;
  const __amdgpu_buffer_rsrc_t rsZ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(BNR ? a.bnr_z : a.out), 0, BNR ? a.M * a.bnr_zs * OES : 0, P_RSRC3);
  const bool stats = BNR || a.bn_sum != nullptr;

  // BNR with TM = 64: every z quad of the tile (16 loads, 32 registers) is issued in the K loop, right
  // after the tile's last LDS-DMA step and BEFORE the next tile's first one: vmcnt retires in order, so
  // the epilogue's wait for z then does not wait for the prefetch of the next tile (z loaded inside the
  // epilogue drained the whole ring at every tile), and the four channel groups' stores of a pixel row
  // follow each other closely (with z waits between them the partial lines were written twice: 2.1x the
  // output bytes, PMC WRITE_SIZE)
  bf16x4 zall[ZALL ? 4 : 1][ZALL ? 2 * MIQ : 1];
  auto load_zall = [&](int m0) {
    int tidv = tid;
    asm volatile("" : "+v"(tidv));
    const int r16 = tidv & 15, h4 = (tidv >> 4) & 3, wr = w_row(tidv >> 6), wc = w_col(tidv >> 6);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int c = n0 + wc * 64 + nt * 16 + 4 * h4;
#pragma unroll
      for (int mt = 0; mt < 2 * MIQ; ++mt) {
        const int m = pix(m0, wr * TM + (mt / MIQ) * HM + (mt % MIQ) * 16 + r16);
        const bool v = c < a.Nout && m < a.M;
        zall[nt][mt] = __builtin_bit_cast(bf16x4, p_ld8(rsZ, v ? (unsigned)((m * a.bnr_zs + c) * OES) : P_OOB));
      }
    }
  };
  auto epilogue = [&](int m0) {
    // lane-derived epilogue indices made opaque here, so that the compiler cannot hoist their
    // per-(mt, nt) offsets out of the tile loop (they would stay live across the K loop and spill)
    int tidv = tid;
    asm volatile("" : "+v"(tidv));
    const int r16 = tidv & 15, h4 = (tidv >> 4) & 3, wr = w_row(tidv >> 6), wc = w_col(tidv >> 6);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int c = n0 + wc * 64 + nt * 16 + 4 * h4;   // first of this lane's 4 channels (GEMM column)
      const bool cv = c < a.Nout;
      const int cl = wc * 64 + nt * 16 + 4 * h4;         // the same, relative to n0
      const float4 b4 = p_lds_f4(&cst[0][cl]);
      const float bias[4] = {b4.x, b4.y, b4.z, b4.w};
      float wsc[4] = {1.f, 1.f, 1.f, 1.f};
      if constexpr (F8) {
        const float4 w4 = p_lds_f4(&cst[1][cl]);
        wsc[0] = w4.x; wsc[1] = w4.y; wsc[2] = w4.z; wsc[3] = w4.w;
      }
      float sc[4], sh[4], mu[4], is[4];
      // BNR: the 2*MIQ z quads of this channel group, all loaded before the first store of the group (a
      // load behind a store waits for it: vmcnt retires in order)
      bf16x4 zq[BNR && !ZALL ? 2 * MIQ : 1];
      if constexpr (BNR) {
        const float4 a4 = p_lds_f4(&cst[1][cl]);
        const float4 s4 = p_lds_f4(&cst[2][cl]);
        const float4 m4 = p_lds_f4(&cst[3][cl]);
        const float4 i4 = p_lds_f4(&cst[4][cl]);
        sc[0] = a4.x; sc[1] = a4.y; sc[2] = a4.z; sc[3] = a4.w;
        sh[0] = s4.x; sh[1] = s4.y; sh[2] = s4.z; sh[3] = s4.w;
        mu[0] = m4.x; mu[1] = m4.y; mu[2] = m4.z; mu[3] = m4.w;
        is[0] = i4.x; is[1] = i4.y; is[2] = i4.z; is[3] = i4.w;
        if constexpr (!ZALL) {
#pragma unroll
          for (int mt = 0; mt < 2 * MIQ; ++mt) {
            const int m = pix(m0, wr * TM + (mt / MIQ) * HM + (mt % MIQ) * 16 + r16);
            const bool v = cv && m < a.M;
            zq[mt] = __builtin_bit_cast(bf16x4, p_ld8(rsZ, v ? (unsigned)((m * a.bnr_zs + c) * OES) : P_OOB));
          }
        }
      }
      // store target of the channel quad: GEMM column c -> (buffer, channel offset)
      int sub = 0, cq = c;
      if (shuffle) { sub = c / a.Cps; cq = c - sub * a.Cps; }
      // (split_c % 16 == 0: the whole 16-channel block of the wave goes to one buffer -- a scalar choice
      //  of the buffer resource, no per-lane waterfall around the store)
      const bool second = split && __builtin_amdgcn_readfirstlane(n0 + wc * 64 + nt * 16) >= a.split_c;
      if (second) cq = c - a.split_c;
      const int ostr = second ? a.out2_stride : a.out_stride;
      // the store target's resource, built from a scalar pointer choice (selecting between two resource
      // objects makes the compiler spill them to the stack and reload per lane)
      const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(second ? a.out2 : a.out, 0,
                                                                         second ? out2_bytes : (int)out_bytes, P_RSRC3);
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mt = 0; mt < 2 * MIQ; ++mt) {
        const int m = pix(m0, wr * TM + (mt / MIQ) * HM + (mt % MIQ) * 16 + r16);
        const bool v = cv && m < a.M;
        float x[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[r] = F8 ? fmaf(acc[mt][nt][r], wsc[r], bias[r]) : acc[mt][nt][r] + bias[r];
          if (a.relu) x[r] = fmaxf(x[r], 0.f);
        }
        bf16x4 o;
        if constexpr (!F32) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16)x[r];
        }
        int pix = m;
        if (shuffle) {
          const int img = m / HWo, rem = m - img * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
          pix = (img * Hq + 2 * yo + (sub >> 1)) * Wq + 2 * xo + (sub & 1);
        }
        // (timing-only ablation, fwd_debug bit 7: every store to an out-of-range offset, dropped)
        const unsigned off = v && !(ADP_DBG(a) & 128) ? (unsigned)((pix * ostr + cq) * oes) : P_OOB;
        if constexpr (F32) {
          const f32x4 o4 = {x[0], x[1], x[2], x[3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, o4), rsO, off, 0, 0);
        } else if (o8) {   // 4 channels -> 4 e4m3 bytes (f8x8_from_f's saturating encode)
          float c8[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) c8[r] = fminf(fmaxf(x[r], -FP8_MAX), FP8_MAX);
          int q = __builtin_amdgcn_cvt_pk_fp8_f32(c8[0], c8[1], 0, false);
          q = __builtin_amdgcn_cvt_pk_fp8_f32(c8[2], c8[3], q, true);
          __builtin_amdgcn_raw_buffer_store_b32((unsigned)q, rsO, off, 0, 0);
        } else {
          p_st8(rsO, off, __builtin_bit_cast(v2u32, o));
        }
        if constexpr (BNR) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float g = (float)o[r], zf = (float)(ZALL ? zall[nt][mt][r] : zq[ZALL ? 0 : mt][r]);   // stored gradient
            const float db = fmaf(zf, sc[r], sh[r]) > 0.f ? g : 0.f;
            s1[r] += db;
            s2[r] += db * (zf - mu[r]) * is[r];
          }
        } else if (stats && v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) { s1[r] += x[r]; s2[r] += x[r] * x[r]; }
        }
      }
      if (stats) {   // over the 16 pixel lanes of the channel quad, then into the block's LDS sums
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s1[r] = row16_sum(s1[r]);
          s2[r] = row16_sum(s2[r]);
        }
        if (r16 == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p_lds_add(&sacc[0][cl + r], s1[r]);
            p_lds_add(&sacc[1][cl + r], s2[r]);
          }
        }
      }
    }
  };
  // wide_st (bf16, no BN-backward reduction): the channel quads of 16-channel groups nt and nt + 1 are
  // joined into 8-channel runs before the store. Lane row h4 (16 lanes, one pixel each) holds channels
  // 16 nt + 4 h4 .. + 3; v_permlane16_swap exchanges the odd rows of group nt with the even rows of group
  // nt + 1, after which row h4 holds channels 16 (nt + (h4 & 1)) + 8 (h4 >> 1) .. + 7 of its pixel: one
  // 16-B store per (pixel, pair of groups) instead of two 8-B ones, 64 contiguous bytes of a pixel per
  // instruction instead of 32. Needs Nout % 16 == 0 and a split point on a 32-channel boundary (host).
  auto epilogue_wide = [&](int m0) {
    if constexpr (!BNR && !F32) {
      int tidv = tid;
      asm volatile("" : "+v"(tidv));
      const int r16 = tidv & 15, h4 = (tidv >> 4) & 3, wr = w_row(tidv >> 6), wc = w_col(tidv >> 6);
#pragma unroll
      for (int np = 0; np < 4; np += 2) {
        float bias[2][4], wsc[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float4 b4 = p_lds_f4(&cst[0][wc * 64 + (np + j) * 16 + 4 * h4]);
          bias[j][0] = b4.x; bias[j][1] = b4.y; bias[j][2] = b4.z; bias[j][3] = b4.w;
          if constexpr (F8) {   // the per-column dequantisation scale (bf16 output)
            const float4 w4 = p_lds_f4(&cst[1][wc * 64 + (np + j) * 16 + 4 * h4]);
            wsc[j][0] = w4.x; wsc[j][1] = w4.y; wsc[j][2] = w4.z; wsc[j][3] = w4.w;
          }
        }
        // this lane's 8-channel run after the exchange, and its store target
        const int cw = n0 + wc * 64 + 16 * (np + (h4 & 1)) + 8 * (h4 >> 1);
        const bool cv = cw < a.Nout;
        int sub = 0, cq = cw;
        if (shuffle) { sub = cw / a.Cps; cq = cw - sub * a.Cps; }
        const bool second = split && __builtin_amdgcn_readfirstlane(n0 + wc * 64 + np * 16) >= a.split_c;
        if (second) cq = cw - a.split_c;
        const int ostr = second ? a.out2_stride : a.out_stride;
        const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(second ? a.out2 : a.out, 0,
                                                                           second ? out2_bytes : (int)out_bytes, P_RSRC3);
        float s1[2][4] = {}, s2[2][4] = {};
#pragma unroll
        for (int mt = 0; mt < 2 * MIQ; ++mt) {
          const int m = pix(m0, wr * TM + (mt / MIQ) * HM + (mt % MIQ) * 16 + r16);
          const bool mv = m < a.M;
          v2u32 o2[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bool qv = mv && n0 + wc * 64 + (np + j) * 16 + 4 * h4 < a.Nout;   // (statistics: own quad)
            float x[4];
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              x[r] = F8 ? fmaf(acc[mt][np + j][r], wsc[j][r], bias[j][r]) : acc[mt][np + j][r] + bias[j][r];
              if (a.relu) x[r] = fmaxf(x[r], 0.f);
              o[r] = (bf16)x[r];
            }
            o2[j] = __builtin_bit_cast(v2u32, o);
            if (stats && qv) {
#pragma unroll
              for (int r = 0; r < 4; ++r) { s1[j][r] += x[r]; s2[j][r] += x[r] * x[r]; }
            }
          }
          const auto e0 = __builtin_amdgcn_permlane16_swap(o2[0].x, o2[1].x, false, false);
          const auto e1 = __builtin_amdgcn_permlane16_swap(o2[0].y, o2[1].y, false, false);
          const v4u32_t st = {e0[0], e1[0], e0[1], e1[1]};
          int pixo = m;
          if (shuffle) {
            const int img = m / HWo, rem = m - img * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
            pixo = (img * Hq + 2 * yo + (sub >> 1)) * Wq + 2 * xo + (sub & 1);
          }
          const unsigned off = mv && cv && !(ADP_DBG(a) & 128) ? (unsigned)((pixo * ostr + cq) * OES) : P_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(st, rsO, off, 0, 0);
        }
        if (stats) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              s1[j][r] = row16_sum(s1[j][r]);
              s2[j][r] = row16_sum(s2[j][r]);
            }
            if (r16 == 0) {
              const int cl = wc * 64 + (np + j) * 16 + 4 * h4;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                p_lds_add(&sacc[0][cl + r], s1[j][r]);
                p_lds_add(&sacc[1][cl + r], s2[j][r]);
              }
            }
          }
        }
      }
    }
  };
  // wide_st = 2: the same 16-B stores in line order. epilogue_wide writes the first 64 B of the wave's 128-B pixel
  // lines (groups 0-1) for all 2 * MIQ pixel groups and only then the second 64 B (groups 2-3): 16 store instructions
  // apart, and with every CU of an XCD in its epilogue at once (8 waves x 128 pixels x 64 B = 64 KiB per CU, 2 MiB per
  // XCD between the two halves of a line) the L2 writes many lines back in halves -- PMC WRITE_SIZE 1.48x the output
  // bytes on every level (profiles/r04c_pmc_dom.txt). Here the two halves of each pixel line leave in consecutive
  // instructions. Same values, same stores: bit-identical.
  auto epilogue_lines = [&](int m0) {
    if constexpr (!BNR && !F32) {
      int tidv = tid;
      asm volatile("" : "+v"(tidv));
      const int r16 = tidv & 15, h4 = (tidv >> 4) & 3, wr = w_row(tidv >> 6), wc = w_col(tidv >> 6);
      float bias[4][4], wsc[4][4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float4 b4 = p_lds_f4(&cst[0][wc * 64 + nt * 16 + 4 * h4]);
        bias[nt][0] = b4.x; bias[nt][1] = b4.y; bias[nt][2] = b4.z; bias[nt][3] = b4.w;
        if constexpr (F8) {
          const float4 w4 = p_lds_f4(&cst[1][wc * 64 + nt * 16 + 4 * h4]);
          wsc[nt][0] = w4.x; wsc[nt][1] = w4.y; wsc[nt][2] = w4.z; wsc[nt][3] = w4.w;
        }
      }
      // per pair of groups (np = 0, 2): this lane's 8-channel run after the exchange and its store target
      int cqp[2], subp[2], ostrp[2];
      bool cvp[2];
      __amdgpu_buffer_rsrc_t rsOp[2];
#pragma unroll
      for (int pi = 0; pi < 2; ++pi) {
        const int np = 2 * pi;
        const int cw = n0 + wc * 64 + 16 * (np + (h4 & 1)) + 8 * (h4 >> 1);
        cvp[pi] = cw < a.Nout;
        subp[pi] = 0;
        cqp[pi] = cw;
        if (shuffle) { subp[pi] = cw / a.Cps; cqp[pi] = cw - subp[pi] * a.Cps; }
        const bool second = split && __builtin_amdgcn_readfirstlane(n0 + wc * 64 + np * 16) >= a.split_c;
        if (second) cqp[pi] = cw - a.split_c;
        ostrp[pi] = second ? a.out2_stride : a.out_stride;
        rsOp[pi] = __builtin_amdgcn_make_buffer_rsrc(second ? a.out2 : a.out, 0, second ? out2_bytes : (int)out_bytes,
                                                     P_RSRC3);
      }
      float s1[4][4] = {}, s2[4][4] = {};
#pragma unroll
      for (int mt = 0; mt < 2 * MIQ; ++mt) {
        const int m = pix(m0, wr * TM + (mt / MIQ) * HM + (mt % MIQ) * 16 + r16);
        const bool mv = m < a.M;
#pragma unroll
        for (int pi = 0; pi < 2; ++pi) {
          v2u32 o2[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int nt = 2 * pi + j;
            const bool qv = mv && n0 + wc * 64 + nt * 16 + 4 * h4 < a.Nout;   // (statistics: own quad)
            float x[4];
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              x[r] = F8 ? fmaf(acc[mt][nt][r], wsc[nt][r], bias[nt][r]) : acc[mt][nt][r] + bias[nt][r];
              if (a.relu) x[r] = fmaxf(x[r], 0.f);
              o[r] = (bf16)x[r];
            }
            o2[j] = __builtin_bit_cast(v2u32, o);
            if (stats && qv) {
#pragma unroll
              for (int r = 0; r < 4; ++r) { s1[nt][r] += x[r]; s2[nt][r] += x[r] * x[r]; }
            }
          }
          const auto e0 = __builtin_amdgcn_permlane16_swap(o2[0].x, o2[1].x, false, false);
          const auto e1 = __builtin_amdgcn_permlane16_swap(o2[0].y, o2[1].y, false, false);
          const v4u32_t st = {e0[0], e1[0], e0[1], e1[1]};
          int pixo = m;
          if (shuffle) {
            const int img = m / HWo, rem = m - img * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
            pixo = (img * Hq + 2 * yo + (subp[pi] >> 1)) * Wq + 2 * xo + (subp[pi] & 1);
          }
          const unsigned off =
              mv && cvp[pi] && !(ADP_DBG(a) & 128) ? (unsigned)((pixo * ostrp[pi] + cqp[pi]) * OES) : P_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(st, rsOp[pi], off, 0, 0);
        }
      }
      if (stats) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1[nt][r] = row16_sum(s1[nt][r]);
            s2[nt][r] = row16_sum(s2[nt][r]);
          }
          if (r16 == 0) {
            const int cl = wc * 64 + nt * 16 + 4 * h4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              p_lds_add(&sacc[0][cl + r], s1[nt][r]);
              p_lds_add(&sacc[1][cl + r], s2[nt][r]);
            }
          }
        }
      }
    }
  };
  // wide_st = 3 (fp8 output): the four 16-channel groups' quads of a lane (one e4m3 dword each) transposed over the
  // lane rows -- v_permlane16_swap on the pairs (0, 1) and (2, 3), then v_permlane32_swap on (0, 2) and (1, 3) --
  // leave lane row h4 with channels 16 h4 .. + 15 of its pixel: one 16-B store per pixel group instead of four
  // 4-B stores (a 64-B fp8 pixel line per instruction and pixel; pixel-shuffle targets are whole 16-channel runs)
  auto epilogue_q8 = [&](int m0) {
    if constexpr (F8) {
      int tidv = tid;
      asm volatile("" : "+v"(tidv));
      const int r16 = tidv & 15, h4 = (tidv >> 4) & 3, wr = w_row(tidv >> 6), wc = w_col(tidv >> 6);
      // pass 1, group by group (8 constants live): each quad -> its e4m3 dword, kept in the accumulator's first
      // register (no extra registers: the 256x256 forms have none to spare)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float4 b4 = p_lds_f4(&cst[0][wc * 64 + nt * 16 + 4 * h4]);
        const float4 w4 = p_lds_f4(&cst[1][wc * 64 + nt * 16 + 4 * h4]);
        const float bias[4] = {b4.x, b4.y, b4.z, b4.w}, wsc[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int mt = 0; mt < 2 * MIQ; ++mt) {
          float c8[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = fmaf(acc[mt][nt][r], wsc[r], bias[r]);
            if (a.relu) x = fmaxf(x, 0.f);
            c8[r] = fminf(fmaxf(x, -FP8_MAX), FP8_MAX);
          }
          int q = __builtin_amdgcn_cvt_pk_fp8_f32(c8[0], c8[1], 0, false);
          q = __builtin_amdgcn_cvt_pk_fp8_f32(c8[2], c8[3], q, true);
          acc[mt][nt][0] = __builtin_bit_cast(float, q);
        }
      }
      const int cw = n0 + wc * 64 + 16 * h4;   // this lane's 16 channels after the transpose
      const bool cv = cw < a.Nout;
      int sub = 0, cq = cw;
      if (shuffle) { sub = cw / a.Cps; cq = cw - sub * a.Cps; }
      const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)out_bytes, P_RSRC3);
      // pass 2, pixel group by pixel group: transpose and store
#pragma unroll
      for (int mt = 0; mt < 2 * MIQ; ++mt) {
        const int m = pix(m0, wr * TM + (mt / MIQ) * HM + (mt % MIQ) * 16 + r16);
        const bool mv = m < a.M;
        unsigned d[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) d[nt] = __builtin_bit_cast(unsigned, acc[mt][nt][0]);
        const auto p01 = __builtin_amdgcn_permlane16_swap(d[0], d[1], false, false);
        const auto p23 = __builtin_amdgcn_permlane16_swap(d[2], d[3], false, false);
        const auto q02 = __builtin_amdgcn_permlane32_swap(p01[0], p23[0], false, false);
        const auto q13 = __builtin_amdgcn_permlane32_swap(p01[1], p23[1], false, false);
        const v4u32_t st = {q02[0], q13[0], q02[1], q13[1]};
        int pixo = m;
        if (shuffle) {
          const int img = m / HWo, rem = m - img * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
          pixo = (img * Hq + 2 * yo + (sub >> 1)) * Wq + 2 * xo + (sub & 1);
        }
        const unsigned off = mv && cv && !(ADP_DBG(a) & 128) ? (unsigned)(pixo * a.out_stride + cq) : P_OOB;
        __builtin_amdgcn_raw_buffer_store_b128(st, rsO, off, 0, 0);
      }
    }
  };
  const bool q8l = F8 && a.wide_st == 3;   // (fp8 output, launcher: Nout % 16, Cps % 16, out_stride % 16)
  // (fp8 forms: bf16 output through the narrow epilogue, fp8 output through epilogue_q8 -- the 16-B bf16 forms are not
  //  compiled into them: with all three epilogues the 256x256 fp8 forms spill)
  const bool wide = EPIC >= 2 || (EPIC < 0 && !BNR && !F32 && !F8 && a.wide_st && a.wide_st != 3);

  bf16x8 fa[MIQ][2], fb0[2][2], fb1[2][2];
  // staggered issue (option tap64p_stagger): waves 4-7 issue their LDS-DMA pieces after their first MFMA
  // cluster instead of right after the barrier. Waves w and w + 4 share a SIMD, so one of them multiplies
  // while the other issues (the issue of a piece costs the issuing wave 60-185 cycles); with every wave
  // issuing after the barrier the DMA issue and the MFMAs serialised on each SIMD (the no-DMA ablation
  // runs the K loop 20 % faster)
  // (issuing each wave's step in two halves spread over the clusters measured 5-9 % slower:
  //  profiles/r02_stagger_ab.txt)
  const bool late = a.stagger && ((__builtin_amdgcn_readfirstlane(wave) >> 2) & 1);
  int hslot = 0, hdy = 0, hdx = 0;   // HALO: halo slot and tap of the step being multiplied
  auto rA = [&](int buf, int h) {
    if constexpr (HALO) readA_halo(hslot, hdy, hdx, h, fa);
    else readA(buf, h, fa);
  };
  auto compute = [&](int buf, bool issue_late) {
    rA(buf, 0);
    readB(buf, 0, fb0);
    mma(fa, fb0, 0, 0);
    if (issue_late) load_next();
    readB(buf, 1, fb1);
    mma(fa, fb1, 0, 1);
    rA(buf, 1);
    mma(fa, fb1, 1, 1);
    mma(fa, fb0, 1, 0);
  };
  // ---- the stream: prologue fills NST - 1 stages; step gs waits for its stage, issues step gs + NST - 1
  // into the stage step gs - 1 read (every wave is past this step's barrier, so nobody reads it), multiplies.
  // The wait counts what was issued after the stage: the NST - 2 younger stages and, when a tile ended
  // inside that window, its EPI_OPS epilogue ops; near the end of the stream (fewer younger stages) it
  // drains everything.
  if (full) {   // the first two tiles (a block that starts late finds them past the end and leaves)
    if (tid == 0) {
      ring[0] = r2;
      ring[1] = r2 + 1;
    }
    __syncthreads();
  }
  if constexpr (WREG) {   // the first chunk's whole halo ahead of the stream (registers -> LDS)
#pragma unroll
    for (int g = 0; g < GH; ++g)
      store_halo_reg(g, 0, load_halo_reg(tile_id(0), 0, g, true), true, (unsigned)(OB0 + tid * 16));
  } else if constexpr (HALO) {   // the first chunk's whole halo ahead of the stream
    const int t0 = tile_id(0);
    if (t0 >= 0) {
#pragma unroll
      for (int g = 0; g < GH; ++g) issue_halo(t0, 0, g, 0);
    }
  }
  if constexpr (WREG) load_w(0);   // (the first load_next stores them into stage 0)
  // dyn: the claim of tile 1 goes out before the prologue's stages, so the wait at the top of step 0 covers it
  int c1val = 0;
  if (dyn && !full && tid == 0) c1val = claim_issue(a.claim + col);
#pragma unroll
  for (int i = 0; i < NST - 1; ++i) load_next();
  int gs = 0, cs = 0, last_epi = -NST;   // step, its stage, step of the latest epilogue
  for (int k = 0;; ++k) {
    const int tk = tile_id(k);
    if (tk < 0) break;   // the block's work is done (uniform)
    const int m0c = m0_of(tk);
#pragma unroll
    for (int i = 0; i < 2 * MIQ; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bool zissued = false;
    int zstep = -NST;   // step whose barrier preceded this tile's z loads
    for (int t = 0; t < nk; ++t, ++gs) {
      // ops younger than stage cs: the NST - 2 stages issued after it, an epilogue in the window, and the
      // z loads when they went out at the previous step (after cs, before that step's stage); a count
      // that is too small only waits longer, so the combinations are covered by the smaller constant
      // (HALO, NST = 2: the stage's weights plus, when this wave issued one, a halo group after them; the
      // halo of a chunk was issued before the weights of the chunk's first step, so it has landed too)
      if constexpr (HALO) {
        // NST = 3: the younger stage's weights are counted, its halo groups not (a smaller count only
        // waits longer)
        if constexpr (WREG) {
          // the stage and the halo groups were written by every wave's ds_write at earlier steps
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (ADP_DBG(a) & 64) {   // timing-only ablation (fwd_debug bit 6): LDS-DMA issued, never waited for
        } else if (gs + NST - 2 >= lsteps) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (last_epi > gs - NST) {
          if (q8l) {
            if (NST == 2 && hg_last) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI_Q + 1 < 63 ? VM_EPI_Q + 1 : 63) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI_Q) : "memory");
          } else if (wide) {
            if (NST == 2 && hg_last) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI_W + 1 < 63 ? VM_EPI_W + 1 : 63) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI_W) : "memory");
          } else if (NST == 2 && hg_last) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI + 1 < 63 ? VM_EPI + 1 : 63) : "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI) : "memory");
          }
        } else if (NST == 2 && hg_last) {
          asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * LOPS) : "memory");
        }
        const int c = t / 9, tp = t - 9 * c;
        hslot = (k * nch + c) & 1;
        hdy = tp / 3;
        hdx = tp - 3 * hdy;
      } else if (gs + NST - 2 >= lsteps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (last_epi > gs - NST && q8l) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI_Q) : "memory");
      else if (last_epi > gs - NST && wide) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI_W) : "memory");
      else if (last_epi > gs - NST) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_EPI) : "memory");
      else if (ZALL && zstep == gs - 1 && NST > 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM_Z) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * LOPS) : "memory");
      if (dyn && !full && gs == 0 && tid == 0) claim_publish<-1>(ring + 1, c1val);   // tile 1 (claimed in the prologue)
      // (timing-only ablation, fwd_debug bit 9: no barrier -- the stages race, the values are garbage)
      if (!(ADP_DBG(a) & 512)) P_BAR();   // stage cs landed for every wave, nobody reads the stage being refilled
      if constexpr (ZALL) {
        if (!zissued && lk > k) {   // the loader is past this tile: z before the next tile's first stage
          load_zall(m0c);
          zissued = true;
          zstep = gs;
        }
      }
      // dyn: when the loader starts tile lk at this step, thread 0 claims tile lk + 1 (an atomic the compiler
      // does not wait for: claim_issue) and publishes it after the multiply, waiting only for the atomic (the
      // step's own LDS-DMA pieces, issued after it, stay in flight); the next barrier makes it visible, ahead
      // of the loader's first use (step NST - 1 of tile lk for the halo form, the next tile's first step else)
      bool claim_now = false;
      int cslot = 0, cval = 0;
      if (dyn && lt == 0) {
        lk_tile = tile_id(lk);
        claim_now = lk_tile >= 0;
        cslot = (lk + 1) & 3;
        if (claim_now && tid == 0) cval = claim_issue(a.claim + col);
      }
      if (!late) load_next();
      compute(cs, late);
      if (claim_now && tid == 0) {
        if (WREG || no_dma) claim_publish<0>(ring + cslot, cval);
        else claim_publish<LOPS>(ring + cslot, cval);
      }
      cs = cs == NST - 1 ? 0 : cs + 1;
    }
    last_epi = gs - 1;
    if (ADP_DBG(a) & 16) {   // timing-only ablation (option fwd_debug bit 4): no epilogue
#pragma unroll
      for (int i = 0; i < 2 * MIQ; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
      last_epi = -NST;   // (no epilogue ops were issued)
      continue;
    }
    if constexpr (EPIC >= 2) epilogue_lines(m0c);
    else if (q8l) epilogue_q8(m0c);
    else if (wide && a.wide_st == 2) epilogue_lines(m0c);
    else if (wide) epilogue_wide(m0c);
    else epilogue(m0c);
  }

  if (dyn && tid == 0) claim_block_done(a.claim, ntn, G);   // (every claim of the block has returned)
  // ---- BatchNorm sums of the block -> its replica of the accumulators (folded by the launcher)
  if (!stats || (ADP_DBG(a) & 2)) return;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  double* rep = a.stat + (size_t)(blockIdx.x & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
  if (tid < BN) {
    const int n = n0 + tid;
    if (n < a.Nout) {
      const int c = shuffle ? n % a.Cps : n;
      atomicAdd(rep + c, sacc[0][tid]);
      atomicAdd(rep + adp::STAT_CMAX + c, sacc[1][tid]);
    }
  }
}

#undef P_BAR

}  // namespace

namespace adp {
// persistent launch for the epilogue forms it covers; 0 = not eligible (the caller falls back).
// Tile / ring (option tap64p_cfg, 0 = from the tap64 tile choice): 1 = 256x256 / 2 stages,
// 2 = 256x128 / 3 stages, 3 = 128x256 / 3 stages.
int launch_fwd_tap64p(FwdArgs& a, hipStream_t s, int tile) {
  if (!option("tap64_persist", 1) || a.K < 128) return 0;   // (two bf16 K steps / one fp8 step at least)
  // fp8: the halo forms with a plain bf16 store (the eval convs of UNetBN.forward_fp8)
  if (a.f8 && (!option("tap64p_f8", 1) || a.out_mode == 2 || a.bn_sum || a.bnr_z ||
               a.CAs % 128 != 0 || a.CBs % 128 != 0))
    return 0;
  if (a.addend || a.mask || a.mask2 || a.accum || a.drop_rate > 0.f || a.scA || a.scB) return 0;
  // f32: the 256x128 halo form (the tap64 256x128 choice, option tap64p_f32), no BN-backward reduction
  if (a.f32 && (!option("tap64p_f32", 1) || tile != 1 || a.bnr_z)) return 0;
  if (a.up != 1 && (a.up != 2 || a.bnr_z)) return 0;   // up = 2: the halo form only (below)
  if (a.out_mode == 1 && (a.Cps % 8 != 0 || a.Nout % a.Cps != 0)) return 0;
  if (a.out_mode == 2 && (a.split_c % 16 != 0 || a.out2_stride % 8 != 0)) return 0;
  if (a.out_stride % 8 != 0 || (a.bnr_z && a.bnr_zs % 8 != 0)) return 0;
  const int Cin_s = a.CAs + a.CBs;
  const int ks = a.f32 ? 32 : 64, es = a.f32 ? 4 : 2;   // K-step channels (bf16 / f32), element bytes
  if (a.CAs % ks != 0 || a.CBs % ks != 0 || a.K != a.kh * a.kw * Cin_s || a.K % ks != 0 || a.Kpad != a.K) return 0;
  // buffer-resource offsets: every operand below 2 GiB
  const size_t lim = (size_t)1 << 31, pix = (size_t)a.Nimg * a.Hs * a.Ws;
  const size_t outb = a.out_mode == 1 ? (size_t)a.M * 4 * a.out_stride * es : (size_t)a.M * a.out_stride * es;
  if (pix * a.CAs * es >= lim || pix * a.CBs * es >= lim || outb >= lim ||
      (size_t)((a.Nout + 63) / 64 * 64) * a.Kpad * es >= lim || (a.out2 && (size_t)a.M * a.out2_stride * es >= lim) ||
      (a.bnr_z && (size_t)a.M * a.bnr_zs * 2 >= lim))
    return 0;
  // auto (tools/bench_kernels.py, bench_convt.py; profiles/r02_tap64p_cfg_ab.txt): the tap64 256x128 choice
  // -> 256x128 / 3 stages; 256x256 -> 256x256 / 2 stages for K >= 512 (3x3 layers: +3-7 % over tap64) and
  // 128x256 / 3 stages for the short ConvTranspose K of 128..256 (+8-15 % over 256x256); the fused BN-backward
  // reduction only on the 256x128 form (its z loads wait behind the prefetch stream, which costs the
  // 256x256 form 5-8 % against tap64's LDS-staged epilogue)
  a.stagger = option("tap64p_stagger", 1);
  // 16-B epilogue stores (bf16, no BN-backward reduction; whole 16-channel groups, split on 32 channels):
  // level 2 forward +6 %, level 3 +3 %, step -1.4 %, bit-identical (profiles/r03_wide_store_ab.txt)
  // (a software-pipelined K loop -- barrier in the middle of the previous step, B half 0 preloaded -- measured
  //  1.5-5 % slower here and was removed: profiles/r03_kpipe_ab.txt)
  // fp8 launches with a bf16 output take them too (option tap64p_wide_f8); fp8 outputs keep 4-B stores
  // tap64p_wide = 2 (default since round 4): the same stores in line order (epilogue_lines): PMC writes 1.48x ->
  // 1.00x the output bytes on levels 2-4, the kernel +1.0-1.3 % on levels 2-3, step 23.51 -> 23.43 ms
  // (profiles/r04c_wlines_*.txt); 1 = the pair-major order of round 3
  const int wide_opt = option("tap64p_wide", 2);
  a.wide_st = wide_opt && !a.f32 && (!a.f8 || (option("tap64p_wide_f8", 0) && !a.out_f8)) && !a.bnr_z &&
              a.Nout % 16 == 0 && (a.out_mode != 2 || a.split_c % 32 == 0)
                  ? (wide_opt == 2 ? 2 : 1)
                  : 0;
  // fp8 output (option tap64p_f8_lines): the lane-transposed 16-B stores of epilogue_q8
  if (a.f8 && a.out_f8 && option("tap64p_f8_lines", 1) && a.Nout % 16 == 0 && a.out_stride % 16 == 0 &&
      (a.out_mode != 1 || a.Cps % 16 == 0))
    a.wide_st = 3;
  int cfg = option("tap64p_cfg", 0);
  if (cfg < 1 || cfg > 3) {
    if (a.bnr_z && tile != 1 && option("tap64p_bnr", 1) < 2) return 0;
    cfg = tile == 1 ? 2 : (a.K <= 256 ? 3 : 1);
  }
  const int BM = cfg == 3 ? 128 : 256, BN = cfg == 2 ? 128 : 256;
  a.ntile_n = (a.Nout + BN - 1) / BN;
  const int mt = (a.M + BM - 1) / BM;
  a.nblocks = mt * a.ntile_n;   // tiles; the grid is persistent
  int grid = std::min(a.nblocks, option("tap64_persist_grid", 256));
  grid -= grid % a.ntile_n;
  if (grid <= 0) grid = a.ntile_n;
  // dynamic tile claiming (option tap64p_claim): robust to CUs held by another stream's kernels (RCCL)
  a.claim = nullptr;
  if (option("tap64p_claim", option("dp_claim", 0)) && a.ntile_n + 1 <= CLAIM_INTS) a.claim = claim_slot();   // (nullptr: static lists)
  // claim_full: only with at least 4 tiles per block (its first claim takes tiles 0 and 1 at once: with fewer,
  // the blocks that start first would take two tiles each and leave the rest idle -- 2x on a 1-tile-per-block launch)
  a.claim_full = option("claim_full", 0) && mt >= 4 * (grid / a.ntile_n);
  const bool bnr = a.bnr_z != nullptr;
  // the halo form (option tap64p_halo): 3x3 stride-1 'same' layers whose output tiles into 8 x 32 patches
  const bool halo_shape = !bnr && option("tap64p_halo", 1) && a.out_mode != 1 && a.kh == 3 && a.kw == 3 &&
                          a.dil == 1 && a.pad == 1 && a.stride == 1 && a.Ho == a.Hs * a.up && a.Wo == a.Ws * a.up &&
                          a.Ho % 8 == 0 && a.Wo % 32 == 0;
  if (a.up != 1 && !(halo_shape && (cfg == 1 || (cfg == 2 && option("tap64p_halo128", 1))))) return 0;
  if (a.f32) {
    if (!halo_shape || cfg != 2) return 0;
    adp::set_kernel("igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, true, -1>");
    hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, true>), dim3(grid), dim3(512), 0,
                       s, a);
    return 1;
  }
  if (a.f8 && !(halo_shape && (cfg == 1 || cfg == 2))) {   // gather form (ConvTranspose, fp8 output)
    adp::set_kernel("igemm_fwd_tap64p_kernel<%d, %d, %d, false, false, true, false, false, -1>", BM, BN, cfg == 1 ? 2 : 3);
    if (cfg == 1) hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 256, 2, false, false, true>), dim3(grid), dim3(512), 0, s, a);
    else if (cfg == 2) hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 128, 3, false, false, true>), dim3(grid), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<128, 256, 3, false, false, true>), dim3(grid), dim3(512), 0, s, a);
    return 1;
  }
  if (a.f8) {
    if (cfg == 1) {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, true, false, false, -1>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 256, 2, false, true, true>), dim3(grid), dim3(512), 0, s, a);
    } else {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 128, 3, false, true, true, false, false, -1>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 128, 3, false, true, true>), dim3(grid), dim3(512), 0, s, a);
    }
    return 1;
  }
  // the four-wave direct-weight form (conv_fwd_w4.hip) for the layers it covers
  if (halo_shape && cfg == 1 && launch_fwd_w4(a, s)) return 1;
  if (halo_shape && cfg == 1 && option("tap64p_wreg", 0)) {   // opt-in: 5-9 % slower (profiles/r03_wreg_ab.txt)
    adp::set_kernel("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, true, false, -1>");
    hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, true>), dim3(grid), dim3(512), 0, s, a);
    return 1;
  }
  // (line-ordered stores, the default: the instance with only that epilogue compiled, option tap64p_epic)
  const bool epic = a.wide_st == 2 && option("tap64p_epic", 1);
  const bool epic3 = epic && !a.claim && option("tap64p_epic3", 1);   // (static tile lists: no claiming code)
  if (halo_shape && cfg == 1) {
    if (epic3 && a.out_mode == 0 && option("tap64p_epic4", 1)) {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 4>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 4>), dim3(grid), dim3(512), 0, s, a);
      return 1;
    }
    if (epic3) {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 3>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 3>), dim3(grid), dim3(512), 0, s, a);
      return 1;
    }
    if (epic) {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 2>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, 2>), dim3(grid), dim3(512), 0, s, a);
      return 1;
    }
    adp::set_kernel("igemm_fwd_tap64p_kernel<256, 256, 2, false, true, false, false, false, -1>");
    hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 256, 2, false, true>), dim3(grid), dim3(512), 0, s, a);
    return 1;
  }
  if (halo_shape && cfg == 2 && option("tap64p_halo128", 1)) {
    if (epic3 && a.out_mode == 0 && option("tap64p_epic4", 1)) {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, false, 4>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, false, 4>), dim3(grid), dim3(512), 0, s, a);
      return 1;
    }
    if (epic3) {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, false, 3>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, false, 3>), dim3(grid), dim3(512), 0, s, a);
      return 1;
    }
    if (epic) {
      adp::set_kernel("igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, false, 2>");
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, false, 2>), dim3(grid), dim3(512), 0, s, a);
      return 1;
    }
    adp::set_kernel("igemm_fwd_tap64p_kernel<256, 128, 3, false, true, false, false, false, -1>");
    hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<256, 128, 3, false, true>), dim3(grid), dim3(512), 0, s, a);
    return 1;
  }
  if (epic && !bnr)
    adp::set_kernel("igemm_fwd_tap64p_kernel<%d, %d, %d, false, false, false, false, false, %d>", BM, BN, cfg == 1 ? 2 : 3,
                    epic3 ? 3 : 2);
  else
    adp::set_kernel("igemm_fwd_tap64p_kernel<%d, %d, %d, %s, false, false, false, false, -1>", BM, BN, cfg == 1 ? 2 : 3, bnr ? "true" : "false");
#define P_LAUNCH(BM_, BN_, NST_)                                                                           \
  do {                                                                                                     \
    if (bnr) hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<BM_, BN_, NST_, true>), dim3(grid), dim3(512), 0, s, a); \
    else if (epic3)                                                                                        \
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<BM_, BN_, NST_, false, false, false, false, false, 3>), dim3(grid), \
                         dim3(512), 0, s, a);                                                             \
    else if (epic)                                                                                         \
      hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<BM_, BN_, NST_, false, false, false, false, false, 2>), dim3(grid), \
                         dim3(512), 0, s, a);                                                             \
    else hipLaunchKernelGGL((igemm_fwd_tap64p_kernel<BM_, BN_, NST_, false>), dim3(grid), dim3(512), 0, s, a);   \
  } while (0)
  if (cfg == 1) P_LAUNCH(256, 256, 2);
  else if (cfg == 2) P_LAUNCH(256, 128, 3);
  else P_LAUNCH(128, 256, 3);
#undef P_LAUNCH
  return 1;
}
}  // namespace adp
