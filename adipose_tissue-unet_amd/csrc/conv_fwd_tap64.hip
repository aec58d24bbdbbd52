// Double-buffered LDS-DMA implicit-GEMM forward kernel ("tap64") for every layer whose channel stride is a
// multiple of 64 — all 3x3 convs of the unet_bn preset after the input layer, their data-gradients,
// the ConvTranspose 2x2/s2 forward (1x1 + pixel-shuffle store) and data-gradient (stride-2 4-tap
// gather). Semantics are those of igemm_fwd_kernel (conv_igemm.hip); only the schedule differs.
//
// Because Cin_s % 64 == 0, each 64-deep K step lies inside one tap and one source, so the per-lane
// gather address of a K step is (row base pixel + tap offset) * stride + channel: a bounds test and
// two adds, no per-lane division.
//
// Schedule: a block of WM x WN waves computes BM x BN = (WM*TM) x (WN*64); each wave a TM x 64 tile
// held as (TM/16) x 4 accumulators of v_mfma_f32_16x16x32_bf16. Every K step (64) is staged in four
// quarter-tiles -- A0/A1 (the upper/lower TM/2 rows of every wave row group) and B0/B1 (the left/right
// 32 columns of every wave column group) -- moved HBM/L2 -> LDS by LDS-DMA (buffer_load ... lds) into a
// lane-linear image whose 16-B chunks are XOR-swizzled on the SOURCE address. Two stages: after ONE
// barrier per K step the next step's four quarters are issued into the idle stage, then the current
// stage is multiplied as the quadrants (A0,B0) (A0,B1) (A1,B1) (A1,B0).
//
// F8 (fp8 e4m3 forward, BASELINE configs[4]): the same schedule with 128-channel K steps — a 128-B LDS row
// then holds 128 fp8 instead of 64 bf16, so staging, swizzle and barriers are unchanged — and one
// block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales; 2x the bf16 rate) per fragment pair
// in place of two 16x16x32 bf16 MFMAs. Each lane feeds both operands the same 32 k values (16-B chunks
// h4 and h4+4 of the row: the bf16 read pattern, conflict-free under the swizzle), so the k order inside
// the instruction cancels out of the dot product.
// The per-output-channel weight scale is applied in the epilogue (FwdArgs::wscale).
#include <algorithm>
#include <type_traits>

#include "conv_common.h"

extern "C" int adp_set_option(const char* name, int value);   // (abi.cpp)

namespace {

__device__ __attribute__((aligned(256))) uint4 tap64_zero_page[64];

constexpr int cmax(int x, int y) { return x > y ? x : y; }

// compiler fence + hardware barrier + compiler fence: keeps LDS reads and LDS-DMA issues on their
// side of the barrier (the s_barrier builtin alone does not order memory operations)
#define T64_BAR()                          \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_s_barrier();          \
    asm volatile("" ::: "memory");         \
  } while (0)

// blocks per CU the LDS footprint allows (2 when two double-buffered stages fit in 80 KB)
template <int WM, int WN, int TM>
constexpr int tap64_occ() { return 2 * (WM * TM + WN * 64) * 128 <= 81920 ? 2 : 1; }

// BUF: operands through buffer resources (raw_ptr_buffer_load_lds): a padding tap or a weight row past
// the matrix is an out-of-range 32-bit offset, which the buffer unit reads as zeros, so an issue is a
// few 32-bit VALU ops (no zero page, no 64-bit address arithmetic, no scalar load of a global address
// inside the loop). The flat-address form is kept for tensors of 2 GiB and more.
// BNR: data-gradient launch with the fused BatchNorm-backward reduction epilogue (epi_rows_bnr).
typedef int v8i32 __attribute__((ext_vector_type(8)));
typedef int v4i32 __attribute__((ext_vector_type(4)));

constexpr unsigned T64_OOB = 0x80000000u;   // buffer offset beyond every resource: reads as zeros
constexpr int T64_RSRC3 = 0x00020000;        // raw buffer descriptor word 3 (gfx9: 32-bit data format)

// one 16-B-per-lane LDS-DMA piece through a buffer resource (a device function: the host pass of the
// kernel templates then never sees the target builtin)
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
}

// F32 (the f32 parity path, adipose_v3 / unet_bn at the reference's precision): 32-channel K steps (a 128-B row
// holds 32 floats: staging, swizzle and barriers unchanged); each 16-B fragment is 4 k values of one row, fed to
// four exact v_mfma_f32_16x16x4_f32 (lane group g supplies k = 4g + j to the j-th one: A and B share the
// permutation, so every k of the step enters the dot product once); f32 epilogue stores.
// KP: the K loop compiled in -- -1 either, chosen at run time by a.kpipe (the fp8 / f32 forms); 0 the plain double
// buffer only; 2 the same without the nearest-x2 upsample gather (launches with up == 1, option tap64_up1); 1 the
// mid-step-barrier loop only (bf16 forms: one loop per instance leaves the register allocator
// one schedule, as the persistent kernel's EPIC does for its epilogues); 4-6 (F32, WN == 1, round 5) the plain
// loop with the zero tails ZT = KP - 3 of FwdArgs::ztail skipped (bit 1: WN == 1 only): bit 0 -- every source is a 64-channel stride whose
// weight columns [48, 64) are zeros (44-channel f32 layers), so the upper 16 channels of every odd K step (the
// source's channels 48-63) are neither read from LDS nor multiplied (the loop runs two steps per trip, so the step
// parity is known at compile time); bit 1 -- Nout == 64 with zero weight rows [48, 64): the 16-column MFMA group
// 48-63 is skipped and its accumulators stay 0. The skipped products are exact zeros: the same values.
template <int WM, int WN, int TM, bool BUF, bool BNR, bool F8, bool F32 = false, int KP = -1>
__global__ __launch_bounds__(WM * WN * 64, (tap64_occ<WM, WN, TM>())) void igemm_fwd_tap64_kernel(FwdArgs a) {
  static_assert(!(F8 && F32), "one operand dtype");
  constexpr int ZT = KP >= 4 ? KP - 3 : 0;
  static_assert(ZT == 0 || (F32 && !BNR && (WN == 1 || ZT == 1)), "zero-tail forms: f32; the N tail on 64-column tiles");
  using TO = typename std::conditional<F32, float, bf16>::type;   // output dtype
  constexpr int NTH = WM * WN * 64;
  constexpr int BM = WM * TM, BN = WN * 64;
  constexpr int ROWB = 128;                        // one K step of one row: 64 bf16 / 128 fp8 / 32 f32
  constexpr int ES = F8 ? 1 : (F32 ? 4 : 2);       // bytes per element
  constexpr int KSTEP = ROWB / ES;                 // K elements per step
  constexpr int QA = BM / 2, QB = BN / 2;          // rows per quarter-tile
  constexpr int GA = QA * 8 / NTH, GB = QB * 8 / NTH;  // glds per thread per quarter
  static_assert(GA >= 1 && GB >= 1 && GA * NTH == QA * 8 && GB * NTH == QB * 8, "quarters must split evenly");
  constexpr int HM = TM / 2;                       // rows of a wave's A quarter
  constexpr int MIQ = TM / 32;                     // 16-row fragments per wave per A quarter
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int OA1 = QA * ROWB, OB0 = BM * ROWB, OB1 = (BM + QB) * ROWB;
  constexpr int EPI = TM * (BN + 4) * 4;
  constexpr int SMEM0 = cmax(cmax(2 * STAGE, EPI), NTH * 16 * 4);
  // BNL (BN-backward reduction, bf16, buffer resources): + the per-channel parameters of the LDS-staged epilogue
  constexpr bool BNRL = BNR && BUF && !F32 && !F8;
  constexpr int SMEM = SMEM0 + (BNRL ? 4 * BN * 4 : 0);
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if constexpr (WM * WN == 8) prio_static<ADP_PRIO_T64>(wave);
  // f32 256x128 (as in the persistent kernel): waves w and w + 4 share a SIMD and take the two column halves
  // (wc = w >> 2); a wave skips the MFMAs of a 32-column group wholly past Nout (option f32_skip)
  const bool SPLIT = F32 && WM == 4 && WN == 2 && a.f32_skip;   // (f32_skip = 0: the bf16 forms' wave layout)
  const int wr = SPLIT ? (wave & 3) : wave / WN, wc = SPLIT ? (wave >> 2) : wave % WN;
  // split-K (FwdArgs::ksplit): block -> (tile, K range); the ranges are contiguous runs of K steps
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  const int lin0 = xcd_remap(blockIdx.x, a.nblocks);
  const int ksid = lin0 % nsplit, lin = lin0 / nsplit;
  const int tn = lin % a.ntile_n, tm = lin / a.ntile_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wcu = SPLIT ? (__builtin_amdgcn_readfirstlane(wave) >> 2) : 0;
  const bool skip0 = SPLIT && n0 + wcu * 64 >= a.Nout;        // (block- and wave-uniform)
  const bool skip1 = SPLIT && n0 + wcu * 64 + 32 >= a.Nout;
  const int pos = lane & 7;
  const int upv = KP == 2 ? 1 : a.up;   // (KP 2: up == 1 at compile time)
  const int HWo = a.Ho * a.Wo, Hv = a.Hs * upv, Wv = a.Ws * upv;
  const int Cin_s = a.CAs + a.CBs;
  const int Wrows = (a.Nout + 63) / 64 * 64;
  const int nk_all = a.K / KSTEP;
  const int kb = (int)((long long)ksid * nk_all / nsplit);
  const int nk = (int)((long long)(ksid + 1) * nk_all / nsplit) - kb;

  // ---- per-thread staging rows: quarter h, instruction i -> quarter row q = i*(NTH/8) + tid/8
  int ry[2][GA], rx[2][GA], rn[2][GA], rc[2][GA], pb[2][GA];   // pb: pixel of tap (0,0) (up == 1)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int q = i * (NTH / 8) + (tid >> 3);
      const int m = m0 + (q / HM) * TM + h * HM + (q % HM);
      const bool v = m < a.M;
      const int mm = v ? m : 0;
      const int n = mm / HWo, rem = mm - n * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
      ry[h][i] = yo * a.stride - a.pad;
      rx[h][i] = xo * a.stride - a.pad;
      rn[h][i] = v ? n * a.Hs : -1;
      pb[h][i] = (n * a.Hs + ry[h][i]) * a.Ws + rx[h][i];
      rc[h][i] = 16 * (pos ^ swz(q));   // byte offset of this lane's 16-B chunk
    }
  const unsigned char* bp[2][GB];
  unsigned bo[2][GB];   // BUF: byte offset of this lane's weight chunk (T64_OOB past the matrix)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int q = i * (NTH / 8) + (tid >> 3);
      const int col = (q / 32) * 64 + h * 32 + (q % 32);
      const bool v = n0 + col < Wrows;
      bo[h][i] = v ? (unsigned)((n0 + col) * a.Kpad * ES + 16 * (pos ^ swz(q))) : T64_OOB;
      bp[h][i] = v ? reinterpret_cast<const unsigned char*>(a.W) + ((size_t)(n0 + col) * a.Kpad) * ES +
                         16 * (pos ^ swz(q))
                   : nullptr;
    }
  const unsigned char* srcA = reinterpret_cast<const unsigned char*>(a.srcA);
  const unsigned char* srcB = reinterpret_cast<const unsigned char*>(a.srcB);
  const int npix = a.Nimg * a.Hs * a.Ws;   // (only the BUF instantiations use the resources)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.srcA, 0, npix * a.CAs * ES, T64_RSRC3);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.CBs ? a.srcB : a.srcA), 0, npix * (a.CBs ? a.CBs : a.CAs) * ES, T64_RSRC3);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, Wrows * a.Kpad * ES, T64_RSRC3);

  // K step -> (tap offsets, source, channel); uniform across the block, advanced incrementally (K steps
  // run channel-chunk-fastest inside a tap, taps row-major). cs = pixel stride in bytes, cb = byte offset
  // of the step's first channel inside its source's pixel, dpix = pixel delta of the tap (up == 1).
  struct Kt { int oy, ox, cs, cb, srcb, dpix, kt; const unsigned char* base; };
  // iterator state: the NEXT step kinfo() returns (split-K: the block's first step kb)
  const int spt = Cin_s / KSTEP;
  int it_ci = (kb % spt) * KSTEP, it_ty = (kb / spt) / a.kw, it_tx = (kb / spt) % a.kw, it_kt = kb;
  auto kinfo = [&]() {
    Kt r;
    r.oy = it_ty * a.dil; r.ox = it_tx * a.dil; r.kt = it_kt;
    r.dpix = r.oy * a.Ws + r.ox;
    if (it_ci < a.CAs) { r.cb = it_ci * ES; r.cs = a.CAs * ES; r.srcb = 0; r.base = srcA + r.cb; }
    else { r.cb = (it_ci - a.CAs) * ES; r.cs = a.CBs * ES; r.srcb = 1; r.base = srcB + r.cb; }
    ++it_kt;
    it_ci += KSTEP;
    if (it_ci >= Cin_s) {
      it_ci = 0;
      if (++it_tx == a.kw) { it_tx = 0; ++it_ty; }
    }
    return r;
  };
  auto issueA = [&](int h, const Kt& k, int buf) {
    unsigned char* dst = smem + buf * STAGE + h * OA1 + wave * 8 * ROWB;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      int yi = ry[h][i] + k.oy, xi = rx[h][i] + k.ox;
      const bool v = rn[h][i] >= 0 && (unsigned)yi < (unsigned)Hv && (unsigned)xi < (unsigned)Wv;
      int pix;
      if (upv == 2) pix = (rn[h][i] + (yi >> 1)) * a.Ws + (xi >> 1);
      else pix = pb[h][i] + k.dpix;
      if constexpr (BUF) {
        const unsigned off = v ? (unsigned)(pix * k.cs + k.cb + rc[h][i]) : T64_OOB;
        buf_lds16(k.srcb ? rsB : rsA, dst + i * (NTH / 8) * ROWB, off);
      } else {
        const void* p = v ? (const void*)(k.base + (size_t)pix * k.cs + rc[h][i]) : (const void*)tap64_zero_page;
        __builtin_amdgcn_global_load_lds(p, (lds_void*)(dst + i * (NTH / 8) * ROWB), 16, 0, 0);
      }
    }
  };
  auto issueB = [&](int h, const Kt& k, int buf) {
    unsigned char* dst = smem + buf * STAGE + (h ? OB1 : OB0) + wave * 8 * ROWB;
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      if constexpr (BUF) {
        const unsigned off = bo[h][i] == T64_OOB ? T64_OOB : bo[h][i] + (unsigned)k.kt * ROWB;
        buf_lds16(rsW, dst + i * (NTH / 8) * ROWB, off);
      } else {
        const void* p = bp[h][i] ? (const void*)(bp[h][i] + (size_t)k.kt * ROWB) : (const void*)tap64_zero_page;
        __builtin_amdgcn_global_load_lds(p, (lds_void*)(dst + i * (NTH / 8) * ROWB), 16, 0, 0);
      }
    }
  };

  const int r16 = lane & 15, h4 = lane >> 4;
  auto readA = [&](int buf, int h, bf16x8 (&fa)[MIQ][2], bool ktail = false) {
    const unsigned char* base = smem + buf * STAGE + h * OA1;
#pragma unroll
    for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if ((ZT & 1) && ktail && s == 1) continue;
        const int q = wr * HM + mi * 16 + r16, c = 4 * s + h4;
        fa[mi][s] = *reinterpret_cast<const bf16x8*>(base + q * ROWB + ((c ^ swz(q)) << 4));
      }
  };
  auto readB = [&](int buf, int h, bf16x8 (&fb)[2][2]) {
    const unsigned char* base = smem + buf * STAGE + (h ? OB1 : OB0);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if ((ZT & 2) && h == 1 && ni == 1) continue;
        const int q = wc * 32 + ni * 16 + r16, c = 4 * s + h4;
        fb[ni][s] = *reinterpret_cast<const bf16x8*>(base + q * ROWB + ((c ^ swz(q)) << 4));
      }
  };

  f32x4 acc[2 * MIQ][4];
#pragma unroll
  for (int i = 0; i < 2 * MIQ; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8 (&fa)[MIQ][2], const bf16x8 (&fb)[2][2], int ha, int hb, bool ktail = false) {
    if constexpr (F32)
      if (hb ? skip1 : skip0) return;
    prio_hi<ADP_PRIO_T64>();
    if constexpr (F8) {
#pragma unroll
      for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[ha * MIQ + mi][hb * 2 + ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              __builtin_bit_cast(v8i32, fa[mi]), __builtin_bit_cast(v8i32, fb[ni]), acc[ha * MIQ + mi][hb * 2 + ni],
              0, 0, 0, 127, 0, 127);
    } else if constexpr (F32) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            if ((ZT & 1) && ktail && s == 1) continue;
            if ((ZT & 2) && hb == 1 && ni == 1) continue;
            const f32x4 av = __builtin_bit_cast(f32x4, fa[mi][s]), bv = __builtin_bit_cast(f32x4, fb[ni][s]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[ha * MIQ + mi][hb * 2 + ni] =
                  __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc[ha * MIQ + mi][hb * 2 + ni], 0, 0, 0);
          }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[ha * MIQ + mi][hb * 2 + ni] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mi][s], fb[ni][s], acc[ha * MIQ + mi][hb * 2 + ni], 0, 0, 0);
    }
    prio_lo<ADP_PRIO_T64>();
  };

  bf16x8 fa[MIQ][2], fb0[2][2], fb1[2][2];
  // double buffering, ONE barrier per K step: stage t+1 is filled while stage t multiplies (the earlier
  // schedules -- a 4-barrier quarter refill with step t+2, issues interleaved with the MFMA clusters, and
  // the guide's two-barrier ping-pong -- measured 6-20 % slower on these shapes: DESIGN.md §3)
  {
    const Kt k0 = kinfo();
    issueA(0, k0, 0); issueB(0, k0, 0); issueB(1, k0, 0); issueA(1, k0, 0);
  }
  // staggered issue (option tap64p_stagger, shared with the persistent kernel): the waves on the second
  // half of the SIMDs (waves w and w + NW/2 share one) issue their LDS-DMA pieces after their first MFMA
  // cluster, so one wave of each SIMD multiplies while the other issues
  constexpr int NW = WM * WN;
  const bool late = a.stagger && NW == 8 && ((__builtin_amdgcn_readfirstlane(wave) >> 2) & 1);
  // KPIPE (option tap64_kpipe): the step's barrier sits in the middle of the previous step. After its third
  // MFMA cluster a wave has read all of stage t it will read (B half 0 was preloaded), so there it waits for
  // stage t + 1 (issued one step earlier), passes the barrier while that cluster's MFMAs run, refills stage t
  // with step t + 2, issues the fourth cluster and preloads stage t + 1's B half 0 behind it. The same
  // fragments and MFMA order: bit-identical.
  const bool kp = KP == 1 || (KP < 0 && a.kpipe);
  if (kp) {
    auto issue_step = [&](int b_) {
      const Kt kk = kinfo();
      issueA(0, kk, b_); issueB(0, kk, b_); issueB(1, kk, b_); issueA(1, kk, b_);
    };
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    T64_BAR();   // stage 0 landed for every wave
    if (nk > 1) issue_step(1);
    readB(0, 0, fb0);
    for (int t = 0; t < nk; ++t) {
      const int buf = t & 1;
      readA(buf, 0, fa);
      mma(fa, fb0, 0, 0);
      readB(buf, 1, fb1);
      mma(fa, fb1, 0, 1);
      readA(buf, 1, fa);
      mma(fa, fb1, 1, 1);
      if (t + 1 < nk) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (only step t + 1 is in flight)
        T64_BAR();   // stage t read by every wave; stage t + 1 landed
        if (!late && t + 2 < nk) issue_step(buf);
      }
      mma(fa, fb0, 1, 0);
      if (t + 1 < nk) {
        readB(buf ^ 1, 0, fb0);
        if (late && t + 2 < nk) issue_step(buf);
      }
    }
  } else if constexpr (ZT != 0) {
    // (the plain loop below, two K steps per trip: the second is the odd one; nk is even, the launcher checks)
    auto step = [&](int t, auto odd) {
      constexpr bool kt = decltype(odd)::value && (ZT & 1);
      const int buf = t & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      T64_BAR();
      auto issue_next = [&]() {
        if (t + 1 < nk) {
          const Kt k1 = kinfo();
          issueA(0, k1, buf ^ 1); issueB(0, k1, buf ^ 1); issueB(1, k1, buf ^ 1); issueA(1, k1, buf ^ 1);
        }
      };
      if (!late) issue_next();
      readA(buf, 0, fa, kt);
      readB(buf, 0, fb0);
      mma(fa, fb0, 0, 0, kt);
      if (late) issue_next();
      readB(buf, 1, fb1);
      mma(fa, fb1, 0, 1, kt);
      readA(buf, 1, fa, kt);
      mma(fa, fb1, 1, 1, kt);
      mma(fa, fb0, 1, 0, kt);
    };
    int t = 0;
    for (; t + 1 < nk; t += 2) {
      step(t, std::false_type{});
      step(t + 1, std::true_type{});
    }
    if (t < nk) step(t, std::false_type{});   // (an odd nk: bit 1 only)
  } else
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    T64_BAR();   // stage t landed for every wave, and nobody reads buffer buf ^ 1 any more
    auto issue_next = [&]() {
      if (t + 1 < nk) {
        const Kt k1 = kinfo();
        issueA(0, k1, buf ^ 1); issueB(0, k1, buf ^ 1); issueB(1, k1, buf ^ 1); issueA(1, k1, buf ^ 1);
      }
    };
    if (!late) issue_next();
    readA(buf, 0, fa);
    readB(buf, 0, fb0);
    mma(fa, fb0, 0, 0);
    if (late) issue_next();
    readB(buf, 1, fb1);
    mma(fa, fb1, 0, 1);
    readA(buf, 1, fa);
    mma(fa, fb1, 1, 1);
    mma(fa, fb0, 1, 0);
  }
  T64_BAR();   // the epilogue reuses the stages

  if (nsplit > 1) {
    // split-K: this K range's accumulators to the tile's partial slab (accumulator i of thread t of split k at
    // [(k NACC + i) NTH + t]: coalesced 16-B stores), then the tile's counter; the last of its nsplit blocks re-zeroes
    // the counter, reads every split's partial in split order (its own too: the sum's order does not depend on which
    // block came last) and runs the epilogue below. Release / acquire at agent scope: the blocks sit on any XCD.
    constexpr int NACC = 2 * MIQ * 4;
    float4* part = reinterpret_cast<float4*>(a.kpart) + (size_t)lin * nsplit * NACC * NTH;
#pragma unroll
    for (int i = 0; i < 2 * MIQ; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = acc[i][j];
        part[(size_t)(ksid * NACC + i * 4 + j) * NTH + tid] = make_float4(v[0], v[1], v[2], v[3]);
      }
    __syncthreads();   // (every wave's stores complete: its vmcnt is drained by the barrier's fence)
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(a.kcnt + lin, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == nsplit - 1;
      if (last) __hip_atomic_store(a.kcnt + lin, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    const int last = flag[0];
    __syncthreads();   // (the flag is read before the epilogue reuses the LDS)
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
    for (int i = 0; i < 2 * MIQ; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 sum = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < nsplit; ++k) {
          const float4 v = part[(size_t)(k * NACC + i * 4 + j) * NTH + tid];
          if (k == 0) sum = f32x4{v.x, v.y, v.z, v.w};
          else sum += f32x4{v.x, v.y, v.z, v.w};
        }
        acc[i][j] = sum;
      }
  }

  if (ADP_DBG(a) & 16) {   // timing-only ablation (option fwd_debug bit 4): no epilogue at all
#pragma unroll
    for (int i = 0; i < 2 * MIQ; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  // ---- BN-backward-reduction epilogue through LDS only (option tap64_bnr_lds, round 5): per wave row group the z rows
  // come in by LDS-DMA while the group's accumulators are staged as bf16 (the values the launch stores, rounded once as
  // grp_from_f rounds them), and the row loop reads dA, z and the per-channel parameters from LDS: no row waits on a
  // global load (epi_rows_bnr issues each row's z load behind that row's store; at level 2 the z reads were two thirds
  // of an epilogue that took 29 % of the launch). Same values and sums, same order: bit-identical.
  if constexpr (BNRL) {
    if (a.bnr_lds && !a.addend && !a.mask) {
      constexpr int LTB = BN + 8;                         // bf16 per staged row (+16 B: rows start on other banks)
      constexpr int ZOFF = TM * LTB * 2;                  // z rows of the group: 16-B chunks, row-major
      constexpr int GPR = BN / 8, RSTEP = NTH / GPR;
      constexpr int ZCH = TM * GPR, GZ = ZCH / NTH;
      static_assert(ZOFF + TM * BN * 2 <= SMEM0 && GZ * NTH == ZCH, "LDS-staged BNR epilogue layout");
      bf16* t16 = reinterpret_cast<bf16*>(smem);
      float* prm = reinterpret_cast<float*>(smem + SMEM0);   // scale | shift | mean | invstd, BN each
      if (tid < BN) {
        const int c = n0 + tid;
        const bool v = c < a.Nout;
        prm[tid] = v ? a.bnr_sc[c] : 0.f;
        prm[BN + tid] = v ? a.bnr_sh[c] : 0.f;
        prm[2 * BN + tid] = v ? a.bnr_mean[c] : 0.f;
        prm[3 * BN + tid] = v ? a.bnr_invstd[c] : 0.f;
      }
      const __amdgpu_buffer_rsrc_t rsZ =
          __builtin_amdgcn_make_buffer_rsrc((void*)a.bnr_z, 0, a.M * a.bnr_zs * 2, T64_RSRC3);
      const int col = lane & 15, rq = (lane >> 4) * 4;
      const int cg = tid % GPR, n = n0 + cg * 8;
      float bs[8], bq[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { bs[j] = 0.f; bq[j] = 0.f; }
      for (int p = 0; p < WM; ++p) {
        const int mb = m0 + p * TM;
#pragma unroll
        for (int i = 0; i < GZ; ++i) {
          const int idx = i * NTH + tid, row = idx / GPR, cc = idx - row * GPR, m = mb + row;
          const unsigned off =
              m < a.M && n0 + cc * 8 < a.Nout ? (unsigned)(((size_t)m * a.bnr_zs + n0 + cc * 8) * 2) : T64_OOB;
          buf_lds16(rsZ, smem + ZOFF + (size_t)(i * NTH + wave * 64) * 16, off);
        }
        if (wr == p) {
#pragma unroll
          for (int mt = 0; mt < 2 * MIQ; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                t16[((mt / MIQ) * HM + (mt % MIQ) * 16 + rq + r) * LTB + wc * 64 + nt * 16 + col] = (bf16)acc[mt][nt][r];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's z chunks landed
        ADP_LDS_BARRIER();                                  // every thread's, and the staging
        if (n < a.Nout) {
          for (int row = tid / GPR; row < TM; row += RSTEP) {
            const int m = mb + row;
            if (m >= a.M) break;
            Grp<bf16> gd, gz;
            gd.v = *reinterpret_cast<const uint4*>(t16 + row * LTB + cg * 8);
            gz.v = *reinterpret_cast<const uint4*>(smem + ZOFF + (size_t)(row * GPR + cg) * 16);
            grp_store(gd, reinterpret_cast<bf16*>(a.out) + (size_t)m * a.out_stride + n);
            float v[8], f[8];
            grp_to_f(gd, v);
            grp_to_f(gz, f);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float4 sc = *reinterpret_cast<const float4*>(prm + cg * 8 + 4 * h);
              const float4 sh = *reinterpret_cast<const float4*>(prm + BN + cg * 8 + 4 * h);
              const float4 mu = *reinterpret_cast<const float4*>(prm + 2 * BN + cg * 8 + 4 * h);
              const float4 is = *reinterpret_cast<const float4*>(prm + 3 * BN + cg * 8 + 4 * h);
              const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
              const float muv[4] = {mu.x, mu.y, mu.z, mu.w}, isv[4] = {is.x, is.y, is.z, is.w};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int jj = 4 * h + j;
                const float db = fmaf(f[jj], scv[j], shv[j]) > 0.f ? v[jj] : 0.f;
                bs[jj] += db;
                bq[jj] += db * (f[jj] - muv[j]) * isv[j];
              }
            }
          }
        }
        ADP_LDS_BARRIER();   // the group's rows are read out: the next group's DMA and staging may overwrite them
      }
      epi_bn_flush<NTH, BN>(a, reinterpret_cast<float*>(smem), n0, tid, bs, bq);
      return;
    }
  }
  // ---- mask / addend epilogue through LDS (option tap64_mask_lds, round 5: the adipose_v3 data gradients). Per half
  // row group the mask and addend rows come in by LDS-DMA while the half's f32 accumulators are staged, so no row
  // waits on a global load (epi_rows loads each row's addend and mask behind that row's store: at level 2 of the bf16
  // adipose_v3 step that epilogue was 36 % of the launch, profiles/r05_mask_epi_probe.log). Plain stores with bias,
  // addend, mask and BatchNorm statistics only (the host checks); epi_rows' arithmetic in its order: bit-identical.
  {
    constexpr int ESZ = F32 ? 4 : 2;
    constexpr int H2 = TM / 2;
    constexpr int MOFF = H2 * (BN + 4) * 4;            // f32 staging of half a row group, then the mask and addend rows
    constexpr int AOFF = MOFF + H2 * BN * ESZ;
    constexpr int CPR = BN * ESZ / 16;                 // 16-B chunks per row
    constexpr bool MAL = BUF && !F8 && !BNR && AOFF + H2 * BN * ESZ <= SMEM0 && (H2 * CPR) % NTH == 0;
    if constexpr (MAL) {
      if (a.mask_lds && (a.mask || a.addend)) {
        constexpr int GQ = H2 * CPR / NTH, GPR = BN / 8, RSTEP = NTH / GPR, LT = BN + 4;
        float* st = reinterpret_cast<float*>(smem);
        const TO* mk = reinterpret_cast<const TO*>(smem + MOFF);
        const TO* ad = reinterpret_cast<const TO*>(smem + AOFF);
        const __amdgpu_buffer_rsrc_t rsM = __builtin_amdgcn_make_buffer_rsrc(
            (void*)a.mask, 0, a.mask ? a.M * a.mask_stride * ESZ : 0, T64_RSRC3);
        const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc(
            (void*)a.addend, 0, a.addend ? a.M * a.addend_stride * ESZ : 0, T64_RSRC3);
        const int col = lane & 15, rq = (lane >> 4) * 4;
        const int cg = tid % GPR, n = n0 + cg * 8;
        float bias[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) bias[j] = a.bias && n + j < a.Nout ? a.bias[n + j] : 0.f;
        float bs[8], bq[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { bs[j] = 0.f; bq[j] = 0.f; }
        for (int p = 0; p < WM; ++p) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int mb = m0 + p * TM + h * H2;
#pragma unroll
            for (int i = 0; i < GQ; ++i) {
              const int idx = i * NTH + tid, row = idx / CPR, cq = idx - row * CPR, m = mb + row;
              const int c = n0 + cq * (16 / ESZ);
              const bool ok = m < a.M && c < a.Nout;
              const size_t lo = (size_t)(i * NTH + wave * 64) * 16;
              if (a.mask) buf_lds16(rsM, smem + MOFF + lo, ok ? (unsigned)(((size_t)m * a.mask_stride + c) * ESZ) : T64_OOB);
              if (a.addend)
                buf_lds16(rsD, smem + AOFF + lo, ok ? (unsigned)(((size_t)m * a.addend_stride + c) * ESZ) : T64_OOB);
            }
            if (wr == p) {
#pragma unroll
              for (int mi = 0; mi < MIQ; ++mi)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                  for (int r = 0; r < 4; ++r)
                    st[(mi * 16 + rq + r) * LT + wc * 64 + nt * 16 + col] = acc[h * MIQ + mi][nt][r];
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's mask / addend chunks landed
            ADP_LDS_BARRIER();
            if (n < a.Nout) {
              for (int row = tid / GPR; row < H2; row += RSTEP) {
                const int m = mb + row;
                if (m >= a.M) break;
                float v[8], f[8];
                const float4* tp = reinterpret_cast<const float4*>(st + row * LT + cg * 8);
                const float4 t0 = tp[0], t1 = tp[1];
                v[0] = t0.x; v[1] = t0.y; v[2] = t0.z; v[3] = t0.w; v[4] = t1.x; v[5] = t1.y; v[6] = t1.z; v[7] = t1.w;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] += bias[j];
                Grp<TO> gr;
                if (a.addend) {
                  grp_load(gr, ad + row * BN + cg * 8);
                  grp_to_f(gr, f);
#pragma unroll
                  for (int j = 0; j < 8; ++j) v[j] += f[j];
                }
                if (a.mask) {
                  grp_load(gr, mk + row * BN + cg * 8);
                  grp_to_f(gr, f);
#pragma unroll
                  for (int j = 0; j < 8; ++j) v[j] = f[j] > 0.f ? v[j] * a.mask_scale : 0.f;
                }
                grp_from_f(gr, v);
                grp_store(gr, reinterpret_cast<TO*>(a.out) + (size_t)m * a.out_stride + n);
                if (a.bn_sum) {
#pragma unroll
                  for (int j = 0; j < 8; ++j) { bs[j] += v[j]; bq[j] += v[j] * v[j]; }
                }
              }
            }
            ADP_LDS_BARRIER();   // the half is read out: the next half's DMA and staging may overwrite it
          }
        }
        if (a.bn_sum) epi_bn_flush<NTH, BN>(a, reinterpret_cast<float*>(smem), n0, tid, bs, bq);
        return;
      }
    }
  }
  // ---- epilogue: one wave row group (TM rows x BN) at a time through LDS
  float* tile = reinterpret_cast<float*>(smem);
  constexpr int LT = BN + 4;
  const int col = lane & 15, rq = (lane >> 4) * 4;
  float bs[8], bq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bs[j] = 0.f; bq[j] = 0.f; }
  for (int p = 0; p < WM; ++p) {
    if (wr == p) {
#pragma unroll
      for (int mt = 0; mt < 2 * MIQ; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            tile[((mt / MIQ) * HM + (mt % MIQ) * 16 + rq + r) * LT + wc * 64 + nt * 16 + col] = acc[mt][nt][r];
    }
    ADP_LDS_BARRIER();
    if constexpr (BNR) epi_rows_bnr<NTH, BN, TO>(a, tile, TM, m0 + p * TM, n0, tid, bs, bq);
    else epi_rows<NTH, BN, F8, TO>(a, tile, TM, m0 + p * TM, n0, tid, bs, bq);
    ADP_LDS_BARRIER();
  }
  if (a.bn_sum || a.bnr_z) epi_bn_flush<NTH, BN>(a, tile, n0, tid, bs, bq);
}

#undef T64_BAR

template <int WM, int WN, int TM>
void launch_cfg(FwdArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM, BN = WN * 64;
  a.ntile_n = (a.Nout + BN - 1) / BN;
  a.nblocks = ((a.M + BM - 1) / BM) * a.ntile_n;
  // split-K (round 6, option tap64_ksplit): a launch whose tiles occupy at most tap64_ksplit_max
  // (192) of the chip's 256 (occupancy 1) or 512 (occupancy 2) block slots -- the f32 path's 32^2 level at BASELINE
  // configs[0]: 48 tiles -- gets up to 8 blocks per tile, each at least 6 K steps; not the zero-tail forms (their loop
  // runs K steps in pairs) or the mid-step-barrier loop
  a.ksplit = 0;
  {
    const int tiles = a.nblocks, nk = a.K / (a.f8 ? 128 : (a.f32 ? 32 : 64));
    const int occ = tap64_occ<WM, WN, TM>();
    if (adp::option("tap64_ksplit", 1) && tiles <= adp::CLAIM_INTS &&
        tiles * occ <= adp::option("tap64_ksplit_max", 192) && !(a.f32 && a.ztail)) {
      const int sp = std::min(std::min(8, (256 * occ) / tiles), nk / 6);
      if (sp >= 2) {
        int* cnt = adp::claim_slot();
        float* part = static_cast<float*>(adp::scratch(7, (size_t)tiles * sp * BM * BN * sizeof(float)));
        if (cnt && part) {
          a.ksplit = sp;
          a.kcnt = cnt;
          a.kpart = part;
          a.kpipe = 0;
          a.nblocks = tiles * sp;
        }
      }
    }
  }
  ::adp_set_option("tap64_ksplit_last", a.ksplit);   // (test hook, adp_get_option)
  const dim3 g(a.nblocks), b(WM * WN * 64);
  // buffer-resource loads need every operand below 2 GiB (32-bit offsets, T64_OOB reserved)
  const int es = a.f8 ? 1 : (a.f32 ? 4 : 2);
  const size_t pix = (size_t)a.Nimg * a.Hs * a.Ws, lim = (size_t)1 << 31;
  const bool buf = adp::option("tap64_buf", 1) && pix * a.CAs * es < lim && pix * a.CBs * es < lim &&
                   (size_t)((a.Nout + 63) / 64 * 64) * a.Kpad * es < lim;
#define T64_LAUNCH(BUFV, BNRV, F8V)                                                                     \
  do {                                                                                                 \
    adp::set_kernel("igemm_fwd_tap64_kernel<%d, %d, %d, %s, %s, %s, false, -1>", WM, WN, TM,            \
                    BUFV ? "true" : "false", BNRV ? "true" : "false", F8V ? "true" : "false");         \
    hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, BUFV, BNRV, F8V>), g, b, 0, s, a);           \
  } while (0)
#define T64_LAUNCH16(BUFV, BNRV)                                                                        \
  do {                                                                                                 \
    if (a.kpipe) {                                                                                     \
      adp::set_kernel("igemm_fwd_tap64_kernel<%d, %d, %d, %s, %s, false, false, 1>", WM, WN, TM,        \
                      BUFV ? "true" : "false", BNRV ? "true" : "false");                               \
      hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, BUFV, BNRV, false, false, 1>), g, b, 0, s, a); \
    } else if (a.up == 1 && adp::option("tap64_up1", 1)) {                                             \
      adp::set_kernel("igemm_fwd_tap64_kernel<%d, %d, %d, %s, %s, false, false, 2>", WM, WN, TM,        \
                      BUFV ? "true" : "false", BNRV ? "true" : "false");                               \
      hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, BUFV, BNRV, false, false, 2>), g, b, 0, s, a); \
    } else {                                                                                           \
      adp::set_kernel("igemm_fwd_tap64_kernel<%d, %d, %d, %s, %s, false, false, 0>", WM, WN, TM,        \
                      BUFV ? "true" : "false", BNRV ? "true" : "false");                               \
      hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, BUFV, BNRV, false, false, 0>), g, b, 0, s, a); \
    }                                                                                                  \
  } while (0)
#define T64_LAUNCH32(BUFV, BNRV)                                                                        \
  do {                                                                                                 \
    adp::set_kernel("igemm_fwd_tap64_kernel<%d, %d, %d, %s, %s, false, true, -1>", WM, WN, TM,          \
                    BUFV ? "true" : "false", BNRV ? "true" : "false");                                 \
    hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, BUFV, BNRV, false, true>), g, b, 0, s, a);   \
  } while (0)
  if (a.f32) {
    // zero tails (FwdArgs::ztail, option f32_ztail): the KP 4-6 instances of the 64-column tile, KP 4 (K tail) of
    // the 256x128 one
    if constexpr ((WN == 1 || WN == 2) && TM == 64) {
      const int zt = adp::option("f32_ztail", 1) && buf && !a.bnr_z && !a.kpipe ? a.ztail & (WN == 1 ? 3 : 1) : 0;
      if constexpr (WN == 2) {
        if (zt) {
          adp::set_kernel("igemm_fwd_tap64_kernel<%d, %d, %d, true, false, false, true, 4>", WM, WN, TM);
          hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, true, false, false, true, 4>), g, b, 0, s, a);
          return;
        }
      } else if (zt) {
        adp::set_kernel("igemm_fwd_tap64_kernel<%d, %d, %d, true, false, false, true, %d>", WM, WN, TM, zt + 3);
        if (zt == 1) hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, true, false, false, true, 4>), g, b, 0, s, a);
        else if (zt == 2) hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, true, false, false, true, 5>), g, b, 0, s, a);
        else hipLaunchKernelGGL((igemm_fwd_tap64_kernel<WM, WN, TM, true, false, false, true, 6>), g, b, 0, s, a);
        return;
      }
    }
    if (a.bnr_z) {
      if (buf) T64_LAUNCH32(true, true);
      else T64_LAUNCH32(false, true);
    } else {
      if (buf) T64_LAUNCH32(true, false);
      else T64_LAUNCH32(false, false);
    }
    return;
  }
  if constexpr (TM == 64) {   // fp8: the 64-row-per-wave tiles only (the 128-row ones spill in the K loop)
    if (a.f8) {               // inference launches: no BN-backward epilogue
      if (buf) T64_LAUNCH(true, false, true);
      else T64_LAUNCH(false, false, true);
      return;
    }
  }
  if (a.bnr_z) {
    if (buf) T64_LAUNCH16(true, true);
    else T64_LAUNCH16(false, true);
  } else {
    if (buf) T64_LAUNCH16(true, false);
    else T64_LAUNCH16(false, false);
  }
#undef T64_LAUNCH
#undef T64_LAUNCH16
#undef T64_LAUNCH32
}

// configurations: 0 = 256x256 (8 waves, 128x64 per wave), 1 = 256x128 (8 waves, 64x64),
// 2 = 512x64 (4 waves, 128x64), 3 = 256x64 (4 waves, 64x64, two blocks per CU)
constexpr int CFG_BM[4] = {256, 256, 512, 256};
constexpr int CFG_BN[4] = {256, 128, 64, 64};
// relative per-block throughput, measured on the unet_bn layer shapes (tools/bench_kernels.py):
// 256x256 > 256x128 > 256x64 (two blocks per CU; the only one used at N = 64, +21-26 % over the
// 4-wave kernel of conv_igemm.hip) ; 512x64 (one wave per SIMD) is never picked.
constexpr double CFG_EFF[4] = {1.0, 0.85, 0.0, 0.6};
// f32 (option f32_eff = 1): the f32 tiles spend 4x the MFMA time per K step, so the 256x64 tile's second
// block per CU buys less than in bf16: 256x128 ran 123 TF per used column against 109 TF for 256x64 on the
// adipose_v3 1024^2 step (profiles/r04c_f32_1024_bench.log: 92.7 TF at 3/4 column use, 109.3 TF at full use)
constexpr double CFG_EFF_F32[4] = {0.0, 1.13, 0.0, 1.0};

}  // namespace

namespace adp {
int launch_fwd_tap64(FwdArgs& a, hipStream_t s) {
  a.stagger = option("tap64p_stagger", 1);
  a.f32_skip = option("f32_skip", 1);
  int mode = option("fwd_tap64", 1);   // 0 off, 1 auto, 2+c force configuration c
  if (mode == 0) return 0;
  // the fused BN-backward epilogue handles plain stores only (what the data-gradient launches use)
  if (a.bnr_z && (a.out_mode != 0 || a.bias || a.relu || a.drop_rate > 0.f || a.accum || a.bn_sum)) return 0;
  const int Cin_s = a.CAs + a.CBs;
  const int ks = a.f8 ? 128 : (a.f32 ? 32 : 64);   // channels per K step (one 128-B LDS row)
  if (a.scA || a.scB || a.CAs % ks != 0 || a.CBs % ks != 0 || a.K != a.kh * a.kw * Cin_s || a.K % ks != 0 ||
      a.Kpad != a.K)
    return 0;
  int cfg = mode - 2;
  // fp8: the persistent halo forms first (256x256 when a 256-wide N tile is at least 3/4 used, else 256x128)
  if (a.f32 && !option("f32_tap", 1)) return 0;
  if (a.f8 && (mode == 1 || cfg == 0 || cfg == 1)) {
    const int t = mode == 1 ? ((a.Nout % 256 == 0 || (a.Nout > 256 && a.Nout % 256 >= 192)) ? 0 : 1) : cfg;
    if (launch_fwd_tap64p(a, s, t)) return 1;
  }
  if (a.f8 && cfg != 1 && cfg != 3) mode = 1;
  if (mode == 1) {
    // score = column utilisation x last-wave utilisation of the 256-CU grid x per-block efficiency
    // a configuration whose N tile is less than 3/4 used is not considered
    double best = 0.0;
    const int f32_eff = a.f32 ? option("f32_eff", 1) : 0;
    const double* eff = f32_eff ? CFG_EFF_F32 : CFG_EFF;
    for (int c = 0; c < 4; ++c) {
      if (a.f8 && CFG_BM[c] * CFG_BN[c] > 256 * 128) continue;   // fp8: 256x128 / 256x64 tiles
      if (a.f32 && c == 0) continue;   // f32: the 256x256 tile spills in its f32 epilogue; 256x128 keeps 156 VGPRs
      const long long tn = (a.Nout + CFG_BN[c] - 1) / CFG_BN[c], tmm = (a.M + CFG_BM[c] - 1) / CFG_BM[c];
      // resident blocks per wave of the grid: 256 CUs x 1 (f32_eff = 2: x 2 for the 256x64 tile, whose LDS
      // (2 x 40 KB) and 4 waves leave room for a second block per CU -- the last-wave fill of the few-tile f32
      // launches, e.g. 128^2 x 352 channels: 384 / 768 blocks)
      const long long slots = (f32_eff >= 2 && c == 3) ? 512 : 256;
      const long long blocks = tn * tmm, waves = (blocks + slots - 1) / slots;
      const double colu = (double)a.Nout / (tn * CFG_BN[c]);
      if (colu < 0.75) continue;
      const double sc = colu * (double)blocks / (waves * slots) * eff[c];
      if (sc > best) { best = sc; cfg = c; }
    }
    if (best <= 0.0) return 0;
  }
  // the persistent kernel for the 256x256 and 256x128 tiles (BNR launches: option tap64p_bnr)
  if ((cfg == 0 || cfg == 1) && !a.f8 && !a.f32 && (!a.bnr_z || option("tap64p_bnr", 1)) && launch_fwd_tap64p(a, s, cfg))
    return 1;
  // f32: the persistent halo form for the 256x128 choice (3x3 stride-1 layers; falls through otherwise)
  if (cfg == 1 && a.f32 && launch_fwd_tap64p(a, s, 1)) return 1;
  a.kpipe = option("tap64_kpipe", 0);   // (opt-in: +1-1.5 % on the BN-backward data gradients, profiles/r03_kpipe_ab.txt)
  // (LDS-staged BN-backward epilogue: level 2 256 -> 256 -9 %, level 3 1024 -> 512 -3 %, others within 1 %;
  //  profiles/r05_bnrlds_kernels.log)
  a.bnr_lds = option("tap64_bnr_lds", 1) && (size_t)a.M * a.bnr_zs * 2 < ((size_t)1 << 31);
  {
    const size_t es = a.f32 ? 4 : 2, lim = (size_t)1 << 31;
    a.mask_lds = option("tap64_mask_lds", 1) && !a.f8 && !a.bnr_z && a.out && a.out_mode == 0 && !a.relu &&
                 a.drop_rate == 0.f && !a.accum && a.out_stride % 8 == 0 &&
                 (!a.mask || ((size_t)a.mask_stride * es % 16 == 0 && (size_t)a.M * a.mask_stride * es < lim)) &&
                 (!a.addend || ((size_t)a.addend_stride * es % 16 == 0 && (size_t)a.M * a.addend_stride * es < lim));
  }
  if (a.f32 && cfg == 0) cfg = 1;
  if (cfg == 0) launch_cfg<2, 4, 128>(a, s);
  else if (cfg == 1) launch_cfg<4, 2, 64>(a, s);
  else if (cfg == 2) launch_cfg<4, 1, 128>(a, s);
  else if (cfg == 3) launch_cfg<4, 1, 64>(a, s);
  else return 0;
  return 1;
}
}  // namespace adp
