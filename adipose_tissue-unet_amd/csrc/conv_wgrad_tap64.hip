// Phase-pipelined LDS-DMA weight-gradient kernel ("wgrad tap64") for layers whose channel stride is
// a multiple of 64 (every unet_bn conv after the input layer, their ConvTranspose layers):
//   dW[n][k] += sum_m dY[m][n] * X(k)[m]      (k = tap * Cin_s + ci, m = output pixel)
// Semantics are those of igemm_wgrad_kernel (conv_igemm.hip); the bias gradient is the separate
// channel-sum launch.
//
// Block = WN x WK waves, dW tile TN x TK = (WN*TNW) x (WK*64); each wave a TNW x 64 tile of
// v_mfma_f32_16x16x32_bf16 accumulators whose A operand (dY^T) and B operand (X^T) are read from the
// natural [pixel][channel] LDS images with ds_read_b64_tr_b16 (MFMA k = pixel). A stage is 64 pixels,
// staged as four quarter images — dY and X for pixels 0-31 (q0) and 32-63 (q1) — moved by
// global_load_lds_dwordx4. Phases: q0 (split into the two n halves of the wave when TNW = 128), then
// q1; a quarter is refilled with stage t+2 (q0) or t+1 (q1) as soon as its reader phases have passed a
// barrier, and each phase pair ends in one counted `s_waitcnt vmcnt` (never 0 in the loop).
//
// Per-lane gather: a thread's 16-B chunk column is fixed for the whole kernel (the row swizzle only
// depends on row bits a thread's rows share), so its tap, source and channel are constants and its
// pixel rows advance by 64 per stage with incremental (image, y, x) coordinates — no divisions in
// the loop.
#include "conv_common.h"
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

namespace {

__device__ __attribute__((aligned(256))) uint4 wg64_zero_page[64];

constexpr unsigned WG_OOB = 0x80000000u;   // buffer offset beyond every resource: reads as zeros
constexpr int WG_RSRC3 = 0x00020000;       // raw buffer descriptor word 3 (gfx9: 32-bit data format)
// one 16-B-per-lane LDS-DMA piece through a buffer resource (device function: the host pass of the
// kernel templates never sees the target builtin)
__device__ __forceinline__ void wg_buf_lds16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
}
// (the same with a wave-uniform scalar offset added to the per-lane one)
__device__ __forceinline__ void wg_buf_lds16s(__amdgpu_buffer_rsrc_t r, void* lds, unsigned off, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, soff, 0, 0);
}
__device__ __forceinline__ void wg_glds16(const void* p, void* lds) {
  __builtin_amdgcn_global_load_lds(p, (lds_void*)lds, 16, 0, 0);
}


#define W64_BAR()                          \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_s_barrier();          \
    asm volatile("" ::: "memory");         \
  } while (0)

struct PixSlot { int m, n, y, x; };

ADP_DEV void slot_init(PixSlot& s, int m, int HWo, int Wo) {
  s.m = m;
  s.n = m / HWo;
  const int rem = m - s.n * HWo;
  s.y = rem / Wo;
  s.x = rem - s.y * Wo;
}
// next stage (pixel + 64) as a branch-free mixed-radix add of (an, ay, ax) = 64 in (image, y, x) digits
struct Adv { int an, ay, ax; };
ADP_DEV void slot_adv(PixSlot& s, const Adv& d, int Ho, int Wo) {
  s.m += 64;
  s.x += d.ax;
  const int cx = s.x >= Wo;
  s.x -= cx ? Wo : 0;
  s.y += d.ay + cx;
  const int cy = s.y >= Ho;
  s.y -= cy ? Ho : 0;
  s.n += d.an + cy;
}

// ds_read_b64_tr_b16 as inline asm: the builtin form makes hipcc wait vmcnt(0) (every LDS-DMA in
// flight) before each read, because it cannot tell the read from the pending DMA writes. The caller
// orders these reads with explicit lgkmcnt waits.
ADP_DEV v4s16 ds_tr16(uint32_t lds_addr) {
  v4s16 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr) : "memory");
  return r;
}
typedef unsigned v4u32_w __attribute__((ext_vector_type(4)));
// LDS float4 read / 16-B write as inline asm: the compiler would put a vmcnt(0) (every LDS-DMA in flight)
// in front of a plain access to the LDS object the DMA writes; the reader waits itself
ADP_DEV float4 wg_lds_f4(uint32_t lds_addr) {
  float4 r;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr) : "memory");
  return r;
}
typedef unsigned v2u32_w __attribute__((ext_vector_type(2)));
ADP_DEV v2u32_w wg_lds_r8(uint32_t lds_addr) {
  v2u32_w r;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr) : "memory");
  return r;
}
ADP_DEV void wg_lds_w16(uint32_t lds_addr, v4u32_w v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr), "v"(v) : "memory");
}
ADP_DEV void wg_lds_w8(uint32_t lds_addr, v2u32_w v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(lds_addr), "v"(v) : "memory");
}
ADP_DEV uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
template <int N>
ADP_DEV void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int RB>
ADP_DEV bf16x8 tr_frag_asm(uint32_t base, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = 16 * (g >> 1) + 4 * (g & 1) + q, r1 = r0 + 8;
  const int col = col0 + 4 * p, chunk = col >> 3, inb = (col & 7) * 2;
  const v4s16 lo = ds_tr16(base + r0 * RB + ((chunk ^ gsw<RB>(r0)) << 4) + inb);
  const v4s16 hi = ds_tr16(base + r1 * RB + ((chunk ^ gsw<RB>(r1)) << 4) + inb);
  bf16x8 r;
  const bf16* l = reinterpret_cast<const bf16*>(&lo);
  const bf16* h = reinterpret_cast<const bf16*>(&hi);
#pragma unroll
  for (int e = 0; e < 4; ++e) { r[e] = l[e]; r[4 + e] = h[e]; }
  return r;
}

template <int WN, int WK, int TNW>
constexpr int wg64_occ() { return 2 * 2 * 32 * (2 * WN * TNW + 2 * WK * 64) <= 81920 ? 2 : 1; }

// RA (row-aligned): Wo % 64 == 0, no upsample and 64-aligned splits, so every 64-pixel stage lies in
// one image row: the stage origin (image, y, x0) is block-uniform (scalar registers) and each
// slot's gather address is that origin plus a per-slot 64-bit constant.
template <int WN, int WK, int TNW, bool TWO_BAR, bool RA>
__global__ __launch_bounds__(WN * WK * 64, (wg64_occ<WN, WK, TNW>())) void igemm_wgrad_tap64_kernel(WgradArgs a) {
  constexpr int NTH = WN * WK * 64;
  constexpr int TN = WN * TNW, TK = WK * 64;
  constexpr int RD = 2 * TN, RX = 2 * TK;              // LDS row bytes (one pixel)
  constexpr int QD = 32 * RD, QX = 32 * RX;            // quarter image bytes
  constexpr int STAGE = 2 * (QD + QX);
  constexpr int CPRD = RD / 16, CPRX = RX / 16;        // 16-B chunks per row
  constexpr int RPID = NTH / CPRD, RPIX = NTH / CPRX;  // rows per glds instruction (whole block)
  constexpr int GD = 32 / RPID, GX = 32 / RPIX;        // glds per thread per quarter
  static_assert(GD >= 1 && GX >= 1 && GD * RPID == 32 && GX * RPIX == 32, "quarters must split evenly");
  static_assert(RPID % 8 == 0 && RPIX % 8 == 0, "a thread's rows must share the swizzle bits");
  constexpr int NH = GD + GX;                          // glds per thread per pixel half
  constexpr bool SPLIT = TNW == 128;                   // two phases (n halves) per pixel half
  constexpr int NB = TNW / 16;                         // 16-row n blocks per wave
  constexpr int NBP = SPLIT ? NB / 2 : NB;             // n blocks per phase
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: LDS-DMA bases in SGPRs
  const int wn = wave / WK, wk = wave % WK;
  // 1-D grid, XCD remap with the tile index fastest: all dW tiles of one pixel split run back to
  // back on one XCD and share its L2 for dY (every tile of the split) and X (neighbouring taps)
  const int tiles = a.ntile_k * a.ntile_n;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / tiles, tile = lin - split * tiles;
  const int tk = tile % a.ntile_k, tn = tile / a.ntile_k;
  const int k0 = tk * TK, n0 = tn * TN;
  const int mbeg = split * a.mchunk;
  const int mend = min(a.M, mbeg + a.mchunk);
  if (mbeg >= mend) return;
  const int ns = (mend - mbeg + 63) / 64;
  const int HWo = a.Ho * a.Wo, Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  const int Cin_s = a.CAs + a.CBs;

  // ---- fixed chunk columns
  const int kx = k0 + 8 * ((tid % CPRX) ^ gsw<RX>(tid / CPRX));
  const bool kvalid = kx < a.K;
  int oy = 0, ox = 0, xcs = a.CAs;
  const bf16* xbase = reinterpret_cast<const bf16*>(a.srcA);
  if (kvalid) {
    const int tap = kx / Cin_s, ci = kx - tap * Cin_s;
    const int ty = tap / a.kw, tx = tap - ty * a.kw;
    oy = ty * a.dil - a.pad;
    ox = tx * a.dil - a.pad;
    if (ci < a.CAs) xbase += ci;
    else { xbase = reinterpret_cast<const bf16*>(a.srcB) + (ci - a.CAs); xcs = a.CBs; }
  }
  const int nd = n0 + 8 * ((tid % CPRD) ^ gsw<RD>(tid / CPRD));
  const bool nvalid = nd < a.Nout;
  int dsub = 0, dc = nd;
  if (a.dy_mode == 1) { dsub = nd / a.Cps; dc = nd - dsub * a.Cps; }
  const bf16* dy = reinterpret_cast<const bf16*>(a.dY);

  // ---- general path: per-slot incremental (image, y, x) coordinates
  PixSlot sx[2][RA ? 1 : GX], sd[2][RA ? 1 : GD];
  Adv adv{0, 0, 0};
  // ---- row-aligned path: per-slot byte addresses relative to the stage origin
  const char* xb[2][GX];
  const char* db[2][GD];
  int xcol[2][GX], drow[2][GD];
  struct StageOrg { int m, n, y, x0; } org[2];
  const int ys_ok_lo = -oy;   // (y*stride + oy) in [0, Hv)  <=>  y*stride in [-oy, Hv - oy)
  if constexpr (RA) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int i = 0; i < GX; ++i) {
        const int r = 32 * q + i * RPIX + tid / CPRX;
        xcol[q][i] = r * a.stride + ox;
        xb[q][i] = reinterpret_cast<const char*>(xbase) + 2LL * ((long long)oy * a.Ws + xcol[q][i]) * xcs;
      }
#pragma unroll
      for (int i = 0; i < GD; ++i) {
        const int r = 32 * q + i * RPID + tid / CPRD;
        drow[q][i] = r;
        const long long e = a.dy_mode == 0 ? (long long)r * a.dy_stride + nd
                                           : ((long long)(dsub >> 1) * 2 * a.Wo + 2 * r + (dsub & 1)) * a.dy_stride + dc;
        db[q][i] = reinterpret_cast<const char*>(dy) + 2 * e;
      }
      org[q].m = mbeg;
      org[q].n = mbeg / HWo;
      const int rem = mbeg - org[q].n * HWo;
      org[q].y = rem / a.Wo;
      org[q].x0 = rem - org[q].y * a.Wo;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int i = 0; i < GX; ++i) slot_init(sx[q][i], mbeg + 32 * q + i * RPIX + tid / CPRX, HWo, a.Wo);
#pragma unroll
      for (int i = 0; i < GD; ++i) slot_init(sd[q][i], mbeg + 32 * q + i * RPID + tid / CPRD, HWo, a.Wo);
    }
    adv.an = 64 / HWo;
    adv.ay = (64 - adv.an * HWo) / a.Wo;
    adv.ax = 64 - adv.an * HWo - adv.ay * a.Wo;
  }

  // issue quarter q of the next stage into buffer buf, then advance to the following stage
  auto issue = [&](int q, int buf) {
    unsigned char* base = smem + buf * STAGE;
    if constexpr (RA) {
      StageOrg& o = org[q];
      const int left = mend - o.m;                                   // valid rows of this stage
      const long long xo = 2LL * (((long long)o.n * a.Hs + o.y * a.stride) * a.Ws + (long long)o.x0 * a.stride);
      const long long dof = a.dy_mode == 0 ? 2LL * o.m * a.dy_stride
                                           : 2LL * (((long long)o.n * 2 * a.Ho + 2 * o.y) * 2 * a.Wo + 2 * o.x0) * a.dy_stride;
      const bool yok = kvalid && o.y * a.stride >= ys_ok_lo && o.y * a.stride + oy < Hv;
      const int x0s = o.x0 * a.stride;
#pragma unroll
      for (int i = 0; i < GD; ++i) {
        const bool ok = nvalid && drow[q][i] < left;
        const void* p = ok ? (const void*)(db[q][i] + dof) : (const void*)wg64_zero_page;
        __builtin_amdgcn_global_load_lds(p, (lds_void*)(base + q * QD + (i * RPID + wave * (64 / CPRD)) * RD), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < GX; ++i) {
        const int xr = 32 * q + i * RPIX + tid / CPRX;
        const bool ok = yok && xr < left && (unsigned)(x0s + xcol[q][i]) < (unsigned)Wv;
        const void* p = ok ? (const void*)(xb[q][i] + xo * xcs) : (const void*)wg64_zero_page;
        __builtin_amdgcn_global_load_lds(p, (lds_void*)(base + 2 * QD + q * QX + (i * RPIX + wave * (64 / CPRX)) * RX),
                                         16, 0, 0);
      }
      o.m += 64;
      o.x0 += 64;
      if (o.x0 >= a.Wo) {
        o.x0 = 0;
        if (++o.y == a.Ho) { o.y = 0; ++o.n; }
      }
    } else {
#pragma unroll
      for (int i = 0; i < GD; ++i) {
        PixSlot& s = sd[q][i];
        size_t off;
        if (a.dy_mode == 0) {
          off = (size_t)s.m * a.dy_stride + nd;
        } else {
          off = (((size_t)s.n * (2 * a.Ho) + 2 * s.y + (dsub >> 1)) * (2 * a.Wo) + 2 * s.x + (dsub & 1)) * a.dy_stride + dc;
        }
        const bool ok = s.m < mend && nvalid;
        const void* p = ok ? (const void*)(dy + off) : (const void*)wg64_zero_page;
        __builtin_amdgcn_global_load_lds(p, (lds_void*)(base + q * QD + (i * RPID + wave * (64 / CPRD)) * RD), 16, 0, 0);
        slot_adv(s, adv, a.Ho, a.Wo);
      }
#pragma unroll
      for (int i = 0; i < GX; ++i) {
        PixSlot& s = sx[q][i];
        int yi = s.y * a.stride + oy, xi = s.x * a.stride + ox;
        const bool ok = s.m < mend && kvalid && (unsigned)yi < (unsigned)Hv && (unsigned)xi < (unsigned)Wv;
        if (a.up == 2) { yi >>= 1; xi >>= 1; }
        const void* p = ok ? (const void*)(xbase + (size_t)((s.n * a.Hs + yi) * a.Ws + xi) * xcs)
                           : (const void*)wg64_zero_page;
        __builtin_amdgcn_global_load_lds(p, (lds_void*)(base + 2 * QD + q * QX + (i * RPIX + wave * (64 / CPRX)) * RX),
                                         16, 0, 0);
        slot_adv(s, adv, a.Ho, a.Wo);
      }
    }
  };

  f32x4 acc[NB][4];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fd[NBP], fx[4];
  const uint32_t sbase = lds_off(smem);
  auto readD = [&](int buf, int q, int h) {
    const uint32_t base = sbase + buf * STAGE + q * QD;
#pragma unroll
    for (int nb = 0; nb < NBP; ++nb) fd[nb] = tr_frag_asm<RD>(base, wn * TNW + (h * NBP + nb) * 16, lane);
  };
  auto readX = [&](int buf, int q) {
    const uint32_t base = sbase + buf * STAGE + 2 * QD + q * QX;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) fx[kb] = tr_frag_asm<RX>(base, wk * 64 + kb * 16, lane);
  };
  // MFMAs of one phase. The fragments come from inline-asm LDS reads issued X first, then dY block by
  // block (2 reads each): wait only for what the next dY block needs (lgkmcnt counts the dY reads
  // still outstanding) and pin the MFMAs below each wait with a scheduling barrier.
  auto mma_nb = [&](auto nbc, int h) {
    constexpr int nb = decltype(nbc)::value;
    if constexpr (nb < NBP) {
      lgkm_wait<2 * (NBP - 1 - nb)>();
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
        acc[h * NBP + nb][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[nb], fx[kb], acc[h * NBP + nb][kb], 0, 0, 0);
    }
  };
  auto mma = [&](int h) {
    __builtin_amdgcn_s_setprio(1);
    mma_nb(std::integral_constant<int, 0>{}, h);
    mma_nb(std::integral_constant<int, 1>{}, h);
    mma_nb(std::integral_constant<int, 2>{}, h);
    mma_nb(std::integral_constant<int, 3>{}, h);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: stage 0 (q0, q1) and stage 1 q0 in flight; wait for stage 0 q0
  issue(0, 0);
  issue(1, 0);
  if (ns > 1) {
    issue(0, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NH) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NH) : "memory");
  }
  W64_BAR();

  for (int t = 0; t < ns; ++t) {
    const int buf = t & 1;
    const bool n1 = t + 1 < ns, n2 = t + 2 < ns;
    // ---- pixel half 0 (q0); q1 of the other buffer is free -> stage t+1 q1
    if (n1) issue(1, buf ^ 1);
    readX(buf, 0);
    readD(buf, 0, 0);
    if (TWO_BAR) W64_BAR();
    mma(0);
    if (SPLIT) {
      if (TWO_BAR) W64_BAR();
      readD(buf, 0, 1);
      if (TWO_BAR) W64_BAR();
      mma(1);
    }
    // retire stage t q1 (issued after it: stage t+1 q0 and q1, iff they exist)
    if (n1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NH) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W64_BAR();
    // ---- pixel half 1 (q1); q0 of this buffer is free -> stage t+2 q0
    if (n2) issue(0, buf);
    readX(buf, 1);
    readD(buf, 1, 0);
    if (TWO_BAR) W64_BAR();
    mma(0);
    if (SPLIT) {
      if (TWO_BAR) W64_BAR();
      readD(buf, 1, 1);
      if (TWO_BAR) W64_BAR();
      mma(1);
    }
    // retire stage t+1 q0 (issued after it: stage t+1 q1, stage t+2 q0 iff it exists)
    if (n2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NH) : "memory");
    else if (n1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NH) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W64_BAR();
  }

  const int col = lane & 15, rq = (lane >> 4) * 4;
  if (ADP_DBG(a) & 1) {   // timing-only ablation: keep the accumulators live, skip the atomics
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) asm volatile("" ::"v"(acc[nb][kb]));
    return;
  }
  // Output: each wave's 16-row blocks are re-shaped through LDS so that every store / atomic covers one
  // whole 256-B row of dW (64 consecutive k). With several pixel splits the partial sums go to a
  // per-split slab by plain stores and a second launch sums the slabs into dW: f32 atomics execute at
  // the memory side at ~1.3 TB/s chip-wide, and the split partials of a step add up to ~2 GB (measured
  // 1.7 ms of atomics per training step). The loop above ended on a barrier: the staging buffers are free.
  constexpr int ES = 68;   // padded row stride (floats) of a wave's 16 x 64 block
  float* blk = reinterpret_cast<float*>(smem) + wave * 16 * ES;
  const int kk = k0 + wk * 64 + lane;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) blk[(rq + r) * ES + kb * 16 + col] = acc[nb][kb][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (a.part) {   // this split's partial slab: plain 256-B row stores, reduced by wgrad_reduce_kernel
      float* slab = a.part + (size_t)split * a.Nout * a.Kpad;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int n = n0 + wn * TNW + nb * 16 + i;
        const float v = blk[i * ES + lane];
        if (n < a.Nout && kk < a.K) slab[(size_t)n * a.Kpad + kk] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int n = n0 + wn * TNW + nb * 16 + i;
        const float v = blk[i * ES + lane];
        if (n < a.Nout && kk < a.K) atomicAdd(a.dW + (size_t)n * a.Kpad + kk, v);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
}

// Persistent halo weight-gradient kernel for the narrow full-resolution layers (3x3, stride 1, dilation
// 1, Cin_s == 64 single source, Nout == 64, plain dY: unet_bn level-0 64->64 convs). The tap64 kernel
// re-gathers every input pixel once per tap (9x) through LDS-DMA and pads K = 576 to three 256-wide
// tiles (a third of its MFMAs multiply zeros). Here one block per CU walks 8 x 32 output patches; per
// patch the 10 x 34 input halo and the 256 x 64 dY tile are moved into LDS once (LDS-DMA, double
// buffered across patches), and wave t (9 waves) accumulates dW_t = sum_p dY[p]^T X[p + off_t] for tap
// t in 16 accumulator tiles that stay in registers for all of the block's patches: each patch row is
// one 32-pixel MFMA k step of transposed LDS reads (both operands with the same row permutation). The
// block's dW partial is added once at the end (256-B rows through LDS, f32 atomics).
// NW = 9: one wave per tap (9 waves on 4 SIMDs: the SIMD holding 3 of them sets the pace). NW = 8: wave
// w owns tap w and a 16 x 32 eighth of tap 8 (output block w >> 1, column blocks 2 (w & 1) + {0, 1}),
// two waves per SIMD with 18 MFMAs each per k step.
//
// BNA (adp_conv_wgrad_bn, NW = 8): the dY tile is not read but computed, adp_bn_bwd_apply of the layer's
// BatchNorm fused. At the first two rows of a patch each thread moves its 4 16-B groups of dA (into the
// next stage's dY image) and of z (into the next stage's halo image, free until its halo is issued) by
// LDS-DMA with the dY swizzle; at row BNA_ROW it waits for its own pieces, applies
// dY = P*dA*(z*s+h > 0) + Q*(z - mean) + R in place (the apply kernel's arithmetic and bf16 rounding; the
// thread's channel group is fixed, so its constants are 8 LDS words each) and -- blocks of input chunk 0
// only -- stores dY for the data-gradient launch; the halo groups follow at rows BNA_ROW..7. No barrier
// and no long-lived registers: every thread reads back only the LDS slots its own DMA wrote.
// CLM: the patch-claiming code compiled in (false: static lists only, the instances of every launch without a claim
// counter -- the register allocation without the claim ring and its waits, as the persistent forward's EPIC = 3)
// PF (round 5): row-pipelined fragments -- each wave issues the LDS reads of patch row pr + 1 before the MFMAs of row
// pr (two fragment sets in registers), and the next patch's row 0 right after the patch barrier, before row 7's MFMAs.
// Without it a wave waits for its own row's reads before every MFMA cluster, and since the waves leave each patch
// barrier together, all 8 waves read at once and then all multiply at once (the two waves of a SIMD do not cover each
// other's read phase): the round-5 ablation (profiles/r05a_wgrad_ablation.log) ran the K loop with no LDS-DMA, no
// barrier and no atomics at only 1.33 PF.
template <int NW, bool BNA = false, int SPR = 8, bool CLM = true, bool PF = false>
__global__ __launch_bounds__(NW * 64, 1) void igemm_wgrad_halop_kernel(WgradArgs a) {
  static_assert(!PF || (NW == 8 && !BNA && !CLM), "PF: the plain static-list 8-wave form");
  constexpr int NTH = NW * 64, RB = 128;
  constexpr int PH = 8, PW = 32, HW = PW + 2, HROWS = (PH + 2) * HW;   // 340 halo pixels
  constexpr int HCH = HROWS * 8, DCH = PH * PW * 8;                     // 16-B chunks per image
  constexpr int GH = (HCH + NTH - 1) / NTH, GD = (DCH + NTH - 1) / NTH;
  constexpr int HBUF = HROWS * RB, DBUF = PH * PW * RB;
  constexpr int STAGE = HBUF + DBUF;
  static_assert(GH + GD <= 2 * PH, "the next patch's LDS-DMA groups are spread over the 8 patch rows");
  static_assert(!BNA || (NW == 8 && GD * NTH == DCH), "BNA: 8 waves, whole dY groups");
  constexpr int BNA_ROW = 3;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE + (BNA ? 6 * 64 * 4 : 0) + 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // = tap
  const int dbg = ADP_DBG(a);   // timing-only ablations (option wgrad_debug): bits 0-3, see below
  prio_static<ADP_PRIO_WGRAD>(wave);
  const int dy = wave / 3, dx = wave - 3 * (wave / 3);
  const int tx_n = a.Wo / PW, ty_n = a.Ho / PH;
  // work unit = (patch, 64-channel input chunk, 64-wide output block); a block keeps one
  // (chunk, output block) combination for all of its patches (its accumulators are that dW block)
  const int nch = (a.CAs + a.CBs) >> 6, combos = nch * (a.Nout >> 6);
  const int T = a.Nimg * tx_n * ty_n, G = gridDim.x / combos;
  const int lin0 = xcd_remap(blockIdx.x, gridDim.x);
  const int combo = lin0 % combos, lin = lin0 / combos;
  const int ch = combo % nch, nblk = combo / nch;
  // patches: the static list lin, lin + G, ... (nt of them), or (dyn, conv_common.h) super-patches of CH
  // consecutive patches claimed from the counter of the block's (chunk, output block) combination: super-patches
  // 0 and 1 are the block's static ones, claim value c is super-patch 2 G + c; super-patch s + 2 is claimed at the
  // start of super-patch s (a compiler-visible atomic: this file is built without the atomic optimizer) and
  // published after the drain at the end of its first patch, before that patch's barrier
  const bool dyn = CLM && a.claim != nullptr;
  const bool full = dyn && a.claim_full;   // every super-patch claimed (0 and 1 by one claim at the start)
  int* ring = reinterpret_cast<int*>(smem + 2 * STAGE + (BNA ? 6 * 64 * 4 : 0));
  const int nt = dyn ? 0 : (lin < T ? (T - lin + G - 1) / G : 0);
  const int CH = dyn ? a.claim_chunk : 1, nsup = (T + CH - 1) / CH;
  auto sup_id = [&](int sidx) -> int {
    const int v = full ? claim_ring_read(ring + (sidx & 3))
                       : sidx < 2 ? lin + sidx * G : 2 * G + claim_ring_read(ring + (sidx & 3));
    return v < nsup ? v : -1;
  };
  auto tile_id = [&](int k) -> int {
    if (!dyn) return k < nt ? lin + k * G : -1;
    const int v = sup_id(k / CH);
    const int t = v * CH + k % CH;
    return v >= 0 && t < T ? t : -1;
  };
  const bool inA = ch * 64 < a.CAs;
  const int xcs = inA ? a.CAs : a.CBs;
  // operands through buffer resources over the whole source / dY tensors (the launcher keeps each below
  // 2 GiB): a halo pixel outside the image is an out-of-range offset and reads as zeros
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(inA ? a.srcA : a.srcB), 0, a.Nimg * a.Hs * a.Ws * xcs * 2, WG_RSRC3);
  // (BNA with dY null: nothing reads dz, a zero-size resource drops its stores)
  const __amdgpu_buffer_rsrc_t rsD =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dY, 0, a.dY ? a.Nimg * a.Ho * a.Wo * a.dy_stride * 2 : 0, WG_RSRC3);
  const __amdgpu_buffer_rsrc_t rsBA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BNA ? a.bna_dA : a.dY), 0, a.Nimg * a.Ho * a.Wo * a.dy_stride * 2, WG_RSRC3);
  const __amdgpu_buffer_rsrc_t rsBZ = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BNA ? a.bna_z : a.dY), 0, a.Nimg * a.Ho * a.Wo * a.dy_stride * 2, WG_RSRC3);
  // per-thread constant parts of the gathers: halo group i -> (pixel delta, row/col offsets, byte offset)
  // up = 2 (nearest-x2 upsample folded into the input gather, adipose_v3's up*_conv1): halo pixel (y0 + hy,
  // x0 + hx) of the conv's input grid is source pixel ((y0 + hy) >> 1, (x0 + hx) >> 1) = (y0 / 2 + (hy >> 1), ...)
  // for the even patch origins, so the per-thread part of the gather stays a constant pixel delta
  const int us = a.up >> 1;
  int hy[GH], hx[GH], hpix[GH], hoff[GH], dpix[GD], doff[GD];
  const int xc0 = (inA ? ch * 64 : ch * 64 - a.CAs) * 2;
#pragma unroll
  for (int i = 0; i < GH; ++i) {
    const int idx = i * NTH + tid, hr = idx >> 3, pos = idx & 7;
    hy[i] = hr / HW - 1;
    hx[i] = hr % HW - 1;
    hpix[i] = (hy[i] >> us) * a.Ws + (hx[i] >> us);
    hoff[i] = xc0 + 16 * (pos ^ gsw<RB>(hr));
  }
#pragma unroll
  for (int i = 0; i < GD; ++i) {
    const int idx = i * NTH + tid, pr = idx >> 3, pos = idx & 7;
    dpix[i] = (pr >> 5) * a.Wo + (pr & 31);
    doff[i] = nblk * 128 + 16 * (pos ^ gsw<RB>(pr));
  }
  // patch k of this block -> origin (image row base, y0, x0) and the pixel indices of its (y0, x0)
  struct Patch { int y0, x0, pbx, pbd; };
  auto patch = [&](int t) {   // (t: the patch index from tile_id, read once per patch and carried)
    Patch P;
    const int px = t % tx_n, r = t / tx_n;
    const int img = r / ty_n;
    P.y0 = (r % ty_n) * PH;
    P.x0 = px * PW;
    P.pbx = (img * a.Hs + (P.y0 >> us)) * a.Ws + (P.x0 >> us);
    P.pbd = (img * a.Ho + P.y0) * a.Wo + P.x0;
    return P;
  };
  auto issue_h = [&](const Patch& P, int i, int buf) {
    const int idx = i * NTH + tid;
    if (i < GH - 1 || idx < HCH) {
      const int gy = P.y0 + hy[i], gx = P.x0 + hx[i];
      const bool ok = (unsigned)gy < (unsigned)(a.Hs << us) && (unsigned)gx < (unsigned)(a.Ws << us);
      const unsigned off = ok ? (unsigned)((P.pbx + hpix[i]) * xcs * 2 + hoff[i]) : WG_OOB;
      wg_buf_lds16(rsX, smem + buf * STAGE + (size_t)(i * NTH + wave * 64) * 16, off);
    }
  };
  auto issue_d = [&](const Patch& P, int i, int buf) {
    const int idx = i * NTH + tid;
    if (i < GD - 1 || idx < DCH) {
      const unsigned off = (unsigned)((P.pbd + dpix[i]) * a.dy_stride * 2 + doff[i]);
      if constexpr (BNA) {   // dA -> the dY image, z -> the (still unused) halo image of the stage
        wg_buf_lds16(rsBA, smem + buf * STAGE + HBUF + (size_t)(i * NTH + wave * 64) * 16, off);
        wg_buf_lds16(rsBZ, smem + buf * STAGE + (size_t)(i * NTH + wave * 64) * 16, off);
      } else {
        wg_buf_lds16(rsD, smem + buf * STAGE + HBUF + (size_t)(i * NTH + wave * 64) * 16, off);
      }
    }
  };
  // the groups of the next patch issued while row pr of this one multiplies: halo first, then dY,
  // two per row until the remaining rows can take one each (BNA: halo only, rows 2..7)
  auto issue_row = [&](const Patch& P, int pr, int buf) {
    if constexpr (BNA) {   // rows 0-1: dA / z groups; rows BNA_ROW..7: the halo, two per row first
      constexpr int HR = PH - BNA_ROW, EXTRA = GH - HR;
      if (pr < 2) {
#pragma unroll
        for (int i = 0; i < GD; ++i)
          if (i / (GD / 2) == pr) issue_d(P, i, buf);
      } else if (SPR != PH && pr >= BNA_ROW) {   // two halo groups a row from BNA_ROW on
#pragma unroll
        for (int gi = 0; gi < GH; ++gi)
          if (gi / 2 == pr - BNA_ROW) issue_h(P, gi, buf);
      } else if (pr >= BNA_ROW) {
        const int r = pr - BNA_ROW;
        const int g0 = r < EXTRA ? 2 * r : EXTRA + r;
        const int g1 = r < EXTRA ? g0 + 1 : -1;
#pragma unroll
        for (int gi = 0; gi < GH; ++gi)
          if (gi == g0 || gi == g1) issue_h(P, gi, buf);
      }
      return;
    }
    constexpr int NG = GH + GD;
    if constexpr (SPR == PH) {   // over all 8 rows: rows 0 .. EXTRA-1 take two groups
      constexpr int EXTRA = NG - PH;
      const int g0 = pr < EXTRA ? 2 * pr : EXTRA + pr;
      const int g1 = pr < EXTRA ? g0 + 1 : -1;
#pragma unroll
      for (int gi = 0; gi < NG; ++gi)
        if (gi == g0 || gi == g1) {
          if (gi < GH) issue_h(P, gi, buf);
          else issue_d(P, gi - GH, buf);
        }
    } else {   // over rows 0 .. SPR-1, ceil(NG / SPR) groups a row: the last rows give the DMA slack
      constexpr int PER = (NG + SPR - 1) / SPR;
#pragma unroll
      for (int gi = 0; gi < NG; ++gi)
        if (gi / PER == pr) {
          if (gi < GH) issue_h(P, gi, buf);
          else issue_d(P, gi - GH, buf);
        }
    }
  };
  // transposed 16x32 fragment of an [row][64 bf16] LDS image whose rows row0 .. row0+31 are the 32
  // pixels of one k step (absolute rows, so the row swizzle matches the one applied on load)
  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, pp = ii & 3;
  const int rr0 = 16 * (g >> 1) + 4 * (g & 1) + q;
  // BNA: the lane terms are re-derived per patch from an opaque copy of the lane id, so that the
  // fragment addresses of the 8 unrolled rows are not hoisted out of the patch loop (they would hold
  // the registers the apply needs)
  int fpp = pp, frr0 = rr0;
  auto frag = [&](uint32_t img_base, int row0, int col0) {
    const int col = col0 + 4 * fpp, chunk = col >> 3, inb = (col & 7) * 2;
    const int R0 = row0 + frr0, R1 = R0 + 8;
    const v4s16 lo = ds_tr16(img_base + R0 * RB + ((chunk ^ gsw<RB>(R0)) << 4) + inb);
    const v4s16 hi = ds_tr16(img_base + R1 * RB + ((chunk ^ gsw<RB>(R1)) << 4) + inb);
    bf16x8 r;
    const bf16* l = reinterpret_cast<const bf16*>(&lo);
    const bf16* h = reinterpret_cast<const bf16*>(&hi);
#pragma unroll
    for (int e = 0; e < 4; ++e) { r[e] = l[e]; r[4 + e] = h[e]; }
    return r;
  };

  // ---- BNA: per-channel constants of this output block in LDS ([6][64]: scale, shift, mean, P, Q, R, as
  // bn_bwd_apply_kernel forms them); the thread's slots hold source channel group bcg for all its groups
  // (the swizzle gsw(pr) depends on row bits its rows share)
  float* bk = reinterpret_cast<float*>(smem + 2 * STAGE);
  const uint32_t sbase = lds_off(smem);
  const int bcg = (tid & 7) ^ gsw<RB>(tid >> 3);
  auto bna_apply = [&](const Patch& P, int buf) {
    if constexpr (BNA) {
      uint32_t og[GD][4];
#pragma unroll
      for (int half = 0; half < 2; ++half) {   // 4 channels at a time: bounds the registers held
        float c[6][4];
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const float4 v = wg_lds_f4(sbase + 2 * STAGE + (q * 64 + bcg * 8 + 4 * half) * 4);
          c[q][0] = v.x; c[q][1] = v.y; c[q][2] = v.z; c[q][3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < GD; ++i) {
          const uint32_t slot = (uint32_t)(i * NTH + tid) * 16 + 8 * half;
          const v2u32_w dv = wg_lds_r8(sbase + buf * STAGE + HBUF + slot);
          const v2u32_w zv = wg_lds_r8(sbase + buf * STAGE + slot);
          const bf16* d = reinterpret_cast<const bf16*>(&dv);
          const bf16* zz = reinterpret_cast<const bf16*>(&zv);
          bf16 o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {   // bn_bwd_apply_kernel's arithmetic and rounding
            const float zf = (float)zz[j];
            const float db = fmaf(zf, c[0][j], c[1][j]) > 0.f ? (float)d[j] : 0.f;
            o[j] = (bf16)fmaf(c[3][j], db, fmaf(c[4][j], zf - c[2][j], c[5][j]));
          }
          const uint32_t* ow = reinterpret_cast<const uint32_t*>(o);
          og[i][2 * half] = ow[0];
          og[i][2 * half + 1] = ow[1];
        }
      }
#pragma unroll
      for (int i = 0; i < GD; ++i) {
        const v4u32_w ov = {og[i][0], og[i][1], og[i][2], og[i][3]};
        wg_lds_w16(sbase + buf * STAGE + HBUF + (uint32_t)(i * NTH + tid) * 16, ov);
        if (ch == 0)
          __builtin_amdgcn_raw_buffer_store_b128(ov, rsD, (unsigned)((P.pbd + dpix[i]) * a.dy_stride * 2 + doff[i]), 0, 0);
      }
      // this thread's z slots are overwritten by its own halo DMA next: the reads above are complete
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  if constexpr (BNA) {
    if (tid < 64) {
      const int cc = nblk * 64 + tid;
      const float k = a.bna_gamma[cc] * a.bna_invstd[cc];
      bk[0 * 64 + tid] = a.bna_sc[cc];
      bk[1 * 64 + tid] = a.bna_sh[cc];
      bk[2 * 64 + tid] = a.bna_mean[cc];
      bk[3 * 64 + tid] = k;
      bk[4 * 64 + tid] = -k * a.bna_invstd[cc] * a.bna_dgamma[cc] * a.bna_inv_count;
      bk[5 * 64 + tid] = -k * a.bna_dbeta[cc] * a.bna_inv_count;
    }
    __syncthreads();
  }

  f32x4 acc[4][4], acc8[2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc8[0] = acc8[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nb8 = wave >> 1, cb8 = 2 * (wave & 1);

  if (full) {   // the first two super-patches (a block that starts late finds them past the end)
    if (tid == 0) {
      const int r = claim_next2(a.claim + combo);
      ring[0] = r;
      ring[1] = r + 1;
    }
    __syncthreads();
  }
  int tcur = tile_id(0);
  const bool any = tcur >= 0;
  if (any) {
    const Patch P0 = patch(tcur);
    if constexpr (BNA) {
#pragma unroll
      for (int i = 0; i < GD; ++i) issue_d(P0, i, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bna_apply(P0, 0);
    }
#pragma unroll
    for (int i = 0; i < GH; ++i) issue_h(P0, i, 0);
    if constexpr (!BNA) {
#pragma unroll
      for (int i = 0; i < GD; ++i) issue_d(P0, i, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W64_BAR();
  }
  if constexpr (PF) {
    struct Frags { bf16x8 fd[4], fx[4], fd8, fx8[2]; };
    Frags F[2];   // fragments of the even / odd patch rows
    // per-lane byte offset of a transposed 16 x 32 fragment whose 32 rows start at row C of an image (the same
    // addressing as frag()); lz: an opaque copy of the lane id, so that the 29 addresses below are rebuilt per
    // patch instead of being held across the loop next to their per-buffer sums
    auto xoff = [&](int C, int col0, int lz) -> uint32_t {
      const int g_ = lz >> 4, i_ = lz & 15;
      const int R = C + 16 * (g_ >> 1) + 4 * (g_ & 1) + (i_ >> 2);
      const int col = col0 + 4 * (i_ & 3), chunk = col >> 3, inb = (col & 7) * 2;
      return (uint32_t)(R * RB + ((chunk ^ gsw<RB>(R)) << 4) + inb);
    };
    // halo rows of patch row pr = 4 q + m start at (pr + dy) * HW + dx: rows pr and pr + 4 differ by 4 HW = 136 rows
    // (a multiple of 8: the same swizzle), so 4 address registers per column block serve all 8 rows with immediate
    // offsets q * 136 * RB; the two 8-row halves of a fragment differ by 8 rows (same swizzle: + 8 RB); dY row pr
    // is + pr * PW * RB
    uint32_t ha[4][4], h8[4][2], da[4], d8;
    auto addrs = [&](uint32_t hb) {
      int lz = lane;
      asm volatile("" : "+v"(lz));
      const int C0 = dy * HW + dx;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) ha[m][cb] = hb + xoff(C0 + HW * m, cb * 16, lz);
#pragma unroll
        for (int j = 0; j < 2; ++j) h8[m][j] = hb + xoff(2 * HW + 2 + HW * m, cb8 * 16 + 16 * j, lz);
      }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) da[nb] = hb + HBUF + xoff(0, nb * 16, lz);
      d8 = hb + HBUF + xoff(0, nb8 * 16, lz);
    };
    auto rd = [](uint32_t ad, auto off) -> bf16x8 {   // two ds_read_b64_tr_b16 at immediate offsets off, off + 8 RB
      v4s16 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(ad), "n"(decltype(off)::value) : "memory");
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(ad), "n"(decltype(off)::value + 8 * RB)
                   : "memory");
      bf16x8 r;
      const bf16* l = reinterpret_cast<const bf16*>(&lo);
      const bf16* h = reinterpret_cast<const bf16*>(&hi);
#pragma unroll
      for (int e = 0; e < 4; ++e) { r[e] = l[e]; r[4 + e] = h[e]; }
      return r;
    };
    // the 22 reads of patch row pr (addresses of the current buffer) in two parts: 14 (dY, tap 8), then 8 (this
    // wave's tap); lgkmcnt holds at most 15, so the wait for the previous row sits between the parts
    auto load_row_a = [&](Frags& f, auto prc) {
      constexpr int pr = decltype(prc)::value, m = pr & 3;
      using HO = std::integral_constant<int, (pr >> 2) * 4 * HW * RB>;
      using DO = std::integral_constant<int, pr * PW * RB>;
      f.fd8 = rd(d8, DO{});
      f.fx8[0] = rd(h8[m][0], HO{});
      f.fx8[1] = rd(h8[m][1], HO{});
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) f.fd[nb] = rd(da[nb], DO{});
    };
    auto load_row_b = [&](Frags& f, auto prc) {
      constexpr int pr = decltype(prc)::value, m = pr & 3;
      using HO = std::integral_constant<int, (pr >> 2) * 4 * HW * RB>;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) f.fx[cb] = rd(ha[m][cb], HO{});
    };
    auto load_row = [&](Frags& f, auto prc) {
      load_row_a(f, prc);
      load_row_b(f, prc);
    };
    if (any) {
      addrs(sbase);
      load_row(F[0], std::integral_constant<int, 0>{});
    }
    for (int k = 0; any; ++k) {
      const int buf = k & 1;
      const int tn = tile_id(k + 1);
      const bool more = tn >= 0;
      const Patch Pn = patch(more ? tn : tcur);
      addrs(sbase + buf * STAGE);
      auto row = [&](auto prc) {
        constexpr int pr = decltype(prc)::value;
        if (more && !(dbg & 2)) issue_row(Pn, pr, buf ^ 1);
        if constexpr (pr < PH - 1) {
          load_row_a(F[(pr + 1) & 1], std::integral_constant<int, pr + 1>{});
          lgkm_wait<14>();   // row pr's fragments (issued one row ago) have landed
          load_row_b(F[(pr + 1) & 1], std::integral_constant<int, pr + 1>{});
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next patch landed (this thread's pieces)
          lgkm_wait<0>();                                      // row 7's fragments: this buffer is read out
          if (!(dbg & 4)) W64_BAR();
          if (more) {                                          // the next patch's row 0 under row 7's MFMAs
            addrs(sbase + (buf ^ 1) * STAGE);
            load_row(F[0], std::integral_constant<int, 0>{});
          }
        }
        const Frags& f = F[pr & 1];
        prio_hi<ADP_PRIO_WGRAD>();
        acc8[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.fd8, f.fx8[0], acc8[0], 0, 0, 0);
        acc8[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.fd8, f.fx8[1], acc8[1], 0, 0, 0);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
            acc[nb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.fd[nb], f.fx[cb], acc[nb][cb], 0, 0, 0);
        prio_lo<ADP_PRIO_WGRAD>();
      };
      row(std::integral_constant<int, 0>{});
      row(std::integral_constant<int, 1>{});
      row(std::integral_constant<int, 2>{});
      row(std::integral_constant<int, 3>{});
      row(std::integral_constant<int, 4>{});
      row(std::integral_constant<int, 5>{});
      row(std::integral_constant<int, 6>{});
      row(std::integral_constant<int, 7>{});
      if (!more) break;
      tcur = tn;
    }
  }
  for (int k = 0; any && !PF; ++k) {
    const int buf = k & 1;
    const int tn = tile_id(k + 1);
    const bool more = tn >= 0;
    const Patch Pn = patch(more ? tn : tcur);
    const bool claim_now = dyn && k % CH == 0 && more && sup_id(k / CH + 1) >= 0;
    int claimed = 0;
    if (claim_now && tid == 0)
      claimed = __hip_atomic_fetch_add(a.claim + combo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (BNA) {
      int lz = lane;
      asm volatile("" : "+v"(lz));
      const int g_ = lz >> 4, i_ = lz & 15;
      fpp = i_ & 3;
      frr0 = 16 * (g_ >> 1) + 4 * (g_ & 1) + (i_ >> 2);
    }
    const uint32_t hbase = sbase + buf * STAGE, dbase = hbase + HBUF;
#pragma unroll
    for (int pr = 0; pr < PH; ++pr) {
      if (BNA && more && pr == BNA_ROW) {   // this thread's dA / z pieces (rows 0-1) have landed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bna_apply(Pn, buf ^ 1);
      }
      if (more && !(dbg & 2)) issue_row(Pn, pr, buf ^ 1);   // (wgrad_debug bit 1: no LDS-DMA after the prologue)
      bf16x8 fd[4], fx[4], fd8, fx8[2];
      if (NW == 8) {
        fd8 = frag(dbase, pr * PW, nb8 * 16);
        fx8[0] = frag(hbase, (pr + 2) * HW + 2, cb8 * 16);
        fx8[1] = frag(hbase, (pr + 2) * HW + 2, cb8 * 16 + 16);
      }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) fd[nb] = frag(dbase, pr * PW, nb * 16);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) fx[cb] = frag(hbase, (pr + dy) * HW + dx, cb * 16);
      // column block cb's MFMAs start as soon as its two reads (and the dY fragments) have landed
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        if (dbg & 8) {   // (wgrad_debug bit 3, timing only: the MFMAs do not wait for their fragments)
          if (cb == 3) lgkm_wait<0>();
        } else if (cb == 0) lgkm_wait<6>();
        else if (cb == 1) lgkm_wait<4>();
        else if (cb == 2) lgkm_wait<2>();
        else lgkm_wait<0>();
        prio_hi<ADP_PRIO_WGRAD>();
        if (NW == 8 && cb == 0) {
          acc8[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd8, fx8[0], acc8[0], 0, 0, 0);
          acc8[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd8, fx8[1], acc8[1], 0, 0, 0);
        }
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          acc[nb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[nb], fx[cb], acc[nb][cb], 0, 0, 0);
        prio_lo<ADP_PRIO_WGRAD>();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next patch landed
    if (claim_now && tid == 0) ring[(k / CH + 2) & 3] = claimed;   // (slot of super-patch s - 2: long done)
    if (!(dbg & 4)) W64_BAR();                          // and nobody reads this buffer any more (bit 2: timing only)
    if (!more) break;
    tcur = tn;
  }
  if (dyn && tid == 0) claim_block_done(a.claim, combos, gridDim.x);   // (every claim of the block has returned)
  if (!any && !a.part) return;   // (dyn: a block that started late found the work taken; a slab gets its zeros)
  if (ADP_DBG(a) & 1) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) asm volatile("" ::"v"(acc[nb][cb]));
    asm volatile("" ::"v"(acc8[0]), "v"(acc8[1]));
    return;
  }
  // dW[n][tap * 64 + c] += acc: each wave's 16-row blocks through LDS, out as 16-B pieces (16 lanes per 256-B row,
  // four rows per instruction; round 5: a quarter of the row form's store instructions, which all blocks issue at
  // once at the end of the launch). Three forms (launcher): f32 atomics into dW; plain stores into this block's slab
  // (block index lin of its combination: a fixed-order reduce launch adds the slabs into dW, so the result does not
  // depend on the order the blocks finish); or, with one block per combination, dW += partial by plain load + store
  // (the block owns those dW elements)
  constexpr int ES = 68;
  float* blk = reinterpret_cast<float*>(smem) + wave * 16 * ES;
  const int col = lane & 15, rq = (lane >> 4) * 4;
  float* dW = a.part ? a.part + ((size_t)lin * a.Nout + (size_t)nblk * 64) * a.Kpad : a.dW + (size_t)nblk * 64 * a.Kpad;
  // (the per-lane part of an address is a 32-bit offset, the row part wave-uniform)
  const int voff = wave * (a.CAs + a.CBs) + ch * 64 + col * 4 + (lane >> 4) * a.Kpad;
  const int lrd = (lane >> 4) * ES + col * 4;
  auto out = [&](auto put) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) blk[(rq + r) * ES + cb * 16 + col] = acc[nb][cb][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
      for (int j = 0; j < 4; ++j)
        put(dW + (size_t)(nb * 16 + j * 4) * a.Kpad + voff, *reinterpret_cast<const float4*>(blk + j * 4 * ES + lrd));
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
  };
  // this wave's eighth of tap 8: rows nb8 * 16 + rq + r, columns cb8 * 16 + {0..31}
  auto out8 = [&](auto put1) {
    if constexpr (NW == 8) {
      const int k8 = 8 * (a.CAs + a.CBs) + ch * 64 + cb8 * 16 + col;
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
        for (int r = 0; r < 4; ++r) put1(dW + (size_t)(nb8 * 16 + rq + r) * a.Kpad + k8 + 16 * j2, acc8[j2][r]);
    }
  };
  if (a.part) {
    out([](float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; });
    out8([](float* p, float v) { *p = v; });
  } else if (a.part_rmw) {
    out([](float* p, float4 v) {
      float4 o = *reinterpret_cast<float4*>(p);
      o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
      *reinterpret_cast<float4*>(p) = o;
    });
    out8([](float* p, float v) { *p += v; });
  } else {
    out([](float* p, float4 v) { atomicAdd(p, v.x); atomicAdd(p + 1, v.y); atomicAdd(p + 2, v.z); atomicAdd(p + 3, v.w); });
    out8([](float* p, float v) { atomicAdd(p, v); });
  }
}

// Round 6: the tap-pair form of the persistent halo weight gradient. The 8-wave form above gives
// each wave one tap (64 x 64) and an eighth of tap 8: per patch row a wave reads 22 fragments (the whole dY^T tile, its
// tap's halo rows, tap 8's share) for 18 MFMAs, and all eight waves read the same dY^T fragments -- the K loop alone ran
// at 1.3-1.5 PF, bounded by LDS fragment reads and their waits, not by the MFMA pipe. Here the two waves of a SIMD
// (w, w + 4) own the same 64 x 144 block of dW -- taps 2p and 2p + 1 and column block p of tap 8 (p = w & 3) -- and split
// the patch rows between them (wave w + 4h takes rows h, h + 2, h + 4, h + 6). One dY^T fragment set (4) then feeds 36
// MFMAs instead of 18: 26 reads per 36 MFMAs, 0.72 reads per MFMA against 1.22, and 104 fragment reads per CU and patch
// row against 176. The LDS images, their swizzle, the LDS-DMA schedule and the block's (chunk, output block) work split
// are those of the 8-wave form. Per row the reads of the next row are issued in two groups between the MFMA clusters
// (G1 = the next dY^T set, double-buffered, + three of the four tap-2p halo fragments after the tap-2p MFMAs; G2 = the
// last tap-2p fragment, the tap-2p+1 set and tap 8's fragment, double-buffered, after the tap-2p+1 MFMAs), so a row's
// first MFMA waits only for reads issued a cluster earlier, and at most 15 reads are ever outstanding (the lgkmcnt
// field). The two waves of a pair add their partial sums in LDS at the end (h = 0 + h = 1: fixed order,
// deterministic) and the block's 64 x 576 partial leaves in 16-B pieces in one of the three output forms of the 8-wave
// form (slab / dW += partial / f32 atomics). Static patch lists only, plain dY (no fused BatchNorm apply).
// LSPR: the next patch's LDS-DMA groups are issued over the wave's first LSPR local rows (of 4).
template <int LSPR, int PIPE>
__global__ __launch_bounds__(512, 1) void igemm_wgrad_halopair_kernel(WgradArgs a) {
  constexpr bool DB = PIPE == 1;
  constexpr int NTH = 512, RB = 128;
  // halo rows padded to HW = 36 pixels (the two extra columns are loaded and never read): rows pr and pr + 2 of a
  // patch then start 72 LDS rows apart, a multiple of 8, so a wave's four rows share one swizzle and one address set
  constexpr int PH = 8, PW = 32, HW = PW + 4, HROWS = (PH + 2) * HW;   // 360 halo pixels
  constexpr int HCH = HROWS * 8, DCH = PH * PW * 8;                     // 16-B chunks per image
  constexpr int GH = (HCH + NTH - 1) / NTH, GD = DCH / NTH;             // 6 halo + 4 dY groups per thread
  constexpr int HBUF = HROWS * RB, DBUF = PH * PW * RB;
  constexpr int STAGE = HBUF + DBUF;
  constexpr int ES = 9 * 64 + 4;   // epilogue: the block's [64][576] f32 partial, row stride 580 (bank-conflict-free)
  static_assert(64 * ES * 4 <= 2 * STAGE, "the epilogue image fits in the two stages");
  static_assert(GD * NTH == DCH && GH + GD == 10 && LSPR >= 1 && LSPR <= 9, "shape");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // timing-only ablations (ablation build, option wgrad_debug): bit 0 no output, bit 1 no LDS-DMA after the prologue,
  // bit 2 no patch barrier, bit 3 the MFMA clusters do not wait for their fragments, bit 4 no wait for the next patch's
  // LDS-DMA before the barrier
  const int dbg = ADP_DBG(a);
  // (the lane id is re-derived by v_mbcnt in a volatile statement wherever the loop needs it, so that neither it nor the
  // thread id occupies a register across the loop)
  auto lane_now = []() -> int {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
  };
  const int p = wave & 3, h = wave >> 2;   // tap pair, row parity
  prio_static<ADP_PRIO_WGRAD>(wave);
  const int t0 = 2 * p, t1 = 2 * p + 1;
  const int dy0 = t0 / 3, dx0 = t0 - 3 * (t0 / 3), dy1 = t1 / 3, dx1 = t1 - 3 * (t1 / 3);
  const int tx_n = a.Wo / PW, ty_n = a.Ho / PH;
  const int nch = (a.CAs + a.CBs) >> 6, combos = nch * (a.Nout >> 6);
  const int T = a.Nimg * tx_n * ty_n, G = gridDim.x / combos;
  const int lin0 = xcd_remap(blockIdx.x, gridDim.x);
  const int combo = lin0 % combos, lin = lin0 / combos;
  const int ch = combo % nch, nblk = combo / nch;
  const int nt = lin < T ? (T - lin + G - 1) / G : 0;
  const bool inA = ch * 64 < a.CAs;
  const int xcs = inA ? a.CAs : a.CBs;
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(inA ? a.srcA : a.srcB), 0, a.Nimg * a.Hs * a.Ws * xcs * 2, WG_RSRC3);
  const __amdgpu_buffer_rsrc_t rsD =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dY, 0, a.Nimg * a.Ho * a.Wo * a.dy_stride * 2, WG_RSRC3);
  const int us = a.up >> 1;
  const int xc0 = (inA ? ch * 64 : ch * 64 - a.CAs) * 2;
  struct Patch { int y0, x0, pbx, pbd; };
  auto patch = [&](int t) {
    Patch P;
    const int px = t % tx_n, r = t / tx_n;
    const int img = r / ty_n;
    P.y0 = (r % ty_n) * PH;
    P.x0 = px * PW;
    P.pbx = (img * a.Hs + (P.y0 >> us)) * a.Ws + (P.x0 >> us);
    P.pbd = (img * a.Ho + P.y0) * a.Wo + P.x0;
    return P;
  };
  // LDS-DMA group gi of this thread (0 .. GH-1 halo, GH .. GH+GD-1 dY): its per-thread constants are rebuilt from an
  // opaque copy of the thread id at each issue (a few VALU under the MFMAs) instead of 32 registers held across the loop
  // LDS-DMA groups (round 6: per-group arithmetic cut to a few VALU). Thread t moves 16-B chunk t & 7 of LDS row
  // r0 + 64 gi (r0 = t >> 3) of an image; that row's swizzle gsw(r0 + 64 gi) = gsw(r0), so the chunk's column on both
  // sides is the same for every group. The halo rows' source-grid (y, x) relative to the patch are packed 10 bits a group
  // in hpk (0x3ff: a row past the halo); a dY group's offset is one per-thread constant plus the patch and group part,
  // which goes into the buffer instruction's scalar offset. The upsample (us = 1) halves the halo's source coordinates:
  // (y0 + hy) >> 1 = (y0 >> 1) + ((hy + 2) >> 1) - 1 for the even patch origins.
  uint32_t hpk[2] = {0u, 0u};
#pragma unroll
  for (int gi = 0; gi < GH; ++gi) {
    const int hr = gi * 64 + (int)(threadIdx.x >> 3);
    const uint32_t v = hr < HROWS ? (uint32_t)((((hr / HW) + us) >> us) << 6 | (((hr % HW) + us) >> us)) : 0x3ffu;
    hpk[gi / 3] |= v << (10 * (gi % 3));
  }
  const int xcs2 = xcs * 2, dys2 = a.dy_stride * 2;
  auto issue_g = [&](const Patch& P, int gi, int buf) {
    const int l = lane_now();
    const int cpos = 16 * ((l & 7) ^ (2 * ((l >> 4) & 3)));   // (gsw(r0) = 2 ((r0 >> 1) & 3), r0 = 8 wave + (l >> 3))
    if (gi < GH) {
      const uint32_t v = (hpk[gi / 3] >> (10 * (gi % 3))) & 0x3ffu;
      if (gi < GH - 1 || v != 0x3ffu) {
        const int hyS = (int)(v >> 6), hxS = (int)(v & 63u);
        const bool ok = (unsigned)((P.y0 >> us) - 1 + hyS) < (unsigned)a.Hs && (unsigned)((P.x0 >> us) - 1 + hxS) < (unsigned)a.Ws;
        const unsigned off = ok ? (unsigned)((hyS * a.Ws + hxS + (P.pbx - a.Ws - 1)) * xcs2 + xc0 + cpos) : WG_OOB;
        wg_buf_lds16(rsX, smem + buf * STAGE + (size_t)(gi * NTH + wave * 64) * 16, off);
      }
    } else {
      const int i = gi - GH;
      const unsigned voff = (unsigned)(((wave >> 2) * a.Wo + 8 * (wave & 3) + (l >> 3)) * dys2 + nblk * 128 + cpos);
      wg_buf_lds16s(rsD, smem + buf * STAGE + HBUF + (size_t)(i * NTH + wave * 64) * 16, voff, (P.pbd + 2 * i * a.Wo) * dys2);
    }
  };
  // the groups of local row j: ceil(10 / LSPR) a row; each group's address arithmetic is fenced off from the next
  // (sched_barrier), so that their temporaries are not all live at once
  // (LSPR 1-4: ceil(10 / LSPR) groups a row over the first LSPR rows; 5, 6, 7: 4-3-3-0, 3-4-3-0, 3-3-4-0; 8: 3-4-3-0 with
  //  the waves of rows 1, 3, .. issuing after their row's first cluster, the others before it)
  auto issue_lrow = [&](const Patch& P, auto jc, int buf) {
    constexpr int j = decltype(jc)::value, NG = GH + GD, PER = LSPR <= 4 ? (NG + LSPR - 1) / LSPR : 3;
    constexpr int B0 = LSPR == 5 ? 4 : 3, B1 = LSPR == 6 || LSPR == 8 ? B0 + 4 : B0 + 3;
    constexpr int lo = LSPR <= 4 ? j * PER : j == 0 ? 0 : j == 1 ? B0 : j == 2 ? B1 : NG;
    constexpr int hi = LSPR <= 4 ? (j + 1) * PER : j == 0 ? B0 : j == 1 ? B1 : NG;
#pragma unroll
    for (int gi = 0; gi < NG; ++gi)
      if (gi >= lo && gi < hi) {
        issue_g(P, gi, buf);
        __builtin_amdgcn_sched_barrier(0);
      }
  };

  // LSPR 9: one group at each MFMA-cluster boundary of rows 0-2 (row start, after tap 2p, after tap 8; two at row 0's
  // start), so that no two pieces are issued back to back
  auto issue_slot = [&](const Patch& P, auto jc, auto bc, int buf) {
    constexpr int sl = 3 * decltype(jc)::value + decltype(bc)::value;
    constexpr int lo = sl == 0 ? 0 : sl + 1, hi = sl + 2;
    if constexpr (decltype(jc)::value < 3) {
#pragma unroll
      for (int gi = lo; gi < hi; ++gi) {
        issue_g(P, gi, buf);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // fragment addresses (per lane byte offsets into a stage; the 8-wave PF form's addressing): local row i is patch row
  // pr = h + 2i; the halo rows of (pr, tap) start at (pr + dy) HW + dx and dY rows at pr PW, so row i is the row-0
  // address + i 2 HW RB (halo) or + i 2 PW RB (dY): the same swizzle, immediate offsets
  auto xoff = [&](int C, int col0, int lz) -> uint32_t {
    const int g_ = lz >> 4, i_ = lz & 15;
    const int R = C + 16 * (g_ >> 1) + 4 * (g_ & 1) + (i_ >> 2);
    const int col = col0 + 4 * (i_ & 3), chunk = col >> 3, inb = (col & 7) * 2;
    return (uint32_t)(R * RB + ((chunk ^ gsw<RB>(R)) << 4) + inb);
  };
  const uint32_t sbase = lds_off(smem);
  // one address per operand family (its cb = 0 column block): the image rows are 128-B aligned and a 16-column block is
  // 2 of a row's 8 swizzled 16-B chunks, so column block cb of the same rows is at address ^ (cb << 5) (the XOR commutes
  // with the swizzle). The XOR sits inside the read statement, so the column-block addresses are never held in
  // registers (13 address registers would be, beside 144 accumulators and 72 fragment registers)
  uint32_t da, ha0, ha1, h8;
  auto addrs = [&](uint32_t hb) {
    const int lz = lane_now();
    da = hb + HBUF + xoff(h * PW, 0, lz);
    ha0 = hb + xoff((h + dy0) * HW + dx0, 0, lz);
    ha1 = hb + xoff((h + dy1) * HW + dx1, 0, lz);
    h8 = hb + xoff((h + 2) * HW + 2, p * 16, lz);
  };
  // fragment = two ds_read_b64_tr_b16 at immediate offsets OFF, OFF + 8 RB from address ad ^ (cb << 5)
  auto rd = [](uint32_t ad, auto cbc, auto off) -> bf16x8 {
    constexpr int cb = decltype(cbc)::value, OFF = decltype(off)::value;
    v4s16 lo, hi;
    if constexpr (cb == 0) {
      asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
                   : "=v"(lo), "=v"(hi) : "v"(ad), "n"(OFF), "n"(OFF + 8 * RB) : "memory");
    } else {
      uint32_t t;
      asm volatile("v_xor_b32 %2, %4, %3\n\tds_read_b64_tr_b16 %0, %2 offset:%5\n\tds_read_b64_tr_b16 %1, %2 offset:%6"
                   : "=v"(lo), "=v"(hi), "=&v"(t) : "v"(ad), "n"(cb << 5), "n"(OFF), "n"(OFF + 8 * RB) : "memory");
    }
    bf16x8 r;
    const bf16* l = reinterpret_cast<const bf16*>(&lo);
    const bf16* hh = reinterpret_cast<const bf16*>(&hi);
#pragma unroll
    for (int e = 0; e < 4; ++e) { r[e] = l[e]; r[4 + e] = hh[e]; }
    return r;
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;
  bf16x8 fd[4], fx0[4], fx1[4], f8;   // dY^T, tap 2p, tap 2p+1, tap 8 (one set each: 52 registers)
  // per local row the MFMA clusters run tap 2p, tap 8, tap 2p+1, and the next row's fragments are read as each cluster
  // frees its registers: after tap 2p the last tap-2p+1 fragment of this row (read a row late, see below) and the next
  // tap-2p set (10 reads), after tap 8 the next tap-8 fragment (2), after tap 2p+1 the next dY^T set and tap-2p+1
  // fragments 0-2 (14). At most 15 reads are ever outstanding (the lgkmcnt field); a row's first cluster waits for the
  // dY^T reads issued at the end of the previous row (the other wave of the SIMD multiplies meanwhile)
  auto load_a = [&](auto ic) {   // (after tap 2p) tap-2p+1 fragment 3 of row i - 1, tap-2p set of row i
    constexpr int i = decltype(ic)::value & 3;
    using HO = std::integral_constant<int, i * 2 * HW * RB>;
    using HP = std::integral_constant<int, ((i + 3) & 3) * 2 * HW * RB>;
    if constexpr (decltype(ic)::value > 0) fx1[3] = rd(ha1, C3{}, HP{});
    fx0[0] = rd(ha0, C0{}, HO{});
    fx0[1] = rd(ha0, C1{}, HO{});
    fx0[2] = rd(ha0, C2{}, HO{});
    fx0[3] = rd(ha0, C3{}, HO{});
  };
  auto load_b = [&](auto ic) {   // (after tap 8) tap-8 fragment of row i
    constexpr int i = decltype(ic)::value & 3;
    using HO = std::integral_constant<int, i * 2 * HW * RB>;
    f8 = rd(h8, C0{}, HO{});
  };
  auto load_c = [&](auto ic) {   // (after tap 2p+1) dY^T set and tap-2p+1 fragments 0-2 of row i
    constexpr int i = decltype(ic)::value & 3;
    using DO = std::integral_constant<int, i * 2 * PW * RB>;
    using HO = std::integral_constant<int, i * 2 * HW * RB>;
    fd[0] = rd(da, C0{}, DO{});
    fd[1] = rd(da, C1{}, DO{});
    fd[2] = rd(da, C2{}, DO{});
    fd[3] = rd(da, C3{}, DO{});
    fx1[0] = rd(ha1, C0{}, HO{});
    fx1[1] = rd(ha1, C1{}, HO{});
    fx1[2] = rd(ha1, C2{}, HO{});
  };
  // DB: the dY^T set double-buffered by local row parity (fd for even rows, fe for odd ones), so the next row's set is
  // read right after this row's tap-2p cluster: G1 = the next dY^T set + tap-2p fragments 0-2 (14 reads, after tap 2p),
  // G1b = tap-2p fragment 3 + tap 8 (4, after tap 8), G2 = the tap-2p+1 set (8, after tap 2p+1); a row's first cluster
  // then waits for reads issued two clusters earlier
  bf16x8 fe[4];
  auto db_g1 = [&](auto ic) {
    constexpr int i = decltype(ic)::value & 3;
    using DO = std::integral_constant<int, i * 2 * PW * RB>;
    using HO = std::integral_constant<int, i * 2 * HW * RB>;
    bf16x8* d = (i & 1) ? fe : fd;
    d[0] = rd(da, C0{}, DO{});
    d[1] = rd(da, C1{}, DO{});
    d[2] = rd(da, C2{}, DO{});
    d[3] = rd(da, C3{}, DO{});
    fx0[0] = rd(ha0, C0{}, HO{});
    fx0[1] = rd(ha0, C1{}, HO{});
    fx0[2] = rd(ha0, C2{}, HO{});
  };
  auto db_g1b = [&](auto ic) {
    constexpr int i = decltype(ic)::value & 3;
    using HO = std::integral_constant<int, i * 2 * HW * RB>;
    fx0[3] = rd(ha0, C3{}, HO{});
    f8 = rd(h8, C0{}, HO{});
  };
  auto db_g2 = [&](auto ic) {
    constexpr int i = decltype(ic)::value & 3;
    using HO = std::integral_constant<int, i * 2 * HW * RB>;
    fx1[0] = rd(ha1, C0{}, HO{});
    fx1[1] = rd(ha1, C1{}, HO{});
    fx1[2] = rd(ha1, C2{}, HO{});
    fx1[3] = rd(ha1, C3{}, HO{});
  };

  // The MFMAs are inline asm accumulating in place ("+v": D = C, one register tuple per accumulator for the whole
  // loop). With the builtin, hipcc rotated the accumulators through other registers (94 of 144 MFMAs had D != C), which
  // at 144 accumulators and 52 fragment registers left no room and spilled. Hazards of the asm form: the A / B
  // fragments are asm LDS reads this code waits for itself (no VALU writes them: tests/test_isa.py), an accumulator is
  // read as C one cluster (>= 4 MFMAs) after the MFMA that wrote it, the zero-initialising moves are fenced off from the
  // first MFMA (acc_fence), and the epilogue's first VALU reads of the last cluster's results come after s_nops.
  auto mma = [](f32x4& c, const bf16x8& x, const bf16x8& y) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(x), "v"(y));
  };
  f32x4 acc0[4][4], acc1[4][4], acc8[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0[i][j] = acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+v"(acc0[i][j]), "+v"(acc1[i][j]));
    }
    acc8[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("" : "+v"(acc8[i]));
  }
  asm volatile("s_nop 4" ::: "memory");   // (acc_fence: VALU writes of the accumulators -> MFMA reads of them as C)

  const bool any = nt > 0;
  if (any) {
    const Patch P0 = patch(lin);
#pragma unroll
    for (int gi = 0; gi < GH + GD; ++gi) issue_g(P0, gi, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W64_BAR();
    addrs(sbase);
    if constexpr (PIPE == 2) {   // row 0's sets in the steady-state order (16, 2, 8 reads)
      fx0[0] = rd(ha0, C0{}, std::integral_constant<int, 0>{});
      fd[0] = rd(da, C0{}, std::integral_constant<int, 0>{});
      fx0[1] = rd(ha0, C1{}, std::integral_constant<int, 0>{});
      fd[1] = rd(da, C1{}, std::integral_constant<int, 0>{});
      fx0[2] = rd(ha0, C2{}, std::integral_constant<int, 0>{});
      fd[2] = rd(da, C2{}, std::integral_constant<int, 0>{});
      fx0[3] = rd(ha0, C3{}, std::integral_constant<int, 0>{});
      fd[3] = rd(da, C3{}, std::integral_constant<int, 0>{});
      lgkm_wait<13>();
      f8 = rd(h8, C0{}, std::integral_constant<int, 0>{});
      lgkm_wait<7>();
      db_g2(std::integral_constant<int, 0>{});
    } else if constexpr (DB) {
      db_g1(std::integral_constant<int, 0>{});
      lgkm_wait<11>();   // (at most 15 reads in flight)
      db_g1b(std::integral_constant<int, 0>{});
      lgkm_wait<7>();
      db_g2(std::integral_constant<int, 0>{});
    } else {
      load_a(std::integral_constant<int, 0>{});   // (the steady-state issue order; row 0's fx1[3] comes with A(1))
      load_b(std::integral_constant<int, 0>{});
      lgkm_wait<1>();   // (at most 15 reads in flight)
      load_c(std::integral_constant<int, 0>{});
    }
  }
  for (int k = 0; k < nt; ++k) {
    const int buf = k & 1;
    const bool more = k + 1 < nt;
    const Patch Pn = patch(more ? lin + (k + 1) * G : lin);
    auto row = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (LSPR == 9) {
        if (more && !(dbg & 2)) issue_slot(Pn, ic, C0{}, buf ^ 1);
      } else if constexpr (i < (LSPR <= 4 ? LSPR : 3)) {
        if (more && !(dbg & 2) && (LSPR != 8 || h == 0)) issue_lrow(Pn, ic, buf ^ 1);
      }
      // issue order up to here: [A(i): fx1(i-1)[3] (not for row 0 of a patch: read before the patch barrier), fx0(i)]
      // [B(i): f8(i)] [C(i): fd(i), fx1(i)[0..2]]; row i needs fd, fx0, f8: only fx1(i)[0..2] (6) may be younger
      if (!(dbg & 8)) lgkm_wait<6>();
      prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          mma(acc0[nb][cb], fd[nb], fx0[cb]);
      prio_lo<ADP_PRIO_WGRAD>();
      if constexpr (LSPR == 8 && i < 3) {
        if (more && !(dbg & 2) && h == 1) issue_lrow(Pn, ic, buf ^ 1);
      }
      if constexpr (LSPR == 9) {
        if (more && !(dbg & 2)) issue_slot(Pn, ic, C1{}, buf ^ 1);
      }
      if constexpr (i == 3) {
        lgkm_wait<0>();                                      // every read of this buffer but fx1(3)[3] has returned;
        if (!(dbg & 16)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's next-patch pieces landed
        fx1[3] = rd(ha1, C3{}, std::integral_constant<int, 3 * 2 * HW * RB>{});
        lgkm_wait<0>();                                      // (and that one: the buffer is read out)
        if (!(dbg & 4)) W64_BAR();
        if (more) {                                          // the next patch's rows, from the other buffer
          addrs(sbase + (buf ^ 1) * STAGE);
          load_a(std::integral_constant<int, 0>{});
        }
      } else {
        lgkm_wait<5>();   // (C(i) has had the tap-2p cluster: at most 15 reads in flight after A(i + 1))
        load_a(std::integral_constant<int, i + 1>{});
      }
      prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) mma(acc8[nb], fd[nb], f8);
      prio_lo<ADP_PRIO_WGRAD>();
      if constexpr (LSPR == 9) {
        if (more && !(dbg & 2)) issue_slot(Pn, ic, C2{}, buf ^ 1);
      }
      if (i < 3 || more) {
        lgkm_wait<13>();
        load_b(std::integral_constant<int, i + 1>{});
      }
      // fx1(i) complete: younger are A(i + 1) minus its first fragment (8) and B(i + 1) (2)
      if (dbg & 8) {
      } else if (i < 3 || more) lgkm_wait<10>();
      else lgkm_wait<0>();
      prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          mma(acc1[nb][cb], fd[nb], fx1[cb]);
      prio_lo<ADP_PRIO_WGRAD>();
      if (i < 3 || more) {
        lgkm_wait<1>();   // (A(i + 1) and B(i + 1) issued a cluster ago)
        load_c(std::integral_constant<int, i + 1>{});
      }
    };
    auto row_db = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i < (LSPR <= 4 ? LSPR : 3)) {
        if (more && !(dbg & 2)) issue_lrow(Pn, ic, buf ^ 1);
      }
      const bf16x8* d = (i & 1) ? fe : fd;
      // issue order: [G1(i)] [G1b(i)] [G2(i)]: row i's first clusters need G1 and G1b, G2 (8) may be younger
      if (!(dbg & 8)) lgkm_wait<8>();
      prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          mma(acc0[nb][cb], d[nb], fx0[cb]);
      prio_lo<ADP_PRIO_WGRAD>();
      lgkm_wait<0>();   // G2(i) too (issued a cluster ago): nothing of row i is in flight
      if constexpr (i == 3) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's pieces of the next patch have landed
        if (!(dbg & 4)) W64_BAR();
        if (more) addrs(sbase + (buf ^ 1) * STAGE);        // the next patch's rows, from the other buffer
      }
      if (i < 3 || more) db_g1(std::integral_constant<int, i + 1>{});
      prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) mma(acc8[nb], d[nb], f8);
      prio_lo<ADP_PRIO_WGRAD>();
      if (i < 3 || more) {
        lgkm_wait<11>();
        db_g1b(std::integral_constant<int, i + 1>{});
      }
      prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          mma(acc1[nb][cb], d[nb], fx1[cb]);
      prio_lo<ADP_PRIO_WGRAD>();
      if (i < 3 || more) {
        lgkm_wait<7>();
        db_g2(std::integral_constant<int, i + 1>{});
      }
    };
    // PIPE 2: the next row's fragments read inside the clusters, each right after the MFMAs that free its registers
    // (dY^T double-buffered): after tap 2p column block cb, its next-row fragment and the next dY^T block cb (4 reads),
    // after tap 8 its next fragment (2), after tap 2p+1 column block cb its next fragment (2). Every fragment is read at
    // least a cluster before its first MFMA. Row 3 needs no LDS reads (its fragments were read during row 2), so the
    // patch barrier sits at its start and its clusters read the next patch's first row from the other buffer.
    auto row_il = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      using NI = std::integral_constant<int, (i + 1) & 3>;
      using DO = std::integral_constant<int, NI::value * 2 * PW * RB>;
      using HO = std::integral_constant<int, NI::value * 2 * HW * RB>;
      if constexpr (i < (LSPR <= 4 ? LSPR : 3)) {
        if (more && !(dbg & 2)) issue_lrow(Pn, ic, buf ^ 1);
      }
      const bf16x8* cur = (i & 1) ? fe : fd;
      bf16x8* nxt = (i & 1) ? fd : fe;
      if constexpr (i == 3) {
        lgkm_wait<0>();                                      // row 3's fragments have landed: the buffer is read out,
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // and this thread's pieces of the next patch have landed
        if (!(dbg & 4)) W64_BAR();
        if (more) addrs(sbase + (buf ^ 1) * STAGE);
      } else if (!(dbg & 8)) {
        lgkm_wait<10>();   // row i's dY^T and tap-2p sets (read during row i - 1's first cluster) have landed
      }
      const bool ld = i < 3 || more;
      auto tap0_cb = [&](auto cbc) {
        constexpr int cb = decltype(cbc)::value;
        prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) mma(acc0[nb][cb], cur[nb], fx0[cb]);
        prio_lo<ADP_PRIO_WGRAD>();
        if (ld) {
          if constexpr (cb > 0) lgkm_wait<11>();   // (at most 15 in flight; by cb = 1 this row's f8, by cb = 3 its fx1)
          fx0[cb] = rd(ha0, cbc, HO{});
          nxt[cb] = rd(da, cbc, DO{});
        }
      };
      tap0_cb(C0{});
      tap0_cb(C1{});
      tap0_cb(C2{});
      tap0_cb(C3{});
      prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) mma(acc8[nb], cur[nb], f8);
      prio_lo<ADP_PRIO_WGRAD>();
      if (ld) {
        lgkm_wait<13>();
        f8 = rd(h8, C0{}, HO{});
      }
      auto tap1_cb = [&](auto cbc) {
        constexpr int cb = decltype(cbc)::value;
        prio_hi<ADP_PRIO_WGRAD>();
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) mma(acc1[nb][cb], cur[nb], fx1[cb]);
        prio_lo<ADP_PRIO_WGRAD>();
        if (ld) {
          lgkm_wait<13>();
          fx1[cb] = rd(ha1, cbc, HO{});
        }
      };
      tap1_cb(C0{});
      tap1_cb(C1{});
      tap1_cb(C2{});
      tap1_cb(C3{});
    };
    if constexpr (PIPE == 2) {
      row_il(std::integral_constant<int, 0>{});
      row_il(std::integral_constant<int, 1>{});
      row_il(std::integral_constant<int, 2>{});
      row_il(std::integral_constant<int, 3>{});
    } else if constexpr (DB) {
      row_db(std::integral_constant<int, 0>{});
      row_db(std::integral_constant<int, 1>{});
      row_db(std::integral_constant<int, 2>{});
      row_db(std::integral_constant<int, 3>{});
    } else {
      row(std::integral_constant<int, 0>{});
      row(std::integral_constant<int, 1>{});
      row(std::integral_constant<int, 2>{});
      row(std::integral_constant<int, 3>{});
    }
  }
  // the last cluster's results (tap 2p+1, column block 3: its last four MFMAs) before any VALU reads them
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc1[0][3]), "+v"(acc1[1][3]), "+v"(acc1[2][3]), "+v"(acc1[3][3]));
  if (!any && !a.part) return;   // (a slab gets its zeros)
  if (dbg & 1) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) asm volatile("" ::"v"(acc0[nb][cb]), "v"(acc1[nb][cb]));
      asm volatile("" ::"v"(acc8[nb]));
    }
    return;
  }
  // epilogue: waves h = 1 put their partial in the [64][ES] image, waves h = 0 add it to theirs (h0 + h1) and put the
  // sum back, then the whole block writes the 64 x 576 partial out in 16-B pieces. (Every LDS read of the loop has
  // returned before the last patch barrier, and no LDS-DMA is in flight after it.)
  float* img = reinterpret_cast<float*>(smem);
  const int lane = lane_now(), tid = wave * 64 + lane;
  const int col = lane & 15, rq = (lane >> 4) * 4;
  auto each = [&](auto fn) {   // (tile, element) -> image index, for the 36 tiles of this pair
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rowi = (nb * 16 + rq + r) * ES + cb * 16 + col;
          fn(acc0[nb][cb][r], rowi + t0 * 64);
          fn(acc1[nb][cb][r], rowi + t1 * 64);
        }
#pragma unroll
      for (int r = 0; r < 4; ++r) fn(acc8[nb][r], (nb * 16 + rq + r) * ES + 8 * 64 + p * 16 + col);
    }
  };
  if (h == 1) each([&](float v, int ix) { img[ix] = v; });
  __syncthreads();
  if (h == 0) each([&](float v, int ix) { img[ix] = v + img[ix]; });
  __syncthreads();
  const int cin = a.CAs + a.CBs;
  float* dW = a.part ? a.part + ((size_t)lin * a.Nout + (size_t)nblk * 64) * a.Kpad : a.dW + (size_t)nblk * 64 * a.Kpad;
#pragma unroll 2
  for (int j = 0; j < 64 * 144 / NTH; ++j) {
    const int idx = j * NTH + tid, n = idx / 144, r = idx - 144 * (idx / 144), tap = r >> 4, c4 = r & 15;
    const float4 v = *reinterpret_cast<const float4*>(img + n * ES + tap * 64 + c4 * 4);
    float* d = dW + (size_t)n * a.Kpad + tap * cin + ch * 64 + c4 * 4;
    if (a.part) {
      *reinterpret_cast<float4*>(d) = v;
    } else if (a.part_rmw) {
      float4 o = *reinterpret_cast<float4*>(d);
      o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
      *reinterpret_cast<float4*>(d) = o;
    } else {
      atomicAdd(d, v.x); atomicAdd(d + 1, v.y); atomicAdd(d + 2, v.z); atomicAdd(d + 3, v.w);
    }
  }
}



template __global__ void igemm_wgrad_halopair_kernel<6, 0>(WgradArgs);
template __global__ void igemm_wgrad_halopair_kernel<6, 1>(WgradArgs);
template __global__ void igemm_wgrad_halopair_kernel<6, 2>(WgradArgs);
template __global__ void igemm_wgrad_halopair_kernel<4, 0>(WgradArgs);
template __global__ void igemm_wgrad_halopair_kernel<8, 0>(WgradArgs);
template __global__ void igemm_wgrad_halopair_kernel<9, 0>(WgradArgs);

// Weight gradient of the input layers (one 8-channel source, 3x3 stride 1, 64 outputs; K = 72): an
// HBM-bound pass over dY (128 B per pixel) and X (16 B per pixel). Persistent, one block per CU, a
// 3-stage LDS-DMA ring of 8 x 32 patches (34 x 10 halo of 16-B pixels + the 256 x 64 dY tile); wave w
// takes patch row w as one 32-pixel MFMA k step for the whole 64 x 80 product: A = dY^T fragments,
// B = "virtual" fragments whose 16 columns are two taps x 8 channels (column j = k = 8 tap + c), read
// with ds_read_b64_tr_b16 from the halo rows of the two taps (the tenth tap column reads a zero row).
// Wave partials meet in LDS (ds_add_f32); one f32 atomic per dW element per block.
// BNA (adp_conv_wgrad_bn on the input layer, unet_bn enc0_conv1): dY = bn_bwd_apply(dA, z) is computed
// here instead of read. Two patches ahead, dA goes by LDS-DMA into the slots of the stage's dY image dY
// would have taken and z into registers (two register sets, the loop unrolled by two); at its patch each
// thread applies bn_bwd_apply_kernel's arithmetic (same rounding: bit-identical dz) to its own slots in
// place. dz is not stored: the launcher takes this form only for dY = NULL (the input layer has no data
// gradient, so nothing reads dz). Replaces the apply pass (dA + z read, dz written) and the dz read.
template <bool BNA>
__global__ __launch_bounds__(512, 1) void igemm_wgrad_cin8_kernel(WgradArgs a) {
  constexpr int NTH = 512, PH = 8, PW = 32, HW = PW + 2, HROWS = (PH + 2) * HW;   // 340 halo pixels
  constexpr int HSLOT = NTH * 16;                  // halo region: one 16-B row per thread (rows >= 340: 0)
  constexpr int GD = PH * PW * 8 / NTH;            // dY 16-B chunks per thread
  constexpr int STAGE = HSLOT + PH * PW * 128, NST = 3;
  constexpr int ZROW = HROWS;                      // an all-zero halo row
  constexpr int CST = BNA ? 6 * 64 * 4 : 0;        // BNA: per-channel scale, shift, mean, P, Q, R
  static_assert(NST * STAGE + CST <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NST * STAGE + CST];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // = patch row
  const int tx_n = a.Wo / PW, ty_n = a.Ho / PH;
  const int T = a.Nimg * tx_n * ty_n, G = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, G);
  const int nt = lin < T ? (T - lin + G - 1) / G : 0;
  const bf16* X = reinterpret_cast<const bf16*>(a.srcA);
  const bf16* D = reinterpret_cast<const bf16*>(a.dY);

  auto patch_origin = [&](int k, int& img, int& y0, int& x0) {
    const int t = lin + k * G;
    const int px = t % tx_n, r = t / tx_n;
    y0 = (r % ty_n) * PH; img = r / ty_n; x0 = px * PW;
  };
  auto issue_halo = [&](int k) {   // 1 LDS-DMA instruction per thread
    int img, y0, x0;
    patch_origin(k, img, y0, x0);
    unsigned char* st = smem + (k % NST) * STAGE;
    const int hr = tid;
    const int gy = y0 - 1 + hr / HW, gx = x0 - 1 + hr % HW;
    const bool ok = hr < HROWS && gy >= 0 && gy < a.Hs && gx >= 0 && gx < a.Ws;
    const void* p = ok ? (const void*)(X + (size_t)((img * a.Hs + gy) * a.Ws + gx) * a.CAs)
                       : (const void*)wg64_zero_page;
    wg_glds16(p, st + wave * 64 * 16);
  };
  // element offset of this thread's dY chunk i of patch k (the same for dA, z and dz)
  auto chunk_off = [&](int k, int i) {
    int img, y0, x0;
    patch_origin(k, img, y0, x0);
    const int idx = i * NTH + tid;
    const int pr = idx >> 3, pos = idx & 7;
    const size_t m = (size_t)(img * a.Ho + y0 + (pr >> 5)) * a.Wo + x0 + (pr & 31);
    return m * a.dy_stride + 8 * (pos ^ gsw<128>(pr));
  };
  auto issue = [&](int k) {   // 1 + GD LDS-DMA instructions per thread
    issue_halo(k);
    unsigned char* st = smem + (k % NST) * STAGE;
#pragma unroll
    for (int i = 0; i < GD; ++i)
      wg_glds16(D + chunk_off(k, i), st + HSLOT + (size_t)(i * NTH + wave * 64) * 16);
  };
  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, pp = ii & 3;
  const int rr0 = 16 * (g >> 1) + 4 * (g & 1) + q;
  auto frag2 = [&](uint32_t a0, uint32_t a1) {
    const v4s16 lo = ds_tr16(a0), hi = ds_tr16(a1);
    bf16x8 r;
    const bf16* l = reinterpret_cast<const bf16*>(&lo);
    const bf16* h = reinterpret_cast<const bf16*>(&hi);
#pragma unroll
    for (int e = 0; e < 4; ++e) { r[e] = l[e]; r[4 + e] = h[e]; }
    return r;
  };

  f32x4 acc[4][5];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t sbase = lds_off(smem);
  auto compute = [&](int k) {   // patch k of stage k % NST, landed and visible to every wave
    const uint32_t hb = sbase + (k % NST) * STAGE, db = hb + HSLOT;
    bf16x8 fd[4], fx[5];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {   // A = dY^T: rows = 16 output channels, k = the wave's 32 pixels
      const int col = nb * 16 + 4 * pp, chunk = col >> 3, inb = (col & 7) * 2;
      const int R0 = wave * PW + rr0, R1 = R0 + 8;
      fd[nb] = frag2(db + R0 * 128 + ((chunk ^ gsw<128>(R0)) << 4) + inb,
                     db + R1 * 128 + ((chunk ^ gsw<128>(R1)) << 4) + inb);
    }
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) {   // B columns 16 kb .. 16 kb + 15 = taps 2 kb, 2 kb + 1 x 8 channels
      const int tap = 2 * kb + (pp >> 1), cb = (pp & 1) * 8;
      const int dy = tap / 3, dx = tap - 3 * (tap / 3);
      const int h0 = tap < 9 ? (wave + dy) * HW + dx + rr0 : ZROW;
      const int h1 = tap < 9 ? h0 + 8 : ZROW;
      fx[kb] = frag2(hb + h0 * 16 + cb, hb + h1 * 16 + cb);
    }
    lgkm_wait<0>();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int kb = 0; kb < 5; ++kb)
        acc[nb][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[nb], fx[kb], acc[nb][kb], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (!BNA) {
    if (nt > 0) issue(0);
    if (nt > 1) issue(1);
    for (int k = 0; k < nt; ++k) {
      if (k + 2 < nt) {
        issue(k + 2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (1 + GD)) : "memory");
      } else if (k + 1 < nt) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 + GD) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      W64_BAR();   // patch k landed for every wave
      compute(k);
      W64_BAR();   // stage k % NST is free for patch k + 3
    }
  } else {
    // per-channel constants of bn_bwd_apply_kernel; this thread's chunks all hold channel group bcg
    // (gsw<128> depends on row bits 1-2, which the thread's rows i * 64 + tid / 8 share)
    const __amdgpu_buffer_rsrc_t rsDA = __builtin_amdgcn_make_buffer_rsrc((void*)a.bna_dA, 0, a.M * a.dy_stride * 2, WG_RSRC3);
    const __amdgpu_buffer_rsrc_t rsZ = __builtin_amdgcn_make_buffer_rsrc((void*)a.bna_z, 0, a.M * a.dy_stride * 2, WG_RSRC3);
    const int bcg = (tid & 7) ^ gsw<128>(tid >> 3);
    float* bk = reinterpret_cast<float*>(smem + NST * STAGE);
    if (tid < 64) {
      const float kk = a.bna_gamma[tid] * a.bna_invstd[tid];
      bk[0 * 64 + tid] = a.bna_sc[tid];
      bk[1 * 64 + tid] = a.bna_sh[tid];
      bk[2 * 64 + tid] = a.bna_mean[tid];
      bk[3 * 64 + tid] = kk;
      bk[4 * 64 + tid] = -kk * a.bna_invstd[tid] * a.bna_dgamma[tid] * a.bna_inv_count;
      bk[5 * 64 + tid] = -kk * a.bna_dbeta[tid] * a.bna_inv_count;
    }
    __syncthreads();
    typedef unsigned v4u_c __attribute__((ext_vector_type(4)));
    // dA by LDS-DMA into the stage's dY image (the slots this thread would have DMA'd dY into), z into
    // registers (2 GD + 1 vector-memory ops per patch with the halo)
    auto load_ops = [&](int k, v4u_c (&zr)[GD]) {
      issue_halo(k);
      unsigned char* st = smem + (k % NST) * STAGE;
#pragma unroll
      for (int i = 0; i < GD; ++i) {
        const unsigned off = (unsigned)(chunk_off(k, i) * 2);
        wg_buf_lds16(rsDA, st + HSLOT + (size_t)(i * NTH + wave * 64) * 16, off);
        zr[i] = __builtin_amdgcn_raw_buffer_load_b128(rsZ, off, 0, 0);
      }
    };
    // dz of this thread's slots of patch k, in place (its own DMA wrote them: no barrier needed before);
    // 8 B at a time (no 16-B result held: registers)
    auto apply = [&](int k, const v4u_c (&zr)[GD]) {
      const uint32_t dimg = sbase + (k % NST) * STAGE + HSLOT;
#pragma unroll
      for (int half = 0; half < 2; ++half) {   // 4 channels at a time: bounds the registers held
        float c[6][4];
#pragma unroll
        for (int qq = 0; qq < 6; ++qq) {
          const float4 v = wg_lds_f4(sbase + NST * STAGE + (qq * 64 + bcg * 8 + 4 * half) * 4);
          c[qq][0] = v.x; c[qq][1] = v.y; c[qq][2] = v.z; c[qq][3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < GD; ++i) {
          const uint32_t slot = dimg + (uint32_t)(i * NTH + tid) * 16 + 8 * half;
          const v2u32_w dv = wg_lds_r8(slot);
          const unsigned zw[2] = {zr[i][2 * half], zr[i][2 * half + 1]};
          const bf16* d = reinterpret_cast<const bf16*>(&dv);
          const bf16* zz = reinterpret_cast<const bf16*>(zw);
          bf16 o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {   // bn_bwd_apply_kernel's arithmetic and rounding
            const float zf = (float)zz[j];
            const float dbv = fmaf(zf, c[0][j], c[1][j]) > 0.f ? (float)d[j] : 0.f;
            o[j] = (bf16)fmaf(c[3][j], dbv, fmaf(c[4][j], zf - c[2][j], c[5][j]));
          }
          wg_lds_w8(slot, *reinterpret_cast<const v2u32_w*>(o));
        }
      }
    };
    constexpr int OPS = 1 + 2 * GD;   // vector-memory ops of one patch's loads
    v4u_c z0[GD], z1[GD];
    // patch k: its loads (issued two patches ago) retired, its dz into the stage, the loads of patch
    // k + 2 into the freed registers, then the multiply. Ops younger than patch k's loads at the wait: the
    // loads of patch k + 1 (OPS)
    auto step = [&](int k, v4u_c (&zr)[GD]) {
      if (k + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      apply(k, zr);
      if (k + 2 < nt) load_ops(k + 2, zr);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      W64_BAR();   // patch k's halo and dz image visible to every wave
      compute(k);
      W64_BAR();   // stage k % NST is free for patch k + 3
    };
    if (nt > 0) load_ops(0, z0);
    if (nt > 1) load_ops(1, z1);
    for (int k = 0; k < nt; k += 2) {
      step(k, z0);
      if (k + 1 < nt) step(k + 1, z1);
    }
  }
  if (nt == 0 && !a.part) return;   // (a slab gets its zeros)
  // wave partials -> LDS [64][80] f32, added in wave order (deterministic) -> this block's slab [64][Kpad] (plain
  // stores, zeros past k = 72; the launcher's fixed-order reduce adds the slabs into dW) or one f32 atomic per
  // element into dW[n][k], k < 72
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* red = reinterpret_cast<float*>(smem);
  __syncthreads();
  const int col = lane & 15, rq = (lane >> 4) * 4;
  for (int w = 0; w < NTH / 64; ++w) {
    if (wave == w) {   // (a lane's (row, column) elements are its own: no race inside the wave)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int kb = 0; kb < 5; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* e = red + (nb * 16 + rq + r) * 80 + kb * 16 + col;
            *e = w == 0 ? acc[nb][kb][r] : *e + acc[nb][kb][r];
          }
    }
    __syncthreads();
  }
  if (a.part) {
    float* slab = a.part + (size_t)blockIdx.x * 64 * a.Kpad;
    for (int i = tid; i < 64 * a.Kpad; i += NTH) {
      const int n = i / a.Kpad, kk = i - n * a.Kpad;
      slab[i] = kk < 72 ? red[n * 80 + kk] : 0.f;
    }
    return;
  }
  for (int i = tid; i < 64 * 72; i += NTH) {
    const int n = i / 72, kk = i - n * 72;
    atomicAdd(a.dW + (size_t)n * a.Kpad + kk, red[n * 80 + kk]);
  }
}

#undef W64_BAR

// (explicit instantiations: without them hipcc emitted no host stub for the <false> form)
template __global__ void igemm_wgrad_cin8_kernel<false>(WgradArgs);
template __global__ void igemm_wgrad_cin8_kernel<true>(WgradArgs);

// dW[n][k] += sum over the splits of part[split][n][k] (n < Nout, k < K = Kpad), 4 floats per thread.
// blockIdx.y = group of SG consecutive splits: one group adds with a plain read-modify-write, several
// groups add their group sums with f32 atomics (SG x fewer atomic bytes than the per-block epilogue).
constexpr int WG_SG = 32;
__global__ void wgrad_reduce_kernel(int splits, size_t slab, const float4* part, float4* dW) {
  const size_t n4 = slab / 4;
  const int s0 = blockIdx.y * WG_SG, s1 = min(splits, s0 + WG_SG);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 acc = part[(size_t)s0 * n4 + i];
    for (int s = s0 + 1; s < s1; ++s) {
      const float4 v = part[(size_t)s * n4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (gridDim.y == 1) {
      float4 d = dW[i];
      d.x += acc.x; d.y += acc.y; d.z += acc.z; d.w += acc.w;
      dW[i] = d;
    } else {
      float* d = reinterpret_cast<float*>(dW + i);
      atomicAdd(d, acc.x); atomicAdd(d + 1, acc.y); atomicAdd(d + 2, acc.z); atomicAdd(d + 3, acc.w);
    }
  }
}

// Fixed-order sum of G partial slabs into dW (dW[i] += sum_g part[g][i]): a 256-thread block takes 32 float4
// elements; its 8 thread groups sum consecutive slab ranges [g0, g1) in order, and group 0 adds the 8 range sums in
// order. The association depends only on G, so two runs give the same bits (unlike f32 atomics).
__device__ __forceinline__ void slab_reduce_block(int G, size_t n4, const float4* __restrict__ part,
                                                  float4* __restrict__ dW, int blk, float4 (&ps)[8][32]) {
  const int e = threadIdx.x & 31, j = threadIdx.x >> 5;
  const size_t i = (size_t)blk * 32 + e;
  const int per = (G + 7) / 8, g0 = min(G, j * per), g1 = min(G, g0 + per);
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    int g = g0;
    for (; g + 4 <= g1; g += 4) {   // four loads in flight, added in order
      const float4 v0 = part[(size_t)g * n4 + i], v1 = part[(size_t)(g + 1) * n4 + i];
      const float4 v2 = part[(size_t)(g + 2) * n4 + i], v3 = part[(size_t)(g + 3) * n4 + i];
      acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
      acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
      acc.x += v2.x; acc.y += v2.y; acc.z += v2.z; acc.w += v2.w;
      acc.x += v3.x; acc.y += v3.y; acc.z += v3.z; acc.w += v3.w;
    }
    for (; g < g1; ++g) {
      const float4 v = part[(size_t)g * n4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  ps[j][e] = acc;
  __syncthreads();
  if (j == 0 && i < n4) {
    float4 s = ps[0][e];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      const float4 v = ps[q][e];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    float4 d = dW[i];
    d.x += s.x; d.y += s.y; d.z += s.z; d.w += s.w;
    dW[i] = d;
  }
}
__global__ __launch_bounds__(256) void wgrad_slab_reduce_kernel(int G, size_t n4, const float4* __restrict__ part,
                                                                float4* __restrict__ dW) {
  __shared__ float4 ps[8][32];
  slab_reduce_block(G, n4, part, dW, blockIdx.x, ps);
}
// the deferred reductions of a backward in one launch (adp_wgrad_defer / adp_wgrad_flush): segment j takes blocks
// [blk0[j], blk0[j + 1]), each block the same arithmetic as wgrad_slab_reduce_kernel (bit-identical sums)
constexpr int SEG_MAX = 32;
struct SegTable {
  int n;
  int blk0[SEG_MAX + 1];
  int G[SEG_MAX];
  unsigned long long n4[SEG_MAX];
  const float4* part[SEG_MAX];
  float4* dst[SEG_MAX];
};
__global__ __launch_bounds__(256) void wgrad_slab_reduce_batched_kernel(SegTable t) {
  __shared__ float4 ps[8][32];
  const int b = blockIdx.x;
  int j = 0;
  while (j + 1 < t.n && b >= t.blk0[j + 1]) ++j;
  slab_reduce_block(t.G[j], (size_t)t.n4[j], t.part[j], t.dst[j], b - t.blk0[j], ps);
}

// Pixel splits: enough blocks to fill the chip (target_blocks), but every split keeps at least
// min_chunk pixels so that the f32 atomic epilogue (blocks x TN x TK x 4 bytes at ~1.3 TB/s) stays
// small against the GEMM.
template <int WN, int WK, int TNW>
void launch_wcfg(WgradArgs& a, hipStream_t s, int target_blocks, int min_chunk) {
  constexpr int TN = WN * TNW, TK = WK * 64;
  a.ntile_k = (a.K + TK - 1) / TK;
  a.ntile_n = (a.Nout + TN - 1) / TN;
  const int tiles = a.ntile_k * a.ntile_n;
  // a one-tile launch (unet_bn's dec0_up ConvTranspose weight gradient: 128 x 256 over 1 M pixels) splits at most
  // wgrad_blocks_1tile (256) ways: one round of one-block-per-CU blocks and half the slabs of the 512-way split,
  // 0.225 -> 0.181 ms (profiles/r06o_convt_wgrad.log); multi-tile launches keep the larger targets (256 for all of
  // them cost adipose_v3's bf16 step 3.5 %, profiles/r06p_v3_bf16_ab.log)
  if (tiles == 1) target_blocks = std::min(target_blocks, adp::option("wgrad_blocks_1tile", 256));
  int splits = (target_blocks + tiles - 1) / tiles;
  const int maxsplit = (a.M + min_chunk - 1) / min_chunk;
  splits = std::max(1, std::min(splits, maxsplit));
  a.mchunk = ((a.M + splits - 1) / splits + 63) / 64 * 64;
  splits = (a.M + a.mchunk - 1) / a.mchunk;
  const bool ra = a.Wo % 64 == 0 && a.up == 1 && adp::option("wgrad_ra", 1);
  a.debug_flags = adp::option("wgrad_debug", 0);
  const bool two = adp::option("tap64_bar", 1) == 2;
  const dim3 grid(tiles * splits), block(WN * WK * 64);
  // split partials: slabs + reduce launch instead of f32 atomics (Kpad == K for every tap64 launch)
  a.part = nullptr;
  const size_t slab = (size_t)a.Nout * a.Kpad;
  // (measured per layer, tools/bench_kernels.py: slabs win 7-14 % on the 256x256 tiles of the >= 256-channel
  // layers, atomics win 4-6 % on the narrow-N tiles, whose slabs are small but split ~1000 ways)
  // (wgrad_det, default on: every split launch writes slabs, summed by the fixed-order reduce: two runs give the
  //  same bits)
  const bool det = adp::option("wgrad_det", 1) != 0;
  if (splits > 1 && (det || adp::option("wgrad_partials", TN >= 256 ? 1 : 0)) && !(ADP_DBG(a) & 1))
    a.part = det ? adp::reduce_part(0, slab * splits * sizeof(float), s)
                 : static_cast<float*>(adp::scratch(0, slab * splits * sizeof(float)));
  adp::set_kernel("igemm_wgrad_tap64_kernel<%d, %d, %d, %s, %s>", WN, WK, TNW, two ? "true" : "false",
                  ra ? "true" : "false");
  if (ra && !two) hipLaunchKernelGGL((igemm_wgrad_tap64_kernel<WN, WK, TNW, false, true>), grid, block, 0, s, a);
  else if (ra) hipLaunchKernelGGL((igemm_wgrad_tap64_kernel<WN, WK, TNW, true, true>), grid, block, 0, s, a);
  else if (!two) hipLaunchKernelGGL((igemm_wgrad_tap64_kernel<WN, WK, TNW, false, false>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((igemm_wgrad_tap64_kernel<WN, WK, TNW, true, false>), grid, block, 0, s, a);
  adp::kernel_end();   // (the split reduce below is a kernel of its own in rocprofv3's list)
  if (a.part && det) {
    adp::slab_reduce(splits, slab / 4, a.part, a.dW, s);
  } else if (a.part) {
    const size_t n4 = slab / 4;
    const int groups = (splits + WG_SG - 1) / WG_SG;
    const int blocks = (int)std::min<size_t>((n4 + 255) / 256, 4096);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks, groups), dim3(256), 0, s, splits, slab,
                       reinterpret_cast<const float4*>(a.part), reinterpret_cast<float4*>(a.dW));
  }
  a.part = nullptr;
}

}  // namespace

namespace adp {
// ---- deferred slab reductions (adp_wgrad_defer / adp_wgrad_flush). Every deterministic weight / bias gradient launch
// is followed by a small reduce launch (~10 us) and, like every launch, a ~5.8 us dependency gap: 21 per training
// step, ~0.34 ms (profiles/r05a: tools/kstats.py, gap analysis in DESIGN.md §3 (30)). Deferred, the slabs go to a
// per-stream arena (chunks kept across steps) and the reductions are recorded; adp_wgrad_flush launches them all as one
// kernel (up to SEG_MAX segments per launch), in the same fixed order: bit-identical gradients.
struct Deferred {
  bool on = false;
  bool fallback = false;                            // the last reduce_part came from scratch: reduce it at once
  std::vector<std::pair<char*, size_t>> chunks;   // (base, bytes) on the key's device, reused across steps
  size_t ci = 0, used = 0;                          // current chunk, bytes used in it
  size_t pending = 0;                               // slab bytes recorded since the last launch of the tables
  std::vector<SegTable> tables;                     // (built as the segments are recorded)
};
static void launch_tables(std::vector<SegTable>& tables, hipStream_t s) {
  for (const SegTable& t : tables)
    if (t.n > 0) hipLaunchKernelGGL(wgrad_slab_reduce_batched_kernel, dim3((unsigned)t.blk0[t.n]), dim3(256), 0, s, t);
  tables.clear();
}
// keyed by (device, stream) like every other piece of library state (round-5 ADVICE): the default stream is handle 0
// on every device, and an arena chunk must live on the device whose launches write it
using DefKey = std::pair<int, hipStream_t>;
static std::mutex g_def_mu;
static std::map<DefKey, Deferred>& deferred_map() {
  static std::map<DefKey, Deferred> m;
  return m;
}
static DefKey def_key(hipStream_t s) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return {dev, s};
}
float* reduce_part(int slot, size_t bytes, hipStream_t s) {
  {
    std::lock_guard<std::mutex> lk(g_def_mu);
    auto it = deferred_map().find(def_key(s));
    if (it != deferred_map().end() && it->second.on) {
      Deferred& d = it->second;
      d.fallback = false;
      bytes = (bytes + 255) / 256 * 256;
      // (option wgrad_defer_mb: once the recorded slabs would pass this many MB, the recorded reductions are
      //  launched first and the arena starts over: the slabs are re-read while they still sit in the MALL, and the
      //  arena's first chunk stays resident)
      const size_t lim = (size_t)std::max(0, option("wgrad_defer_mb", 64)) << 20;
      if (lim && d.pending + bytes > lim && !d.tables.empty()) {
        launch_tables(d.tables, s);
        d.ci = 0;
        d.used = 0;
        d.pending = 0;
      }
      while (d.ci < d.chunks.size() && d.used + bytes > d.chunks[d.ci].second) { ++d.ci; d.used = 0; }
      if (d.ci == d.chunks.size()) {   // (first steps only: a new chunk, kept until adp_wgrad_release)
        const size_t sz = std::max(bytes, (size_t)256 << 20);
        void* p = nullptr;
        if (hipMalloc(&p, sz) != hipSuccess) {
          // no arena: this launch's slabs go to the scratch slot and its reduction runs at once (slab_reduce), still
          // in a fixed order (round-5 ADVICE: it fell back to the f32 atomics and left a stale error)
          (void)hipGetLastError();
          d.fallback = true;
          return static_cast<float*>(scratch(slot, bytes));
        }
        d.chunks.push_back({static_cast<char*>(p), sz});
        d.used = 0;
      }
      d.pending += bytes;
      float* r = reinterpret_cast<float*>(d.chunks[d.ci].first + d.used);
      d.used += bytes;
      return r;
    }
  }
  return static_cast<float*>(scratch(slot, bytes));
}
void slab_reduce(int G, size_t n4, const float* part, float* dst, hipStream_t s) {
  {
    std::lock_guard<std::mutex> lk(g_def_mu);
    auto it = deferred_map().find(def_key(s));
    if (it != deferred_map().end() && it->second.on && !it->second.fallback) {
      Deferred& d = it->second;
      // segments of one launch run concurrently: a destination already in the open table (the same gradient
      // accumulated twice) starts a new table, launched after it
      bool clash = false;
      if (!d.tables.empty()) {
        const SegTable& o = d.tables.back();
        const float4* lo = reinterpret_cast<const float4*>(dst);
        for (int j = 0; j < o.n && !clash; ++j) clash = lo < o.dst[j] + o.n4[j] && o.dst[j] < lo + n4;
      }
      if (d.tables.empty() || d.tables.back().n == SEG_MAX || clash) {
        d.tables.emplace_back();
        d.tables.back().n = 0;
        d.tables.back().blk0[0] = 0;
      }
      SegTable& t = d.tables.back();
      const int j = t.n++;
      t.G[j] = G;
      t.n4[j] = n4;
      t.part[j] = reinterpret_cast<const float4*>(part);
      t.dst[j] = reinterpret_cast<float4*>(dst);
      t.blk0[j + 1] = t.blk0[j] + (int)((n4 + 31) / 32);
      return;
    }
    if (it != deferred_map().end()) it->second.fallback = false;
  }
  hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3((unsigned)((n4 + 31) / 32)), dim3(256), 0, s, G, n4,
                     reinterpret_cast<const float4*>(part), reinterpret_cast<float4*>(dst));
}
int wgrad_defer(hipStream_t s, int on) {
  std::lock_guard<std::mutex> lk(g_def_mu);
  Deferred& d = deferred_map()[def_key(s)];
  if (!on && !d.tables.empty()) { set_error("adp_wgrad_defer: reductions pending (adp_wgrad_flush first)"); return -1; }
  d.on = on != 0 && option("wgrad_defer", 1);   // (option wgrad_defer = 0: every reduction launched at once)
  return 0;
}
// launch the pending reductions of stream s (stream-ordered after the launches that wrote their slabs) and end the
// deferral; the arena is reused by the next deferred launches, which are ordered after these reductions
int wgrad_flush(hipStream_t s) {
  std::vector<SegTable> tables;
  {
    std::lock_guard<std::mutex> lk(g_def_mu);
    Deferred& d = deferred_map()[def_key(s)];
    tables.swap(d.tables);
    d.on = false;
    d.ci = 0;
    d.used = 0;
    d.pending = 0;
  }
  launch_tables(tables, s);
  return 0;
}
// free the arena of (current device, stream s) and forget the stream (an arena per stream that ever
// deferred, never freed; a destroyed stream's reused handle inherited it). Synchronises s first; an error with
// reductions pending (flush first).
int wgrad_release(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_def_mu);
  auto it = deferred_map().find(def_key(s));
  if (it == deferred_map().end()) return 0;
  if (!it->second.tables.empty()) { set_error("adp_wgrad_release: reductions pending (adp_wgrad_flush first)"); return -1; }
  if (!it->second.chunks.empty() && hipStreamSynchronize(s) != hipSuccess) {
    set_error("adp_wgrad_release: stream synchronisation failed");
    return -1;
  }
  for (auto& c : it->second.chunks) (void)hipFree(c.first);
  deferred_map().erase(it);
  return 0;
}
// (test hook) the number of arena chunks of (current device, stream s)
int wgrad_arena_chunks(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_def_mu);
  auto it = deferred_map().find(def_key(s));
  return it == deferred_map().end() ? 0 : (int)it->second.chunks.size();
}
// shapes of the persistent halo weight-gradient kernel
static bool halop_ok(const WgradArgs& a) {
  const int cin = a.CAs + a.CBs;
  return option("wgrad_halop", 1) && !a.scA && !a.scB && a.CAs % 64 == 0 && a.CBs % 64 == 0 && a.kh == 3 &&
         a.kw == 3 && a.dil == 1 && a.pad == 1 && a.stride == 1 && (a.up == 1 || a.up == 2) && a.Ho == a.Hs * a.up &&
         a.Wo == a.Ws * a.up &&
         a.Ho % 8 == 0 && a.Wo % 32 == 0 && a.Nout % 64 == 0 && a.dy_mode == 0 && a.K == 9 * cin &&
         a.Kpad == a.K && a.dy_stride % 8 == 0 && a.dy_stride >= a.Nout &&
         // buffer-resource offsets: every operand below 2 GiB
         (size_t)a.Nimg * a.Hs * a.Ws * std::max(a.CAs, a.CBs) * 2 < ((size_t)1 << 31) &&
         (size_t)a.Nimg * a.Ho * a.Wo * a.dy_stride * 2 < ((size_t)1 << 31);
}

// BatchNorm-backward apply fused into the halo weight gradient: every block of input chunk c recomputes
// its output block's dY tile, so only layers with at most wgrad_bna_maxch (default 1) 64-channel input
// chunks take it (levels 0-1 of unet_bn; deeper layers re-read dA/z once per chunk)
// shapes of the input-layer weight-gradient kernel (one 8-channel source, 64 outputs)
static bool cin8_ok(const WgradArgs& a) {
  return option("wgrad_cin8", 1) && !a.scA && a.CAs == 8 && a.CBs == 0 && a.kh == 3 && a.kw == 3 && a.dil == 1 &&
         a.pad == 1 && a.stride == 1 && a.up == 1 && a.Ho == a.Hs && a.Wo == a.Ws && a.Ho % 8 == 0 && a.Wo % 32 == 0 &&
         a.Nout == 64 && a.dy_mode == 0 && a.K == 72 && a.Kpad >= 72 && a.dy_stride % 8 == 0 && a.dy_stride >= 64;
}
bool wgrad_bna_fusable(const WgradArgs& a) {
  // (launch_wgrad_tap64 takes the halo kernel only with wgrad_tap64 != 0: with it off, the fused form would
  //  fall through to a kernel that reads a dY nothing has computed)
  if (!(a.bna_dA && a.bna_z && option("wgrad_tap64", 1) != 0 && option("wgrad_bna", 1))) return false;
  // the input layer (option wgrad_cin8_bna), when nothing reads dz (dY = NULL: the kernel stores none);
  // dA / z through buffer resources below 2 GiB
  if (cin8_ok(a) && !a.dY && option("wgrad_cin8_bna", 1) && (size_t)a.M * a.dy_stride * 2 < ((size_t)1 << 31))
    return true;
  return option("wgrad_halop_waves", 8) == 8 && halop_ok(a) && (a.CAs + a.CBs) / 64 <= option("wgrad_bna_maxch", 1);
}

// configurations: 0 = 256x256 (8 waves, 128x64 per wave), 1 = 128x256 (8 waves, 64x64),
// 2 = 64x256 (4 waves, 64x64, two blocks per CU)
int launch_wgrad_tap64(WgradArgs& a, hipStream_t s) {
  const int mode = option("wgrad_tap64", 1);   // 0 off, 1 auto, 2+c force configuration c
  if (mode == 0) return 0;
  if (cin8_ok(a)) {   // (bna_dA set: the caller checked wgrad_bna_fusable)
    const int tiles = a.Nimg * (a.Ho / 8) * (a.Wo / 32);
    const int grid = std::max(1, std::min(tiles, option("wgrad_cin8_grid", 256)));
    // wgrad_det (default on): per-block slabs [grid][64][Kpad] + the fixed-order reduce instead of f32 atomics
    a.part = option("wgrad_det", 1) && !(ADP_DBG(a) & 1)
                 ? reduce_part(0, (size_t)grid * 64 * a.Kpad * sizeof(float), s) : nullptr;
    if (a.bna_dA) {
      adp::set_kernel("igemm_wgrad_cin8_kernel<true>");
      hipLaunchKernelGGL((igemm_wgrad_cin8_kernel<true>), dim3(grid), dim3(512), 0, s, a);
    } else {
      adp::set_kernel("igemm_wgrad_cin8_kernel<false>");
      hipLaunchKernelGGL((igemm_wgrad_cin8_kernel<false>), dim3(grid), dim3(512), 0, s, a);
    }
    if (a.part) {
      adp::kernel_end();
      slab_reduce(grid, (size_t)64 * a.Kpad / 4, a.part, a.dW, s);
      a.part = nullptr;
    }
    return 1;
  }
  const int cin = a.CAs + a.CBs;
  if (halop_ok(a)) {   // option wgrad_halop: 0 off, else every eligible shape
    const int combos = (cin / 64) * (a.Nout / 64);
    const int tiles = a.Nimg * (a.Ho / 8) * (a.Wo / 32);
    int per = std::max(1, std::min(tiles, option("wgrad_halop_grid", 256) / combos));
    a.debug_flags = option("wgrad_debug", 0);
    // dynamic patch claiming (option wgrad_halop_claim; nullptr from claim_slot: static lists)
    a.claim = option("wgrad_halop_claim", option("dp_claim", 0)) && combos + 1 <= CLAIM_INTS ? claim_slot() : nullptr;
    a.claim_chunk = std::max(1, option("wgrad_halop_claim_chunk", 4));   // patches per claim
    if (a.claim) per = std::min(per, (tiles + a.claim_chunk - 1) / a.claim_chunk);   // (<= super-patches)
    // claim_full only with at least 4 super-patches per block (its first claim takes two at once)
    a.claim_full = option("claim_full", 0) && (tiles + a.claim_chunk - 1) / a.claim_chunk >= 4 * per;
    const int grid = per * combos;
    const bool stat_inst = !a.claim && option("wgrad_halop_static", 1);   // (the CLM = false instances)
    // output form (option wgrad_det, default on): static lists write per-block slabs summed in a fixed order by
    // wgrad_slab_reduce_kernel (one block per combination: dW += partial in place), so two runs give the same bits;
    // wgrad_det = 0 or claimed patches: f32 atomics in the order blocks finish
    a.part = nullptr;
    a.part_rmw = 0;
    const bool det = !a.claim && option("wgrad_det", 1) && !(ADP_DBG(a) & 1);
    if (det && per == 1 && ((uintptr_t)a.dW & 15) == 0) a.part_rmw = 1;   // (16-B pieces of dW: aligned dW only)
    else if (det) a.part = reduce_part(0, (size_t)per * a.Nout * a.Kpad * sizeof(float), s);
    // (a failed scratch allocation leaves part null: the atomic form)
    if (a.bna_dA) {   // the caller checked wgrad_bna_fusable
      if (option("wgrad_halop_spread", 4) == 8) {
        adp::set_kernel("igemm_wgrad_halop_kernel<8, true, 8, true, false>");
        hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, true, 8>), dim3(grid), dim3(512), 0, s, a);
      } else if (stat_inst) {
        adp::set_kernel("igemm_wgrad_halop_kernel<8, true, 4, false, false>");
        hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, true, 4, false>), dim3(grid), dim3(512), 0, s, a);
      } else {   // halo groups two a row over rows 3-5
        adp::set_kernel("igemm_wgrad_halop_kernel<8, true, 4, true, false>");
        hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, true, 4>), dim3(grid), dim3(512), 0, s, a);
      }
    } else if (stat_inst && option("wgrad_halop_pair", 1)) {
      // (round 6, default: the tap-pair form -- two waves of a SIMD own taps 2p, 2p + 1 and a quarter of tap 8 and split
      //  the patch rows; option wgrad_halop_pair = 0 keeps the one-tap-per-wave forms below)
      // (options wgrad_pair_spread: the LDS-DMA schedule LSPR; wgrad_pair_pipe: the fragment-read schedule PIPE)
      const int spr = option("wgrad_pair_spread", 6), pipe = option("wgrad_pair_pipe", 0);
#define ADP_PAIR(L, D)                                                                                              \
  if (spr == L && pipe == D) {                                                                                      \
    adp::set_kernel("igemm_wgrad_halopair_kernel<" #L ", " #D ">");                                                \
    hipLaunchKernelGGL((igemm_wgrad_halopair_kernel<L, D>), dim3(grid), dim3(512), 0, s, a);                       \
  } else
      ADP_PAIR(6, 0) ADP_PAIR(6, 1) ADP_PAIR(6, 2) ADP_PAIR(4, 0) ADP_PAIR(8, 0) ADP_PAIR(9, 0) {
        set_error("wgrad_pair_spread / wgrad_pair_pipe: (6, 0 / 1 / 2), (4, 0), (8, 0) or (9, 0)");
        return -1;
      }
#undef ADP_PAIR
    } else if (option("wgrad_halop_waves", 8) == 9) {
      adp::set_kernel("igemm_wgrad_halop_kernel<9, false, 8, true, false>");
      hipLaunchKernelGGL(igemm_wgrad_halop_kernel<9>, dim3(grid), dim3(576), 0, s, a);
    } else if (stat_inst && (option("wgrad_halop_pf", 2) == 2 ||
                             (option("wgrad_halop_pf", 2) == 1 && a.M <= option("wgrad_halop_pf_maxm", 1 << 19)))) {
      // (row-pipelined form; option wgrad_halop_pf 0 never, 1 only where M <= 2^19 pixels, 2 always -- the default:
      //  at levels 0-1 the plain loop is 1-4 % ahead per launch (profiles/r05_wgrad_variants.log) but the step does not
      //  move (22.627 vs 22.632 ms, r05_pfauto_ab.log), and one instance for every launch keeps the step's dominant
      //  kernel the same instantiation round to round)
      // (option wgrad_halop_spread: the next patch's LDS-DMA over patch rows 0-3 (4, default) or 0-7 (8))
      const int spr = option("wgrad_halop_spread", 4);
      if (spr == 8) {
        adp::set_kernel("igemm_wgrad_halop_kernel<8, false, 8, false, true>");
        hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, false, 8, false, true>), dim3(grid), dim3(512), 0, s, a);
      } else {   // (rows 0-1 / row 0 only: -1..-16 % / -2..-4 % at L0-L4, profiles/r05k_spread*_ab.log)
        adp::set_kernel("igemm_wgrad_halop_kernel<8, false, 4, false, true>");
        hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, false, 4, false, true>), dim3(grid), dim3(512), 0, s, a);
      }
    } else if (stat_inst && option("wgrad_halop_spread", 4) != 8) {
      adp::set_kernel("igemm_wgrad_halop_kernel<8, false, 4, false, false>");
      hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, false, 4, false>), dim3(grid), dim3(512), 0, s, a);
    } else {
      // the next patch's loads over rows 0-3 (3 groups a row) leave 4 rows of DMA slack before the patch
      // barrier: +1-3 % on every level but 0 64->64 against rows 0-7, step -0.3 %
      // (profiles/r02_wgrad_spread_ab.txt); option wgrad_halop_spread=8 keeps the all-rows schedule
      if (option("wgrad_halop_spread", 4) == 8) {
        adp::set_kernel("igemm_wgrad_halop_kernel<8, false, 8, true, false>");
        hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, false, 8>), dim3(grid), dim3(512), 0, s, a);
      } else {
        adp::set_kernel("igemm_wgrad_halop_kernel<8, false, 4, true, false>");
        hipLaunchKernelGGL((igemm_wgrad_halop_kernel<8, false, 4>), dim3(grid), dim3(512), 0, s, a);
      }
    }
    if (a.part) {   // (a kernel of its own in rocprofv3's list and outside the conv's event bracket)
      adp::kernel_end();
      slab_reduce(per, (size_t)a.Nout * a.Kpad / 4, a.part, a.dW, s);
      a.part = nullptr;
    }
    return 1;
  }
  if (a.bna_dA) return 0;   // only the halo kernel computes dY itself (the caller runs the apply, then a fallback)
  const int Cin_s = a.CAs + a.CBs;
  if (a.scA || a.scB || a.CAs % 64 != 0 || a.CBs % 64 != 0 || a.K != a.kh * a.kw * Cin_s || a.K % 64 != 0 ||
      a.Kpad != a.K)
    return 0;
  int cfg = mode - 2;
  if (mode == 1) cfg = a.Nout >= 192 ? 0 : a.Nout > 64 ? 1 : 2;
  // block targets measured on the unet_bn layer shapes (tools/bench_kernels.py)
  const int target = option("wgrad_blocks", cfg == 0 ? 1024 : cfg == 1 ? 2048 : 4096);
  const int min_chunk = option("wgrad_min_chunk", cfg == 0 ? 2048 : 1024);
  if (cfg == 0) launch_wcfg<2, 4, 128>(a, s, target, min_chunk);
  else if (cfg == 1) launch_wcfg<2, 4, 64>(a, s, target, min_chunk);
  else if (cfg == 2) launch_wcfg<1, 4, 64>(a, s, target, min_chunk);
  else return 0;
  return 1;
}
}  // namespace adp
