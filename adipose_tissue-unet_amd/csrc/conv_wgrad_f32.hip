// f32 weight gradient on the LDS-DMA staging of the bf16 kernels (the reference-precision path every drop-in
// CLI defaults to; an opt-in alternative to the register-staged igemm_wgrad_kernel<float> of conv_igemm.hip,
// option wgrad_f32=1: slower on adipose_v3's channel widths, see launch_wgrad_f32):
//   dW[n][k] += sum_m dY[m][n] * X(k)[m]      (k = tap * Cin_s + ci, m = output pixel)
// Block = WN x WK waves, dW tile (WN*64) x (WK*64), each wave a 64 x 64 tile of exact v_mfma_f32_16x16x4_f32
// accumulators. A stage is 32 output pixels: the dY rows (TN f32 channels) and the gathered X rows (TK f32
// k-columns, 4 consecutive channels of one tap per 16-B chunk: f32 channel strides are multiples of 4) are
// moved into LDS by global_load_lds_dwordx4 in their natural [pixel][channel] layout, double-buffered with one
// barrier per stage. MFMA k = pixel: for each 4-pixel k step a lane reads one f32 of dY^T and one of X^T
// (16 consecutive channels of one pixel row per 16 lanes), with the 16-B chunk of row r stored at position
// c ^ (4 (r & 3)) so that the four rows of a k step fall into four distinct 64-B bank groups.
// Splits of the pixel range write per-split slabs reduced by a second launch (wide tiles) or add with f32
// atomics (narrow tiles), as the bf16 tap64 weight gradient does.
#include "conv_common.h"

namespace {

__device__ __attribute__((aligned(256))) uint4 wf_zero_page[64];

ADP_DEV uint32_t wf_lds(const void* p) { return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p; }
// LDS reads as inline asm: the compiler would wait for every LDS-DMA in flight before a plain read
ADP_DEV float wf_rd(uint32_t addr) {
  float r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}
template <int N>
ADP_DEV void wf_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
ADP_DEV int fsw(int r) { return (r & 3) << 2; }

struct WfSlot { int m, n, y, x; };
ADP_DEV void wf_init(WfSlot& s, int m, int HWo, int Wo) {
  s.m = m;
  s.n = m / HWo;
  const int rem = m - s.n * HWo;
  s.y = rem / Wo;
  s.x = rem - s.y * Wo;
}
struct WfAdv { int an, ay, ax; };
ADP_DEV void wf_adv(WfSlot& s, const WfAdv& d, int Ho, int Wo) {   // pixel + 32, branch-free mixed radix
  s.m += 32;
  s.x += d.ax;
  const int cx = s.x >= Wo;
  s.x -= cx ? Wo : 0;
  s.y += d.ay + cx;
  const int cy = s.y >= Ho;
  s.y -= cy ? Ho : 0;
  s.n += d.an + cy;
}

template <int WN, int WK>
__global__ __launch_bounds__(WN * WK * 64, 1) void igemm_wgrad_f32_kernel(WgradArgs a) {
  constexpr int NTH = WN * WK * 64, TN = WN * 64, TK = WK * 64;
  constexpr int RD = 4 * TN, RX = 4 * TK;              // LDS row bytes (one pixel)
  constexpr int QD = 32 * RD, QX = 32 * RX, STAGE = QD + QX;
  constexpr int CPRD = RD / 16, CPRX = RX / 16;        // 16-B chunks per row
  constexpr int RPID = NTH / CPRD, RPIX = NTH / CPRX;  // rows per LDS-DMA instruction (whole block)
  constexpr int GD = 32 / RPID, GX = 32 / RPIX;        // LDS-DMA instructions per thread per stage
  static_assert(GD >= 1 && GX >= 1 && GD * RPID == 32 && GX * RPIX == 32, "stage rows split evenly");
  static_assert(RPID % 4 == 0 && RPIX % 4 == 0 && CPRD >= 16 && CPRX >= 16, "a thread's rows share the swizzle");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WK, wk = wave % WK;
  const int tiles = a.ntile_k * a.ntile_n;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / tiles, tile = lin - split * tiles;
  const int tk = tile % a.ntile_k, tn = tile / a.ntile_k;
  const int k0 = tk * TK, n0 = tn * TN;
  const int mbeg = split * a.mchunk;
  const int mend = min(a.M, mbeg + a.mchunk);
  if (mbeg >= mend) return;
  const int ns = (mend - mbeg + 31) / 32;
  const int HWo = a.Ho * a.Wo, Hv = a.Hs * a.up, Wv = a.Ws * a.up;
  const int Cin_s = a.CAs + a.CBs;

  // ---- this thread's fixed chunk columns (X: 4 channels of one tap; dY: 4 output channels)
  const int kx = k0 + 4 * ((tid % CPRX) ^ fsw(tid / CPRX));
  const bool kvalid = kx < a.K;
  int oy = 0, ox = 0, xcs = a.CAs;
  const float* xbase = reinterpret_cast<const float*>(a.srcA);
  if (kvalid) {
    const int tap = kx / Cin_s, ci = kx - tap * Cin_s;
    const int ty = tap / a.kw, tx = tap - ty * a.kw;
    oy = ty * a.dil - a.pad;
    ox = tx * a.dil - a.pad;
    if (ci < a.CAs) xbase += ci;
    else { xbase = reinterpret_cast<const float*>(a.srcB) + (ci - a.CAs); xcs = a.CBs; }
  }
  const int nd = n0 + 4 * ((tid % CPRD) ^ fsw(tid / CPRD));
  const bool nvalid = nd < a.Nout;
  int dsub = 0, dc = nd;
  if (a.dy_mode == 1) { dsub = nd / a.Cps; dc = nd - dsub * a.Cps; }
  const float* dy = reinterpret_cast<const float*>(a.dY);

  WfSlot sx[GX], sd[GD];
#pragma unroll
  for (int i = 0; i < GX; ++i) wf_init(sx[i], mbeg + i * RPIX + tid / CPRX, HWo, a.Wo);
#pragma unroll
  for (int i = 0; i < GD; ++i) wf_init(sd[i], mbeg + i * RPID + tid / CPRD, HWo, a.Wo);
  WfAdv adv;
  adv.an = 32 / HWo;
  adv.ay = (32 - adv.an * HWo) / a.Wo;
  adv.ax = 32 - adv.an * HWo - adv.ay * a.Wo;

  // the next stage into buffer buf (every thread GD + GX pieces), then advance the slots by 32 pixels
  auto issue = [&](int buf) {
    unsigned char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < GD; ++i) {
      WfSlot& s = sd[i];
      size_t off;
      if (a.dy_mode == 0) off = (size_t)s.m * a.dy_stride + nd;
      else off = (((size_t)s.n * (2 * a.Ho) + 2 * s.y + (dsub >> 1)) * (2 * a.Wo) + 2 * s.x + (dsub & 1)) * a.dy_stride + dc;
      const bool ok = s.m < mend && nvalid;
      const void* p = ok ? (const void*)(dy + off) : (const void*)wf_zero_page;
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(base + i * RPID * RD + wave * 1024), 16, 0, 0);
      wf_adv(s, adv, a.Ho, a.Wo);
    }
#pragma unroll
    for (int i = 0; i < GX; ++i) {
      WfSlot& s = sx[i];
      int yi = s.y * a.stride + oy, xi = s.x * a.stride + ox;
      const bool ok = s.m < mend && kvalid && (unsigned)yi < (unsigned)Hv && (unsigned)xi < (unsigned)Wv;
      if (a.up == 2) { yi >>= 1; xi >>= 1; }
      const void* p = ok ? (const void*)(xbase + (size_t)((s.n * a.Hs + yi) * a.Ws + xi) * xcs)
                         : (const void*)wf_zero_page;
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(base + QD + i * RPIX * RX + wave * 1024), 16, 0, 0);
      wf_adv(s, adv, a.Ho, a.Wo);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment offsets of this lane inside a row (before the row's swizzle): dY^T column n, X^T column k
  const int li = lane & 15, lg = lane >> 4;
  int dcol[4], xcol[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    dcol[b] = wn * 64 + b * 16 + li;
    xcol[b] = wk * 64 + b * 16 + li;
  }
  const uint32_t sbase = wf_lds(smem);
  float fa[2][4], fb[2][4];
  auto read_ks = [&](int buf, int ks, float (&A)[4], float (&B)[4]) {
    const int r = ks * 4 + lg, sw = fsw(r);
    const uint32_t rd = sbase + buf * STAGE + r * RD, rx = sbase + buf * STAGE + QD + r * RX;
#pragma unroll
    for (int b = 0; b < 4; ++b) A[b] = wf_rd(rd + ((((dcol[b] >> 2) ^ sw) << 4) | ((dcol[b] & 3) << 2)));
#pragma unroll
    for (int b = 0; b < 4; ++b) B[b] = wf_rd(rx + ((((xcol[b] >> 2) ^ sw) << 4) | ((xcol[b] & 3) << 2)));
  };
  auto mma_ks = [&](const float (&A)[4], const float (&B)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) acc[nb][kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[nb], B[kb], acc[nb][kb], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  issue(0);
  for (int t = 0; t < ns; ++t) {
    const int buf = t & 1;
    // stage t landed for every wave, and every wave is done with stage t - 1 (its buffer takes stage t + 1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < ns) issue(buf ^ 1);
    read_ks(buf, 0, fa[0], fb[0]);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if (ks + 1 < 8) {
        read_ks(buf, ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
        wf_lgkm<8>();
      } else {
        wf_lgkm<0>();
      }
      mma_ks(fa[ks & 1], fb[ks & 1]);
    }
  }
  __syncthreads();   // the stage buffers become the epilogue's staging rows

  // dW rows: each wave's 16-row blocks through LDS into 256-B rows (64 consecutive k per store / atomic)
  constexpr int ES = 68;
  float* blk = reinterpret_cast<float*>(smem) + wave * 16 * ES;
  const int col = lane & 15, rq = (lane >> 4) * 4;
  const int kk = k0 + wk * 64 + lane;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) blk[(rq + r) * ES + kb * 16 + col] = acc[nb][kb][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (a.part) {
      // the reduce adds whole Nout x Kpad slabs: the K..Kpad-1 pad columns are written as zeros (the tiles
      // cover them, ntile_k * TK >= round_up(K, 64) >= Kpad), never left with another launch's scratch
      float* slab = a.part + (size_t)split * a.Nout * a.Kpad;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int n = n0 + wn * 64 + nb * 16 + i;
        if (n < a.Nout && kk < a.Kpad) slab[(size_t)n * a.Kpad + kk] = kk < a.K ? blk[i * ES + lane] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int n = n0 + wn * 64 + nb * 16 + i;
        if (n < a.Nout && kk < a.K) atomicAdd(a.dW + (size_t)n * a.Kpad + kk, blk[i * ES + lane]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
}

// dW[n][k] += sum over the splits of part[split][n][k] (k < Kpad), 4 floats per thread
__global__ void wgrad_f32_reduce_kernel(int splits, size_t slab, const float4* part, float4* dW) {
  const size_t n4 = slab / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 acc = dW[i];
    for (int s = 0; s < splits; ++s) {
      const float4 v = part[(size_t)s * n4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    dW[i] = acc;
  }
}


// ---------------------------------------------------------------------------------------------------------------
// Persistent halo form of the f32 weight gradient (3x3, stride 1, dilation 1, 'same'; f32 channel strides that are
// multiples of 32 from one or two sources, Nout a multiple of 32; the nearest-x2 input gather of adipose_v3's
// up*_conv1 layers): the f32 counterpart of igemm_wgrad_halop_kernel (conv_wgrad_tap64.hip). The gathered kernel
// above re-reads every input pixel once per tap and tiles K = 9 Cin_s in 64-wide blocks that run part-empty on
// adipose_v3's 44 * 2^l widths; here a block keeps one (32-channel input chunk, 64-channel output block) pair
// and walks 4 x 32 output patches: per patch the 6 x 34 input halo (26 KiB) and the 128 x 64 dY tile (32 KiB)
// are moved into LDS once by LDS-DMA (double-buffered: the next patch's pieces ride on the rows of this one),
// and wave w keeps the 16 x 16 dW block (output rows 16 (w >> 1), input columns 16 (w & 1)) of all nine taps in
// 36 accumulator registers. A 4-pixel k step of v_mfma_f32_16x16x4_f32 reads one f32 of dY^T and, per tap, one
// f32 of the shifted halo (ds_read_b32, 16 consecutive channels of one pixel per 16 lanes); the 16-B chunk q of
// row r sits at q ^ 4 (r & 1), so the two rows a 32-lane group reads fall into disjoint banks. Exact f32
// products, f32 accumulation; one f32 atomic add per dW element and block at the end.
constexpr int HF_PH = 4, HF_PW = 32, HF_HW = HF_PW + 2, HF_HROWS = (HF_PH + 2) * HF_HW;   // 204 halo pixels
// LDS read with a compile-time byte offset on a per-lane base: the uniform part of every fragment address of the
// unrolled k loop is an immediate, so the loop holds 4 base registers instead of 320 addresses
template <int OFF>
ADP_DEV float wf_rdo(uint32_t addr) {
  float r;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF) : "memory");
  return r;
}
// (a device function: the builtin inside a kernel template fails the host pass's substitution)
__device__ __forceinline__ void hf_buf_lds16(__amdgpu_buffer_rsrc_t rs, void* lds, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, off, 0, 0, 0);
}
// halo geometry of the dilated form (below): the 32 patch columns in SPLIT segments of 32 / SPLIT, each segment with
// its own two halo columns; SPLIT 1 is the dilation-1 layout (34 halo columns)
template <int SPLIT>
constexpr int hf_hw() { return HF_PW + 2 * SPLIT; }
template <int SPLIT>
constexpr int hf_col(int c) { return c + 2 * (c / (HF_PW / SPLIT)); }
// k step S of a patch (pixel row S / 8, pixels 4 (S % 8) .. + 3): dY^T element and the tap-shifted halo elements of
// the taps in TM (all 9 by default; the tap-split waves of the T3 form take 5 or 4)
#define HF_B(t) \
  if constexpr ((TM >> (t)) & 1) B[t] = wf_rdo<((r + (t) / 3) * HW + hc) * 128>(bbase[(t) % 3]);
template <int S, int SPLIT, int TM = 0x1FF>
ADP_DEV void hf_read(uint32_t abase, const uint32_t (&bbase)[3], float& A, float (&B)[9]) {
  constexpr int r = S / 8, xs = S % 8, HW = hf_hw<SPLIT>(), hc = hf_col<SPLIT>(4 * xs);
  A = wf_rdo<(r * HF_PW + 4 * xs) * 256>(abase);
  HF_B(0) HF_B(1) HF_B(2) HF_B(3) HF_B(4) HF_B(5) HF_B(6) HF_B(7) HF_B(8)
}
#undef HF_B
// the 32 k steps of a patch, software-pipelined one step deep (the reads of step S + 1 in flight while step S
// multiplies); at the first step of each pixel row the row's share of the next patch's LDS-DMA goes out
#define HF_M(t) \
  if constexpr ((TM >> (t)) & 1) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[cur], fb[cur][t], acc[t], 0, 0, 0);
template <int S, int SPLIT = 1, int TM = 0x1FF, typename RowIssue>
ADP_DEV void hf_steps(uint32_t abase, const uint32_t (&bbase)[3], float (&fa)[2], float (&fb)[2][9], f32x4 (&acc)[9],
                      float& db, const RowIssue& row_issue) {
  constexpr int NS = HF_PH * HF_PW / 4, cur = S & 1, NRD = 1 + __builtin_popcount(TM);
  if constexpr (S % 8 == 0) row_issue(S / 8);
  if constexpr (S + 1 < NS) {
    hf_read<S + 1, SPLIT, TM>(abase, bbase, fa[cur ^ 1], fb[cur ^ 1]);
    wf_lgkm<NRD>();
  } else {
    wf_lgkm<0>();
  }
  __builtin_amdgcn_s_setprio(1);
  HF_M(0) HF_M(1) HF_M(2) HF_M(3) HF_M(4) HF_M(5) HF_M(6) HF_M(7) HF_M(8)
  __builtin_amdgcn_s_setprio(0);
  db += fa[cur];   // (the bias gradient: every dY element of the patch passes one lane's A operand once)
  if constexpr (S + 1 < NS) hf_steps<S + 1, SPLIT, TM>(abase, bbase, fa, fb, acc, db, row_issue);
}
#undef HF_M
// Z3 (round 6): the multi-row wave of a chunk tail with 3 row blocks -- taps 7 and 8 (halo row r + 2, columns + 1 and
// + 2) of all three 16-row blocks: three dY^T elements and two halo elements per k step, six MFMAs into acc[0..5]
template <int S>
ADP_DEV void hf_read_mr(const uint32_t (&abase)[3], const uint32_t (&bbase)[3], float (&A)[3], float (&B)[2]) {
  constexpr int r = S / 8, xs = S % 8, HW = hf_hw<1>(), hc = hf_col<1>(4 * xs);
  A[0] = wf_rdo<(r * HF_PW + 4 * xs) * 256>(abase[0]);
  A[1] = wf_rdo<(r * HF_PW + 4 * xs) * 256>(abase[1]);
  A[2] = wf_rdo<(r * HF_PW + 4 * xs) * 256>(abase[2]);
  B[0] = wf_rdo<((r + 2) * HW + hc) * 128>(bbase[1]);
  B[1] = wf_rdo<((r + 2) * HW + hc) * 128>(bbase[2]);
}
template <int S, typename RowIssue>
ADP_DEV void hf_steps_mr(const uint32_t (&abase)[3], const uint32_t (&bbase)[3], float (&fa)[2][3], float (&fb)[2][2],
                         f32x4 (&acc)[9], const RowIssue& row_issue) {
  constexpr int NS = HF_PH * HF_PW / 4, cur = S & 1;
  if constexpr (S % 8 == 0) row_issue(S / 8);
  if constexpr (S + 1 < NS) {
    hf_read_mr<S + 1>(abase, bbase, fa[cur ^ 1], fb[cur ^ 1]);
    wf_lgkm<5>();
  } else {
    wf_lgkm<0>();
  }
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int rr = 0; rr < 3; ++rr) {
    acc[2 * rr] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[cur][rr], fb[cur][0], acc[2 * rr], 0, 0, 0);
    acc[2 * rr + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[cur][rr], fb[cur][1], acc[2 * rr + 1], 0, 0, 0);
  }
  __builtin_amdgcn_s_setprio(0);
  if constexpr (S + 1 < NS) hf_steps_mr<S + 1>(abase, bbase, fa, fb, acc, row_issue);
}
// T3 (round 6): output blocks with 3 real 16-row blocks (adipose_v3's level-0 44 outputs) leave rows 48-63 to the
// waves 6 and 7, i.e. SIMDs 2 and 3 idle half the time while SIMDs 0 and 1 run two full waves. In the T3 form the
// third row block is split by taps: waves 4 / 5 take its taps 0-4, waves 6 / 7 taps 5-8, so the SIMDs run 14, 14, 13
// and 13 tap blocks per k step instead of 18, 18, 9 and 9.
template <bool T3>
__global__ __launch_bounds__(512, 1) void igemm_wgrad_halo_f32_kernel(WgradArgs a) {
  constexpr int NTH = 512, CI = 32, NB = 64;
  constexpr int HRB = CI * 4, DRB = NB * 4;                    // LDS row bytes: halo pixel, dY pixel
  constexpr int NPIX = HF_PH * HF_PW;                          // 128 output pixels per patch
  constexpr int HBUF = HF_HROWS * HRB, DBUF = NPIX * DRB, STAGE = HBUF + DBUF;
  constexpr int HCH = HF_HROWS * (HRB / 16), DCH = NPIX * (DRB / 16);   // 16-B pieces per patch
  constexpr int GH = (HCH + NTH - 1) / NTH, GD = DCH / NTH;
  static_assert(GD * NTH == DCH && GH + GD <= 2 * HF_PH, "pieces: two per patch row");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tx_n = a.Wo / HF_PW, ty_n = a.Ho / HF_PH;
  const int Cin_s = a.CAs + a.CBs, nch = Cin_s / CI, nnb = (a.Nout + NB - 1) / NB, combos = nch * nnb;
  const int T = a.Nimg * tx_n * ty_n;
  const int lin0 = xcd_remap(blockIdx.x, gridDim.x);
  int combo, lin, G;
  if (a.zt_n) {   // zero tails: weighted block ranges per combination (the launcher's table)
    combo = 0;
    while (combo + 1 < a.zt_n && lin0 >= a.zt_cstart[combo + 1]) ++combo;
    lin = lin0 - a.zt_cstart[combo];
    G = a.zt_cstart[combo + 1] - a.zt_cstart[combo];
  } else {
    G = gridDim.x / combos;
    combo = lin0 % combos;
    lin = lin0 / combos;
  }
  const int ch = combo % nch, nblk = combo / nch;
  const int nt = lin < T ? (T - lin + G - 1) / G : 0;
  if (nt == 0) return;   // (uniform)
  // zero tails: a chunk with <= 16 real input channels has hm useful 16 x 16 blocks (output rows 16 w, input columns
  // 0-15), one per wave 0 .. hm - 1 -- one wave per SIMD instead of two --, and the other waves only stage
  // row tails (zt_mode >= 16): an output block with <= 2 real 16-row blocks takes them on waves 0 .. 2 rb - 1 (both
  // column blocks), one wave per SIMD as well
  const int zm = a.zt_n ? a.zt_mode[combo] : 0, hm = zm & 15;
  const bool rt = (zm & 16) != 0, t3 = T3 && (zm & 32) != 0;   // (row tails; T3: the tap-split third row block)
  // Z3 (T3 instance): a chunk tail with 3 row blocks -- waves 0-2 take taps 0-6 of row block w, wave 3 taps 7-8 of all
  // three (SIMD loads 7, 7, 7, 6 tap blocks instead of 9, 9, 9, 0), waves 4-7 stage
  const bool z3 = T3 && (zm & 64) != 0;
  const bool idle = hm > 0 && !t3 && wave >= (z3 ? 4 : rt ? 2 * hm : hm);
  const bool inA = ch * CI < a.CAs;
  const int xcs = inA ? a.CAs : a.CBs;
  const int us = a.up >> 1;
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(inA ? a.srcA : a.srcB), 0, a.Nimg * a.Hs * a.Ws * xcs * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsD =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dY, 0, a.Nimg * a.Ho * a.Wo * a.dy_stride * 4, 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  // per-thread constant parts of the gathers (a halo row holds CI channels in 8 chunks, a dY row NB in 16)
  const int xc0 = (inA ? ch * CI : ch * CI - a.CAs) * 4;
  int hy[GH], hx[GH], hoff[GH];
#pragma unroll
  for (int i = 0; i < GH; ++i) {
    const int idx = i * NTH + tid, hr = idx >> 3, pos = idx & 7;
    hy[i] = hr / HF_HW - 1;
    hx[i] = hr % HF_HW - 1;
    hoff[i] = xc0 + 16 * (pos ^ (4 * (hr & 1)));
  }
  int dpix[GD], doff[GD];
  bool dok[GD];
#pragma unroll
  for (int i = 0; i < GD; ++i) {
    const int idx = i * NTH + tid, pr = idx >> 4, q = (idx & 15) ^ (4 * (pr & 1));
    dpix[i] = (pr >> 5) * a.Wo + (pr & 31);
    doff[i] = (nblk * NB + 4 * q) * 4;
    dok[i] = nblk * NB + 4 * q < a.Nout;
  }
  struct Patch { int img, y0, x0, pbd; };
  auto patch = [&](int k) {
    Patch P;
    const int t = lin + k * G;
    const int px = t % tx_n, r = t / tx_n;
    P.img = r / ty_n;
    P.y0 = (r % ty_n) * HF_PH;
    P.x0 = px * HF_PW;
    P.pbd = (P.img * a.Ho + P.y0) * a.Wo + P.x0;
    return P;
  };
  auto issue_h = [&](const Patch& P, int i, int buf) {
    const int idx = i * NTH + tid;
    if (i < GH - 1 || idx < HCH) {
      const int gy = P.y0 + hy[i], gx = P.x0 + hx[i];
      const bool ok = (unsigned)gy < (unsigned)(a.Hs << us) && (unsigned)gx < (unsigned)(a.Ws << us);
      const unsigned off =
          ok ? (unsigned)(((P.img * a.Hs + (gy >> us)) * a.Ws + (gx >> us)) * xcs * 4 + hoff[i]) : OOB;
      hf_buf_lds16(rsX, smem + buf * STAGE + (size_t)(i * NTH + wave * 64) * 16, off);
    }
  };
  auto issue_d = [&](const Patch& P, int i, int buf) {
    const unsigned off = dok[i] ? (unsigned)((P.pbd + dpix[i]) * a.dy_stride * 4 + doff[i]) : OOB;
    hf_buf_lds16(rsD, smem + buf * STAGE + HBUF + (size_t)(i * NTH + wave * 64) * 16, off);
  };
  // the next patch's pieces, two per patch row (halo first)
  auto issue_row = [&](const Patch& P, int r, int buf) {
#pragma unroll
    for (int g = 0; g < GH + GD; ++g)
      if (g / 2 == r) {
        if (g < GH) issue_h(P, g, buf);
        else issue_d(P, g - GH, buf);
      }
  };

  f32x4 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db = 0.f;
  const bool zc = hm && !rt && !t3;   // (chunk tails: one 16-column block, a 16-row block per wave)
  const int wn = zc ? (z3 && wave == 3 ? 0 : wave) : (t3 ? min(wave >> 1, 2) : wave >> 1), wc = zc ? 0 : wave & 1;
  // T3: waves 4 / 5 the taps 0-4 of row block 2, waves 6 / 7 its taps 5-8 (tap masks 0x01F / 0x1E0); Z3: waves 0-2
  // taps 0-6 (0x07F), wave 3 the multi-row taps 7-8 (tsel 4)
  const int tsel = t3 ? (wave < 4 ? 0 : wave < 6 ? 1 : 2) : z3 ? (wave < 3 ? 3 : 4) : 0;
  const int tmask = tsel == 0 ? 0x1FF : tsel == 1 ? 0x01F : tsel == 2 ? 0x1E0 : tsel == 3 ? 0x07F : 0x180;
  const int li = lane & 15, lg = lane >> 4;
  const int ncol = wn * 16 + li, ccol = wc * 16 + li;   // this lane's dY column (output channel), X column
  const uint32_t sbase = wf_lds(smem);
  // per-lane parts of the fragment addresses: row r * 32 + 4 xs + lg of the dY tile, row (r + dy) * 34 + 4 xs +
  // lg + dx of the halo; the rows' swizzle parity is that of lg (+ dx), the rest of the address is uniform
  const uint32_t a_lane = lg * DRB + ((((ncol >> 2) ^ (4 * (lg & 1))) << 4) | ((ncol & 3) << 2));
  uint32_t b_lane[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
    b_lane[dx] = (lg + dx) * HRB + ((((ccol >> 2) ^ (4 * ((lg + dx) & 1))) << 4) | ((ccol & 3) << 2));
  uint32_t a_lane_mr[3];   // (Z3's multi-row wave: the dY^T columns of row blocks 0-2)
#pragma unroll
  for (int rr = 0; rr < 3; ++rr) {
    const int nc = rr * 16 + li;
    a_lane_mr[rr] = lg * DRB + ((((nc >> 2) ^ (4 * (lg & 1))) << 4) | ((nc & 3) << 2));
  }

  {
    const Patch P0 = patch(0);
#pragma unroll
    for (int i = 0; i < GH; ++i) issue_h(P0, i, 0);
#pragma unroll
    for (int i = 0; i < GD; ++i) issue_d(P0, i, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (idle) {   // (staging only: the same pieces, barriers and waits as the multiplying waves)
    for (int k = 0; k < nt; ++k) {
      const int buf = k & 1;
      if (k + 1 < nt) {
        const Patch Pn = patch(k + 1);
#pragma unroll
        for (int r = 0; r < HF_PH; ++r) issue_row(Pn, r, buf ^ 1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    return;
  }
  for (int k = 0; k < nt; ++k) {
    const int buf = k & 1;
    const bool more = k + 1 < nt;
    const Patch Pn = patch(more ? k + 1 : k);
    const uint32_t hb = sbase + buf * STAGE;
    const uint32_t abase = hb + HBUF + a_lane;
    const uint32_t bbase[3] = {hb + b_lane[0], hb + b_lane[1], hb + b_lane[2]};
    float fa[2], fb[2][9];
    auto row_issue = [&](int r) { if (more) issue_row(Pn, r, buf ^ 1); };
    if (!T3 || tsel == 0) {
      hf_read<0, 1>(abase, bbase, fa[0], fb[0]);
      hf_steps<0>(abase, bbase, fa, fb, acc, db, row_issue);
    } else if (tsel == 1) {
      hf_read<0, 1, 0x01F>(abase, bbase, fa[0], fb[0]);
      hf_steps<0, 1, 0x01F>(abase, bbase, fa, fb, acc, db, row_issue);
    } else if (tsel == 2) {
      hf_read<0, 1, 0x1E0>(abase, bbase, fa[0], fb[0]);
      hf_steps<0, 1, 0x1E0>(abase, bbase, fa, fb, acc, db, row_issue);
    } else if (tsel == 3) {
      hf_read<0, 1, 0x07F>(abase, bbase, fa[0], fb[0]);
      hf_steps<0, 1, 0x07F>(abase, bbase, fa, fb, acc, db, row_issue);
    } else {
      const uint32_t ab3[3] = {hb + HBUF + a_lane_mr[0], hb + HBUF + a_lane_mr[1], hb + HBUF + a_lane_mr[2]};
      float fa3[2][3], fb2[2][2];
      hf_read_mr<0>(ab3, bbase, fa3[0], fb2[0]);
      hf_steps_mr<0>(ab3, bbase, fa3, fb2, acc, row_issue);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next patch landed
    __syncthreads();                                    // and nobody reads this stage any more
  }
  // bias gradient (a.bias_part: the launcher's per-block rows, summed in a fixed order by its slab reduce): the
  // column-block-0 waves of the chunk-0 blocks hold each output channel's dY sum over the block's pixels in the four
  // lane rows
  if (a.bias_part && ch == 0 && wc == 0 && tsel != 4) {   // (Z3's multi-row wave sums no bias)
    db += __shfl_xor(db, 16, 64);
    db += __shfl_xor(db, 32, 64);
    const int n = nblk * NB + ncol;
    if (lg == 0 && n < a.Nout) a.bias_part[(size_t)lin * a.Nout + n] = db;
  }
  // dW[n][tap * Cin_s + ch * CI + ccol] += acc[tap][r], n = nblk * NB + wn * 16 + 4 lg + r (the wave's taps)
  const int kc = ch * CI + ccol;
  if (T3 && tsel == 4) {   // Z3's multi-row wave: acc[2 rb + (tap - 7)] of row block rb
#pragma unroll
    for (int rb = 0; rb < 3; ++rb)
#pragma unroll
      for (int t = 7; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nblk * NB + rb * 16 + 4 * lg + r;
          if (n < a.Nout) atomicAdd(a.dW + (size_t)n * a.Kpad + t * Cin_s + kc, acc[2 * rb + t - 7][r]);
        }
    return;
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nblk * NB + wn * 16 + 4 * lg + r;
      if (n < a.Nout && ((tmask >> t) & 1)) atomicAdd(a.dW + (size_t)n * a.Kpad + t * Cin_s + kc, acc[t][r]);
    }
}
template __global__ void igemm_wgrad_halo_f32_kernel<false>(WgradArgs);
template __global__ void igemm_wgrad_halo_f32_kernel<true>(WgradArgs);

// Dilated form of the halo weight gradient (3x3, stride 1, dilation d > 1, 'same'; adipose_v3's bottleneck
// dilate2..dilate6 at d = 2 .. 32, which ran on the register-staged kernel at ~85 TF). A dilation-d conv is d x d
// independent dilation-1 convs on the sub-lattices y = a (mod d), x = b (mod d), so a patch is 4 sub-lattice rows
// (image rows y0 + d r) by 32 output columns, and its halo the same 6 x 34 layout as above: output (r, c) reads halo
// (r + ty, c + tx). Where a sub-lattice row is narrower than 32 (Wo / d < 32) the 32 columns are SPLIT segments of
// Wo / d columns on SPLIT neighbouring sub-lattices b0 .. b0 + SPLIT - 1, each with its own two halo columns (32 + 2
// SPLIT halo columns; the k loop's fragment addresses stay compile-time: hf_col). The pieces are the same 16-B LDS-DMA
// gathers of whole 128-B channel chunks (a strided pixel costs what a neighbouring one does).
// Work: the (channel chunk, output block) x patch items of a layer are cut into gridDim.x contiguous ranges, one per
// block, so the 66 combinations of a 352 -> 352 layer fill every CU (the dilation-1 form gives each combination a
// whole number of blocks: 198 of 256 there); a block flushes its accumulators with f32 atomics where its range
// changes combination, as the dilation-1 form does at its end.
template <int SPLIT>
__global__ __launch_bounds__(512, 1) void igemm_wgrad_halo_f32_dil_kernel(WgradArgs a) {
  constexpr int NTH = 512, CI = 32, NB = 64;
  constexpr int HW = hf_hw<SPLIT>(), SEGW = HF_PW / SPLIT, HROWS = (HF_PH + 2) * HW;
  constexpr int HRB = CI * 4, DRB = NB * 4, NPIX = HF_PH * HF_PW;
  constexpr int HBUF = HROWS * HRB, DBUF = NPIX * DRB, STAGE = HBUF + DBUF;
  constexpr int HCH = HROWS * (HRB / 16), DCH = NPIX * (DRB / 16);
  constexpr int GH = (HCH + NTH - 1) / NTH, GD = DCH / NTH, GT = GH + GD;
  static_assert(GD * NTH == DCH && GT <= 3 * HF_PH, "pieces: at most three per patch row");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int d = a.dil;
  const int nxq = a.Wo / d / SEGW, nbg = d / SPLIT, nyq = a.Ho / d / HF_PH;
  const int T = a.Nimg * d * nyq * nbg * nxq;   // patches per combination
  const int Cin_s = a.CAs + a.CBs, nch = Cin_s / CI, nnb = (a.Nout + NB - 1) / NB, combos = nch * nnb;
  const int G = gridDim.x, blk = xcd_remap(blockIdx.x, G);
  const long long I = (long long)combos * T;
  const int it0 = (int)(I * blk / G), it1 = (int)(I * (blk + 1) / G);
  if (it0 >= it1) return;   // (uniform)
  const size_t npx = (size_t)a.Nimg * a.Hs * a.Ws;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.srcA, 0, npx * a.CAs * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.CBs ? a.srcB : a.srcA), 0, npx * a.CBs * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsD =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dY, 0, a.Nimg * a.Ho * a.Wo * a.dy_stride * 4, 0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  // per-thread parts of the gathers: halo piece -> image row / column offset from the patch origin and byte offset
  // inside the 32-channel chunk; dY piece -> pixel offset and channel inside the 64-channel block
  int hy[GH], hx[GH], hl[GH];
#pragma unroll
  for (int i = 0; i < GH; ++i) {
    const int idx = i * NTH + tid, hr = idx >> 3, pos = idx & 7;
    const int hrow = hr / HW, hcol = hr % HW, sg = hcol / (SEGW + 2), hc = hcol % (SEGW + 2);
    hy[i] = d * (hrow - 1);
    hx[i] = sg + d * (hc - 1);
    hl[i] = 16 * (pos ^ (4 * (hr & 1)));
  }
  int dpix[GD], dq[GD];
#pragma unroll
  for (int i = 0; i < GD; ++i) {
    const int idx = i * NTH + tid, pr = idx >> 4, q = (idx & 15) ^ (4 * (pr & 1));
    const int r = pr >> 5, c = pr & 31;
    dpix[i] = d * r * a.Wo + c / SEGW + d * (c % SEGW);
    dq[i] = 4 * q;
  }
  struct Cmb { int ch, nb, xcs, xc0; bool inA; };
  auto cmb = [&](int c) {
    Cmb C;
    C.ch = c % nch;
    C.nb = c / nch;
    C.inA = C.ch * CI < a.CAs;
    C.xcs = C.inA ? a.CAs : a.CBs;
    C.xc0 = (C.inA ? C.ch * CI : C.ch * CI - a.CAs) * 4;
    return C;
  };
  struct Patch { int img, y0, x0, pbd; };
  auto patch = [&](int t) {   // t -> (img, sub-lattice row a, patch row, column group b0, patch column)
    Patch P;
    const int px = t % nxq, t1 = t / nxq, bg = t1 % nbg, t2 = t1 / nbg, yq = t2 % nyq, t3 = t2 / nyq;
    P.img = t3 / d;
    P.y0 = t3 % d + d * yq * HF_PH;
    P.x0 = bg * SPLIT + d * px * SEGW;
    P.pbd = (P.img * a.Ho + P.y0) * a.Wo + P.x0;
    return P;
  };
  auto issue_h = [&](const Patch& P, const Cmb& C, int i, int buf) {
    const int idx = i * NTH + tid;
    if (i < GH - 1 || idx < HCH) {
      const int gy = P.y0 + hy[i], gx = P.x0 + hx[i];
      const bool ok = (unsigned)gy < (unsigned)a.Hs && (unsigned)gx < (unsigned)a.Ws;
      const unsigned off = ok ? (unsigned)(((P.img * a.Hs + gy) * a.Ws + gx) * C.xcs * 4 + C.xc0 + hl[i]) : OOB;
      hf_buf_lds16(C.inA ? rsA : rsB, smem + buf * STAGE + (size_t)(i * NTH + wave * 64) * 16, off);
    }
  };
  auto issue_d = [&](const Patch& P, const Cmb& C, int i, int buf) {
    const int cc = C.nb * NB + dq[i];
    const unsigned off = cc < a.Nout ? (unsigned)((P.pbd + dpix[i]) * a.dy_stride * 4 + cc * 4) : OOB;
    hf_buf_lds16(rsD, smem + buf * STAGE + HBUF + (size_t)(i * NTH + wave * 64) * 16, off);
  };
  auto issue_row = [&](const Patch& P, const Cmb& C, int r, int buf) {   // the pieces that ride on patch row r
#pragma unroll
    for (int g = 0; g < GT; ++g)
      if (g * HF_PH / GT == r) {
        if (g < GH) issue_h(P, C, g, buf);
        else issue_d(P, C, g - GH, buf);
      }
  };

  f32x4 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db = 0.f;
  const int wn = wave >> 1, wc = wave & 1;
  const int li = lane & 15, lg = lane >> 4;
  const int ncol = wn * 16 + li, ccol = wc * 16 + li;
  const uint32_t sbase = wf_lds(smem);
  const uint32_t a_lane = lg * DRB + ((((ncol >> 2) ^ (4 * (lg & 1))) << 4) | ((ncol & 3) << 2));
  uint32_t b_lane[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
    b_lane[dx] = (lg + dx) * HRB + ((((ccol >> 2) ^ (4 * ((lg + dx) & 1))) << 4) | ((ccol & 3) << 2));

  {
    const Cmb C0 = cmb(it0 / T);
    const Patch P0 = patch(it0 % T);
#pragma unroll
    for (int i = 0; i < GH; ++i) issue_h(P0, C0, i, 0);
#pragma unroll
    for (int i = 0; i < GD; ++i) issue_d(P0, C0, i, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int it = it0; it < it1; ++it) {
    const int buf = (it - it0) & 1;
    const bool more = it + 1 < it1;
    const int itn = more ? it + 1 : it;
    const Cmb Cn = cmb(itn / T);
    const Patch Pn = patch(itn % T);
    const uint32_t hb = sbase + buf * STAGE;
    const uint32_t abase = hb + HBUF + a_lane;
    const uint32_t bbase[3] = {hb + b_lane[0], hb + b_lane[1], hb + b_lane[2]};
    float fa[2], fb[2][9];
    hf_read<0, SPLIT>(abase, bbase, fa[0], fb[0]);
    hf_steps<0, SPLIT>(abase, bbase, fa, fb, acc, db, [&](int r) { if (more) issue_row(Pn, Cn, r, buf ^ 1); });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next item landed
    __syncthreads();                                    // and nobody reads this stage any more
    if (more && (it + 1) % T != 0) continue;
    // the block's last item of this combination: bias row (block blk of the launcher's [G][Nout] rows) and dW atomics
    const Cmb C = cmb(it / T);
    if (a.bias_part && C.ch == 0 && wc == 0) {
      float s = db;
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const int n = C.nb * NB + ncol;
      if (lg == 0 && n < a.Nout) a.bias_part[(size_t)blk * a.Nout + n] = s;
    }
    const int kc = C.ch * CI + ccol;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = C.nb * NB + wn * 16 + 4 * lg + r;
        if (n < a.Nout) atomicAdd(a.dW + (size_t)n * a.Kpad + t * Cin_s + kc, acc[t][r]);
        acc[t][r] = 0.f;
      }
    db = 0.f;
  }
}

template __global__ void igemm_wgrad_halo_f32_dil_kernel<1>(WgradArgs);
template __global__ void igemm_wgrad_halo_f32_dil_kernel<2>(WgradArgs);
template __global__ void igemm_wgrad_halo_f32_dil_kernel<4>(WgradArgs);
template __global__ void igemm_wgrad_halo_f32_dil_kernel<8>(WgradArgs);

// f32 weight gradient of a one-real-channel input layer (adipose_v3's down1_conv1: the gray tile in an 8-channel
// stride, <= 64 output channels): dW[n][t * 8] = sum_p dY[p][n] X[p + off_t][0] and dB[n] = sum_p dY[p][n]. The
// products are 2 M x 64 x 10 per 1024^2 tile -- nothing -- and dY is 256 B a pixel: the launch streams dY once. The
// generic register-staged kernel tiled K = 72 in 64-wide blocks and ran at ~1.5 TB/s. Here one v_mfma_f32_16x16x4_f32
// per 4 pixels and 16 channels: A = the tap-shifted input (row i = tap i < 9, row 9 = ones for the bias, k = pixel),
// B = dY (k = pixel, column j = channel 4 j + q of block q: one float4 load per lane and 4 pixels, 1 KB per wave
// instruction). 8 waves a block, each a strided run of 4-pixel steps; the waves' sums are added in LDS in wave order
// and each block writes one slab (dW layout, zero pad columns) and one bias row, summed in a fixed order by the slab
// reduce: deterministic.
__global__ __launch_bounds__(512) void wgrad_in1_f32_kernel(WgradArgs a, float* part, float* bpart) {
  constexpr int NW = 8, UNR = 8;
  __shared__ float red[NW][64 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = gridDim.x, blk = blockIdx.x;
  const int per = ((a.M + G - 1) / G + 4 * NW - 1) / (4 * NW) * (4 * NW);
  const int p0 = blk * per, p1 = min(a.M, p0 + per);
  const int i = lane & 15, kq = lane >> 4;
  const int ty = i / 3 - 1, tx = i % 3 - 1;
  const int HW = a.Ho * a.Wo;
  const float* X = reinterpret_cast<const float*>(a.srcA);
  const float4* dy4 = reinterpret_cast<const float4*>(a.dY);
  const int ds4 = a.dy_stride / 4;
  f32x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int pb = p0 + 4 * wave; pb < p1; pb += 4 * NW * UNR) {
    float av[UNR];
    float4 bv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int p = pb + u * 4 * NW + kq;
      const bool in = p < p1;
      bv[u] = in ? dy4[(size_t)p * ds4 + i] : float4{0.f, 0.f, 0.f, 0.f};
      float v = 0.f;
      if (in && i < 10) {
        if (i == 9) {
          v = 1.f;
        } else {
          const int n = p / HW, rem = p - n * HW, y = rem / a.Wo, x = rem - y * a.Wo;
          const int yy = y + ty, xx = x + tx;
          if ((unsigned)yy < (unsigned)a.Hs && (unsigned)xx < (unsigned)a.Ws)
            v = X[((size_t)(n * a.Hs + yy) * a.Ws + xx) * a.CAs];
        }
      }
      av[u] = v;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u].x, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u].y, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u].z, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u].w, acc[3], 0, 0, 0);
    }
  }
  // D[i][j] of block q at lane j + 16 (i >> 2), register i & 3: tap / ones row i, channel n = 4 j + q
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][(4 * (lane & 15) + q) * 16 + 4 * (lane >> 4) + r] = acc[q][r];
  __syncthreads();
  // slab: [Nout][Kpad] (tap t at column 8 t, the other columns zero), bias row [Nout]
  float* slab = part + (size_t)blk * a.Nout * a.Kpad;
  for (int e = tid; e < a.Nout * a.Kpad; e += 512) {
    const int n = e / a.Kpad, c = e - n * a.Kpad;
    float v = 0.f;
    if ((c & 7) == 0 && c < 72) {
      const int t = c >> 3;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[w][n * 16 + t];
    }
    slab[e] = v;
  }
  if (bpart)
    for (int n = tid; n < a.Nout; n += 512) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[w][n * 16 + 9];
      bpart[(size_t)blk * a.Nout + n] = v;
    }
}

template <int WN, int WK>
void launch_f32cfg(WgradArgs& a, hipStream_t s) {
  constexpr int TN = WN * 64, TK = WK * 64;
  a.ntile_k = (a.K + TK - 1) / TK;
  a.ntile_n = (a.Nout + TN - 1) / TN;
  const int tiles = a.ntile_k * a.ntile_n;
  const int target = adp::option("wgrad_f32_blocks", 1024), min_chunk = adp::option("wgrad_f32_min_chunk", 1024);
  int splits = (target + tiles - 1) / tiles;
  const int maxsplit = (a.M + min_chunk - 1) / min_chunk;
  splits = std::max(1, std::min(splits, maxsplit));
  a.mchunk = ((a.M + splits - 1) / splits + 31) / 32 * 32;
  splits = (a.M + a.mchunk - 1) / a.mchunk;
  const size_t slab = (size_t)a.Nout * a.Kpad;
  a.part = nullptr;
  if (splits > 1 && adp::option("wgrad_f32_partials", TN >= 256 ? 1 : 0))
    a.part = static_cast<float*>(adp::scratch(0, slab * splits * sizeof(float)));
  adp::set_kernel("igemm_wgrad_f32_kernel<%d, %d>", WN, WK);
  hipLaunchKernelGGL((igemm_wgrad_f32_kernel<WN, WK>), dim3(tiles * splits), dim3(WN * WK * 64), 0, s, a);
  adp::kernel_end();
  if (a.part) {
    const int blocks = (int)std::min<size_t>((slab / 4 + 255) / 256, 4096);
    hipLaunchKernelGGL(wgrad_f32_reduce_kernel, dim3(blocks), dim3(256), 0, s, splits, slab,
                       reinterpret_cast<const float4*>(a.part), reinterpret_cast<float4*>(a.dW));
  }
}

}  // namespace

namespace adp {
// f32 weight gradient on the LDS-DMA kernel: any stride / dilation / padding / nearest-x2 gather, one or two
// sources, plain or pixel-shuffle dY, no BN-apply on load; 0 = not eligible (the caller falls back)
int launch_wgrad_f32(WgradArgs& a, hipStream_t s) {
  // opt-in: on adipose_v3's f32 layers (44 * 2^l channels, K = 9 Cin_s) its 64-granular N tiles and 128-512-wide
  // K tiles run 39-66 % full, and it measured 62-64 TF against the register-staged kernel's 84 TF
  // (profiles/r03_wgrad_f32_ab.txt)
  if (a.scA || a.scB || a.bna_dA) return 0;
  const int Cin_s = a.CAs + a.CBs;
  // one real input channel (the caller's hint) in a stride of 8, <= 64 outputs (option wgrad_f32_in1)
  if (option("wgrad_f32_in1", 1) && a.ca_real == 1 && a.CAs == 8 && a.CBs == 0 && a.kh == 3 && a.kw == 3 &&
      a.dil == 1 && a.pad == 1 && a.stride == 1 && a.up == 1 && a.Ho == a.Hs && a.Wo == a.Ws && a.Nout <= 64 &&
      a.Nout % 4 == 0 && a.dy_mode == 0 && a.K == 72 && a.Kpad >= 72 && a.Kpad % 4 == 0 && a.dy_stride % 4 == 0 &&
      a.dy_stride >= 64 && a.srcA && a.M > 0) {
    const int G = std::max(1, std::min(option("wgrad_f32_in1_grid", 256), (a.M + 31) / 32));
    float* part = reduce_part(0, (size_t)G * a.Nout * a.Kpad * sizeof(float), s);
    float* bpart = a.dB ? reduce_part(3, (size_t)G * a.Nout * sizeof(float), s) : nullptr;
    if (part && (bpart || !a.dB)) {
      adp::set_kernel("wgrad_in1_f32_kernel");
      hipLaunchKernelGGL(wgrad_in1_f32_kernel, dim3(G), dim3(512), 0, s, a, part, bpart);
      adp::kernel_end();
      slab_reduce(G, (size_t)a.Nout * a.Kpad / 4, part, a.dW, s);
      if (bpart) {
        slab_reduce(G, (size_t)a.Nout / 4, bpart, a.dB, s);
        a.dB = nullptr;   // (done: the caller's channel-sum launch is skipped)
      }
      return 1;
    }
  }
  // the persistent halo form (option wgrad_f32_halo): 3x3 stride-1 'same' layers of 32-channel multiples
  if (option("wgrad_f32_halo", 1) && a.kh == 3 && a.kw == 3 && a.dil == 1 && a.pad == 1 && a.stride == 1 &&
      (a.up == 1 || a.up == 2) && a.Ho == a.Hs * a.up && a.Wo == a.Ws * a.up && a.Ho % HF_PH == 0 &&
      a.Wo % HF_PW == 0 && a.CAs % 32 == 0 && a.CBs % 32 == 0 && a.Nout % 32 == 0 && a.dy_mode == 0 &&
      a.K == 9 * Cin_s && a.Kpad >= a.K && a.dy_stride % 4 == 0 && a.dy_stride >= a.Nout &&
      a.srcA && (!a.CBs || a.srcB) &&
      (size_t)a.Nimg * a.Hs * a.Ws * std::max(a.CAs, a.CBs) * 4 < ((size_t)1 << 31) &&
      (size_t)a.M * a.dy_stride * 4 < ((size_t)1 << 31)) {
    const int nch = Cin_s / 32, combos = nch * ((a.Nout + 63) / 64);
    const int tiles = a.Nimg * (a.Ho / HF_PH) * (a.Wo / HF_PW);
    const int target = option("wgrad_f32_halo_grid", 256);
    const int per = std::max(1, std::min(tiles, target / combos));
    int grid = per * combos;
    // zero tails (the caller's real channel counts; option wgrad_f32_zt): a combination whose input chunk holds
    // <= 16 real channels runs its <= 4 useful 16 x 16 blocks one per SIMD, and since round 6 one whose output
    // block holds <= 2 real 16-row blocks runs them on 2 rb waves (row tails, option wgrad_f32_rt); either takes
    // ~60 % of a full patch's time (option wgrad_f32_zt_w, percent; 50 and 70 measured slower,
    // profiles/r06f_f32_wgrad_probe.log) and gets blocks in proportion
    a.zt_n = 0;
    bool t3 = false;   // (a combination in the tap-split form: the T3 instance)
    if (option("wgrad_f32_zt", 1) && combos <= std::min(ZT_MAX, option("wgrad_f32_zt_max", ZT_MAX)) &&
        (a.ca_real > 0 || a.cb_real > 0 || a.nout_real > 0)) {
      const bool rows_too = option("wgrad_f32_rt", 1) && a.nout_real > 0;
      const bool t3_ok = option("wgrad_f32_t3", 1) && a.nout_real > 0;
      // (per-mode weights, profiles/r06ab_probe.log: chunk tails 60 %, row tails 55 % -- the level-1 layers ran 2-4 %
      //  faster at 55 than at 60, the level-0 chunk tails 5 % slower --, the T3 split 85 %)
      const double wt = option("wgrad_f32_zt_w", 60) / 100.0, w3 = option("wgrad_f32_t3_w", 85) / 100.0;
      const double wr = option("wgrad_f32_rt_w", 55) / 100.0, wz3 = option("wgrad_f32_z3_w", 47) / 100.0;
      const bool z3_ok = option("wgrad_f32_z3", 1) != 0;
      double w[ZT_MAX], tot = 0.0;
      bool any = false;
      for (int c = 0; c < combos; ++c) {
        const int ch = c % nch, nb = c / nch;
        const bool inA = ch * 32 < a.CAs;
        const int rsrc = inA ? a.ca_real : a.cb_real, c0 = inA ? ch * 32 : ch * 32 - a.CAs;
        const int rin = rsrc > 0 ? std::min(32, std::max(0, rsrc - c0)) : 32;
        const int rows = a.nout_real > 0 ? std::min(64, std::max(0, a.nout_real - nb * 64)) : 64;
        const int rb = (rows + 15) / 16;
        a.zt_mode[c] = rin <= 16 && rb == 3 && z3_ok ? 64 + 3
                       : rin <= 16 && rb >= 1         ? rb
                       : rows_too && rb >= 1 && rb <= 2 ? 16 + rb
                       : t3_ok && rb == 3             ? 32 + 3
                                                      : 0;
        any = any || a.zt_mode[c] > 0;
        t3 = t3 || a.zt_mode[c] >= 32;
        w[c] = a.zt_mode[c] >= 64 ? wz3 : a.zt_mode[c] >= 32 ? w3 : a.zt_mode[c] >= 16 ? wr : a.zt_mode[c] > 0 ? wt : 1.0;
        tot += w[c];
      }
      if (any) {
        // blocks per combination: one each, then greedily to the combination with the longest weighted time
        // w ceil(tiles / n) until the target is reached (never more blocks than the target: a second round of
        // blocks would double the launch)
        (void)tot;
        int n[ZT_MAX], used = combos;
        for (int c = 0; c < combos; ++c) n[c] = 1;
        while (used < target) {
          int best = -1;
          double bt = 0.0;
          for (int c = 0; c < combos; ++c) {
            const double t = w[c] * ((tiles + n[c] - 1) / n[c]);
            if (n[c] < tiles && t > bt) { bt = t; best = c; }
          }
          if (best < 0) break;
          ++n[best];
          ++used;
        }
        a.zt_n = combos;
        a.zt_cstart[0] = 0;
        for (int c = 0; c < combos; ++c) a.zt_cstart[c + 1] = a.zt_cstart[c] + n[c];
        grid = a.zt_cstart[combos];
      }
    }
    // the bias gradient in the same pass (option wgrad_f32_bias): per-block rows [G0][Nout] (G0 = the blocks of
    // each chunk-0 combination), zeroed first (blocks without patches and idle waves write nothing), then the
    // fixed-order slab reduce into dB -- instead of a channel-sum launch that reads dY once more
    a.bias_part = nullptr;
    int g0 = 0;
    if (a.dB && a.Nout % 4 == 0 && option("wgrad_f32_bias", 1)) {
      // (one row per block index of the chunk-0 combinations; a combination with fewer blocks leaves its other
      // rows zero)
      g0 = per;
      if (a.zt_n) {
        g0 = 0;
        for (int c = 0; c < combos; c += nch) g0 = std::max(g0, a.zt_cstart[c + 1] - a.zt_cstart[c]);
      }
      a.bias_part = reduce_part(3, (size_t)g0 * a.Nout * sizeof(float), s);
      if (a.bias_part && hipMemsetAsync(a.bias_part, 0, (size_t)g0 * a.Nout * sizeof(float), s) != hipSuccess)
        a.bias_part = nullptr;
    }
    t3 = t3 && a.zt_n;
    adp::set_kernel(t3 ? "igemm_wgrad_halo_f32_kernel<true>" : "igemm_wgrad_halo_f32_kernel<false>");
    if (t3) hipLaunchKernelGGL((igemm_wgrad_halo_f32_kernel<true>), dim3(grid), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((igemm_wgrad_halo_f32_kernel<false>), dim3(grid), dim3(512), 0, s, a);
    if (a.bias_part) {
      adp::kernel_end();
      slab_reduce(g0, (size_t)a.Nout / 4, a.bias_part, a.dB, s);
      a.dB = nullptr;   // (done: the caller's channel-sum launch is skipped)
      a.bias_part = nullptr;
    }
    adp::kernel_end();
    return 1;
  }
  // the dilated halo form (option wgrad_f32_dil): the same layers at dilation d > 1 whose sub-lattices tile into
  // 4-row patches and whose rows into 32 / SPLIT-column segments (SPLIT <= 8, d a multiple of SPLIT)
  if (option("wgrad_f32_dil", 1) && a.kh == 3 && a.kw == 3 && a.dil > 1 && a.pad == a.dil && a.stride == 1 &&
      a.up == 1 && a.Ho == a.Hs && a.Wo == a.Ws && a.Ho % a.dil == 0 && a.Wo % a.dil == 0 &&
      (a.Ho / a.dil) % HF_PH == 0 && a.CAs % 32 == 0 && a.CBs % 32 == 0 && a.Nout % 32 == 0 && a.dy_mode == 0 &&
      a.K == 9 * Cin_s && a.Kpad >= a.K && a.dy_stride % 4 == 0 && a.dy_stride >= a.Nout && a.srcA &&
      (!a.CBs || a.srcB) && (size_t)a.Nimg * a.Hs * a.Ws * std::max(a.CAs, a.CBs) * 4 < ((size_t)1 << 31) &&
      (size_t)a.M * a.dy_stride * 4 < ((size_t)1 << 31)) {
    const int wq = a.Wo / a.dil;
    const int split = wq >= HF_PW ? (wq % HF_PW == 0 ? 1 : 0) : (HF_PW % wq == 0 ? HF_PW / wq : 0);
    if (split >= 1 && split <= 8 && a.dil % split == 0) {
      const int combos = Cin_s / 32 * ((a.Nout + 63) / 64);
      const long long items = (long long)combos * a.Nimg * (a.Ho / HF_PH) * (a.Wo / HF_PW);
      const int grid = (int)std::max(1LL, std::min<long long>(items, option("wgrad_f32_dil_grid", 256)));
      a.zt_n = 0;
      a.bias_part = nullptr;
      if (a.dB && a.Nout % 4 == 0 && option("wgrad_f32_bias", 1)) {
        a.bias_part = reduce_part(3, (size_t)grid * a.Nout * sizeof(float), s);
        if (a.bias_part && hipMemsetAsync(a.bias_part, 0, (size_t)grid * a.Nout * sizeof(float), s) != hipSuccess)
          a.bias_part = nullptr;
      }
      adp::set_kernel("igemm_wgrad_halo_f32_dil_kernel<%d>", split);
      if (split == 1) hipLaunchKernelGGL((igemm_wgrad_halo_f32_dil_kernel<1>), dim3(grid), dim3(512), 0, s, a);
      else if (split == 2) hipLaunchKernelGGL((igemm_wgrad_halo_f32_dil_kernel<2>), dim3(grid), dim3(512), 0, s, a);
      else if (split == 4) hipLaunchKernelGGL((igemm_wgrad_halo_f32_dil_kernel<4>), dim3(grid), dim3(512), 0, s, a);
      else hipLaunchKernelGGL((igemm_wgrad_halo_f32_dil_kernel<8>), dim3(grid), dim3(512), 0, s, a);
      if (a.bias_part) {
        adp::kernel_end();
        slab_reduce(grid, (size_t)a.Nout / 4, a.bias_part, a.dB, s);
        a.dB = nullptr;
        a.bias_part = nullptr;
      }
      adp::kernel_end();
      return 1;
    }
  }
  if (!option("wgrad_f32", 0)) return 0;
  if (a.CAs % 4 != 0 || a.CBs % 4 != 0 || a.K != a.kh * a.kw * Cin_s || a.Kpad % 4 != 0 || a.Kpad < a.K ||
      a.dy_stride % 4 != 0 || a.Nout % 4 != 0 || (a.dy_mode == 1 && a.Cps % 4 != 0))
    return 0;
  if (!a.srcA || (a.CBs && !a.srcB)) return 0;
  int cfg = option("wgrad_f32_cfg", 0);   // 1: 64 x 512, 2: 128 x 256, 3: 256 x 128 (n x k tile)
  if (cfg < 1 || cfg > 3) cfg = a.Nout <= 64 ? 1 : a.Nout <= 128 ? 2 : 3;
  if (cfg == 1) launch_f32cfg<1, 8>(a, s);
  else if (cfg == 2) launch_f32cfg<2, 4>(a, s);
  else launch_f32cfg<4, 2>(a, s);
  return 1;
}
}  // namespace adp
