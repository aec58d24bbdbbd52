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
  if (!option("wgrad_f32", 0) || a.scA || a.scB || a.bna_dA) return 0;
  const int Cin_s = a.CAs + a.CBs;
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
