// Shared pieces of the implicit-GEMM convolution kernels (conv_igemm.hip, conv_fwd_tap64.hip):
// the forward-shaped launch arguments, the XCD-aware block remap and the LDS-staged epilogue.
#pragma once
#include "common.h"

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
  // fused BatchNorm-backward reduction of the stored output (see adp_conv_io.bnr_*)
  const void* bnr_z; int bnr_zs;
  const float* bnr_sc; const float* bnr_sh; const float* bnr_mean; const float* bnr_invstd;
  float* bnr_dgamma; float* bnr_dbeta;
  int M;
  int ntile_n;           // gridDim decomposition helper
  int nblocks;
  // fp8 (OCP e4m3fn) forward launches: operands are fp8, acc[n] is dequantised by wscale[n] (per GEMM
  // column; activations carry no scale); out_f8 stores the output as fp8 too (else bf16)
  int f8;
  const float* wscale;
  int out_f8;
  int stagger;           // persistent forward: waves 4-7 issue their LDS-DMA after the first MFMA cluster
  int wide_st;           // persistent forward: 16-B epilogue stores (channel pairs joined by permlane16_swap)
  int kpipe;             // tap64 kernel: mid-step barrier, next step's B half 0 preloaded (option tap64_kpipe)
  int debug_flags;       // timing-only ablations (option "fwd_debug"): bit1 skips the BN-statistics atomics
  double* stat;          // BatchNorm accumulator replicas (f64) (adp::stat_scratch) for bn_sum / bnr_* launches
  int defer_fold;        // bn_sum launch whose replica sums adp_bn_finalize_fold adds in (adp_conv_desc)
  int f32;               // f32 launch on the LDS-DMA tap kernel (32-channel K steps, f32 MFMA)
  int f32_skip;          // f32 256x128 tiles: 32-column groups past Nout skip their MFMAs (option f32_skip)
  int* claim;            // persistent kernels: dynamic tile claiming counters (adp::claim_slot), nullptr = static lists
  int claim_chunk;       // tiles per claim (halo forward: consecutive patches taken together)
  int claim_full;        // claiming: every tile claimed, none static (option claim_full; conv_common.h)
  void* act_out;         // with scA / shA: relu(srcA * scA + shA) stored here too (adp_conv_io.act_outA)
  int bnr_lds;           // tap64 BN-backward-reduction launches: the LDS-staged epilogue (option tap64_bnr_lds)
  int mask_lds;          // tap64 mask / addend launches: mask and addend rows by LDS-DMA (option tap64_mask_lds)
  int ca_real;           // adp_conv_desc.CA_real (0 = unknown)
  int ztail;             // zero tails of the weights (adp_conv_desc CA_real / CB_real / Nout_real): bit 0 every source a
                         // 64-channel stride with <= 48 real channels, bit 1 Nout == 64 with <= 48 real columns
  // tap64 split-K (round 6, option tap64_ksplit): ksplit > 1 blocks per output tile, each a contiguous K range; the
  // partial accumulators go to kpart, the tile's last block (counter kcnt[tile], re-zeroed by it) sums them in split
  // order and runs the epilogue
  int ksplit;
  float* kpart;
  int* kcnt;
};

// weight-gradient launch arguments: dW[n][k] += sum_m dY[m][n] * X(k)[m]
constexpr int ZT_MAX = 40;   // combinations the f32 halo weight gradient's zero-tail table holds
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
  int debug_flags;      // timing-only ablations (tools/bench_kernels.py): bit0 skips the dW atomics
  float* part;          // tap64: per-split partial dW slabs [split][Nout][Kpad] (plain stores), reduced
                        // into dW by a second launch; nullptr -> f32 atomics into dW (halo weight gradient: one
                        // slab per block index within its (chunk, output block) combination, fixed-order reduce)
  int part_rmw;         // halo weight gradient with one block per combination: dW += partial by plain
                        // load + store (the block owns its dW rows), no slab, no atomics
  // fused BatchNorm-backward apply (adp_conv_wgrad_bn): dY = bn_bwd_apply(bna_dA, bna_z) of the layer's
  // BatchNorm, computed on load and stored into dY (all three [M][dy_stride]); bna_dA == nullptr: plain dY
  const void* bna_dA; const void* bna_z;
  const float* bna_sc; const float* bna_sh; const float* bna_mean; const float* bna_invstd;
  const float* bna_gamma; const float* bna_dgamma; const float* bna_dbeta;
  float bna_inv_count;
  int* claim;           // persistent halo weight gradient: dynamic tile claiming counters (nullptr: static lists)
  int claim_chunk;      // patches per claim
  int claim_full;       // every super-patch claimed, none static (option claim_full)
  // f32 halo weight gradient, zero tails (adp_conv_desc CA_real / CB_real / Nout_real; 0 = unknown): zt_n > 0 ->
  // combination c takes the blocks [zt_cstart[c], zt_cstart[c + 1]); zt_mode[c] > 0 -> its input chunk has <= 16 real
  // channels, and waves 0 .. zt_mode[c] - 1 take its useful 16 x 16 blocks (one per wave), the others only stage
  int ca_real, cb_real, nout_real;
  int zt_n;
  // (zt_mode[c] >= 16: row tails -- the output block holds zt_mode[c] - 16 <= 2 real 16-row blocks and waves 0 ..
  // 2 (zt_mode[c] - 16) - 1 take them with both input column blocks; round 6)
  int zt_cstart[ZT_MAX + 1];
  int zt_mode[ZT_MAX];
  float* bias_part;     // f32 halo weight gradient: per-block bias-gradient rows (option wgrad_f32_bias)
};

// LDS-only workgroup barrier for epilogues: this wave's LDS traffic complete, then s_barrier. Unlike
// __syncthreads() (whose workgroup fence waits for vmcnt = 0) it does not stall behind the wave's own
// global stores or loads still in flight; use it only where the barrier orders LDS accesses alone.
#define ADP_LDS_BARRIER()                                     \
  do {                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
    __builtin_amdgcn_s_barrier();                             \
    asm volatile("" ::: "memory");                            \
  } while (0)

namespace {

// sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15), every lane receives it: xor-1 and xor-2 quad
// permutes, then the half-row and row mirrors (after the quad steps the lanes of a quad hold equal values,
// so a mirror adds exactly what xor 4 / xor 8 would) -- the butterfly of __shfl_xor(v, 1..8) term for term,
// as four DPP-modified VALU adds instead of four ds_bpermute round trips through the LDS pipe
// MFMA-cluster wave priority of the hot K loops, per kernel family (build-time, A/B only): 0 = s_setprio 1
// around each MFMA cluster (default); 1 = no priority changes; 2 = the second-dispatched half of a 512-thread
// block (waves 4-7) at priority 1 for the whole kernel, no per-cluster flips; 3 = the first half instead.
// Same-box A/B of library builds (profiles/r03_prio_ab.txt): on the forwards every mode is within the 1-2 %
// drift of consecutive runs on one box; on the persistent weight gradient modes 1-3 cost 3-4 %.
#ifndef ADP_PRIO_FWD
#define ADP_PRIO_FWD 0
#endif
#ifndef ADP_PRIO_WGRAD
#define ADP_PRIO_WGRAD 0
#endif
#ifndef ADP_PRIO_T64
#define ADP_PRIO_T64 0   // the non-persistent tap kernel (conv_fwd_tap64.hip)
#endif
template <int M>
__device__ __forceinline__ void prio_hi() {
  if constexpr (M == 0) __builtin_amdgcn_s_setprio(1);
}
template <int M>
__device__ __forceinline__ void prio_lo() {
  if constexpr (M == 0) __builtin_amdgcn_s_setprio(0);
}
template <int M>
__device__ __forceinline__ void prio_static(int wave) {
  if constexpr (M == 2) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  } else if constexpr (M == 3) {   // (A/B only: the first-dispatched half instead)
    if (wave < 4) __builtin_amdgcn_s_setprio(1);
  }
}
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

typedef __attribute__((address_space(3))) void lds_void;
typedef short v4s16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s16 lds_v4s16;


// XCD-aware bijective remap of the linear block id: each XCD (blocks b, b+8, ...) receives a
// contiguous run of tiles, N-tile fastest, so the A (activation) panel of one M-tile is shared
// through one XCD's L2 by all its N-tiles.
ADP_DEV int xcd_remap(int bid, int nwg) {
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// ------------------------------------------------ dynamic tile claiming (persistent kernels)
// A persistent kernel whose blocks walk static tile lists (lin, lin + G, ...) runs ~2x long when a kernel on
// another stream (RCCL's all-reduce blocks) holds a few CUs: the blocks that find no free CU run their whole
// list after the others (profiles/r03_contention_probe.txt). With claiming, a block takes its next tile from
// a per-N-column counter (claim[col], vector atomics at agent scope, one tile ahead of the multiply so the
// cross-tile prefetch stays), and a block that starts late finds the work taken. claim[nclaim] counts the
// blocks that are done; the last one re-zeroes the counters, so the next launch on the slot starts from 0.
// read of a claimed tile id from the block's LDS ring as inline asm: a plain LDS read gets an s_waitcnt vmcnt(0)
// in front whenever LDS-DMA or a claim atomic may be in flight (the compiler cannot tell the ring from the DMA
// targets), which would drain the prefetch or wait for the pending claim
ADP_DEV int claim_ring_read(const int* p) {
  int r;
  const unsigned addr = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
  return __builtin_amdgcn_readfirstlane(r);
}
// (the prologue's synchronous claim of a block's first two tiles; the atomic optimizer's wave form is fine here)
ADP_DEV int claim_next2(int* cnt) {
  return __hip_atomic_fetch_add(cnt, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// In the K loop the claim must not stall. The atomic is compiler-visible (so every use of its result is ordered
// after its return by the compiler's own vmcnt accounting), in files built without the atomic optimizer
// (-amdgpu-atomic-optimizer-strategy=None, Makefile NOATOMOPT), whose wave form would broadcast the result at once
// and put an s_waitcnt vmcnt(0) right behind the atomic, draining the LDS-DMA prefetch. claim_publish stores the
// value into the LDS ring a step later; the compiler waits for the atomic in front of it (round 4 kept the atomic
// in inline asm with a hand-counted vmcnt, which the compiler could not see: a copy of the pending register in
// between would have read a stale tile id -- round-4 ADVICE; tests/test_isa.py walks the code for such reads)
ADP_DEV int claim_issue(int* cnt) {
  return __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (NYOUNG: kept for the call sites' documentation of how many vector-memory ops follow the atomic; the wait is the
// compiler's)
template <int NYOUNG>
ADP_DEV void claim_publish(int* lds, int r) {
  const unsigned addr = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(r) : "memory");
}
// claim_full (option claim_full): a block's first two tiles are claimed too -- one synchronous claim of two at
// the start (claim_next2) -- instead of being its static ones. With static first tiles a block whose CU is
// held by another stream's kernel when the launch starts still owns them and runs them after everyone else
// is done (+4.3 ms per step with 8 CUs held for 20 ms: profiles/r04_contention_probe.txt); claimed, a late
// block finds the work taken and leaves. The price is the claim's round trip at the start of every block.
// every block calls this exactly once, after its last claim (thread 0; nclaim counters + the done count)
ADP_DEV void claim_block_done(int* claim, int nclaim, int G) {
  const int done = __hip_atomic_fetch_add(claim + nclaim, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (done == G - 1) {
    for (int i = 0; i < nclaim; ++i) __hip_atomic_store(claim + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(claim + nclaim, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// XOR swizzle of the 16-B chunks of a 128-B LDS row (rows of 64 bf16): chunk c of row r is stored at
// position c ^ swz(r); makes the 16x16x32 MFMA fragment reads (16 rows x one 16-B chunk per 16-lane
// group) bank-conflict free.
ADP_DEV int swz(int r) { return (r >> 1) & 7; }

// ------------------------------------------------ transposed fragment reads (weight gradient)
// Operands X[pixel][k] and dY[pixel][n] sit in LDS as linear rows of RB bytes (pixel = row); 16-B
// chunk c of row r is stored at chunk position c ^ gsw(r), gsw(r) = 2*(r & 7) for RB >= 256 and
// 2*((r >> 1) & 3) for RB = 128, which spreads the 8 rows read by one 32-lane half of a
// ds_read_b64_tr_b16 over 8 distinct 32-B bank slots. Inside a 32-pixel MFMA k step the pixel order
// is permuted, rho(8g+e) = 16(g>>1) + 8(e>>2) + 4(g&1) + (e&3), so that the 8 rows one half-wave
// reads are 8 consecutive LDS rows (both operands use the same permutation).
template <int RB>
ADP_DEV int gsw(int r) { return RB >= 256 ? 2 * (r & 7) : 2 * ((r >> 1) & 3); }

template <int RB>
ADP_DEV bf16x8 tr_frag_sw(const unsigned char* base, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = row0 + 16 * (g >> 1) + 4 * (g & 1) + q;
  const int r1 = r0 + 8;
  const int col = col0 + 4 * p;
  const int chunk = col >> 3, inb = (col & 7) * 2;
  const unsigned char* a0 = base + r0 * RB + ((chunk ^ gsw<RB>(r0)) << 4) + inb;
  const unsigned char* a1 = base + r1 * RB + ((chunk ^ gsw<RB>(r1)) << 4) + inb;
  v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(a0));
  v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(a1));
  bf16x8 r;
  const bf16* l = reinterpret_cast<const bf16*>(&lo);
  const bf16* h = reinterpret_cast<const bf16*>(&hi);
#pragma unroll
  for (int e = 0; e < 4; ++e) { r[e] = l[e]; r[4 + e] = h[e]; }
  return r;
}

// ---------------------------------------------------------------- LDS-staged bf16 epilogue
// `tile` holds `rows` x BN f32 accumulators (row stride BN + 4) for output pixels m0.. and GEMM
// columns n0..; NTH threads each own one 8-column group (cg = tid % (BN/8)) and walk the rows.
// Applies bias, ReLU, dropout, the pixel-shuffle / split / addend / mask / accumulate store modes
// and collects per-channel partial sums into bs/bq: BatchNorm statistics (sum, sum of squares) of the
// stored values, or with bnr_z the BatchNorm-backward sums (db, db*xhat) of the stored gradient.
// F8: fp8 launch — acc * wscale[n] before the bias, fp8 or bf16 store (compiled only into the fp8
// kernels, so the bf16 kernels keep their register budget)
template <int NTH, int BN, bool F8 = false, typename TO = bf16>
ADP_DEV void epi_rows(const FwdArgs& a, const float* tile, int rows, int m0, int n0, int tid,
                      float (&bs)[8], float (&bq)[8]) {
  constexpr int LT = BN + 4;
  constexpr int GPR = BN / 8;
  static_assert(NTH % GPR == 0, "epilogue: threads must tile the row groups");
  constexpr int RSTEP = NTH / GPR;
  const int cg = tid % GPR;
  const int n = n0 + cg * 8;
  if (n >= a.Nout) return;
  const int HWo = a.Ho * a.Wo;
  float bias[8], wsc[F8 ? 8 : 1];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias[j] = a.bias ? a.bias[a.out_mode == 1 ? (n + j) % a.Cps : n + j] : 0.f;
  if constexpr (F8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) wsc[j] = a.wscale[n + j];
  }
  for (int row = tid / GPR; row < rows; row += RSTEP) {
    const int m = m0 + row;
    if (m >= a.M) break;
    float v[8];
    const float4* tp = reinterpret_cast<const float4*>(tile + row * LT + cg * 8);
    float4 t0 = tp[0], t1 = tp[1];
    v[0] = t0.x; v[1] = t0.y; v[2] = t0.z; v[3] = t0.w; v[4] = t1.x; v[5] = t1.y; v[6] = t1.z; v[7] = t1.w;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (F8) v[j] = fmaf(v[j], wsc[j], bias[j]);
      else v[j] += bias[j];
      if (a.relu) v[j] = fmaxf(v[j], 0.f);
    }
    if (a.drop_rate > 0.f) {
      const float ks = 1.f / (1.f - a.drop_rate);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float u = adp_uniform(a.drop_seed, (uint64_t)m * (uint64_t)a.Nout + n + j);
        v[j] = (u >= a.drop_rate) ? v[j] * ks : 0.f;
      }
    }
    Grp<TO> gr;
    if (a.out_mode == 1) {
      int sub = n / a.Cps, c = n - sub * a.Cps;
      int nimg = m / HWo, rem = m - nimg * HWo, yo = rem / a.Wo, xo = rem - yo * a.Wo;
      size_t pix = ((size_t)nimg * (2 * a.Ho) + 2 * yo + (sub >> 1)) * (2 * a.Wo) + 2 * xo + (sub & 1);
      if constexpr (F8) {
        if (a.out_f8) {
          *reinterpret_cast<uint2*>(reinterpret_cast<unsigned char*>(a.out) + pix * a.out_stride + c) = f8x8_from_f(v);
          continue;
        }
      }
      grp_from_f(gr, v);
      grp_store(gr, reinterpret_cast<TO*>(a.out) + pix * a.out_stride + c);
    } else if (a.out_mode == 2 && n >= a.split_c) {
      const int c = n - a.split_c;
      if (a.mask2) {
        float mk[8];
        grp_load(gr, reinterpret_cast<const TO*>(a.mask2) + (size_t)m * a.mask2_stride + c);
        grp_to_f(gr, mk);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = mk[j] > 0.f ? v[j] * a.mask2_scale : 0.f;
      }
      grp_from_f(gr, v);
      grp_store(gr, reinterpret_cast<TO*>(a.out2) + (size_t)m * a.out2_stride + c);
      if (a.bn_sum) {   // channel sums of the out2 part too (e.g. a ConvTranspose bias gradient)
#pragma unroll
        for (int j = 0; j < 8; ++j) { bs[j] += v[j]; bq[j] += v[j] * v[j]; }
      }
      continue;
    } else {
      if (!a.out) continue;
      if constexpr (F8) {   // fp8 launches: plain store (the host rejects addend / mask / accum / BN sums)
        if (a.out_f8) {
          *reinterpret_cast<uint2*>(reinterpret_cast<unsigned char*>(a.out) + (size_t)m * a.out_stride + n) =
              f8x8_from_f(v);
          continue;
        }
      }
      float f[8];
      if (a.addend) {
        grp_load(gr, reinterpret_cast<const TO*>(a.addend) + (size_t)m * a.addend_stride + n);
        grp_to_f(gr, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += f[j];
      }
      if (a.mask) {
        grp_load(gr, reinterpret_cast<const TO*>(a.mask) + (size_t)m * a.mask_stride + n);
        grp_to_f(gr, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f[j] > 0.f ? v[j] * a.mask_scale : 0.f;
      }
      grp_from_f(gr, v);
      grp_store(gr, reinterpret_cast<TO*>(a.out) + (size_t)m * a.out_stride + n);
      if (a.accum) {
        float* ap = a.accum + (size_t)m * a.accum_stride + n;
        float r[8];
        grp_to_f(gr, r);   // accumulate the value as stored (bf16-rounded), like the generic path
#pragma unroll
        for (int j = 0; j < 8; ++j) ap[j] += r[j];
      }
    }
    if (a.bn_sum) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { bs[j] += v[j]; bq[j] += v[j] * v[j]; }
    }
  }
}

// Epilogue of a data-gradient launch with the fused BatchNorm-backward reduction (bnr_*): plain store
// of the gradient dA (+addend, *mask), then the sums db = dA*(z*scale+shift > 0) and db*xhat over the
// stored (bf16-rounded) dA, exactly what adp_bn_bwd_reduce would read. Kept separate from epi_rows so
// that the per-channel parameters cost registers only in the kernels that use them (they are read
// per row from L1 rather than held across the row loop).
template <int NTH, int BN, typename TO = bf16>
ADP_DEV void epi_rows_bnr(const FwdArgs& a, const float* tile, int rows, int m0, int n0, int tid,
                          float (&bs)[8], float (&bq)[8]) {
  constexpr int LT = BN + 4;
  constexpr int GPR = BN / 8;
  constexpr int RSTEP = NTH / GPR;
  const int cg = tid % GPR;
  const int n = n0 + cg * 8;
  if (n >= a.Nout) return;
  for (int row = tid / GPR; row < rows; row += RSTEP) {
    const int m = m0 + row;
    if (m >= a.M) break;
    float v[8], f[8];
    const float4* tp = reinterpret_cast<const float4*>(tile + row * LT + cg * 8);
    float4 t0 = tp[0], t1 = tp[1];
    v[0] = t0.x; v[1] = t0.y; v[2] = t0.z; v[3] = t0.w; v[4] = t1.x; v[5] = t1.y; v[6] = t1.z; v[7] = t1.w;
    Grp<TO> gr;
    if (a.addend) {
      grp_load(gr, reinterpret_cast<const TO*>(a.addend) + (size_t)m * a.addend_stride + n);
      grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += f[j];
    }
    if (a.mask) {
      grp_load(gr, reinterpret_cast<const TO*>(a.mask) + (size_t)m * a.mask_stride + n);
      grp_to_f(gr, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = f[j] > 0.f ? v[j] * a.mask_scale : 0.f;
    }
    grp_from_f(gr, v);
    grp_store(gr, reinterpret_cast<TO*>(a.out) + (size_t)m * a.out_stride + n);
    grp_to_f(gr, v);   // the stored (rounded) gradient
    if (ADP_DBG(a) & 8192) grp_zero(gr);   // (timing-only ablation, fwd_debug bit 13: no z loads)
    else grp_load(gr, reinterpret_cast<const TO*>(a.bnr_z) + (size_t)m * a.bnr_zs + n);
    grp_to_f(gr, f);
    if (ADP_DBG(a) & 16384) continue;   // (fwd_debug bit 14: no sums)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 sc = *reinterpret_cast<const float4*>(a.bnr_sc + n + 4 * h);
      const float4 sh = *reinterpret_cast<const float4*>(a.bnr_sh + n + 4 * h);
      const float4 mu = *reinterpret_cast<const float4*>(a.bnr_mean + n + 4 * h);
      const float4 is = *reinterpret_cast<const float4*>(a.bnr_invstd + n + 4 * h);
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

// Threads with equal column group hold partial BN sums of the same 8 channels: reduce them through
// LDS (`red` needs NTH*16 floats; caller guarantees no pending reads of it), then one atomic per
// channel and block.
template <int NTH, int BN>
ADP_DEV void epi_bn_flush(const FwdArgs& a, float* red, int n0, int tid, const float (&bs)[8],
                          const float (&bq)[8]) {
  constexpr int GPR = BN / 8;
  if (ADP_DBG(a) & 2) return;
  ADP_LDS_BARRIER();
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[tid * 16 + j] = bs[j]; red[tid * 16 + 8 + j] = bq[j]; }
  ADP_LDS_BARRIER();
  if (tid < BN) {
    const int gg = tid >> 3, j = tid & 7;
    float s = 0.f, q = 0.f;
    for (int t = gg; t < NTH; t += GPR) { s += red[t * 16 + j]; q += red[t * 16 + 8 + j]; }
    const int nn = n0 + tid;
    if (nn < a.Nout) {
      const int c = a.out_mode == 1 ? nn % a.Cps : nn;
      // replica of this block (folded into bn_sum/bn_sq or bnr_dbeta/bnr_dgamma by the launcher)
      const unsigned blk = blockIdx.x + blockIdx.y * gridDim.x;
      double* rep = a.stat + (size_t)(blk & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
      atomicAdd(rep + c, (double)s);
      atomicAdd(rep + adp::STAT_CMAX + c, (double)q);
    }
  }
}

}  // namespace

namespace adp {
// conv_fwd_tap64.hip: 8-phase LDS-DMA forward kernel for layers whose channel stride is a multiple
// of 64 (every 64-deep K step lies inside one tap). Returns 1 if it launched, 0 if not eligible.
int launch_fwd_tap64(FwdArgs& a, hipStream_t s);
// conv_fwd_tap64p.hip: persistent 256x256 form of the same kernel with the tile boundary pipelined
// (next tile's first stage in flight during a register epilogue); called by launch_fwd_tap64.
int launch_fwd_tap64p(FwdArgs& a, hipStream_t s, int tile);   // tile: tap64 config 0 (256x256) / 1 (256x128)
// conv_fwd_halo.hip: halo-reuse 3x3 kernel for narrow (<= 128 output channels) stride-1 layers.
int launch_fwd_halo(FwdArgs& a, hipStream_t s);
// conv_fwd_w4.hip: four-wave persistent halo forward (weights straight to registers) for 3x3 'same'
// layers with Nout % 256 == 0; called by launch_fwd_tap64p for its 256x256 halo shapes.
int launch_fwd_w4(FwdArgs& a, hipStream_t s);
int launch_fwd_cin8(FwdArgs& a, hipStream_t s);   // conv_fwd_cin8.hip: input layers (one 8-channel source)
int launch_fwd_cin8_f32(FwdArgs& a, hipStream_t s);   // conv_fwd_cin8.hip: f32 3x3 input layers
// conv_fwd_halo_f8.hip: fp8 forward of 3x3 layers with 64-channel sources (one, or two concatenated)
int launch_fwd_halop_f8(FwdArgs& a, hipStream_t s);
// conv_wgrad_tap64.hip: phase-pipelined LDS-DMA weight-gradient kernel for the same layers.
int launch_wgrad_tap64(WgradArgs& a, hipStream_t s);
// dst[i] += sum_g part[g][i] over G slabs of n4 float4 each, in an order fixed by G alone (deterministic); recorded
// instead of launched while the stream defers (adp_wgrad_defer), launched batched by adp_wgrad_flush
void slab_reduce(int G, size_t n4, const float* part, float* dst, hipStream_t s);
// the slabs of one such reduction: library scratch `slot`, or (deferring stream) the stream's arena
float* reduce_part(int slot, size_t bytes, hipStream_t s);
// conv_wgrad_f32.hip: f32 weight gradient on LDS-DMA staging (32-pixel stages, exact f32 MFMA)
int launch_wgrad_f32(WgradArgs& a, hipStream_t s);
// the persistent halo weight-gradient kernel takes this launch with the BatchNorm-backward apply fused
bool wgrad_bna_fusable(const WgradArgs& a);
}
