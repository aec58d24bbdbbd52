// fp8 e4m3 forward of the 64-channel 3x3 layers (unet_bn level 0 and the level-1 layer fed by pool0: BASELINE
// configs[4], UNetBN.forward_fp8). The bf16 network runs these layers on igemm_fwd_halop_kernel (conv_fwd_halo.hip):
// one 512-thread block per CU, all nine weight taps resident in LDS, the 10 x 34 input halo of an 8 x 32 output
// patch read by every tap. Here the same structure with fp8 operands and v_mfma_scale_f32_16x16x128_f8f6f4:
//   * a K step is 128 fp8 values. One 64-channel source (Cin_s = 64): a step is the tap PAIR (2p, 2p + 1) -- lane
//     group h4 supplies channels 16 h4 .. + 15 of tap 2p (first 16 B of its operand) and of tap 2p + 1 (second
//     16 B); five steps, the fifth pairing tap 8 with zero weights. Two 64-channel sources (Cin_s = 128, the
//     decoder's concat): a step is one tap, first 16 B from source A, second from source B. The weight rows of a
//     step are the packed [N][K] row's bytes [128 p, 128 p + 128) in both cases (K = tap * Cin_s + channel), so A
//     and B share the K permutation and the layer's packed fp8 weights (pack_weights_fp8) are used as they are.
//   * the halo is one 64-B LDS row per pixel and source (chunk c of row r at c ^ ((r >> 1) & 3): conflict-free for
//     the 16 consecutive rows a ds_read_b128 lane group reads from any base row), 21.25 KiB per source; weights
//     5 or 9 steps x 64 rows x 128 B = 40 / 72 KiB, loaded once per block.
//   * epilogue: acc * wscale[n] + bias[n] (the eval BatchNorm folded in by UNetBN: dequantisation x BN scale, BN
//     shift), ReLU, and an fp8 or bf16 store. fp8: the four channel quads of a lane (one dword each) are transposed
//     across the four lane rows by v_permlane16_swap + v_permlane32_swap, after which lane row h4 holds channels
//     16 h4 .. + 15 of its pixel: one 16-B store per lane, 1 KiB of consecutive pixels per instruction. bf16: the
//     channel-quad pairs of halop's wide epilogue (16-B stores, both halves of a pixel's 128-B line back to back).
// Static tile lists (eval forward: no all-reduce holds CUs); the next tile's halo is prefetched into registers.
#include "conv_common.h"

namespace {

constexpr int Q_PH = 8, Q_PW = 32, Q_HW = 34, Q_HROWS = 340;
constexpr int Q_HROWB = 64;                          // 64 fp8 channels per halo LDS row
constexpr int Q_HPIECE = Q_HROWS * 4;                // 16-B pieces per source image (1360)
constexpr int Q_HPAD = 1408;                         // per-image piece range padded to whole waves (22 x 64)
constexpr int Q_HSTR = Q_HPAD * 16;                  // LDS bytes per source image (incl. the pad pieces)
__device__ __attribute__((aligned(256))) uint4 q_zero_page[64];
__device__ __forceinline__ int q_hswz(int r) { return (r >> 1) & 3; }

#define Q_LDS_BAR()                                           \
  do {                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        \
    __builtin_amdgcn_s_barrier();                             \
    asm volatile("" ::: "memory");                            \
  } while (0)

template <int NCH>
constexpr int halop_f8_lds() {
  return (NCH == 1 ? 5 : 9) * 64 * 128 + NCH * Q_HSTR + 2 * 64 * 4;
}

template <int NCH, bool PIPE>
__global__ __launch_bounds__(512, 1) void igemm_fwd_halop_f8_kernel(FwdArgs a) {
  constexpr int NTH = 512, BN = 64, NF = 4;
  constexpr int NSTEP = NCH == 1 ? 5 : 9;
  constexpr int WROW = 128;
  constexpr int WBYTES = NSTEP * BN * WROW;
  constexpr int GW = WBYTES / 16 / NTH;                           // resident weight pieces per thread
  constexpr int GH = (NCH * Q_HPAD + NTH - 1) / NTH;              // halo pieces per thread per tile
  constexpr int OFF_H = WBYTES, OFF_C = OFF_H + NCH * Q_HSTR;
  static_assert(GW * NTH * 16 == WBYTES, "weights split evenly");
  static_assert(halop_f8_lds<NCH>() <= 160 * 1024, "LDS");
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  typedef int v8i32 __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(1024))) unsigned char smem[halop_f8_lds<NCH>()];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // = patch row
  const int tx_n = a.Wo / Q_PW, ty_n = a.Ho / Q_PH;
  const int T = a.nblocks, G = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, G);
  const int NT = a.ntile_n;                                    // 64-wide output blocks
  const int nt = lin < T ? (T - lin + G - 1) / G : 0;
  if (nt == 0) return;
  const int nh = lin % NT, n0 = 64 * nh;
  const int Wrows = (a.Nout + 63) / 64 * 64;
  auto tile_id = [&](int k) -> int { return k < nt ? lin / NT + k * (G / NT) : -1; };   // patch index
  auto origin = [&](int t, int& img, int& y0, int& x0) {
    const int px = t % tx_n, r = t / tx_n;
    y0 = (r % ty_n) * Q_PH;
    img = r / ty_n;
    x0 = px * Q_PW;
  };
  // halo piece i of this thread for the patch at (img, y0, x0): source image s, pixel hr, chunk position hp;
  // nullptr = zero (outside the image) or nothing to load (pad pieces / past the last image)
  const unsigned char* srcA = reinterpret_cast<const unsigned char*>(a.srcA);
  const unsigned char* srcB = reinterpret_cast<const unsigned char*>(a.srcB);
  auto piece_src = [&](int img, int y0, int x0, int i, bool& want) -> const uint4* {
    const int idx = i * NTH + tid;
    const int s = idx >= Q_HPAD ? 1 : 0, pin = idx - s * Q_HPAD;
    want = s < NCH && pin < Q_HPIECE;
    if (!want) return nullptr;
    const int hr = pin >> 2, hp = pin & 3;
    const int gy = y0 - 1 + hr / Q_HW, gx = x0 - 1 + hr % Q_HW;
    if ((unsigned)gy >= (unsigned)a.Hs || (unsigned)gx >= (unsigned)a.Ws) return nullptr;
    const unsigned char* base = s ? srcB : srcA;
    const int cs = s ? a.CBs : a.CAs;
    return reinterpret_cast<const uint4*>(base + (size_t)((img * a.Hs + gy) * a.Ws + gx) * cs + 16 * (hp ^ q_hswz(hr)));
  };
  // LDS slot of piece i (wave-uniform base for LDS-DMA: the pad range keeps a wave inside one source image)
  auto piece_lds = [&](int i) -> int {
    const int idx = i * NTH + tid, s = idx >= Q_HPAD ? 1 : 0;
    return OFF_H + s * Q_HSTR + (idx - s * Q_HPAD) * 16;
  };

  // ---- prologue: resident weights (step p row q: packed row n0 + q, K bytes [128 p, 128 p + 128), chunk position
  // pos holding source chunk pos ^ swz(q); K bytes past the layer's K read zero), constants, the first halo
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(a.W);
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int idx = i * NTH + tid;
    const int p = idx / (BN * 8), rem = idx - p * (BN * 8), q = rem >> 3, pos = rem & 7;
    const int kb = p * WROW + 16 * (pos ^ swz(q));
    const void* src = n0 + q < Wrows && kb < a.K ? (const void*)(Wb + (size_t)(n0 + q) * a.Kpad + kb) : (const void*)q_zero_page;
    __builtin_amdgcn_global_load_lds(src, (lds_void*)(smem + (size_t)(i * NTH + wave * 64) * 16), 16, 0, 0);
  }
  {
    int img0, y00, x00;
    origin(tile_id(0), img0, y00, x00);
#pragma unroll
    for (int i = 0; i < GH; ++i) {
      bool want;
      const uint4* p = piece_src(img0, y00, x00, i, want);
      if (__builtin_amdgcn_readfirstlane(i * NTH + wave * 64) < NCH * Q_HPAD)   // (wave-uniform: a whole pad wave skips)
        __builtin_amdgcn_global_load_lds(p ? (const void*)p : (const void*)q_zero_page,
                                         (lds_void*)(smem + __builtin_amdgcn_readfirstlane(piece_lds(i) - lane * 16)),
                                         16, 0, 0);
    }
  }
  float* cst = reinterpret_cast<float*>(smem + OFF_C);   // [2][64]: bias | wscale
  if (tid < BN) {
    const int c = n0 + tid;
    const bool v = c < a.Nout;
    cst[tid] = (a.bias && v) ? a.bias[c] : 0.f;
    cst[BN + tid] = v ? a.wscale[c] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int r16 = lane & 15, h4 = lane >> 4;
  const bool o8 = a.out_f8 != 0;
  unsigned char* obase = reinterpret_cast<unsigned char*>(a.out);
  const int oes = o8 ? 1 : 2;
  const __amdgpu_buffer_rsrc_t rsO =
      __builtin_amdgcn_make_buffer_rsrc((void*)obase, 0, a.M * a.out_stride * oes, 0x00020000);

  f32x4 acc[2][NF];
  for (int k = 0;; ++k) {
    const int t = tile_id(k);
    if (t < 0) break;
    const int tn = tile_id(k + 1);
    const bool more = tn >= 0;
    int img, y0, x0;
    origin(t, img, y0, x0);
    const int mrow = (img * a.Ho + y0 + wave) * a.Wo + x0;   // first output pixel of this wave's patch row
    // the next tile's halo into registers (stored after this tile's taps)
    uint4 hreg[GH];
    if (more) {
      int img1, y01, x01;
      origin(tn, img1, y01, x01);
#pragma unroll
      for (int i = 0; i < GH; ++i) {
        bool want;
        const uint4* p = piece_src(img1, y01, x01, i, want);
        hreg[i] = p ? *p : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K loop, software-pipelined by one step: the fragments of step p + 1 are read from LDS while step p multiplies
    // (two named fragment sets, steps taken in pairs; a fully unrolled loop hoisted every step's reads and spilled)
    struct Frag { bf16x8 fb[NF][2], fa[2][2]; };
    auto load_frag = [&](int p, Frag& F) {
      const unsigned char* Wp = smem + p * BN * WROW;
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int q = nf * 16 + r16, c = 4 * s + h4;
          F.fb[nf][s] = *reinterpret_cast<const bf16x8*>(Wp + q * WROW + ((c ^ swz(q)) << 4));
        }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // one source: tap 2p + s (tap 9 = the zero-weight padding: any valid row, tap 8's); two sources: tap p,
        // source s
        const int tap = NCH == 1 ? (2 * p + s < 9 ? 2 * p + s : 8) : p;
        const int dy = tap / 3, dx = tap - 3 * (tap / 3);
        const unsigned char* Hs_ = smem + OFF_H + (NCH == 1 ? 0 : s) * Q_HSTR;
#pragma unroll
        for (int mf = 0; mf < 2; ++mf) {
          const int hr = (wave + dy) * Q_HW + mf * 16 + r16 + dx;
          F.fa[mf][s] = *reinterpret_cast<const bf16x8*>(Hs_ + hr * Q_HROWB + ((h4 ^ q_hswz(hr)) << 4));
        }
      }
    };
    auto mma = [&](const Frag& F) {
#pragma unroll
      for (int mf = 0; mf < 2; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)   // transposed: rows = output channels, columns = pixels
          acc[mf][nf] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              __builtin_bit_cast(v8i32, F.fb[nf]), __builtin_bit_cast(v8i32, F.fa[mf]), acc[mf][nf], 0, 0, 0, 127, 0, 127);
    };
    Frag FA, FB;
    if constexpr (PIPE) {   // (option halop_f8_pipe, default 1)
      load_frag(0, FA);
#pragma unroll 1
      for (int p = 0; p < NSTEP; p += 2) {
        if (p + 1 < NSTEP) load_frag(p + 1, FB);
        mma(FA);
        if (p + 1 < NSTEP) {
          if (p + 2 < NSTEP) load_frag(p + 2, FA);
          mma(FB);
        }
      }
    } else {   // one step at a time: each step's reads, then its MFMAs
#pragma unroll 1
      for (int p = 0; p < NSTEP; ++p) {
        load_frag(p, FA);
        mma(FA);
      }
    }
    // ---- epilogue: lane (r16, h4) holds channels 16 nf + 4 h4 .. + 3 of pixel mrow + 16 mf + r16
#pragma unroll
    for (int mf = 0; mf < 2; ++mf) {
      const int m = mrow + mf * 16 + r16;
      float x[NF][4];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
        const float4 b4 = *reinterpret_cast<const float4*>(cst + nf * 16 + 4 * h4);
        const float4 w4 = *reinterpret_cast<const float4*>(cst + BN + nf * 16 + 4 * h4);
        const float bb[4] = {b4.x, b4.y, b4.z, b4.w}, ww[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[nf][r] = fmaf(acc[mf][nf][r], ww[r], bb[r]);
          if (a.relu) x[nf][r] = fmaxf(x[nf][r], 0.f);
        }
      }
      if (o8) {
        unsigned d[NF];
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          float c8[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) c8[r] = fminf(fmaxf(x[nf][r], -FP8_MAX), FP8_MAX);
          int qv = __builtin_amdgcn_cvt_pk_fp8_f32(c8[0], c8[1], 0, false);
          qv = __builtin_amdgcn_cvt_pk_fp8_f32(c8[2], c8[3], qv, true);
          d[nf] = (unsigned)qv;
        }
        // 4 x 4 transpose over the lane rows: afterwards lane row h4 holds groups (row 0..3) of quad h4
        const auto p01 = __builtin_amdgcn_permlane16_swap(d[0], d[1], false, false);
        const auto p23 = __builtin_amdgcn_permlane16_swap(d[2], d[3], false, false);
        const auto q02 = __builtin_amdgcn_permlane32_swap(p01[0], p23[0], false, false);
        const auto q13 = __builtin_amdgcn_permlane32_swap(p01[1], p23[1], false, false);
        const v4u st = {q02[0], q13[0], q02[1], q13[1]};
        const unsigned off = n0 + 16 * h4 < a.Nout ? (unsigned)(m * a.out_stride + n0 + 16 * h4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(st, rsO, off, 0, 0);
      } else {
#pragma unroll
        for (int np = 0; np < NF; np += 2) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          typedef unsigned v2u __attribute__((ext_vector_type(2)));
          bf16x4 o0, o1;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            o0[r] = (bf16)x[np][r];
            o1[r] = (bf16)x[np + 1][r];
          }
          const v2u u0 = __builtin_bit_cast(v2u, o0), u1 = __builtin_bit_cast(v2u, o1);
          const auto e0 = __builtin_amdgcn_permlane16_swap(u0.x, u1.x, false, false);
          const auto e1 = __builtin_amdgcn_permlane16_swap(u0.y, u1.y, false, false);
          const v4u st = {e0[0], e1[0], e0[1], e1[1]};
          const int cw = 16 * (np + (h4 & 1)) + 8 * (h4 >> 1);
          const unsigned off = n0 + cw < a.Nout ? (unsigned)((m * a.out_stride + n0 + cw) * 2) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b128(st, rsO, off, 0, 0);
        }
      }
    }
    if (more) {
      Q_LDS_BAR();   // every wave is done with this tile's halo
#pragma unroll
      for (int i = 0; i < GH; ++i) {
        const int idx = i * NTH + tid, s = idx >= Q_HPAD ? 1 : 0;
        if (s < NCH && idx - s * Q_HPAD < Q_HPIECE) *reinterpret_cast<uint4*>(smem + piece_lds(i)) = hreg[i];
      }
      Q_LDS_BAR();
    }
  }
}

#undef Q_LDS_BAR

}  // namespace

namespace adp {
// fp8 forward of a 3x3 stride-1 'same' layer whose sources are 64 fp8 channels (one source, or two concatenated):
// Nout a multiple of 64, plain store (bias, ReLU, fp8 or bf16 output). 0 = not eligible.
int launch_fwd_halop_f8(FwdArgs& a, hipStream_t s) {
  if (!option("halop_f8", 1)) return 0;
  const int Cin_s = a.CAs + a.CBs;
  if (a.CAs != 64 || (a.CBs != 0 && a.CBs != 64) || a.kh != 3 || a.kw != 3 || a.dil != 1 || a.pad != 1 ||
      a.stride != 1 || a.up != 1 || a.Ho != a.Hs || a.Wo != a.Ws || a.Ho % Q_PH != 0 || a.Wo % Q_PW != 0 ||
      a.K != 9 * Cin_s || a.Kpad < a.K || a.Nout % 64 != 0 || a.out_mode != 0 || !a.out || a.bn_sum || a.bnr_z ||
      a.addend || a.mask || a.accum || a.drop_rate > 0.f || a.scA || a.scB)
    return 0;
  if (a.out_stride % (a.out_f8 ? 16 : 8) != 0) return 0;
  const size_t lim = (size_t)1 << 31;
  if ((size_t)a.M * a.out_stride * (a.out_f8 ? 1 : 2) >= lim) return 0;
  a.ntile_n = a.Nout / 64;
  const bool pipe = option("halop_f8_pipe", 1);   // K loop software-pipelined by one step
  const int tiles = a.Nimg * (a.Ho / Q_PH) * (a.Wo / Q_PW) * a.ntile_n;
  a.nblocks = tiles;
  int grid = std::max(1, std::min(tiles, option("halo_persist_grid", 256)));
  grid -= grid % a.ntile_n;
  if (grid == 0) grid = a.ntile_n;
  adp::set_kernel("igemm_fwd_halop_f8_kernel<%d, %s>", a.CBs == 0 ? 1 : 2, pipe ? "true" : "false");
  if (a.CBs == 0) {
    if (pipe) hipLaunchKernelGGL((igemm_fwd_halop_f8_kernel<1, true>), dim3(grid), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((igemm_fwd_halop_f8_kernel<1, false>), dim3(grid), dim3(512), 0, s, a);
  } else {
    if (pipe) hipLaunchKernelGGL((igemm_fwd_halop_f8_kernel<2, true>), dim3(grid), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((igemm_fwd_halop_f8_kernel<2, false>), dim3(grid), dim3(512), 0, s, a);
  }
  return 1;
}
}  // namespace adp
