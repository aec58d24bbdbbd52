// Input-layer forward convolution ("cin8"): one 8-channel source group (the network input, channel
// stride 8: 3 RGB or 1 gray channel + zero pad), K = taps * 8 <= 96, N <= 64 output channels.
// unet_bn enc0_conv1 (3 -> 64) and adipose_v3 down1_conv1 (1 -> 44, train_adipose_unet_v3.py:668).
//
// The layer is HBM-bound on its 64-channel output (AI ~ 9 FLOP/B), so it needs no LDS staging: the
// whole weight matrix lives in registers as MFMA A fragments (W[co][k], 16 output channels x 32 k per
// fragment) and each lane loads its B fragment — the 8 channels of one tap of one output pixel, one
// 16-B load — straight from global memory (the 3x3 neighbourhood re-reads hit L1/L2). The product is
// C^T = W X^T: lane l holds 4 consecutive output channels 4(l>>4)+i (+16 mb) of pixel l & 15, stored
// as one 8-B vector per 16-channel block. BatchNorm statistics of the stored values are kept per lane
// and reduced once per wave (shuffles over the 16 lanes of a channel quad, one atomic per channel into
// the wave's replica of the BatchNorm accumulators, adp::stat_scratch).
#include "conv_common.h"

namespace {
typedef unsigned C8v2u32 __attribute__((ext_vector_type(2)));

template <int KS, int UNR>
__global__ __launch_bounds__(256) void igemm_fwd_cin8_kernel(FwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, h4 = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  const bf16* W = reinterpret_cast<const bf16*>(a.W);
  const bf16* src = reinterpret_cast<const bf16*>(a.srcA);
  bf16* out = reinterpret_cast<bf16*>(a.out);

  bf16x8 wf[4][KS];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[mb][ks] = *reinterpret_cast<const bf16x8*>(W + (size_t)(16 * mb + r16) * a.Kpad + 32 * ks + 8 * h4);
  const int ntaps = a.kh * a.kw;
  int toy[KS], tox[KS];
  bool tval[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int t = 4 * ks + h4;
    tval[ks] = t < ntaps;
    const int ty = t / a.kw, tx = t - ty * a.kw;
    toy[ks] = ty * a.dil - a.pad;
    tox[ks] = tx * a.dil - a.pad;
  }
  float bias[4][4], s1[4][4], s2[4][4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 16 * mb + 4 * h4 + i;
      bias[mb][i] = (a.bias && co < a.Nout) ? a.bias[co] : 0.f;
      s1[mb][i] = 0.f;
      s2[mb][i] = 0.f;
    }
  const int HWo = a.Ho * a.Wo;
  const int groups = (a.M + 15) / 16;
  const bf16x8 zero = {};
  for (int g0 = wave * UNR; g0 < groups; g0 += nwaves * UNR) {
    bf16x8 xb[UNR][KS];
    int mm[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int m = (g0 + u) * 16 + r16;
      mm[u] = m;
      const bool mv = g0 + u < groups && m < a.M;
      const int mc = mv ? m : 0;
      const int n = mc / HWo, rem = mc - n * HWo, y = rem / a.Wo, x = rem - y * a.Wo;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int yi = y + toy[ks], xi = x + tox[ks];
        const bool ok = mv && tval[ks] && (unsigned)yi < (unsigned)a.Hs && (unsigned)xi < (unsigned)a.Ws;
        xb[u][ks] = ok ? *reinterpret_cast<const bf16x8*>(src + ((size_t)(n * a.Hs + yi) * a.Ws + xi) * 8) : zero;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      f32x4 acc[4];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mb][ks], xb[u][ks], acc[mb], 0, 0, 0);
      const int m = mm[u];
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      if (a.out_f8) {
        // fp8 e4m3 output (UNetBN.forward_fp8's level-0 operand; no statistics): each 16-channel block's quad is one
        // dword; a 4 x 4 transpose over the lane rows (v_permlane16_swap, then v_permlane32_swap) leaves lane row h4
        // with channels 16 h4 .. + 15 of its pixel, one 16-B store (Nout == 64, the launcher checks)
        const bool mv = g0 + u < groups && m < a.M;
        unsigned d[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          float c8[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = acc[mb][i] + bias[mb][i];
            if (a.relu) v = fmaxf(v, 0.f);
            c8[i] = fminf(fmaxf(v, -FP8_MAX), FP8_MAX);
          }
          int qv = __builtin_amdgcn_cvt_pk_fp8_f32(c8[0], c8[1], 0, false);
          qv = __builtin_amdgcn_cvt_pk_fp8_f32(c8[2], c8[3], qv, true);
          d[mb] = (unsigned)qv;
        }
        const auto p01 = __builtin_amdgcn_permlane16_swap(d[0], d[1], false, false);
        const auto p23 = __builtin_amdgcn_permlane16_swap(d[2], d[3], false, false);
        const auto q02 = __builtin_amdgcn_permlane32_swap(p01[0], p23[0], false, false);
        const auto q13 = __builtin_amdgcn_permlane32_swap(p01[1], p23[1], false, false);
        if (mv)
          *reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(a.out) + (size_t)m * a.out_stride + 16 * h4) =
              make_uint4(q02[0], q13[0], q02[1], q13[1]);
        continue;
      }
      if (a.wide_st) {
        // 16-B stores: the quads of 16-channel blocks mb and mb + 1 joined by v_permlane16_swap (lane row h4
        // then holds channels 16 (mb + (h4 & 1)) + 8 (h4 >> 1) .. + 7), before the lane-divergent tail test
        const bool mv = g0 + u < groups && m < a.M;
        C8v2u32 o2[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const bool qv = mv && 16 * mb + 4 * h4 < a.Nout;
          float v[4];
          bf16x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = acc[mb][i] + bias[mb][i];
            if (a.relu) v[i] = fmaxf(v[i], 0.f);
            if (qv) { s1[mb][i] += v[i]; s2[mb][i] += v[i] * v[i]; }
            o[i] = (bf16)v[i];
          }
          o2[mb] = __builtin_bit_cast(C8v2u32, o);
        }
#pragma unroll
        for (int p = 0; p < 4; p += 2) {
          const auto e0 = __builtin_amdgcn_permlane16_swap(o2[p].x, o2[p + 1].x, false, false);
          const auto e1 = __builtin_amdgcn_permlane16_swap(o2[p].y, o2[p + 1].y, false, false);
          const int cw = 16 * (p + (h4 & 1)) + 8 * (h4 >> 1);
          if (mv && cw < a.Nout)
            *reinterpret_cast<uint4*>(out + (size_t)m * a.out_stride + cw) = make_uint4(e0[0], e1[0], e0[1], e1[1]);
        }
        continue;
      }
      if (g0 + u >= groups || m >= a.M) continue;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int co0 = 16 * mb + 4 * h4;
        if (co0 >= a.Nout) continue;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = acc[mb][i] + bias[mb][i];
          if (a.relu) v[i] = fmaxf(v[i], 0.f);
          s1[mb][i] += v[i];
          s2[mb][i] += v[i] * v[i];
        }
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)v[i];
        *reinterpret_cast<bf16x4*>(out + (size_t)m * a.out_stride + co0) = o;
      }
    }
  }
  if (!a.bn_sum || (ADP_DBG(a) & 2)) return;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = row16_sum(s1[mb][i]), y = row16_sum(s2[mb][i]);
      const int co = 16 * mb + 4 * h4 + i;
      if (r16 == 0 && co < a.Nout) {   // this wave's replica; the launcher folds them into bn_sum / bn_sq
        double* rep = a.stat + (size_t)(wave & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
        atomicAdd(rep + co, (double)x);
        atomicAdd(rep + adp::STAT_CMAX + co, (double)y);
      }
    }
}

// Pipelined form (opt-in: option cin8_pf = 1, with source and output < 2 GiB): the same product and
// store layout, with every access a buffer load / store whose out-of-range offset stands for "padding"
// or "past the end" (reads 0, writes dropped) and the ReLU / validity tests as selects, so the loop has
// no branch. Passes alternate between two register sets: the gathers of pass k + 1 are issued before
// pass k's MFMAs and stores, and the wait before pass k's MFMAs counts exactly the later pass's loads
// and this pass's stores (vmcnt retires in order), so gather latency hides behind the previous pass.
// Measured at unet_bn's 1024^2 x 4 input layer: 0.245 ms against 0.242 for the plain form (gather latency
// is not what bounds it), so it stays opt-in, with a bit-exactness test.
template <int KS, int UNR>
__global__ __launch_bounds__(256) void igemm_fwd_cin8p_kernel(FwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, h4 = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  const bf16* W = reinterpret_cast<const bf16*>(a.W);
  const int HWo = a.Ho * a.Wo;
  const int nimg = (a.M + HWo - 1) / HWo;
  const __amdgpu_buffer_rsrc_t rsX =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.srcA, 0, nimg * a.Hs * a.Ws * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsO =
      __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.M * a.out_stride * 2, 0x00020000);
  constexpr unsigned OOB = 0x80000000u;

  bf16x8 wf[4][KS];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[mb][ks] = *reinterpret_cast<const bf16x8*>(W + (size_t)(16 * mb + r16) * a.Kpad + 32 * ks + 8 * h4);
  const int ntaps = a.kh * a.kw;
  int toy[KS], tox[KS];
  bool tval[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int t = 4 * ks + h4;
    tval[ks] = t < ntaps;
    const int ty = t / a.kw, tx = t - ty * a.kw;
    toy[ks] = ty * a.dil - a.pad;
    tox[ks] = tx * a.dil - a.pad;
  }
  const float lo = a.relu ? 0.f : -INFINITY;
  float bias[4][4], s1[4][4], s2[4][4];
  bool cval[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    cval[mb] = 16 * mb + 4 * h4 < a.Nout;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 16 * mb + 4 * h4 + i;
      bias[mb][i] = (a.bias && co < a.Nout) ? a.bias[co] : 0.f;
      s1[mb][i] = 0.f;
      s2[mb][i] = 0.f;
    }
  }
  const int groups = (a.M + 15) / 16;
  const int step = nwaves * UNR;

  auto gather = [&](int g, bf16x8 (&xv)[UNR][KS]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int m = (g + u) * 16 + r16;
      const bool mv = m < a.M;
      const int mc = mv ? m : 0;
      const int n = mc / HWo, rem = mc - n * HWo, y = rem / a.Wo, x = rem - y * a.Wo;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int yi = y + toy[ks], xi = x + tox[ks];
        const bool ok = mv && tval[ks] && (unsigned)yi < (unsigned)a.Hs && (unsigned)xi < (unsigned)a.Ws;
        const unsigned off = ok ? (unsigned)(((n * a.Hs + yi) * a.Ws + xi) * 16) : OOB;
        xv[u][ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsX, off, 0, 0));
      }
    }
  };
  auto pass = [&](int g, const bf16x8 (&xv)[UNR][KS]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      f32x4 acc[4];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mb][ks], xv[u][ks], acc[mb], 0, 0, 0);
      const int m = (g + u) * 16 + r16;
      const bool mv = m < a.M;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int co0 = 16 * mb + 4 * h4;
        const bool ok = mv && cval[mb];
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = fmaxf(acc[mb][i] + bias[mb][i], lo);
          const float vs = ok ? v[i] : 0.f;
          s1[mb][i] += vs;
          s2[mb][i] += vs * vs;
        }
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)v[i];
        const unsigned off = ok ? (unsigned)(((size_t)m * a.out_stride + co0) * 2) : OOB;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(C8v2u32, o), rsO, off, 0, 0);
      }
    }
  };
  bf16x8 xa[UNR][KS], xb[UNR][KS];
  int g0 = wave * UNR;
  if (g0 < groups) gather(g0, xa);
  for (; g0 < groups; g0 += 2 * step) {
    gather(g0 + step, xb);   // (a pass past the end gathers zeros from out-of-range offsets)
    pass(g0, xa);
    if (g0 + step >= groups) break;
    gather(g0 + 2 * step, xa);
    pass(g0 + step, xb);
  }
  if (!a.bn_sum || (ADP_DBG(a) & 2)) return;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = row16_sum(s1[mb][i]), y = row16_sum(s2[mb][i]);
      const int co = 16 * mb + 4 * h4 + i;
      if (r16 == 0 && co < a.Nout) {
        double* rep = a.stat + (size_t)(wave & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
        atomicAdd(rep + co, (double)x);
        atomicAdd(rep + adp::STAT_CMAX + co, (double)y);
      }
    }
}

template <int KS, int UNR>
void launch_cin8_u(FwdArgs& a, hipStream_t s) {
  const int groups = (a.M + 15) / 16;
  // (4 groups per pass on 2048 waves: 0.255 -> 0.239 ms at unet_bn's 1024^2 x 4 input layer,
  //  profiles/r02_cin8_ab.txt)
  const int waves = std::max(1, std::min((groups + UNR - 1) / UNR, adp::option("cin8_waves", 2048)));
  const size_t HWo = (size_t)a.Ho * a.Wo;
  const size_t src_bytes = ((size_t)a.M + HWo - 1) / HWo * a.Hs * a.Ws * 16, out_bytes = (size_t)a.M * a.out_stride * 2;
  if (adp::option("cin8_pf", 0) && !a.out_f8 && src_bytes < (1ull << 31) && out_bytes < (1ull << 31)) {
    adp::set_kernel("igemm_fwd_cin8p_kernel<%d, %d>", KS, UNR);
    hipLaunchKernelGGL((igemm_fwd_cin8p_kernel<KS, UNR>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
    return;
  }
  adp::set_kernel("igemm_fwd_cin8_kernel<%d, %d>", KS, UNR);
  hipLaunchKernelGGL((igemm_fwd_cin8_kernel<KS, UNR>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
}
template <int KS>
void launch_cin8(FwdArgs& a, hipStream_t s) {
  const int unr = adp::option("cin8_unr", 4);
  if (unr == 4) launch_cin8_u<KS, 4>(a, s);
  else if (unr == 1) launch_cin8_u<KS, 1>(a, s);
  else launch_cin8_u<KS, 2>(a, s);
}

// f32 form (round 5; the drop-in CLIs' default dtype, adipose_v3 down1_conv1 at the reference's precision): the same
// product on exact v_mfma_f32_16x16x4_f32 -- a 4-deep k step is one channel quad of one tap: lane l supplies
// W[16 mb + (l & 15)][8 t + 4 q + (l >> 4)] (registers for the whole launch) and X[pixel l & 15][tap t][channel
// 4 q + (l >> 4)] (one 4-B gather), so C^T = W X^T lands as in the bf16 form: lane l holds channels 16 mb + 4 (l >> 4)
// + i of pixel l & 15, one 16-B store per 16-channel block. Q = 1 when the caller's CA_real <= 4 (adp_conv_desc v19:
// the weight columns of channels 4-7 are zeros, e.g. the gray input): one quad per tap. 3x3 taps. The generic
// register-staged kernel it replaces ran this layer at ~1 TB/s (0.59 ms of the 1024^2 B=2 f32 step).
template <int Q, int UNR>
__global__ __launch_bounds__(256) void igemm_fwd_cin8_f32_kernel(FwdArgs a) {
  constexpr int T = 9;
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, h4 = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  const float* W = reinterpret_cast<const float*>(a.W);
  const float* src = reinterpret_cast<const float*>(a.srcA);
  float* out = reinterpret_cast<float*>(a.out);
  float wf[4][T][Q];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int q = 0; q < Q; ++q) wf[mb][t][q] = W[(size_t)(16 * mb + r16) * a.Kpad + 8 * t + 4 * q + h4];
  float bias[4][4], s1[4][4], s2[4][4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 16 * mb + 4 * h4 + i;
      bias[mb][i] = (a.bias && co < a.Nout) ? a.bias[co] : 0.f;
      s1[mb][i] = 0.f;
      s2[mb][i] = 0.f;
    }
  const int HWo = a.Ho * a.Wo;
  const int groups = (a.M + 15) / 16;
  for (int g0 = wave * UNR; g0 < groups; g0 += nwaves * UNR) {
    float xb[UNR][T][Q];
    int mm[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int m = (g0 + u) * 16 + r16;
      mm[u] = m;
      const bool mv = g0 + u < groups && m < a.M;
      const int mc = mv ? m : 0;
      const int n = mc / HWo, rem = mc - n * HWo, y = rem / a.Wo, x = rem - y * a.Wo;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int yi = y + (t / 3) * a.dil - a.pad, xi = x + (t % 3) * a.dil - a.pad;
        const bool ok = mv && (unsigned)yi < (unsigned)a.Hs && (unsigned)xi < (unsigned)a.Ws;
        const float* p = src + ((size_t)(n * a.Hs + yi) * a.Ws + xi) * 8 + h4;
#pragma unroll
        for (int q = 0; q < Q; ++q) xb[u][t][q] = ok ? p[4 * q] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      f32x4 acc[4];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
            acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[mb][t][q], xb[u][t][q], acc[mb], 0, 0, 0);
      const int m = mm[u];
      if (g0 + u >= groups || m >= a.M) continue;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int co0 = 16 * mb + 4 * h4;
        if (co0 >= a.Nout) continue;
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float x = acc[mb][i] + bias[mb][i];
          if (a.relu) x = fmaxf(x, 0.f);
          s1[mb][i] += x;
          s2[mb][i] += x * x;
          v[i] = x;
        }
        *reinterpret_cast<f32x4*>(out + (size_t)m * a.out_stride + co0) = v;
      }
    }
  }
  if (!a.bn_sum) return;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = row16_sum(s1[mb][i]), y = row16_sum(s2[mb][i]);
      const int co = 16 * mb + 4 * h4 + i;
      if (r16 == 0 && co < a.Nout) {   // this wave's replica; the launcher folds them into bn_sum / bn_sq
        double* rep = a.stat + (size_t)(wave & (adp::STAT_REPL - 1)) * 2 * adp::STAT_CMAX;
        atomicAdd(rep + co, (double)x);
        atomicAdd(rep + adp::STAT_CMAX + co, (double)y);
      }
    }
}

}  // namespace

namespace adp {
// bf16 forward of an input layer: one 8-channel source, K = taps*8 <= 96, Nout <= 64 (weights packed
// [round_up(Nout, 64)][Kpad]), plain store with bias / ReLU / BN statistics.
int launch_fwd_cin8(FwdArgs& a, hipStream_t s) {
  if (option("fwd_cin8", 1) == 0) return 0;
  const int taps = a.kh * a.kw;
  if (a.CAs != 8 || a.CBs != 0 || a.scA || a.up != 1 || a.stride != 1 || taps > 12 || a.K != taps * 8 ||
      a.Kpad < (a.K + 31) / 32 * 32 || a.Nout > 64 || a.Nout % 8 != 0 || a.out_mode != 0 || !a.out ||
      a.out_stride % 4 != 0 || a.addend || a.mask || a.accum || a.drop_rate > 0.f || a.bnr_z)
    return 0;
  // fp8 output (desc out_fp8 on a bf16 launch): 64 channels, 16-B aligned pixel rows, no statistics
  if (a.out_f8 && (a.Nout != 64 || a.out_stride % 16 != 0 || a.bn_sum)) return 0;
  // 16-B output stores (option cin8_wide): every 8-channel run wholly inside or outside Nout (Nout % 8 == 0)
  a.wide_st = option("cin8_wide", 1) && a.out_stride % 8 == 0;
  const int ks = (a.K + 31) / 32;
  if (ks == 1) launch_cin8<1>(a, s);
  else if (ks == 2) launch_cin8<2>(a, s);
  else launch_cin8<3>(a, s);
  return 1;
}

// f32 forward of a 3x3 input layer (igemm_fwd_cin8_f32_kernel): one 8-channel source, Nout <= 64, plain store with
// bias / ReLU / BN statistics; 16-B aligned output rows
int launch_fwd_cin8_f32(FwdArgs& a, hipStream_t s) {
  if (option("fwd_cin8_f32", 1) == 0) return 0;
  if (a.CAs != 8 || a.CBs != 0 || a.scA || a.up != 1 || a.stride != 1 || a.kh != 3 || a.kw != 3 || a.K != 72 ||
      a.Kpad < 72 || a.Nout > 64 || a.Nout % 4 != 0 || a.out_mode != 0 || !a.out || a.out_stride % 4 != 0 ||
      ((uintptr_t)a.out & 15) != 0 || a.addend || a.mask || a.accum || a.drop_rate > 0.f || a.bnr_z || a.out_f8)
    return 0;
  const int groups = (a.M + 15) / 16, unr = 4;
  const int waves = std::max(1, std::min((groups + unr - 1) / unr, option("cin8_waves", 2048)));
  if (a.ca_real > 0 && a.ca_real <= 4) {
    adp::set_kernel("igemm_fwd_cin8_f32_kernel<1, 4>");
    hipLaunchKernelGGL((igemm_fwd_cin8_f32_kernel<1, 4>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
  } else {
    adp::set_kernel("igemm_fwd_cin8_f32_kernel<2, 4>");
    hipLaunchKernelGGL((igemm_fwd_cin8_f32_kernel<2, 4>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
  }
  return 1;
}
}  // namespace adp
