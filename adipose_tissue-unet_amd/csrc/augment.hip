// Training-time augmentation and normalisation of gray tiles on the GPU (src/utils/data.py:13-264,
// 398-429; TileDataset, train_adipose_unet_v3.py:568-607). The host draws every random parameter in
// the reference's RandomState order (adipose_amd/augment.py); these kernels do the pixel work on f32
// (H, W) planes. Arithmetic follows numpy's float32 evaluation order where the reference is numpy
// (separate roundings, no fused multiply-add), and OpenCV's documented semantics where it is cv2:
//   resize INTER_LINEAR   src = (dst + 0.5) * in/out - 0.5, clamped to the edge (float coefficients)
//   resize INTER_NEAREST  src = floor(dst * in/out), clamped
//   GaussianBlur(0,0,s)   separable, ksize = round(8s + 1) | 1, BORDER_REFLECT_101, f32 taps
//   remap INTER_LINEAR    maps rounded to 1/32 pixel (INTER_TAB_SIZE), BORDER_REFLECT
//   remap INTER_NEAREST   maps rounded to the nearest pixel, BORDER_CONSTANT 0
// (cv2 is not installed here: those five are restatements, "parity unpinned" in the tests).
#include "common.h"
#include "../../include/adipose_hip.h"

namespace {

constexpr int TPB = 256;
inline int nblk(size_t n) {
  size_t b = (n + TPB - 1) / TPB;
  return (int)std::min<size_t>(std::max<size_t>(b, 1), 16384);
}

// np.rot90(x, k) (counter-clockwise) then fliplr (axis 1) then flipud (axis 0): dst is (Ho, Wo)
__global__ void geom_kernel(int H, int W, const float* src, float* dst, int k, int flr, int fud) {
  const int Ho = (k & 1) ? W : H, Wo = (k & 1) ? H : W;
  const size_t n = (size_t)Ho * Wo;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    int y = (int)(i / Wo), x = (int)(i % Wo);
    if (fud) y = Ho - 1 - y;
    if (flr) x = Wo - 1 - x;
    int sy, sx;   // rot90 k: out[y][x] = in[...]
    switch (k & 3) {
      case 0: sy = y; sx = x; break;
      case 1: sy = x; sx = W - 1 - y; break;
      case 2: sy = H - 1 - y; sx = W - 1 - x; break;
      default: sy = H - 1 - x; sx = y; break;
    }
    dst[i] = src[(size_t)sy * W + sx];
  }
}

// mode 0 brightness: clip(x*f, 0, 255); 1 contrast: clip((x - m)*f + m, 0, 255); 2 gamma: (x/255)^g * 255;
// 3 z-score (x - m) / f (TileDataset zscore, train_adipose_unet_v3.py:589-590, f = std + 1e-10)
__global__ void photo_kernel(size_t n, const float* src, float* dst, int mode, float f, float m) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const float x = src[i];
    float y;
    if (mode == 0) y = fminf(fmaxf(__fmul_rn(x, f), 0.f), 255.f);
    else if (mode == 1) y = fminf(fmaxf(__fadd_rn(__fmul_rn(__fsub_rn(x, m), f), m), 0.f), 255.f);
    else if (mode == 2) y = __fmul_rn(powf(__fdiv_rn(x, 255.f), f), 255.f);
    else y = __fdiv_rn(__fsub_rn(x, m), f);
    dst[i] = y;
  }
}

// image + noise (f64, as numpy promotes), clipped to [0, 255] in f64, rounded to f32 once
__global__ void noise_kernel(size_t n, const float* src, const double* noise, float* dst) {
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
    dst[i] = (float)fmin(fmax((double)src[i] + noise[i], 0.0), 255.0);
}

// sum (f64) of a plane -> *out (for contrast's image.mean())
__global__ void sum_kernel(size_t n, const float* src, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) s += src[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double red[TPB / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < TPB / 64; ++w) t += red[w];
    atomicAdd(out, t);
  }
}

ADP_DEV int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}
ADP_DEV int reflect(int p, int n) {   // BORDER_REFLECT: fedcba|abcdef|fedcba
  while (p < 0 || p >= n) p = p < 0 ? -p - 1 : 2 * n - 1 - p;
  return p;
}

// one separable pass of a Gaussian (taps w[0..2r]); axis 0 = along x (rows), 1 = along y (columns)
template <typename T>
__global__ void blur_kernel(int H, int W, const T* src, T* dst, const float* w, int r, int axis) {
  const size_t n = (size_t)H * W;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int y = (int)(i / W), x = (int)(i % W);
    T acc = 0;
    for (int t = -r; t <= r; ++t) {
      const T v = axis == 0 ? src[(size_t)y * W + reflect101(x + t, W)] : src[(size_t)reflect101(y + t, H) * W + x];
      acc += (T)w[t + r] * v;
    }
    dst[i] = acc;
  }
}

// cv2.resize of (H, W) to (Hn, Wn), then the reference's center crop (Hn >= H) or pad to (H, W)
// (image: numpy 'reflect' = BORDER_REFLECT_101, mask: constant 0). nearest: INTER_NEAREST (masks).
__global__ void scale_kernel(int H, int W, int Hn, int Wn, const float* src, float* dst, int nearest) {
  const size_t n = (size_t)H * W;
  const float sy = (float)H / (float)Hn, sx = (float)W / (float)Wn;   // cv2: inv_scale = src / dst
  const bool zoom_in = Hn >= H;
  const int oy = zoom_in ? (Hn - H) / 2 : (H - Hn) / 2, ox = zoom_in ? (Wn - W) / 2 : (W - Wn) / 2;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int y = (int)(i / W), x = (int)(i % W);
    int yr, xr;   // coordinate in the resized (Hn, Wn) image
    if (zoom_in) {
      yr = y + oy; xr = x + ox;
    } else {
      yr = y - oy; xr = x - ox;
      if (yr < 0 || yr >= Hn || xr < 0 || xr >= Wn) {
        if (nearest) { dst[i] = 0.f; continue; }
        yr = reflect101(yr, Hn);
        xr = reflect101(xr, Wn);
      }
    }
    float v;
    if (nearest) {
      const int ys = min((int)floorf(yr * sy), H - 1), xs = min((int)floorf(xr * sx), W - 1);
      v = src[(size_t)ys * W + xs];
    } else {
      float fy = (yr + 0.5f) * sy - 0.5f, fx = (xr + 0.5f) * sx - 0.5f;
      int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
      fy -= y0; fx -= x0;
      if (y0 < 0) { y0 = 0; fy = 0.f; }
      if (x0 < 0) { x0 = 0; fx = 0.f; }
      if (y0 >= H - 1) { y0 = H - 1; fy = 0.f; }
      if (x0 >= W - 1) { x0 = W - 1; fx = 0.f; }
      const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
      const float a = src[(size_t)y0 * W + x0], b = src[(size_t)y0 * W + x1];
      const float c = src[(size_t)y1 * W + x0], d = src[(size_t)y1 * W + x1];
      v = (a * (1.f - fx) + b * fx) * (1.f - fy) + (c * (1.f - fx) + d * fx) * fy;
    }
    dst[i] = v;
  }
}

// elastic remap: map_y = f32(y + dy*alpha), map_x = f32(x + dx*alpha) (dx, dy: the blurred f64 fields)
__global__ void remap_kernel(int H, int W, const float* src, const float* msrc, const double* dx, const double* dy,
                             double alpha, float* dst, float* mdst) {
  const size_t n = (size_t)H * W;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int y = (int)(i / W), x = (int)(i % W);
    const float my = (float)((double)y + dy[i] * alpha), mx = (float)((double)x + dx[i] * alpha);
    // image: INTER_LINEAR on 1/32-pixel fixed-point maps, BORDER_REFLECT
    const int X = (int)rintf(mx * 32.f), Y = (int)rintf(my * 32.f);
    const int x0 = X >> 5, y0 = Y >> 5;
    const float fx = (X & 31) * (1.f / 32.f), fy = (Y & 31) * (1.f / 32.f);
    const int xa = reflect(x0, W), xb = reflect(x0 + 1, W), ya = reflect(y0, H), yb = reflect(y0 + 1, H);
    const float a = src[(size_t)ya * W + xa], b = src[(size_t)ya * W + xb];
    const float c = src[(size_t)yb * W + xa], d = src[(size_t)yb * W + xb];
    dst[i] = (a * (1.f - fx) + b * fx) * (1.f - fy) + (c * (1.f - fx) + d * fx) * fy;
    // mask: INTER_NEAREST (maps rounded), BORDER_CONSTANT 0
    const int xn = (int)rintf(mx), yn = (int)rintf(my);
    mdst[i] = (xn >= 0 && xn < W && yn >= 0 && yn < H) ? msrc[(size_t)yn * W + xn] : 0.f;
  }
}

// ---- exact order statistics (np.percentile, linear) by a 3-pass radix select on the f32 bit pattern
ADP_DEV uint32_t fkey(float f) {   // monotone map f32 -> u32
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
ADP_DEV float fval(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k); }

// state per plane: sel[q] = {prefix, rank remaining} for 4 ranks; hist [4][2048]
struct SelState { uint32_t prefix[4]; uint32_t rank[4]; };
constexpr int RB = 11, NB = 1 << RB;   // 11 + 11 + 10 bits

__global__ void sel_hist_kernel(size_t n, const float* src, const SelState* st, int pass, unsigned* hist) {
  __shared__ unsigned h[4][NB];
  for (int i = threadIdx.x; i < 4 * NB; i += TPB) (&h[0][0])[i] = 0;
  __syncthreads();
  const int shift = pass == 0 ? 21 : pass == 1 ? 10 : 0;
  const uint32_t bits = pass == 2 ? 10 : 11;
  const uint32_t pmask = pass == 0 ? 0u : pass == 1 ? 0xFFE00000u : 0xFFFFFC00u;
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const uint32_t k = fkey(src[i]);
    const uint32_t b = (k >> shift) & ((1u << bits) - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if ((k & pmask) == st->prefix[q]) atomicAdd(&h[q][b], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * NB; i += TPB)
    if ((&h[0][0])[i]) atomicAdd(hist + i, (&h[0][0])[i]);
}

__global__ void sel_init_kernel(SelState* st, unsigned* hist, uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3) {
  if (blockIdx.x == 0 && threadIdx.x < 4) {
    const uint32_t r[4] = {r0, r1, r2, r3};
    st->prefix[threadIdx.x] = 0;
    st->rank[threadIdx.x] = r[threadIdx.x];
  }
  for (int i = blockIdx.x * TPB + threadIdx.x; i < 4 * NB; i += gridDim.x * TPB) hist[i] = 0;
}

// block q: find the bin holding rank[q] (chunked parallel scan), fold it into prefix[q], re-zero hist[q]
__global__ void sel_scan_kernel(SelState* st, int pass, unsigned* hist) {
  const int q = blockIdx.x, t = threadIdx.x;
  const int shift = pass == 0 ? 21 : pass == 1 ? 10 : 0;
  constexpr int PER = NB / TPB;   // 8 bins per thread
  unsigned* h = hist + q * NB;
  unsigned v[PER], tot = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) { v[j] = h[t * PER + j]; tot += v[j]; }
  __shared__ unsigned part[TPB];
  __shared__ unsigned base[TPB];
  part[t] = tot;
  __syncthreads();
  if (t == 0) {
    unsigned acc = 0;
    for (int i = 0; i < TPB; ++i) { base[i] = acc; acc += part[i]; }
  }
  __syncthreads();
  const uint32_t r = st->rank[q];
  __syncthreads();   // every thread has read rank before the owner updates it
  if (r >= base[t] && r < base[t] + tot) {
    uint32_t rr = r - base[t];
    int j = 0;
    for (; j < PER; ++j) {
      if (rr < v[j]) break;
      rr -= v[j];
    }
    st->prefix[q] |= (uint32_t)(t * PER + j) << shift;
    st->rank[q] = rr;
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) h[t * PER + j] = 0;   // ready for the next pass
}

// percentile normalisation: p = lerp of the order statistics (numpy 'linear', in f64), then
// clip((x - p_lo) / max(p_hi - p_lo, 1e-3), 0, 1) evaluated as the reference's pinned numpy 1.23.5 does
// (value-based casting: the f64 scalars are rounded to f32 and the array arithmetic is f32; numpy >= 2
// would evaluate in f64 -- at most 1 ulp apart) (data.py:398-429)
__global__ void pct_norm_kernel(size_t n, const float* src, const SelState* st, double tlo, double thi, float* dst,
                                float* pout) {
  auto lerp = [](double a, double b, double t) {   // numpy._lerp
    const double d = b - a;
    return t >= 0.5 ? b - d * (1.0 - t) : a + d * t;
  };
  const double plo = lerp(fval(st->prefix[0]), fval(st->prefix[1]), tlo);
  const double phi = lerp(fval(st->prefix[2]), fval(st->prefix[3]), thi);
  const float plo32 = (float)plo, den32 = (float)fmax(phi - plo, 1e-3);
  if (blockIdx.x == 0 && threadIdx.x == 0 && pout) { pout[0] = (float)plo; pout[1] = (float)phi; }
  for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
    dst[i] = fminf(fmaxf(__fdiv_rn(__fsub_rn(src[i], plo32), den32), 0.f), 1.f);
}

}  // namespace

extern "C" int adp_aug_geom(int H, int W, const float* src, float* dst, int k, int flip_lr, int flip_ud,
                            adp_stream_t st) {
  ADP_REQUIRE(H > 0 && W > 0 && src && dst && src != dst, "adp_aug_geom: bad arguments (out of place only)");
  hipLaunchKernelGGL(geom_kernel, dim3(nblk((size_t)H * W)), dim3(TPB), 0, (hipStream_t)st, H, W, src, dst, k & 3,
                     flip_lr, flip_ud);
  return adp::check_launch("adp_aug_geom");
}

extern "C" int adp_aug_photometric(size_t n, const float* src, float* dst, int mode, float f, float m,
                                   adp_stream_t st) {
  ADP_REQUIRE(mode >= 0 && mode <= 3 && src && dst,
              "adp_aug_photometric: mode 0 brightness, 1 contrast, 2 gamma, 3 z-score");
  hipLaunchKernelGGL(photo_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, n, src, dst, mode, f, m);
  return adp::check_launch("adp_aug_photometric");
}

extern "C" int adp_aug_noise(size_t n, const float* src, const double* noise, float* dst, adp_stream_t st) {
  hipLaunchKernelGGL(noise_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, n, src, noise, dst);
  return adp::check_launch("adp_aug_noise");
}

extern "C" int adp_aug_sum(size_t n, const float* src, double* out, adp_stream_t st) {
  hipLaunchKernelGGL(sum_kernel, dim3(std::min(nblk(n), 1024)), dim3(TPB), 0, (hipStream_t)st, n, src, out);
  return adp::check_launch("adp_aug_sum");
}

extern "C" int adp_aug_blur(int dtype64, int H, int W, const void* src, void* tmp, void* dst, const float* taps,
                            int radius, adp_stream_t st) {
  ADP_REQUIRE(radius >= 0 && taps && src && tmp && dst, "adp_aug_blur: bad arguments");
  hipStream_t s = (hipStream_t)st;
  const int nb = nblk((size_t)H * W);
  if (dtype64) {
    hipLaunchKernelGGL(blur_kernel<double>, dim3(nb), dim3(TPB), 0, s, H, W, (const double*)src, (double*)tmp, taps,
                       radius, 0);
    hipLaunchKernelGGL(blur_kernel<double>, dim3(nb), dim3(TPB), 0, s, H, W, (const double*)tmp, (double*)dst, taps,
                       radius, 1);
  } else {
    hipLaunchKernelGGL(blur_kernel<float>, dim3(nb), dim3(TPB), 0, s, H, W, (const float*)src, (float*)tmp, taps,
                       radius, 0);
    hipLaunchKernelGGL(blur_kernel<float>, dim3(nb), dim3(TPB), 0, s, H, W, (const float*)tmp, (float*)dst, taps,
                       radius, 1);
  }
  return adp::check_launch("adp_aug_blur");
}

extern "C" int adp_aug_scale(int H, int W, int Hn, int Wn, const float* src, float* dst, int nearest, adp_stream_t st) {
  ADP_REQUIRE(Hn > 0 && Wn > 0 && (Hn >= H) == (Wn >= W) && src != dst, "adp_aug_scale: bad arguments");
  hipLaunchKernelGGL(scale_kernel, dim3(nblk((size_t)H * W)), dim3(TPB), 0, (hipStream_t)st, H, W, Hn, Wn, src, dst,
                     nearest);
  return adp::check_launch("adp_aug_scale");
}

extern "C" int adp_aug_remap(int H, int W, const float* src, const float* msrc, const double* dx, const double* dy,
                             double alpha, float* dst, float* mdst, adp_stream_t st) {
  ADP_REQUIRE(src != dst && msrc != mdst, "adp_aug_remap: out of place only");
  hipLaunchKernelGGL(remap_kernel, dim3(nblk((size_t)H * W)), dim3(TPB), 0, (hipStream_t)st, H, W, src, msrc, dx, dy,
                     alpha, dst, mdst);
  return adp::check_launch("adp_aug_remap");
}

// work: >= 16 + 4*2048*4 bytes of device scratch (SelState + histograms), caller-owned
extern "C" int adp_percentile_normalize(size_t n, const float* src, float* dst, double p_low, double p_high,
                                        void* work, float* p_out, adp_stream_t st) {
  ADP_REQUIRE(n > 0 && src && dst && work && p_low >= 0 && p_high <= 100 && p_low <= p_high,
              "adp_percentile_normalize: bad arguments");
  hipStream_t s = (hipStream_t)st;
  const double pl = p_low / 100.0 * (double)(n - 1), ph = p_high / 100.0 * (double)(n - 1);
  const uint32_t l0 = (uint32_t)floor(pl), h0 = (uint32_t)floor(ph);
  SelState* sd = reinterpret_cast<SelState*>(work);
  unsigned* hist = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(work) + 64);
  hipLaunchKernelGGL(sel_init_kernel, dim3(8), dim3(TPB), 0, s, sd, hist, l0, (uint32_t)std::min<size_t>(l0 + 1, n - 1),
                     h0, (uint32_t)std::min<size_t>(h0 + 1, n - 1));
  const int nb = std::min(nblk(n), 1024);
  for (int pass = 0; pass < 3; ++pass) {
    hipLaunchKernelGGL(sel_hist_kernel, dim3(nb), dim3(TPB), 0, s, n, src, sd, pass, hist);
    hipLaunchKernelGGL(sel_scan_kernel, dim3(4), dim3(TPB), 0, s, sd, pass, hist);
  }
  hipLaunchKernelGGL(pct_norm_kernel, dim3(nblk(n)), dim3(TPB), 0, s, n, src, sd, pl - floor(pl), ph - floor(ph), dst,
                     p_out);
  return adp::check_launch("adp_percentile_normalize");
}
