// BoundaryRefiner.refine (Segmentation/full_evaluation_enhanced.py:332-393) on the GPU, for one (H, W) f32
// probability map:
//   m = uint8(mask * 255) (truncation; values outside [0, 1] clamped first)
//   eroded / dilated = cv2.erode / cv2.dilate(m, ellipse(k))   (OpenCV's default morphology border: pixels
//                                                              outside the image take no part)
//   boundary = (dilated > 0) xor (eroded > 0)
//   filtered = cv2.bilateralFilter(m, d, sigma_color, sigma_space)   (radius d / 2, circular window, f32 weights
//              exp(-r^2 / (2 sigma_space^2)) * exp(-|v - v0|^2 / (2 sigma_color^2)), BORDER_REFLECT_101,
//              round-half-even of sum / wsum; the scalar accumulation order of OpenCV's 8u kernel)
//   refined = boundary ? filtered : m; then MORPH_OPEN (erode, dilate) and MORPH_CLOSE (dilate, erode)
//   out = f32(refined / 255.0)
// The ellipse is getStructuringElement(MORPH_ELLIPSE, (k, k)): row i spans the columns [c - dx, c + dx] with
// dx = round(c * sqrt((r^2 - (i - r)^2) / r^2)) (computed by the caller, passed as row extents).
// Every pass is one HBM-bound u8 plane sweep (1 MiB per 1024^2 tile); cv2 itself is absent here, so the
// pixel output is checked against the numpy restatement in oracle/numpy_ref.py (parity unpinned vs cv2).
#include "common.h"
#include "../../include/adipose_hip.h"

namespace {

constexpr int TPB = 256;
constexpr int KMAX = 31;

struct Footprint {
  int k;
  int j1[KMAX], j2[KMAX];
};

int grid_for(size_t n) { return (int)std::max<size_t>(1, std::min<size_t>((n + TPB - 1) / TPB, 8192)); }

__global__ void to_u8_kernel(size_t n, const float* __restrict__ mask, unsigned char* __restrict__ m) {
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const float v = __fmul_rn(fminf(fmaxf(mask[i], 0.f), 1.f), 255.f);
    m[i] = (unsigned char)(int)v;   // astype(np.uint8) of a value in [0, 255]: truncation
  }
}

// grey erosion (is_max = 0) / dilation (1) with the footprint, pixels outside the image ignored
__global__ void morph_kernel(int H, int W, const unsigned char* __restrict__ src, unsigned char* __restrict__ dst,
                             Footprint fp, int is_max) {
  const size_t n = (size_t)H * W;
  const int r = fp.k / 2;
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int y = (int)(i / W), x = (int)(i % W);
    int v = is_max ? 0 : 255;
    for (int a = 0; a < fp.k; ++a) {
      const int yy = y + a - r;
      if (yy < 0 || yy >= H) continue;
      const unsigned char* row = src + (size_t)yy * W;
      for (int b = fp.j1[a]; b < fp.j2[a]; ++b) {
        const int xx = x + b - r;
        if (xx < 0 || xx >= W) continue;
        const int s = row[xx];
        v = is_max ? max(v, s) : min(v, s);
      }
    }
    dst[i] = (unsigned char)v;
  }
}

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

// boundary band from the eroded / dilated planes, the bilateral filter inside it, m outside it
__global__ void band_bilateral_kernel(int H, int W, const unsigned char* __restrict__ m,
                                      const unsigned char* __restrict__ er, const unsigned char* __restrict__ di,
                                      unsigned char* __restrict__ out, int radius, double cspace, double ccolor) {
  __shared__ float cw[256];
  __shared__ float sw[(2 * 15 + 1) * (2 * 15 + 1)];
  __shared__ int sdy[(2 * 15 + 1) * (2 * 15 + 1)], sdx[(2 * 15 + 1) * (2 * 15 + 1)];
  __shared__ int nk;
  for (int t = threadIdx.x; t < 256; t += TPB) cw[t] = (float)exp((double)t * t * ccolor);
  if (threadIdx.x == 0) {   // OpenCV's offset order: rows -radius..radius, columns -radius..radius, r <= radius
    int k = 0;
    for (int a = -radius; a <= radius; ++a)
      for (int b = -radius; b <= radius; ++b) {
        const double rr = sqrt((double)a * a + (double)b * b);
        if (rr > radius) continue;
        sw[k] = (float)exp(rr * rr * cspace);
        sdy[k] = a;
        sdx[k] = b;
        ++k;
      }
    nk = k;
  }
  __syncthreads();
  const size_t n = (size_t)H * W;
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
    const int v0 = m[i];
    if ((di[i] > 0) == (er[i] > 0)) {
      out[i] = (unsigned char)v0;
      continue;
    }
    const int y = (int)(i / W), x = (int)(i % W);
    float sum = 0.f, wsum = 0.f;
    for (int k = 0; k < nk; ++k) {
      const int v = m[(size_t)reflect101(y + sdy[k], H) * W + reflect101(x + sdx[k], W)];
      const float w = __fmul_rn(sw[k], cw[abs(v - v0)]);
      sum = __fadd_rn(sum, __fmul_rn((float)v, w));
      wsum = __fadd_rn(wsum, w);
    }
    const float q = __fdiv_rn(sum, wsum);
    out[i] = (unsigned char)min(max((int)rintf(q), 0), 255);
  }
}

__global__ void to_f32_kernel(size_t n, const unsigned char* __restrict__ m, float* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
    out[i] = (float)((double)m[i] / 255.0);
}

}  // namespace

extern "C" int adp_boundary_refine(int H, int W, const float* mask, int ksize, const int* row_lo, const int* row_hi,
                                   int d, float sigma_color, float sigma_space, void* work, float* out,
                                   adp_stream_t st) {
  ADP_REQUIRE(H > 0 && W > 0 && mask && work && out && row_lo && row_hi && ksize >= 1 && ksize <= KMAX,
              "adp_boundary_refine: positive H, W, 1 <= ksize <= 31, every buffer and the footprint rows");
  // cv2.bilateralFilter's parameter handling: sigma <= 0 -> 1, radius = d / 2 (d <= 0: 1.5 sigma_space), >= 1
  const float scol = sigma_color <= 0.f ? 1.f : sigma_color, sspa = sigma_space <= 0.f ? 1.f : sigma_space;
  int radius = d <= 0 ? (int)lrint(sspa * 1.5) : d / 2;
  radius = std::max(radius, 1);
  ADP_REQUIRE(radius <= 15, "adp_boundary_refine: bilateral diameter above 31");
  Footprint fp{};
  fp.k = ksize;
  for (int i = 0; i < ksize; ++i) {
    ADP_REQUIRE(row_lo[i] >= 0 && row_hi[i] <= ksize && row_lo[i] <= row_hi[i], "adp_boundary_refine: bad footprint row");
    fp.j1[i] = row_lo[i];
    fp.j2[i] = row_hi[i];
  }
  hipStream_t s = (hipStream_t)st;
  const size_t n = (size_t)H * W;
  unsigned char* m = static_cast<unsigned char*>(work);
  unsigned char* a = m + n;
  unsigned char* b = a + n;
  unsigned char* c = b + n;
  const int g = grid_for(n);
  hipLaunchKernelGGL(to_u8_kernel, dim3(g), dim3(TPB), 0, s, n, mask, m);
  hipLaunchKernelGGL(morph_kernel, dim3(g), dim3(TPB), 0, s, H, W, m, a, fp, 0);   // eroded
  hipLaunchKernelGGL(morph_kernel, dim3(g), dim3(TPB), 0, s, H, W, m, b, fp, 1);   // dilated
  hipLaunchKernelGGL(band_bilateral_kernel, dim3(g), dim3(TPB), 0, s, H, W, m, a, b, c, radius,
                     -0.5 / ((double)sspa * sspa), -0.5 / ((double)scol * scol));
  hipLaunchKernelGGL(morph_kernel, dim3(g), dim3(TPB), 0, s, H, W, c, a, fp, 0);   // open: erode
  hipLaunchKernelGGL(morph_kernel, dim3(g), dim3(TPB), 0, s, H, W, a, b, fp, 1);   //       dilate
  hipLaunchKernelGGL(morph_kernel, dim3(g), dim3(TPB), 0, s, H, W, b, a, fp, 1);   // close: dilate
  hipLaunchKernelGGL(morph_kernel, dim3(g), dim3(TPB), 0, s, H, W, a, b, fp, 0);   //        erode
  hipLaunchKernelGGL(to_f32_kernel, dim3(g), dim3(TPB), 0, s, n, b, out);
  return adp::check_launch("adp_boundary_refine");
}
