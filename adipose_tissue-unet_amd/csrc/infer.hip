// Inference-side plumbing on the GPU: input normalisation (+TTA view transform folded into the
// load), TTA de-augment + mean, and Gaussian/linear blending of sliding-window tiles.
//   predict_single normalisation        Segmentation/segmentation_inference.py:153-158
//   TestTimeAugmentation (8 D4 views)    Segmentation/segmentation_inference.py:181-229,
//                                        Segmentation/full_evaluation_enhanced.py:522-600
//   GaussianBlender / LinearBlender      Segmentation/full_evaluation_enhanced.py:115-204
#include "common.h"
#include "../../include/adipose_hip.h"

namespace {
constexpr int TPB = 256;
inline int nblk(size_t n, int cap = 8192) {
  size_t b = (n + TPB - 1) / TPB;
  return (int)(b < (size_t)cap ? (b ? b : 1) : cap);
}

// View v of the input image A (S x S): V[a][b] = A[g_v(a,b)], matching the reference transforms
// 0 ident, 1 rot90 (np.rot90 k=1, CCW), 2 rot180, 3 rot270, 4 flipH (axis 1), 5 flipV (axis 0),
// 6 flipH(rot90), 7 flipV(rot90).
ADP_DEV void view_src(int v, int a, int b, int S, int& i, int& j) {
  switch (v) {
    case 1: i = b; j = S - 1 - a; break;
    case 2: i = S - 1 - a; j = S - 1 - b; break;
    case 3: i = S - 1 - b; j = a; break;
    case 4: i = a; j = S - 1 - b; break;
    case 5: i = S - 1 - a; j = b; break;
    case 6: i = S - 1 - b; j = S - 1 - a; break;
    case 7: i = b; j = a; break;
    default: i = a; j = b; break;
  }
}
// inverse: original pixel (i,j) is predicted at view pixel (a,b)
ADP_DEV void view_dst(int v, int i, int j, int S, int& a, int& b) {
  switch (v) {
    case 1: a = S - 1 - j; b = i; break;
    case 2: a = S - 1 - i; b = S - 1 - j; break;
    case 3: a = j; b = S - 1 - i; break;
    case 4: a = i; b = S - 1 - j; break;
    case 5: a = S - 1 - i; b = j; break;
    case 6: a = S - 1 - j; b = S - 1 - i; break;
    case 7: a = j; b = i; break;
    default: a = i; b = j; break;
  }
}

template <typename T>
__global__ void prep_kernel(int N, int H, int W, int Cin, const float* src, long long row_stride,
                            long long img_stride, float mean, float stdv, int view, int Cs, T* dst) {
  // reference: (image - mean) / (std + 1e-10) in float32 (segmentation_inference.py:155)
  const float den = stdv + 1e-10f;
  size_t total = (size_t)N * H * W;
  for (size_t p = blockIdx.x * (size_t)TPB + threadIdx.x; p < total; p += (size_t)gridDim.x * TPB) {
    int b = (int)(p % W);
    size_t t = p / W;
    int a = (int)(t % H), n = (int)(t / H);
    int i, j;
    view_src(view, a, b, H, i, j);
    const float* s = src + (size_t)n * img_stride + ((size_t)i * row_stride + j) * Cin;
    T* d = dst + p * Cs;
    for (int c = 0; c < Cs; ++c) d[c] = from_f<T>(c < Cin ? __fdiv_rn(__fsub_rn(s[c], mean), den) : 0.f);
  }
}

struct ViewList { int v[8]; };

__global__ void tta_merge_kernel(int H, int W, int nv, ViewList views, const float* probs, float* out) {
  size_t total = (size_t)H * W;
  for (size_t p = blockIdx.x * (size_t)TPB + threadIdx.x; p < total; p += (size_t)gridDim.x * TPB) {
    int j = (int)(p % W), i = (int)(p / W);
    float s = 0.f;
    for (int k = 0; k < nv; ++k) {
      int a, b;
      view_dst(views.v[k], i, j, H, a, b);
      s += probs[(size_t)k * total + (size_t)a * W + b];
    }
    out[p] = s / (float)nv;
  }
}

__global__ void blend_accum_kernel(int H, int W, int T, int y0, int x0, const float* tile,
                                   const float* wmap, float* acc, float* wsum) {
  size_t total = (size_t)T * T;
  for (size_t p = blockIdx.x * (size_t)TPB + threadIdx.x; p < total; p += (size_t)gridDim.x * TPB) {
    int j = (int)(p % T), i = (int)(p / T);
    int y = y0 + i, x = x0 + j;
    if (y >= H || x >= W) continue;
    float w = wmap ? wmap[p] : 1.f;
    size_t o = (size_t)y * W + x;
    // separate roundings (hipcc contracts a*b+c into v_fmac by default): bit-identical to numpy's
    // accumulator += tile * weight
    {
#pragma clang fp contract(off)
      acc[o] = acc[o] + tile[p] * w;
    }
    wsum[o] = __fadd_rn(wsum[o], w);
  }
}

__global__ void blend_final_kernel(size_t n, const float* acc, const float* wsum, float fl, float* out) {
  for (size_t p = blockIdx.x * (size_t)TPB + threadIdx.x; p < n; p += (size_t)gridDim.x * TPB)
    out[p] = __fdiv_rn(acc[p], fmaxf(wsum[p], fl));  // IEEE division, as numpy
}
}  // namespace

extern "C" int adp_prep_input(int dtype, int N, int H, int W, int Cin, const float* src, long long src_row_stride,
                              long long src_img_stride, float mean, float stdv, int view, int Cs, void* dst,
                              adp_stream_t st) {
  ADP_REQUIRE(view >= 0 && view < 8, "adp_prep_input: view must be 0..7");
  ADP_REQUIRE(view == 0 || view == 4 || view == 5 || H == W, "adp_prep_input: rotated views need square tiles");
  ADP_REQUIRE(Cs >= Cin && Cs % 8 == 0, "adp_prep_input: bad channel stride");
  if (src_row_stride <= 0) src_row_stride = W;
  if (src_img_stride <= 0) src_img_stride = (long long)H * src_row_stride * Cin;
  ADP_REQUIRE(src_row_stride >= W, "adp_prep_input: row stride smaller than the tile width");
  size_t n = (size_t)N * H * W;
  if (dtype == ADP_F32)
    hipLaunchKernelGGL(prep_kernel<float>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, H, W, Cin, src,
                       src_row_stride, src_img_stride, mean, stdv, view, Cs, (float*)dst);
  else if (dtype == ADP_BF16)
    hipLaunchKernelGGL(prep_kernel<bf16>, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, N, H, W, Cin, src,
                       src_row_stride, src_img_stride, mean, stdv, view, Cs, (bf16*)dst);
  else { adp::set_error("adp_prep_input: bad dtype"); return -1; }
  return adp::check_launch("adp_prep_input");
}

extern "C" int adp_tta_merge(int H, int W, int nv, const int* views, const float* probs, float* out,
                             adp_stream_t st) {
  ADP_REQUIRE(nv > 0 && nv <= 8 && H == W && views, "adp_tta_merge: need 1..8 views on a square tile");
  ViewList vl{};
  for (int k = 0; k < nv; ++k) {
    ADP_REQUIRE(views[k] >= 0 && views[k] < 8, "adp_tta_merge: view out of range");
    vl.v[k] = views[k];
  }
  size_t n = (size_t)H * W;
  hipLaunchKernelGGL(tta_merge_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, H, W, nv, vl, probs, out);
  return adp::check_launch("adp_tta_merge");
}

extern "C" int adp_blend_accum(int H, int W, int T, int y0, int x0, const float* tile, const float* weight,
                               float* acc, float* wsum, adp_stream_t st) {
  ADP_REQUIRE(y0 >= 0 && x0 >= 0 && T > 0, "adp_blend_accum: bad tile position");
  size_t n = (size_t)T * T;
  hipLaunchKernelGGL(blend_accum_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, H, W, T, y0, x0, tile,
                     weight, acc, wsum);
  return adp::check_launch("adp_blend_accum");
}

extern "C" int adp_blend_finalize(size_t n, const float* acc, const float* wsum, float fl, float* out,
                                  adp_stream_t st) {
  hipLaunchKernelGGL(blend_final_kernel, dim3(nblk(n)), dim3(TPB), 0, (hipStream_t)st, n, acc, wsum, fl, out);
  return adp::check_launch("adp_blend_finalize");
}
