// Shared device/host helpers for libadipose_hip (gfx950 / CDNA4 only).
//
// Layout conventions used by every kernel in this library:
//   * activations are NHWC, channel stride padded to a multiple of 8 ("group" = 8 channels
//     = 16 B in bf16, 32 B in f32); pad channels are kept at zero by construction;
//   * GEMM weights are stored [Npad][Kpad] (output channel major, K contiguous) with
//     K = taps * Cin_stride, Kpad = round_up(K, 32), Npad = round_up(N, 64);
//   * f32 is the parity dtype (exact f32 MFMA), bf16 the throughput dtype (f32 accumulate).
#pragma once
#include <hip/hip_runtime.h>

// Timing-only ablation switches (options fwd_debug / wgrad_debug) are read by the kernels only in a library built
// with -DADP_ABLATION (make ABLATION=1: tools that measure ablations build that variant into ab/). In the product build
// ADP_DBG is the constant 0 and every ablation branch compiles away: as run-time branches inside the K loops they cost
// the halo weight gradient 8 % (its waits were selected per column block at run time; profiles/r05_bisect.log).
#ifdef ADP_ABLATION
#define ADP_DBG(a) ((a).debug_flags)
#else
#define ADP_DBG(a) 0
#endif
#include <stdint.h>
#include <algorithm>
#include <cmath>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define ADP_DEV __device__ __forceinline__

enum AdpDtype { ADP_F32 = 0, ADP_BF16 = 1, ADP_FP8 = 2 };

// ---- OCP fp8 e4m3fn (gfx950 v_cvt_*_fp8): saturating encode of 8 values into 8 bytes, decode one byte
constexpr float FP8_MAX = 448.f;
ADP_DEV uint2 f8x8_from_f(const float* v) {
  float c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = fminf(fmaxf(v[j], -FP8_MAX), FP8_MAX);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
}
ADP_DEV void f8x8_to_f(uint2 q, float* f) {
  f[0] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 0); f[1] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 1);
  f[2] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 2); f[3] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 3);
  f[4] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 0); f[5] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 1);
  f[6] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 2); f[7] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 3);
}

// 8-channel group as raw bytes: 16 B for bf16, 32 B for f32.
template <typename T> struct Grp;
template <> struct Grp<bf16> { uint4 v; };
template <> struct Grp<float> { uint4 v[2]; };

ADP_DEV float to_f(float x) { return x; }
ADP_DEV float to_f(bf16 x) { return (float)x; }
template <typename T> ADP_DEV T from_f(float x);
template <> ADP_DEV float from_f<float>(float x) { return x; }
template <> ADP_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

ADP_DEV void grp_zero(Grp<bf16>& g) { g.v = make_uint4(0, 0, 0, 0); }
ADP_DEV void grp_zero(Grp<float>& g) { g.v[0] = make_uint4(0, 0, 0, 0); g.v[1] = g.v[0]; }
ADP_DEV void grp_load(Grp<bf16>& g, const bf16* p) { g.v = *reinterpret_cast<const uint4*>(p); }
ADP_DEV void grp_load(Grp<float>& g, const float* p) {
  g.v[0] = reinterpret_cast<const uint4*>(p)[0];
  g.v[1] = reinterpret_cast<const uint4*>(p)[1];
}
ADP_DEV void grp_store(const Grp<bf16>& g, bf16* p) { *reinterpret_cast<uint4*>(p) = g.v; }
ADP_DEV void grp_store(const Grp<float>& g, float* p) {
  reinterpret_cast<uint4*>(p)[0] = g.v[0];
  reinterpret_cast<uint4*>(p)[1] = g.v[1];
}
ADP_DEV void grp_to_f(const Grp<bf16>& g, float* f) {
  const bf16* e = reinterpret_cast<const bf16*>(&g.v);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)e[j];
}
ADP_DEV void grp_to_f(const Grp<float>& g, float* f) {
  const float* e = reinterpret_cast<const float*>(&g.v[0]);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = e[j];
}
ADP_DEV void grp_from_f(Grp<bf16>& g, const float* f) {
  bf16* e = reinterpret_cast<bf16*>(&g.v);
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = (bf16)f[j];
}
ADP_DEV void grp_from_f(Grp<float>& g, const float* f) {
  float* e = reinterpret_cast<float*>(&g.v[0]);
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = f[j];
}

// Stateless counter-based RNG for dropout (lowbias32 mix of seed and element index):
// the mask is never stored, backward derives it from the stored post-dropout activation.
ADP_DEV uint32_t adp_hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
ADP_DEV float adp_uniform(uint32_t seed, uint64_t idx) {
  uint32_t h = adp_hash(seed ^ adp_hash((uint32_t)idx ^ adp_hash((uint32_t)(idx >> 32) + 0x9e3779b9U)));
  return (h >> 8) * (1.0f / 16777216.0f);
}

ADP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- host side error plumbing
#ifdef __cplusplus
#include <string>
namespace adp {
void set_error(const std::string& msg);
int check_launch(const char* what);
int option(const char* name, int dflt);  // runtime switches set through adp_set_option
// blocks of `kernel` (threads per block, dynamic LDS bytes) that fit on the device at once: occupancy per
// CU x CU count (cached per kernel and device) -- the grid of a grid-stride kernel whose blocks should all
// be resident (no second round of blocks, no tail)
int resident_grid(const void* kernel, int threads, size_t smem = 0);
// name of the kernel the last conv launch of this thread used (adp_last_kernel), printf-style
void set_kernel(const char* fmt, ...);
// per-launch timing (adp_timing): the stream of the conv launch in progress (set at the ABI entry), and the
// end mark of its main kernel (call right after launching it; set_kernel marks the start)
void set_launch_stream(hipStream_t s);
void kernel_end();
// Replicated per-channel accumulators for the BatchNorm sums (statistics of a conv output, or the
// BN-backward dbeta/dgamma reductions). Atomics execute at the memory side and serialise per
// address, so thousands of blocks adding into the same C values queue behind each other (measured:
// ~17 ns per add per address, 1.75 ms per training step); blocks add into replica (block & 63)
// instead and stat_fold() sums the replicas into the caller's accumulators and re-zeroes them.
// The replicas are f64 (round 4): each producer adds f32 partials summed in a fixed order, and f64 sums
// of them in the atomics' run-dependent order round to the same f32 (deterministic BatchNorm statistics).
// Per device, lazily allocated and zeroed; launches that use it must be ordered on one stream.
constexpr int STAT_REPL = 64, STAT_CMAX = 2048;
double* stat_scratch();   // [STAT_REPL][2][STAT_CMAX] f64, or nullptr (error set) if allocation failed or a
                         // deferred fold is pending
// bn_defer_fold bookkeeping: a launch that leaves its sums in the replicas records (C, sum, stream); only the
// adp_bn_finalize_fold with the same three may take the replicas next (stat_scratch_fold clears the record)
int defer_fold_begin(int C, const float* sum, hipStream_t s);
double* stat_scratch_fold(int C, const float* sum, hipStream_t s);
int bn_fold_reset(hipStream_t s);   // adp_bn_fold_reset
// dynamic tile claiming: a zeroed slot of CLAIM_INTS counters for one persistent launch (a ring of CLAIM_SLOTS per
// device, handed out in turn; a launch leaves its slot zeroed again), or nullptr (error set)
constexpr int CLAIM_SLOTS = 64, CLAIM_INTS = 512;
int* claim_slot();
// per-device growable scratch (slot 0: weight-gradient split partials / slabs, 1: dz of the unfused BN-backward
// weight gradient, 2: metrics, 3: bias-gradient block sums); growing synchronises the device
void* scratch(int slot, size_t bytes);
// deferred weight-gradient slab reductions of a stream (adp_wgrad_defer / adp_wgrad_flush; conv_wgrad_tap64.hip)
int wgrad_defer(hipStream_t s, int on);
int wgrad_flush(hipStream_t s);
int wgrad_release(hipStream_t s);
int wgrad_arena_chunks(hipStream_t s);
int stat_fold(int C, float* dst0, float* dst1, hipStream_t s);   // elementwise.hip
// the same over replica channels [c0, c0 + C) into dst0[0..C) (and dst1 unless nullptr)
int stat_fold_at(int c0, int C, float* dst0, float* dst1, hipStream_t s);
}  // namespace adp
#define ADP_REQUIRE(cond, msg)          \
  do {                                  \
    if (!(cond)) {                      \
      adp::set_error(msg);              \
      return -1;                        \
    }                                   \
  } while (0)
#endif
