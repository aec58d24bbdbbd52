// Inter-kernel gap probe: does the idle time between two dependent kernels on one stream grow with the dirty data
// the first one leaves in the L2s (written back at its end-of-kernel release)? Kernel `writer<AUX>` stores `mb` MB
// with buffer-store cache policy AUX (0 default, 2 nt, 16 sc1, 17 sc0|sc1, 19 nt|sc0|sc1), kernel `tiny` follows;
// run under `rocprofv3 --kernel-trace` and read tiny's start minus writer's end (tools/probes/gap_summary.py).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ __launch_bounds__(256) void writer(unsigned* out, unsigned n16, unsigned seed) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, n16 * 16u, 0x00020000);
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) {
    const v4u v = {i ^ seed, i + seed, i * 3u, seed};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, i * 16u, 0, AUX);
  }
}
__global__ void tiny(unsigned* flag) {
  if (threadIdx.x == 0) flag[0] += 1;
}
// a persistent-kernel-shaped launch: 256 blocks x 512 threads, LDS bytes per block set by the template, a short
// busy loop, one store per thread
template <int LDSB>
__global__ __launch_bounds__(512) void fat(unsigned* out, int iters) {
  __shared__ unsigned sm[LDSB / 4];
  unsigned v = threadIdx.x;
  sm[threadIdx.x % (LDSB / 4)] = v;
  __syncthreads();
  for (int i = 0; i < iters; ++i) v = v * 1664525u + sm[(v + i) % (LDSB / 4)];
  out[blockIdx.x * 512 + threadIdx.x] = v;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  unsigned* buf = nullptr;
  unsigned* flag = nullptr;
  const size_t maxmb = 1024;
  if (hipMalloc(&buf, maxmb << 20) != hipSuccess || hipMalloc(&flag, 256) != hipSuccess) return 1;
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) return 1;
  const int sizes[] = {0, 4, 16, 64, 256, 1024};
  for (int r = 0; r < reps; ++r)
    for (int mb : sizes) {
      const unsigned n16 = (unsigned)(((size_t)mb << 20) / 16);
      const dim3 g(2048), b(256);
      hipLaunchKernelGGL(writer<0>, g, b, 0, s, buf, n16, 1u);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, flag);
      hipLaunchKernelGGL(writer<2>, g, b, 0, s, buf, n16, 2u);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, flag);
      hipLaunchKernelGGL(writer<16>, g, b, 0, s, buf, n16, 3u);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, flag);
      hipLaunchKernelGGL(writer<17>, g, b, 0, s, buf, n16, 4u);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, flag);
      hipLaunchKernelGGL(writer<19>, g, b, 0, s, buf, n16, 5u);
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, flag);
      if (hipStreamSynchronize(s) != hipSuccess) return 2;
      printf("rep %d mb %d done\n", r, mb);
    }
  // fat -> fat pairs: LDS 4 KB and 160 KB per block (one block per CU), ~50 us each
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(fat<4096>, dim3(256), dim3(512), 0, s, buf, 20000);
    hipLaunchKernelGGL(fat<4096>, dim3(256), dim3(512), 0, s, buf, 20000);
    hipLaunchKernelGGL(fat<163840>, dim3(256), dim3(512), 0, s, buf, 20000);
    hipLaunchKernelGGL(fat<163840>, dim3(256), dim3(512), 0, s, buf, 20000);
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, flag);
    hipLaunchKernelGGL(fat<163840>, dim3(256), dim3(512), 0, s, buf, 20000);
    hipLaunchKernelGGL(writer<0>, dim3(2048), dim3(256), 0, s, buf, (unsigned)((256u << 20) / 16), 9u);
    hipLaunchKernelGGL(fat<163840>, dim3(256), dim3(512), 0, s, buf, 20000);
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
  }
  hipFree(buf);
  hipFree(flag);
  return 0;
}
