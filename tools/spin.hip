// Contention probe helper (tools/contention_probe.py): a kernel whose blocks only sleep, each holding 96 KiB
// of LDS (one per CU, and no persistent conv block fits beside it), to stand in for the RCCL blocks that occupy CUs while the data-parallel step runs. Not part
// of the product library. Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/libspin.so tools/spin.hip
#include <hip/hip_runtime.h>

extern "C" __global__ void spin_kernel(int iters) {
  extern __shared__ char lds[];
  if (threadIdx.x == 0) lds[0] = 0;
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
}

extern "C" int spin_launch(int blocks, int iters, int lds_bytes, void* stream) {
  if (hipFuncSetAttribute((const void*)spin_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), lds_bytes, (hipStream_t)stream, iters);
  return (int)hipGetLastError();
}
