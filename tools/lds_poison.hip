// Diagnostic (tools/lds_poison_bisect.py): fill LDS words [begin, end) of every CU with `pattern` and
// the rest with zero, so the next kernel's workgroups start on it.  Vector (ds_write) stores only.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void lds_poison_range_kernel(uint32_t pattern, int begin, int end) {
  extern __shared__ uint32_t lds_words[];
  for (int i = threadIdx.x; i < 163840 / 4; i += 256) lds_words[i] = (i >= begin && i < end) ? pattern : 0u;
  __syncthreads();
}

extern "C" int lds_poison_range(uint32_t pattern, int begin, int end) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  if (hipFuncSetAttribute((const void*)lds_poison_range_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840) !=
      hipSuccess)
    return -1;
  hipLaunchKernelGGL(lds_poison_range_kernel, dim3(8 * cus), dim3(256), 163840, 0, pattern, begin, end);
  if (hipGetLastError() != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
