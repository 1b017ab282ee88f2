// MEASUREMENT AID (not product code): bandwidth of a kernel that reads or
// writes pinned host memory directly over PCIe (zero-copy), against
// hipMemcpyAsync, to size a fused staging path.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                              size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    d[i] = __builtin_nontemporal_load(s + i);
}

extern "C" int hostbw_copy(const void* src, void* dst, size_t bytes, int blocks, void* stream) {
  hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src,
                     (u32x4*)dst, bytes / 16);
  return (int)hipGetLastError();
}
