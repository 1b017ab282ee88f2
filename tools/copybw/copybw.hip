// copybw.hip -- measurement aid for bench.py (not product code): HBM copy
// kernels, 16 B per lane.  bench.py reports the fastest form's rate as the
// measured copy ceiling next to the aggregate kernel's roofline fraction
// (MI355X_MICROARCH.md lists 6.29 TB/s for a float4 copy).
//   mode 0: grid-stride, 2048 x 256 threads, 4 loads in flight per lane
//   mode 1: one element per thread (a grid of n/256 workgroups), plain loads
//   mode 2: as 1 with nontemporal loads
//   mode 3: as 0 with nontemporal loads
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_stride(const u32x4* __restrict__ src,
                                                   u32x4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const u32x4 a = ld<NT>(src + i), b = ld<NT>(src + i + stride),
                c = ld<NT>(src + i + 2 * stride), d = ld<NT>(src + i + 3 * stride);
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = ld<NT>(src + i);
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_flat(const u32x4* __restrict__ src,
                                                 u32x4* __restrict__ dst, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = ld<NT>(src + i);
}

extern "C" int copybw_copy_mode(void* dst, const void* src, size_t bytes, int mode,
                                void* stream) {
  const size_t n = bytes / 16;
  const hipStream_t s = (hipStream_t)stream;
  const dim3 flat((unsigned)((n + 255) / 256)), grid(2048), blk(256);
  switch (mode) {
    case 0: hipLaunchKernelGGL(copy_stride<false>, grid, blk, 0, s, (const u32x4*)src, (u32x4*)dst, n); break;
    case 1: hipLaunchKernelGGL(copy_flat<false>, flat, blk, 0, s, (const u32x4*)src, (u32x4*)dst, n); break;
    case 2: hipLaunchKernelGGL(copy_flat<true>, flat, blk, 0, s, (const u32x4*)src, (u32x4*)dst, n); break;
    case 3: hipLaunchKernelGGL(copy_stride<true>, grid, blk, 0, s, (const u32x4*)src, (u32x4*)dst, n); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// the form bench.py reports (the fastest measured: flat, nontemporal loads)
extern "C" int copybw_copy(void* dst, const void* src, size_t bytes, void* stream) {
  return copybw_copy_mode(dst, src, bytes, 2, stream);
}
