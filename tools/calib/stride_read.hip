// Sampled-read calibration (not product code): how long does it take to read
// ONE 8-B key per S bytes of a 1 GB array, against reading all of it?  If the
// memory side fetches whole 128-B lines, a 1-in-16 key sample (S = 128) costs
// as much as the full read; with 64-B sectors it costs half.  This decides
// whether a partition that samples every 16th push key can be cheaper than
// the stream partition that reads every key (psg_partition.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void sampled(const uint64_t* __restrict__ p, size_t nsamp, size_t step, unsigned* sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsamp; i += stride)
    acc ^= __builtin_nontemporal_load(p + i * step);
  if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (unsigned)acc;
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
__global__ void full(const u64x2* __restrict__ p, size_t n, unsigned* sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64x2 v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (unsigned)acc;
}

int main() {
  const size_t bytes = 1ull << 30;
  uint64_t* p;
  unsigned* sink;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  hipMemset(p, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const dim3 g(256 * 32), blk(256);
  auto run = [&](const char* name, size_t step) {
    float best = 1e9f;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a, 0);
      if (step == 0)
        hipLaunchKernelGGL(full, g, blk, 0, 0, (const u64x2*)p, bytes / 16, sink);
      else
        hipLaunchKernelGGL(sampled, g, blk, 0, 0, p, bytes / (8 * step), step, sink);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep > 0 && ms < best) best = ms;
    }
    printf("%-10s stride %5zu B: %.4f ms  (%.2f TB/s of the array)\n", name, step ? step * 8 : 16,
           best, bytes / (best * 1e-3) / 1e12);
  };
  run("full", 0);
  for (size_t s : {1, 2, 4, 8, 16, 32, 64}) run("sampled", s);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
