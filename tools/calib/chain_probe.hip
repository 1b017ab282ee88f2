// Dependent-load latency in the snappy table walk's pattern (not product
// code): one wave walks a 512 KB buffer by dependent 64-byte windows (one
// byte per lane, the next window ~3 KB on, its position depending on a byte
// of the current one, as a literal's length does), after waves 1-3 did or
// did not pull the buffer into L2 first.  Prints clocks per dependent load.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define AS1 __attribute__((address_space(1)))

__global__ __launch_bounds__(256) void chain(const uint8_t* __restrict__ buf, uint32_t n,
                                             int prefetch, int steps, unsigned long long* out) {
  const AS1 uint8_t* s0 = (const AS1 uint8_t*)buf;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  if (w > 0 && prefetch) {
    uint32_t acc = 0;
    for (uint32_t x0 = (tid - 64u) * 128u; x0 < n; x0 += 8u * 192u * 128u) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t x = x0 + (uint32_t)k * 192u * 128u;
        v[k] = x < n ? (uint32_t)s0[x] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc ^= v[k];
    }
    asm volatile("" ::"v"(acc));
  }
  __syncthreads();
  if (w != 0) return;
  uint32_t q = 0;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < steps; ++i) {
    const uint32_t la = q + lane < n ? (uint32_t)s0[q + lane] : 0u;
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)la, 5);
    q = (q + 3000u + (b & 1u)) % (n - 64u);
  }
  const unsigned long long t1 = clock64();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = q;
  }
}

int main() {
  const uint32_t n = 512u << 10;
  uint8_t* buf;
  unsigned long long* out;
  hipMalloc(&buf, n);
  hipMalloc(&out, 16);
  hipMemset(buf, 7, n);
  unsigned long long h[2];
  for (int pf = 0; pf < 2; ++pf)
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(chain, dim3(1), dim3(256), 0, 0, buf, n, pf, 170, out);
      hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
      printf("prefetch %d rep %d: %.0f clocks per dependent window load\n", pf, rep,
             (double)h[0] / 170.0);
    }
  return 0;
}
