// psg_darling.hip -- the server's model update fused onto the resident
// aggregate: Darling::updateWeight (src/linear_method/darling.cc:437-477),
// run by the server on received(time) = (G, U) of a feature block
// (darling.cc:251-262).
//
// For server position k = lo + i of channel `grp` with active_set bit k set:
//   g = G[i], u = U[i] / eta + 1e-10, g_pos = g + lambda, g_neg = g - lambda
//   d = -w, vio = 0
//   if w == 0:  g_pos < 0 -> vio = -g_pos;  else g_neg > 0 -> vio = g_neg;
//               else g_pos > T && g_neg < -T -> clear bit k, w = NaN(all
//               ones, darling.cc:13-15), next k
//   violation = max(violation, vio)
//   if g_pos <= u*w: d = -g_pos/u;  else if g_neg >= u*w: d = -g_neg/u
//   d = min(delta[k], max(-delta[k], d));  delta[k] = newDelta(d) =
//   min(delta_max, 2|d| + .1) (darling.h:31-33);  w += d
// f64 throughout, IEEE ops in the reference's order (the library is built
// with -ffp-contract=off: no fused multiply-adds), std::min/std::max as the
// ternaries they are -- bit-exact with the CPU.
//
// Layout: one lane per server position; a wave covers 64 positions = two
// words of the active-set bitmap (bit k of word k/32), aligned to words,
// so the new bits leave by one ballot and two 32-bit stores, no atomics.
// The violation is a max on the bit pattern (every vio is a non-negative
// double, so its bits order like its value): a wave max, a max over the
// workgroup's four waves, one atomic max into one of kVioSlots slots (one
// per 64-B line, picked by workgroup), then a one-workgroup pass folds the
// slots and re-zeroes them. A single address took every wave's atomic
// before: on the first update of a model (w = 0, so most positions
// violate) 262,144 atomics serialised at one L2 channel, 2.98 ms against
// 0.133 ms for a later update of the same 16.8 M positions (r05 trace).  HBM-bound: 8 (G) + 8 (U) + 2x8 (w) + 2x8 (delta) bytes
// per position plus the bitmap.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_internal.h"

namespace psg {

namespace {

__device__ __forceinline__ double dmin(double a, double b) { return b < a ? b : a; }  // std::min
__device__ __forceinline__ double dmax(double a, double b) { return a < b ? b : a; }  // std::max

__device__ __forceinline__ unsigned long long wave_max(unsigned long long v) {
  for (int s = 32; s >= 1; s >>= 1) {
    const unsigned long long o = (unsigned long long)__shfl_xor((long long)v, s, 64);
    v = o > v ? o : v;
  }
  return v;
}

__global__ __launch_bounds__(256) void darling_kernel(const double* __restrict__ G,
                                                      const double* __restrict__ U,
                                                      double* __restrict__ w,
                                                      double* __restrict__ delta,
                                                      uint32_t* __restrict__ active,
                                                      uint64_t lo, uint64_t n, DarlingParam P,
                                                      const unsigned long long* __restrict__ bad,
                                                      unsigned long long* __restrict__ slots) {
  if (*bad) return;  // a push of this block failed to match: the reference aborted
  const uint64_t base = lo & ~31ull;
  const uint64_t k = base + ((uint64_t)blockIdx.x * 256u + threadIdx.x);
  const int lane = threadIdx.x & 63;
  const bool in = k >= lo && k < lo + n;
  const uint64_t end = lo + n;
  const bool wordok = (k >> 5) <= ((end - 1) >> 5);  // word inside the range's words
  uint32_t word = 0;
  if (wordok) word = active[k >> 5];
  bool bit = (word >> (k & 31)) & 1u;
  double vio = 0;
  if (in && bit) {
    const uint64_t i = k - lo;
    const double g = G[i], u = U[i] / P.eta + 1e-10;
    const double g_pos = g + P.lambda, g_neg = g - P.lambda;
    double wk = w[k];
    double d = -wk;
    bool inactive = false;
    if (wk == 0) {
      if (g_pos < 0) {
        vio = -g_pos;
      } else if (g_neg > 0) {
        vio = g_neg;
      } else if (g_pos > P.kkt && g_neg < -P.kkt) {
        inactive = true;
      }
    }
    if (inactive) {
      bit = false;
      w[k] = __longlong_as_double((long long)~0ull);  // kInactiveValue_
    } else {
      if (g_pos <= u * wk) {
        d = -g_pos / u;
      } else if (g_neg >= u * wk) {
        d = -g_neg / u;
      }
      const double dk = delta[k];
      d = dmin(dk, dmax(-dk, d));
      delta[k] = dmin(P.delta_max, 2 * fabs(d) + .1);
      wk += d;
      w[k] = wk;
    }
  }
  // new bitmap words: lanes 0 and 32 store the two words of this wave
  const unsigned long long m = __ballot(bit);
  if ((lane & 31) == 0 && wordok) {
    const uint32_t nw = (uint32_t)(m >> lane);
    if (nw != word) active[k >> 5] = nw;
  }
  // violation: max over the wave, the workgroup, then one atomic per workgroup
  unsigned long long vb = wave_max((unsigned long long)__double_as_longlong(vio));
  __shared__ unsigned long long wmax[4];
  if (lane == 0) wmax[threadIdx.x >> 6] = vb;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) vb = wmax[i] > vb ? wmax[i] : vb;
    if (vb)
      __hip_atomic_fetch_max(slots + (blockIdx.x % kVioSlots) * 8, vb, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the slots' max into *vio; the slots back to zero for the next update
__global__ __launch_bounds__(kVioSlots) void darling_vio_kernel(unsigned long long* __restrict__ slots,
                                                                unsigned long long* __restrict__ vio) {
  unsigned long long vb = slots[threadIdx.x * 8];
  slots[threadIdx.x * 8] = 0;
  vb = wave_max(vb);
  __shared__ unsigned long long wmax[kVioSlots / 64];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = vb;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kVioSlots / 64; ++i) vb = wmax[i] > vb ? wmax[i] : vb;
    *vio = vb;
  }
}

__global__ __launch_bounds__(256) void bitmap_fill_kernel(uint32_t* __restrict__ a, uint64_t nbits) {
  const uint64_t wi = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint64_t nw = (nbits + 31) >> 5;
  if (wi >= nw) return;
  const uint64_t left = nbits - wi * 32;
  a[wi] = left >= 32 ? 0xffffffffu : ((1u << left) - 1u);
}

__global__ __launch_bounds__(256) void fill_f64_kernel(double* __restrict__ a, uint64_t n, double v) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i < n) a[i] = v;
}

__global__ __launch_bounds__(256) void popcount_kernel(const uint32_t* __restrict__ a, uint64_t nw,
                                                       unsigned long long* __restrict__ out) {
  const uint64_t wi = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  unsigned long long c = wi < nw ? (unsigned long long)__popc(a[wi]) : 0ull;
  for (int s = 32; s >= 1; s >>= 1) c += (unsigned long long)__shfl_xor((long long)c, s, 64);
  if ((threadIdx.x & 63) == 0 && c)
    __hip_atomic_fetch_add(out, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

hipError_t launch_darling(const double* G, const double* U, double* w, double* delta,
                          uint32_t* active, uint64_t lo, uint64_t n, const DarlingParam& P,
                          const unsigned long long* bad, unsigned long long* slots,
                          unsigned long long* vio, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(vio, 0, 8, s);
  const uint64_t span = lo + n - (lo & ~31ull);
  const uint64_t blocks = (span + 255) / 256;
  hipLaunchKernelGGL(darling_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, G, U, w, delta,
                     active, lo, n, P, bad, slots);
  hipLaunchKernelGGL(darling_vio_kernel, dim3(1), dim3(kVioSlots), 0, s, slots, vio);
  return hipGetLastError();
}

hipError_t launch_darling_init(double* delta, uint32_t* active, uint64_t n, double delta_init,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill_f64_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, delta,
                     n, delta_init);
  return launch_bitmap_fill(active, n, s);
}

hipError_t launch_bitmap_fill(uint32_t* active, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t nw = (n + 31) / 32;
  hipLaunchKernelGGL(bitmap_fill_kernel, dim3((uint32_t)((nw + 255) / 256)), dim3(256), 0, s,
                     active, n);
  return hipGetLastError();
}

hipError_t launch_popcount(const uint32_t* a, uint64_t nw, unsigned long long* out, hipStream_t s) {
  if (nw == 0) return hipSuccess;
  hipLaunchKernelGGL(popcount_kernel, dim3((uint32_t)((nw + 255) / 256)), dim3(256), 0, s, a, nw,
                     out);
  return hipGetLastError();
}

}  // namespace psg
