// psg_device.h -- device helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psg {
namespace dev {

// ----------------------------------------------------------------------
// wave-cooperative k-ary search: first index i in [0, n) whose key
// satisfies (upper ? S[i] > key : S[i] >= key); n if none.  64 probes per
// round -> ceil(log64 n)+1 dependent global loads instead of log2 n.
// Every lane of the wave must call it with the same arguments.
// ----------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_search(const uint64_t* __restrict__ S,
                                                uint64_t n, uint64_t key,
                                                bool upper, int lane) {
  uint64_t lo = 0, hi = n;  // answer in [lo, hi]
  while (hi > lo) {
    const uint64_t len = hi - lo;
    const uint64_t step = (len + 63) >> 6;
    const uint64_t idx = lo + (uint64_t)(lane + 1) * step - 1;
    bool pred = true;  // probes past the range count as "true"
    if (idx < hi) {
      const uint64_t s = S[idx];
      pred = upper ? (s > key) : (s >= key);
    }
    const unsigned long long mask = __ballot(pred);
    if (mask == 0) {
      lo = hi;
      break;
    }
    const uint64_t f = (uint64_t)(__ffsll((long long)mask) - 1);
    const uint64_t nlo = lo + f * step;
    uint64_t nhi = lo + (f + 1) * step - 1;
    if (nhi > hi) nhi = hi;
    lo = nlo;
    hi = nhi;
  }
  return lo;
}

// lower_bound(S, xl) inside a bracket with S[a] < xl <= S[c]: interpolation
// probes (pushes of murmur-hashed keys are near-uniform), bisection, then
// the last <= 15 candidates in one round trip.  One lane per search.
__device__ __forceinline__ uint64_t bracket_lower_bound(const uint64_t* S, uint64_t xl,
                                                        uint64_t a, uint64_t c, uint64_t ka,
                                                        uint64_t kc) {
  for (int it = 0; it < 6 && c - a > 16u; ++it) {
    const double f = (double)(xl - ka) / (double)(kc - ka);
    uint64_t mid = a + 1 + (uint64_t)(f * (double)(c - a - 1));
    mid = mid < c ? mid : c - 1;
    const uint64_t km = S[mid];
    if (km < xl) {
      a = mid;
      ka = km;
    } else {
      c = mid;
      kc = km;
    }
  }
  while (c - a > 16u) {
    const uint64_t mid = a + ((c - a) >> 1);
    if (S[mid] < xl) a = mid; else c = mid;
  }
  // independent loads of S[a+1 .. c-1] (indices clamped to c, where
  // S[c] >= xl counts 0)
  uint32_t below = 0;
#pragma unroll
  for (uint32_t i = 1; i < 16u; ++i) {
    const uint64_t idx = a + i < c ? a + i : c;
    below += S[idx] < xl ? 1u : 0u;
  }
  return a + 1u + below;
}

// lower_bound(S[0, n), x) by bracket_lower_bound: in [0, n] whatever S holds
__device__ __forceinline__ uint64_t interp_lower_bound(const uint64_t* S, uint64_t n, uint64_t x) {
  if (n == 0) return 0;
  const uint64_t k0 = S[0], kn = S[n - 1];
  if (x <= k0) return 0;
  if (x > kn) return n;
  return bracket_lower_bound(S, x, 0, n - 1, k0, kn);
}

// lower_bound over a sorted LDS array of n <= 2*TILE-1 keys: fixed trip
// count (log2(TILE)+1 probes), so the wave never diverges on the loop.
template <int TILE>
__device__ __forceinline__ int lds_lower_bound(const uint64_t* a, int n,
                                               uint64_t k) {
  int pos = 0;
#pragma unroll
  for (int step = TILE; step > 0; step >>= 1) {
    const int c = pos + step;
    if (c <= n && a[c - 1] < k) pos = c;
  }
  return pos;
}

__device__ __forceinline__ uint64_t gl_lower_bound(const uint64_t* __restrict__ a,
                                                   uint64_t n, uint64_t k) {
  uint64_t lo = 0, len = n;
  while (len > 0) {
    const uint64_t half = len >> 1;
    if (a[lo + half] < k) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo;
}

// Exclusive scan across an NT-thread workgroup.  wsum: LDS scratch of NT/64
// words.  Contains two barriers; callers separate consecutive uses with a
// barrier of their own.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum,
                                                    uint32_t* total) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  constexpr int kW = NT / 64;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    uint32_t s = lane < kW ? wsum[lane] : 0u;
#pragma unroll
    for (int d = 1; d < kW; d <<= 1) {
      const uint32_t y = __shfl_up(s, d, 64);
      if (lane >= d) s += y;
    }
    if (lane < kW) wsum[lane] = s;
  }
  __syncthreads();
  *total = wsum[kW - 1];
  return (w > 0 ? wsum[w - 1] : 0u) + x - v;
}

// Scale of the tile kernels' bucket map bucket(x) = umulhi(x, mul): every
// x <= r32 (< 2^32) lands below nb.  An f32 reciprocal with a 2^-20 margin
// (reciprocal ~2^-23, conversions and products 2^-24 each) replaces the
// 64-bit integer division floor(nb * 2^32 / (r32 + 1)), which compiles to a
// ~100-instruction scalar routine in every wave; only the spread of keys over
// buckets depends on the exact value, not what a search finds.
__device__ __forceinline__ uint32_t bucket_scale(uint64_t r32, uint32_t nb) {
  const float f = (float)nb * 4294967296.0f * (1.0f - 0x1p-20f) *
                  __builtin_amdgcn_rcpf((float)(r32 + 1ull));
  return f >= 4294967295.0f ? 0xffffffffu : (uint32_t)f;
}

// One step of the per-key fold in push-arrival order.  p = push index in
// this launch, lp = last push index in this launch that held the key (-1:
// none yet).  Serial (the reference default) adds +0.0 for every absent
// later push (kv_vector.h:200); since x + 0.0 == x except -0.0 -> +0.0 and
// the operation is idempotent, one "+ 0" per run of absent pushes is exact.
template <typename V>
__device__ __forceinline__ V fold_step(V acc, int lp, int p, V v,
                                       bool parallel, bool cont) {
  if (p == 0 && !cont) return v;  // the first push is assigned (:195-196)
  if (!parallel) {
    const bool gap = (lp >= 0) ? (p - lp > 1) : (cont && p > 0);
    if (gap) acc = acc + V(0);
  }
  return acc + v;
}


}  // namespace dev
}  // namespace psg
