// psg_stream3.hip -- streaming aggregate kernel v8 (the default): v7's
// one-wave-per-coarse-range structure with the slot searches of a batch of
// pushes interleaved.
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267); see psg_stream2.hip for the fold rules.
//
// Why v8: v7 measured latency-bound on each wave's own dependency chain
// (DESIGN.md §4.2): per window a bucket read, 3-4 dependent LDS probes and
// the accumulator read-modify-write, window after window.  Only the fold has
// to respect push order; the searches do not.  v8 therefore runs the searches
// of NPW windows level by level together (NPW independent LDS chains in
// flight per wave), then folds the windows in push order.  A push whose
// window was entirely inside the tile continues (sequentially) before the
// next push folds, so the per-slot fold order is still the arrival order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "psg_device.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))

namespace psg {

namespace {

constexpr int kFT = 256;  // fine tile slots (4 per lane)

template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}
template <typename T>
__device__ __forceinline__ AS1 T* GW(T* p) {
  return (AS1 T*)p;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// lower_bound of k in a[off, off+N) (N a power of two; a padded past the end)
template <int N>
__device__ __forceinline__ uint32_t lb_pow2(const uint64_t* a, uint32_t off, uint64_t k) {
  const char* ab = (const char*)a;
  uint32_t o = off * 8;
#pragma unroll
  for (int step = N / 2; step > 0; step >>= 1) {
    const uint64_t v = *(const uint64_t*)(ab + o + 8 * (step - 1));
    o = (v < k) ? o + 8 * step : o;
  }
  const uint64_t v = *(const uint64_t*)(ab + o);
  o = (v < k) ? o + 8 : o;
  return o >> 3;
}

template <typename V>
__device__ __forceinline__ V fold1(V acc, int lp, int p, V v, bool parallel, bool cont) {
  const bool gap = !parallel && ((lp >= 0) ? (p - lp > 1) : (cont && p > 0));
  const V a1 = gap ? acc + V(0) : acc;
  return (p == 0 && !cont) ? v : a1 + v;
}

// NPW: windows (pushes) per batch; WPS: waves per SIMD; LNB: log2 buckets
// per fine tile; PR: first windows sized by the push's expected share.
template <typename V, int M, int NPW, int WPS, int LNB, int PR>
__global__ __launch_bounds__(64, WPS) void stream3_kernel(const TileDesc* __restrict__ tiles) {
  constexpr int kNB = 1 << LNB;
  __shared__ __attribute__((aligned(16))) uint64_t dk[kFT + 16];
  __shared__ V acc[M * kFT];
  __shared__ int16_t lastl[kFT];
  __shared__ uint32_t btab[kNB + 1];

  const int lane = threadIdx.x;
  const TileDesc T = tiles[blockIdx.x];
  const uint32_t np = T.np;  // <= 64 (host guarantees)
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  const uint32_t ncs = T.nt;
  const uint32_t nft = (ncs + kFT - 1) / kFT;
  const uint64_t* Dg = T.dk;

  // lane p: push p's cursor, coarse end, key/value pointers, window size
  uint32_t cur = 0, cend = 0, pred = 64;
  uint64_t kp = 0;
  uint64_t vp[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) vp[mi] = 0;
  if ((uint32_t)lane < np) {
    cur = G(T.seg)[lane];
    cend = G(T.seg)[np + lane];
    kp = (uint64_t)G(T.pkeys)[lane];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) vp[mi] = (uint64_t)G(T.pvals)[(size_t)lane * M + mi];
    if (PR && ncs > 0) {
      const float mu = (float)(cend - cur) * (float)kFT / (float)ncs;
      const float w = mu + 2.0f * __builtin_sqrtf(mu) + 4.0f;
      pred = w >= 64.0f ? 64u : (uint32_t)w + 1u;
    }
  }
  if (lane < 16) dk[kFT + lane] = ~0ull;
  V* outb[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) outb[mi] = (V*)G(T.out)[mi] + T.slot0;
  // retire the set-up loads here (see psg_stream2.hip)
  __builtin_amdgcn_s_waitcnt(0);

  // window of push p at its cursor: W keys; lanes past the coarse end hold ~0
  auto load_window = [&](uint64_t& wk, V (&wv)[M], uint32_t p, uint32_t W) {
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(cur, p);
    const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(cend, p);
    const uint32_t n = e - c < W ? e - c : W;
    const uint64_t* sk = (const uint64_t*)readlane64(kp, p);
    const bool act = (uint32_t)lane < n;
    wk = act ? G(sk)[c + lane] : ~0ull;
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      const V* sv = (const V*)readlane64(vp[mi], p);
      wv[mi] = act ? G(sv)[c + lane] : V(0);
    }
  };
  auto first_w = [&](uint32_t p) -> uint32_t {
    return PR ? (uint32_t)__builtin_amdgcn_readlane(pred, p) : 64u;
  };

  for (uint32_t ft = 0; ft < nft; ++ft) {
    const uint32_t base = ft * kFT;
    const int nt = (int)(ncs - base < (uint32_t)kFT ? ncs - base : (uint32_t)kFT);
    const bool last_tile = ft + 1 == nft;

    // ---- one round trip: D keys, bound, first batch of windows
    uint64_t dreg[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = base + (uint32_t)lane + 64u * k;
      dreg[k] = i < ncs ? G(Dg)[i] : ~0ull;
    }
    const uint64_t bound = last_tile ? ~0ull : G(Dg)[base + kFT];
    uint64_t wk[NPW];
    V wv[NPW][M];
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      if ((uint32_t)q < np) load_window(wk[q], wv[q], q, first_w(q));
      else wk[q] = ~0ull;
    }

    // ---- install the tile: D, accumulators, bucket table
#pragma unroll
    for (int k = 0; k < 4; ++k) dk[lane + 64 * k] = dreg[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = lane * 4 + j;
      lastl[s] = -1;
#pragma unroll
      for (int mi = 0; mi < M; ++mi)
        acc[mi * kFT + s] = (cont && s < nt) ? G(outb[mi] + base)[s] : V(0);
    }
    __syncthreads();
    const uint64_t klo =
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)dreg[0]) |
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(dreg[0] >> 32)) << 32);
    const uint64_t range = dk[nt - 1] - klo;
    const int bits = range ? 64 - __builtin_clzll(range) : 0;
    const int shift = bits > LNB ? bits - LNB : 0;
    // btab[b] = first slot whose key >= klo + (b << shift)
#pragma unroll
    for (int r = 0; r < kNB / 64; ++r) {
      const uint64_t d = (uint64_t)(lane + 64 * r) << shift;
      const uint64_t key = d > ~0ull - klo ? ~0ull : klo + d;
      const uint32_t sb = lb_pow2<kFT>(dk, 0, key);
      btab[lane + 64 * r] = sb < (uint32_t)nt ? sb : (uint32_t)nt;
    }
    if (lane == 0) btab[kNB] = (uint32_t)nt;
    __syncthreads();

    // window's in-tile prefix (sorted pushes: a ballot against the bound)
    auto in_tile = [&](uint64_t key, uint32_t p, uint32_t W) -> uint32_t {
      bool inb;
      if (last_tile) {  // the rest of the coarse range: every loaded key
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(cur, p);
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(cend, p);
        inb = (uint32_t)lane < (e - c < W ? e - c : W);
      } else {
        inb = key < bound;
      }
      const unsigned long long bal = __ballot(inb);
      return (~bal == 0ull) ? 64u : (uint32_t)__builtin_ctzll(~bal);
    };
    auto bucket = [&](uint64_t k) -> uint32_t {
      const uint64_t dlt = k - klo;
      return (k < klo) ? 0u
             : (dlt >> shift) < (uint64_t)kNB ? (uint32_t)(dlt >> shift)
                                              : (uint32_t)kNB;
    };
    // order check, fold (push order), carry, failures, cursor
    auto fold_window = [&](uint64_t k, const V (&val)[M], uint32_t pos, bool found, uint32_t Lq,
                           uint32_t p, int& carry, uint32_t& fails) {
      const bool act = (uint32_t)lane < Lq;
      const uint32_t prev_in = __shfl_up(pos, 1, 64);
      const int prev = lane == 0 ? carry : (int)prev_in;
      const bool ok = act && (int)pos < nt && found && prev < (int)pos;
      if (ok) {
        const int lp = lastl[pos];
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          acc[mi * kFT + pos] = fold1<V>(acc[mi * kFT + pos], lp, (int)p, val[mi], parallel, cont);
        lastl[pos] = (int16_t)p;
      }
      if (Lq > 0) carry = (int)__shfl(pos, (int)Lq - 1, 64);
      fails += (uint32_t)__popcll(__ballot(act && !ok));
      if (lane == (int)p) cur += Lq;
      (void)k;
    };
    // one window alone (continuations): search then fold
    auto process1 = [&](uint64_t key, const V (&val)[M], uint32_t p, uint32_t W, int& carry,
                        uint32_t& fails) -> uint32_t {
      const uint32_t Lq = in_tile(key, p, W);
      const uint64_t k = (uint32_t)lane < Lq ? key : ~0ull;
      const uint32_t b = bucket(k);
      const uint32_t lo = btab[b], hi = btab[b < (uint32_t)kNB ? b + 1 : b];
      uint32_t pos;
      bool found;
      if (hi - lo <= 8u) {
        const uint64_t v0 = dk[lo], v4 = dk[lo + 4];
        uint32_t j = v4 <= k ? lo + 4 : lo;
        found = v0 == k || v4 == k;
        const uint64_t v2 = dk[j + 2];
        j = v2 <= k ? j + 2 : j;
        const uint64_t v1 = dk[j + 1];
        j = v1 <= k ? j + 1 : j;
        found = found || v2 == k || v1 == k;
        pos = j;
      } else {
        pos = lb_pow2<kFT>(dk, 0, k);
        found = dk[pos] == k;
      }
      fold_window(k, val, pos, found, Lq, p, carry, fails);
      return Lq;
    };
    auto rest = [&](uint32_t p, uint32_t Lq, uint32_t W, int& carry, uint32_t& fails) {
      while (Lq == W) {
        uint64_t k2;
        V v2[M];
        load_window(k2, v2, p, 64u);
        Lq = process1(k2, v2, p, 64u, carry, fails);
        W = 64u;
      }
    };
    auto flush_fails = [&](uint32_t p, uint32_t fails) {
      if (fails && lane == 0)
        __hip_atomic_fetch_add(GW(T.fail) + p, (unsigned long long)fails, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };

    // ---- a batch of NPW windows: searches level by level, folds in order.
    // Candidates lo..lo+7 of a narrow bucket: last key <= k by lifting
    // (reads {lo, lo+4}, then j+2, then j+1); found iff some read == k.
    auto batch = [&](uint32_t b0) {
      uint32_t Lq[NPW], pos[NPW], lo[NPW], hi[NPW];
      uint64_t kk[NPW];
      bool fnd[NPW];
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        const bool live = b0 + q < np;
        Lq[q] = live ? in_tile(wk[q], b0 + q, first_w(b0 + q)) : 0u;
        kk[q] = (uint32_t)lane < Lq[q] ? wk[q] : ~0ull;
        const uint32_t b = bucket(kk[q]);
        lo[q] = btab[b];
        hi[q] = btab[b < (uint32_t)kNB ? b + 1 : b];
      }
      uint64_t v0[NPW], v4[NPW];
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        v0[q] = dk[lo[q]];
        v4[q] = dk[lo[q] + 4];
      }
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        pos[q] = v4[q] <= kk[q] ? lo[q] + 4 : lo[q];
        fnd[q] = v0[q] == kk[q] || v4[q] == kk[q];
      }
      uint64_t v2[NPW];
#pragma unroll
      for (int q = 0; q < NPW; ++q) v2[q] = dk[pos[q] + 2];
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        pos[q] = v2[q] <= kk[q] ? pos[q] + 2 : pos[q];
        fnd[q] = fnd[q] || v2[q] == kk[q];
      }
      uint64_t v1[NPW];
#pragma unroll
      for (int q = 0; q < NPW; ++q) v1[q] = dk[pos[q] + 1];
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        pos[q] = v1[q] <= kk[q] ? pos[q] + 1 : pos[q];
        fnd[q] = fnd[q] || v1[q] == kk[q];
        if (hi[q] - lo[q] > 8u) {  // rare: a crowded bucket, full search
          pos[q] = lb_pow2<kFT>(dk, 0, kk[q]);
          fnd[q] = dk[pos[q]] == kk[q];
        }
      }
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        if (b0 + q < np) {
          int carry = -1;
          uint32_t fails = 0;
          fold_window(kk[q], wv[q], pos[q], fnd[q], Lq[q], b0 + q, carry, fails);
          rest(b0 + q, Lq[q], first_w(b0 + q), carry, fails);
          flush_fails(b0 + q, fails);
        }
      }
    };

    batch(0);
    for (uint32_t b0 = NPW; b0 < np; b0 += NPW) {
#pragma unroll
      for (int q = 0; q < NPW; ++q)
        if (b0 + q < np) load_window(wk[q], wv[q], b0 + q, first_w(b0 + q));
      batch(b0);
    }
    __syncthreads();

    // ---- trailing absent pushes (serial: one "+ 0.0"), store 4 slots/lane
    {
      const int s0 = lane * 4;
      V res[M][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int lp = lastl[s0 + j];
        const bool gap = !parallel && ((lp >= 0) ? (lp < (int)np - 1) : (cont && np > 0));
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          const V a = acc[mi * kFT + s0 + j];
          res[mi][j] = gap ? a + V(0) : a;
        }
      }
      if (s0 + 4 <= nt) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          V* o = outb[mi] + base + s0;
          if ((reinterpret_cast<uintptr_t>(o) & 15u) == 0u) {
            if constexpr (sizeof(V) == 4) {
              typedef float f4 __attribute__((ext_vector_type(4)));
              const f4 w = {res[mi][0], res[mi][1], res[mi][2], res[mi][3]};
              *(AS1 f4*)GW(o) = w;
            } else {
              typedef double d2 __attribute__((ext_vector_type(2)));
              const d2 w0 = {res[mi][0], res[mi][1]};
              const d2 w1 = {res[mi][2], res[mi][3]};
              ((AS1 d2*)GW(o))[0] = w0;
              ((AS1 d2*)GW(o))[1] = w1;
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) GW(o)[j] = res[mi][j];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (s0 + j < nt) {
#pragma unroll
            for (int mi = 0; mi < M; ++mi) GW(outb[mi] + base)[s0 + j] = res[mi][j];
          }
      }
    }
    __syncthreads();
  }
}

template <typename V, int M, int NPW, int WPS, int LNB, int PR>
hipError_t go3(const TileDesc* t, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL((stream3_kernel<V, M, NPW, WPS, LNB, PR>), dim3(n), dim3(64), 0, s, t);
  return hipGetLastError();
}

template <typename V, int M>
hipError_t launch_s3m(const TileDesc* t, uint32_t n, hipStream_t s) {
  if constexpr (sizeof(V) == 4 && M == 1) {
    static const int variant = [] {
      const char* e = getenv("PSG_STREAM3_VARIANT");  // benchmarking aid
      return e ? atoi(e) : 0;
    }();
    switch (variant) {
      case 1: return go3<V, M, 4, 8, 7, 0>(t, n, s);
      case 2: return go3<V, M, 2, 8, 7, 1>(t, n, s);
      case 3: return go3<V, M, 2, 8, 6, 0>(t, n, s);
      case 4: return go3<V, M, 3, 8, 7, 0>(t, n, s);
      default: break;
    }
  }
  return go3<V, M, 2, 8, 7, 0>(t, n, s);
}

template <typename V>
hipError_t launch_s3v(int m, const TileDesc* t, uint32_t n, hipStream_t s) {
  switch (m) {
    case 1: return launch_s3m<V, 1>(t, n, s);
    case 2: return launch_s3m<V, 2>(t, n, s);
    case 3: return launch_s3m<V, 3>(t, n, s);
    case 4: return launch_s3m<V, 4>(t, n, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_stream3(int dtype, int m, const TileDesc* d_tiles, uint32_t ncoarse,
                                    hipStream_t stream) {
  if (ncoarse == 0) return hipSuccess;
  return dtype == 0 ? launch_s3v<float>(m, d_tiles, ncoarse, stream)
                    : launch_s3v<double>(m, d_tiles, ncoarse, stream);
}

}  // namespace psg
