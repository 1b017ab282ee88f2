// psg_stream4.hip -- streaming aggregate kernel v9 (the default): v7's
// one-wave-per-coarse-range structure, software-pipelined.
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267); see psg_stream2.hip for the fold rules.
//
// Why v9: ablations of v7 on the bench workload put its
// skeleton (loads, tile install, ballots, stores) at 0.153 ms -- about the
// HBM rate -- and the slot search + fold at another 0.10 ms that did not
// overlap with memory: a wave computing has nothing in flight.  v9 keeps the
// next batch of push windows in flight (two register sets, A/B) while it
// searches and folds the current batch.  The batches of a tile are unrolled
// at compile time (NB batches of NPW pushes; the host picks the instance by
// the job's push count) so that every load/use distance is straight-line
// code and the compiler's wait counts stay exact.
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
// per fine tile; PR: first windows sized by the push's expected share;
// NB: batches per tile (compile time; np <= NB * NPW).
template <typename V, int M, int NPW, int WPS, int LNB, int PR, int NB>
__global__ __launch_bounds__(64, WPS) void stream4_kernel(const TileDesc* __restrict__ tiles) {
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
  const uint32_t nb = (np + NPW - 1) / NPW;
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

  auto first_w = [&](uint32_t p) -> uint32_t {
    return PR ? (uint32_t)__builtin_amdgcn_readlane(pred, p) : 64u;
  };
  // window of push p at its cursor: W keys.  Lanes past the coarse end
  // re-read its last key (masked by `window_mask`): unconditional loads, so
  // no register is written while a load to it may be in flight, which would
  // make the compiler drain every outstanding load (vmcnt(0)) first.
  // An empty window (or a lane p >= np, whose cursor and end are 0) reads
  // the tile's first server key instead: always a valid address.
  auto load_window = [&](uint64_t& wk, V (&wv)[M], uint32_t p, uint32_t W) {
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(cur, p);
    const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(cend, p);
    const uint32_t n = e - c < W ? e - c : W;
    const bool any = n > 0u;
    const uint32_t i = !any ? 0u : (uint32_t)lane < n ? (uint32_t)lane : n - 1u;
    const uint64_t* sk = any ? (const uint64_t*)readlane64(kp, p) + c : Dg;
    wk = G(sk)[i];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      const V* sv = any ? (const V*)readlane64(vp[mi], p) + c : (const V*)Dg;
      wv[mi] = G(sv)[i];
    }
  };
  // lanes of push p's window (at its cursor, W wide) that hold keys
  auto window_mask = [&](uint32_t p, uint32_t W) -> bool {
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(cur, p);
    const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(cend, p);
    return (uint32_t)lane < (e - c < W ? e - c : W);
  };
  auto load_batch = [&](uint64_t (&wk)[NPW], V (&wv)[NPW][M], uint32_t b) {
#pragma unroll
    for (int q = 0; q < NPW; ++q) load_window(wk[q], wv[q], b * NPW + q, first_w(b * NPW + q));
  };
  // server keys of fine tile ft (4 per lane, strided) and the next tile's first
  auto load_tile = [&](uint64_t (&dr)[4], uint64_t& bnd, uint32_t ft) {
    const uint32_t base = ft * kFT;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = base + (uint32_t)lane + 64u * k;
      dr[k] = i < ncs ? G(Dg)[i] : ~0ull;
    }
    bnd = ft + 1 == nft ? ~0ull : G(Dg)[base + kFT];
  };

  for (uint32_t ft = 0; ft < nft; ++ft) {
    uint64_t ka[NPW], kb[NPW];
    V va[NPW][M], vb[NPW][M];
    const uint32_t base = ft * kFT;
    const int nt = (int)(ncs - base < (uint32_t)kFT ? ncs - base : (uint32_t)kFT);
    const bool last_tile = ft + 1 == nft;
    // ---- one round trip: server keys, bound, first batch of windows
    uint64_t dreg[4], bound;
    load_tile(dreg, bound, ft);
    load_batch(ka, va, 0);

    // ---- install the tile: D, accumulators, bucket table
#pragma unroll
    for (int k = 0; k < 4; ++k) dk[lane + 64 * k] = dreg[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) lastl[lane * 4 + j] = -1;
    if (cont) {  // continuing an aggregate of an earlier launch
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int s = lane * 4 + j;
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          const V v = G(outb[mi] + base)[s < nt ? s : nt - 1];
          acc[mi * kFT + s] = s < nt ? v : V(0);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < M; ++mi) acc[mi * kFT + lane * 4 + j] = V(0);
    }
    __syncthreads();
    const uint64_t klo = dk[0];
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

    // ---- one window of push p: its share of this tile, searched, checked,
    //      folded in arrival order.  Returns the window's in-tile count.
    auto process = [&](uint64_t key, const V (&val)[M], uint32_t p, uint32_t W, int& carry,
                       uint32_t& fails) -> uint32_t {
      // the rest of the coarse range (last tile) or the keys below the bound
      const bool inb = window_mask(p, W) && (last_tile || key < bound);
      const unsigned long long bal = __ballot(inb);
      const uint32_t Lq = (~bal == 0ull) ? 64u : (uint32_t)__builtin_ctzll(~bal);
      const bool act = (uint32_t)lane < Lq;
      const uint64_t k = act ? key : ~0ull;
      const uint64_t dlt = k - klo;
      const uint32_t b = (k < klo) ? 0u
                         : (dlt >> shift) < (uint64_t)kNB ? (uint32_t)(dlt >> shift)
                                                          : (uint32_t)kNB;
      const uint32_t lo = btab[b];
      const uint32_t hi = btab[b < (uint32_t)kNB ? b + 1 : b];
      uint32_t pos;
      if (hi - lo <= 8u) pos = lb_pow2<8>(dk, lo, k);
      else pos = lb_pow2<kFT>(dk, 0, k);
      const bool found = dk[pos] == k;
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
      return Lq;
    };
    // push p after its first window: keep streaming while a whole window
    // fell in the tile (a short window -- sentinel lanes -- reached the end)
    auto rest = [&](uint32_t p, uint32_t Lq, uint32_t W, int& carry, uint32_t& fails) {
      while (Lq == W) {
        uint64_t k2;
        V v2[M];
        load_window(k2, v2, p, 64u);
        Lq = process(k2, v2, p, 64u, carry, fails);
        W = 64u;
      }
    };
    auto run_batch = [&](const uint64_t (&wk)[NPW], const V (&wv)[NPW][M], uint32_t b) {
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        const uint32_t p = b * NPW + q;
        if (p < np) {
          int carry = -1;
          uint32_t fails = 0;
          const uint32_t Lq = process(wk[q], wv[q], p, first_w(p), carry, fails);
          rest(p, Lq, first_w(p), carry, fails);
          if (fails && lane == 0)
            __hip_atomic_fetch_add(GW(T.fail) + p, (unsigned long long)fails, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    };

    // ---- batches, software-pipelined over the A/B window sets: while one
    //      set is searched and folded the next batch is in flight
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if ((uint32_t)b < nb) {
        if ((uint32_t)b + 1 < nb) {
          if (b & 1) load_batch(ka, va, b + 1);
          else load_batch(kb, vb, b + 1);
        }
        if (b & 1) run_batch(kb, vb, b);
        else run_batch(ka, va, b);
      }
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

template <typename V, int M, int NPW, int WPS, int LNB, int PR, int NB>
hipError_t go4(const TileDesc* t, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL((stream4_kernel<V, M, NPW, WPS, LNB, PR, NB>), dim3(n), dim3(64), 0, s, t);
  return hipGetLastError();
}

// instance by push count: NB batches of NPW windows cover the job's pushes
template <typename V, int M, int NPW, int WPS, int LNB, int PR>
hipError_t go4n(const TileDesc* t, uint32_t n, uint32_t maxnp, hipStream_t s) {
  if (maxnp <= 2 * NPW) return go4<V, M, NPW, WPS, LNB, PR, 2>(t, n, s);
  if (maxnp <= 4 * NPW) return go4<V, M, NPW, WPS, LNB, PR, 4>(t, n, s);
  if (maxnp <= 8 * NPW) return go4<V, M, NPW, WPS, LNB, PR, 8>(t, n, s);
  return go4<V, M, NPW, WPS, LNB, PR, (kStreamMaxPush + NPW - 1) / NPW>(t, n, s);
}

template <typename V, int M>
hipError_t launch_s4m(const TileDesc* t, uint32_t n, uint32_t maxnp, hipStream_t s) {
  if constexpr (sizeof(V) == 4 && M == 1) {
    static const int variant = [] {
      const char* e = getenv("PSG_STREAM4_VARIANT");  // benchmarking aid
      return e ? atoi(e) : 0;
    }();
    switch (variant) {
      case 1: return go4n<V, M, 2, 8, 7, 0>(t, n, maxnp, s);
      case 2: return go4n<V, M, 2, 7, 7, 1>(t, n, maxnp, s);
      case 3: return go4n<V, M, 4, 6, 7, 0>(t, n, maxnp, s);
      case 4: return go4n<V, M, 1, 8, 7, 0>(t, n, maxnp, s);
      case 5: return go4n<V, M, 4, 7, 7, 0>(t, n, maxnp, s);
      default: break;
    }
  }
  // f32, m = 1: 72 VGPRs at NB = 4 -> 7 waves/SIMD; wider values: 6
  return go4n<V, M, 2, (sizeof(V) == 4 && M == 1) ? 7 : 6, 7, 0>(t, n, maxnp, s);
}

template <typename V>
hipError_t launch_s4v(int m, const TileDesc* t, uint32_t n, uint32_t maxnp, hipStream_t s) {
  switch (m) {
    case 1: return launch_s4m<V, 1>(t, n, maxnp, s);
    case 2: return launch_s4m<V, 2>(t, n, maxnp, s);
    case 3: return launch_s4m<V, 3>(t, n, maxnp, s);
    case 4: return launch_s4m<V, 4>(t, n, maxnp, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_stream4(int dtype, int m, const TileDesc* d_tiles, uint32_t ncoarse,
                                    uint32_t maxnp, hipStream_t stream) {
  if (ncoarse == 0) return hipSuccess;
  return dtype == 0 ? launch_s4v<float>(m, d_tiles, ncoarse, maxnp, stream)
                    : launch_s4v<double>(m, d_tiles, ncoarse, maxnp, stream);
}

}  // namespace psg
