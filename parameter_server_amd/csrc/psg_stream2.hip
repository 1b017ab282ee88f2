// psg_stream2.hip -- streaming aggregate kernel v7 (the default): one wave
// per coarse range of 4096 server slots, built for occupancy.
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267): out[j] = fold over pushes p in arrival
// order of V_p[k] where S_p[k] == D[lo+j]; the first push assigns, later
// pushes add, and the serial path adds +0.0 for absent pushes (one "+0.0"
// per run of absent pushes is exact, see fold1).
//
// Measured on MI355X (DESIGN.md "Kernels"): this path is latency-bound and
// hidden by wave-level parallelism, so every register spent on software
// pipelining cost more (fewer resident waves) than it won.  The kernel is
// therefore the smallest loop that streams the data:
//   * a workgroup is one wave; lane p holds push p's cursor and coarse end
//     (coarse boundaries come from the partition kernel, 1 per 4096 slots);
//   * per fine tile of 256 slots: the D keys and the first batch of push
//     windows (64 keys per push) are one round trip; a ballot of each window
//     against the next tile's first key gives the tile's share of the push
//     (sorted pushes: a prefix), so fine boundaries need no search;
//   * pushes are folded strictly in arrival order, straight into an LDS
//     accumulator (a wave executes in lockstep and its LDS accesses are
//     ordered; barriers only order the compiler where lanes read statically
//     addressed slots other lanes wrote);
//   * slot search through a 64-bucket table (4 probes when the bucket window
//     is <= 8 slots, 9-probe full search otherwise);
//   * order check on slot positions: all keys matched + strictly increasing
//     slots <=> sorted, unique, inside the range (reference matched == n).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "psg_device.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))

namespace psg {

namespace {

constexpr int kFT = 256;   // fine tile slots (4 per lane)
constexpr int kMaxNB = 256;  // buckets per fine tile (template LNB: 64..256)

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
__device__ __forceinline__ V fold1(V acc, int lp, int p, V v, bool parallel,
                                   bool cont) {
  const bool gap = !parallel && ((lp >= 0) ? (p - lp > 1) : (cont && p > 0));
  const V a1 = gap ? acc + V(0) : acc;
  return (p == 0 && !cont) ? v : a1 + v;
}

// SR: slot search by dependent probes from the bucket start (0), one round
//     of wide window reads (1), or last-key-<=-k lifting over 8 candidates
//     with the value carried (2: 3 dependent LDS levels, no re-read)
// BTT: bucket table by per-bucket searches (0) or slot transitions (1)
// PR: first window of a push per tile sized by its expected share (1) or 64 (0)
// LNB: log2 of the buckets per fine tile
// DG: diagnostic ablation (benchmarking only, results invalid): 1 = no fold,
//     2 = no search and no fold
template <typename V, int M, int NPW, int WPS, int SR = 0, int BTT = 0, int PR = 1, int LNB = 6,
          int DG = 0>
__global__ __launch_bounds__(64, WPS) void stream2_kernel(const TileDesc* __restrict__ tiles) {
  constexpr int kNB = 1 << LNB;
  static_assert(kNB <= kMaxNB, "bucket table");
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
      // expected keys of push p per fine tile, + 2 sigma (Poisson) + 4: a
      // short first window leaves fewer over-fetched keys to re-read next tile
      const float mu = (float)(cend - cur) * (float)kFT / (float)ncs;
      const float w = mu + 2.0f * __builtin_sqrtf(mu) + 4.0f;
      pred = w >= 64.0f ? 64u : (uint32_t)w + 1u;
    }
  }
  if (lane < 16) dk[kFT + lane] = ~0ull;
  V* outb[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) outb[mi] = (V*)G(T.out)[mi] + T.slot0;
  // Retire the set-up loads here: left pending into the tile loop, they make
  // the compiler's wait insertion put a vmcnt(0) in front of every window
  // load (the per-push cursors read by readlane), serialising round trips.
  __builtin_amdgcn_s_waitcnt(0);

  // window of push p at its cursor: W keys; lanes past the coarse end hold
  // ~0, which is never below a tile bound
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

  for (uint32_t ft = 0; ft < nft; ++ft) {
    const uint32_t base = ft * kFT;
    const int nt = (int)(ncs - base < (uint32_t)kFT ? ncs - base : (uint32_t)kFT);
    const bool last_tile = ft + 1 == nft;
    V* outp[M];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) outp[mi] = outb[mi] + base;

    auto first_w = [&](uint32_t p) -> uint32_t {
      return PR ? (uint32_t)__builtin_amdgcn_readlane(pred, p) : 64u;
    };
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
      for (int mi = 0; mi < M; ++mi) acc[mi * kFT + s] = (cont && s < nt) ? G(outp[mi])[s] : V(0);
    }
    __syncthreads();
    const uint64_t klo =
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)dreg[0]) |
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(dreg[0] >> 32)) << 32);
    const uint64_t range = dk[nt - 1] - klo;
    const int bits = range ? 64 - __builtin_clzll(range) : 0;
    const int shift = bits > LNB ? bits - LNB : 0;
    if constexpr (DG >= 3) {
      if (lane == 0) btab[kNB] = (uint32_t)nt;
    } else if constexpr (BTT == 0) {
#pragma unroll
      for (int r = 0; r < kNB / 64; ++r) {
        const uint64_t d = (uint64_t)(lane + 64 * r) << shift;
        const uint64_t key = d > ~0ull - klo ? ~0ull : klo + d;
        const uint32_t sb = lb_pow2<kFT>(dk, 0, key);
        btab[lane + 64 * r] = sb < (uint32_t)nt ? sb : (uint32_t)nt;
      }
      if (lane == 0) btab[kNB] = (uint32_t)nt;
    } else {
      // btab[b] = first slot whose bucket >= b: a slot opens the buckets
      // between its predecessor's and its own; the last slot closes the table
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t up = __shfl_up(dreg[k], 1, 64);
        const uint64_t wrap = k > 0 ? __shfl(dreg[k > 0 ? k - 1 : 0], 63, 64) : 0ull;
        const uint64_t prevkey = lane > 0 ? up : wrap;
        const int sidx = lane + 64 * k;
        if (sidx < nt) {
          const int bcur = (int)((dreg[k] - klo) >> shift);
          const int bprev = sidx == 0 ? -1 : (int)((prevkey - klo) >> shift);
          for (int b = bprev + 1; b <= bcur; ++b) btab[b] = (uint32_t)sidx;
          if (sidx == nt - 1)
            for (int b = bcur + 1; b <= kNB; ++b) btab[b] = (uint32_t)nt;
        }
      }
    }
    __syncthreads();

    // ---- one window of push p: its share of this tile, searched, checked,
    //      folded in arrival order.  Returns the window's in-tile count.
    auto process = [&](uint64_t key, const V (&val)[M], uint32_t p, uint32_t W, int& carry,
                       uint32_t& fails) -> uint32_t {
      bool inb;
      if (last_tile) {  // the rest of the coarse range: every loaded key
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(cur, p);
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(cend, p);
        inb = (uint32_t)lane < (e - c < W ? e - c : W);
      } else {
        inb = key < bound;
      }
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
      bool found;
      if constexpr (DG >= 2) {
        pos = (uint32_t)lane * 4u + (lo & 1u);
        found = act;
      } else if constexpr (SR == 2) {
        // last slot with key <= k among lo..lo+7, its key carried along;
        // dk is ~0 past the tile, so the candidates never leave the array
        uint64_t val;
        if (hi - lo <= 8u) {
          const uint64_t v0 = dk[lo], v4 = dk[lo + 4];
          uint32_t j = v4 <= k ? lo + 4 : lo;
          val = v4 <= k ? v4 : v0;
          const uint64_t v2 = dk[j + 2];
          j = v2 <= k ? j + 2 : j;
          val = v2 <= k ? v2 : val;
          const uint64_t v1 = dk[j + 1];
          j = v1 <= k ? j + 1 : j;
          val = v1 <= k ? v1 : val;
          pos = j;
        } else {
          pos = lb_pow2<kFT>(dk, 0, k);
          val = dk[pos];
        }
        found = val == k;
      } else if constexpr (SR == 1) {
        if (hi - lo <= 8u) {
          // one round of 5 independent 16-byte reads covers [lo, lo+8]
          const uint32_t w0 = lo & ~1u;
          typedef uint64_t u2 __attribute__((ext_vector_type(2)));
          const u2* wp = (const u2*)(dk + w0);
          uint32_t cnt = 0;
          found = false;
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            const u2 v = wp[i];
            cnt += (v.x < k ? 1u : 0u) + (v.y < k ? 1u : 0u);
            found = found || v.x == k || v.y == k;
          }
          pos = w0 + cnt;
        } else {
          pos = lb_pow2<kFT>(dk, 0, k);
          found = dk[pos] == k;
        }
      } else {
        if (hi - lo <= 8u) pos = lb_pow2<8>(dk, lo, k);
        else pos = lb_pow2<kFT>(dk, 0, k);
        found = dk[pos] == k;
      }
      const uint32_t prev_in = __shfl_up(pos, 1, 64);
      const int prev = DG >= 2 ? -1 : lane == 0 ? carry : (int)prev_in;
      const bool ok = act && (int)pos < nt && found && prev < (int)pos;
      if (DG == 0 && ok) {
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
    auto flush_fails = [&](uint32_t p, uint32_t fails) {
      if (fails && lane == 0)
        __hip_atomic_fetch_add(GW(T.fail) + p, (unsigned long long)fails, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };

#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      if ((uint32_t)q < np) {
        int carry = -1;
        uint32_t fails = 0;
        const uint32_t Lq = process(wk[q], wv[q], q, first_w(q), carry, fails);
        rest(q, Lq, first_w(q), carry, fails);
        flush_fails(q, fails);
      }
    }
    // later pushes in batches of NPW: windows of a batch load together
    for (uint32_t b0 = NPW; b0 < np; b0 += NPW) {
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        if (b0 + q < np) load_window(wk[q], wv[q], b0 + q, first_w(b0 + q));
      }
#pragma unroll
      for (int q = 0; q < NPW; ++q) {
        if (b0 + q < np) {
          int carry = -1;
          uint32_t fails = 0;
          const uint32_t Lq = process(wk[q], wv[q], b0 + q, first_w(b0 + q), carry, fails);
          rest(b0 + q, Lq, first_w(b0 + q), carry, fails);
          flush_fails(b0 + q, fails);
        }
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
          V* o = outp[mi] + s0;
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
            for (int mi = 0; mi < M; ++mi) GW(outp[mi])[s0 + j] = res[mi][j];
          }
      }
    }
    __syncthreads();
  }
}

template <typename V, int M, int NPW, int WPS, int SR = 0, int BTT = 0, int PR = 1, int LNB = 6,
          int DG = 0>
hipError_t go(const TileDesc* t, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL((stream2_kernel<V, M, NPW, WPS, SR, BTT, PR, LNB, DG>), dim3(n), dim3(64), 0,
                     s, t);
  return hipGetLastError();
}

template <typename V, int M>
hipError_t launch_s2m(const TileDesc* t, uint32_t n, hipStream_t s) {
  if constexpr (sizeof(V) == 4 && M == 1) {
    static const int variant = [] {
      const char* e = getenv("PSG_STREAM2_VARIANT");  // benchmarking aid
      return e ? atoi(e) : 0;
    }();
    switch (variant) {
      case 1: return go<V, M, 2, 8, 0, 0, 0>(t, n, s);  // 64-key first windows
      case 2: return go<V, M, 2, 8, 1, 0, 1>(t, n, s);  // wide reads
      case 3: return go<V, M, 2, 8, 0, 1, 1>(t, n, s);  // transitions
      case 4: return go<V, M, 4, 8, 0, 0, 1>(t, n, s);
      case 5: return go<V, M, 1, 8, 0, 0, 1>(t, n, s);
      case 6: return go<V, M, 4, 8, 2, 0, 0, 7>(t, n, s);  // last<=k search, 128 buckets
      case 7: return go<V, M, 4, 8, 0, 0, 0>(t, n, s);
      case 8: return go<V, M, 4, 8, 2, 0, 0, 8>(t, n, s);  // 256 buckets
      case 9: return go<V, M, 2, 8, 2, 0, 0, 7>(t, n, s);
      case 10: return go<V, M, 4, 8, 0, 0, 0, 7>(t, n, s);
      case 21: return go<V, M, 4, 8, 0, 0, 0, 7, 1>(t, n, s);  // ablations of 10
      case 22: return go<V, M, 4, 8, 0, 0, 0, 7, 2>(t, n, s);
      case 23: return go<V, M, 4, 8, 0, 0, 0, 7, 3>(t, n, s);  // + no bucket table
      default: break;
    }
  }
  return go<V, M, 2, 8>(t, n, s);
}

template <typename V>
hipError_t launch_s2v(int m, const TileDesc* t, uint32_t n, hipStream_t s) {
  switch (m) {
    case 1: return launch_s2m<V, 1>(t, n, s);
    case 2: return launch_s2m<V, 2>(t, n, s);
    case 3: return launch_s2m<V, 3>(t, n, s);
    case 4: return launch_s2m<V, 4>(t, n, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_stream2(int dtype, int m, const TileDesc* d_tiles,
                                    uint32_t ncoarse, hipStream_t stream) {
  if (ncoarse == 0) return hipSuccess;
  return dtype == 0 ? launch_s2v<float>(m, d_tiles, ncoarse, stream)
                    : launch_s2v<double>(m, d_tiles, ncoarse, stream);
}

}  // namespace psg
