// psg_tile.hip -- aggregate kernel v13 ("tile"): one workgroup of TS/4
// threads per tile of TS server slots; every load of the tile is issued
// before any of it is used.
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267): out[j] = fold over pushes p in arrival
// order of V_p[k] where S_p[k] == D[lo+j]; the first push assigns, later
// pushes add, and the serial path adds +0.0 for absent pushes (one "+0.0"
// per run of absent pushes is exact, see dev::fold_step).
//
// Shape:
//   * the partition kernel has cut every push at every tile's first server
//     key, so push q's keys of this tile are S_q[seg[t][q], seg[t+1][q]);
//   * thread i takes element i of every push's piece (a "round" of up to
//     NT elements per push), so all element loads are independent,
//     coalesced, and in flight together with the tile's D keys;
//   * D goes to LDS with a bucket table over its key range (2 buckets per
//     slot): a search is one table read and one or two key reads;
//   * the fold runs push by push (a barrier between pushes), so each slot
//     sees its contributions in arrival order without atomics; sums and
//     "last push holding the slot" live in LDS;
//   * stores are 256 B per wave instruction;
//   * consecutive tiles run on one XCD (blocks b and b+8 share one), so the
//     cache lines two neighbouring tiles' pieces share are read once.
// Order check: inside a push's piece the matched positions must increase
// strictly and every key must be found; the piece boundaries come from the
// tile's key bounds, so this is the reference's matched == n <=> sorted,
// unique, inside the range.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_device.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))

namespace psg {

namespace {

template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}
template <typename T>
__device__ __forceinline__ AS1 T* GW(T* p) {
  return (AS1 T*)p;
}

constexpr int kGP = 8;  // pushes per group (elements in flight per thread)

template <int TS>
struct Geo {
  static constexpr int NT = TS / 4;   // threads
  static constexpr int SPT = 4;       // slots per thread
  static constexpr int NB = 2 * TS;   // buckets
  static constexpr int LNB = TS == 512 ? 10 : TS == 1024 ? 11 : TS == 2048 ? 12 : 13;
  static_assert((1 << LNB) == NB, "bucket count");
  static_assert(TS <= 0x7ffe, "u16 positions");
};

// blocks b and b+8 share an XCD (observed dispatch, speed only): give each
// XCD a contiguous run of tiles
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + j;
}

template <typename V, int M, int TS>
__global__ __launch_bounds__(TS / 4) void tile_kernel(const TileDesc* __restrict__ tiles) {
  using Gm = Geo<TS>;
  constexpr int NT = Gm::NT, SPT = Gm::SPT, NB = Gm::NB, LNB = Gm::LNB;
  __shared__ __attribute__((aligned(16))) uint64_t dk[TS + 8];
  __shared__ __attribute__((aligned(16))) uint16_t btab[NB + 8];
  __shared__ __attribute__((aligned(16))) V acc[M][TS];
  __shared__ __attribute__((aligned(16))) uint16_t lastl[TS];  // last push + 1 holding the slot
  __shared__ __attribute__((aligned(16))) uint16_t spos[kGP][NT];
  __shared__ int carry[kGP];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const TileDesc& T = tiles[xcd_tile(blockIdx.x, gridDim.x)];
  const uint32_t np = T.np;
  const uint32_t nt = T.nt;
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  const uint64_t* Dg = T.dk;

  // ---- group 0's element loads first: they are the long pole
  uint32_t c[kGP], len[kGP];
  uint64_t ek[kGP];
  V ev[kGP][M];
  uint32_t rounds = 0;
  auto group_bounds = [&](uint32_t g0) {
    const uint32_t gp = np - g0 < (uint32_t)kGP ? np - g0 : (uint32_t)kGP;
    uint32_t mx = 0;
#pragma unroll
    for (int q = 0; q < kGP; ++q) {
      c[q] = 0;
      len[q] = 0;
      if ((uint32_t)q < gp) {
        const uint32_t a = G(T.seg)[g0 + q];
        const uint32_t b = G(T.seg)[np + g0 + q];
        c[q] = a;
        len[q] = b > a ? b - a : 0u;
        if (b < a && tid == 0)  // pieces out of order: the push is unsorted
          __hip_atomic_fetch_add(GW(T.fail) + g0 + q, 1ull, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        mx = len[q] > mx ? len[q] : mx;
      }
    }
    rounds = __builtin_amdgcn_readfirstlane((mx + NT - 1) / NT);
  };
  // a pass folds one round of every push of the group (qsel < 0) or, when a
  // piece spans several rounds, one round of push qsel: the fold order must
  // stay push-major
  auto load_round = [&](uint32_t g0, uint32_t r, int qsel) {
#pragma unroll
    for (int q = 0; q < kGP; ++q) {
      const uint32_t i = r * NT + (uint32_t)tid;
      if ((qsel < 0 || q == qsel) && i < len[q]) {
        const uint32_t x = c[q] + i;
        ek[q] = G(T.pkeys[g0 + q])[x];
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          ev[q][mi] = G((const V*)T.pvals[(size_t)(g0 + q) * M + mi])[x];
      }
    }
  };
  if (np) {
    group_bounds(0);
    if (rounds <= 1) load_round(0, 0, -1);
  }

  // ---- D keys (and continued sums): slot s = tid + NT i
  uint64_t d[SPT];
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const uint32_t s = (uint32_t)(tid + i * NT);
    d[i] = s < nt ? G(Dg)[s] : ~0ull;
  }
  V a0[SPT][M];
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const uint32_t s = (uint32_t)(tid + i * NT);
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      a0[i][mi] = V(0);
      if (cont && s < nt) a0[i][mi] = G((const V*)T.out[mi] + T.slot0)[s];
    }
  }

  // ---- install D, sums, lastl
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const int s = tid + i * NT;
    dk[s] = d[i];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) acc[mi][s] = a0[i][mi];
    lastl[s] = 0;
  }
  if (tid < 8) dk[TS + tid] = ~0ull;
  if (tid < kGP) carry[tid] = -1;

  // bucket of a key: (k - klo) >> shift, clamped (keys outside the tile's
  // range land in an end bucket and are not found there)
  const uint64_t klo = G(Dg)[0];
  const uint64_t khi = G(Dg)[nt - 1];
  const uint64_t range = khi - klo;
  const int bits = range ? 64 - __builtin_clzll(range) : 0;
  const int shift = bits > LNB ? bits - LNB : 0;
  auto bucket = [&](uint64_t k) -> uint32_t {
    const uint64_t bb = (k - klo) >> shift;
    return bb < (uint64_t)NB ? (uint32_t)bb : (uint32_t)(NB - 1);
  };
  __syncthreads();

  // ---- bucket table: btab[b] = first slot whose bucket >= b, btab[NB] = nt
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const uint32_t s = (uint32_t)(tid + i * NT);
    if (s < nt) {
      const int b = (int)bucket(d[i]);
      const int bp = s ? (int)bucket(dk[s - 1]) : -1;
      for (int x = bp + 1; x <= b; ++x) btab[x] = (uint16_t)s;
      if (s == nt - 1)
        for (int x = b + 1; x <= NB; ++x) btab[x] = (uint16_t)nt;
    }
  }
  __syncthreads();

  // ---- groups of pushes; passes of NT elements per push
  for (uint32_t g0 = 0; g0 < np; g0 += kGP) {
    if (g0) {
      group_bounds(g0);
      if (tid < kGP) carry[tid] = -1;  // read after the pass's first barrier
    }
    const uint32_t gp = np - g0 < (uint32_t)kGP ? np - g0 : (uint32_t)kGP;
    const bool wide = rounds <= 1;
    const uint32_t npass = wide ? 1u : gp * rounds;
    for (uint32_t ps = 0; ps < npass; ++ps) {
      const int qsel = wide ? -1 : (int)(ps / rounds);
      const uint32_t r = wide ? 0u : ps % rounds;
      if (g0 || !wide) load_round(g0, r, qsel);
      const uint32_t i = r * NT + (uint32_t)tid;
      auto act = [&](int q) { return (qsel < 0 || q == qsel) && i < len[q]; };
      // search
      uint32_t pos[kGP];
      bool fnd[kGP];
#pragma unroll
      for (int q = 0; q < kGP; ++q) {
        pos[q] = 0xffffu;
        fnd[q] = false;
        if (act(q)) {
          const uint64_t k = ek[q];
          const uint32_t b = bucket(k);
          uint32_t l = btab[b];
          uint32_t n = (uint32_t)btab[b + 1] - l;
          while (n > 4u) {
            const uint32_t half = n >> 1;
            if (dk[l + half - 1] < k) {
              l += half;
              n -= half;
            } else {
              n = half;
            }
          }
          const uint64_t k0 = dk[l], k1 = dk[l + 1], k2 = dk[l + 2], k3 = dk[l + 3];
          const bool l0 = n > 0u && k0 < k, l1 = n > 1u && k1 < k;
          const bool l2 = n > 2u && k2 < k, l3 = n > 3u && k3 < k;
          pos[q] = l + (l0 ? 1u : 0u) + (l1 ? 1u : 0u) + (l2 ? 1u : 0u) + (l3 ? 1u : 0u);
          fnd[q] = (n > 0u && k0 == k) | (n > 1u && k1 == k) | (n > 2u && k2 == k) |
                   (n > 3u && k3 == k);
          spos[q][tid] = fnd[q] ? (uint16_t)pos[q] : (uint16_t)0xffffu;
        }
      }
      __syncthreads();
      // order check: strictly increasing positions inside each piece
      bool ok[kGP];
#pragma unroll
      for (int q = 0; q < kGP; ++q) {
        ok[q] = false;
        if ((uint32_t)q < gp && (qsel < 0 || q == qsel)) {
          const bool a = act(q);
          if (a) {
            const int prev = tid ? (int)spos[q][tid - 1] : carry[q];
            ok[q] = fnd[q] && (int)pos[q] > prev;
          }
          const uint64_t bad = __ballot(a && !ok[q]);
          if (bad && lane == 0)
            __hip_atomic_fetch_add(GW(T.fail) + g0 + q, (unsigned long long)__popcll(bad),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      // fold, push by push in arrival order
#pragma unroll
      for (int q = 0; q < kGP; ++q) {
        if ((uint32_t)q < gp && (qsel < 0 || q == qsel)) {
          if (ok[q]) {
            const uint32_t p = g0 + (uint32_t)q;
            const uint32_t s = pos[q];
            const uint32_t l1 = lastl[s];
            const bool first = p == 0u && !cont;
            const bool gap = !parallel && l1 < p;
#pragma unroll
            for (int mi = 0; mi < M; ++mi) {
              const V a = acc[mi][s];
              const V ag = gap ? a + V(0) : a;
              acc[mi][s] = first ? ev[q][mi] : ag + ev[q][mi];
            }
            lastl[s] = (uint16_t)(p + 1u);
          }
          __syncthreads();
        }
      }
      // carry: the round's last element of each piece
#pragma unroll
      for (int q = 0; q < kGP; ++q) {
        if (act(q) && (i + 1u == len[q] || tid == NT - 1))
          carry[q] = fnd[q] ? (int)pos[q] : 0xffff;
      }
      __syncthreads();
    }
  }

  // ---- trailing "+0.0" of absent last pushes (serial), stores
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const uint32_t s = (uint32_t)(tid + i * NT);
    if (s < nt) {
      const bool gap = !parallel && (uint32_t)lastl[s] < np;
#pragma unroll
      for (int mi = 0; mi < M; ++mi) {
        const V a = acc[mi][s];
        GW((V*)T.out[mi] + T.slot0)[s] = gap ? a + V(0) : a;
      }
    }
  }
}

template <typename V, int M, int TS>
hipError_t go(const TileDesc* t, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL((tile_kernel<V, M, TS>), dim3(n), dim3(TS / 4), 0, s, t);
  return hipGetLastError();
}

template <typename V, int TS>
hipError_t launch_m(int m, const TileDesc* t, uint32_t n, hipStream_t s) {
  switch (m) {
    case 1: return go<V, 1, TS>(t, n, s);
    case 2: return go<V, 2, TS>(t, n, s);
    case 3: return go<V, 3, TS>(t, n, s);
    case 4: return go<V, 4, TS>(t, n, s);
    default: return hipErrorInvalidValue;
  }
}

template <typename V>
hipError_t launch_ts(int tile, int m, const TileDesc* t, uint32_t n, hipStream_t s) {
  switch (tile) {
    case 1024: return launch_m<V, 1024>(m, t, n, s);
    case 2048: return launch_m<V, 2048>(m, t, n, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool tile_size_ok(int tile) { return tile == 1024 || tile == 2048; }

hipError_t launch_aggregate_tile(int dtype, int m, int tile, const TileDesc* d_tiles,
                                 uint32_t ntiles, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  return dtype == 0 ? launch_ts<float>(tile, m, d_tiles, ntiles, stream)
                    : launch_ts<double>(tile, m, d_tiles, ntiles, stream);
}

}  // namespace psg
