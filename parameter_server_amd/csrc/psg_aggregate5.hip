// psg_aggregate5.hip -- aggregate kernel v5 (one workgroup per tile).
//
// Same contract and bit-exact output as the v2/v4 kernels (reference
// KVVector::serialSetValue / parallelSetValue, kv_vector.h:84-204, over
// match / oldMatch, message.h:134-267).  Relative to v4:
//
//   * slot search through a per-tile bucket table: bucket(k) =
//     (k - D[0]) >> shift with TILE/4 buckets over the tile's key range;
//     btab[b] = first slot of bucket b, so lower_bound(k) lies in
//     [btab[b], btab[b+1]] and a 4-probe search covers windows <= 8 slots
//     (uniform / hashed / contiguous keys); wider windows fall back to the
//     full sentinel-padded search;
//   * an element alone in its slot within the chunk (one mask bit) folds
//     directly into the LDS accumulator; only slots with >= 2 pushes in the
//     chunk ("hot") stage their values, in push order, for one folding
//     thread each.  No per-chunk rank scan, no full scatter.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_device.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))

namespace psg {

using namespace dev;

namespace {

constexpr uint32_t kInv = 0xFFFFFFFFu;
constexpr uint32_t kLiBits = 25;
constexpr uint32_t kLiMask = (1u << kLiBits) - 1u;

template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}
template <typename T>
__device__ __forceinline__ AS1 T* GW(T* p) {
  return (AS1 T*)p;
}

template <typename V, int M, int TILE, int NT>
struct L5 {
  static constexpr int kSPT = TILE / NT;
  static constexpr int kChunk = NT * kEPT;
  static constexpr int kNB = TILE / 4;                          // buckets
  static constexpr size_t dk = 0;                               // u64[TILE + 8]
  static constexpr size_t mask = dk + 8 * (TILE + 8);           // u64[TILE]
  static constexpr size_t acc = mask + 8 * TILE;                // V[M][TILE]
  static constexpr size_t last = acc + sizeof(V) * M * TILE;    // i16[TILE]
  static constexpr size_t hoff = last + 2 * TILE;               // u16[TILE]
  static constexpr size_t hot = hoff + 2 * TILE;                // u16[TILE]
  static constexpr size_t btab = hot + 2 * TILE;                // u32[kNB + 1]
  static constexpr size_t hv = (btab + 4 * (kNB + 1) + 15) / 16 * 16;  // V[kChunk*M]
  static constexpr size_t epos = hv;                            // u16[kChunk] (aliases hv)
  static constexpr size_t hvb = sizeof(V) * M * kChunk > 2 * kChunk
                                    ? sizeof(V) * M * kChunk : 2 * kChunk;
  static constexpr size_t bpush = hv + hvb;                     // u32[kChunk/64]
  static constexpr size_t gk = bpush + 4 * (kChunk / 64);       // ptr[kGroup]
  static constexpr size_t gv = gk + 8 * kGroup;                 // ptr[kGroup*M]
  static constexpr size_t wsum = gv + 8 * kGroup * M;           // u32[16]
  static constexpr size_t misc = wsum + 64;                     // u32[16]
  static constexpr size_t pstart = misc + 64;                   // u32[np+1], u32[np]
  __host__ __device__ static size_t bytes(uint32_t maxnp) {
    return (pstart + 4 * (2 * (size_t)maxnp + 1) + 15) / 16 * 16;
  }
};

enum { kMiscHot = 0, kMiscCarry = 1, kMiscHv = 2 };

__device__ __forceinline__ uint32_t locate(const uint32_t* pstart, uint32_t pf,
                                           uint32_t pl, uint32_t e) {
  uint32_t p = pf;
#pragma unroll
  for (uint32_t step = 32; step > 0; step >>= 1) {
    const uint32_t c = p + step;
    const uint32_t cc = c < pl ? c : pl - 1;
    p = (c < pl && pstart[cc] <= e) ? c : p;
  }
  return p;
}

template <int TILE>
__device__ __forceinline__ uint32_t lb_padded(const uint64_t* a, uint64_t k) {
  const char* ab = (const char*)a;
  uint32_t off = 0;
#pragma unroll
  for (int step = TILE / 2; step > 0; step >>= 1) {
    const uint64_t v = *(const uint64_t*)(ab + off + 8 * (step - 1));
    off = (v < k) ? off + 8 * step : off;
  }
  const uint64_t v = *(const uint64_t*)(ab + off);
  off = (v < k) ? off + 8 : off;
  return off >> 3;
}

template <typename V>
__device__ __forceinline__ V fold1(V acc, int lp, int p, V v, bool parallel,
                                   bool cont) {
  const bool gap = !parallel && ((lp >= 0) ? (p - lp > 1) : (cont && p > 0));
  const V a1 = gap ? acc + V(0) : acc;
  return (p == 0 && !cont) ? v : a1 + v;
}

template <typename V, int M, int TILE, int NT>
__global__ __launch_bounds__(NT) void aggregate_v5_kernel(
    const TileDesc* __restrict__ tiles, uint32_t maxnp) {
  using L = L5<V, M, TILE, NT>;
  constexpr int SPT = L::kSPT;
  constexpr int CHUNK = L::kChunk;
  constexpr int NB = L::kNB;
  constexpr int LOGNB = __builtin_ctz(NB);
  static_assert(SPT == 4, "4 slots per thread");
  static_assert(NB <= NT, "one bucket per thread");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* dk = (uint64_t*)(smem + L::dk);
  unsigned long long* mask = (unsigned long long*)(smem + L::mask);
  V* accl = (V*)(smem + L::acc);
  int16_t* lastl = (int16_t*)(smem + L::last);
  uint16_t* hoff = (uint16_t*)(smem + L::hoff);
  uint16_t* hot = (uint16_t*)(smem + L::hot);
  uint32_t* btab = (uint32_t*)(smem + L::btab);
  V* hv = (V*)(smem + L::hv);
  uint16_t* epos = (uint16_t*)(smem + L::epos);
  uint32_t* bpush = (uint32_t*)(smem + L::bpush);
  const uint64_t** gk = (const uint64_t**)(smem + L::gk);
  const V** gv = (const V**)(smem + L::gv);
  uint32_t* wsum = (uint32_t*)(smem + L::wsum);
  uint32_t* misc = (uint32_t*)(smem + L::misc);
  uint32_t* pstart = (uint32_t*)(smem + L::pstart);
  uint32_t* segb = pstart + maxnp + 1;

  const int tid = threadIdx.x;
  const int s0 = tid * SPT;
  const TileDesc T = tiles[blockIdx.x];
  const int nt = (int)T.nt;
  const uint32_t np = T.np;
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  V* outp[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) outp[mi] = (V*)T.out[mi] + T.slot0;

  // ---- tile setup (one round trip): D (sentinel padded), segments, first
  //      push group, accumulators, last-push indices
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int i = tid + k * NT;
    dk[i] = i < nt ? G(T.dk)[i] : ~0ull;
  }
  if (tid < 8) dk[TILE + tid] = ~0ull;
  for (uint32_t p = tid; p < np; p += NT) {
    const uint32_t b = G(T.seg)[p];
    segb[p] = b;
    pstart[p] = G(T.seg)[np + p] - b;
  }
  {
    const uint32_t g0 = np < (uint32_t)kGroup ? np : (uint32_t)kGroup;
    for (uint32_t q = tid; q < g0 * (1 + M); q += NT) {
      if (q < g0) gk[q] = G(T.pkeys)[q];
      else gv[q - g0] = (const V*)G(T.pvals)[q - g0];
    }
  }
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    lastl[s0 + j] = -1;
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
      accl[mi * TILE + s0 + j] = (cont && s0 + j < nt) ? G(outp[mi])[s0 + j] : V(0);
  }
  __syncthreads();
  // bucket table over [D[0], D[nt-1]]
  const uint64_t klo = dk[0];
  const uint64_t range = nt > 0 ? dk[nt - 1] - klo : 0ull;
  const int bits = range ? 64 - __builtin_clzll(range) : 0;
  const int shift = bits > LOGNB ? bits - LOGNB : 0;
  if (tid <= NB) {
    uint32_t s = (uint32_t)nt;
    if (tid < NB) {
      const uint64_t d = (uint64_t)tid << shift;
      const uint64_t key = d > ~0ull - klo ? ~0ull : klo + d;
      s = lb_padded<TILE>(dk, key);
      s = s < (uint32_t)nt ? s : (uint32_t)nt;
    }
    btab[tid] = s;
  }
  uint32_t E = 0;
  for (uint32_t c0 = 0; c0 < np; c0 += NT) {
    const uint32_t idx = c0 + tid;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<NT>(idx < np ? pstart[idx] : 0u, wsum, &tot);
    if (idx < np) pstart[idx] = E + ex;
    E += tot;
    __syncthreads();
  }
  if (tid == 0) pstart[np] = E;

  uint32_t gbase = 0;
  for (uint32_t e0 = 0; e0 < E;) {
    __syncthreads();
    uint32_t pf;
    {
      int lo = 0, hi = (int)np - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pstart[mid] <= e0) lo = mid; else hi = mid - 1;
      }
      pf = (uint32_t)lo;
    }
    const uint32_t pl = (pf + kGroup < np) ? pf + kGroup : np;
    uint32_t e1 = e0 + CHUNK;
    if (e1 > E) e1 = E;
    if (e1 > pstart[pl]) e1 = pstart[pl];
    if (pf < gbase || pl > gbase + kGroup) {  // uniform: stage push pointers
      gbase = pf;
      const uint32_t w = pl - pf;
      for (uint32_t q = tid; q < w * (1 + M); q += NT) {
        if (q < w) gk[q] = G(T.pkeys)[pf + q];
        else gv[q - w] = (const V*)G(T.pvals)[(size_t)pf * M + (q - w)];
      }
    }
#pragma unroll
    for (int k = 0; k < SPT; ++k) mask[tid + k * NT] = 0ull;
    if (tid == 0) {
      misc[kMiscHot] = 0;
      misc[kMiscHv] = 0;
    }
    {
      const uint32_t nblk = (e1 - e0 + 63) >> 6;
      for (uint32_t b = tid; b < nblk; b += NT) {
        const uint32_t eb = e0 + (b << 6);
        const uint32_t p = locate(pstart, pf, pl, eb);
        const uint32_t elast = eb + 63 < e1 ? eb + 63 : e1 - 1;
        bpush[b] = p | (pstart[p + 1] > elast ? 0x80000000u : 0u);
      }
    }
    __syncthreads();

    // ---- loads (branch-free; lanes past the chunk re-load its last element)
    uint64_t ekey[kEPT];
    uint32_t einfo[kEPT];
    V ev[kEPT][M];
#pragma unroll
    for (int r = 0; r < kEPT; ++r) {
      const uint32_t e = e0 + (uint32_t)tid + (uint32_t)r * NT;
      const bool valid = e < e1;
      const uint32_t ec = valid ? e : e1 - 1;
      const uint32_t bi = __builtin_amdgcn_readfirstlane(bpush[(ec - e0) >> 6]);
      uint32_t p = bi & 0x7FFFFFFFu;
      if (!(bi >> 31)) p = locate(pstart, p, pl, ec);
      const uint32_t li = ec - pstart[p];
      const uint64_t i = (uint64_t)segb[p] + li;
      ekey[r] = G(gk[p - gbase])[i];
#pragma unroll
      for (int mi = 0; mi < M; ++mi) ev[r][mi] = G(gv[(p - gbase) * M + mi])[i];
      einfo[r] = valid ? (((p - pf) << kLiBits) | (li < kLiMask ? li : kLiMask)) : kInv;
    }

    // ---- slot search through the bucket table, mask bit, slot position
    uint32_t spos[kEPT];
#pragma unroll
    for (int r = 0; r < kEPT; ++r) {
      const uint64_t k = ekey[r];
      const uint64_t d = k - klo;
      const uint32_t b = (k < klo) ? 0u : (d >> shift) < (uint64_t)NB ? (uint32_t)(d >> shift) : NB;
      const uint32_t lo = btab[b];
      const uint32_t hi = btab[b + (b < (uint32_t)NB ? 1 : 0)];
      spos[r] = lo;
      if (hi - lo > 8u) spos[r] = kInv;  // wide window: full search below
      else {
        uint32_t off = lo * 8;
        const char* ab = (const char*)dk;
#pragma unroll
        for (int step = 4; step > 0; step >>= 1) {
          const uint64_t v = *(const uint64_t*)(ab + off + 8 * (step - 1));
          off = (v < k) ? off + 8 * step : off;
        }
        const uint64_t v = *(const uint64_t*)(ab + off);
        off = (v < k) ? off + 8 : off;
        spos[r] = off >> 3;
      }
    }
#pragma unroll
    for (int r = 0; r < kEPT; ++r)
      if (spos[r] == kInv) spos[r] = lb_padded<TILE>(dk, ekey[r]);
    uint32_t rec[kEPT];
#pragma unroll
    for (int r = 0; r < kEPT; ++r) {
      const uint32_t e = e0 + (uint32_t)tid + (uint32_t)r * NT;
      const uint32_t b = einfo[r] >> kLiBits;
      const int pos = (int)spos[r];
      const bool ok = einfo[r] != kInv && pos < nt && dk[pos] == ekey[r];
      if (ok) atomicOr(&mask[pos], 1ull << b);
      rec[r] = ok ? ((uint32_t)pos | (b << 16)) : kInv;
      epos[e - e0] = ok ? (uint16_t)pos : (uint16_t)0xFFFFu;
      if (einfo[r] != kInv && !ok)
        __hip_atomic_fetch_add(GW(T.fail) + pf + b, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();

    // ---- singles fold directly; hot slots register; order check
    uint32_t hrank[kEPT];
    {
      const uint32_t carry = misc[kMiscCarry];
#pragma unroll
      for (int r = 0; r < kEPT; ++r) {
        hrank[r] = kInv;
        if (rec[r] == kInv) continue;
        const int pos = (int)(rec[r] & 0xFFFFu);
        const int b = (int)(rec[r] >> 16);
        const int p = (int)pf + b;
        const unsigned long long mk = mask[pos];
        if ((mk & (mk - 1ull)) == 0ull) {  // alone in its slot: fold now
          const int lp = lastl[pos];
#pragma unroll
          for (int mi = 0; mi < M; ++mi)
            accl[mi * TILE + pos] = fold1<V>(accl[mi * TILE + pos], lp, p, ev[r][mi],
                                            parallel, cont);
          lastl[pos] = (int16_t)p;
        } else {
          const uint32_t rk = (uint32_t)__popcll(mk & ((1ull << b) - 1ull));
          hrank[r] = rk;
          if (rk == 0u) {  // the slot's first contributor registers it
            const uint32_t h = atomicAdd(&misc[kMiscHot], 1u);
            hot[h] = (uint16_t)pos;
            hoff[pos] = (uint16_t)atomicAdd(&misc[kMiscHv], (uint32_t)__popcll(mk));
          }
        }
      }
#pragma unroll
      for (int r = 0; r < kEPT; ++r) {
        const uint32_t e = e0 + (uint32_t)tid + (uint32_t)r * NT;
        if (rec[r] != kInv && (einfo[r] & kLiMask) > 0) {
          const uint32_t prev = e > e0 ? epos[e - 1 - e0] : carry;
          if (!(prev < (rec[r] & 0xFFFFu)))
            __hip_atomic_fetch_add(GW(T.fail) + pf + (einfo[r] >> kLiBits), 1ull,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    const uint32_t next_carry = epos[e1 - 1 - e0];  // before hv overwrites epos
    __syncthreads();
    const uint32_t nhot = misc[kMiscHot];
    if (tid == 0) misc[kMiscCarry] = next_carry;
    if (nhot > 0) {  // uniform
#pragma unroll
      for (int r = 0; r < kEPT; ++r) {
        if (hrank[r] != kInv) {
          const int pos = (int)(rec[r] & 0xFFFFu);
#pragma unroll
          for (int mi = 0; mi < M; ++mi) hv[(hoff[pos] + hrank[r]) * M + mi] = ev[r][mi];
        }
      }
      __syncthreads();
      for (uint32_t h = tid; h < nhot; h += NT) {
        const int slot = hot[h];
        unsigned long long mk = mask[slot];
        const uint32_t o = hoff[slot];
        const int lp0 = lastl[slot];
        int lp = lp0;
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          unsigned long long m2 = mk;
          uint32_t rr = o;
          lp = lp0;
          V a = accl[mi * TILE + slot];
          while (m2) {
            const int p = (int)pf + (__ffsll((long long)m2) - 1);
            m2 &= m2 - 1ull;
            a = fold1<V>(a, lp, p, hv[(rr++) * M + mi], parallel, cont);
            lp = p;
          }
          accl[mi * TILE + slot] = a;
        }
        lastl[slot] = (int16_t)lp;
      }
    }
    e0 = e1;
  }
  __syncthreads();

  // ---- trailing absent pushes (serial path: one "+ 0.0"), store
  V res[M][SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int lp = lastl[s0 + j];
    const bool gap = !parallel && ((lp >= 0) ? (lp < (int)np - 1) : (cont && np > 0));
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      const V a = accl[mi * TILE + s0 + j];
      res[mi][j] = gap ? a + V(0) : a;
    }
  }
  if (s0 + SPT <= nt) {
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
        for (int j = 0; j < SPT; ++j) GW(o)[j] = res[mi][j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (s0 + j < nt) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) GW(outp[mi])[s0 + j] = res[mi][j];
      }
    }
  }
}

template <typename V, int M, int G_>
hipError_t launch_one5(const TileDesc* d_tiles, uint32_t ntiles, uint32_t maxnp,
                       hipStream_t stream) {
  constexpr int TILE = geo_tile(G_), NT = geo_threads(G_);
  using L = L5<V, M, TILE, NT>;
  const size_t lds = L::bytes(maxnp);
  auto kern = aggregate_v5_kernel<V, M, TILE, NT>;
  if (lds > 65536) {
    static size_t attr = 0;
    if (attr < lds) {
      hipError_t e = hipFuncSetAttribute((const void*)kern,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds);
      if (e != hipSuccess) return e;
      attr = lds;
    }
  }
  hipLaunchKernelGGL(kern, dim3(ntiles), dim3(NT), lds, stream, d_tiles, maxnp);
  return hipGetLastError();
}

template <typename V, int M>
hipError_t launch_geo5(int geo, const TileDesc* t, uint32_t n, uint32_t maxnp,
                       hipStream_t s) {
  switch (geo) {
    case kGeoS: return launch_one5<V, M, kGeoS>(t, n, maxnp, s);
    case kGeoM: return launch_one5<V, M, kGeoM>(t, n, maxnp, s);
    case kGeoL: return launch_one5<V, M, kGeoL>(t, n, maxnp, s);
    default: return hipErrorInvalidValue;
  }
}

template <typename V>
hipError_t launch_m5(int m, int geo, const TileDesc* t, uint32_t n, uint32_t maxnp,
                     hipStream_t s) {
  switch (m) {
    case 1: return launch_geo5<V, 1>(geo, t, n, maxnp, s);
    case 2: return launch_geo5<V, 2>(geo, t, n, maxnp, s);
    case 3: return launch_geo5<V, 3>(geo, t, n, maxnp, s);
    case 4: return launch_geo5<V, 4>(geo, t, n, maxnp, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_v5(int dtype, int m, int geo, const TileDesc* d_tiles,
                               uint32_t ntiles, uint32_t maxnp, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  return dtype == 0 ? launch_m5<float>(m, geo, d_tiles, ntiles, maxnp, stream)
                    : launch_m5<double>(m, geo, d_tiles, ntiles, maxnp, stream);
}

}  // namespace psg
