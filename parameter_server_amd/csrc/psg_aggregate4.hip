// psg_aggregate4.hip -- lean aggregate kernel (one workgroup per tile).
//
// Same contract and bit-exact output as aggregate_kernel (psg_aggregate.hip;
// reference KVVector::serialSetValue / parallelSetValue, kv_vector.h:84-204,
// over match / oldMatch, message.h:134-267), with the instruction stream
// cut down (DESIGN.md "Kernels"):
//
//   * element -> push: one wave-uniform lookup per round when the wave's 64
//     elements belong to one push (the common case), a 6-probe branchless
//     search otherwise;
//   * slot search: the D tile is padded with UINT64_MAX sentinels to a power
//     of two; log2(TILE)+1 unguarded probes on a byte offset, so each probe
//     is one ds_read_b64 with an immediate offset + compare + select;
//   * push order is checked on slot positions (u16 in LDS): all keys matched
//     and strictly increasing slots <=> strictly increasing keys inside the
//     range, i.e. the reference's matched == n (kv_vector.h:134,192);
//   * fold: a slot with one contribution in the chunk is folded in O(1) by
//     its owner; slots with >= 2 (cross-push duplicates) go to a compacted
//     hot list folded in push order by one thread each, so waves no longer
//     loop max(popcount) times per slot;
//   * accumulators and last-push indices live in LDS for the whole tile.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

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
struct L4 {
  static constexpr int kSPT = TILE / NT;
  static constexpr int kChunk = NT * kEPT;
  static constexpr size_t dk = 0;                               // u64[TILE]
  static constexpr size_t mask = dk + 8 * TILE;                 // u64[TILE]
  static constexpr size_t acc = mask + 8 * TILE;                // V[M][TILE]
  static constexpr size_t base = acc + sizeof(V) * M * TILE;    // u16[TILE]
  static constexpr size_t sorted = base + 2 * TILE;             // V[kChunk] + dummy
  static constexpr size_t epos = sorted;                        // u16[kChunk], aliases sorted
  static constexpr size_t bpush = sorted + sizeof(V) * kChunk + 16;  // u32[kChunk/64]
  static constexpr size_t last = bpush + 4 * (kChunk / 64);     // i16[TILE]
  static constexpr size_t hot = last + 2 * TILE;                // u16[TILE]
  static constexpr size_t gk = hot + 2 * TILE;                  // ptr[kGroup]
  static constexpr size_t gv = gk + 8 * kGroup;                 // ptr[kGroup*M]
  static constexpr size_t wsum = gv + 8 * kGroup * M;           // u32[16]
  static constexpr size_t misc = wsum + 64;                     // u32[16]
  static constexpr size_t pstart = misc + 64;                   // u32[np+1], u32[np]
  __host__ __device__ static size_t bytes(uint32_t maxnp) {
    return (pstart + 4 * (2 * (size_t)maxnp + 1) + 15) / 16 * 16;
  }
};

enum { kMiscHot = 0, kMiscCarry = 1 };

// largest p in [pf, pl) with pstart[p] <= e  (pl - pf <= 64)
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

// branchless lower_bound over a sentinel-padded power-of-two tile; works on
// byte offsets so every probe is one ds_read_b64 with an immediate offset.
template <int TILE>
__device__ __forceinline__ int lb_padded(const uint64_t* a, uint64_t k) {
  const char* ab = (const char*)a;
  uint32_t off = 0;
#pragma unroll
  for (int step = TILE / 2; step > 0; step >>= 1) {
    const uint64_t v = *(const uint64_t*)(ab + off + 8 * (step - 1));
    off = (v < k) ? off + 8 * step : off;
  }
  const uint64_t v = *(const uint64_t*)(ab + off);
  off = (v < k) ? off + 8 : off;
  return (int)(off >> 3);
}

// one fold step in push-arrival order (fold_step in psg_device.h), branchless
template <typename V>
__device__ __forceinline__ V fold1(V acc, int lp, int p, V v, bool parallel,
                                   bool cont) {
  const bool gap = !parallel && ((lp >= 0) ? (p - lp > 1) : (cont && p > 0));
  const V a1 = gap ? acc + V(0) : acc;
  return (p == 0 && !cont) ? v : a1 + v;
}

// MODE (diagnostic ablation, 0 = the product kernel): 1 = loads + store
// only, 2 = + slot search and mask, 3 = + ranks (no scatter/fold).
template <typename V, int M, int TILE, int NT, int MODE = 0>
__global__ __launch_bounds__(NT) void aggregate_v4_kernel(
    const TileDesc* __restrict__ tiles, uint32_t maxnp) {
  using L = L4<V, M, TILE, NT>;
  constexpr int SPT = L::kSPT;
  constexpr int CHUNK = L::kChunk;
  static_assert(SPT == 4, "4 slots per thread");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* dk = (uint64_t*)(smem + L::dk);
  unsigned long long* mask = (unsigned long long*)(smem + L::mask);
  V* accl = (V*)(smem + L::acc);
  uint16_t* base = (uint16_t*)(smem + L::base);
  V* sorted = (V*)(smem + L::sorted);
  uint16_t* epos = (uint16_t*)(smem + L::epos);
  uint32_t* bpush = (uint32_t*)(smem + L::bpush);
  int16_t* lastl = (int16_t*)(smem + L::last);
  uint16_t* hot = (uint16_t*)(smem + L::hot);
  const uint64_t** gk = (const uint64_t**)(smem + L::gk);
  const V** gv = (const V**)(smem + L::gv);
  uint32_t* wsum = (uint32_t*)(smem + L::wsum);
  uint32_t* misc = (uint32_t*)(smem + L::misc);
  uint32_t* pstart = (uint32_t*)(smem + L::pstart);
  uint32_t* segb = pstart + maxnp + 1;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int s0 = tid * SPT;
  const TileDesc T = tiles[blockIdx.x];
  const int nt = (int)T.nt;
  const uint32_t np = T.np;
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  V* outp[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) outp[mi] = (V*)T.out[mi] + T.slot0;

  // ---- tile setup: D (sentinel padded), segments, first push group,
  //      accumulators, last-push indices: one round trip
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int i = tid + k * NT;
    dk[i] = i < nt ? G(T.dk)[i] : ~0ull;
  }
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
  __syncthreads();

  uint32_t gbase = 0;
  for (uint32_t e0 = 0; e0 < E;) {
    // chunk bounds (uniform)
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
      __syncthreads();
      gbase = pf;
      const uint32_t w = pl - pf;
      for (uint32_t q = tid; q < w * (1 + M); q += NT) {
        if (q < w) gk[q] = G(T.pkeys)[pf + q];
        else gv[q - w] = (const V*)G(T.pvals)[(size_t)pf * M + (q - w)];
      }
    }
#pragma unroll
    for (int k = 0; k < SPT; ++k) mask[tid + k * NT] = 0ull;
    if (tid == 0) misc[kMiscHot] = 0;
    // push of the first element of every 64-element block of the chunk, and
    // whether the whole block lies in that push (bit 31)
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

    // ---- 2a. every element load of the chunk, branch-free (lanes past the
    //          chunk re-load its last element and are masked off below)
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
      if (!(bi >> 31)) p = locate(pstart, p, pl, ec);  // wave-uniform branch
      const uint32_t li = ec - pstart[p];
      const uint64_t i = (uint64_t)segb[p] + li;
      ekey[r] = G(gk[p - gbase])[i];
#pragma unroll
      for (int mi = 0; mi < M; ++mi) ev[r][mi] = G(gv[(p - gbase) * M + mi])[i];
      einfo[r] = valid ? (((p - pf) << kLiBits) | (li < kLiMask ? li : kLiMask)) : kInv;
    }

    if constexpr (MODE == 1) {
      V sink = V(0);
#pragma unroll
      for (int r = 0; r < kEPT; ++r)
        if (einfo[r] != kInv) sink += ev[r][0] + V(ekey[r] & 1u);
      accl[s0] += sink;
      __syncthreads();
      e0 = e1;
      continue;
    }
    // ---- 2b. slot of every element (independent chains interleave), mask
    //          bit, slot position for the order check
    uint32_t rec[kEPT];
    int spos[kEPT];
#pragma unroll
    for (int r = 0; r < kEPT; ++r) spos[r] = lb_padded<TILE>(dk, ekey[r]);
#pragma unroll
    for (int r = 0; r < kEPT; ++r) {
      const uint32_t e = e0 + (uint32_t)tid + (uint32_t)r * NT;
      const uint32_t b = einfo[r] >> kLiBits;
      const int pos = spos[r];
      const bool ok = einfo[r] != kInv && pos < nt && dk[pos] == ekey[r];
      if (ok) atomicOr(&mask[pos], 1ull << b);
      rec[r] = ok ? ((uint32_t)pos | (b << 16)) : kInv;
      epos[e - e0] = ok ? (uint16_t)pos : (uint16_t)0xFFFFu;
      if (einfo[r] != kInv && !ok)
        __hip_atomic_fetch_add(GW(T.fail) + pf + b, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();

    if constexpr (MODE == 2) {
      e0 = e1;
      continue;
    }
    // ---- 3. counts -> rank bases; hot list; order check
    unsigned long long mymask[SPT];
    uint32_t mybase[SPT];
    {
      uint32_t c[SPT], csum = 0;
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        mymask[j] = mask[s0 + j];
        c[j] = (uint32_t)__popcll(mymask[j]);
        csum += c[j];
        if (c[j] >= 2) hot[atomicAdd(&misc[kMiscHot], 1u)] = (uint16_t)(s0 + j);
      }
      uint32_t tot;
      uint32_t run = block_excl_scan<NT>(csum, wsum, &tot);
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        mybase[j] = run;
        base[s0 + j] = (uint16_t)run;
        run += c[j];
      }
    }
    {
      const uint32_t carry = misc[kMiscCarry];
#pragma unroll
      for (int r = 0; r < kEPT; ++r) {
        const uint32_t e = e0 + (uint32_t)tid + (uint32_t)r * NT;
        const uint32_t prev = e > e0 ? epos[e - 1 - e0] : carry;
        if (rec[r] != kInv && (einfo[r] & kLiMask) > 0) {
          if (!(prev < (rec[r] & 0xFFFFu)))
            __hip_atomic_fetch_add(GW(T.fail) + pf + (einfo[r] >> kLiBits), 1ull,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    const uint32_t next_carry = epos[e1 - 1 - e0];  // before sorted overwrites epos
    __syncthreads();
    const uint32_t nhot = misc[kMiscHot];
    if (tid == 0) misc[kMiscCarry] = next_carry;

    if constexpr (MODE == 3) {
      e0 = e1;
      continue;
    }
    // ---- 4. scatter into (slot, push) order; fold singles and hot slots
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
#pragma unroll
      for (int r = 0; r < kEPT; ++r) {
        const bool ok = rec[r] != kInv;
        const int pos = (int)(rec[r] & 0x07FFu) & (TILE - 1);
        const int b = (int)((rec[r] >> 16) & 63u);
        const unsigned long long below = (1ull << b) - 1ull;
        const uint32_t rank = base[pos] + (uint32_t)__popcll(mask[pos] & below);
        sorted[ok ? rank : (uint32_t)CHUNK] = ev[r][mi];
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        const unsigned long long mk = mymask[j];
        const bool single = mk != 0ull && (mk & (mk - 1ull)) == 0ull;
        const int p = (int)pf + (__ffsll((long long)mk) - 1);
        const int lp = lastl[s0 + j];
        V* a = &accl[mi * TILE + s0 + j];
        const V cur = *a;
        const V nv = fold1<V>(cur, lp, p, sorted[mybase[j] < (uint32_t)CHUNK ? mybase[j] : CHUNK],
                              parallel, cont);
        *a = single ? nv : cur;
        if (mi == M - 1 && single) lastl[s0 + j] = (int16_t)p;
      }
      for (uint32_t h = tid; h < nhot; h += NT) {
        const int slot = hot[h];
        unsigned long long mk = mask[slot];
        uint32_t rr = base[slot];
        int lp = lastl[slot];
        V a = accl[mi * TILE + slot];
        while (mk) {
          const int p = (int)pf + (__ffsll((long long)mk) - 1);
          mk &= mk - 1ull;
          a = fold1<V>(a, lp, p, sorted[rr++], parallel, cont);
          lp = p;
        }
        accl[mi * TILE + slot] = a;
        if (mi == M - 1) lastl[slot] = (int16_t)lp;
      }
      __syncthreads();
    }
    e0 = e1;
  }

  // ---- 5. trailing absent pushes (serial path: one "+ 0.0"), store
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

template <typename V, int M, int G_, int MODE = 0>
hipError_t launch_one4(const TileDesc* d_tiles, uint32_t ntiles, uint32_t maxnp,
                       hipStream_t stream) {
  constexpr int TILE = geo_tile(G_), NT = geo_threads(G_);
  using L = L4<V, M, TILE, NT>;
  const size_t lds = L::bytes(maxnp);
  auto kern = aggregate_v4_kernel<V, M, TILE, NT, MODE>;
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
hipError_t launch_geo4(int geo, const TileDesc* t, uint32_t n, uint32_t maxnp,
                       hipStream_t s) {
  if constexpr (sizeof(V) == 4 && M == 1) {
    static const int mode = [] {
      const char* e = getenv("PSG_AGG_MODE");  // diagnostic ablation only
      return e ? atoi(e) : 0;
    }();
    if (mode == 1) return launch_one4<V, M, kGeoM, 1>(t, n, maxnp, s);
    if (mode == 2) return launch_one4<V, M, kGeoM, 2>(t, n, maxnp, s);
    if (mode == 3) return launch_one4<V, M, kGeoM, 3>(t, n, maxnp, s);
  }
  switch (geo) {
    case kGeoS: return launch_one4<V, M, kGeoS>(t, n, maxnp, s);
    case kGeoM: return launch_one4<V, M, kGeoM>(t, n, maxnp, s);
    case kGeoL: return launch_one4<V, M, kGeoL>(t, n, maxnp, s);
    default: return hipErrorInvalidValue;
  }
}

template <typename V>
hipError_t launch_m4(int m, int geo, const TileDesc* t, uint32_t n, uint32_t maxnp,
                     hipStream_t s) {
  switch (m) {
    case 1: return launch_geo4<V, 1>(geo, t, n, maxnp, s);
    case 2: return launch_geo4<V, 2>(geo, t, n, maxnp, s);
    case 3: return launch_geo4<V, 3>(geo, t, n, maxnp, s);
    case 4: return launch_geo4<V, 4>(geo, t, n, maxnp, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_v4(int dtype, int m, int geo, const TileDesc* d_tiles,
                               uint32_t ntiles, uint32_t maxnp, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  return dtype == 0 ? launch_m4<float>(m, geo, d_tiles, ntiles, maxnp, stream)
                    : launch_m4<double>(m, geo, d_tiles, ntiles, maxnp, stream);
}

}  // namespace psg
