// psg_aggregate.hip -- the hot path: per-(channel, time) aggregation of N
// sorted pushes into the resident server key range, on gfx950.
//
// Reference: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-137, 171-204) over oldMatch / match
// (src/system/message.h:134-267), with the push range located by
// SArray::findRange (src/base/shared_array_inl.h:164-171).
//
// Two launches per batch of jobs:
//   partition: one lane per (job, tile boundary, push): interpolation search
//              of the tile's first server key in the push.
//   aggregate: one workgroup per tile of server slots:
//     1. one scalar round trip for the TileDesc; then the D tile, the
//        tile's push segments and the push pointers load together;
//     2. chunks of <= NT*kEPT elements from <= 64 pushes: every element
//        load of the chunk is issued before any dependent work; then a
//        strict-order check against the predecessor key (shuffle / one
//        load at wave or segment edges), an LDS lower_bound for the slot,
//        and an LDS atomic OR of bit (p - pf) into mask[slot];
//     3. popcount(mask) -> workgroup scan -> each element's rank in
//        (slot, push) order: a stable counting sort, no value atomics;
//     4. each thread folds its 4 slots in push order (bit-exact reference
//        order, serial/parallel zero semantics) in registers across chunks;
//     5. one 16-B store per thread and value array.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_device.h"
#include "psg_internal.h"

namespace psg {

using namespace dev;

namespace {

constexpr uint32_t kInvalid = 0xFFFFFFFFu;

// partition: one lane per (job, push p, tile boundary b), 64 consecutive
// boundaries of one push per wave.  Boundary b < ntiles is
// lower_bound(S_p, D[b*tile]); b == ntiles is upper_bound(S_p, D[nslots-1])
// (SArray::findRange, shared_array_inl.h:164-171, restated per tile).
// Interpolation search: the reference's keys are hashed (murmur,
// example_parser.cc:205-208), so a push is near-uniform over its key range
// and about 3 probes bracket the answer in <= 16 keys at 128 K; bisection
// narrows skewed cases to 16 (at most 6 interpolation probes first) and one
// batch of 15 independent loads finishes.
__global__ __launch_bounds__(256) void partition_kernel(
    const JobDev* __restrict__ jobs, const uint32_t* __restrict__ item_job,
    uint32_t nitems) {
  const uint32_t item = __builtin_amdgcn_readfirstlane((blockIdx.x * 256u + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (item >= nitems) return;
  const uint32_t j = __builtin_amdgcn_readfirstlane(item_job[item]);
  const JobDev& J = jobs[j];
  const uint32_t local = item - J.part_begin;
  const uint32_t ng = (J.ntiles + 64u) >> 6;  // ceil((ntiles + 1) / 64)
  // group-major: the waves of one boundary group (all pushes) are adjacent,
  // so they share workgroups/XCDs (the group's D keys hit in L2) and their
  // interleaved seg[b * npush + p] writes land close together in time
  const uint32_t g = local / J.npush;
  const uint32_t p = local - g * J.npush;
  (void)ng;
  const uint32_t b = (g << 6) + (uint32_t)lane;
  const bool valid = b <= J.ntiles;
  uint64_t res = 0;
  if (J.nslots > 0) {
    const uint64_t* S = J.pkeys[p];
    const uint64_t n = J.pn[p];
    const uint32_t bc = valid ? b : J.ntiles;
    const bool up = bc == J.ntiles;
    const uint64_t x = up ? J.dkeys[J.nslots - 1] : J.dkeys[(uint64_t)bc * J.tile];
    // upper_bound(x) == lower_bound(x + 1): D never holds 2^64-1
    const uint64_t xl = up ? x + 1ull : x;
    const uint64_t k0 = n ? S[0] : 0ull, kn = n ? S[n - 1] : 0ull;
    if (n == 0 || xl <= k0) {
      res = 0;
    } else if (xl > kn) {
      res = n;
    } else {
      // invariant S[a] < xl <= S[c]; interpolation probes, then bisection
      uint64_t a = 0, c = n - 1, ka = k0, kc = kn;
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
      // the last <= 15 candidates in one round trip: independent loads of
      // S[a+1 .. c-1] (indices clamped to c, where S[c] >= xl counts 0)
      uint32_t below = 0;
#pragma unroll
      for (uint32_t i = 1; i < 16u; ++i) {
        const uint64_t idx = a + i < c ? a + i : c;
        below += S[idx] < xl ? 1u : 0u;
      }
      res = a + 1u + below;
    }
  }
  if (valid) {
    J.seg[(size_t)b * J.npush + p] = (uint32_t)res;
    if (b == 0) J.fail[p] = 0ull;  // the aggregate launch follows in-stream
  }
}

template <typename V, int M, int TILE, int NT>
struct AggLayout {
  static constexpr int kSPT = TILE / NT;
  static constexpr int kChunk = NT * kEPT;
  static constexpr size_t dk = 0;                                  // u64[TILE]
  static constexpr size_t mask = dk + 8 * TILE;                    // u64[TILE]
  static constexpr size_t base = mask + 8 * TILE;                  // u32[TILE]
  static constexpr size_t sorted = base + 4 * TILE;                // V[kChunk]
  static constexpr size_t gk = sorted + sizeof(V) * kChunk;        // ptr[kGroup]
  static constexpr size_t gv = gk + 8 * kGroup;                    // ptr[kGroup*M]
  static constexpr size_t wsum = gv + 8 * kGroup * M;              // u32[16]
  static constexpr size_t pstart = wsum + 64;                      // u32[np+1], u32[np]
  static size_t bytes(uint32_t maxnp) {
    return (pstart + 4 * (2 * (size_t)maxnp + 1) + 15) / 16 * 16;
  }
};

template <typename V, int M, int TILE, int NT>
__global__ __launch_bounds__(NT) void aggregate_kernel(
    const TileDesc* __restrict__ tiles, uint32_t maxnp) {
  using L = AggLayout<V, M, TILE, NT>;
  constexpr int SPT = L::kSPT;
  constexpr int CHUNK = L::kChunk;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* dk = (uint64_t*)(smem + L::dk);
  unsigned long long* mask = (unsigned long long*)(smem + L::mask);
  uint32_t* base = (uint32_t*)(smem + L::base);
  V* sorted = (V*)(smem + L::sorted);
  const uint64_t** gk = (const uint64_t**)(smem + L::gk);
  const V** gv = (const V**)(smem + L::gv);
  uint32_t* wsum = (uint32_t*)(smem + L::wsum);
  uint32_t* pstart = (uint32_t*)(smem + L::pstart);
  uint32_t* segb = pstart + maxnp + 1;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const TileDesc T = tiles[blockIdx.x];
  const int nt = (int)T.nt;
  const uint32_t np = T.np;
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;

  // 1. D tile, segments, pointers of the first push group: one round trip
  for (int i = tid; i < nt; i += NT) dk[i] = T.dk[i];
  for (uint32_t p = tid; p < np; p += NT) {
    const uint32_t b = T.seg[p];
    segb[p] = b;
    pstart[p] = T.seg[np + p] - b;
  }
  {
    const uint32_t g0 = np < (uint32_t)kGroup ? np : (uint32_t)kGroup;
    for (uint32_t q = tid; q < g0 * (1 + M); q += NT) {
      if (q < g0) gk[q] = T.pkeys[q];
      else gv[q - g0] = (const V*)T.pvals[(size_t)((q - g0) / M) * M + (q - g0) % M];
    }
  }
  V* outp[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) outp[mi] = (V*)T.out[mi] + T.slot0;
  __syncthreads();
  // exclusive scan of the segment lengths -> pstart, pstart[np] = E
  uint32_t E = 0;
  for (uint32_t c0 = 0; c0 < np; c0 += NT) {
    const uint32_t idx = c0 + tid;
    const uint32_t v = idx < np ? pstart[idx] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<NT>(v, wsum, &tot);
    if (idx < np) pstart[idx] = E + ex;
    E += tot;
    __syncthreads();
  }
  if (tid == 0) pstart[np] = E;

  const int s0 = tid * SPT;
  V acc[M][SPT];
  int lastp[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    lastp[j] = -1;
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
      acc[mi][j] = (cont && s0 + j < nt) ? outp[mi][s0 + j] : V(0);
  }
  __syncthreads();

  uint32_t gbase = 0;  // pushes whose pointers sit in gk/gv: [gbase, gbase+64)
  for (uint32_t e0 = 0; e0 < E;) {
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
    if (pf < gbase || pl > gbase + kGroup) {  // uniform: reload push pointers
      gbase = pf;
      for (uint32_t q = tid; q < (pl - pf) * (1 + M); q += NT) {
        const uint32_t w = pl - pf;
        if (q < w) gk[q] = T.pkeys[pf + q];
        else gv[q - w] = (const V*)T.pvals[(size_t)(pf + (q - w) / M) * M + (q - w) % M];
      }
    }
    for (int i = tid; i < nt; i += NT) mask[i] = 0ull;
    __syncthreads();

    // 2a. issue every load of the chunk
    uint64_t key[kEPT], prevg[kEPT];
    V vv[kEPT][M];
    uint32_t eli[kEPT];  // element index in its push's tile segment
    int eb[kEPT];        // p - pf, or -1 for no element
#pragma unroll
    for (int r = 0; r < kEPT; ++r) {
      const uint32_t e = e0 + (uint32_t)tid + (uint32_t)r * NT;
      key[r] = 0;
      prevg[r] = 0;
      eli[r] = 0;
      eb[r] = -1;
#pragma unroll
      for (int mi = 0; mi < M; ++mi) vv[r][mi] = V(0);
      if (e < e1) {
        int lo = (int)pf, hi = (int)pl - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (pstart[mid] <= e) lo = mid; else hi = mid - 1;
        }
        const uint32_t p = (uint32_t)lo;
        const uint32_t li = e - pstart[p];
        const uint64_t i = (uint64_t)segb[p] + li;
        const uint64_t* sk = gk[p - gbase];
        key[r] = sk[i];
#pragma unroll
        for (int mi = 0; mi < M; ++mi) vv[r][mi] = gv[(p - gbase) * M + mi][i];
        if (i > 0 && (li == 0 || lane == 0)) prevg[r] = sk[i - 1];
        eli[r] = li;
        eb[r] = (int)(p - pf);
      }
    }
    // 2b. order check, slot search, mask bit
    uint32_t rec[kEPT];
#pragma unroll
    for (int r = 0; r < kEPT; ++r) {
      const uint64_t prevk = __shfl_up(key[r], 1, 64);
      rec[r] = kInvalid;
      if (eb[r] >= 0) {
        const uint32_t b = (uint32_t)eb[r];
        const uint32_t li = eli[r];
        const uint32_t p = pf + b;
        const uint64_t i = (uint64_t)segb[p] + li;
        bool ok = true;
        if (i > 0) ok = ((li == 0 || lane == 0) ? prevg[r] : prevk) < key[r];
        const uint32_t Lp = pstart[p + 1] - pstart[p];
        int pos;
        if (Lp == (uint32_t)nt && dk[li] == key[r])
          pos = (int)li;  // dense segment: the slot is the offset
        else
          pos = lds_lower_bound<TILE>(dk, nt, key[r]);
        ok = ok && pos < nt && dk[pos] == key[r];
        if (ok) {
          const unsigned long long bit = 1ull << b;
          const unsigned long long old = atomicOr(&mask[pos], bit);
          ok = (old & bit) == 0ull;
        }
        if (ok)
          rec[r] = (uint32_t)pos | (b << 16);
        else
          atomicAdd(&T.fail[p], 1ull);
      }
    }
    __syncthreads();

    // 3. contribution counts -> ranks
    unsigned long long mymask[SPT];
    uint32_t mybase[SPT];
    {
      uint32_t c[SPT], csum = 0;
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        mymask[j] = (s0 + j < nt) ? mask[s0 + j] : 0ull;
        c[j] = (uint32_t)__popcll(mymask[j]);
        csum += c[j];
      }
      uint32_t tot;
      uint32_t run = block_excl_scan<NT>(csum, wsum, &tot);
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        mybase[j] = run;
        if (s0 + j < nt) base[s0 + j] = run;
        run += c[j];
      }
    }
    __syncthreads();

    // 4. scatter into (slot, push) order, fold in push order
    int newlast[SPT];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
#pragma unroll
      for (int r = 0; r < kEPT; ++r) {
        if (rec[r] != kInvalid) {
          const int pos = (int)(rec[r] & 0xFFFFu);
          const int b = (int)(rec[r] >> 16);
          const unsigned long long below = (1ull << b) - 1ull;
          sorted[base[pos] + (uint32_t)__popcll(mask[pos] & below)] = vv[r][mi];
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < SPT; ++j) {
        unsigned long long mk = mymask[j];
        uint32_t rr = mybase[j];
        int lp = lastp[j];
        V a = acc[mi][j];
        while (mk) {
          const int b = __ffsll((long long)mk) - 1;
          mk &= mk - 1ull;
          const int p = (int)pf + b;
          a = fold_step<V>(a, lp, p, sorted[rr++], parallel, cont);
          lp = p;
        }
        acc[mi][j] = a;
        newlast[j] = lp;
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < SPT; ++j) lastp[j] = newlast[j];
    e0 = e1;
  }

  // trailing absent pushes of the serial path: one "+ 0.0"
  if (!parallel) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int lp = lastp[j];
      const bool gap = (lp >= 0) ? (lp < (int)np - 1) : (cont && np > 0);
      if (gap) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) acc[mi][j] = acc[mi][j] + V(0);
      }
    }
  }

  // 5. store
  static_assert(SPT == 4, "4 slots per thread");
  if (s0 + SPT <= nt) {
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      V* o = outp[mi] + s0;
      if ((reinterpret_cast<uintptr_t>(o) & 15u) == 0u) {
        if constexpr (sizeof(V) == 4) {
          float4 w;
          w.x = acc[mi][0]; w.y = acc[mi][1]; w.z = acc[mi][2]; w.w = acc[mi][3];
          *reinterpret_cast<float4*>(o) = w;
        } else {
          double2 w0, w1;
          w0.x = acc[mi][0]; w0.y = acc[mi][1];
          w1.x = acc[mi][2]; w1.y = acc[mi][3];
          reinterpret_cast<double2*>(o)[0] = w0;
          reinterpret_cast<double2*>(o)[1] = w1;
        }
      } else {
#pragma unroll
        for (int j = 0; j < SPT; ++j) o[j] = acc[mi][j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (s0 + j < nt) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) outp[mi][s0 + j] = acc[mi][j];
      }
    }
  }
}

template <typename V, int M, int G>
hipError_t launch_one(const TileDesc* d_tiles, uint32_t ntiles, uint32_t maxnp,
                      hipStream_t stream) {
  constexpr int TILE = geo_tile(G), NT = geo_threads(G);
  using L = AggLayout<V, M, TILE, NT>;
  const size_t lds = L::bytes(maxnp);
  auto kern = aggregate_kernel<V, M, TILE, NT>;
  if (lds > 65536) {
    static bool attr = false;  // per instantiation
    if (!attr) {
      hipError_t e = hipFuncSetAttribute((const void*)kern,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds);
      if (e != hipSuccess) return e;
      attr = true;
    }
  }
  hipLaunchKernelGGL(kern, dim3(ntiles), dim3(NT), lds, stream, d_tiles, maxnp);
  return hipGetLastError();
}

template <typename V, int M>
hipError_t launch_geo(int geo, const TileDesc* t, uint32_t n, uint32_t maxnp,
                      hipStream_t s) {
  switch (geo) {
    case kGeoS: return launch_one<V, M, kGeoS>(t, n, maxnp, s);
    case kGeoM: return launch_one<V, M, kGeoM>(t, n, maxnp, s);
    case kGeoL: return launch_one<V, M, kGeoL>(t, n, maxnp, s);
    default: return hipErrorInvalidValue;
  }
}

template <typename V>
hipError_t launch_m(int m, int geo, const TileDesc* t, uint32_t n, uint32_t maxnp,
                    hipStream_t s) {
  switch (m) {
    case 1: return launch_geo<V, 1>(geo, t, n, maxnp, s);
    case 2: return launch_geo<V, 2>(geo, t, n, maxnp, s);
    case 3: return launch_geo<V, 3>(geo, t, n, maxnp, s);
    case 4: return launch_geo<V, 4>(geo, t, n, maxnp, s);
    default: return hipErrorInvalidValue;
  }
}

template <typename V, int M>
size_t lds_geo(int geo, uint32_t maxnp) {
  switch (geo) {
    case kGeoS: return AggLayout<V, M, geo_tile(kGeoS), geo_threads(kGeoS)>::bytes(maxnp);
    case kGeoM: return AggLayout<V, M, geo_tile(kGeoM), geo_threads(kGeoM)>::bytes(maxnp);
    default: return AggLayout<V, M, geo_tile(kGeoL), geo_threads(kGeoL)>::bytes(maxnp);
  }
}

}  // namespace

hipError_t launch_partition(const JobDev* d_jobs, const uint32_t* d_item_job,
                            uint32_t nitems, hipStream_t stream) {
  if (nitems == 0) return hipSuccess;
  const uint32_t blocks = (nitems + 3u) / 4u;
  hipLaunchKernelGGL(partition_kernel, dim3(blocks), dim3(256), 0, stream, d_jobs,
                     d_item_job, nitems);
  return hipGetLastError();
}

size_t aggregate_lds_bytes(int geo, int dtype, int m, uint32_t maxnp) {
  if (dtype == 0) {
    switch (m) {
      case 1: return lds_geo<float, 1>(geo, maxnp);
      case 2: return lds_geo<float, 2>(geo, maxnp);
      case 3: return lds_geo<float, 3>(geo, maxnp);
      default: return lds_geo<float, 4>(geo, maxnp);
    }
  }
  switch (m) {
    case 1: return lds_geo<double, 1>(geo, maxnp);
    case 2: return lds_geo<double, 2>(geo, maxnp);
    case 3: return lds_geo<double, 3>(geo, maxnp);
    default: return lds_geo<double, 4>(geo, maxnp);
  }
}

hipError_t launch_aggregate(int dtype, int m, int geo, const TileDesc* d_tiles,
                            uint32_t ntiles, uint32_t maxnp, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  return dtype == 0 ? launch_m<float>(m, geo, d_tiles, ntiles, maxnp, stream)
                    : launch_m<double>(m, geo, d_tiles, ntiles, maxnp, stream);
}

}  // namespace psg
