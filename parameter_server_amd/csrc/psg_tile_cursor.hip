// psg_tile_cursor.hip -- the aggregate kernel for plans of long pieces with
// no partition pass: every workgroup walks a contiguous run of tiles (a
// CHUNK) of one job and keeps, per push, a CURSOR -- the index of the push's
// first key not yet merged -- so a tile's piece of push q starts where the
// previous tile's ended and its end is found by the element loads
// themselves: the first key >= the next tile's first server key.
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267), exactly as psg_tile.hip (same search, order
// check, wave-ordered fold, contributor counts and trailing +0.0): out[j] =
// fold over pushes in arrival order of V_p[k] where S_p[k] == D[lo + j].
// What changes is only where a tile's pieces come from:
//   psg_tile.hip    the partition kernel (psg_partition.hip) cut every push
//                   at every tile boundary first (one more launch, 0.19 GB
//                   of reads for cfg2) and each tile reads its bounds back;
//   here            a push's keys are read once, in tile order: a wave loads
//                   kr rounds of 64 consecutive keys of each of its pushes
//                   from the cursor, and a key belongs to the tile iff it
//                   precedes the first key >= the next tile's first server
//                   key (the lower_bound of message.h:96-99 / findRange,
//                   found by one ballot per round).  Keys past the piece are
//                   the next tile's and are read again there from L2.
// Shape: a 256-thread workgroup (4 waves), 1024-slot tiles, the plan's
// resident bucket index; pushes in groups of 8, wave w holding pushes 2w and
// 2w + 1 of the group (kr <= 3 rounds each: the host picks this form when a
// piece, mean + 4 sigma, fits 3 rounds); the fold runs wave by wave, so
// arrival order holds per slot with no atomics.  A piece longer than kr
// rounds (rare) is finished round by round inside its wave's fold step,
// before the wave's next push.  Chunk boundaries: a chunk starts from
// lower_bound(push, its first tile's first key); each chunk xors its start
// and its end cursors into the boundary word it shares with its neighbour,
// so a nonzero word (a push whose keys are not sorted) reaches
// psg_plan_matched; the job's first and last chunks write the covered range.
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

constexpr int kTS = kTileSlots;  // 1024 slots per tile
constexpr int kNT = kTS / 4;     // 256 threads, thread t owns slots 4t..4t+3
constexpr int kNW = kNT / 64;    // 4 waves
constexpr int kNB = kTS;         // one bucket per slot (the resident index's map)
constexpr int kPPW = 2;          // pushes per wave per group
constexpr int kGP = kNW * kPPW;  // pushes per group
constexpr int kRR = 3;           // rounds per push at most
constexpr int kCap = kPPW * kRR; // rounds a wave holds

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (uint64_t)uni((uint32_t)v) | (uint64_t)uni((uint32_t)(v >> 32)) << 32;
}

// blocks b and b+8 share an XCD (observed dispatch, speed only): neighbouring
// chunks (which share the cache lines at their boundary) on one XCD
__device__ __forceinline__ uint32_t xcd_map(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + j;
}

template <typename V, int M>
constexpr int occupancy() {
  constexpr int lds = (kTS + 4) * 8 + (kNB + 8) * 2 + M * (int)sizeof(V) * kTS + kTS * 4 + 32 * 4;
  constexpr int w = (163840 / lds) * kNW / 4;
  return w >= 8 ? 8 : (w < 1 ? 1 : w);
}

template <typename V, int M, int KR>
__global__ __launch_bounds__(kNT, (occupancy<V, M>())) void cursor_kernel(
    const CursorJob* __restrict__ jobs, const CursorChunk* __restrict__ chunks, uint32_t nchunks,
    uint32_t* __restrict__ bx) {
  __shared__ __attribute__((aligned(16))) uint64_t dk[kTS + 4];  // + sentinels ~0
  __shared__ __attribute__((aligned(16))) uint32_t bt32[(kNB + 8) / 2];
  uint16_t* const bt = (uint16_t*)bt32;
  __shared__ __attribute__((aligned(16))) V acc[M][kTS];
  __shared__ __attribute__((aligned(16))) uint32_t cnt[kTS];  // pushes holding the slot
  __shared__ uint32_t cur[32];                                // cursors
  __shared__ uint32_t sh_ovf;                                 // a piece past kr rounds

  const uint32_t w = uni((uint32_t)threadIdx.x >> 6);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const uint32_t ci = xcd_map(blockIdx.x, gridDim.x);
  if (ci >= nchunks) return;
  const CursorChunk C = chunks[ci];
  const CursorJob& J = jobs[C.job];
  const uint32_t np = J.np;
  const bool parallel = (J.flags & kFlagParallel) != 0;
  const bool cont = (J.flags & kFlagCont) != 0;
  constexpr uint32_t kr = KR;  // rounds per push (the job's J.kr, a template argument)
  const uint64_t* const D = J.dkeys;

  // ---- start cursors: lower_bound(push q, the chunk's first key); the
  // chunk boundary word gets them xored in, the job's first chunk writes the
  // covered range's start
  {
    const uint64_t k0 = G(D)[(uint64_t)C.t0 * kTS];
    for (uint32_t q = w; q < np; q += kNW) {
      const uint64_t* kp = (const uint64_t*)uni64((uint64_t)G(J.pkeys)[q]);
      const uint64_t n = uni64(G(J.pn)[q]);
      const uint32_t c = (uint32_t)dev::wave_search(kp, n, k0, false, lane);
      if (lane == 0) {
        cur[q] = c;
        if (C.t0 == 0) GW(J.seg)[q] = c;
        else atomicXor(bx + (size_t)ci * 32u + q, c);
      }
    }
  }
  if (tid == 0) sh_ovf = 0u;
  __syncthreads();

  for (uint32_t t = C.t0; t < C.t1; ++t) {
    // the thread id afresh per tile (opaque): values derived from it are
    // recomputed in the loop instead of hoisted out of it, where they would
    // hold VGPRs across the whole loop (and spill at the 64-VGPR budget)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const uint32_t s0 = 4u * (uint32_t)tid;
    const uint64_t slot0 = (uint64_t)t * kTS;
    const uint64_t* Dg = D + slot0;
    const uint32_t nt = (uint32_t)(J.nslots - slot0 < (uint64_t)kTS ? J.nslots - slot0 : kTS);
    // the piece bound: keys < the next tile's first key; the job's last tile
    // takes every key <= D[nslots - 1] (open: D ends at 2^64 - 1)
    const bool lastt = t + 1 == J.ntiles;
    const uint64_t dl = lastt ? G(D)[J.nslots - 1] : G(Dg)[kTS];
    const bool open = lastt && dl == ~0ull;
    const uint64_t nxt = lastt ? dl + 1ull : dl;

    const uint64_t klo = G(Dg)[0];
    const uint64_t khi = G(Dg)[nt - 1];
    const uint64_t range = khi - klo;
    const int bits = range ? 64 - __builtin_clzll(range) : 0;
    const int sh2 = bits > 32 ? bits - 32 : 0;
    const uint64_t r32 = range >> sh2;
    const uint32_t mul = dev::bucket_scale(r32, kNB);
    auto bucket = [&](uint64_t k) -> uint32_t {
      const uint64_t x = (k - klo) >> sh2;
      const uint32_t xs = x > r32 ? 0xffffffffu : (uint32_t)x;
      const uint32_t b = __umulhi(xs, mul);
      return b < (uint32_t)(kNB - 1) ? b : (uint32_t)(kNB - 1);
    };
    // the tile kernel's search (psg_tile.hip): bucket, a 4-key window from
    // the bucket start (the lower bound unless *deep: a bucket of more than 4
    // keys with all 4 below k, ~0.4 % of keys), *hit = k found
    auto search = [&](uint64_t k, bool* hit, bool* deep) -> uint32_t {
      const uint32_t b = bucket(k);
      const uint32_t l = bt[b];
      const uint32_t n = (uint32_t)bt[b + 1] - l;
      const uint64_t* wk = dk + l;
      const uint64_t k0 = wk[0], k1 = wk[1], k2 = wk[2], k3 = wk[3];
      const uint32_t c = (uint32_t)(k0 < k) + (uint32_t)(k1 < k) + (uint32_t)(k2 < k) +
                         (uint32_t)(k3 < k);
      const uint32_t p = l + c;
      const uint64_t eq = __ballot(k0 == k) | __ballot(k1 == k) | __ballot(k2 == k) |
                          __ballot(k3 == k);
      *hit = ((eq >> lane) & 1ull) && p < nt;
      *deep = c == 4u && n > 4u;
      return p;
    };
    // the rest of a long bucket, bisected (lanes with *deep only)
    auto bisect = [&](uint64_t k, bool* hit) -> uint32_t {
      const uint32_t b = bucket(k);
      uint32_t lo = bt[b] + 4u, m = (uint32_t)bt[b + 1] - lo;
      while (m > 0u) {
        const uint32_t half = m >> 1;
        if (dk[lo + half] < k) {
          lo += half + 1u;
          m -= half + 1u;
        } else {
          m = half;
        }
      }
      *hit = lo < nt && dk[lo] == k;
      return lo;
    };

    for (uint32_t g0 = 0; g0 < np || g0 == 0; g0 += kGP) {
      int lane = threadIdx.x & 63;
      asm volatile("" : "+v"(lane));
      // ---- this wave's pushes of the group: kr rounds from the cursor each
      uint64_t ek[kCap];
      V ev[kCap][M];
      uint32_t hv = 0;  // bit r: round r's element exists in its push
      uint32_t qn[kPPW], qc[kPPW];  // push index (np: none), cursor
#pragma unroll
      for (int p = 0; p < kPPW; ++p) {
        const uint32_t q = g0 + 2u * w + (uint32_t)p;
        qn[p] = q < np ? q : np;
        qc[p] = q < np ? uni(cur[q]) : 0u;
      }
#pragma unroll
      for (int p = 0; p < kPPW; ++p) {
        const uint32_t q = qn[p];
        if (q < np) {
          const uint64_t* kp = (const uint64_t*)uni64((uint64_t)G(J.pkeys)[q]) + qc[p];
          // keys left in the push past the cursor (pushes hold < 2^32 keys)
          const uint32_t rem = (uint32_t)uni64(G(J.pn)[q]) - qc[p];
#pragma unroll
          for (int r = 0; r < kRR; ++r) {
            const int rr = p * kRR + r;
            if ((uint32_t)r < kr) {
              const bool have = rem > 64u * r && (uint32_t)lane < rem - 64u * r;
              hv |= (uint32_t)have << rr;
              if (have) ek[rr] = G(kp + 64u * r)[lane];
#pragma unroll
              for (int mi = 0; mi < M; ++mi) {
                const V* vp = (const V*)uni64((uint64_t)G(J.pvals)[(size_t)q * M + mi]) + qc[p];
                if (have) ev[rr][mi] = G(vp + 64u * r)[lane];
              }
            }
          }
        }
      }
      if (g0 == 0) {
        // ---- D keys, resident bucket table, continued sums, loaded after
        // the first group's element loads were issued (both in flight at
        // once; D's registers live only up to their LDS stores) and
        // installed with the counts (first group)
        uint64_t d[4];
        if (s0 + 3u < nt && ((uintptr_t)Dg & 15u) == 0u) {
          const u64x2 x0 = __builtin_nontemporal_load((const AS1 u64x2*)(Dg + s0));
          const u64x2 x1 = __builtin_nontemporal_load((const AS1 u64x2*)(Dg + s0 + 2));
          d[0] = x0.x; d[1] = x0.y; d[2] = x1.x; d[3] = x1.y;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint64_t o = ~0ull;
            asm volatile("" : "+v"(o));
            d[j] = s0 + j < nt ? G(Dg)[s0 + j] : o;
          }
        }
        const u32x2 btw =
            __builtin_nontemporal_load((const AS1 u32x2*)(J.bt + (size_t)t * (kNB / 2)) + tid);
        V a0[M][4];
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            a0[mi][j] = (cont && s0 + j < nt) ? G((const V*)J.out[mi] + slot0)[s0 + j] : V(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dk[s0 + j] = d[j];
#pragma unroll
          for (int mi = 0; mi < M; ++mi) acc[mi][s0 + j] = a0[mi][j];
        }
        {
          // opaque constants: made here, not hoisted out of the tile loop
          // (held in VGPRs across it they spill at the 64-VGPR budget)
          uint32_t z = 0, o = ~0u;
          asm volatile("" : "+v"(z), "+v"(o));
          *(u32x4*)&cnt[s0] = u32x4{z, z, z, z};
          if (tid < 4) dk[kTS + tid] = (uint64_t)o << 32 | o;
        }
        *(u32x2*)&bt32[2 * tid] = btw;
        if (tid == 0) bt[kNB] = (uint16_t)nt;
        __syncthreads();  // (A) the tile's tables
      }

      // ---- piece bounds: the first key of a round that is past the push or
      // >= nxt ends the piece; rounds after it hold no piece element
      uint32_t inp = 0;    // bit r: in the piece
      uint32_t ends[kPPW];  // piece end (push index)
      uint32_t ovf = 0;     // bit p: the piece continues past kr rounds
#pragma unroll
      for (int p = 0; p < kPPW; ++p) {
        ends[p] = qc[p];
        bool closed = qn[p] >= np;
#pragma unroll
        for (int r = 0; r < kRR; ++r) {
          const int rr = p * kRR + r;
          if ((uint32_t)r < kr && !closed) {
            const bool in = ((hv >> rr) & 1u) && (open || ek[rr] < nxt);
            const uint64_t out = __ballot(!in);
            const uint32_t f = out ? (uint32_t)__builtin_ctzll(out) : 64u;
            inp |= (uint32_t)((uint32_t)lane < f) << rr;
            ends[p] += f;
            closed = f < 64u;
          }
        }
        if (!closed) ovf |= 1u << p;
      }

      // ---- search every round holding piece elements, then the rare deep
      // buckets, then the order check (per push: positions strictly increase
      // along its rounds)
      uint32_t pos[kCap];
      uint32_t fd = 0, dp = 0;  // bit r: found / deep
#pragma unroll
      for (int rr = 0; rr < kCap; ++rr) {
        pos[rr] = 0;
        if ((uint32_t)(rr % kRR) < kr && qn[rr / kRR] < np && __ballot((inp >> rr) & 1u)) {
          bool hit, deep;
          pos[rr] = search(ek[rr], &hit, &deep);
          fd |= (uint32_t)hit << rr;
          dp |= (uint32_t)deep << rr;
        }
      }
      if (__ballot((dp & inp) != 0u)) {
#pragma unroll
        for (int rr = 0; rr < kCap; ++rr) {
          if (((dp & inp) >> rr) & 1u) {
            bool hit;
            pos[rr] = bisect(ek[rr], &hit);
            fd = (fd & ~(1u << rr)) | (uint32_t)hit << rr;
          }
        }
      }
      uint32_t okb = 0;
#pragma unroll
      for (int p = 0; p < kPPW; ++p) {
        int prev0 = -1;
#pragma unroll
        for (int r = 0; r < kRR; ++r) {
          const int rr = p * kRR + r;
          if ((uint32_t)r < kr && qn[p] < np) {
            const int prev =
                __builtin_amdgcn_update_dpp(prev0, (int)pos[rr], 0x138, 0xf, 0xf, false);
            okb |= (uint32_t)((((inp & fd) >> rr) & 1u) && (int)pos[rr] > prev) << rr;
            prev0 = __builtin_amdgcn_readlane((int)pos[rr], 63);
          }
        }
      }
      // a piece running past kr rounds (rare) sends the whole group down the
      // slow path below, which keeps arrival order with no assumption
      if (ovf && lane == 0) sh_ovf = 1u;
      __syncthreads();  // (C)
      const bool slow = uni(sh_ovf) != 0u;
      if (!slow) {
        // contributor counts, match failures (per push)
#pragma unroll
        for (int p = 0; p < kPPW; ++p) {
          uint32_t nbad = 0;
#pragma unroll
          for (int r = 0; r < kRR; ++r) {
            const int rr = p * kRR + r;
            if ((uint32_t)r < kr && qn[p] < np) {
              const bool ok = (okb >> rr) & 1u;
              if (!parallel && ok)
                __hip_atomic_fetch_add(&cnt[pos[rr]], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
              nbad += (uint32_t)__popcll(__ballot(((inp >> rr) & 1u) && !ok));
            }
          }
          if (nbad && lane == 0)
            __hip_atomic_fetch_add(GW(J.fail) + qn[p], (unsigned long long)nbad, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        // ---- fold, wave by wave (waves hold consecutive pushes): arrival order
        for (uint32_t st = 0; st < (uint32_t)kNW; ++st) {
          if (st == w) {
#pragma unroll
            for (int rr = 0; rr < kCap; ++rr) {
              if ((uint32_t)(rr % kRR) < kr && ((okb >> rr) & 1u)) {
                const bool first = qn[rr / kRR] == 0u && !cont;
                const uint32_t s = pos[rr];
#pragma unroll
                for (int mi = 0; mi < M; ++mi)
                  acc[mi][s] = first ? ev[rr][mi] : acc[mi][s] + ev[rr][mi];
              }
            }
            // the next tile's cursors (read after the barriers that follow)
            if (lane == 0) {
#pragma unroll
              for (int p = 0; p < kPPW; ++p)
                if (qn[p] < np) cur[qn[p]] = ends[p];
            }
          }
          __syncthreads();
        }
      } else {
        // ---- slow path: wave 0 merges the group's pushes one after another,
        // a round of 64 keys at a time, each piece to its end
        if (w == 0) {
          const uint32_t ge = np - g0 < (uint32_t)kGP ? np - g0 : (uint32_t)kGP;
          for (uint32_t q = g0; q < g0 + ge; ++q) {
            const uint64_t* kp = (const uint64_t*)uni64((uint64_t)G(J.pkeys)[q]);
            const uint64_t n = uni64(G(J.pn)[q]);
            const bool first = q == 0u && !cont;
            uint32_t e = uni(cur[q]);
            int prev0 = -1;
            uint32_t nbad = 0;
            for (;;) {
              const uint64_t i = (uint64_t)e + lane;
              const bool have = i < n;
              uint64_t k = ~0ull;
              V v[M];
#pragma unroll
              for (int mi = 0; mi < M; ++mi) v[mi] = V(0);
              if (have) {
                k = G(kp)[i];
#pragma unroll
                for (int mi = 0; mi < M; ++mi)
                  v[mi] = G((const V*)uni64((uint64_t)G(J.pvals)[(size_t)q * M + mi]))[i];
              }
              const bool in0 = have && (open || k < nxt);
              const uint64_t out = __ballot(!in0);
              const uint32_t f = out ? (uint32_t)__builtin_ctzll(out) : 64u;
              const bool in = (uint32_t)lane < f;
              bool hit = false, deep = false;
              uint32_t ps = search(k, &hit, &deep);
              if (__ballot(in && deep))
                if (in && deep) ps = bisect(k, &hit);
              const int prev = __builtin_amdgcn_update_dpp(prev0, (int)ps, 0x138, 0xf, 0xf, false);
              const bool ok = in && hit && (int)ps > prev;
              if (!parallel && ok)
                __hip_atomic_fetch_add(&cnt[ps], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
              if (ok) {
#pragma unroll
                for (int mi = 0; mi < M; ++mi) acc[mi][ps] = first ? v[mi] : acc[mi][ps] + v[mi];
              }
              nbad += (uint32_t)__popcll(__ballot(in && !ok));
              prev0 = __builtin_amdgcn_readlane((int)ps, 63);
              e += f;
              if (f < 64u) break;
            }
            if (lane == 0) {
              cur[q] = e;
              if (nbad)
                __hip_atomic_fetch_add(GW(J.fail) + q, (unsigned long long)nbad, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          if (lane == 0) sh_ovf = 0u;
        }
        __syncthreads();
      }
      if (np == 0) break;
    }

    // ---- the "+0.0" of absent pushes (serial), stores (psg_tile.hip)
    V res[M][4];
    {
      const u32x4 cn = *(const u32x4*)&cnt[s0];
      const uint32_t ncontrib[4] = {cn.x, cn.y, cn.z, cn.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool gap = !parallel && ncontrib[j] != np;
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          const V a = acc[mi][s0 + j];
          res[mi][j] = gap ? a + V(0) : a;
        }
      }
    }
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      V* o = (V*)J.out[mi] + slot0 + s0;
      if (s0 + 3u < nt && ((uintptr_t)o & 15u) == 0u) {
        if constexpr (sizeof(V) == 4) {
          typedef float f4 __attribute__((ext_vector_type(4)));
          const f4 v = {res[mi][0], res[mi][1], res[mi][2], res[mi][3]};
          __builtin_nontemporal_store(v, (AS1 f4*)GW(o));
        } else {
          typedef double d2 __attribute__((ext_vector_type(2)));
          const d2 v0 = {res[mi][0], res[mi][1]};
          const d2 v1 = {res[mi][2], res[mi][3]};
          __builtin_nontemporal_store(v0, (AS1 d2*)GW(o));
          __builtin_nontemporal_store(v1, (AS1 d2*)GW(o) + 1);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (s0 + j < nt) GW(o)[j] = res[mi][j];
      }
    }
    __syncthreads();  // (B) every read of this tile's LDS before the next install
  }

  // ---- end cursors: the next chunk's boundary word, or the covered range's end
  if ((uint32_t)tid < np) {
    const uint32_t c = cur[tid];
    if (C.t1 == J.ntiles) GW(J.seg)[(size_t)J.ntiles * np + tid] = c;
    else atomicXor(bx + (size_t)(ci + 1) * 32u + tid, c);
  }
}

template <typename V, int M>
hipError_t go(int kr, const CursorJob* j, const CursorChunk* c, uint32_t n, uint32_t* bx,
              hipStream_t s) {
  switch (kr) {
    case 1: hipLaunchKernelGGL((cursor_kernel<V, M, 1>), dim3(n), dim3(kNT), 0, s, j, c, n, bx); break;
    case 2: hipLaunchKernelGGL((cursor_kernel<V, M, 2>), dim3(n), dim3(kNT), 0, s, j, c, n, bx); break;
    case 3: hipLaunchKernelGGL((cursor_kernel<V, M, 3>), dim3(n), dim3(kNT), 0, s, j, c, n, bx); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename V>
hipError_t launch_m(int m, int kr, const CursorJob* j, const CursorChunk* c, uint32_t n,
                    uint32_t* bx, hipStream_t s) {
  switch (m) {
    case 1: return go<V, 1>(kr, j, c, n, bx, s);
    case 2: return go<V, 2>(kr, j, c, n, bx, s);
    case 3: return go<V, 3>(kr, j, c, n, bx, s);
    case 4: return go<V, 4>(kr, j, c, n, bx, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_cursor(int dtype, int m, int kr, const CursorJob* d_jobs,
                                   const CursorChunk* d_chunks, uint32_t nchunks, uint32_t* bx,
                                   hipStream_t stream) {
  if (nchunks == 0) return hipSuccess;
  return dtype == 0 ? launch_m<float>(m, kr, d_jobs, d_chunks, nchunks, bx, stream)
                    : launch_m<double>(m, kr, d_jobs, d_chunks, nchunks, bx, stream);
}

}  // namespace psg
