// psg_rows.hip -- aggregate kernel v10 ("rows"): one wave per coarse range of
// C server slots whose keys sit in LDS; every push key of the range streams
// through exactly once, packed into full 64-lane rows across push boundaries.
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267): out[j] = fold over pushes p in arrival
// order of V_p[k] where S_p[k] == D[lo+j]; the first push assigns, later
// pushes add, and the serial path adds +0.0 for absent pushes (one "+0.0"
// per run of absent pushes is exact, see fold_q).
//
// Why this shape.  Counters on the earlier
// tile-window kernels (v7/v9) showed ~820 VALU instructions per 256 server
// slots: eight per-push windows per fine tile, each about half full, each
// paying its own bookkeeping, plus a per-tile bucket table built by binary
// searches.  Here:
//   * the partition kernel gives, per push, the segment [c_p, e_p) of keys
//     inside the range; the segments are concatenated (exclusive scan over
//     the lanes that hold the pushes) and cut into rows of 64 keys, so a row
//     is full except the last one of the range, whatever the push sizes;
//   * a lane's key address is an SGPR base + 8 * its row index; only rows
//     that cross a push boundary select a second base (v_cndmask);
//   * rows are prefetched R deep in registers (loads never wait on LDS);
//   * the slot search is a bucket table over the range (about one slot per
//     bucket for hashed keys) built once per range by an LDS histogram and a
//     scan, then 4 candidate keys read in one LDS round trip; a bucket
//     longer than 4 is narrowed by binary search first (skewed key sets stay
//     correct, just slower);
//   * the fold is an LDS read-modify-write in push order: a row holding
//     pushes q..q' folds them one exec mask at a time (SGPR masks through
//     inverse_ballot), so two pushes that share a slot inside one row keep
//     their arrival order;
//   * order check: all keys found + strictly increasing slots within a
//     push's segment <=> the push is sorted, unique and inside the range
//     (the reference's matched == n).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

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

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// lanes [lo, hi) as a wave mask (0 <= lo <= hi <= 64)
__device__ __forceinline__ uint64_t lane_range(uint32_t lo, uint32_t hi) {
  const uint64_t a = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  const uint64_t b = lo >= 64 ? ~0ull : ((1ull << lo) - 1ull);
  return a & ~b;
}

// C: server slots per sub-tile (power of two, >= 256); R: rows in flight.
// A wave owns a span of up to kMaxSub sub-tiles of one partition range.
template <typename V, int M, int C, int R, int WPS>
__global__ __launch_bounds__(64, WPS) void rows_kernel(const TileDesc* __restrict__ tiles) {
  constexpr int NB = 2 * C;  // buckets: about half a slot each for hashed keys
  constexpr int LNB = __builtin_ctz(NB);
  constexpr int SPL = C / 64;   // slots per lane
  constexpr int EPL = NB / 64;  // bucket entries per lane (scan)
  static_assert(SPL % 4 == 0 && EPL % 8 == 0, "C >= 256");
  static_assert(C <= 4096, "u16 bucket starts");
  // dk doubles as the bucket histogram (u32[NB + 4]) before D is installed
  __shared__ __attribute__((aligned(16))) uint64_t dk[C + 8];
  __shared__ __attribute__((aligned(16))) uint16_t btab[NB + 8];  // first slot of bucket b
  __shared__ __attribute__((aligned(16))) V acc[M * C];
  __shared__ __attribute__((aligned(16))) uint8_t lastl[C];  // last push + 1 that held the slot
  __shared__ uint32_t nfail[64];
  __shared__ uint32_t bnd[(kRowsMaxSub + 1) * 64];  // segment starts, [point][push]
  static_assert((NB + 4) * 4 <= (C + 8) * 8, "histogram fits in dk");

  const int lane = threadIdx.x;
  const TileDesc T = tiles[blockIdx.x];
  const uint32_t np = T.np;  // <= 64 (host guarantees)
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  const uint32_t nt = T.nt;  // span slots, 1 .. kRowsMaxSub * C
  const uint32_t nsub = (nt + C - 1) / C;
  const uint64_t* Dg = T.dk;
  const uint32_t soff = T.sub & 0xffffu;  // span offset inside its partition range
  const uint32_t pslots = T.sub >> 16;    // slots of that range

  nfail[lane] = 0u;
  auto out_of = [&](int mi) -> V* { return (V*)T.out[mi] + T.slot0; };
  if (np == 0) {  // no pushes: the (continued) sums as they are
    if (!cont) {
      for (uint32_t s = (uint32_t)lane; s < nt; s += 64u) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) GW(out_of(mi))[s] = V(0);
      }
    }
    return;
  }

  // ---- lane p < np: push p's segment [c_p, e_p) of the partition range
  const uint32_t pl = (uint32_t)lane < np ? (uint32_t)lane : np - 1;
  const uint32_t c_raw = G(T.seg)[pl];
  const uint32_t e_raw = G(T.seg)[np + pl];
  const uint64_t kb_raw = (uint64_t)G(T.pkeys)[pl];
  uint64_t vb_raw[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) vb_raw[mi] = (uint64_t)G(T.pvals)[(size_t)pl * M + mi];

  // ---- bnd[j][p] = first key of push p at or after D[j C] (j = 0..nsub).
  //      A point strictly inside the partition range is located by
  //      interpolating its index in [c_p, e_p) and reading the 64 keys
  //      around it (lines the rows re-read from cache), four points x
  //      kRowsInlinePush pushes per round trip; a miss (skewed keys) falls
  //      back to a wave search.  Points on the range's edges are c_p / e_p.
  const uint32_t bstride = np <= (uint32_t)kRowsInlinePush ? (uint32_t)kRowsInlinePush : 64u;
  if ((uint32_t)lane < np) {
    bnd[lane] = soff == 0u ? c_raw : 0u;
    bnd[nsub * bstride + lane] = soff + nt >= pslots ? e_raw : 0u;
  }
  {
    // interior points j in [jlo, jhi]
    const uint32_t jlo = soff == 0u ? 1u : 0u;
    const uint32_t jhi = soff + nt >= pslots ? nsub - 1u : nsub;
    for (uint32_t j0 = jlo; j0 <= jhi && jhi != ~0u; j0 += 4u) {
      uint64_t wk[4 * kRowsInlinePush];
#pragma unroll
      for (int i = 0; i < 4 * kRowsInlinePush; ++i) {
        const uint32_t j = j0 + (uint32_t)(i / kRowsInlinePush);
        const uint32_t q = min((uint32_t)(i % kRowsInlinePush), np - 1u);
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(c_raw, q);
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(e_raw, q);
        const uint32_t o = soff + min(j * (uint32_t)C, nt);
        const bool need = j <= jhi && (uint32_t)(i % kRowsInlinePush) < np && e > c;
        const uint32_t est = c + (uint32_t)((float)(e - c) * ((float)o / (float)pslots));
        const uint32_t wmax = e - c > 64u ? e - 64u : c;
        const uint32_t w0 = min(max(est, c + 32u) - 32u, wmax);
        const uint32_t nv = min(64u, e - w0);
        const uint64_t kp = need ? readlane64(kb_raw, q) : (uint64_t)Dg;
        const uint32_t idx = need ? w0 + min((uint32_t)lane, nv - 1u) : 0u;
        wk[i] = ((const AS1 uint64_t*)kp)[idx];
      }
#pragma unroll
      for (int i = 0; i < 4 * kRowsInlinePush; ++i) {
        const uint32_t j = j0 + (uint32_t)(i / kRowsInlinePush);
        const uint32_t q = (uint32_t)(i % kRowsInlinePush);
        if (j > jhi || q >= np) continue;
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(c_raw, q);
        const uint32_t e = (uint32_t)__builtin_amdgcn_readlane(e_raw, q);
        uint32_t res = c;
        if (e > c) {
          const uint32_t o = soff + min(j * (uint32_t)C, nt);
          const uint32_t est = c + (uint32_t)((float)(e - c) * ((float)o / (float)pslots));
          const uint32_t wmax = e - c > 64u ? e - 64u : c;
          const uint32_t w0 = min(max(est, c + 32u) - 32u, wmax);
          const uint32_t nv = min(64u, e - w0);
          const uint64_t x = G(Dg)[min(j * (uint32_t)C, nt)];
          const uint32_t cw =
              (uint32_t)__builtin_popcountll(__ballot((uint32_t)lane < nv && wk[i] < x));
          res = w0 + cw;
          if ((cw == 0u && w0 > c) || (cw == nv && w0 + nv < e)) {
            const uint64_t* S = (const uint64_t*)readlane64(kb_raw, q);
            res = c + (uint32_t)dev::wave_search(S + c, e - c, x, false, lane);
          }
        }
        if (lane == 0) bnd[j * bstride + q] = res;
      }
    }
  }
  __syncthreads();

  uint64_t dreg[SPL];
  const uint32_t qs_mask = parallel ? 0u : ~0u;  // parallel path: no gap canonicalisation

  // results of sub-tile j: trailing absent pushes (serial: one "+ 0.0"),
  // 4 slots per lane per store
  auto store_sub = [&](uint32_t j) {
    const uint32_t base = j * (uint32_t)C;
    const uint32_t ntj = min((uint32_t)C, nt - base);
#pragma unroll
    for (int jj = 0; jj < SPL / 4; ++jj) {
      const uint32_t s0 = (uint32_t)(jj * 256 + lane * 4);
      const uint32_t ll = *(const uint32_t*)&lastl[s0];
      V res[M][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t l1 = (ll >> (8 * u)) & 0xffu;
        const bool gap = !parallel && l1 < np;
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          const V a = acc[mi * C + s0 + u];
          res[mi][u] = gap ? a + V(0) : a;
        }
      }
#pragma unroll
      for (int mi = 0; mi < M; ++mi) {
        V* o = out_of(mi) + base + s0;
        if (s0 + 4 <= ntj && (reinterpret_cast<uintptr_t>(o) & 15u) == 0u) {
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
          for (int u = 0; u < 4; ++u)
            if (s0 + u < ntj) GW(o)[u] = res[mi][u];
        }
      }
    }
  };

  for (uint32_t jsub = 0; jsub < nsub; ++jsub) {
    const uint32_t base = jsub * (uint32_t)C;
    const uint32_t ntj = min((uint32_t)C, nt - base);
    const uint64_t* Dj = Dg + base;

    // ---- this sub-tile's segments [lo_p, hi_p), packed at offset excl
    const uint32_t lo_p = bnd[jsub * bstride + pl];
    const uint32_t hi_p = bnd[(jsub + 1) * bstride + pl];
#pragma unroll
    for (int i = 0; i < SPL; ++i) {
      const uint32_t s = (uint32_t)(i * 64 + lane);
      dreg[i] = G(Dj)[s < ntj ? s : ntj - 1];
    }
    const uint64_t khi = G(Dj)[ntj - 1];
    const bool own = (uint32_t)lane < np;
    // only an unsorted push makes lower_bound non-monotone
    const bool neg = own && (e_raw < c_raw || hi_p < lo_p);
    const uint32_t cnt = (own && !neg) ? hi_p - lo_p : 0u;
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    const uint32_t excl = incl - cnt;  // lanes >= np: excl = incl = total
    // row element g of push p sits at kb_p + 8 g
    const uint64_t kb = kb_raw + 8ull * lo_p - 8ull * excl;
    uint64_t vb[M];
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
      vb[mi] = vb_raw[mi] + sizeof(V) * (uint64_t)lo_p - sizeof(V) * (uint64_t)excl;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
    const uint32_t nrows = (total + 63u) >> 6;
    const uint64_t nonempty = __ballot(cnt > 0u);
    if (neg && jsub == 0) nfail[lane] = 1u;

    // the pushes of the row starting at element g0: the first one (its
    // segment holds g0; pushes are concatenated in order, so those ending at
    // or before g0 are a prefix of the lanes) and the non-empty ones that
    // start inside (g0, g0 + 64)
    auto row_first = [&](uint32_t g0) -> uint32_t {
      const uint32_t q = (uint32_t)__builtin_popcountll(__ballot(incl <= g0));
      return q < np ? q : np - 1;
    };
    auto row_inner = [&](uint32_t g0) -> uint64_t {
      return __ballot(excl - g0 - 1u < 63u) & nonempty;
    };

    // ---- row loads: lane g = 64 r + lane of the concatenated segments;
    //      lanes past the end re-read the last element (masked in process)
    const uint32_t glim = (total ? total : 1u) - 1u;
    auto load_row = [&](uint32_t r, uint64_t& key, V (&val)[M]) {
      const uint32_t g0 = r << 6;
      const uint32_t q0 = row_first(g0);
      const uint64_t inner = row_inner(g0);
      uint64_t kp0 = readlane64(kb, q0);
      uint64_t vp0[M];
#pragma unroll
      for (int mi = 0; mi < M; ++mi) vp0[mi] = readlane64(vb[mi], q0);
      if (total == 0u) {  // nothing to stream: a valid dummy address
        kp0 = (uint64_t)Dg;
#pragma unroll
        for (int mi = 0; mi < M; ++mi) vp0[mi] = (uint64_t)Dg;
      }
      const uint32_t gi = min(g0 + (uint32_t)lane, glim);
      if (inner == 0ull) {  // the row lies inside one push: SGPR bases
        key = *(const AS1 uint64_t*)(kp0 + 8ull * gi);
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          val[mi] = *(const AS1 V*)(vp0[mi] + sizeof(V) * (uint64_t)gi);
      } else {  // pushes start inside the row: per-lane bases
        uint64_t kp = kp0;
        uint64_t vp[M];
#pragma unroll
        for (int mi = 0; mi < M; ++mi) vp[mi] = vp0[mi];
        for (uint64_t in2 = inner; in2; in2 &= in2 - 1) {
          const uint32_t q = (uint32_t)__builtin_ctzll(in2);
          const bool ge = gi >= (uint32_t)__builtin_amdgcn_readlane(excl, q);
          kp = ge ? readlane64(kb, q) : kp;
#pragma unroll
          for (int mi = 0; mi < M; ++mi) vp[mi] = ge ? readlane64(vb[mi], q) : vp[mi];
        }
        key = *(const AS1 uint64_t*)(kp + 8ull * gi);
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          val[mi] = *(const AS1 V*)(vp[mi] + sizeof(V) * (uint64_t)gi);
      }
    };

    uint64_t rk[R];
    V rv[R][M];
#pragma unroll
    for (int q = 0; q < R; ++q) load_row((uint32_t)q, rk[q], rv[q]);

    // ---- results of the previous sub-tile leave while the loads fly
    if (jsub > 0) store_sub(jsub - 1);

    // ---- install: accumulators, bucket histogram (in dk) -> scan -> btab, D
    if (cont) {  // rare: continue the sums of an earlier launch
      for (uint32_t s = (uint32_t)lane; s < (uint32_t)C; s += 64u) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          acc[mi * C + s] = s < ntj ? G(out_of(mi) + base)[s] : V(0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < SPL; ++i) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) acc[mi * C + i * 64 + lane] = V(0);
      }
    }
    uint32_t* hist = (uint32_t*)dk;
    for (int i = lane; i < NB + 4; i += 64) hist[i] = 0u;
    {
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      const u4 z = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < C / 1024; ++i) ((u4*)lastl)[i * 64 + lane] = z;
      if constexpr (C < 1024) {
        if (lane < C / 16) ((u4*)lastl)[lane] = z;
      }
    }
    __syncthreads();
    const uint64_t klo = readlane64(dreg[0], 0);
    const uint64_t range = khi - klo;
    const int bits = range ? 64 - __builtin_clzll(range) : 0;
    const int shift = bits > LNB ? bits - LNB : 0;
#pragma unroll
    for (int i = 0; i < SPL; ++i) {
      // D is sorted, so (k - klo) >> shift < NB needs no clamp; the clamped
      // copies past ntj count into a spare cell
      const uint32_t s = (uint32_t)(i * 64 + lane);
      const uint32_t b = (uint32_t)((dreg[i] - klo) >> shift) + 1u;
      __hip_atomic_fetch_add(&hist[s < ntj ? b : (uint32_t)(NB + 2)], 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    {
      // btab[b] = slots with bucket < b = inclusive scan of hist (count of
      // bucket b sits at b + 1)
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      const u4* hp = (const u4*)&hist[lane * EPL];
      uint32_t v[EPL];
#pragma unroll
      for (int i = 0; i < EPL / 4; ++i) {
        const u4 c = hp[i];
        v[4 * i] = c.x;
        v[4 * i + 1] = c.y;
        v[4 * i + 2] = c.z;
        v[4 * i + 3] = c.w;
      }
#pragma unroll
      for (int i = 1; i < EPL; ++i) v[i] += v[i - 1];
      uint32_t x = v[EPL - 1];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
      }
      const uint32_t bs = x - v[EPL - 1];
      u4* bp = (u4*)&btab[lane * EPL];
#pragma unroll
      for (int i = 0; i < EPL / 8; ++i) {
        u4 w;
        w.x = (v[8 * i] + bs) | ((v[8 * i + 1] + bs) << 16);
        w.y = (v[8 * i + 2] + bs) | ((v[8 * i + 3] + bs) << 16);
        w.z = (v[8 * i + 4] + bs) | ((v[8 * i + 5] + bs) << 16);
        w.w = (v[8 * i + 6] + bs) | ((v[8 * i + 7] + bs) << 16);
        bp[i] = w;
      }
      if (lane == 0) btab[NB] = (uint16_t)ntj;
    }
    __syncthreads();  // histogram read before D overwrites it
#pragma unroll
    for (int i = 0; i < SPL; ++i) dk[i * 64 + lane] = dreg[i];
    // candidates past the sub-tile read ~0 (never below a key)
    for (uint32_t i = ntj + (uint32_t)lane; i < (uint32_t)C + 8u; i += 64u) dk[i] = ~0ull;
    __syncthreads();
    auto bucket = [&](uint64_t k) -> uint32_t {
      const uint64_t bb = (k - klo) >> shift;
      return bb < (uint64_t)NB ? (uint32_t)bb : (uint32_t)(NB - 1);
    };

    // ---- process rows in order
    int carry = -1;
    auto process_row = [&](uint32_t r, uint64_t key, const V (&val)[M]) {
      const uint32_t g0 = r << 6;
      const uint32_t q0 = row_first(g0);
      const uint64_t inner = row_inner(g0);
      const uint64_t actm = lane_range(0u, total - g0 < 64u ? total - g0 : 64u);
      // slot search: bucket -> [l, l + n) -> (binary narrowing) -> 4 candidates
      const uint32_t b = bucket(key);
      uint32_t l = btab[b];
      uint32_t n = (uint32_t)btab[b + 1] - l;
      while (n > 4u) {
        const uint32_t half = n >> 1;
        if (dk[l + half - 1] < key) {
          l += half;
          n -= half;
        } else {
          n = half;
        }
      }
      const uint64_t c0 = dk[l], c1 = dk[l + 1], c2 = dk[l + 2], c3 = dk[l + 3];
      const uint32_t pos = l + (c0 < key ? 1u : 0u) + (c1 < key ? 1u : 0u) +
                           (c2 < key ? 1u : 0u) + (c3 < key ? 1u : 0u);
      const bool found = (c0 == key) | (c1 == key) | (c2 == key) | (c3 == key);
      // order check: each push segment's first key compares with -1, the
      // row's lane 0 with the previous row's lane 63 (same push)
      uint64_t starts = (uint32_t)__builtin_amdgcn_readlane(excl, q0) == g0 ? 1ull : 0ull;
      for (uint64_t in2 = inner; in2; in2 &= in2 - 1) {
        const uint32_t q = (uint32_t)__builtin_ctzll(in2);
        starts |= 1ull << ((uint32_t)__builtin_amdgcn_readlane(excl, q) - g0);
      }
      const int prev_in = __builtin_amdgcn_update_dpp(carry, (int)pos, 0x138, 0xf, 0xf, false);
      const int prev = __builtin_amdgcn_inverse_ballot_w64(starts) ? -1 : prev_in;
      const uint64_t okm = __ballot(found && (int)pos > prev) & actm;
      const uint64_t badm = actm & ~okm;
      // fold push by push (arrival order inside the row)
      uint32_t q = q0, a0 = 0;
      uint64_t rest = inner;
      for (;;) {
        uint32_t a1 = 64u, qn = 0u;
        if (rest) {
          qn = (uint32_t)__builtin_ctzll(rest);
          rest &= rest - 1;
          a1 = (uint32_t)__builtin_amdgcn_readlane(excl, qn) - g0;
        }
        const uint64_t segm = lane_range(a0, a1);
        if (__builtin_amdgcn_inverse_ballot_w64(segm & okm)) {
          const uint32_t l1 = lastl[pos];
          const bool gap = l1 < (q & qs_mask);  // absent since the last contribution
          const bool first = q == 0u && !cont;  // the first push is assigned
#pragma unroll
          for (int mi = 0; mi < M; ++mi) {
            const V a = acc[mi * C + pos];
            const V a1v = gap ? a + V(0) : a;
            acc[mi * C + pos] = first ? val[mi] : a1v + val[mi];
          }
          lastl[pos] = (uint8_t)(q + 1u);
        }
        const uint32_t nbad = (uint32_t)__builtin_popcountll(segm & badm);
        if (nbad && lane == 0) nfail[q] += nbad;
        if (a1 >= 64u) break;
        a0 = a1;
        q = qn;
      }
      carry = __builtin_amdgcn_readlane((int)pos, 63);
    };

    // whole chunks of R rows (each step refills its register set R rows
    // ahead), then the last < R rows with no further loads: no step leaves
    // the loop early, so the wait counts stay exact on every path
    uint32_t r0 = 0;
    for (; r0 + R <= nrows; r0 += R) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        process_row(r0 + q, rk[q], rv[q]);
        load_row(r0 + q + R, rk[q], rv[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < R; ++q)
      if (r0 + q < nrows) process_row(r0 + q, rk[q], rv[q]);
    __syncthreads();
  }
  store_sub(nsub - 1);
  if ((uint32_t)lane < np && nfail[lane])
    __hip_atomic_fetch_add(GW(T.fail) + lane, (unsigned long long)nfail[lane], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

template <typename V, int M, int C, int R, int WPS>
hipError_t go(const TileDesc* t, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL((rows_kernel<V, M, C, R, WPS>), dim3(n), dim3(64), 0, s, t);
  return hipGetLastError();
}

template <typename V, int M>
hipError_t launch_m(int C, const TileDesc* t, uint32_t n, hipStream_t s) {
  static const int rr = [] {
    const char* e = getenv("PSG_ROWS_R");  // benchmarking aid: rows in flight
    return e ? atoi(e) : 8;
  }();
  if (C == 2048) return go<V, M, 2048, 8, 1>(t, n, s);
  if (C == 512) return rr == 4 ? go<V, M, 512, 4, 4>(t, n, s) : go<V, M, 512, 8, 4>(t, n, s);
  if (C == 256) return go<V, M, 256, 4, 8>(t, n, s);
  if (rr == 4) return go<V, M, 1024, 4, 2>(t, n, s);
  if (rr == 6) return go<V, M, 1024, 6, 2>(t, n, s);
  return go<V, M, 1024, 8, 2>(t, n, s);
}

template <typename V>
hipError_t launch_v(int m, int C, const TileDesc* t, uint32_t n, hipStream_t s) {
  switch (m) {
    case 1: return launch_m<V, 1>(C, t, n, s);
    case 2: return launch_m<V, 2>(C, t, n, s);
    case 3: return launch_m<V, 3>(C, t, n, s);
    case 4: return launch_m<V, 4>(C, t, n, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

int rows_tile() {
  static const int c = [] {
    const char* e = getenv("PSG_ROWS_TILE");  // benchmarking aid: 1024 / 2048
    const int v = e ? atoi(e) : 1024;
    return (v == 2048 || v == 512 || v == 256) ? v : 1024;
  }();
  return c;
}

hipError_t launch_aggregate_rows(int dtype, int m, const TileDesc* d_tiles, uint32_t ncoarse,
                                 hipStream_t stream) {
  if (ncoarse == 0) return hipSuccess;
  const int C = rows_tile();
  return dtype == 0 ? launch_v<float>(m, C, d_tiles, ncoarse, stream)
                    : launch_v<double>(m, C, d_tiles, ncoarse, stream);
}

}  // namespace psg
