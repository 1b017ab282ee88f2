// psg_stream.hip -- streaming aggregate kernel (v6): one wave per coarse
// range of server slots, fine tiles walked in key order, pushes folded in
// arrival order straight into an LDS accumulator.
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267): out[j] = fold over pushes p in arrival
// order of V_p[k] where S_p[k] == D[lo+j]; the first push assigns, later
// pushes add, and the serial path adds an explicit +0.0 for absent pushes.
//
// Structure (DESIGN.md "Kernels"):
//   * a workgroup is ONE wave (64 lanes): no s_barrier anywhere; LDS
//     accesses of a wave are ordered, so the sequential per-push fold below
//     is race-free and in push order by construction;
//   * the wave owns a coarse range of <= 16 fine tiles x 256 slots; the
//     partition kernel only finds the coarse boundaries (one per 4096
//     slots).  Lane p keeps push p's cursor and coarse end;
//   * per fine tile, push p's next 64 keys are one wave load; a ballot
//     against the next tile's first key gives exactly how many belong to
//     this tile (sorted pushes: a prefix), so the fine boundaries fall out of
//     data the tile needs anyway;
//   * slot search: 64-bucket table over the fine tile's key range, 4 LDS
//     probes for windows <= 8 slots, full 9-probe search otherwise;
//   * order check on slot positions (shuffle within a window, carry across
//     windows): all keys matched + strictly increasing slots <=> the push is
//     sorted, unique and inside the range (reference matched == n);
//   * software pipeline: right after a tile's ballots, the next tile's D keys
//     and first windows are issued into a second register set, so HBM
//     streams under the search/fold of the current tile.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "psg_device.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))

namespace psg {

namespace {

constexpr int kFT = 256;            // fine tile slots (4 per lane)
constexpr int kNB = 64;             // buckets per fine tile
constexpr int kStreamCT = 16;       // fine tiles per coarse range
constexpr uint32_t kInvPos = 0xFFFFFFFFu;
static_assert(kFT * kStreamCT == 4096, "coarse tile = 4096 slots");

template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}
template <typename T>
__device__ __forceinline__ AS1 T* GW(T* p) {
  return (AS1 T*)p;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

template <int N>
__device__ __forceinline__ uint32_t lb_pow2(const uint64_t* a, uint32_t off, uint64_t k) {
  // lower_bound in a[off .. off + N] (N power of two), byte offsets
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

template <typename V, int M, int NPW>
struct Staged {
  uint64_t dreg[4];   // D keys of the tile: slots lane + 64k
  uint64_t bkey;      // first key of the following tile (or ~0)
  uint64_t wk[NPW];   // window keys, push q of the first batch, lane = offset
  V wv[NPW][M];
  uint32_t wc[NPW];   // window start (uniform)
  uint32_t wn[NPW];   // window valid lanes (uniform)
};

// Design knobs (benchmarked variants; see launch_sm):
//   BT: bucket table by one 9-probe search per bucket (0) or slot transitions (1)
//   PH: per push search+check+fold fused (0) or phased over the batch (1)
//   PF: prefetch the next tile under the current one (1) or not (0)
template <typename V, int M, int NPW, int BT, int PH, int PF>
__global__ __launch_bounds__(64) void stream_kernel(const TileDesc* __restrict__ tiles) {
  __shared__ uint64_t dk[kFT + 8];
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

  // lane p: push p's cursor, coarse end, pointers
  uint32_t cur = 0, cend = 0;
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
  }
  if (lane < 8) dk[kFT + lane] = ~0ull;
  const uint32_t nb0 = np < (uint32_t)NPW ? np : (uint32_t)NPW;

  auto load_d = [&](Staged<V, M, NPW>& s, uint32_t ft) {
    const uint32_t base = ft * kFT;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = base + (uint32_t)lane + 64u * k;
      s.dreg[k] = i < ncs ? G(Dg)[i] : ~0ull;
    }
    s.bkey = (ft + 1 < nft) ? G(Dg)[base + kFT] : ~0ull;
  };
  auto load_window = [&](uint64_t& wk, V (&wv)[M], uint32_t& wc, uint32_t& wn, uint32_t p) {
    const uint32_t c = __builtin_amdgcn_readlane(cur, p);
    const uint32_t e = __builtin_amdgcn_readlane(cend, p);
    const uint32_t n = e - c < 64u ? e - c : 64u;
    wc = c;
    wn = n;
    const uint64_t* sk = (const uint64_t*)readlane64(kp, p);
    const bool act = (uint32_t)lane < n;
    const uint32_t i = act ? c + lane : c;  // clamped: always a valid address when n > 0
    wk = (act) ? G(sk)[i] : ~0ull;
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      const V* sv = (const V*)readlane64(vp[mi], p);
      wv[mi] = act ? G(sv)[i] : V(0);
    }
  };
  auto load_batch0 = [&](Staged<V, M, NPW>& s) {
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      if ((uint32_t)q < nb0) load_window(s.wk[q], s.wv[q], s.wc[q], s.wn[q], q);
      else { s.wk[q] = ~0ull; s.wn[q] = 0; s.wc[q] = 0; }
    }
  };

  Staged<V, M, NPW> A, B;
  if (nft > 0) {
    load_d(A, 0);
    load_batch0(A);
  }

  for (uint32_t ft = 0; ft < nft; ++ft) {
    const uint32_t base = ft * kFT;
    const int nt = (int)(ncs - base < (uint32_t)kFT ? ncs - base : (uint32_t)kFT);
    const uint64_t bound = A.bkey;
    const bool last_tile = ft + 1 == nft;  // takes every element up to the coarse end
    V* outp[M];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) outp[mi] = (V*)T.out[mi] + T.slot0 + base;

    // ---- install the tile: D keys, accumulators, bucket table
#pragma unroll
    for (int k = 0; k < 4; ++k) dk[lane + 64 * k] = A.dreg[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = lane * 4 + j;
      lastl[s] = -1;
#pragma unroll
      for (int mi = 0; mi < M; ++mi) acc[mi * kFT + s] = (cont && s < nt) ? G(outp[mi])[s] : V(0);
    }
    // lanes read slots other lanes wrote: order the LDS accesses (the
    // compiler reasons per thread; for a one-wave workgroup this is cheap)
    __syncthreads();
    const uint64_t klo =
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)A.dreg[0]) |
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(A.dreg[0] >> 32)) << 32);
    const uint64_t khi = dk[nt - 1];
    const uint64_t range = khi - klo;
    const int bits = range ? 64 - __builtin_clzll(range) : 0;
    const int shift = bits > 6 ? bits - 6 : 0;
    if constexpr (BT == 0) {
      const uint64_t d = (uint64_t)lane << shift;
      const uint64_t key = d > ~0ull - klo ? ~0ull : klo + d;
      const uint32_t sb = lb_pow2<kFT>(dk, 0, key);
      btab[lane] = sb < (uint32_t)nt ? sb : (uint32_t)nt;
      if (lane == 0) btab[kNB] = (uint32_t)nt;
    } else {
      // btab[b] = first slot whose bucket >= b: every slot whose bucket is
      // larger than its predecessor's writes the buckets it opens; the last
      // slot closes the table up to kNB (btab[kNB] = nt).
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int sidx = lane + 64 * k;
        if (sidx < nt) {
          const int bcur = (int)((A.dreg[k] - klo) >> shift);
          const int bprev = sidx == 0 ? -1 : (int)((dk[sidx - 1] - klo) >> shift);
          for (int b = bprev + 1; b <= bcur; ++b) btab[b] = (uint32_t)sidx;
          if (sidx == nt - 1)
            for (int b = bcur + 1; b <= kNB; ++b) btab[b] = (uint32_t)nt;
        }
      }
    }

    __syncthreads();
    // ---- ballots of the first batch: how much of each window is this tile's
    uint32_t L[NPW];
    bool more = false;  // some window ended inside this tile's range
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      const bool inb = (uint32_t)lane < A.wn[q] && (last_tile || A.wk[q] < bound);
      const unsigned long long bal = __ballot(inb);
      const uint32_t pre = (~bal == 0ull) ? 64u : (uint32_t)__builtin_ctzll(~bal);
      L[q] = pre;
      more = more || (pre == 64u && A.wn[q] == 64u && A.wc[q] + 64u < __builtin_amdgcn_readlane(cend, q));
      if (lane == q) cur = A.wc[q] + pre;
    }
    // ---- prefetch the next tile under this tile's search + fold
    const bool pref = PF && !more && np <= (uint32_t)NPW && ft + 1 < nft;
    if (pref) {
      load_d(B, ft + 1);
      load_batch0(B);
    }

    // ---- process pushes in arrival order
    auto process = [&](uint64_t key, const V (&val)[M], uint32_t Lq, uint32_t p,
                       int& carry) -> uint32_t {
      // returns the number of failed elements (uniform)
      const bool act = (uint32_t)lane < Lq;
      const uint64_t k = act ? key : ~0ull;
      const uint64_t dlt = k - klo;
      const uint32_t b = (k < klo) ? 0u : (dlt >> shift) < (uint64_t)kNB ? (uint32_t)(dlt >> shift) : (uint32_t)kNB;
      const uint32_t lo = btab[b];
      const uint32_t hi = btab[b < (uint32_t)kNB ? b + 1 : b];
      uint32_t pos;
      if (hi - lo <= 8u) pos = lb_pow2<8>(dk, lo, k);
      else pos = lb_pow2<kFT>(dk, 0, k);
      const uint32_t prev_in = __shfl_up(pos, 1, 64);
      const int prev = lane == 0 ? carry : (int)prev_in;
      const bool ok = act && (int)pos < nt && dk[pos] == k && prev < (int)pos;
      if (ok) {
        const int lp = lastl[pos];
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          acc[mi * kFT + pos] = fold1<V>(acc[mi * kFT + pos], lp, (int)p, val[mi], parallel, cont);
        lastl[pos] = (int16_t)p;
      }
      if (Lq > 0) carry = (int)__shfl(pos, (int)Lq - 1, 64);
      const unsigned long long bad = __ballot(act && !ok);
      return (uint32_t)__popcll(bad);
    };
    auto extra_windows = [&](uint32_t p, uint32_t c, int& carry) {
      // push p filled a whole window inside this tile: keep streaming it
      uint32_t fails = 0;
      for (;;) {
        const uint32_t e = __builtin_amdgcn_readlane(cend, p);
        if (c >= e) break;
        uint64_t wk;
        V wv[M];
        uint32_t wc, wn;
        if (lane == (int)p) cur = c;
        load_window(wk, wv, wc, wn, p);
        const bool inb = (uint32_t)lane < wn && (last_tile || wk < bound);
        const unsigned long long bal = __ballot(inb);
        const uint32_t pre = (~bal == 0ull) ? 64u : (uint32_t)__builtin_ctzll(~bal);
        fails += process(wk, wv, pre, p, carry);
        c = wc + pre;
        if (lane == (int)p) cur = c;
        if (!(pre == 64u && wn == 64u)) break;
      }
      return fails;
    };
    if constexpr (PH == 0) {
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      if ((uint32_t)q < nb0) {
        int carry = -1;
        uint32_t fails = process(A.wk[q], A.wv[q], L[q], q, carry);
        if (L[q] == 64u && A.wn[q] == 64u)
          fails += extra_windows(q, A.wc[q] + 64u, carry);
        if (fails && lane == 0)
          __hip_atomic_fetch_add(GW(T.fail) + q, (unsigned long long)fails,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    } else {
    // first batch in three phases: (a) every slot search (independent,
    // interleaved), (b) order checks, (c) the in-order fold (short LDS
    // read-modify-write chain per push)
    uint32_t pos[NPW];
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      const bool act = (uint32_t)lane < L[q];
      const uint64_t k = act ? A.wk[q] : ~0ull;
      const uint64_t dlt = k - klo;
      const uint32_t b = (k < klo) ? 0u : (dlt >> shift) < (uint64_t)kNB ? (uint32_t)(dlt >> shift) : (uint32_t)kNB;
      const uint32_t lo = btab[b];
      const uint32_t hi = btab[b < (uint32_t)kNB ? b + 1 : b];
      pos[q] = (hi - lo <= 8u) ? lb_pow2<8>(dk, lo, k) : kInvPos;
    }
#pragma unroll
    for (int q = 0; q < NPW; ++q)
      if (pos[q] == kInvPos) pos[q] = lb_pow2<kFT>(dk, 0, (uint32_t)lane < L[q] ? A.wk[q] : ~0ull);
    bool okq[NPW];
    bool needx = false;
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      const bool act = (uint32_t)lane < L[q];
      const uint32_t prev_in = __shfl_up(pos[q], 1, 64);
      const int prev = lane == 0 ? -1 : (int)prev_in;
      okq[q] = act && (int)pos[q] < nt && dk[pos[q]] == A.wk[q] && prev < (int)pos[q];
      const unsigned long long bad = __ballot(act && !okq[q]);
      if (bad && lane == 0)
        __hip_atomic_fetch_add(GW(T.fail) + q, (unsigned long long)__popcll(bad),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      needx = needx || (L[q] == 64u && A.wn[q] == 64u);
    }
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      if (okq[q]) {
        const uint32_t ps = pos[q];
        const int lp = lastl[ps];
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          acc[mi * kFT + ps] = fold1<V>(acc[mi * kFT + ps], lp, q, A.wv[q][mi], parallel, cont);
        lastl[ps] = (int16_t)q;
      }
      if (needx && L[q] == 64u && A.wn[q] == 64u) {
        // push q filled a window inside this tile (dense data): stream the
        // rest of it before push q+1 (arrival order)
        int carry = (int)__shfl(pos[q], 63, 64);
        const uint32_t fails = extra_windows(q, A.wc[q] + 64u, carry);
        if (fails && lane == 0)
          __hip_atomic_fetch_add(GW(T.fail) + q, (unsigned long long)fails,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    }
    for (uint32_t p = NPW; p < np; ++p) {  // later pushes: streamed directly
      int carry = -1;
      const uint32_t fails = extra_windows(p, __builtin_amdgcn_readlane(cur, p), carry);
      if (fails && lane == 0)
        __hip_atomic_fetch_add(GW(T.fail) + p, (unsigned long long)fails,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

    if (ft + 1 < nft) {
      if (pref) {
        A = B;
      } else {
        load_d(A, ft + 1);
        load_batch0(A);
      }
    }
  }
}

template <typename V, int M>
hipError_t launch_sm(const TileDesc* t, uint32_t n, hipStream_t s) {
  if constexpr (sizeof(V) == 4 && M == 1) {
    static const int variant = [] {
      const char* e = getenv("PSG_STREAM_VARIANT");  // benchmarking aid
      return e ? atoi(e) : 0;
    }();
    switch (variant) {
      case 1: hipLaunchKernelGGL((stream_kernel<V, M, 8, 1, 0, 1>), dim3(n), dim3(64), 0, s, t); return hipGetLastError();
      case 2: hipLaunchKernelGGL((stream_kernel<V, M, 8, 0, 1, 1>), dim3(n), dim3(64), 0, s, t); return hipGetLastError();
      case 3: hipLaunchKernelGGL((stream_kernel<V, M, 8, 1, 1, 1>), dim3(n), dim3(64), 0, s, t); return hipGetLastError();
      case 4: hipLaunchKernelGGL((stream_kernel<V, M, 8, 0, 0, 0>), dim3(n), dim3(64), 0, s, t); return hipGetLastError();
      case 5: hipLaunchKernelGGL((stream_kernel<V, M, 4, 0, 0, 1>), dim3(n), dim3(64), 0, s, t); return hipGetLastError();
      default: break;
    }
  }
  hipLaunchKernelGGL((stream_kernel<V, M, 8, 0, 0, 1>), dim3(n), dim3(64), 0, s, t);
  return hipGetLastError();
}

template <typename V>
hipError_t launch_sv(int m, const TileDesc* t, uint32_t n, hipStream_t s) {
  switch (m) {
    case 1: return launch_sm<V, 1>(t, n, s);
    case 2: return launch_sm<V, 2>(t, n, s);
    case 3: return launch_sm<V, 3>(t, n, s);
    case 4: return launch_sm<V, 4>(t, n, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_stream(int dtype, int m, const TileDesc* d_tiles,
                                   uint32_t ncoarse, hipStream_t stream) {
  if (ncoarse == 0) return hipSuccess;
  return dtype == 0 ? launch_sv<float>(m, d_tiles, ncoarse, stream)
                    : launch_sv<double>(m, d_tiles, ncoarse, stream);
}

}  // namespace psg
