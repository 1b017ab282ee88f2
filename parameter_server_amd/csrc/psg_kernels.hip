// psg_kernels.hip -- hand-written gfx950 (CDNA4) kernels of the server-side
// push aggregation path.  No MFMA: this is an integer merge + float
// segmented sum, bound by HBM bandwidth (DESIGN.md "Kernels").
//
// Reference semantics restated here (wakensky/parameter_server):
//   aggregate  <- KVVector::serialSetValue / parallelSetValue
//                 (src/parameter/kv_vector.h:84-137, 171-204) built on
//                 oldMatch / match (src/system/message.h:134-267)
//   partition  <- SArray::findRange + sliceKeyOrderedMsg lower_bounds
//                 (src/base/shared_array_inl.h:164-171, message.h:96-99)
//   gather     <- KVVector::serialGetValue (kv_vector.h:215-227)
//   union      <- SArray::setUnion (shared_array_inl.h:155-162)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_internal.h"

namespace psg {

namespace {

constexpr uint32_t kInvalid = 0xFFFFFFFFu;

// ----------------------------------------------------------------------
// wave-cooperative k-ary search: first index i in [0, n) whose key
// satisfies (upper ? S[i] > key : S[i] >= key); n if none.  64 probes per
// round -> ceil(log64 n)+1 dependent global loads instead of log2 n.
// Every lane of the wave must call it with the same arguments.
// ----------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_search(const uint64_t* __restrict__ S,
                                                uint64_t n, uint64_t key,
                                                bool upper, int lane) {
  uint64_t lo = 0, hi = n;  // answer in [lo, hi]
  while (hi > lo) {
    const uint64_t len = hi - lo;
    const uint64_t step = (len + 63) >> 6;
    const uint64_t idx = lo + (uint64_t)(lane + 1) * step - 1;
    bool pred = true;  // probes past the range count as "true"
    if (idx < hi) {
      const uint64_t s = S[idx];
      pred = upper ? (s > key) : (s >= key);
    }
    const unsigned long long mask = __ballot(pred);
    if (mask == 0) {
      lo = hi;
      break;
    }
    const uint64_t f = (uint64_t)(__ffsll((long long)mask) - 1);
    const uint64_t nlo = lo + f * step;
    uint64_t nhi = lo + (f + 1) * step - 1;
    if (nhi > hi) nhi = hi;
    lo = nlo;
    hi = nhi;
  }
  return lo;
}

// lower_bound over a sorted LDS array of n <= 2*kTile-1 keys: fixed trip
// count (12 probes), so the wave never diverges on the loop itself.
__device__ __forceinline__ int lds_lower_bound(const uint64_t* a, int n,
                                               uint64_t k) {
  int pos = 0;
#pragma unroll
  for (int step = kTile; step > 0; step >>= 1) {
    const int c = pos + step;
    if (c <= n && a[c - 1] < k) pos = c;
  }
  return pos;
}

__device__ __forceinline__ uint64_t gl_lower_bound(const uint64_t* __restrict__ a,
                                                   uint64_t n, uint64_t k) {
  uint64_t lo = 0, len = n;
  while (len > 0) {
    const uint64_t half = len >> 1;
    if (a[lo + half] < k) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo;
}

// Exclusive scan across a kThreads workgroup.  wsum: LDS scratch of
// kThreads/64 words.  Contains two barriers; callers separate consecutive
// uses with a barrier of their own.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum,
                                                    uint32_t* total) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  constexpr int kW = kThreads / 64;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    uint32_t s = lane < kW ? wsum[lane] : 0u;
#pragma unroll
    for (int d = 1; d < kW; d <<= 1) {
      const uint32_t y = __shfl_up(s, d, 64);
      if (lane >= d) s += y;
    }
    if (lane < kW) wsum[lane] = s;
  }
  __syncthreads();
  *total = wsum[kW - 1];
  return (w > 0 ? wsum[w - 1] : 0u) + x - v;
}

// One step of the per-key fold in push-arrival order.  p = push index in
// this launch, lp = last push index in this launch that held the key (-1:
// none yet).  Serial (the reference default) adds +0.0 for every absent
// later push (kv_vector.h:200); since x + 0.0 == x except -0.0 -> +0.0 and
// the operation is idempotent, one "+ 0" per run of absent pushes is exact.
template <typename V>
__device__ __forceinline__ V fold_step(V acc, int lp, int p, V v,
                                       bool parallel, bool cont) {
  if (p == 0 && !cont) return v;  // the first push is assigned (:195-196)
  if (!parallel) {
    const bool gap = (lp >= 0) ? (p - lp > 1) : (cont && p > 0);
    if (gap) acc = acc + V(0);
  }
  return acc + v;
}

template <typename V>
struct AggSmem {
  uint64_t dk[kTile];            // server keys of this tile
  uint64_t mask[kTile];          // bit b: push pf+b holds this key (this chunk)
  uint32_t base[kTile];          // exclusive prefix of popcount(mask)
  V sorted[kChunk];              // chunk values in (slot, push) order
  uint32_t pstart[kMaxPush + 1]; // element offset of each push's segment
  uint32_t segb[kMaxPush];       // first index of each push's segment
  uint32_t wsum[kThreads / 64];
};

// ----------------------------------------------------------------------
// partition: one wave per (job, tile boundary b, push p).
// ----------------------------------------------------------------------
__global__ __launch_bounds__(256) void partition_kernel(
    const JobDev* __restrict__ jobs, int njobs, uint32_t nitems) {
  const uint32_t item = (blockIdx.x * 256u + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (item >= nitems) return;
  int jlo = 0, jhi = njobs - 1;
  while (jlo < jhi) {
    const int mid = (jlo + jhi + 1) >> 1;
    if (jobs[mid].part_begin <= item) jlo = mid; else jhi = mid - 1;
  }
  const JobDev& J = jobs[jlo];
  const uint32_t local = item - J.part_begin;
  const uint32_t b = local / J.npush;
  const uint32_t p = local - b * J.npush;
  uint64_t res = 0;
  if (J.nslots > 0) {
    const bool upper = (b == J.ntiles);
    const uint64_t key =
        upper ? J.dkeys[J.nslots - 1] : J.dkeys[(uint64_t)b * kTile];
    res = wave_search(J.pkeys[p], J.pn[p], key, upper, lane);
  }
  if (lane == 0) {
    J.seg[local] = (uint32_t)res;
    if (b == 0) J.fail[p] = 0ull;  // the aggregate launch follows in-stream
  }
}

// ----------------------------------------------------------------------
// aggregate: one workgroup per tile of kTile server slots.
//
//  1. D tile -> LDS; push segments of the tile (from partition) -> LDS
//     prefix table.
//  2. Chunks of <= kChunk push elements spanning <= kGroup pushes: each
//     lane loads (key, values) coalesced, checks strict order against its
//     predecessor (shuffle / one load at wave edges), finds the slot by a
//     12-probe LDS lower_bound and sets bit (p - pf) of mask[slot] with an
//     LDS atomic OR.
//  3. popcount(mask) -> workgroup scan -> base; each element's rank =
//     base[slot] + popcount(mask[slot] below its bit): the (slot, push)
//     order, i.e. a stable counting sort with no atomics on values.
//  4. Each thread folds its kSPT slots' contributions in push order into
//     registers (bit-exact reference order), across chunks.
//  5. One coalesced store per thread of its kSPT sums.
// ----------------------------------------------------------------------
template <typename V, int M>
__global__ __launch_bounds__(kThreads, 2) void aggregate_kernel(
    const JobDev* __restrict__ jobs, int njobs) {
  __shared__ AggSmem<V> sm;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const uint32_t g = blockIdx.x;

  int jlo = 0, jhi = njobs - 1;
  while (jlo < jhi) {
    const int mid = (jlo + jhi + 1) >> 1;
    if (jobs[mid].tile_begin <= g) jlo = mid; else jhi = mid - 1;
  }
  const JobDev* __restrict__ J = &jobs[jlo];
  const uint32_t t = g - J->tile_begin;
  const uint32_t np = J->npush;
  const uint64_t slot0 = (uint64_t)t * kTile;
  const uint64_t rem = J->nslots - slot0;
  const int nt = rem < (uint64_t)kTile ? (int)rem : kTile;
  const bool parallel = (J->flags & kFlagParallel) != 0;
  const bool cont = (J->flags & kFlagCont) != 0;

  // 1. server keys of the tile, push segments
  {
    const uint64_t* __restrict__ dk = J->dkeys + slot0;
    for (int i = tid; i < nt; i += kThreads) sm.dk[i] = dk[i];
  }
  uint32_t myseg = 0;
  if ((uint32_t)tid < np) {
    const uint32_t b = J->seg[(size_t)t * np + tid];
    const uint32_t e = J->seg[(size_t)(t + 1) * np + tid];
    sm.segb[tid] = b;
    myseg = e - b;
  }
  uint32_t E;
  {
    const uint32_t ex = block_excl_scan(myseg, sm.wsum, &E);
    if ((uint32_t)tid < np) sm.pstart[tid] = ex;
    if (tid == 0) sm.pstart[np] = E;
  }

  const int s0 = tid * kSPT;
  V acc[M][kSPT];
  int lastp[kSPT];
  V* outp[M];
#pragma unroll
  for (int mi = 0; mi < M; ++mi) outp[mi] = (V*)J->out[mi] + slot0;
#pragma unroll
  for (int j = 0; j < kSPT; ++j) {
    lastp[j] = -1;
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
      acc[mi][j] = (cont && s0 + j < nt) ? outp[mi][s0 + j] : V(0);
  }
  __syncthreads();

  for (uint32_t e0 = 0; e0 < E;) {
    // push containing e0: largest p < np with pstart[p] <= e0
    uint32_t pf;
    {
      int lo = 0, hi = (int)np - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sm.pstart[mid] <= e0) lo = mid; else hi = mid - 1;
      }
      pf = (uint32_t)lo;
    }
    const uint32_t pl = (pf + kGroup < np) ? pf + kGroup : np;
    uint32_t e1 = e0 + kChunk;
    if (e1 > E) e1 = E;
    if (e1 > sm.pstart[pl]) e1 = sm.pstart[pl];

    for (int i = tid; i < nt; i += kThreads) sm.mask[i] = 0ull;
    __syncthreads();

    // 2. locate every element of the chunk
    uint32_t rec[kEPT];
    V vv[kEPT][M];
#pragma unroll
    for (int r = 0; r < kEPT; ++r) {
      const uint32_t e = e0 + (uint32_t)tid + (uint32_t)r * kThreads;
      const bool act = e < e1;
      uint32_t p = pf, li = 0;
      uint64_t key = 0, i = 0;
      rec[r] = kInvalid;
#pragma unroll
      for (int mi = 0; mi < M; ++mi) vv[r][mi] = V(0);
      if (act) {
        int lo = (int)pf, hi = (int)pl - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (sm.pstart[mid] <= e) lo = mid; else hi = mid - 1;
        }
        p = (uint32_t)lo;
        li = e - sm.pstart[p];
        i = (uint64_t)sm.segb[p] + li;
        key = J->pkeys[p][i];
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          vv[r][mi] = ((const V*)J->pvals[(size_t)p * M + mi])[i];
      }
      const uint64_t prevk = __shfl_up(key, 1, 64);
      const uint32_t prevp = __shfl_up(p, 1, 64);
      if (act) {
        bool ok = true;
        if (i > 0) {  // strict order vs the push's previous key (kv_vector.h:134,192)
          const uint64_t pk = (li > 0 && lane > 0 && prevp == p)
                                  ? prevk
                                  : J->pkeys[p][i - 1];
          ok = pk < key;
        }
        const uint32_t L = sm.pstart[p + 1] - sm.pstart[p];
        int pos;
        if (L == (uint32_t)nt && sm.dk[li] == key)
          pos = (int)li;  // dense segment: the slot is the offset
        else
          pos = lds_lower_bound(sm.dk, nt, key);
        ok = ok && pos < nt && sm.dk[pos] == key;
        if (ok) {
          const unsigned long long bit = 1ull << (p - pf);
          const unsigned long long old =
              atomicOr((unsigned long long*)&sm.mask[pos], bit);
          ok = (old & bit) == 0ull;
        }
        if (ok)
          rec[r] = (uint32_t)pos | ((p - pf) << 16);
        else
          atomicAdd(&J->fail[p], 1ull);
      }
    }
    __syncthreads();

    // 3. per-slot contribution counts -> ranks
    unsigned long long mymask[kSPT];
    uint32_t mybase[kSPT];
    {
      uint32_t c[kSPT], csum = 0;
#pragma unroll
      for (int j = 0; j < kSPT; ++j) {
        mymask[j] = (s0 + j < nt) ? sm.mask[s0 + j] : 0ull;
        c[j] = (uint32_t)__popcll(mymask[j]);
        csum += c[j];
      }
      uint32_t tot;
      uint32_t run = block_excl_scan(csum, sm.wsum, &tot);
#pragma unroll
      for (int j = 0; j < kSPT; ++j) {
        mybase[j] = run;
        if (s0 + j < nt) sm.base[s0 + j] = run;
        run += c[j];
      }
    }
    __syncthreads();

    // 4. scatter values into (slot, push) order, fold in push order
    int newlast[kSPT];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
#pragma unroll
      for (int r = 0; r < kEPT; ++r) {
        if (rec[r] != kInvalid) {
          const int pos = (int)(rec[r] & 0xFFFFu);
          const int b = (int)(rec[r] >> 16);
          const unsigned long long below = (1ull << b) - 1ull;
          const uint32_t rank =
              sm.base[pos] + (uint32_t)__popcll(sm.mask[pos] & below);
          sm.sorted[rank] = vv[r][mi];
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kSPT; ++j) {
        unsigned long long mk = mymask[j];
        uint32_t rr = mybase[j];
        int lp = lastp[j];
        V a = acc[mi][j];
        while (mk) {
          const int b = __ffsll((long long)mk) - 1;
          mk &= mk - 1ull;
          const int p = (int)pf + b;
          a = fold_step<V>(a, lp, p, sm.sorted[rr++], parallel, cont);
          lp = p;
        }
        acc[mi][j] = a;
        newlast[j] = lp;
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < kSPT; ++j) lastp[j] = newlast[j];
    e0 = e1;
  }

  // trailing absent pushes of the serial path: one "+ 0.0"
  if (!parallel) {
#pragma unroll
    for (int j = 0; j < kSPT; ++j) {
      const int lp = lastp[j];
      const bool gap = (lp >= 0) ? (lp < (int)np - 1) : (cont && np > 0);
      if (gap) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) acc[mi][j] = acc[mi][j] + V(0);
      }
    }
  }

  // 5. store
  if (s0 + kSPT <= nt) {
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
        for (int j = 0; j < kSPT; ++j) o[j] = acc[mi][j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kSPT; ++j) {
      if (s0 + j < nt) {
#pragma unroll
        for (int mi = 0; mi < M; ++mi) outp[mi][s0 + j] = acc[mi][j];
      }
    }
  }
}

// ----------------------------------------------------------------------
// gather (pull reply): out[i] = W[pos(req[i])], 0 where absent or where
// req[i] repeats req[i-1] (the reference merge walk advances past a match,
// message.h:256-260, so a repeated request key reads 0).
// ----------------------------------------------------------------------
template <typename V>
__global__ __launch_bounds__(256) void gather_kernel(
    const uint64_t* __restrict__ D, uint64_t nd, const V* __restrict__ W,
    const uint64_t* __restrict__ req, uint64_t nreq, V* __restrict__ out,
    unsigned long long* __restrict__ matched) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  bool found = false;
  if (i < nreq) {
    const uint64_t k = req[i];
    const uint64_t pos = gl_lower_bound(D, nd, k);
    V v = V(0);
    if (pos < nd && D[pos] == k && (i == 0 || req[i - 1] != k)) {
      v = W[pos];
      found = true;
    }
    out[i] = v;
  }
  const unsigned long long m = __ballot(found);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(matched, (unsigned long long)__popcll(m));
}

__global__ __launch_bounds__(256) void check_sorted_kernel(
    const uint64_t* __restrict__ k, uint64_t n, unsigned long long* bad) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const bool b = (i > 0 && i < n) && !(k[i - 1] < k[i]);
  const unsigned long long m = __ballot(b);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, (unsigned long long)__popcll(m));
}

// ----------------------------------------------------------------------
// two-input union (strictly increasing a, b):
//   keep[j] = b[j] not in a;  kb = exclusive scan of keep;
//   out[kb[j] + |a < b[j]|] = b[j] for kept j;  out[i + kb(|b < a[i]|)] = a[i]
// ----------------------------------------------------------------------
constexpr int kScanBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanBlock * kScanItems;

__device__ __forceinline__ uint32_t wg256_excl_scan(uint32_t v, uint32_t* ws,
                                                    uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < kScanBlock / 64; ++q) {
    if (q < w) pre += ws[q];
    tot += ws[q];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

__global__ __launch_bounds__(kScanBlock) void union_mark_kernel(
    const uint64_t* __restrict__ a, uint64_t na, const uint64_t* __restrict__ b,
    uint64_t nb, uint32_t* __restrict__ keep, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t ws[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint32_t cnt = 0;
#pragma unroll 4
  for (int q = 0; q < kScanItems; ++q) {
    const uint64_t j = base + (uint64_t)q * kScanBlock + threadIdx.x;
    if (j < nb) {
      const uint64_t k = b[j];
      const uint64_t pos = gl_lower_bound(a, na, k);
      const uint32_t kp = (pos < na && a[pos] == k) ? 0u : 1u;
      keep[j] = kp;
      cnt += kp;
    }
  }
  uint32_t tot;
  wg256_excl_scan(cnt, ws, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// single workgroup: exclusive scan of nblk block sums; d_nout = na + total
__global__ __launch_bounds__(kScanBlock) void union_scan_kernel(
    uint32_t* __restrict__ bsum, uint32_t nblk, uint64_t na,
    uint64_t* __restrict__ d_nout, uint32_t* __restrict__ d_total) {
  __shared__ uint32_t ws[kScanBlock / 64];
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < nblk; c0 += kScanBlock) {
    const uint32_t idx = c0 + threadIdx.x;
    const uint32_t v = idx < nblk ? bsum[idx] : 0u;
    uint32_t tot;
    const uint32_t ex = wg256_excl_scan(v, ws, &tot);
    if (idx < nblk) bsum[idx] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    *d_total = carry;
    *d_nout = na + carry;
  }
}

__global__ __launch_bounds__(kScanBlock) void union_scatter_b_kernel(
    const uint64_t* __restrict__ a, uint64_t na, const uint64_t* __restrict__ b,
    uint64_t nb, uint32_t* __restrict__ keep, const uint32_t* __restrict__ bsum,
    uint64_t* __restrict__ out) {
  __shared__ uint32_t ws[kScanBlock / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  // thread-contiguous items so one scan covers the block in order
  const uint64_t j0 = base + (uint64_t)threadIdx.x * kScanItems;
  uint32_t f[kScanItems];
  uint32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < kScanItems; ++q) {
    const uint64_t j = j0 + q;
    f[q] = j < nb ? keep[j] : 0u;
    cnt += f[q];
  }
  uint32_t tot;
  uint32_t run = bsum[blockIdx.x] + wg256_excl_scan(cnt, ws, &tot);
#pragma unroll
  for (int q = 0; q < kScanItems; ++q) {
    const uint64_t j = j0 + q;
    if (j < nb) {
      keep[j] = run;  // becomes kb[j]
      if (f[q]) {
        const uint64_t k = b[j];
        out[run + gl_lower_bound(a, na, k)] = k;
      }
      run += f[q];
    }
  }
}

__global__ __launch_bounds__(256) void union_scatter_a_kernel(
    const uint64_t* __restrict__ a, uint64_t na, const uint64_t* __restrict__ b,
    uint64_t nb, const uint32_t* __restrict__ kb,
    const uint32_t* __restrict__ d_total, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= na) return;
  const uint64_t k = a[i];
  const uint64_t lb = gl_lower_bound(b, nb, k);
  const uint64_t c = lb < nb ? kb[lb] : *d_total;
  out[i + c] = k;
}

// sliceKeyOrderedMsg positions: one wave per separator (message.h:96-99)
__global__ __launch_bounds__(256) void slice_kernel(
    const uint64_t* __restrict__ keys, uint64_t n, uint64_t kb, uint64_t ke,
    const uint64_t* __restrict__ sep, int nsep, uint64_t* __restrict__ pos) {
  const int s = (int)((blockIdx.x * 256u + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= nsep) return;
  uint64_t k = sep[s];
  if (k > ke) k = ke;
  if (k < kb) k = kb;
  const uint64_t r = wave_search(keys, n, k, false, lane);
  if (lane == 0) pos[s] = r;
}

}  // namespace

// ----------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------
hipError_t launch_partition(const JobDev* d_jobs, int njobs, uint32_t nitems,
                            hipStream_t stream) {
  if (nitems == 0) return hipSuccess;
  const uint32_t blocks = (nitems + 3u) / 4u;
  hipLaunchKernelGGL(partition_kernel, dim3(blocks), dim3(256), 0, stream,
                     d_jobs, njobs, nitems);
  return hipGetLastError();
}

template <typename V>
static hipError_t launch_aggregate_t(int m, const JobDev* d_jobs, int njobs,
                                     uint32_t ntiles, hipStream_t stream) {
  switch (m) {
    case 1: hipLaunchKernelGGL((aggregate_kernel<V, 1>), dim3(ntiles), dim3(kThreads), 0, stream, d_jobs, njobs); break;
    case 2: hipLaunchKernelGGL((aggregate_kernel<V, 2>), dim3(ntiles), dim3(kThreads), 0, stream, d_jobs, njobs); break;
    case 3: hipLaunchKernelGGL((aggregate_kernel<V, 3>), dim3(ntiles), dim3(kThreads), 0, stream, d_jobs, njobs); break;
    case 4: hipLaunchKernelGGL((aggregate_kernel<V, 4>), dim3(ntiles), dim3(kThreads), 0, stream, d_jobs, njobs); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_aggregate(int dtype, int m, const JobDev* d_jobs, int njobs,
                            uint32_t ntiles, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  return dtype == 0 ? launch_aggregate_t<float>(m, d_jobs, njobs, ntiles, stream)
                    : launch_aggregate_t<double>(m, d_jobs, njobs, ntiles, stream);
}

hipError_t launch_gather(int dtype, const uint64_t* dkeys, uint64_t nd,
                         const void* dvals, const uint64_t* req, uint64_t nreq,
                         void* out, unsigned long long* matched,
                         hipStream_t stream) {
  if (nreq == 0) return hipSuccess;
  const uint64_t blocks = (nreq + 255) / 256;
  if (dtype == 0)
    hipLaunchKernelGGL(gather_kernel<float>, dim3((uint32_t)blocks), dim3(256), 0,
                       stream, dkeys, nd, (const float*)dvals, req, nreq,
                       (float*)out, matched);
  else
    hipLaunchKernelGGL(gather_kernel<double>, dim3((uint32_t)blocks), dim3(256), 0,
                       stream, dkeys, nd, (const double*)dvals, req, nreq,
                       (double*)out, matched);
  return hipGetLastError();
}

hipError_t launch_check_sorted(const uint64_t* keys, uint64_t n,
                               unsigned long long* bad, hipStream_t stream) {
  if (n < 2) return hipSuccess;
  hipLaunchKernelGGL(check_sorted_kernel, dim3((uint32_t)((n + 255) / 256)),
                     dim3(256), 0, stream, keys, n, bad);
  return hipGetLastError();
}

size_t union_scratch_bytes(uint64_t nb) {
  const uint64_t nblk = (nb + kScanTile - 1) / kScanTile;
  return (size_t)(nb * 4 + nblk * 4 + 64);
}

hipError_t launch_union(const uint64_t* a, uint64_t na, const uint64_t* b,
                        uint64_t nb, uint64_t* out, void* scratch,
                        uint64_t* d_nout, hipStream_t stream) {
  uint32_t* keep = (uint32_t*)scratch;
  const uint32_t nblk = (uint32_t)((nb + kScanTile - 1) / kScanTile);
  uint32_t* bsum = keep + nb;
  uint32_t* d_total = bsum + nblk;
  if (nb > 0) {
    hipLaunchKernelGGL(union_mark_kernel, dim3(nblk), dim3(kScanBlock), 0,
                       stream, a, na, b, nb, keep, bsum);
  }
  hipLaunchKernelGGL(union_scan_kernel, dim3(1), dim3(kScanBlock), 0, stream,
                     bsum, nblk, na, d_nout, d_total);
  if (nb > 0) {
    hipLaunchKernelGGL(union_scatter_b_kernel, dim3(nblk), dim3(kScanBlock), 0,
                       stream, a, na, b, nb, keep, bsum, out);
  }
  if (na > 0) {
    hipLaunchKernelGGL(union_scatter_a_kernel, dim3((uint32_t)((na + 255) / 256)),
                       dim3(256), 0, stream, a, na, b, nb, keep, d_total, out);
  }
  return hipGetLastError();
}

hipError_t launch_slice(const uint64_t* keys, uint64_t n, uint64_t kb,
                        uint64_t ke, const uint64_t* sep, int nsep,
                        uint64_t* pos, hipStream_t stream) {
  if (nsep <= 0) return hipSuccess;
  hipLaunchKernelGGL(slice_kernel, dim3((uint32_t)((nsep + 3) / 4)), dim3(256), 0,
                     stream, keys, n, kb, ke, sep, nsep, pos);
  return hipGetLastError();
}

}  // namespace psg
