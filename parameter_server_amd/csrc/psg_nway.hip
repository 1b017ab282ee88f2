// psg_nway.hip -- N-way merge of sorted pushes into their merged key set
// (SURVEY 7 step 4): the union of the pushes' keys and, with values, the
// per-key sums over the pushes in arrival order.
//
// Reference semantics:
//   keys  SArray::setUnion applied push after push (shared_array_inl.h:
//         155-162, std::set_union; the key-only branch of
//         KVVector::serialSetValue, kv_vector.h:177-182): the sorted set of
//         every pushed key, duplicates across pushes collapsed;
//   sums  KVVector::serialSetValue / parallelSetValue (kv_vector.h:84-204)
//         over D = that union: per key, push 0 assigns if it holds the key
//         (the others start from the memset +0.0), later pushes add in
//         arrival order, and the serial path adds one +0.0 when some push
//         lacked the key (the dense `+=` of absent pushes).
//
// Pipeline (one stream, no host wait; psg_nway_run):
//   0. candidates: every s-th key of every push, gathered into one array
//                                                              (nw_gather)
//   1. its rank estimate A(c) = s * sum_q (candidates of push q below c):
//      searches of the small candidate lists, staged in LDS, instead of the
//      pushes (R(c) = sum_q lower_bound(push q, c) lies in [A, A + K(s - 1)])
//                                                              (nw_rank)
//   2. splitter of rank bucket b = the largest candidate with
//      floor(A / C') == b (atomic max on the key: A is monotone in the key)
//                                                              (nw_bucket)
//   3. prefix max over the buckets (empty buckets: empty tiles) (nw_split)
//   4. per (tile, push) the piece bounds: lower_bound of the splitters
//                                                              (nw_seg)
//   5. one workgroup per tile (nw_tile):
//      - loads its K pieces (keys, and values into LDS), checks each piece
//        strictly increasing and inside the tile's key range;
//      - merges the K sorted runs in LDS with a merge-path tree
//        (ceil(log2 K) rounds; each thread merges 8 outputs in registers,
//        stable, so equal keys keep push order);
//      - wavefront ballot for run heads (key != previous), block prefix
//        scan for the unique index; decoupled look-back across tiles (tiles
//        in ticket order) for the global offset;
//      - segmented sum of each run in push order; the merged keys and sums
//        staged compacted in LDS and written coalesced.
// Tile size: tile t holds R(split[t]) - R(split[t-1]) elements.
// R(split[t]) <= A(split[t]) + K(s-1) < (t+1) C' + K(s-1); the candidate
// after split[t-1] in key order lies in bucket >= t and at most K
// candidates (one per push) equal split[t-1], so A(split[t-1]) >= t C' - K s;
// hence a tile spans at most C' + 2 K s - K elements <= kCap (C' = kCap -
// 2 K s): no tile overflows, whatever the key distribution.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "psg_device.h"
#include "psg_host.h"
#include "psg_internal.h"

namespace psg {

namespace {

constexpr int kNT = 256;            // threads per tile workgroup
constexpr int kPer = 8;             // merged elements per thread
constexpr int kCap = kNT * kPer;    // elements per tile (LDS)
constexpr int kMaxRuns = 64;        // pushes per merge (runs per tile)

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// global (not flat) accesses: a flat access also counts on lgkmcnt, so the
// LDS waits of the rank and tile stages would wait for loads in flight too
#define AS1 __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}
template <typename T>
__device__ __forceinline__ AS1 T* GW(T* p) {
  return (AS1 T*)p;
}

struct NwArgs {
  const uint64_t* const* keys;  // [K] push keys
  const void* const* vals;      // [K * M] push values (M > 0)
  const uint64_t* n;            // [K]
  const uint64_t* cbase;        // [K + 1] first candidate of each push
  uint64_t* candk;              // [ncand] candidate keys, push by push
  uint32_t* rank;               // [ncand] A(c)
  uint64_t* split;              // [B] splitter keys
  uint32_t* seg;                // [(T + 1) * K] piece starts, tile-major
  unsigned long long* state;    // [T] look-back words
  unsigned long long* bad;      // order violations / overflow
  unsigned long long* nout;     // merged key count
  uint64_t* out_keys;
  void* const* out_vals;        // [M]
  uint64_t ncand;
  uint32_t K, B, T, s, cw;      // pushes, buckets, tiles, sample stride, bucket width C'
  uint32_t flags;
};

// A batch of independent merges (psg_nway_create_batch: e.g. the 64
// aggregates of a bench step) runs as ONE pipeline: each stage is one launch
// over the work items of every merge, which find their merge by a binary
// search over the stage's prefix counts.  The tile stage deals tiles by a
// global ticket, so a tile's look-back only waits on tiles of its merge
// that are already running.
struct NwBatch {
  const NwArgs* args;       // [nm]
  const uint64_t* wpre;     // [nm + 1] rank-stage workgroups before merge j
  const uint64_t* cpre;     // [nm + 1] candidates before merge j
  const uint64_t* spre;     // [nm + 1] seg entries ((T + 1) K) before merge j
  const uint64_t* tpre;     // [nm + 1] tiles before merge j
  unsigned int* ticket;     // tile tickets
  uint32_t nm;
  uint32_t rr;              // tickets round-robin over the merges (1) or merge by merge (0)
};

// merge j of item x: the last j with pre[j] <= x (pre non-decreasing)
__device__ __forceinline__ uint32_t merge_of(const uint64_t* pre, uint32_t nm, uint64_t x) {
  uint32_t lo = 0, hi = nm;  // pre[lo] <= x < pre[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

// the push owning candidate c: the last q with cbase[q] <= c
__device__ __forceinline__ uint32_t owner(const NwArgs& a, uint64_t c) {
  uint32_t lo = 0, hi = a.K;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.cbase[mid] <= c) lo = mid; else hi = mid;
  }
  return lo;
}

// 0. the candidates: candidate i of push q is its key (i + 1) s - 1
__global__ __launch_bounds__(256) void nw_gather_kernel(NwBatch b, uint64_t ncand) {
  const uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (g >= ncand) return;
  const uint32_t j = merge_of(b.cpre, b.nm, g);
  const NwArgs& a = b.args[j];
  const uint64_t c = g - b.cpre[j];
  const uint32_t q = owner(a, c);
  a.candk[c] = a.keys[q][(c - a.cbase[q]) * a.s + a.s - 1];
}

// 1. A(c) for every candidate c: a workgroup takes kRkChunk candidates of
// one merge (16 per thread, in registers) and walks the merge's K candidate
// lists: each list is staged in LDS (coalesced) and searched there, and the
// counts are summed in registers -- no atomics, no global search chains.  A
// list longer than the LDS stage is searched in global memory (interpolation
// probes, then a bisection: exact for any key distribution).
// Candidates per thread: 16 when the batch fills the chip with workgroups of
// 4,096 candidates; a small batch (one merge: 8 such workgroups for cfg2)
// takes 4 or 1 per thread, so its lists are searched by more workgroups at
// once instead of by a few long chains of LDS reads.
constexpr uint32_t kRkList = 8192;           // candidates of one list staged in LDS (64 KB)
template <uint32_t kRkPer>
__global__ __launch_bounds__(256) void nw_rank_kernel(NwBatch b) {
  constexpr uint32_t kRkChunk = 256 * kRkPer;  // candidates per workgroup
  __shared__ uint64_t lst[kRkList];
  const uint32_t item = blockIdx.x;
  const uint32_t j = uni(merge_of(b.wpre, b.nm, item));
  const NwArgs& a = b.args[j];
  const uint64_t c0 = (uint64_t)(item - b.wpre[j]) * kRkChunk;
  const uint32_t t = threadIdx.x;
  uint64_t mine[kRkPer];
  uint32_t acc[kRkPer];
  // thread t holds kRkPer consecutive candidates (sorted while they lie in
  // one push's run): a list is then searched once per thread and walked for
  // the rest, not searched kRkPer times (r05: profiles/r05_ab_nway.txt)
#pragma unroll
  for (uint32_t i = 0; i < kRkPer; ++i) {
    const uint64_t c = c0 + kRkPer * t + i;
    mine[i] = c < a.ncand ? G(a.candk)[c] : ~0ull;
    acc[i] = 0;
  }
  for (uint32_t r = 0; r < a.K; ++r) {
    const uint64_t q0 = a.cbase[r];
    const uint32_t L = (uint32_t)(a.cbase[r + 1] - q0);
    // one candidate per thread (a small batch): each search straight in the
    // list in global memory (L2-resident), no staging round per list
    if (kRkPer > 1 && L <= kRkList) {
      __syncthreads();  // the previous list's searches are done
      for (uint32_t x = t; x < L; x += 256) lst[x] = G(a.candk)[q0 + x];
      __syncthreads();
      uint32_t pos = 0;  // lower_bound(lst[0, L), mine[i - 1])
#pragma unroll
      for (uint32_t i = 0; i < kRkPer; ++i) {
        const uint64_t k = mine[i];
        // from the previous candidate's position when k does not go back
        // (same push run): a few steps forward, else a bisection of the rest
        uint32_t lo = (i > 0 && k >= mine[i - 1]) ? pos : 0u;
#pragma unroll
        for (int st = 0; st < 2; ++st) lo += (lo < L && lst[lo] < k) ? 1u : 0u;
        uint32_t n = lo < L && lst[lo] < k ? L - lo : 0u;
        if (i == 0 || k < mine[i - 1]) {  // a new run (or the first): the whole list
          lo = 0;
          n = L;
        }
        while (n > 0) {
          const uint32_t h = n >> 1;
          if (lst[lo + h] < k) {
            lo += h + 1;
            n -= h + 1;
          } else {
            n = h;
          }
        }
        pos = lo;
        acc[i] += lo;
      }
    } else {
#pragma unroll
      for (uint32_t i = 0; i < kRkPer; ++i)
        acc[i] += (uint32_t)dev::interp_lower_bound(a.candk + q0, L, mine[i]);
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < kRkPer; ++i) {
    const uint64_t c = c0 + kRkPer * t + i;
    if (c < a.ncand) GW(a.rank)[c] = a.s * acc[i];
  }
}

// 2. splitter of bucket floor(R / C') = its largest candidate key
// (consecutive candidates of one push have increasing keys and ranks, so
// about C' / (K s) neighbours share a bucket: only the lane whose right
// neighbour does not dominate it -- same merge and bucket, key not smaller
// -- issues the atomic)
__global__ __launch_bounds__(256) void nw_bucket_kernel(NwBatch b, uint64_t ncand) {
  const uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const bool in = g < ncand;
  uint32_t j = 0, bk = 0xffffffffu;
  uint64_t key = 0;
  if (in) {
    j = merge_of(b.cpre, b.nm, g);
    const NwArgs& a = b.args[j];
    const uint64_t c = g - b.cpre[j];
    key = a.candk[c];
    bk = a.rank[c] / a.cw;
  }
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nj = (uint32_t)__shfl_down((int)j, 1, 64);
  const uint32_t nb = (uint32_t)__shfl_down((int)bk, 1, 64);
  const uint64_t nk = (uint64_t)__shfl_down((long long)key, 1, 64);
  const bool dominated = lane < 63u && g + 1 < ncand && nj == j && nb == bk && nk >= key;
  if (in && !dominated && bk < b.args[j].B)
    atomicMax((unsigned long long*)b.args[j].split + bk, (unsigned long long)key);
}

// 3. prefix max (one workgroup per merge): splitters non-decreasing, empty
// buckets repeat the previous splitter (an empty tile)
__global__ __launch_bounds__(256) void nw_split_kernel(NwBatch bt) {
  __shared__ uint64_t wmax[4];
  __shared__ uint64_t carry;
  const NwArgs& a = bt.args[blockIdx.x];
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t b0 = 0; b0 < a.B; b0 += 256) {
    const uint32_t b = b0 + threadIdx.x;
    uint64_t x = b < a.B ? a.split[b] : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(x, d, 64);
      if (lane >= d && y > x) x = y;
    }
    if (lane == 63) wmax[w] = x;
    __syncthreads();
    uint64_t pre = carry;
    for (int v = 0; v < w; ++v) pre = wmax[v] > pre ? wmax[v] : pre;
    x = x > pre ? x : pre;
    if (b < a.B) a.split[b] = x;
    __syncthreads();
    if (threadIdx.x == 255) carry = x;
    __syncthreads();
  }
}

// 4. seg[t * K + q] = first index of push q in tile t: 0 (t = 0),
// lower_bound(push q, split[t - 1]) (0 < t < T), n_q (t = T)
__global__ __launch_bounds__(256) void nw_seg_kernel(NwBatch b, uint64_t nseg) {
  const uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (g >= nseg) return;
  const uint32_t j = merge_of(b.spre, b.nm, g);
  const NwArgs& a = b.args[j];
  const uint64_t id = g - b.spre[j];
  const uint32_t t = (uint32_t)(id / a.K), q = (uint32_t)(id - (uint64_t)t * a.K);
  uint64_t v;
  if (t == 0) v = 0;
  else if (t == a.T) v = a.n[q];
  else v = dev::interp_lower_bound(a.keys[q], a.n[q], a.split[t - 1]);
  a.seg[id] = (uint32_t)v;
}

constexpr uint64_t kFlagAgg = 1ull << 62, kFlagPre = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;

#ifdef PSG_NWAY_PROF
// diagnostic build only (tools/nway_probe.py --prof): per tile (first 65,536
// tickets), shader clocks at the phase boundaries of nw_tile_kernel
__device__ unsigned long long g_nwprof[65536][8];
#define NP_MARK(i) np_t[i] = clock64()
#else
#define NP_MARK(i) do { } while (0)
#endif

// LDS layout of the tile's keys and source indices: XOR swizzles inside
// aligned blocks (no extra LDS).  Lane l's elements e = 8 l + x land in u64
// bank slot 8 (l mod 4) + (x ^ (l / 4 mod 8)) for keys and in dword bank
// 4 (l mod 8) + (x / 2 ^ (l / 8 mod 4)) for source indices, so the loads'
// installs, the merge walks and write-backs of a wave's 32 lanes hit 32
// different banks instead of 4 or 8 (r05: batch 1.49 -> 1.41 ms,
// profiles/r05_ab_nway.txt)
#define SWK(e) ((e) ^ (((e) >> 5) & 7u))
#define SWI(e) ((e) ^ ((((e) >> 6) & 3u) << 1))


// 5. the tile merge
template <typename V, int M>
__global__ __launch_bounds__(kNT) void nw_tile_kernel(NwBatch bt) {
  constexpr int kM = M > 0 ? M : 1;
  constexpr int kVC = M > 0 ? kCap : 1;
  // keys (merged in place) and the source position of each key, at the
  // swizzled indices SWK / SWI (above)
  __shared__ __attribute__((aligned(16))) uint64_t sk[kCap];
  __shared__ uint16_t si[kCap];
  __shared__ __attribute__((aligned(16))) V sv[kM][kVC];      // values by source position
  __shared__ uint32_t roff[kMaxRuns + 1];                     // run offsets (never changed)
  __shared__ const uint64_t* pkey[kMaxRuns];                  // piece starts (keys)
  __shared__ const V* pval[kMaxRuns * kM];                    // piece starts (values)
  __shared__ uint32_t wsum[kNT / 64];
  __shared__ uint32_t sh_t, sh_err;
  __shared__ unsigned long long sh_base;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#ifdef PSG_NWAY_PROF
  unsigned long long np_t[8];
#endif

  // ---- ticket: tiles in dispatch order (the look-back waits only on
  // tickets taken by workgroups that are already running), then its merge
  if (tid == 0) {
    sh_t = atomicAdd(bt.ticket, 1u);
    sh_err = 0;
  }
  __syncthreads();
  const uint32_t g = uni(sh_t);
  // round robin (batches): ticket g is tile g / nm of merge g mod nm, so the
  // tiles in flight spread over every merge and a tile's predecessor in its
  // merge started nm tickets earlier -- its look-back finds an inclusive
  // prefix at once instead of waiting down a chain of running neighbours
  // (r05: profiles/r05_ab_nway.txt).  A ticket past a merge's last tile
  // (merges of fewer tiles) is idle.
  uint32_t jm, t;
  if (bt.rr) {
    jm = g % bt.nm;
    t = g / bt.nm;
  } else {
    jm = uni(merge_of(bt.tpre, bt.nm, g));
    t = (uint32_t)(g - bt.tpre[jm]);
  }
  const NwArgs& a = bt.args[jm];
  if (t >= a.T) return;
  const uint32_t K = a.K;
  const bool parallel = (a.flags & kFlagParallel) != 0;

  NP_MARK(0);
  // ---- piece table: wave 0, one lane per push
  if (w == 0) {
    uint32_t len = 0;
    if ((uint32_t)lane < K) {
      const uint32_t s0 = G(a.seg)[(size_t)t * K + lane], s1 = G(a.seg)[(size_t)(t + 1) * K + lane];
      len = s1 > s0 ? s1 - s0 : 0u;
      pkey[lane] = a.keys[lane] + s0;
#pragma unroll
      for (int mi = 0; mi < M; ++mi)
        pval[lane * M + mi] = (const V*)a.vals[(size_t)lane * M + mi] + s0;
    }
    uint32_t x = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if ((uint32_t)lane < K) roff[lane + 1] = x;
    if (lane == 0) roff[0] = 0;
    if (lane == 63 && x > (uint32_t)kCap) sh_err = 1;  // excluded by the splitters (header)
  }
  __syncthreads();
  if (sh_err) {
    // never expected: report, and merge nothing (an empty tile still
    // publishes its count, so later tiles' look-back ends)
    if (tid == 0) {
      atomicAdd(a.bad, 1ull << 32);
      roff[K] = 0;
      for (uint32_t q = 0; q < K; ++q) roff[q] = 0;
    }
    __syncthreads();
  }
  const uint32_t E = uni(roff[K]);

  NP_MARK(1);
  // ---- load the pieces: thread tid takes elements [8 tid, 8 tid + 8) of
  // the concatenated pieces (one search of the run offsets, then a walk), so
  // every load of the tile is in flight at once; then keys, source
  // positions and values into LDS, and the order check: each piece strictly
  // increasing and inside the tile's key range [split[t-1], split[t]), so
  // the pieces concatenate to the sorted pushes (std::set_union's
  // precondition)
  uint32_t viol = 0;
  uint64_t kk[kPer];      // this thread's elements (keys), in load order
  uint32_t qs = 0;        // bit x: element e0 + x starts a piece
  {
    const uint32_t e0 = (uint32_t)tid * kPer;
    uint32_t q = 0;
    {
      uint32_t hi = K;  // the last q with roff[q] <= e0
      while (hi - q > 1) {
        const uint32_t mid = (q + hi) >> 1;
        if (roff[mid] <= e0) q = mid; else hi = mid;
      }
    }
    V vv[kPer][kM];
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      const uint32_t e = e0 + x;
      kk[x] = 0;
#pragma unroll
      for (int mi = 0; mi < kM; ++mi) vv[x][mi] = V(0);
      if (e < E) {
        while (roff[q + 1] <= e) ++q;
        const uint32_t i = e - roff[q];
        qs |= (uint32_t)(i == 0u) << x;
        kk[x] = G(pkey[q])[i];
#pragma unroll
        for (int mi = 0; mi < M; ++mi) vv[x][mi] = G(pval[q * M + mi])[i];
      }
    }
    const uint64_t klo = t > 0 ? a.split[t - 1] : 0ull;
    const bool open = t + 1 >= a.T;
    const uint64_t khi = open ? ~0ull : a.split[t];
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      const uint32_t e = e0 + x;
      if (e < E) {
        sk[SWK(e)] = kk[x];
        si[SWI(e)] = (uint16_t)e;
#pragma unroll
        for (int mi = 0; mi < M; ++mi) sv[mi][e] = vv[x][mi];
        // within the thread's run: the previous element from registers; at
        // a piece start only the range; the run's first element against the
        // previous thread's last, after the barrier
        const bool inr = kk[x] >= klo && (open || kk[x] < khi);
        const bool ord = x == 0 || ((qs >> x) & 1u) || kk[x - 1] < kk[x];
        viol += inr && ord ? 0u : 1u;
      }
    }
    __syncthreads();
    if (e0 < E && e0 > 0 && !(qs & 1u) && !(sk[SWK(e0 - 1)] < kk[0])) ++viol;
  }
  NP_MARK(2);
  // ---- merge-path tree: round `width` merges runs [r0, r0 + width) and
  // [r0 + width, r0 + 2 width) (original run indices; the offsets of merged
  // runs are original run offsets); stable, so equal keys keep push order
  const uint32_t k0 = (uint32_t)tid * kPer;
  // this thread's 8 outputs of the last round stay in registers (the run
  // heads and the segmented sums read them there)
  uint64_t rk[kPer];
  uint16_t ri[kPer];
  if (K <= 1) {  // one run: already in order
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      rk[x] = k0 + x < E ? sk[SWK(k0 + x)] : 0ull;
      ri[x] = k0 + x < E ? si[SWI(k0 + x)] : (uint16_t)0;
    }
  }
  for (uint32_t width = 1; width < K; width <<= 1) {
    uint32_t A0 = 0, B0 = 0, B1 = 0, i = 0, j = 0;  // current pair and merge position
    uint64_t ka = 0, kb = 0;                         // sk[A0 + i], sk[B0 + j] (when in range)
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      const uint32_t k = k0 + x;
      rk[x] = 0;
      ri[x] = 0;
      if (k < E) {
        if (x == 0 || k >= B1) {
          // the pair whose merged region holds k, and the merge path there
          uint32_t r0 = 0;
          while (r0 + 2 * width < K && roff[r0 + 2 * width] <= k) r0 += 2 * width;
          const uint32_t r1 = r0 + width < K ? r0 + width : K;
          const uint32_t r2 = r0 + 2 * width < K ? r0 + 2 * width : K;
          A0 = roff[r0];
          B0 = roff[r1];
          B1 = roff[r2];
          const uint32_t la = B0 - A0, lb = B1 - B0, d = k - A0;
          uint32_t lo = d > lb ? d - lb : 0u, hi = d < la ? d : la;
          while (lo < hi) {  // A elements among the first d outputs
            const uint32_t mid = (lo + hi) >> 1;
            if (sk[SWK(A0 + mid)] <= sk[SWK(B0 + d - mid - 1)]) lo = mid + 1;
            else hi = mid;
          }
          i = lo;
          j = d - lo;
          ka = i < la ? sk[SWK(A0 + i)] : 0ull;
          kb = j < lb ? sk[SWK(B0 + j)] : 0ull;
        }
        // one LDS key read per output: the side taken advances
        const uint32_t la = B0 - A0, lb = B1 - B0;
        const bool takeA = j >= lb || (i < la && ka <= kb);
        rk[x] = takeA ? ka : kb;
        ri[x] = si[SWI(takeA ? A0 + i : B0 + j)];
        if (takeA) {
          ++i;
          ka = i < la ? sk[SWK(A0 + i)] : 0ull;
        } else {
          ++j;
          kb = j < lb ? sk[SWK(B0 + j)] : 0ull;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < kPer; ++x)
      if (k0 + x < E) {
        sk[SWK(k0 + x)] = rk[x];
        si[SWI(k0 + x)] = ri[x];
      }
    __syncthreads();
  }

  NP_MARK(3);
  // ---- run heads (a key differing from the previous one), unique index
  uint32_t heads = 0, nh = 0;
  {
    const uint64_t before = k0 > 0 && k0 < E ? sk[SWK(k0 - 1)] : 0ull;
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      const uint32_t e = k0 + x;
      const bool h = e < E && (e == 0 || (x == 0 ? before : rk[x - 1]) != rk[x]);
      heads |= (uint32_t)h << x;
      nh += h ? 1u : 0u;
    }
  }
  uint32_t incl = nh;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  for (int d = 32; d > 0; d >>= 1) viol += __shfl_xor(viol, d, 64);
  if (lane == 0 && viol) atomicAdd(a.bad, (unsigned long long)viol);
  __syncthreads();
  uint32_t U = 0, first_u = incl - nh;
#pragma unroll
  for (int v = 0; v < kNT / 64; ++v) {
    first_u += v < w ? wsum[v] : 0u;
    U += wsum[v];
  }

  NP_MARK(4);
  // ---- this tile's unique count for the look-back of later tiles: as
  // early as it is known (the sums below do not need the offset, so they
  // run while predecessors finish)
  if (w == 0 && lane == 0 && t > 0)
    __hip_atomic_store(a.state + t, kFlagAgg | (unsigned long long)U, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  // ---- segmented sums of this thread's runs, in push order
  uint64_t hk[kPer];
  V hs[kPer][kM];
#pragma unroll
  for (int x = 0; x < kPer; ++x) {
    hk[x] = 0;
#pragma unroll
    for (int mi = 0; mi < kM; ++mi) hs[x][mi] = V(0);
    if ((heads >> x) & 1u) {
      const uint64_t key = rk[x];
      hk[x] = key;
      if constexpr (M > 0) {
        // the run [e, f): push 0 (run 0's sources) assigns, later pushes
        // add to the memset +0.0 or to it; serial: one trailing +0.0 when
        // a push lacked the key (kv_vector.h:195-201).  The run's part in
        // this thread's outputs from registers, the rest (a run crossing
        // into the next thread's outputs) from LDS
        V acc[M];
#pragma unroll
        for (int mi = 0; mi < M; ++mi) acc[mi] = V(0);
        const uint32_t p0 = roff[1];
        uint32_t cnt = 0;
        bool open = true;
#pragma unroll
        for (int y = x; y < kPer; ++y) {
          open = open && k0 + y < E && rk[y] == key;
          if (open) {
            const uint32_t src = ri[y];
#pragma unroll
            for (int mi = 0; mi < M; ++mi) acc[mi] = src < p0 ? sv[mi][src] : acc[mi] + sv[mi][src];
            ++cnt;
          }
        }
        uint32_t f = k0 + kPer;
        while (open && f < E && sk[SWK(f)] == key) {
          const uint32_t src = si[SWI(f)];
#pragma unroll
          for (int mi = 0; mi < M; ++mi) acc[mi] = src < p0 ? sv[mi][src] : acc[mi] + sv[mi][src];
          ++cnt;
          ++f;
        }
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          hs[x][mi] = (!parallel && cnt < K) ? acc[mi] + V(0) : acc[mi];
      }
    }
  }
  NP_MARK(5);
  // ---- decoupled look-back (wave 0): this tile's global offset
  if (w == 0) {
    unsigned long long excl = 0;
    if (t > 0) {
      // 256 predecessors per step (4 per lane, lane l at distances 4l..4l+3,
      // the loads independent): the nearest inclusive prefix ends the sum
      int64_t j = (int64_t)t - 1;
      uint32_t spins = 0;
      for (;;) {
        unsigned long long st4[4];
        int dpre = 1 << 30, dinv = 1 << 30;  // nearest inclusive / unpublished
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int d = 4 * lane + c;
          const int64_t idx = j - d;
          st4[c] = idx >= 0 ? __hip_atomic_load(a.state + idx, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)
                            : kFlagPre;  // before tile 0: an inclusive prefix of 0
          const unsigned long long fl = st4[c] & ~kValMask;
          if (fl == kFlagPre && d < dpre) dpre = d;
          if (fl == 0 && d < dinv) dinv = d;
        }
        for (int o = 32; o > 0; o >>= 1) {
          const int x = __shfl_xor(dpre, o, 64), y = __shfl_xor(dinv, o, 64);
          dpre = x < dpre ? x : dpre;
          dinv = y < dinv ? y : dinv;
        }
        if (dinv < dpre && dinv < 256) {  // a predecessor has not published yet
          if (++spins > (1u << 22)) {  // never expected: report and stop waiting
            if (lane == 0) atomicAdd(a.bad, 1ull << 40);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
          continue;
        }
        unsigned long long v = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (4 * lane + c <= dpre) v += st4[c] & kValMask;
        for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
        excl += v;
        if (dpre < 256) break;
        j -= 256;
      }
    }
    if (lane == 0) {
      __hip_atomic_store(a.state + t, kFlagPre | (excl + U), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1 == a.T) *a.nout = excl + U;
      sh_base = excl;
    }
  }

  __syncthreads();  // every read of sk / si / sv is done; sh_base is set
  // compacted: unique u of the tile at LDS position u
  {
    uint32_t u = first_u;
#pragma unroll
    for (int x = 0; x < kPer; ++x) {
      if ((heads >> x) & 1u) {
        sk[u] = hk[x];
#pragma unroll
        for (int mi = 0; mi < M; ++mi) sv[mi][u] = hs[x][mi];
        ++u;
      }
    }
  }
  __syncthreads();
  NP_MARK(6);
  const unsigned long long base = sh_base;
  for (uint32_t e = tid; e < U; e += kNT) {
    GW(a.out_keys)[base + e] = sk[e];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) GW((V*)a.out_vals[mi])[base + e] = sv[mi][e];
  }
  NP_MARK(7);
#ifdef PSG_NWAY_PROF
  if (tid == 0 && g < 65536u)
    for (int i = 0; i < 8; ++i) g_nwprof[g][i] = np_t[i];
#endif
}

template <typename V, int M>
hipError_t launch_tile(const NwBatch& b, uint64_t tiles, hipStream_t s) {
  hipLaunchKernelGGL((nw_tile_kernel<V, M>), dim3((uint32_t)tiles), dim3(kNT), 0, s, b);
  return hipGetLastError();
}

template <typename V>
hipError_t launch_tile_m(int m, const NwBatch& b, uint64_t tiles, hipStream_t s) {
  switch (m) {
    case 0: return launch_tile<V, 0>(b, tiles, s);
    case 1: return launch_tile<V, 1>(b, tiles, s);
    case 2: return launch_tile<V, 2>(b, tiles, s);
    case 3: return launch_tile<V, 3>(b, tiles, s);
    case 4: return launch_tile<V, 4>(b, tiles, s);
    default: return hipErrorInvalidValue;
  }
}

size_t al256(size_t x) { return (x + 255) / 256 * 256; }

}  // namespace

// One merge's shape: sample stride s and bucket width C' (header: a tile
// holds <= C' + K s + K elements), candidates, buckets, tiles.
struct NwShape {
  uint32_t K = 0, s = 1, cw = 1, B = 1, T = 2;
  uint64_t ncand = 0;
  std::vector<uint64_t> cbase;
  void plan(uint32_t k, const uint64_t* pn) {
    K = k;
    uint64_t ntot = 0;
    for (uint32_t q = 0; q < K; ++q) ntot += pn[q];
    s = std::max<uint32_t>(1, kCap / (8 * std::max<uint32_t>(K, 1)));
    cw = kCap - 2 * K * s;
    cbase.assign(K + 1, 0);
    for (uint32_t q = 0; q < K; ++q) cbase[q + 1] = cbase[q] + pn[q] / s;
    ncand = cbase[K];
    B = (uint32_t)(ntot / cw + 1);
    T = B + 1;
    if (K == 0) B = T = 0;  // no pushes: no work, the merged count stays 0
  }
  // rank workgroups at `per` candidates per thread
  uint64_t waves(uint32_t per) const { return (ncand + 256u * per - 1) / (256u * per); }
};

// Device scratch of a batch of nm merges: [tables: per merge key / value /
// length / candidate-base / output pointer arrays; NwArgs[nm]; prefix
// counts][zeroed per run: per merge rank, splitters, look-back words; the
// ticket; per merge (bad, nout)][per merge piece starts].  The tables are
// written once (upload); a run clears one region and enqueues 5 launches.
struct NwLayout {
  uint32_t nm = 0;
  int m = 0;
  std::vector<NwShape> sh;
  struct Off { size_t k, v, n, cb, ov, rank, split, state, seg, candk; };
  std::vector<Off> off;
  size_t o_args = 0, o_pre = 0, o_zero = 0, o_ticket = 0, o_misc = 0, zero_len = 0, bytes = 0;
  uint64_t nwaves = 0, ncand = 0, nseg = 0, ntiles = 0;
  uint64_t maxT = 0;  // the most tiles of one merge (round-robin tickets: maxT * nm)
  uint32_t rk_per = 16;  // rank-stage candidates per thread (16, 4 or 1)

  // pn: the merges' push lengths back to back, npush[j] per merge
  void plan(uint32_t nmerge, const uint32_t* npush, const uint64_t* pn, int mm) {
    nm = nmerge;
    m = mm;
    sh.assign(nm, NwShape{});
    off.assign(nm, Off{});
    size_t o = 0, pcur = 0;
    for (uint32_t j = 0; j < nm; ++j) {
      sh[j].plan(npush[j], pn + pcur);
      pcur += npush[j];
      const uint32_t K = npush[j];
      Off& f = off[j];
      f.k = o; o = al256(o + 8 * (size_t)K);
      f.v = o; o = al256(o + 8 * (size_t)K * m);
      f.n = o; o = al256(o + 8 * (size_t)K);
      f.cb = o; o = al256(o + 8 * (size_t)(K + 1));
      f.ov = o; o = al256(o + 8 * (size_t)std::max(m, 1));
    }
    o_args = o; o = al256(o + sizeof(NwArgs) * (size_t)nm);
    o_pre = o; o = al256(o + 8 * 4 * (size_t)(nm + 1));
    o_zero = o;
    for (uint32_t j = 0; j < nm; ++j) {
      Off& f = off[j];
      f.rank = o; o = al256(o + 4 * sh[j].ncand);
      f.split = o; o = al256(o + 8 * (size_t)sh[j].B);
      f.state = o; o = al256(o + 8 * (size_t)sh[j].T);
    }
    o_ticket = o; o = al256(o + 8);
    o_misc = o; o = al256(o + 16 * (size_t)nm);  // per merge: bad, nout
    zero_len = o - o_zero;
    for (uint32_t j = 0; j < nm; ++j) {
      off[j].seg = o;
      o = al256(o + 4 * (size_t)(sh[j].T + 1) * sh[j].K);
      off[j].candk = o;
      o = al256(o + 8 * sh[j].ncand);
    }
    bytes = o;
    nwaves = ncand = nseg = ntiles = maxT = 0;
    // the fewest candidates per thread that still gives >= 512 rank workgroups
    uint64_t w16 = 0, w4 = 0;
    for (const NwShape& x : sh) {
      w16 += x.waves(16);
      w4 += x.waves(4);
    }
    rk_per = w16 >= 512 ? 16u : (w4 >= 512 ? 4u : 1u);
    for (const NwShape& x : sh) {
      nwaves += x.waves(rk_per);
      ncand += x.ncand;
      nseg += (uint64_t)(x.T + 1) * x.K;
      ntiles += x.T;
      maxT = std::max<uint64_t>(maxT, x.T);
    }
  }
#ifndef PSG_NW_RR
#define PSG_NW_RR 1
#endif
  // round-robin tickets run maxT * nm workgroups: only where that stays
  // within a small factor of the tiles (a skewed batch -- one large merge and
  // many one-tile merges -- would launch mostly idle workgroups)
  bool rr() const { return PSG_NW_RR && nm > 1 && maxT * nm <= 2 * ntiles; }
  uint64_t tickets() const { return rr() ? maxT * nm : ntiles; }

  unsigned long long* misc(char* b, uint32_t j) const {
    return (unsigned long long*)(b + o_misc) + 2 * (size_t)j;
  }

  NwBatch batch(char* b) const {
    NwBatch B{};
    B.args = (const NwArgs*)(b + o_args);
    const uint64_t* pre = (const uint64_t*)(b + o_pre);
    B.wpre = pre;
    B.cpre = pre + (nm + 1);
    B.spre = pre + 2 * (size_t)(nm + 1);
    B.tpre = pre + 3 * (size_t)(nm + 1);
    B.ticket = (unsigned int*)(b + o_ticket);
    B.nm = nm;
    B.rr = rr() ? 1u : 0u;
    return B;
  }

  // the tables into the scratch b (one copy on st; synchronous: the host
  // image is freed on return).  Arrays as plan(): pk / pn / pv back to back
  // over the merges, out_keys[j], out_vals[j * m + i].
  hipError_t upload(char* b, const uint64_t* const* pk, const void* const* pv,
                    const uint64_t* pn, uint64_t* const* out_keys, const void* const* ov,
                    uint32_t flags, hipStream_t st) const {
    std::vector<char> h(o_zero, 0);
    std::vector<NwArgs> args(nm);
    std::vector<uint64_t> pre(4 * (size_t)(nm + 1), 0);
    size_t pcur = 0;
    for (uint32_t j = 0; j < nm; ++j) {
      const NwShape& x = sh[j];
      const Off& f = off[j];
      const uint32_t K = x.K;
      if (K) memcpy(h.data() + f.k, pk + pcur, 8 * (size_t)K);
      if (K && m) memcpy(h.data() + f.v, pv + pcur * m, 8 * (size_t)K * m);
      if (K) memcpy(h.data() + f.n, pn + pcur, 8 * (size_t)K);
      memcpy(h.data() + f.cb, x.cbase.data(), 8 * (size_t)(K + 1));
      if (m) memcpy(h.data() + f.ov, ov + (size_t)j * m, 8 * (size_t)m);
      pcur += K;
      NwArgs& A = args[j];
      A.keys = (const uint64_t* const*)(b + f.k);
      A.vals = (const void* const*)(b + f.v);
      A.n = (const uint64_t*)(b + f.n);
      A.cbase = (const uint64_t*)(b + f.cb);
      A.candk = (uint64_t*)(b + f.candk);
      A.out_vals = (void* const*)(b + f.ov);
      A.rank = (uint32_t*)(b + f.rank);
      A.split = (uint64_t*)(b + f.split);
      A.state = (unsigned long long*)(b + f.state);
      A.bad = misc(b, j);
      A.nout = misc(b, j) + 1;
      A.seg = (uint32_t*)(b + f.seg);
      A.out_keys = out_keys[j];
      A.ncand = x.ncand;
      A.K = K;
      A.B = x.B;
      A.T = x.T;
      A.s = x.s;
      A.cw = x.cw;
      A.flags = flags;
      pre[j + 1] = pre[j] + x.waves(rk_per);
      pre[(nm + 1) + j + 1] = pre[(nm + 1) + j] + x.ncand;
      pre[2 * (nm + 1) + j + 1] = pre[2 * (nm + 1) + j] + (uint64_t)(x.T + 1) * K;
      pre[3 * (nm + 1) + j + 1] = pre[3 * (nm + 1) + j] + x.T;
    }
    memcpy(h.data() + o_args, args.data(), sizeof(NwArgs) * nm);
    memcpy(h.data() + o_pre, pre.data(), 8 * pre.size());
    hipError_t e = hipMemcpyAsync(b, h.data(), o_zero, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
  }
};

// one run of the batch: clear, then the 5 stages, each one launch over every
// merge (merges of no pushes have no work items; their count stays 0)
hipError_t nway_enqueue(char* b, const NwLayout& L, int dtype, hipStream_t st) {
  hipError_t e = hipMemsetAsync(b + L.o_zero, 0, L.zero_len, st);
  if (e != hipSuccess || L.ntiles == 0) return e;
  const NwBatch B = L.batch(b);
  if (L.ncand) {
    hipLaunchKernelGGL(nw_gather_kernel, dim3((uint32_t)((L.ncand + 255) / 256)), dim3(256), 0, st,
                       B, L.ncand);
    if (L.rk_per == 16)
      hipLaunchKernelGGL(nw_rank_kernel<16>, dim3((uint32_t)L.nwaves), dim3(256), 0, st, B);
    else if (L.rk_per == 4)
      hipLaunchKernelGGL(nw_rank_kernel<4>, dim3((uint32_t)L.nwaves), dim3(256), 0, st, B);
    else
      hipLaunchKernelGGL(nw_rank_kernel<1>, dim3((uint32_t)L.nwaves), dim3(256), 0, st, B);
    hipLaunchKernelGGL(nw_bucket_kernel, dim3((uint32_t)((L.ncand + 255) / 256)), dim3(256), 0, st,
                       B, L.ncand);
  }
  hipLaunchKernelGGL(nw_split_kernel, dim3(L.nm), dim3(256), 0, st, B);
  if (L.nseg)
    hipLaunchKernelGGL(nw_seg_kernel, dim3((uint32_t)((L.nseg + 255) / 256)), dim3(256), 0, st, B,
                       L.nseg);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return dtype == PSG_F32 ? launch_tile_m<float>(L.m, B, L.tickets(), st)
                          : launch_tile_m<double>(L.m, B, L.tickets(), st);
}

// One keys-only union on `st` into out_keys (>= sum(n) entries), scratch
// from the caller (>= nway_scratch_bytes): the context's key union
// (psg_key_union*).  *d_bad / *d_nout: the device words psg_nway_result reads.
size_t nway_scratch_bytes(uint32_t K, const uint64_t* pn) {
  NwLayout L;
  L.plan(1, &K, pn, 0);
  return L.bytes;
}

hipError_t nway_union_enqueue(uint32_t K, const uint64_t* const* pk, const uint64_t* pn,
                              uint64_t* out_keys, void* scratch, unsigned long long** d_bad,
                              hipStream_t st) {
  NwLayout L;
  L.plan(1, &K, pn, 0);
  char* b = (char*)scratch;
  uint64_t* ok[1] = {out_keys};
  hipError_t e = L.upload(b, pk, nullptr, pn, ok, nullptr, 0, st);
  if (e != hipSuccess) return e;
  *d_bad = L.misc(b, 0);  // [bad, nout]
  return nway_enqueue(b, L, PSG_F32, st);
}

}  // namespace psg

using psg::fail;

struct psg_nway {
  int device = 0, dtype = 0, m = 0;
  uint32_t nm = 0;
  uint64_t ntot = 0;              // keys over all pushes
  uint64_t bytes = 0;             // algorithmic bytes read by a run
  void* blob = nullptr;
  psg::NwLayout layout;
  hipStream_t last = nullptr;
};

namespace {

int nway_create(int device, int dtype, int m, unsigned flags, int nmerge, const int* npush,
                const uint64_t* const* keys, const uint64_t* n, const void* const* vals,
                uint64_t* const* out_keys, void* const* out_vals, psg_nway** out) {
  using namespace psg;
  if (!out || nmerge < 1 || !npush || !out_keys) return fail(PSG_ERR_ARG, "null argument");
  if (dtype != PSG_F32 && dtype != PSG_F64) return fail(PSG_ERR_ARG, "dtype %d", dtype);
  if (m < 0 || m > PSG_MAX_VALUE_ARRAYS || (m > 0 && !out_vals))
    return fail(PSG_ERR_ARG, "m=%d", m);
  size_t tot_push = 0;
  for (int j = 0; j < nmerge; ++j) {
    if (npush[j] < 0) return fail(PSG_ERR_ARG, "merge %d: %d pushes", j, npush[j]);
    if (!out_keys[j]) return fail(PSG_ERR_ARG, "merge %d: null out_keys", j);
    for (int i = 0; i < m; ++i)
      if (!out_vals[(size_t)j * m + i]) return fail(PSG_ERR_ARG, "merge %d: null out_vals", j);
    tot_push += (size_t)npush[j];
  }
  if (tot_push && (!keys || !n || (m > 0 && !vals))) return fail(PSG_ERR_ARG, "null argument");
  HIP_TRY(hipSetDevice(device));
  // empty pushes are ignored (kv_vector.h:90,177): push 0 of a merge is its
  // first non-empty one
  std::vector<const uint64_t*> pk;
  std::vector<const void*> pv;
  std::vector<uint64_t> pn;
  std::vector<uint32_t> kept(nmerge, 0);
  uint64_t ntot = 0;
  size_t p = 0;
  for (int j = 0; j < nmerge; ++j) {
    uint64_t mt = 0;
    for (int e = 0; e < npush[j]; ++e, ++p) {
      if (n[p] == 0) continue;
      if (!keys[p]) return fail(PSG_ERR_ARG, "merge %d push %d: null keys", j, e);
      pk.push_back(keys[p]);
      for (int i = 0; i < m; ++i) {
        if (!vals[p * m + i]) return fail(PSG_ERR_ARG, "merge %d push %d: null values", j, e);
        pv.push_back(vals[p * m + i]);
      }
      pn.push_back(n[p]);
      ++kept[j];
      mt += n[p];
    }
    if (kept[j] > (uint32_t)kMaxRuns)
      return fail(PSG_ERR_ARG, "merge %d: %u pushes > %d per merge", j, kept[j], kMaxRuns);
    if (mt >= (1ull << 32))
      return fail(PSG_ERR_ARG, "merge %d: %llu keys >= 2^32", j, (unsigned long long)mt);
    ntot += mt;
  }
  psg_nway* u = new psg_nway();
  u->device = device;
  u->dtype = dtype;
  u->m = m;
  u->nm = (uint32_t)nmerge;
  u->ntot = ntot;
  u->layout.plan((uint32_t)nmerge, kept.data(), pn.data(), m);
  if (hipMalloc(&u->blob, u->layout.bytes) != hipSuccess) {
    const size_t want = u->layout.bytes;
    delete u;
    return fail(PSG_ERR_OOM, "nway: %zu bytes", want);
  }
  const hipError_t e = u->layout.upload(
      (char*)u->blob, pk.data(), pv.data(), pn.data(), out_keys, (const void* const*)out_vals,
      (flags & PSG_PARALLEL_MATCH) ? kFlagParallel : 0u, nullptr);
  if (e != hipSuccess) {
    (void)hipFree(u->blob);
    delete u;
    return fail(PSG_ERR_DEVICE, "nway set-up: %s", hipGetErrorString(e));
  }
  // SURVEY 8d general form, the read side: every push's keys and values
  // (the merged output adds |union| * (8 + m s_V), known after a run)
  u->bytes = ntot * (8 + (uint64_t)m * (dtype == PSG_F32 ? 4 : 8));
  *out = u;
  return PSG_OK;
}

}  // namespace

extern "C" {

#ifdef PSG_NWAY_PROF
int psg_debug_nway_prof(unsigned long long* out, uint32_t n) {
  if (n > 65536) n = 65536;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(psg::g_nwprof), (size_t)n * 64) == hipSuccess ? 0 : -1;
}
#endif

int psg_nway_max_push(void) { return psg::kMaxRuns; }

int psg_nway_create(int device, int dtype, int m, unsigned flags, int npush,
                    const uint64_t* const* keys, const uint64_t* n, const void* const* vals,
                    uint64_t* out_keys, void* const* out_vals, psg_nway** out) {
  if (npush < 0) return fail(PSG_ERR_ARG, "npush %d", npush);
  uint64_t* ok[1] = {out_keys};
  return nway_create(device, dtype, m, flags, 1, &npush, keys, n, vals, ok, out_vals, out);
}

int psg_nway_create_batch(int device, int dtype, int m, unsigned flags, int nmerge,
                          const int* npush, const uint64_t* const* keys, const uint64_t* n,
                          const void* const* vals, uint64_t* const* out_keys,
                          void* const* out_vals, psg_nway** out) {
  return nway_create(device, dtype, m, flags, nmerge, npush, keys, n, vals, out_keys, out_vals,
                     out);
}

int psg_nway_run(psg_nway* u, void* stream) {
  if (!u) return fail(PSG_ERR_ARG, "null merge");
  HIP_TRY(hipSetDevice(u->device));
  hipStream_t st = (hipStream_t)stream;
  u->last = st;
  HIP_TRY(psg::nway_enqueue((char*)u->blob, u->layout, u->dtype, st));
  return PSG_OK;
}

int psg_nway_count_dev(psg_nway* u, unsigned long long** nout) {
  if (!u || !nout) return fail(PSG_ERR_ARG, "null argument");
  *nout = u->layout.misc((char*)u->blob, 0) + 1;
  return PSG_OK;
}

int psg_nway_result(psg_nway* u, uint64_t* nout) {
  if (!u) return fail(PSG_ERR_ARG, "null merge");
  HIP_TRY(hipSetDevice(u->device));
  if (u->last) HIP_TRY(hipStreamSynchronize(u->last));
  std::vector<unsigned long long> h(2 * (size_t)u->nm);  // per merge: bad, nout
  HIP_TRY(hipMemcpy(h.data(), u->layout.misc((char*)u->blob, 0), 8 * h.size(),
                    hipMemcpyDeviceToHost));
  unsigned long long dev = 0, bad = 0;
  for (uint32_t j = 0; j < u->nm; ++j) {
    if (nout) nout[j] = h[2 * j + 1];
    dev |= h[2 * j] >> 32;
    bad += h[2 * j] & 0xffffffffull;
  }
  if (dev) return fail(PSG_ERR_DEVICE, "nway: tile overflow / look-back timeout (%llx)", dev);
  if (bad)
    return fail(PSG_ERR_UNSORTED, "nway: %llu keys out of order (pushes must be strictly "
                "increasing)", bad);
  return PSG_OK;
}

int psg_nway_bytes(psg_nway* u, uint64_t* bytes, uint64_t* kv) {
  if (!u) return fail(PSG_ERR_ARG, "null merge");
  if (bytes) *bytes = u->bytes;
  if (kv) *kv = u->ntot;
  return PSG_OK;
}

int psg_nway_destroy(psg_nway* u) {
  if (!u) return PSG_OK;
  (void)hipSetDevice(u->device);
  if (u->last) (void)hipStreamSynchronize(u->last);
  (void)hipFree(u->blob);
  delete u;
  return PSG_OK;
}

}  // extern "C"
