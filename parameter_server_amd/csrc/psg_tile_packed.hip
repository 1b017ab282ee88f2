// psg_tile_packed.hip -- the aggregate kernel for sparse jobs (many short
// pieces per tile): one 512-thread workgroup (8 waves) per tile of
// kTS = 2048 server slots (twice the tile kernel's: a push's piece per tile
// doubles, so each round's loads touch half as many pushes' pages per
// element; 4 workgroups, 32 waves per CU).  Jobs whose pieces are long go to psg_tile.hip's push-uniform
// rounds instead (the runtime picks by mean piece length, kPackBelow).
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267): out[j] = fold over pushes p in arrival
// order of V_p[k] where S_p[k] == D[lo+j]; the first push assigns, later
// pushes add, and the serial path adds +0.0 for every absent push (one
// "+0.0" per run of absent pushes is exact: x + 0.0 + 0.0 == x + 0.0).
//
// Shape:
//   * the partition (psg_partition.hip) has cut every push at every tile:
//     push q's keys of this tile are S_q[seg(q, t), seg(q, t+1));
//   * pushes are taken in groups of <= kG = 256 (waves 0 and 1, two per
//     lane; cfg5's 256 pushes are one group: one table chain and, at
//     ~8 keys per push per tile, one pass per tile) whose
//     elements fit one pass; the group's pieces are concatenated push-major
//     and cut into ROUNDS of 64 consecutive elements, so a round may hold the
//     tail of one piece and the heads of the next (short pieces of many
//     sparse pushes fill a round instead of leaving it mostly idle); each
//     push's lane writes its elements' push index into an LDS map, so a lane
//     finds its element's push with one LDS read;
//   * each wave takes a contiguous run of rounds per pass and issues all
//     its element loads before the tile's bucket table is built;
//   * D goes to LDS; a bucket table (1 bucket per slot over the tile's key
//     range, one high multiply) turns a search into one table read and one
//     paired key read;
//   * the fold runs wave by wave (8 barrier steps): rounds are push-major
//     and waves hold contiguous runs of them, so every slot sees its
//     contributions in arrival order with no atomics.  Inside one round two
//     pushes can hit one slot: a per-wave slot bitmap detects that, and such
//     a round folds push by push in lane (= push) order;
//   * thread t owns slots 4t..4t+3: 16-B loads of D and 16-B stores;
//   * consecutive tiles run on one XCD (blocks b and b+8 share one), so the
//     cache lines two neighbouring tiles' pieces share are read once.
// Order check: inside a push's piece the matched positions must increase
// strictly and every key must be found; the piece boundaries come from the
// tile's key bounds, so this is the reference's matched == n <=> sorted,
// unique, inside the range.
//
// Cursor form (CUR, plans of <= 256 pushes on a resident index): no
// partition pass.  A workgroup walks a CHUNK of consecutive tiles of one job
// and keeps each push's cursor (the first key not merged yet) in LDS as the
// piece pointer itself; two lanes per push (all 8 waves) load the 16 keys at
// the cursor, and the piece is the keys before the first one >= the next
// tile's first server key (lower_bound, message.h:96-99).  The same lanes
// touch the piece's value lines, so the pass's element loads that follow hit
// L2: each push key is read from HBM once per run (the partition read every
// key once more, cfg5: 0.58 GB).  Piece pointers then point at the piece's
// END with its length in the top 16 bits (device addresses are < 2^48), so
// the next tile starts there; pieces are cut at kTS keys (keys past it can
// only fail, and do so in the next tile).  Chunk boundaries: each chunk
// starts from lower_bound(push, its first key) and xors its start and end
// cursors into the word it shares with its neighbour (a nonzero word = an
// unsorted push); the job's first and last chunks write the covered range.
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

#ifndef PSG_SKELETON
#define PSG_SKELETON 0  // diagnostic A/B builds: 1 = loads and stores only
#endif

constexpr int kTS = kPackTileSlots;  // slots per tile
constexpr int kNT = kTS / 4;         // threads (512 for 2048-slot tiles)
constexpr int kNW = kNT / 64;    // waves
constexpr int kSPT = kTS / kNT;  // slots per thread (contiguous)
constexpr int kNB = kTS;         // buckets (one per slot: the LDS budget of 4 workgroups per CU)
constexpr int kBPT = kNB / kNT;  // bucket-table entries per thread in the scan
constexpr int kCap = 5;          // rounds a wave holds per pass
constexpr int kG = 256;          // pushes per group (waves 0 and 1, two per lane)
constexpr int kECap = kNW * kCap * 64;  // elements per group: one pass
static_assert(kSPT == 4 && kBPT == 4, "layout");
static_assert(kTS <= 0x7ffe, "u16 positions");
static_assert(kG <= 256, "u8 element -> push map, 8-bit push field of a round entry");
static_assert(kECap >= kTS, "a piece (<= kTS keys) always fits a group");
static_assert(kNT / 2 == kG, "cursor form: two lanes per push");
static_assert(kTS < 65536, "cursor form: a piece length in 16 bits");
constexpr uint64_t kPtrMask = (1ull << 48) - 1;  // cursor form: pointer bits of a piece word
#ifndef PSG_PC_TOUCH
#define PSG_PC_TOUCH 1  // A/B builds: 0 = the cursor phase does not touch the value lines
#endif

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

#ifndef PSG_DDMA
#define PSG_DDMA 1  // A/B builds: 0 = D and the resident bucket table through registers
#endif
// 16 B per lane from global memory straight into LDS (gfx950 LDS-DMA), as
// in psg_tile.hip: inline asm (the builtin made the compiler wait for it at
// the next reuse of its address registers); readers wait with dma_wait()
typedef __attribute__((address_space(3))) void* LdsPtr;
__device__ __forceinline__ void dma16(const void* g, void* lds) {
  const uint32_t la = (uint32_t)(uintptr_t)(LdsPtr)lds;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(la)
      : "memory");
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// a barrier for LDS writes that leaves vector-memory operations in flight
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// the lane index recomputed from nothing (mbcnt over a full mask), so a value
// needed late in the kernel does not keep the thread-id register live (at 64
// VGPRs it is the value that would be spilled to scratch: HBM writes)
__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// blocks b and b+8 share an XCD (observed dispatch, speed only): give each
// XCD a contiguous run of tiles
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + j;
}

// inclusive 64-lane prefix sum by DPP (row shifts, then row broadcasts):
// immediate lane controls, so no per-lane shuffle addresses stay live
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// waves per SIMD the LDS allows (8 for the f32, m = 1 case: 4 workgroups per CU):
// the register budget follows it through __launch_bounds__
// D, buckets, sums, last-push marks, group tables, element map, bitmap,
// per-wave words (40.9 KB for 2048-slot tiles, f32, m = 1)
template <typename V, int M>
constexpr int lds_bytes() {
  return (kTS + 8) * 8 + (kTS + 8) * 2 + M * (int)sizeof(V) * kTS + 2 * kTS + 4 * (kG + 1) +
         kECap + 8 * kG * (1 + M) + 12 * kNW + 48;
}
template <typename V, int M>
constexpr int occupancy() {
  constexpr int lds = lds_bytes<V, M>();
  // waves per SIMD (the launch bound's unit): workgroups per CU x waves / 4
  constexpr int w = (163840 / lds) * kNW / 4;
  return w >= 8 ? 8 : (w < 1 ? 1 : w);
}

// rounds of 64 consecutive elements of the concatenated pieces: a round
// can hold several pushes
template <typename V, int M, bool CUR>
__global__ __launch_bounds__(kNT, (occupancy<V, M>())) void tile_packed_kernel(
    const TileDesc* __restrict__ tiles, uint32_t ntiles, const CursorChunk* __restrict__ chunks,
    uint32_t nchunks, uint32_t* __restrict__ bx) {
  __shared__ __attribute__((aligned(16))) uint64_t dk[kTS + 8];
  // bucket starts (u16); the histogram counts in it as packed pairs by 32-bit atomics
  __shared__ __attribute__((aligned(16))) uint32_t bt32[(kNB + 8) / 2];
  uint16_t* const bt = (uint16_t*)bt32;
  __shared__ __attribute__((aligned(16))) V acc[M][kTS];
  // last push holding the slot, relative to the group base g0: last + 2 - g0,
  // 0 when it precedes g0 - 1 (<= kG + 1 for any push count)
  __shared__ __attribute__((aligned(16))) uint16_t lastl[kTS];
  // pre[q] = elements of the group before push q; ep[e] = push of the
  // group's element e (written by the push's lane: one LDS read per element
  // instead of a search over pre)
  __shared__ uint32_t pre[kG + 1];
  __shared__ uint8_t ep[kECap];
  __shared__ uint64_t pkp[kG], pvp[kG * M];  // piece starts (keys, values)
  __shared__ int lastpos[kNW];
  __shared__ int pcarry;
  __shared__ uint32_t wsum[kNW];
  // pushes in the group, elements of the group, wave 0's element count
  __shared__ uint32_t gsh[3];
  // pushes of the group whose piece overflowed (an unsorted or duplicated
  // push): phase B recounts them; rare, so not kept in registers
  __shared__ uint32_t ovf[kG / 32];

  const uint32_t w = uni((uint32_t)threadIdx.x >> 6);
  const int tid = threadIdx.x;
  // the tiles of this workgroup: one (partition form), or a chunk (cursor form)
  uint32_t tb, te, ci = 0;
  if constexpr (CUR) {
    ci = xcd_tile(blockIdx.x, gridDim.x);
    if (ci >= nchunks) return;
    tb = chunks[ci].t0;
    te = chunks[ci].t1;
  } else {
    tb = xcd_tile(blockIdx.x, gridDim.x);
    if (tb >= ntiles) return;
    te = tb + 1u;
  }
  // cursor form: keys of push tid >> 1 not merged yet (both lanes of the pair)
  uint32_t rem = 0;
  if constexpr (CUR) {
    // start cursors: lower_bound(push q, the chunk's first server key)
    const TileDesc& T0 = tiles[tb];
    const uint32_t q = (uint32_t)tid >> 1;
    if (q < T0.np) {
      const uint64_t* S = G(T0.pkeys)[q];
      const uint64_t n = G(T0.pn)[q];
      const uint64_t c = dev::interp_lower_bound(S, n, G(T0.dk)[0]);
      rem = (uint32_t)(n - c);
      if ((tid & 1) == 0) {
        pkp[q] = (uint64_t)(S + c);
        if (T0.slot0 == 0) GW(const_cast<uint32_t*>(T0.seg))[(size_t)q * T0.stride] = (uint32_t)c;
        else atomicXor(bx + (size_t)ci * kG + q, (uint32_t)c);
      } else {
#pragma unroll
        for (int mi = 0; mi < M; ++mi)
          pvp[q * M + mi] = (uint64_t)((const V*)G(T0.pvals)[(size_t)q * M + mi] + c);
      }
    }
    // the pair's other lane reads pkp[q] next: LDS accesses of one wave are
    // in order, the fences keep the compiler from moving them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  for (uint32_t ti = tb;; ++ti) {  // the partition form: one tile, no loop
  // the thread id afresh per tile (opaque): values derived from it are
  // recomputed in the loop instead of held (and spilled) across it
  int tid = threadIdx.x;
  if constexpr (CUR) asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const TileDesc& T = tiles[ti];
  const uint32_t np = T.np;
  const uint32_t nt = T.nt;
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  const uint64_t* Dg = T.dk;

  // ---- push tables of a group: waves 0 and 1, pushes w*128 + lane and
  // w*128 + 64 + lane.  Phase A loads the pieces, writes their start
  // pointers and each wave's own inclusive prefix of the lengths (pre[q+1])
  // into LDS; phase B (after a barrier: wave 1 needs wave 0's total) turns
  // them into the group's prefix, keeps the pushes whose elements fit one
  // pass and writes the element -> push map.  Nothing stays in registers
  // across the barrier but the group size.
  uint32_t tgq = 0;
  // a piece's overflow: keys past the tile or bounds out of order (they
  // cannot all match)
  auto piece = [&](uint32_t q, uint32_t* a_out, uint32_t* over) -> uint32_t {
    const uint32_t* sg = T.seg + (size_t)q * T.stride;
    const uint32_t n = (uint32_t)G(T.pn)[q];
    uint32_t a = G(sg)[0], b = G(sg)[T.segb];
    // bounds from a failed partition (an unsorted push) stay inside the push
    a = a < n ? a : n;
    b = b < n ? b : n;
    *over = b < a ? 1u : (b - a > (uint32_t)kTS ? b - a - (uint32_t)kTS : 0u);
    *a_out = a;
    return b > a ? (b - a < (uint32_t)kTS ? b - a : (uint32_t)kTS) : 0u;
  };
  auto tables_a = [&](uint32_t g0) {
    if (w < 2) {
      // a fresh copy of the lane id per call: otherwise the compiler hoists
      // the lane-derived LDS addresses out of the push-group loop and, at
      // 64 VGPRs, spills them to scratch in every workgroup (HBM writes)
      int lane = (int)lane_id();
      asm volatile("" : "+v"(lane));
      tgq = np - g0 < (uint32_t)kG ? np - g0 : (uint32_t)kG;
      uint32_t len[2], ov[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        len[h] = 0;
        ov[h] = 0;
        const uint32_t ql = 128u * w + (uint32_t)lane + 64u * h;
        if (ql < tgq) {
          const uint32_t q = g0 + ql;
          uint32_t a;
          len[h] = piece(q, &a, &ov[h]);
          // a push that does not fit this group's pass is written again
          // (at its new index) by the next group's phase A
          pkp[ql] = (uint64_t)(G(T.pkeys)[q] + a);
#pragma unroll
          for (int mi = 0; mi < M; ++mi)
            pvp[ql * M + mi] = (uint64_t)((const V*)G(T.pvals)[(size_t)q * M + mi] + a);
        }
      }
      // elements through each push, inside this wave
      const uint32_t x0 = wave_scan_incl(len[0]);
      const uint32_t x1 = wave_scan_incl(len[1]) + uni(__builtin_amdgcn_readlane((int)x0, 63));
      const uint32_t ql0 = 128u * w + (uint32_t)lane;
      if (ql0 < tgq) pre[ql0 + 1] = x0;
      if (ql0 + 64u < tgq) pre[ql0 + 65] = x1;
      if (w == 0 && lane == 63) gsh[2] = x1;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const unsigned long long om = __ballot(ov[h] != 0u);
        if (lane < 2) ovf[4u * w + 2u * h + lane] = (uint32_t)(om >> (32 * lane));
      }
      if (w == 0 && lane == 0) {
        uint32_t z = 0;  // opaque zero: not a constant kept (and spilled) across the loop
        asm volatile("" : "+v"(z));
        gsh[0] = z;
        gsh[1] = z;
      }
    }
  };
  auto tables_b = [&](uint32_t g0) {
    if (w < 2) {
      int lane = (int)lane_id();
      asm volatile("" : "+v"(lane));
      const uint32_t base = w == 1 ? uni(gsh[2]) : 0u;
      uint32_t xl[2], pl[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // all reads before any write
        const uint32_t ql = 128u * w + (uint32_t)lane + 64u * h;
        xl[h] = ql < tgq ? pre[ql + 1] : 0u;
        pl[h] = (h == 0 && lane == 0) || ql >= tgq ? 0u : pre[ql];
      }
      uint32_t fit = 0, emax = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t ql = 128u * w + (uint32_t)lane + 64u * h;
        const uint32_t x = xl[h] + base;
        // the group: the pushes whose elements fit one pass (a prefix; >= 1:
        // a piece is <= kTS)
        const bool in = ql < tgq && x <= (uint32_t)kECap;
        fit += (uint32_t)__popcll(__ballot(in));
        if (in) {
          if ((ovf[ql >> 5] >> (ql & 31u)) & 1u) {  // recount the overflow (rare)
            uint32_t a, over;
            (void)piece(g0 + ql, &a, &over);
            __hip_atomic_fetch_add(GW(T.fail) + g0 + ql, (unsigned long long)over,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          pre[ql + 1] = x;
#pragma nounroll
          for (uint32_t e = x - (xl[h] - pl[h]); e < x; ++e) ep[e] = (uint8_t)ql;
          emax = x;  // increasing with ql: the last fitting push's count
        }
      }
      // wave maximum of the fitting counts
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)emax, o, 64);
        emax = y > emax ? y : emax;
      }
      if (lane == 0) {
        __hip_atomic_fetch_add(&gsh[0], fit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_max(&gsh[1], emax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (w == 0) pre[0] = 0;
      }
    }
  };
  // ---- cursor form: the tables of the group at g0 from the cursors, all 8
  // waves, push g0 + (t >> 1) on lanes t (h = 0) and t + 1 (h = 1).  Phase A
  // (`first`: the tile's first group) finds each piece: the pair loads the
  // 16 keys at the cursor (8 each), the piece ends before the first key >=
  // the next tile's first key (16 more at a time for a longer piece), and
  // moves the piece words to the piece's end.  A later group of the same
  // tile reads the lengths back from the words.  Returns the push's piece
  // length (h = 0 lanes) and its wave-inclusive prefix in *x; the wave
  // totals go to wsum.
  const bool lastt = CUR && (T.flags & kFlagLastTile) != 0u;
  const uint64_t dlast = lastt ? G(Dg)[nt - 1] : 0ull;
  // the piece bound: keys < the next tile's first key; the job's last tile
  // takes every key <= D[nslots - 1] (open: D ends at 2^64 - 1)
  const bool open = lastt && dlast == ~0ull;
  const uint64_t nxt = !CUR ? 0ull : lastt ? dlast + 1ull : G(Dg)[kTS];
  auto cur_a = [&](uint32_t g0, bool first, uint32_t* x) -> uint32_t {
    uint32_t t = (uint32_t)threadIdx.x;
    asm volatile("" : "+v"(t));
    const uint32_t h = t & 1u, q = g0 + (t >> 1);
    const bool own = q < np;
    uint32_t len = 0;
    if (first) {
      uint64_t st = 0;
      auto piece8 = [&](uint32_t b) -> uint32_t {  // keys [b + 8h, b + 8h + 8): leading keys < nxt
        const uint32_t o = b + 8u * h;
        const uint32_t avail = rem > o ? rem - o : 0u;
        const AS1 uint64_t* S = G((const uint64_t*)st) + o;
        uint32_t lt = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint64_t k = (uint32_t)j < avail ? S[j] : ~0ull;
          lt |= (uint32_t)((uint32_t)j < avail && (open || k < nxt)) << j;
        }
        return (uint32_t)__builtin_ctz(~lt);
      };
      uint32_t f = 8;
      if (own) {
        st = pkp[q] & kPtrMask;
        f = piece8(0);
#if PSG_PC_TOUCH
        // the piece's value lines (its first 16 values), so the pass's
        // element loads find them in L2
        const uint32_t o = 8u * h;
        if (rem > o) {
          const uint32_t e = rem - o < 8u ? rem - o - 1u : 7u;
#pragma unroll
          for (int mi = 0; mi < M; ++mi) {
            const AS1 V* pv = G((const V*)pvp[q * M + mi]) + o;
            const V v0 = pv[0], v1 = pv[e];
            asm volatile("" ::"v"(v0), "v"(v1));
          }
        }
#endif
      }
      const uint32_t fo = (uint32_t)__shfl_xor((int)f, 1, 64);
      len = (h ? fo : f) < 8u ? (h ? fo : f) : 8u + (h ? f : fo);
      if (own && len == 16u && rem > 16u) {  // a longer piece (rare): 16 keys a step
        for (uint32_t b = 16;; b += 16) {
          const uint32_t g = piece8(b);
          const uint32_t go = (uint32_t)__shfl_xor((int)g, 1, 64);
          const uint32_t l = (h ? go : g) < 8u ? (h ? go : g) : 8u + (h ? g : go);
          len = b + l;
          if (l < 16u || b + 16u >= rem || len >= (uint32_t)kTS) break;
        }
      }
      len = len < (uint32_t)kTS ? len : (uint32_t)kTS;
      if (own) {
        if (h == 0u) {
          pkp[q] = (st + 8ull * len) | (uint64_t)len << 48;
        } else {
#pragma unroll
          for (int mi = 0; mi < M; ++mi) pvp[q * M + mi] += (uint64_t)len * sizeof(V);
        }
        rem -= len;
      }
    } else {
      len = own ? (uint32_t)(pkp[q] >> 48) : 0u;
    }
    const uint32_t lv = own && h == 0u ? len : 0u;
    *x = wave_scan_incl(lv);
    if (lane_id() == 63u) wsum[w] = *x;
    if (t == 0u) {
      uint32_t z = 0;  // opaque zero (as in tables_a)
      asm volatile("" : "+v"(z));
      gsh[0] = z;
      gsh[1] = z;
    }
    return lv;
  };
  // phase B (after a barrier): the group's prefix, the pushes whose elements
  // fit one pass (a prefix of them), the element -> push map
  auto cur_b = [&](uint32_t g0, uint32_t lv, uint32_t x) {
    uint32_t t = (uint32_t)threadIdx.x;
    asm volatile("" : "+v"(t));
    const uint32_t ql = t >> 1;
    uint32_t base = 0;
#pragma unroll
    for (uint32_t v = 0; v < (uint32_t)kNW - 1u; ++v) base += v < w ? wsum[v] : 0u;
    const uint32_t X = x + base;  // elements of the group through push ql
    // X grows with ql, so the pushes that fit are a prefix
    const bool in = (t & 1u) == 0u && g0 + ql < np && X <= (uint32_t)kECap;
    const uint32_t fit = (uint32_t)__popcll(__ballot(in));
    uint32_t emax = in ? X : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t y = (uint32_t)__shfl_xor((int)emax, o, 64);
      emax = y > emax ? y : emax;
    }
    if (in) {
      pre[ql + 1] = X;
#pragma nounroll
      for (uint32_t e = X - lv; e < X; ++e) ep[e] = (uint8_t)ql;
    }
    if (lane_id() == 0u) {
      __hip_atomic_fetch_add(&gsh[0], fit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_max(&gsh[1], emax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (t == 0u) pre[0] = 0;
  };
  // ---- D keys, continued sums: thread t owns slots 4t..4t+3
  const uint32_t s0i = 4u * (uint32_t)tid;
  // the plan's resident bucket table (psg_tile.hip bucket_index_kernel<64>:
  // the same 2048 buckets over the same tile)
  const uint32_t* Bg = T.bt;
  // full tiles of the partition form: D and the resident bucket table by
  // LDS-DMA, left in flight across barriers (1) and (1b) and the element
  // loads (through registers, D had to land before (1) and the element
  // loads went out after it; psg_tile.hip, profiles/r05_phases_cfg2.txt)
  const bool dma = !CUR && PSG_DDMA && nt == (uint32_t)kTS && ((uintptr_t)Dg & 15u) == 0u &&
                   ((uintptr_t)Bg & 15u) == 0u;
  auto issue_dma = [&]() {
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // kTS / 2 16-B units: 2 wave instructions per wave
      const uint32_t c = 2u * w + (uint32_t)j;
      dma16(Dg + 128u * c + 2u * (uint32_t)lane, (char*)dk + 1024u * c);
    }
    static_assert(kNB / 512 <= kNW, "one 1-KB unit of the bucket table per wave at most");
    if (Bg && w < (uint32_t)kNB / 512u)
      dma16((const char*)Bg + 1024u * w + 16u * (uint32_t)lane, (char*)bt32 + 1024u * w);
  };
  if (dma && w >= 2) issue_dma();
  if (np) {
    if constexpr (!CUR) tables_a(0);
  }
  if (dma && w < 2) issue_dma();  // after waves 0-1's table loads: their waits do not wait for D
  if (!dma) {
    // through registers, loaded and installed on this branch only, drained
    // at its end (the compiler's merged wait state otherwise put a vmcnt(0)
    // on the LDS-DMA path)
    uint64_t d[4];
    if (s0i + 3u < nt && ((uintptr_t)Dg & 15u) == 0u) {
      const u64x2 x0 = *(const AS1 u64x2*)(Dg + s0i);
      const u64x2 x1 = *(const AS1 u64x2*)(Dg + s0i + 2);
      d[0] = x0.x; d[1] = x0.y; d[2] = x1.x; d[3] = x1.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = s0i + j < nt ? G(Dg)[s0i + j] : ~0ull;
    }
    u32x2 btw = {0u, 0u};
    if (Bg) btw = __builtin_nontemporal_load((const AS1 u32x2*)Bg + tid);
#pragma unroll
    for (int j = 0; j < 4; ++j) dk[s0i + j] = d[j];
    if (Bg) *(u32x2*)&bt[tid * kBPT] = btw;
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  }
  // cursor form: the pieces, while D and the index are in flight
  uint32_t cx = 0, clv = 0;
  if constexpr (CUR) {
    if (np) clv = cur_a(0, true, &cx);
  }

  // ---- sums, lastl; clear the histogram and the bitmaps (constants as
  // opaque values: hoisted out of the cursor form's tile loop they would
  // hold VGPRs across it, and spill).  The continued sums on their own
  // branch, drained there (as above)
  uint32_t ones = ~0u, one = 1u;
  if constexpr (CUR) asm volatile("" : "+v"(ones), "+v"(one));
  if (cont) {
    V a0[M][4];
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        a0[mi][j] = s0i + j < nt ? G((const V*)T.out[mi] + T.slot0)[s0i + j] : V(0);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mi][s0i + j] = a0[mi][j];
  } else {
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mi][s0i + j] = V(0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) lastl[s0i + j] = (uint16_t)one;  // last = -1 = g0 - 1
  if (tid < 8) dk[kTS + tid] = (uint64_t)ones << 32 | ones;
  {
    uint32_t z = 0;  // opaque zero: not a hoisted (and spilled) constant vector
    asm volatile("" : "+v"(z));
    if (!Bg) *(u32x2*)&bt[tid * kBPT] = u32x2{z, z};  // a cleared histogram
    if (Bg && tid == 0) bt[kNB] = (uint16_t)nt;  // past the table's kNB entries
  }
  if (tid == 0) pcarry = (int)ones;
  if (dma)
    lds_barrier();  // (1) pieces scanned, sums (D and the bucket table in flight)
  else
    __syncthreads();  // (1) pieces scanned, D, cleared histogram (or the resident bucket table)
  if (np) {
    if constexpr (CUR) cur_b(0, clv, cx);
    else tables_b(0);
  }
  if (dma)
    lds_barrier();  // (1b) the group's tables
  else
    __syncthreads();  // (1b) the group's tables

  // ---- a pass: this wave's run of rounds, loaded into registers
  uint32_t gp = np ? uni(gsh[0]) : 0u;
  uint32_t Et = np ? uni(gsh[1]) : 0u;  // elements of the group
  uint32_t U = (Et + 63u) >> 6;        // rounds of the group
  uint32_t done = 0, g0 = 0;
  uint32_t nrw = 0, ua = 0, Rw = 0;
  // per lane and held round r, 10 bits: q | first-of-piece << 8 | exists << 9
  // (packed 3 rounds per register)
  uint32_t rp[(kCap + 2) / 3];
  uint64_t ek[kCap];
  V ev[kCap][M];
  uint32_t mmask = 0;  // wave-uniform: bit r = round r holds more than one push
  auto load_pass = [&]() {
    const uint32_t rem = U - done;
    Rw = (rem + kNW - 1) / kNW;
    Rw = Rw < (uint32_t)kCap ? Rw : (uint32_t)kCap;
    ua = done + w * Rw;
    const uint32_t ub = ua + Rw < U ? ua + Rw : U;
    nrw = ub > ua ? ub - ua : 0u;
    mmask = 0;
#pragma unroll
    for (int r = 0; r < (kCap + 2) / 3; ++r) rp[r] = 0;
#pragma unroll
    for (int r = 0; r < kCap; ++r) {
      if ((uint32_t)r < nrw) {
        const uint32_t R = ua + (uint32_t)r;
        const uint32_t e = R * 64u + (uint32_t)lane;
        const bool have = e < Et;
        // push of element e; lane 0 holds the round's first element, which
        // exists, so its push is a safe address for the lanes past the end
        uint32_t q = ep[have ? e : R * 64u];
        const uint32_t qlo = uni(q);
        mmask |= (__ballot(have && q != qlo) != 0 ? 1u : 0u) << r;
        if constexpr (CUR) {
          // piece words point at the piece's end: element e is `back` before it
          const uint64_t pw = pkp[g0 + q];
          const uint32_t back = have ? pre[q + 1] - e : 1u;
          const bool head = have && back == (uint32_t)(pw >> 48);
          rp[r / 3] |= (q | (uint32_t)head << 8 | (uint32_t)have << 9) << (10 * (r % 3));
          ek[r] = *(G((const uint64_t*)(pw & kPtrMask)) - back);
#pragma unroll
          for (int mi = 0; mi < M; ++mi) ev[r][mi] = *(G((const V*)pvp[(g0 + q) * M + mi]) - back);
        } else {
          const uint32_t i = have ? e - pre[q] : 0u;
          rp[r / 3] |= (q | (uint32_t)(have && i == 0u) << 8 | (uint32_t)have << 9) << (10 * (r % 3));
          ek[r] = G((const uint64_t*)pkp[q])[i];
#pragma unroll
          for (int mi = 0; mi < M; ++mi) ev[r][mi] = G((const V*)pvp[q * M + mi])[i];
        }
      }
    }
  };
  if (U) load_pass();
  if (dma) {  // (1c) D and the bucket table landed (with the element loads)
    dma_wait();
    __syncthreads();
  }

  // bucket of a key: the tile's key range [klo, khi] scaled onto [0, kNB) by
  // one 32x32 high multiply; keys outside the range land in an end bucket
  // and are not found there.  klo, khi from LDS: a global read here would
  // wait for every load in flight
  const uint64_t klo = uni64(dk[0]);
  const uint64_t khi = uni64(dk[nt - 1]);
  const uint64_t range = khi - klo;
  const int bits = range ? 64 - __builtin_clzll(range) : 0;
  const int s2 = bits > 32 ? bits - 32 : 0;
  const uint64_t r32 = range >> s2;  // < 2^32
  const uint32_t mul = dev::bucket_scale(r32, kNB);
  auto bucket = [&](uint64_t k) -> uint32_t {
    const uint64_t x = (k - klo) >> s2;
    return x > r32 ? (uint32_t)(kNB - 1) : __umulhi((uint32_t)x, mul);
  };

  // ---- bucket table: histogram, exclusive scan -> bt[b] = first slot of bucket b
  // (skipped when the plan's resident index supplied it).  D keys back from
  // LDS: the registers that held them are free during the pass's element
  // loads.  `again`: a rebuild after the collision bitmaps used the table's
  // LDS (context flushes whose tile takes another pass): cleared first.
  auto build_bt = [&](bool again) {
    const uint32_t t = 64u * w + lane_id();
    const uint32_t sb = 4u * t;
    if (again) {
      uint32_t z = 0;
      asm volatile("" : "+v"(z));
      *(u32x2*)&bt[t * kBPT] = u32x2{z, z};
      __syncthreads();
    }
    const u64x2 y0 = *(const u64x2*)&dk[sb];
    const u64x2 y1 = *(const u64x2*)&dk[sb + 2];
    const uint64_t dd[4] = {y0.x, y0.y, y1.x, y1.y};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (sb + j < nt)
      {  // counts <= kTS < 2^16: no carry between the packed halves
        const uint32_t b = bucket(dd[j]);
        __hip_atomic_fetch_add(&bt32[b >> 1], 1u << (16 * (b & 1u)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    __syncthreads();  // (2)
    {
      const u32x2 h = *(const u32x2*)&bt[t * kBPT];
      uint32_t e[kBPT] = {h.x & 0xffffu, h.x >> 16, h.y & 0xffffu, h.y >> 16};
      uint32_t tot = 0;
#pragma unroll
      for (int j = 0; j < kBPT; ++j) {
        const uint32_t c = e[j];
        e[j] = tot;
        tot += c;
      }
      const uint32_t x = wave_scan_incl(tot);
      if (lane_id() == 63u) wsum[w] = x;
      __syncthreads();  // (3)
      uint32_t off = x - tot;
#pragma unroll
      for (uint32_t v = 0; v < (uint32_t)kNW - 1u; ++v) off += v < w ? wsum[v] : 0u;
      const u32x2 o = {(e[0] + off) | (e[1] + off) << 16, (e[2] + off) | (e[3] + off) << 16};
      *(u32x2*)&bt[t * kBPT] = o;
      if (t == 0) bt[kNB] = (uint16_t)nt;
    }
    __syncthreads();  // (4)
  };
  if (!Bg) build_bt(false);

  for (;;) {
    if (!U) {  // this group of pushes has no keys in the tile, or is done
      g0 += gp;
      if (g0 >= np) break;
      // rebase lastl on the new group: last == g0 - 1 -> 1, older -> 0
#pragma unroll
      for (int j = 0; j < 4; ++j) lastl[s0i + j] = lastl[s0i + j] == gp + 1u ? 1 : 0;
      if constexpr (CUR) {
        uint32_t x;
        const uint32_t lv = cur_a(g0, false, &x);
        __syncthreads();
        cur_b(g0, lv, x);
      } else {
        tables_a(g0);
        __syncthreads();
        tables_b(g0);
      }
      __syncthreads();
      gp = uni(gsh[0]);
      Et = uni(gsh[1]);
      U = (Et + 63u) >> 6;
      done = 0;
      if (U) load_pass();
      continue;
    }
    auto re = [&](int r) -> uint32_t { return (rp[r / 3] >> (10 * (r % 3))) & 0x3ffu; };
#if PSG_SKELETON == 1
    // diagnostic (A/B builds only): the loads and stores, no search, check
    // or fold -- the memory side's own time
    {
      V t = V(0);
#pragma unroll
      for (int r = 0; r < kCap; ++r)
        if ((uint32_t)r < nrw && ((re(r) >> 9) & 1u)) t += ev[r][0] + (V)(uint32_t)(ek[r] & 1u);
      acc[0][s0i] += t;
      done += kNW * Rw;
      if (done < U) {
        load_pass();
        continue;
      }
      U = 0;
      continue;
    }
#endif
    // ---- search every held round
    uint32_t pos[kCap];
    uint32_t okm = 0;  // per lane: bit r = found; bit 8 + r = found and in order
#pragma unroll
    for (int r = 0; r < kCap; ++r) {
      pos[r] = 0;
      if ((uint32_t)r < nrw) {
        const uint64_t k = ek[r];
        const uint32_t b = bucket(k);
        uint32_t l = bt[b];
        uint32_t n = (uint32_t)bt[b + 1] - l;
        while (n > 2u) {  // crowded bucket
          const uint32_t half = n >> 1;
          if (dk[l + half - 1] < k) {
            l += half;
            n -= half;
          } else {
            n = half;
          }
        }
        const uint64_t k0 = dk[l], k1 = dk[l + 1];
        pos[r] = l + ((n > 0u && k0 < k) ? 1u : 0u) + ((n > 1u && k1 < k) ? 1u : 0u);
        okm |= (uint32_t)((n > 0u && k0 == k) || (n > 1u && k1 == k)) << r;
      }
    }
    int mylast = 0;  // position held by lane 63 in this wave's last round
#pragma unroll
    for (int r = 0; r < kCap; ++r)
      if ((uint32_t)r + 1u == nrw) mylast = (int)pos[r];
    if (nrw && lane == 63) lastpos[w] = mylast;
    __syncthreads();  // (5) lastpos of every wave

    // ---- order check: strictly increasing positions inside a piece
#pragma unroll
    for (int r = 0; r < kCap; ++r) {
      if ((uint32_t)r < nrw) {
        int prev0;  // position of the element before lane 0's
        if (r > 0) prev0 = __builtin_amdgcn_readlane((int)pos[r - 1], 63);
        else prev0 = w > 0 ? lastpos[w - 1] : pcarry;
        int prev = __builtin_amdgcn_update_dpp(prev0, (int)pos[r], 0x138, 0xf, 0xf, false);
        if ((re(r) >> 8) & 1u) prev = -1;  // first element of its piece
        const bool ok = ((re(r) >> 9) & 1u) && ((okm >> r) & 1u) && (int)pos[r] > prev;
        okm |= (uint32_t)ok << (8 + r);
      }
    }
    // elements that exist but did not match: one ballot per pass; counted per
    // push only when there are any
    {
      uint32_t exist = 0;
#pragma unroll
      for (int r = 0; r < kCap; ++r) exist |= ((re(r) >> 9) & 1u) << r;
      const uint32_t badm = exist & ~(okm >> 8);
      if (__ballot(badm != 0u)) {
#pragma unroll
        for (int r = 0; r < kCap; ++r)
          if ((badm >> r) & 1u)
            __hip_atomic_fetch_add(GW(T.fail) + g0 + (re(r) & 255u), 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#if PSG_SKELETON == 2
    // diagnostic: loads, stores, search and order check; no collision test
    // and no fold
    {
      V t = V(0);
#pragma unroll
      for (int r = 0; r < kCap; ++r)
        if ((uint32_t)r < nrw && ((okm >> (8 + r)) & 1u)) t += ev[r][0] + (V)pos[r];
      acc[0][s0i] += t;
      done += kNW * Rw;
      if (done < U) {
        load_pass();
        continue;
      }
      U = 0;
      continue;
    }
#endif
    const uint32_t inpass = (U - done) < kNW * Rw ? U - done : kNW * Rw;
    const uint32_t wl = (inpass - 1) / Rw;  // wave holding the pass's last round
    // ---- rounds holding several pushes: do two of them hit one slot?
    // cl[r] (wave-uniform): the lanes of round r that found their slot's bit
    // already set -- each names a slot hit more than once in the round.
    // Every wave at once, each with its own bitmap in the bucket table's LDS
    // (free once every search of the pass is done, (5); put back -- from the
    // plan's resident index, or rebuilt -- if another pass or group searches).
    unsigned long long cl[kCap];
#pragma unroll
    for (int r = 0; r < kCap; ++r) cl[r] = 0;
    auto collide = [&](uint32_t* cb) {
      if (mmask) {
#pragma unroll
        for (int r = 0; r < kCap; ++r) {
          if ((mmask >> r) & 1u) {
            const bool ok = (okm >> (8 + r)) & 1u;
            const uint32_t s = pos[r], bit = 1u << (s & 31u);
            uint32_t old = 0;
            if (ok) old = __hip_atomic_fetch_or(&cb[s >> 5], bit, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WAVEFRONT);
            cl[r] = __ballot(ok && (old & bit));
            if (ok) cb[s >> 5] = 0u;
          }
        }
      }
    };
    static_assert(kNW * (kTS / 32) <= (kNB + 8) / 2 && kTS / 32 == 64, "per-wave bitmaps in bt");
    {
      uint32_t* const cb = bt32 + w * (kTS / 32);
      cb[lane_id()] = 0u;  // this wave's bitmap (its own LDS accesses stay in order)
      collide(cb);
    }
    // ---- fold, wave by wave (rounds are push-major)
    for (uint32_t st = 0; st < (uint32_t)kNW; ++st) {
      if (st == w) {
#pragma unroll
        for (int r = 0; r < kCap; ++r) {
          if ((uint32_t)r < nrw) {
            bool pend = (okm >> (8 + r)) & 1u;
            const uint32_t q = re(r) & 255u;
            const uint32_t s = pos[r];
            const bool first = g0 + q == 0u && !cont;
            auto apply = [&]() {
              const uint32_t l1 = lastl[s];
              const bool gap = !parallel && l1 <= q;  // last < g0 + q - 1
#pragma unroll
              for (int mi = 0; mi < M; ++mi) {
                const V a = acc[mi][s];
                const V ag = gap ? a + V(0) : a;
                acc[mi][s] = first ? ev[r][mi] : ag + ev[r][mi];
              }
              lastl[s] = (uint16_t)(q + 2u);
            };
            const unsigned long long cm = cl[r];
            if (!cm) {
              if (pend) apply();  // no two lanes of the round on one slot
            } else {
              // lanes on a slot that cm names must go in lane order, which is
              // push order (rounds cut the push-major concatenation); every
              // other lane has a slot of its own and applies at once
              bool inv = false;
              for (unsigned long long t = cm; t; t &= t - 1) {
                const uint32_t sl =
                    (uint32_t)__builtin_amdgcn_readlane((int)s, (int)__builtin_ctzll(t));
                inv |= s == sl;
              }
              if (pend && !inv) {
                apply();
                pend = false;
              }
              // then, per pass, the lowest pending lane of each shared slot
              // (passes = the largest multiplicity, almost always 2)
              for (;;) {
                const unsigned long long im = __ballot(pend);
                if (!im) break;
                bool lowest = pend;
                for (unsigned long long t = im; t; t &= t - 1) {
                  const int j = (int)__builtin_ctzll(t);
                  const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((int)s, j);
                  if (j < lane && s == sl) lowest = false;
                }
                if (lowest) {
                  apply();
                  pend = false;
                }
              }
            }
          }
        }
        if (w == wl && lane == 63) pcarry = mylast;
      }
      __syncthreads();
    }
    // the bucket table back from the resident index when another pass or
    // group searches it (its first half held the collision bitmaps)
    if (done + kNW * Rw < U || g0 + gp < np) {
      if (Bg) {
        const uint32_t t = 64u * w + lane_id();
        *(u32x2*)&bt[t * kBPT] = __builtin_nontemporal_load((const AS1 u32x2*)Bg + t);
        __syncthreads();
      } else {
        build_bt(true);
      }
    }

    // ---- next pass, or next group of pushes
    done += kNW * Rw;
    if (done < U) {
      load_pass();
      continue;
    }
    U = 0;  // group finished
    if (w == 0 && lane_id() == 0u) pcarry = -1;
  }

  // ---- trailing "+0.0" of absent last pushes (serial), stores
  const uint32_t gl = g0 - gp;  // base of the last group (0 without pushes)
  // the slot offset afresh (an opaque thread id): kept live across the main
  // loop it is the one value the 64-VGPR budget spills to scratch
  uint32_t s0 = 64u * w + lane_id();
  asm volatile("" : "+v"(s0));
  s0 *= 4u;
  V res[M][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // gap iff last < np - 1
    const bool gap = !parallel && (uint32_t)lastl[s0 + j] < np - gl + 1u;
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      const V a = acc[mi][s0 + j];
      res[mi][j] = gap ? a + V(0) : a;
    }
  }
#pragma unroll
  for (int mi = 0; mi < M; ++mi) {
    V* o = (V*)T.out[mi] + T.slot0 + s0;
    if (s0 + 3u < nt && ((uintptr_t)o & 15u) == 0u) {
      if constexpr (sizeof(V) == 4) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 v = {res[mi][0], res[mi][1], res[mi][2], res[mi][3]};
        *(AS1 f4*)GW(o) = v;
      } else {
        typedef double d2 __attribute__((ext_vector_type(2)));
        const d2 v0 = {res[mi][0], res[mi][1]};
        const d2 v1 = {res[mi][2], res[mi][3]};
        ((AS1 d2*)GW(o))[0] = v0;
        ((AS1 d2*)GW(o))[1] = v1;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (s0 + j < nt) GW(o)[j] = res[mi][j];
    }
  }
  if constexpr (!CUR) {
    break;
  } else {
    if (ti + 1u >= te) break;
    __syncthreads();  // the next tile's installs overwrite what the stores read
  }
  }  // tiles of the chunk
  if constexpr (CUR) {
    // end cursors: into the boundary word shared with the next chunk, or the
    // covered range's end (the job's last tile)
    const TileDesc& T1 = tiles[te - 1u];
    uint32_t t = (uint32_t)threadIdx.x;  // fresh: the loop's ids are dead
    asm volatile("" : "+v"(t));
    const uint32_t q = t >> 1;
    if (q < T1.np && (t & 1u) == 0u) {
      const uint32_t c = (uint32_t)(((pkp[q] & kPtrMask) - (uint64_t)G(T1.pkeys)[q]) / 8u);
      if (T1.flags & kFlagLastTile) GW(const_cast<uint32_t*>(T1.seg))[(size_t)q * T1.stride + T1.segb] = c;
      else atomicXor(bx + (size_t)(ci + 1u) * kG + q, c);
    }
  }
}

template <typename V, int M>
hipError_t go(const TileDesc* t, uint32_t n, const CursorChunk* ch, uint32_t nch, uint32_t* bx,
              hipStream_t s) {
  if constexpr (lds_bytes<V, M>() <= 163840) {
    if (ch)
      hipLaunchKernelGGL((tile_packed_kernel<V, M, true>), dim3(nch), dim3(kNT), 0, s, t, n, ch,
                         nch, bx);
    else
      hipLaunchKernelGGL((tile_packed_kernel<V, M, false>), dim3(n), dim3(kNT), 0, s, t, n, ch,
                         nch, bx);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;  // larger tiles (A/B builds) hold fewer value arrays
  }
}

template <typename V>
hipError_t launch_m(int m, const TileDesc* t, uint32_t n, const CursorChunk* ch, uint32_t nch,
                    uint32_t* bx, hipStream_t s) {
  switch (m) {
    case 1: return go<V, 1>(t, n, ch, nch, bx, s);
    case 2: return go<V, 2>(t, n, ch, nch, bx, s);
    case 3: return go<V, 3>(t, n, ch, nch, bx, s);
    case 4: return go<V, 4>(t, n, ch, nch, bx, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_tile_packed(int dtype, int m, const TileDesc* d_tiles,
                                        uint32_t ntiles, hipStream_t stream,
                                        const CursorChunk* d_chunks, uint32_t nchunks,
                                        uint32_t* bx) {
  if (ntiles == 0 || (d_chunks && nchunks == 0)) return hipSuccess;
  return dtype == 0 ? launch_m<float>(m, d_tiles, ntiles, d_chunks, nchunks, bx, stream)
                    : launch_m<double>(m, d_tiles, ntiles, d_chunks, nchunks, bx, stream);
}

}  // namespace psg
