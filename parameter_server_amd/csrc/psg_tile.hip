// psg_tile.hip -- the aggregate kernel for long pieces (push-uniform rounds):
// one workgroup per tile of kTS server slots (1024 slots and 256 threads, or
// 2048 and 512 for jobs of more than 32 pushes), built for
// instruction efficiency.  psg_tile_packed.hip is its form for many short
// pieces (rounds that pack several pushes).
//
// Reference semantics: KVVector::serialSetValue / parallelSetValue
// (src/parameter/kv_vector.h:84-204) over oldMatch / match
// (src/system/message.h:134-267): out[j] = fold over pushes p in arrival
// order of V_p[k] where S_p[k] == D[lo+j]; the first push assigns, later
// pushes add, and the serial path adds +0.0 for absent pushes: one "+0.0"
// after the fold, iff a push lacked the key, is bit-identical (see the
// stores).
//
// Shape:
//   * the partition (psg_partition.hip) has cut every push at every tile's
//     first server key, so push q's keys of this tile are
//     S_q[seg(q, t), seg(q, t+1)) (strides in the TileDesc);
//   * the pieces are split into "rounds" of 64 consecutive keys of ONE push,
//     numbered push-major; each wave takes a contiguous run of rounds, so a
//     round's push (pointers, bounds) is wave-uniform and every element load
//     is a coalesced 512 B (keys) / 256 B (f32 values) wave access;
//   * all of a wave's element loads are issued before the tile's bucket
//     table is built, so they overlap it;
//   * D goes to LDS; a bucket table (1 bucket per slot, the tile's key range
//     scaled by one high multiply; a plan's resident index, or built here by
//     histogram + scan) turns a search into one table read and one paired
//     key read;
//   * the fold runs wave by wave (4 barrier steps): rounds are push-major
//     and waves hold contiguous runs of them, so every slot sees its
//     contributions in arrival order with no atomics; sums and per-slot
//     contributor counts (serial mode) live in LDS;
//   * thread t owns slots 4t..4t+3: 16-B loads of D and 16-B stores;
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
#ifndef KCAP64
#define KCAP64 7
#endif

namespace psg {

#ifndef PSG_SKELETON
#define PSG_SKELETON 0  // diagnostic A/B builds (profiles/r03_ab_fold.txt): 1, 2 skip phases
#endif
#ifdef PSG_PHASES
// diagnostic build only (tools/phases.py): shader clocks between the phase
// marks of thread 0 of every workgroup, summed in registers and stored once
// per tile (one row per tile of the last launch)
constexpr int kPhTiles = 1 << 17;
__device__ uint32_t g_phase[kPhTiles][8];
#define PH(i) do { const unsigned long long _t = clock64(); \
    ph_acc[i] += (uint32_t)(_t - ph_t); ph_t = _t; } while (0)
#else
#define PH(i) do { } while (0)
#endif

namespace {

template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}
template <typename T>
__device__ __forceinline__ AS1 T* GW(T* p) {
  return (AS1 T*)p;
}

// Two forms, by pushes per group (one lane of wave 0 each):
//   32 pushes: 1024-slot tiles, 256 threads;
//   64 pushes (jobs of more than 32 pushes): 2048-slot tiles (kWideSlots),
//      512 threads -- each push's piece per tile doubles,
//      so its push-uniform rounds are fuller (cfg3: ~30 -> ~60 of 64 lanes).
constexpr int ts_of(int g) { return g == 64 ? kWideSlots : kTileSlots; }
constexpr int nt_of(int g) { return ts_of(g) / 4; }
// one bucket per slot in both forms: a plan's resident index is then 2 B per
// slot of HBM reads per run (2 per slot measured 2.5 % slower on cfg2,
// profiles/r03_ab_index.txt)
constexpr int nb_of(int g) { return ts_of(g); }
constexpr int cb_of(int g) { return ts_of(g) / 64 > 16 ? 5 : 4; }  // round-chunk bits
static_assert(ts_of(64) <= 0x7ffe, "u16 positions");

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

#ifndef PSG_FUSECNT
#define PSG_FUSECNT 1  // A/B builds: 0 = sums and contributor counts in separate arrays
#endif
#ifndef PSG_DDMA
#define PSG_DDMA 1  // A/B builds: 0 = D and the resident bucket table through registers
#endif
// 16 B per lane from global memory straight into LDS (gfx950 LDS-DMA): lane l
// writes lds + 16 l; nontemporal (D and the bucket table are read by one tile)
// Issued by inline asm (M0 saved and restored, as the compiler reserves it):
// the builtin form made the compiler's wait-count pass wait for the DMA at
// the next reuse of its address registers, i.e. right after issuing it.  The
// compiler does not see these loads, so readers of the LDS they fill wait
// for them explicitly (dma_wait); its own vmcnt waits stay correct, only
// more conservative (the DMAs are older than its loads).
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
__device__ __forceinline__ void dma_wait() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// a workgroup barrier that makes LDS writes visible but leaves vector-memory
// operations (LDS-DMA, loads) in flight: __syncthreads() would wait for them
// (its release fence waits vmcnt(0) while an LDS-DMA is pending)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0); vmcnt and expcnt not waited for
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// blocks b and b+8 share an XCD (observed dispatch, speed only): give each
// XCD a contiguous run of tiles
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + j;
}

// inclusive 64-lane prefix sum by DPP (row shifts, then row broadcasts):
// immediate lane controls, so no per-lane shuffle addresses stay live (the
// __shfl_up form kept six address VGPRs alive across the kernel and spilled
// them at 8 waves/SIMD)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}


// workgroups per CU the LDS allows (8 for the f32, m = 1 headline case):
// the register budget follows it through __launch_bounds__
template <typename V, int M, int kGroup>
constexpr int occupancy() {
  constexpr int ts = ts_of(kGroup), nw = nt_of(kGroup) / 64;
  constexpr int lds = (ts + 4) * 8 + (nb_of(kGroup) + 8) * 2 + M * (int)sizeof(V) * ts +
                      ts * (kGroup == 32 ? 4 : 2) + (kGroup + 1) * 4 + kGroup * 12 + kGroup * M * 8 +
                      nw * 8 + 8;
  // waves per SIMD (the launch bound's unit): workgroups per CU x waves / 4
  constexpr int w = (163840 / lds) * nw / 4;
#ifdef PSG_OCC64
  if (kGroup == 64) return PSG_OCC64;  // A/B builds: fewer waves, more registers per round
#endif
  return w >= 8 ? 8 : (w < 1 ? 1 : w);
}

template <typename V, int M, int kGroup>
__global__ __launch_bounds__(nt_of(kGroup), (occupancy<V, M, kGroup>())) void tile_kernel(
    const TileDesc* __restrict__ tiles, uint32_t ntiles) {
  constexpr int kTS = ts_of(kGroup);   // slots per tile
  constexpr int kNT = nt_of(kGroup);   // threads
  constexpr int kNW = kNT / 64;        // waves
  constexpr int kNB = nb_of(kGroup);   // buckets
  constexpr int kBPT = kNB / kNT;      // bucket-table entries per thread in the scan
  constexpr int kCB = cb_of(kGroup);   // bits of a round's chunk index
  static_assert(kTS / kNT == 4 && kBPT == 4, "layout");
  // rounds a wave holds per pass: 6 at 8 workgroups per CU (64 VGPRs); the
  // 64-push form runs 7 per CU and affords 8 (4 waves x 8 = 32 rounds: a
  // group of 64 one-round pieces in 2 passes)
  constexpr int kCap = kGroup == 64 ? KCAP64 : 6;
  __shared__ __attribute__((aligned(16))) uint64_t dk[kTS + 4];  // + sentinels ~0: the search window reads up to slot nt + 3
  // bucket starts (u16); the histogram counts in it as packed pairs by 32-bit atomics
  __shared__ __attribute__((aligned(16))) uint32_t bt32[(kNB + 8) / 2];
  uint16_t* const bt = (uint16_t*)bt32;
  // 1024-slot single-value f32 form: the sum and the contributor count of a
  // slot interleaved in one 8-B word (cnt32[2s], cnt32[2s + 1]), so the fold
  // updates both with one 8-B read and one 8-B write and the order check
  // issues no LDS atomic
  constexpr bool kFuse = PSG_FUSECNT && kGroup == 32 && M == 1 && sizeof(V) == 4;
  __shared__ __attribute__((aligned(16))) V acc[kFuse ? 1 : M][kFuse ? 1 : kTS];
  // serial mode: pushes holding the slot (u16 pairs, counted by non-returning
  // LDS adds during the search, off the fold's dependency chain): the fold
  // adds the "+0.0" of absent pushes as ONE trailing +0.0 when the count is
  // below np (see the stores)
  // 1024-slot form: one u32 per slot (the add is a constant 1); the
  // 2048-slot form keeps u16 pairs (LDS: 4 workgroups per CU)
  constexpr bool kCntW = kGroup == 32;
  __shared__ __attribute__((aligned(16))) uint32_t cnt32[kFuse ? 2 * kTS : kCntW ? kTS : kTS / 2];
#define ACC(mi, s) (*(kFuse ? (V*)&cnt32[2u * (s)] : &acc[mi][s]))
  __shared__ uint32_t rpre[kGroup + 1];             // rounds before push q of the group
  __shared__ uint32_t pln[kGroup];                  // piece length
  __shared__ uint64_t pkp[kGroup], pvp[kGroup * M];  // piece starts (keys, values)
  __shared__ int lastpos[kNW];
  __shared__ int pcarry;
  __shared__ uint32_t wsum[kNW];

  const uint32_t w = uni((uint32_t)threadIdx.x >> 6);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const uint32_t ti = xcd_tile(blockIdx.x, gridDim.x);
  if (ti >= ntiles) return;
#ifdef PSG_PHASES
  unsigned long long ph_t = clock64();
  uint32_t ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  const TileDesc& T = tiles[ti];
  const uint32_t np = T.np;
  const uint32_t nt = T.nt;
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  const uint64_t* Dg = T.dk;

  // ---- push tables of a group (wave 0, one lane per push), round prefix
  auto load_tables = [&](uint32_t g0) {
    if (w == 0) {
      // a fresh copy of the lane id per call: otherwise the compiler hoists
      // the lane-derived LDS addresses out of the push-group loop and, at
      // 64 VGPRs, spills them to scratch in every workgroup (HBM writes)
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      const uint32_t gp = np - g0 < (uint32_t)kGroup ? np - g0 : (uint32_t)kGroup;
      uint32_t nr = 0;
      if ((uint32_t)lane < gp) {
        const uint32_t q = g0 + (uint32_t)lane;
        const uint32_t* sg = T.seg + (size_t)q * T.stride;
        // every load of the table first (one round trip, not two)
        const uint32_t n = (uint32_t)G(T.pn)[q];
        uint32_t a = G(sg)[0], b = G(sg)[T.segb];
        const uint64_t* kp = G(T.pkeys)[q];
        const V* vp[M];
#pragma unroll
        for (int mi = 0; mi < M; ++mi) vp[mi] = (const V*)G(T.pvals)[(size_t)q * M + mi];
        // bounds from a failed partition (an unsorted push) stay inside the push
        a = a < n ? a : n;
        b = b < n ? b : n;
        // pieces out of order (the push is unsorted) or longer than the tile
        // (duplicates): those keys cannot all match
        const uint32_t over = b < a ? 1u : (b - a > (uint32_t)kTS ? b - a - (uint32_t)kTS : 0u);
        if (over)
          __hip_atomic_fetch_add(GW(T.fail) + q, (unsigned long long)over, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        // a piece lies inside one tile, so it holds at most kTS keys
        const uint32_t len = b > a ? (b - a < (uint32_t)kTS ? b - a : (uint32_t)kTS) : 0u;
        pln[lane] = len;
        pkp[lane] = (uint64_t)(kp + a);
#pragma unroll
        for (int mi = 0; mi < M; ++mi) pvp[lane * M + mi] = (uint64_t)(vp[mi] + a);
        nr = (len + 63u) >> 6;
      }
      const uint32_t x = wave_scan_incl(nr);
      if (lane < kGroup) rpre[lane + 1] = x;
      if (lane == 0) rpre[0] = 0;
    }
  };
  // ---- D keys, continued sums: thread t owns slots 4t..4t+3
  const uint32_t s0 = 4u * (uint32_t)tid;
  const uint32_t* Bg = T.bt;
  // full tiles: D (and a plan's resident bucket table) by LDS-DMA, issued
  // before the push tables are waited for and left in flight across barrier
  // (1) and the element loads, so D's HBM trip overlaps theirs (through
  // registers, D had to land before barrier (1), and the element loads went
  // out only after it: r05 phase clocks, profiles/r05_phases_cfg2.txt)
  const bool dma = PSG_DDMA && nt == (uint32_t)kTS && ((uintptr_t)Dg & 15u) == 0u &&
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
  if (dma && w != 0) issue_dma();
  if (np) load_tables(0);
  if (dma && w == 0) issue_dma();  // after wave 0's table loads: its wait for them does not wait for D
  // through registers (partial or unaligned tiles): loaded and installed
  // on this branch only, so no load of it is pending where the LDS-DMA
  // path rejoins (a pending one would make the compiler wait for all, D's
  // LDS-DMA included, at the next reuse of its registers)
  if (!dma) {
    uint64_t d[4];
    if (s0 + 3u < nt && ((uintptr_t)Dg & 15u) == 0u) {
      // D is read by this tile only: nontemporal (same-box A/B: ~1-3 % faster
      // on cfg2/cfg3 with the nontemporal sum stores; not the element loads,
      // whose lines neighbouring tiles share)
      const u64x2 x0 = __builtin_nontemporal_load((const AS1 u64x2*)(Dg + s0));
      const u64x2 x1 = __builtin_nontemporal_load((const AS1 u64x2*)(Dg + s0 + 2));
      d[0] = x0.x; d[1] = x0.y; d[2] = x1.x; d[3] = x1.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = s0 + j < nt ? G(Dg)[s0 + j] : ~0ull;
    }
    // the resident bucket table (plans): kBPT u16 entries per thread
    u32x2 btw = {0u, 0u};
    if (Bg) btw = __builtin_nontemporal_load((const AS1 u32x2*)Bg + tid);
#pragma unroll
    for (int j = 0; j < 4; ++j) dk[s0 + j] = d[j];
    if (Bg) {
      bt32[tid * (kBPT / 2)] = btw.x;
      bt32[tid * (kBPT / 2) + 1] = btw.y;
    }
    // drained here, explicitly: the compiler's merge of this branch's wait
    // state into the LDS-DMA path otherwise left a vmcnt(0) on that path
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  }
  // ---- sums, counts; clear the histogram.  The continued sums only on
  // their own (uniform) branch, for the same reason
  if (cont) {
    V a0[M][4];
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        a0[mi][j] = s0 + j < nt ? G((const V*)T.out[mi] + T.slot0)[s0 + j] : V(0);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0), on this branch only (see above)
    if constexpr (kFuse) {
      *(u32x4*)&cnt32[8 * tid] = u32x4{__float_as_uint(a0[0][0]), 0u, __float_as_uint(a0[0][1]), 0u};
      *(u32x4*)&cnt32[8 * tid + 4] = u32x4{__float_as_uint(a0[0][2]), 0u, __float_as_uint(a0[0][3]), 0u};
    } else {
#pragma unroll
      for (int mi = 0; mi < M; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[mi][s0 + j] = a0[mi][j];
    }
  } else if constexpr (kFuse) {
    *(u32x4*)&cnt32[8 * tid] = u32x4{0u, 0u, 0u, 0u};
    *(u32x4*)&cnt32[8 * tid + 4] = u32x4{0u, 0u, 0u, 0u};
  } else {
#pragma unroll
    for (int mi = 0; mi < M; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mi][s0 + j] = V(0);
  }
  if constexpr (kFuse) {
  } else if constexpr (kCntW) {
    *(u32x4*)&cnt32[4 * tid] = u32x4{0u, 0u, 0u, 0u};
  } else {
    cnt32[2 * tid] = 0u;
    cnt32[2 * tid + 1] = 0u;
  }
  if (tid < 4) dk[kTS + tid] = ~0ull;
  if (Bg) {  // resident table: installed above or by the LDS-DMA
    if (tid == 0) bt[kNB] = (uint16_t)nt;  // past its kNB entries
  } else {
    uint32_t z = 0;  // zero
#pragma unroll
    for (int i = 0; i < kBPT / 2; ++i) bt32[tid * (kBPT / 2) + i] = z;
  }
  if (tid == 0) pcarry = -1;
  if (dma)
    lds_barrier();  // (1) tables, sums, counts (D and the bucket table still in flight)
  else
    __syncthreads();  // (1) tables, D, cleared histogram (or the resident bucket table)
  PH(0);

  // ---- a pass: this wave's run of rounds, loaded into registers
  uint32_t done = 0, U = np ? uni(rpre[np < (uint32_t)kGroup ? np : kGroup]) : 0u;
  uint32_t g0 = 0;
  uint32_t nrw = 0, ua = 0, Rw = 0;
  uint32_t re[kCap];  // round: q << kCB | chunk (the same in every lane)
  uint64_t ek[kCap];
  V ev[kCap][M];
  // per lane, bit r of round r (VGPR bit words, not SGPR lane masks; one
  // word each keeps the shifted bits inline constants): the element exists,
  // it was found, it was found and in order
  uint32_t hv = 0, fd = 0, okb = 0;
  auto load_pass = [&]() {
    const uint32_t rem = U - done;
    Rw = (rem + kNW - 1) / kNW;
    Rw = Rw < (uint32_t)kCap ? Rw : (uint32_t)kCap;
    ua = done + w * Rw;
    const uint32_t ub = ua + Rw < U ? ua + Rw : U;
    nrw = ub > ua ? ub - ua : 0u;
    hv = 0;
    // the group's push table, one push per lane (lane q = push g0 + q), from
    // LDS in one round trip; a round's push is then a ballot over the lanes'
    // round ends and its bounds and pointers are lane reads: no dependent
    // LDS reads per round
    const uint32_t gp = np - g0 < (uint32_t)kGroup ? np - g0 : (uint32_t)kGroup;
    uint32_t t_len = 0, t_end = 0xffffffffu;
    uint64_t t_kp = 0, t_vp[M];
#pragma unroll
    for (int mi = 0; mi < M; ++mi) t_vp[mi] = 0;
    if ((uint32_t)lane < gp) {
      t_len = pln[lane];
      t_end = rpre[lane + 1];
      t_kp = pkp[lane];
#pragma unroll
      for (int mi = 0; mi < M; ++mi) t_vp[mi] = pvp[lane * M + mi];
    }
#pragma unroll
    for (int r = 0; r < kCap; ++r) {
      re[r] = 0;
      if ((uint32_t)r < nrw) {
        const uint32_t ru = ua + (uint32_t)r;
        const uint32_t q = (uint32_t)__popcll(__ballot(t_end <= ru));
        const uint32_t rs = q ? (uint32_t)__builtin_amdgcn_readlane((int)t_end, (int)q - 1) : 0u;
        const uint32_t c = ru - rs;
        re[r] = q << kCB | c;
        const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)t_len, (int)q);
        const bool have = c * 64u + (uint32_t)lane < len;
        hv |= (uint32_t)have << r;
        const uint64_t kp = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)t_kp, (int)q) |
                            (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(t_kp >> 32), (int)q) << 32;
        if (have) ek[r] = G((const uint64_t*)kp + 64u * c)[lane];
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          const uint64_t vp =
              (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)t_vp[mi], (int)q) |
              (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(t_vp[mi] >> 32), (int)q) << 32;
          if (have) ev[r][mi] = G((const V*)vp + 64u * c)[lane];
        }
      }
    }
  };
  if (U) load_pass();
  if (dma) {  // (1b) D and the bucket table landed (with the element loads)
    dma_wait();
    __syncthreads();
  }
  PH(1);

  // bucket of a key: the tile's key range [klo, khi] scaled onto [0, kNB) by
  // one 32x32 high multiply; keys outside the range land in an end bucket
  // and are not found there
  // (from LDS: D is installed; a global read here would wait for every
  // load in flight, the LDS-DMA of D included)
  const uint64_t klo = uni64(dk[0]);
  const uint64_t khi = uni64(dk[nt - 1]);
  const uint64_t range = khi - klo;
  const int bits = range ? 64 - __builtin_clzll(range) : 0;
  const int s2 = bits > 32 ? bits - 32 : 0;
  const uint64_t r32 = range >> s2;  // < 2^32
  const uint32_t mul = dev::bucket_scale(r32, kNB);
  auto bucket = [&](uint64_t k) -> uint32_t {
    const uint64_t x = (k - klo) >> s2;
    // no branch: an out-of-range x saturates, and the clamp puts it in the
    // end bucket (umulhi(r32, mul) < kNB for every in-range x)
    const uint32_t xs = x > r32 ? 0xffffffffu : (uint32_t)x;
    const uint32_t b = __umulhi(xs, mul);
    return b < (uint32_t)(kNB - 1) ? b : (uint32_t)(kNB - 1);
  };


  // ---- bucket table: histogram, exclusive scan -> bt[b] = first slot of bucket b
  // (skipped when the plan's resident index supplied it).  D keys back from
  // LDS: the registers that held them are free during the pass's element
  // loads (8 waves/SIMD leave 64 VGPRs)
  if (!Bg) {
  const u64x2 y0 = *(const u64x2*)&dk[s0];
  const u64x2 y1 = *(const u64x2*)&dk[s0 + 2];
  const uint64_t dd[4] = {y0.x, y0.y, y1.x, y1.y};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (s0 + j < nt)
    {  // counts <= kTS < 2^16: no carry between the packed halves
      const uint32_t b = bucket(dd[j]);
      __hip_atomic_fetch_add(&bt32[b >> 1], 1u << (16 * (b & 1u)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  __syncthreads();  // (2)
  {
    uint32_t e[kBPT];
#pragma unroll
    for (int i = 0; i < kBPT / 2; ++i) {
      const uint32_t h = bt32[tid * (kBPT / 2) + i];
      e[2 * i] = h & 0xffffu;
      e[2 * i + 1] = h >> 16;
    }
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < kBPT; ++j) {
      const uint32_t c = e[j];
      e[j] = tot;
      tot += c;
    }
    const uint32_t x = wave_scan_incl(tot);
    if (lane == 63) wsum[w] = x;
    __syncthreads();  // (3)
    uint32_t off = x - tot;
#pragma unroll
    for (uint32_t v = 0; v < (uint32_t)kNW - 1u; ++v) off += v < w ? wsum[v] : 0u;
#pragma unroll
    for (int i = 0; i < kBPT / 2; ++i)
      bt32[tid * (kBPT / 2) + i] = (e[2 * i] + off) | (e[2 * i + 1] + off) << 16;
    if (tid == 0) bt[kNB] = (uint16_t)nt;
  }
  __syncthreads();  // (4)
  }
  PH(2);

  for (;;) {
    if (!U) {  // this group of pushes has no keys in the tile, or is done
      g0 += kGroup;
      if (g0 >= np) break;
      load_tables(g0);
      __syncthreads();
      U = uni(rpre[np - g0 < (uint32_t)kGroup ? np - g0 : kGroup]);
      done = 0;
      if (U) load_pass();
      continue;
    }
#if PSG_SKELETON == 1
    // diagnostic (A/B builds only): the loads and stores of the kernel, no
    // search and no fold -- the memory side's own time
    {
      V t = V(0);
#pragma unroll
      for (int r = 0; r < kCap; ++r)
        if ((uint32_t)r < nrw && ((hv >> r) & 1u)) t += ev[r][0] + (V)(uint32_t)(ek[r] & 1u);
      ACC(0, s0) += t;
      done += kNW * Rw;
      if (done < U) {
        load_pass();
        continue;
      }
      U = 0;
      continue;
    }
#endif
    // ---- search every held round: one bucket-table read, then a window of
    // the 4 server keys from the bucket start, compared without branches.
    // The bucket map is monotone, so every key past the bucket is > k (and
    // the sentinels ~0 past the tile are >= k): c = window keys below k is
    // the lower bound inside the bucket whenever the bucket holds <= 4 keys
    // or c < 4, and k is present iff a window key equals it at a position
    // inside the tile.  One bucket per slot (Poisson occupancy): c == 4 with
    // more keys left in the bucket is ~0.4 % of keys; those finish below.
    uint32_t pos[kCap];
    fd = 0;
    okb = 0;
    uint32_t deep = 0;  // bit r: this lane's key lies past its round's window
#pragma unroll
    for (int r = 0; r < kCap; ++r) {
      pos[r] = 0;
      if ((uint32_t)r < nrw) {
        const uint64_t k = ek[r];
        const uint32_t b = bucket(k);
        const uint32_t l = bt[b];
        const uint32_t n = (uint32_t)bt[b + 1] - l;
        const uint64_t* wk = dk + l;
        const uint64_t k0 = wk[0], k1 = wk[1], k2 = wk[2], k3 = wk[3];
        const uint32_t c = (uint32_t)(k0 < k) + (uint32_t)(k1 < k) + (uint32_t)(k2 < k) +
                           (uint32_t)(k3 < k);
        const uint32_t p = l + c;
        pos[r] = p;
        // equality as lane masks (4 compares + 3 scalar ors)
        const uint64_t eq = __ballot(k0 == k) | __ballot(k1 == k) | __ballot(k2 == k) |
                            __ballot(k3 == k);
        const bool hit = ((eq >> lane) & 1ull) && p < nt;
        fd |= (uint32_t)hit << r;
        deep |= (uint32_t)(c == 4u && n > 4u) << r;
      }
    }
    if (__ballot(deep != 0u)) {  // long buckets: bisect the rest of the bucket
#pragma unroll
      for (int r = 0; r < kCap; ++r) {
        if ((deep >> r) & 1u) {
          const uint64_t k = ek[r];
          const uint32_t b = bucket(k);
          uint32_t l = bt[b] + 4u;
          uint32_t n = (uint32_t)bt[b + 1] - l;
          while (n > 0u) {
            const uint32_t half = n >> 1;
            if (dk[l + half] < k) {
              l += half + 1u;
              n -= half + 1u;
            } else {
              n = half;
            }
          }
          pos[r] = l;
          fd |= (uint32_t)(l < nt && dk[l] == k) << r;
        }
      }
    }
    int mylast = 0;  // position held by lane 63 in this wave's last round
#pragma unroll
    for (int r = 0; r < kCap; ++r)
      if ((uint32_t)r + 1u == nrw) mylast = (int)pos[r];
    if (nrw && lane == 63) lastpos[w] = mylast;
    __syncthreads();  // (5) lastpos of every wave
    PH(3);
#if PSG_SKELETON == 2
    // diagnostic: loads, stores and the search, no order check and no fold
    {
      V t = V(0);
#pragma unroll
      for (int r = 0; r < kCap; ++r)
        if ((uint32_t)r < nrw && ((fd >> r) & 1u)) t += ev[r][0] + (V)pos[r];
      ACC(0, s0) += t;
      done += kNW * Rw;
      if (done < U) {
        load_pass();
        continue;
      }
      U = 0;
      continue;
    }
#endif

    // ---- order check
#pragma unroll
    for (int r = 0; r < kCap; ++r) {
      if ((uint32_t)r < nrw) {
        int prev0;
        if ((re[r] & ((1u << kCB) - 1u)) == 0u) prev0 = -1;  // first round of the piece
        else if (r > 0) prev0 = __builtin_amdgcn_readlane((int)pos[r - 1], 63);
        else prev0 = w > 0 ? lastpos[w - 1] : pcarry;
        const int prev = __builtin_amdgcn_update_dpp(prev0, (int)pos[r], 0x138, 0xf, 0xf, false);
#if PSG_SKELETON == 4
        const bool ok = ((hv & fd) >> r & 1u) && prev != 0x7fffffff;  // diagnostic: no order test
#else
        const bool ok = ((hv & fd) >> r & 1u) && (int)pos[r] > prev;
#endif
        okb |= (uint32_t)ok << r;
        if (!kFuse && !parallel && ok)
          __hip_atomic_fetch_add(kCntW ? &cnt32[pos[r]] : &cnt32[pos[r] >> 1],
                                 kCntW ? 1u : 1u << (16u * (pos[r] & 1u)),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    // elements that exist but did not match: one ballot per pass, counts per
    // round only when there are any
    if (__ballot((hv & ~okb) != 0u)) {
#pragma unroll
      for (int r = 0; r < kCap; ++r) {
        const uint64_t bad = __ballot(((hv & ~okb) >> r & 1u) != 0u);
        if ((uint32_t)r < nrw && bad && lane == 0)
          __hip_atomic_fetch_add(GW(T.fail) + g0 + (re[r] >> kCB),
                                 (unsigned long long)__popcll(bad), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
    }

    // ---- fold, wave by wave (rounds are push-major)
    const uint32_t inpass = (U - done) < kNW * Rw ? U - done : kNW * Rw;
    const uint32_t wl = (inpass - 1) / Rw;  // wave holding the pass's last round
#if PSG_SKELETON == 3
    // diagnostic: every wave folds at once (racy: wrong sums on shared slots),
    // the cost of the wave-ordered fold's serialisation
    for (uint32_t st = 0; st < 1u; ++st) {
      {
#else
    for (uint32_t st = 0; st < (uint32_t)kNW; ++st) {
      if (st == w) {
#endif
#pragma unroll
        for (int r = 0; r < kCap; ++r) {
          if ((uint32_t)r < nrw && ((okb >> r) & 1u)) {
            const uint32_t q = re[r] >> kCB;
            const uint32_t s = pos[r];
            const bool first = g0 + q == 0u && !cont;
            if constexpr (kFuse) {
              u32x2* const p = (u32x2*)&cnt32[2u * s];
              const u32x2 x = *p;
              const V sum = first ? ev[r][0] : __uint_as_float(x.x) + ev[r][0];
              *p = u32x2{__float_as_uint(sum), x.y + 1u};
            } else {
#pragma unroll
              for (int mi = 0; mi < M; ++mi) acc[mi][s] = first ? ev[r][mi] : acc[mi][s] + ev[r][mi];
            }
          }
        }
        if (w == wl && lane == 63) pcarry = mylast;
      }
      __syncthreads();
    }
    PH(4);

    // ---- next pass, or next group of pushes
    done += kNW * Rw;
    if (done < U) {
      load_pass();
      continue;
    }
    U = 0;  // group finished
    if (tid == 0) pcarry = -1;
  }

  PH(5);
  // ---- the "+0.0" of absent pushes (serial), stores.  The reference adds
  // +0.0 for every push lacking the key (kv_vector.h:200); adding +0.0 is
  // the identity except on -0.0 (-> +0.0) and a signalling NaN (quieted),
  // and once either happened later adds keep the result, so the fold over
  // the present values followed by ONE +0.0 iff some push lacked the key is
  // bit-identical to the reference's dense fold
  V res[M][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t ncontrib = kFuse   ? cnt32[2u * (s0 + j) + 1u]
                              : kCntW ? cnt32[s0 + j]
                                      : (uint32_t)((const uint16_t*)cnt32)[s0 + j];
    const bool gap = !parallel && ncontrib != np;
#pragma unroll
    for (int mi = 0; mi < M; ++mi) {
      const V a = ACC(mi, s0 + j);
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
  PH(6);
#ifdef PSG_PHASES
  if (tid == 0 && ti < (uint32_t)kPhTiles)
    for (int i = 0; i < 8; ++i) g_phase[ti][i] = ph_acc[i];
#endif
}

// The bucket table of every tile, from D alone (a plan's resident index,
// built once at plan creation: the plan contract fixes D for its
// lifetime).  Exactly the tile kernel's histogram + scan with the same
// bucket map, written out as the kNB u16 bucket starts of each tile.
template <int kTSl>
__global__ __launch_bounds__(kTSl / 4) void bucket_index_kernel(
    const TileDesc* __restrict__ tiles, uint32_t ntiles, uint32_t* __restrict__ out) {
  constexpr int kNT = kTSl / 4;
  constexpr int kNW = kNT / 64;
  constexpr int kNB = kTSl;  // one bucket per slot (every kernel's map)
  constexpr int kBPT = kNB / kNT;
  __shared__ __attribute__((aligned(16))) uint32_t bt32[(kNB + 8) / 2];
  __shared__ uint32_t wsum[kNW];
  const uint32_t ti = blockIdx.x;
  if (ti >= ntiles) return;
  const TileDesc& T = tiles[ti];
  const uint32_t nt = T.nt;
  const uint64_t* Dg = T.dk;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = uni((uint32_t)tid >> 6);
  const uint32_t s0 = 4u * (uint32_t)tid;
  const uint64_t klo = G(Dg)[0];
  const uint64_t khi = G(Dg)[nt - 1];
  const uint64_t range = khi - klo;
  const int bits = range ? 64 - __builtin_clzll(range) : 0;
  const int s2 = bits > 32 ? bits - 32 : 0;
  const uint64_t r32 = range >> s2;
  const uint32_t mul = dev::bucket_scale(r32, kNB);
#pragma unroll
  for (int i = 0; i < kBPT / 2; ++i) bt32[tid * (kBPT / 2) + i] = 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (s0 + j < nt) {
      const uint64_t x = (G(Dg)[s0 + j] - klo) >> s2;
      const uint32_t b = x > r32 ? (uint32_t)(kNB - 1) : __umulhi((uint32_t)x, mul);
      __hip_atomic_fetch_add(&bt32[b >> 1], 1u << (16 * (b & 1u)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  __syncthreads();
  uint32_t e[kBPT];
#pragma unroll
  for (int i = 0; i < kBPT / 2; ++i) {
    const uint32_t h = bt32[tid * (kBPT / 2) + i];
    e[2 * i] = h & 0xffffu;
    e[2 * i + 1] = h >> 16;
  }
  uint32_t tot = 0;
#pragma unroll
  for (int j = 0; j < kBPT; ++j) {
    const uint32_t c = e[j];
    e[j] = tot;
    tot += c;
  }
  const uint32_t x = wave_scan_incl(tot);
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t off = x - tot;
#pragma unroll
  for (uint32_t v = 0; v < (uint32_t)kNW - 1u; ++v) off += v < w ? wsum[v] : 0u;
  uint32_t* o = out + (size_t)ti * (kNB / 2);
#pragma unroll
  for (int i = 0; i < kBPT / 2; ++i)
    o[tid * (kBPT / 2) + i] = (e[2 * i] + off) | (e[2 * i + 1] + off) << 16;
}

#ifndef PSG_PAD_LDS
#define PSG_PAD_LDS 0  // diagnostic A/B builds only: dynamic LDS per workgroup that
                       // lowers the workgroups per CU at unchanged code
#endif
template <typename V, int M>
hipError_t go(const TileDesc* t, uint32_t n, int form, hipStream_t s) {
  if (form == 1)
    hipLaunchKernelGGL((tile_kernel<V, M, 64>), dim3(n), dim3(nt_of(64)), PSG_PAD_LDS, s, t, n);
  else
    hipLaunchKernelGGL((tile_kernel<V, M, 32>), dim3(n), dim3(nt_of(32)), PSG_PAD_LDS, s, t, n);
  return hipGetLastError();
}

template <typename V>
hipError_t launch_m(int m, const TileDesc* t, uint32_t n, int form, hipStream_t s) {
  switch (m) {
    case 1: return go<V, 1>(t, n, form, s);
    case 2: return go<V, 2>(t, n, form, s);
    case 3: return go<V, 3>(t, n, form, s);
    case 4: return go<V, 4>(t, n, form, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

#ifdef PSG_PHASES
// out: ntiles x 8 u32 rows of the last launch
extern "C" int psg_debug_phases(uint32_t* out, uint32_t ntiles) {
  if (ntiles > (uint32_t)kPhTiles) ntiles = kPhTiles;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), (size_t)ntiles * 32) == hipSuccess ? 0 : -1;
}
#endif

uint32_t bucket_index_words(uint32_t tile_slots) { return tile_slots / 2u; }

hipError_t launch_bucket_index(const TileDesc* d_tiles, uint32_t ntiles, uint32_t tile_slots,
                               uint32_t* out, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  switch (tile_slots) {
    case 1024:
      hipLaunchKernelGGL(bucket_index_kernel<1024>, dim3(ntiles), dim3(256), 0, stream, d_tiles,
                         ntiles, out);
      break;
    case 2048:
      hipLaunchKernelGGL(bucket_index_kernel<2048>, dim3(ntiles), dim3(512), 0, stream, d_tiles,
                         ntiles, out);
      break;
    case 4096:
      hipLaunchKernelGGL(bucket_index_kernel<4096>, dim3(ntiles), dim3(1024), 0, stream, d_tiles,
                         ntiles, out);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_aggregate_tile(int dtype, int m, const TileDesc* d_tiles, uint32_t ntiles,
                                 int form, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  return dtype == 0 ? launch_m<float>(m, d_tiles, ntiles, form, stream)
                    : launch_m<double>(m, d_tiles, ntiles, form, stream);
}

}  // namespace psg
