// psg_tile_staged.hip -- the staged form of the long-piece aggregate kernel
// (psg_tile.hip): persistent workgroups, each walking an XCD-contiguous run
// of tiles, with every byte a tile reads (its D keys, its resident bucket
// index and the push pieces) moved into LDS by LDS-DMA one tile AHEAD of the
// search and fold.  The tile kernel loads a tile, then computes it, and a
// workgroup in its search/fold phases has no HBM load in flight (r05 phase
// clocks: 53 % of a tile); here tile t+1's DMA is in flight for the whole of
// tile t's search, order check and fold, and tile t-1's sums are stored then
// too, so the memory side never waits on the compute side.
//
// Reference semantics (identical to psg_tile.hip, bit for bit):
// KVVector::serialSetValue / parallelSetValue (src/parameter/kv_vector.h:84-204)
// over oldMatch / match (src/system/message.h:134-267): out[j] = fold over
// pushes p in arrival order of V_p[k] where S_p[k] == D[lo+j]; the first push
// assigns, later pushes add; serial mode: one trailing "+0.0" iff a push
// lacked the key.
//
// Shape:
//   * 256 threads, 2 workgroups per CU (LDS: two 32 KB stages + two 8 KB
//     sum/count buffers); grid = 2 x CUs, workgroup L takes tiles
//     [L*n/G, (L+1)*n/G) with L XCD-major, so an XCD walks one contiguous run;
//   * a stage is [D: 516 units][bucket index: 129 units][pieces] in 16-B
//     units; the pieces (every push's keys, then every push's values, each a
//     16-B aligned superset of the piece) are packed back to back, and one
//     DMA instruction moves 64 consecutive units, each lane finding its
//     piece by a uniform walk over the (<= 3) piece starts inside its 64;
//   * the descriptor pipeline runs three tiles ahead: tile t+3's descriptor,
//     t+2's seg bounds and push pointers, t+1's piece table (the DMA plan)
//     -- all loaded while tile t computes, all landed by the top-of-tile wait;
//   * search, order check and the wave-ordered fold are psg_tile.hip's,
//     reading keys and values from the stage (conflict-free consecutive
//     reads) instead of registers;
//   * a tile whose pieces exceed the stage (adversarial shapes only; cfg2's
//     tiles use ~60 % of it) reads its pieces from global memory instead:
//     same code, slower, bit-identical.
// The host picks this form for plans/flushes of <= 31 pushes per job, one
// f32 value array and no continued aggregates (psg_runtime.hip); everything
// else runs psg_tile.hip.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "psg_device.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))

namespace psg {

#ifndef PSG_STAGED_SKELETON
#define PSG_STAGED_SKELETON 0  // diagnostic A/B builds: 1 = DMA + stores only, no search/fold
#endif

namespace {

constexpr int kTS = kTileSlots;  // 1024 slots per tile
constexpr int kNT = 256;         // threads
constexpr int kNW = kNT / 64;    // waves
constexpr int kNB = kTS;         // buckets (one per slot, as every tile kernel)
constexpr int kDU = 516;         // D region: 513 units (an 8-B offset) + 4 sentinel keys
constexpr int kBU = 129;         // bucket index region: kNB u16 + bt[kNB]
constexpr int kPU0 = kDU + kBU;  // first piece unit
#ifndef PSG_STAGE_UNITS
#define PSG_STAGE_UNITS 2000
#endif
constexpr int kStageU = PSG_STAGE_UNITS;  // 16-B units per stage (2 stages + sums: 2 workgroups/CU)
constexpr int kPC = kStageU - kPU0;       // piece capacity, units
constexpr int kCap = 12;                  // rounds a wave holds per pass
constexpr int kMaxNp = 31;                // pushes per job (2 x np piece segments + lanes)
static_assert(kTS / kNT == 4, "thread t owns slots 4t..4t+3");
static_assert(2 * kStageU * 16 + 2 * 2 * kTS * 4 + 256 <= 81920, "two workgroups per CU");

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}
template <typename T>
__device__ __forceinline__ AS1 T* GW(T* p) {
  return (AS1 T*)p;
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
  return (uint64_t)rl((uint32_t)v, l) | (uint64_t)rl((uint32_t)(v >> 32), l) << 32;
}

// inclusive 64-lane prefix sum by DPP (psg_tile.hip's)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// 16 B per lane from global memory into LDS (gfx950 LDS-DMA): lane l writes
// lds + 16 l.  Inline asm (M0 saved and restored), as in psg_tile.hip: the
// compiler does not see these loads, so every reader waits for them
// explicitly (a full vmcnt wait and a barrier at the top of each tile).
typedef __attribute__((address_space(3))) void* LdsPtr;
__device__ __forceinline__ void dma16(const void* g, const void* lds) {
  const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LdsPtr)lds);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(la)
      : "memory");
}
__device__ __forceinline__ void dma16_nt(const void* g, const void* lds) {
  const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LdsPtr)lds);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(la)
      : "memory");
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// a workgroup barrier that leaves vector-memory operations (the next tile's
// LDS-DMA, the previous tile's stores) in flight: __syncthreads() would wait
// for them (psg_tile.hip)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0); vmcnt and expcnt not waited for
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// TileDesc as 26 dwords, one per lane (a descriptor costs one VGPR per stage
// of the pipeline); fields by readlane
static_assert(sizeof(TileDesc) == 104, "TileDesc layout");
constexpr uint32_t kDescW = sizeof(TileDesc) / 4;
#define DF32(d, f) rl((d), (uint32_t)(offsetof(TileDesc, f) / 4))
#define DF64(d, f) (rl((d), (uint32_t)(offsetof(TileDesc, f) / 4)) | \
                    (uint64_t)rl((d), (uint32_t)(offsetof(TileDesc, f) / 4) + 1u) << 32)

// A tile's push table, one push per lane (lane q < np), as loaded: seg
// bounds, push pointers, lengths; plus the job's first output pointer.
struct Raw {
  uint32_t a, b;
  uint64_t n, kp, vp, out0;
};
// A tile's plan: per lane q < np the piece (first key / value address,
// length) and the prefixes that place it in a stage; per tile the scalars
// the DMA, compute and store steps need.  The pieces are staged in groups of
// consecutive pushes whose units fit the stage: one group for every tile of
// the bench shapes (cfg2 uses ~60 % of a stage); a tile of more piece bytes
// stages its later groups itself, synchronously (rare, slower, same result).
struct Plan {
  uint64_t ks, vs;    // per lane: global addresses of the piece's first key / value
  uint32_t len;       // per lane: piece length
  uint32_t kx, vx;    // per lane: exclusive prefixes of key units / value units (totals past np)
  uint32_t ci;        // per lane: inclusive prefix of key + value units
  uint32_t rend;      // per lane: inclusive prefix of rounds (~0 past np)
  uint64_t dg, bg;    // D of the tile, its resident bucket index (0: built here)
  float* out;         // the tile's first output slot
  uint32_t nt, np, par;  // slots, pushes, parallel match
  uint32_t nr;        // rounds
};
// One group's placement in the stage: pushes [q0, q1), per lane q in it the
// first unit (from the piece base) of its keys and of its values.
struct Layout {
  uint32_t q0, q1, npu;
  uint32_t pk, pv;
};

__device__ __forceinline__ uint32_t load_desc(const TileDesc* tiles, uint32_t t, uint32_t t_end,
                                              int lane) {
  return (t < t_end && lane < (int)kDescW) ? G((const uint32_t*)(tiles + t))[lane] : 0u;
}

__device__ __forceinline__ Raw load_raw(uint32_t d, bool valid, int lane) {
  Raw r{0u, 0u, 0ull, 0ull, 0ull, 0ull};
  if (!valid) return r;
  const uint32_t np = DF32(d, np);
  const uint32_t stride = DF32(d, stride), segb = DF32(d, segb);
  const uint32_t* seg = (const uint32_t*)DF64(d, seg);
  const uint64_t* const* pk = (const uint64_t* const*)DF64(d, pkeys);
  const void* const* pv = (const void* const*)DF64(d, pvals);
  const uint64_t* pn = (const uint64_t*)DF64(d, pn);
  void* const* out = (void* const*)DF64(d, out);
  r.out0 = (uint64_t)G(out)[0];
  if ((uint32_t)lane < np) {
    const uint32_t q = (uint32_t)lane;
    r.a = G(seg)[(size_t)q * stride];
    r.b = G(seg)[(size_t)q * stride + segb];
    r.n = G(pn)[q];
    r.kp = (uint64_t)G(pk)[q];
    r.vp = (uint64_t)G(pv)[q];
  }
  return r;
}

// The plan of a tile from its descriptor and push table.  `count`: this wave
// reports the pieces that cannot all match (wave 0 only, once per tile).
__device__ __forceinline__ Plan make_plan(uint32_t d, const Raw& r, bool valid, int lane,
                                          bool count) {
  Plan p;
  p.ks = p.vs = 0;
  p.len = p.kx = p.vx = p.ci = 0;
  p.rend = 0xffffffffu;
  p.dg = p.bg = 0;
  p.out = nullptr;
  p.nt = p.np = p.par = p.nr = 0;
  if (!valid) return p;
  p.nt = DF32(d, nt);
  p.np = DF32(d, np);
  p.par = (DF32(d, flags) & kFlagParallel) ? 1u : 0u;
  p.dg = DF64(d, dk);
  p.bg = DF64(d, bt);
  p.out = (float*)rl64(r.out0, 0) + DF64(d, slot0);
  uint32_t ku = 0, vu = 0, nr = 0;
  if ((uint32_t)lane < p.np) {
    const uint32_t n = r.n < 0xffffffffull ? (uint32_t)r.n : 0xffffffffu;
    // bounds from a failed partition (an unsorted push) stay inside the push
    const uint32_t a = r.a < n ? r.a : n, b = r.b < n ? r.b : n;
    // pieces out of order (an unsorted push) or longer than the tile
    // (duplicates): those keys cannot all match (psg_tile.hip load_tables)
    const uint32_t over = b < a ? 1u : (b - a > (uint32_t)kTS ? b - a - (uint32_t)kTS : 0u);
    if (count && over)
      __hip_atomic_fetch_add(GW((unsigned long long*)DF64(d, fail)) + lane, (unsigned long long)over,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t len = b > a ? (b - a < (uint32_t)kTS ? b - a : (uint32_t)kTS) : 0u;
    p.len = len;
    p.ks = r.kp + 8ull * a;
    p.vs = r.vp + 4ull * a;
    if (len) {
      ku = (uint32_t)(((p.ks + 8ull * len + 15ull) >> 4) - (p.ks >> 4));
      vu = (uint32_t)(((p.vs + 4ull * len + 15ull) >> 4) - (p.vs >> 4));
    }
    nr = (len + 63u) >> 6;
  }
  const uint32_t ki = wave_scan_incl(ku), vi = wave_scan_incl(vu), ri = wave_scan_incl(nr);
  p.kx = ki - ku;
  p.vx = vi - vu;
  p.ci = ki + vi;
  p.nr = rl(ri, 63);
  p.rend = (uint32_t)lane < p.np ? ri : 0xffffffffu;
  return p;
}

// The group of pushes starting at q0: the longest run whose units fit the
// stage (a piece is at most 513 + 257 units, so every group holds a push)
__device__ __forceinline__ Layout layout(const Plan& p, uint32_t q0, int lane) {
  Layout g;
  g.q0 = q0;
  const uint32_t base = q0 ? rl(p.ci, q0 - 1u) : 0u;
  const bool in = (uint32_t)lane >= q0 && (uint32_t)lane < p.np && p.ci - base <= (uint32_t)kPC;
  g.q1 = q0 + (uint32_t)__popcll(__ballot(in));
  const uint32_t k0 = rl(p.kx, q0), v0 = rl(p.vx, q0);
  const uint32_t KU = rl(p.kx, g.q1) - k0, VU = rl(p.vx, g.q1) - v0;
  g.pk = p.kx - k0;
  g.pv = KU + p.vx - v0;
  g.npu = KU + VU;
  return g;
}

// This wave's share of the DMA of a group's pieces into stage S (and, with
// `head`, of the tile's D and bucket index first): instructions g = w, w+4,
// ... over [D units][index units][piece units], 64 units each.  D and the
// index are read by this tile only (nontemporal); the pieces' edge lines are
// shared with the neighbouring tiles of the run (default policy).
__device__ __forceinline__ void issue_dma(const Plan& p, const Layout& L, uint8_t* S, uint32_t w,
                                          int lane, bool head) {
  const uint64_t dga = p.dg & ~15ull;
  const uint32_t nud = head ? (uint32_t)(((p.dg + 8ull * p.nt + 15ull) >> 4) - (p.dg >> 4)) : 0u;
  const uint32_t iD = (nud + 63u) >> 6;
  const uint32_t iB = head && p.bg ? 2u : 0u;
  const uint32_t iP = (L.npu + 63u) >> 6;
  const uint32_t nI = iD + iB + iP, q0 = L.q0, nq = L.q1 - L.q0;
  for (uint32_t g = w; g < nI; g += kNW) {
    if (g < iD) {
      const uint32_t u = 64u * g + (uint32_t)lane;
      if (u < nud) dma16_nt((const void*)(dga + 16ull * u), S + 1024u * g);
    } else if (g < iD + iB) {
      const uint32_t j = g - iD;
      dma16_nt((const void*)(p.bg + 1024ull * j + 16ull * (uint32_t)lane), S + 16u * kDU + 1024u * j);
    } else {
      const uint32_t u0 = 64u * (g - iD - iB), u = u0 + (uint32_t)lane;
      // unit u's segment: the last of the 2 nq segments (keys of pushes
      // q0..q1-1, then their values) whose first unit is <= u; the walk
      // visits only the segment starts inside [u0, u0 + 64)
      const bool lv = (uint32_t)lane >= q0 && (uint32_t)lane < L.q1;
      const uint32_t c0 = (uint32_t)__popcll(__ballot(lv && L.pk <= u0)) +
                          (uint32_t)__popcll(__ballot(lv && L.pv <= u0));
      // unit address of segment k's first unit, minus that unit's index
      auto segbase = [&](uint32_t k) -> uint64_t {
        return k < nq ? (rl64(p.ks, q0 + k) >> 4) - rl(L.pk, q0 + k)
                      : (rl64(p.vs, q0 + k - nq) >> 4) - rl(L.pv, q0 + k - nq);
      };
      uint64_t gm = segbase(c0 - 1u);
      for (uint32_t k = c0; k < 2u * nq; ++k) {
        const uint32_t P = k < nq ? rl(L.pk, q0 + k) : rl(L.pv, q0 + k - nq);
        if (P > u0 + 63u) break;
        const uint64_t gk = segbase(k);
        if (u >= P) gm = gk;
      }
      if (u < L.npu) dma16((const void*)((gm + u) << 4), S + 16u * (kPU0 + u0));
    }
  }
}

// Tile sums out of sum/count buffer SB (thread t: slots 4t..4t+3), with the
// serial "+0.0" of absent pushes (psg_tile.hip, kv_vector.h:200); the
// buffer is cleared for the tile after next.
__device__ __forceinline__ void store_tile(uint32_t* SB, float* out, uint32_t nt, uint32_t np,
                                           uint32_t par, int tid) {
  const uint32_t s0 = 4u * (uint32_t)tid;
  const u32x4 x0 = *(const u32x4*)&SB[8 * tid];
  const u32x4 x1 = *(const u32x4*)&SB[8 * tid + 4];
  const float a[4] = {__uint_as_float(x0.x), __uint_as_float(x0.z), __uint_as_float(x1.x),
                      __uint_as_float(x1.z)};
  const uint32_t c[4] = {x0.y, x0.w, x1.y, x1.w};
  float res[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) res[j] = (!par && c[j] != np) ? a[j] + 0.0f : a[j];
  float* o = out + s0;
  if (s0 + 3u < nt && ((uintptr_t)o & 15u) == 0u) {
    const f32x4 v = {res[0], res[1], res[2], res[3]};
    __builtin_nontemporal_store(v, (AS1 f32x4*)GW(o));
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (s0 + (uint32_t)j < nt) GW(o)[j] = res[j];
  }
  *(u32x4*)&SB[8 * tid] = u32x4{0u, 0u, 0u, 0u};
  *(u32x4*)&SB[8 * tid + 4] = u32x4{0u, 0u, 0u, 0u};
}

__global__ __launch_bounds__(kNT, 2) void staged_kernel(const TileDesc* __restrict__ tiles,
                                                        uint32_t ntiles) {
  __shared__ __attribute__((aligned(16))) uint8_t stg[2][kStageU * 16];
  // per slot: the sum's bits and the contributor count (psg_tile.hip's fused
  // f32 form), two buffers: tile t folds into one while t-1's is stored
  __shared__ __attribute__((aligned(16))) uint32_t sums[2][2 * kTS];
  __shared__ int lastpos[kNW];
  __shared__ int pcarry;
  __shared__ uint32_t wsum[kNW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const uint32_t w = uni((uint32_t)tid >> 6);
  // workgroup L of G (G a multiple of 8; blocks b and b+8 share an XCD:
  // speed only): L XCD-major, tiles [L n / G, (L+1) n / G)
  const uint32_t nb = gridDim.x;
  const uint32_t L = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
  const uint32_t t_begin = (uint32_t)((uint64_t)L * ntiles / nb);
  const uint32_t t_end = (uint32_t)((uint64_t)(L + 1) * ntiles / nb);
  if (t_begin >= t_end) return;

  // ---- pipeline fill: descriptors of tiles 0..3 of the run, push tables of
  // 0..2, plans of 0 and 1, tile 0's DMA
  uint32_t d0 = load_desc(tiles, t_begin, t_end, lane);
  uint32_t d1 = load_desc(tiles, t_begin + 1, t_end, lane);
  uint32_t d2 = load_desc(tiles, t_begin + 2, t_end, lane);
  uint32_t d3 = load_desc(tiles, t_begin + 3, t_end, lane);
  Raw r2 = load_raw(d2, t_begin + 2 < t_end, lane);
  Plan p0, p1;
  {
    const Raw r0 = load_raw(d0, true, lane);
    const Raw r1 = load_raw(d1, t_begin + 1 < t_end, lane);
    p0 = make_plan(d0, r0, true, lane, w == 0);
    p1 = make_plan(d1, r1, t_begin + 1 < t_end, lane, w == 0);
  }
  issue_dma(p0, layout(p0, 0u, lane), stg[0], w, lane, true);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    *(u32x4*)&sums[b][8 * tid] = u32x4{0u, 0u, 0u, 0u};
    *(u32x4*)&sums[b][8 * tid + 4] = u32x4{0u, 0u, 0u, 0u};
  }
  // the previous tile (stored one tile late)
  float* pm_out = nullptr;
  uint32_t pm_nt = 0, pm_np = 0, pm_par = 0;

  for (uint32_t t = t_begin; t < t_end; ++t) {
    const uint32_t i = t - t_begin;
    uint8_t* const S = stg[i & 1u];
    uint32_t* const SU = sums[i & 1u];
    const uint32_t nt = p0.nt, np = p0.np;
    uint64_t* const dk = (uint64_t*)(S + (p0.dg & 15ull));
    uint32_t* const bt32 = (uint32_t*)(S + 16 * kDU);
    uint16_t* const bt = (uint16_t*)bt32;

    // ---- (A) tile t's stage has landed: every wave waits for its own DMA;
    // the wave that moved D's last unit overwrites what it brought past slot
    // nt - 1 with the window's sentinels
    dma_wait();
    {
      const uint32_t nud = (uint32_t)(((p0.dg + 8ull * nt + 15ull) >> 4) - (p0.dg >> 4));
      if (w == ((nud + 63u) / 64u - 1u) % (uint32_t)kNW && lane < 4) dk[nt + (uint32_t)lane] = ~0ull;
      if (p0.bg) {
        if (tid == 0) bt[kNB] = (uint16_t)nt;
      } else {
#pragma unroll
        for (int k = 0; k < kNB / 2 / kNT; ++k) bt32[tid * (kNB / 2 / kNT) + k] = 0u;
      }
      if (tid == 0) pcarry = -1;
    }
    __syncthreads();

    // ---- (B) tile t+1's DMA, t+2's plan, t+3's push table, t+4's descriptor
    issue_dma(p1, layout(p1, 0u, lane), stg[(i + 1u) & 1u], w, lane, true);
    const Raw r3 = load_raw(d3, t + 3 < t_end, lane);
    const uint32_t d4 = load_desc(tiles, t + 4, t_end, lane);
    const Plan p2 = make_plan(d2, r2, t + 2 < t_end, lane, w == 0);

    // ---- (C) tile t-1's sums out; its buffer is the one tile t+1 folds into
    if (i > 0) store_tile(sums[(i + 1u) & 1u], pm_out, pm_nt, pm_np, pm_par, tid);

    // ---- (D) tile t: bucket map of its key range (psg_tile.hip)
    const uint64_t klo = ((uint64_t)uni((uint32_t)(dk[0] >> 32)) << 32) | uni((uint32_t)dk[0]);
    const uint64_t khi = ((uint64_t)uni((uint32_t)(dk[nt - 1] >> 32)) << 32) | uni((uint32_t)dk[nt - 1]);
    const uint64_t range = khi - klo;
    const int bits = range ? 64 - __builtin_clzll(range) : 0;
    const int sh = bits > 32 ? bits - 32 : 0;
    const uint64_t r32 = range >> sh;
    const uint32_t mul = dev::bucket_scale(r32, kNB);
    auto bucket = [&](uint64_t k) -> uint32_t {
      const uint64_t x = (k - klo) >> sh;
      const uint32_t xs = x > r32 ? 0xffffffffu : (uint32_t)x;
      const uint32_t b = __umulhi(xs, mul);
      return b < (uint32_t)(kNB - 1) ? b : (uint32_t)(kNB - 1);
    };
    const uint32_t s0 = 4u * (uint32_t)tid;
    if (!p0.bg) {  // no resident index (context flushes): histogram + scan here
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (s0 + j < nt) {
          const uint32_t b = bucket(dk[s0 + j]);
          __hip_atomic_fetch_add(&bt32[b >> 1], 1u << (16 * (b & 1u)), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      lds_barrier();
      uint32_t e[4];
      {
        const uint32_t h0 = bt32[2 * tid], h1 = bt32[2 * tid + 1];
        e[0] = h0 & 0xffffu;
        e[1] = h0 >> 16;
        e[2] = h1 & 0xffffu;
        e[3] = h1 >> 16;
      }
      uint32_t tot = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t c = e[j];
        e[j] = tot;
        tot += c;
      }
      const uint32_t x = wave_scan_incl(tot);
      if (lane == 63) wsum[w] = x;
      lds_barrier();
      uint32_t off = x - tot;
#pragma unroll
      for (uint32_t v = 0; v < (uint32_t)kNW - 1u; ++v) off += v < w ? wsum[v] : 0u;
      bt32[2 * tid] = (e[0] + off) | (e[1] + off) << 16;
      bt32[2 * tid + 1] = (e[2] + off) | (e[3] + off) << 16;
      if (tid == 0) bt[kNB] = (uint16_t)nt;
      lds_barrier();
    }

    // ---- (E) groups of pushes (one unless the pieces exceed the stage),
    // passes: this wave's run of rounds (64 consecutive keys of one push,
    // push-major), keys and values from the stage.  No compiler-visible
    // vector-memory load in here: a wait for one would also wait for tile
    // t+1's DMA.
    for (uint32_t q0 = 0;;) {
      const Layout Lg = layout(p0, q0, lane);
      if (q0 > 0) {  // a later group: its pieces into the stage now (rare)
        issue_dma(p0, Lg, S, w, lane, false);
        dma_wait();
        lds_barrier();
      }
      const uint32_t R0 = q0 ? rl(p0.rend, q0 - 1u) : 0u;
      const uint32_t R1 = Lg.q1 ? rl(p0.rend, Lg.q1 - 1u) : 0u;
      const uint32_t U = R1 - R0;
#if PSG_STAGED_SKELETON == 1
      {  // diagnostic: the stage is read (one key and value per lane per round), no search/fold
        float tsum = 0.f;
        for (uint32_t ru = R0 + w; ru < R1; ru += kNW) {
          const uint32_t q = (uint32_t)__popcll(__ballot(p0.rend <= ru));
          const uint32_t rs = q ? rl(p0.rend, q - 1u) : 0u;
          const uint32_t ii = 64u * (ru - rs) + (uint32_t)lane;
          if (ii < rl(p0.len, q)) {
            const uint32_t kb = 16u * (kPU0 + rl(Lg.pk, q)) + (rl((uint32_t)p0.ks, q) & 15u);
            const uint32_t vb = 16u * (kPU0 + rl(Lg.pv, q)) + (rl((uint32_t)p0.vs, q) & 15u);
            tsum += *(const float*)(S + vb + 4u * ii) +
                    (float)(uint32_t)(*(const uint64_t*)(S + kb + 8u * ii) & 1u);
          }
        }
        SU[2u * s0] = __float_as_uint(__uint_as_float(SU[2u * s0]) + tsum + (float)(uint32_t)dk[s0]);
        SU[2u * s0 + 1u] = np;
        lds_barrier();
      }
#else
      for (uint32_t done = 0; done < U;) {
        uint32_t Rw = (U - done + kNW - 1) / kNW;
        Rw = Rw < (uint32_t)kCap ? Rw : (uint32_t)kCap;
        const uint32_t ua = R0 + done + w * Rw;
        const uint32_t ub = ua + Rw < R1 ? ua + Rw : R1;
        const uint32_t nrw = ub > ua ? ub - ua : 0u;
        uint32_t re[kCap];
        uint64_t ek[kCap];
        float ev[kCap];
        uint32_t hv = 0;
#pragma unroll
        for (int r = 0; r < kCap; ++r) {
          re[r] = 0;
          ek[r] = 0;
          ev[r] = 0.f;
          if ((uint32_t)r < nrw) {
            const uint32_t ru = ua + (uint32_t)r;
            const uint32_t q = (uint32_t)__popcll(__ballot(p0.rend <= ru));
            const uint32_t rs = q ? rl(p0.rend, q - 1u) : 0u;
            const uint32_t c = ru - rs;
            re[r] = q << 5 | c;
            const uint32_t ii = 64u * c + (uint32_t)lane;
            const bool have = ii < rl(p0.len, q);
            hv |= (uint32_t)have << r;
            const uint32_t kb = 16u * (kPU0 + rl(Lg.pk, q)) + (rl((uint32_t)p0.ks, q) & 15u);
            const uint32_t vb = 16u * (kPU0 + rl(Lg.pv, q)) + (rl((uint32_t)p0.vs, q) & 15u);
            if (have) {
              ek[r] = *(const uint64_t*)(S + kb + 8u * ii);
              ev[r] = *(const float*)(S + vb + 4u * ii);
            }
          }
        }
        // search: psg_tile.hip's window over the 4 keys at the bucket start,
        // bisection past it for the rare long bucket
        uint32_t pos[kCap];
        uint32_t fd = 0, okb = 0, deep = 0;
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
            const uint64_t eq = __ballot(k0 == k) | __ballot(k1 == k) | __ballot(k2 == k) |
                                __ballot(k3 == k);
            const bool hit = ((eq >> lane) & 1ull) && p < nt;
            fd |= (uint32_t)hit << r;
            deep |= (uint32_t)(c == 4u && n > 4u) << r;
          }
        }
        if (__ballot(deep != 0u)) {
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
        int mylast = 0;
#pragma unroll
        for (int r = 0; r < kCap; ++r)
          if ((uint32_t)r + 1u == nrw) mylast = (int)pos[r];
        if (nrw && lane == 63) lastpos[w] = mylast;
        lds_barrier();  // lastpos of every wave

        // order check: matched positions strictly increase inside a piece
#pragma unroll
        for (int r = 0; r < kCap; ++r) {
          if ((uint32_t)r < nrw) {
            int prev0;
            if ((re[r] & 31u) == 0u) prev0 = -1;  // first round of the piece
            else if (r > 0) prev0 = __builtin_amdgcn_readlane((int)pos[r - 1], 63);
            else prev0 = w > 0 ? lastpos[w - 1] : pcarry;
            const int prev = __builtin_amdgcn_update_dpp(prev0, (int)pos[r], 0x138, 0xf, 0xf, false);
            const bool ok = ((hv & fd) >> r & 1u) && (int)pos[r] > prev;
            okb |= (uint32_t)ok << r;
          }
        }
        if (__ballot((hv & ~okb) != 0u)) {
          unsigned long long* const fail = (unsigned long long*)DF64(d0, fail);
#pragma unroll
          for (int r = 0; r < kCap; ++r) {
            const uint64_t bad = __ballot(((hv & ~okb) >> r & 1u) != 0u);
            if ((uint32_t)r < nrw && bad && lane == 0)
              __hip_atomic_fetch_add(GW(fail) + (re[r] >> 5), (unsigned long long)__popcll(bad),
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }

        // fold, wave by wave (rounds are push-major: arrival order per slot)
        const uint32_t inpass = (U - done) < kNW * Rw ? U - done : kNW * Rw;
        const uint32_t wl = (inpass - 1) / Rw;
        for (uint32_t st = 0; st < (uint32_t)kNW; ++st) {
          if (st == w) {
#pragma unroll
            for (int r = 0; r < kCap; ++r) {
              if ((uint32_t)r < nrw && ((okb >> r) & 1u)) {
                const uint32_t q = re[r] >> 5;
                u32x2* const sp = (u32x2*)&SU[2u * pos[r]];
                const u32x2 x = *sp;
                const float sum = q == 0u ? ev[r] : __uint_as_float(x.x) + ev[r];
                *sp = u32x2{__float_as_uint(sum), x.y + 1u};
              }
            }
            if (w == wl && lane == 63) pcarry = mylast;
          }
          lds_barrier();
        }
        done += kNW * Rw;
      }
#endif
      q0 = Lg.q1;
      if (q0 >= np) break;
    }
    lds_barrier();  // the stage and the sums are complete (and free)

    // ---- rotate the pipeline
    pm_out = p0.out;
    pm_nt = nt;
    pm_np = np;
    pm_par = p0.par;
    d0 = d1;
    d1 = d2;
    d2 = d3;
    d3 = d4;
    r2 = r3;
    p0 = p1;
    p1 = p2;
  }
  // the run's last tile
  store_tile(sums[(t_end - t_begin - 1u) & 1u], pm_out, pm_nt, pm_np, pm_par, tid);
}

}  // namespace

hipError_t launch_aggregate_staged(const TileDesc* d_tiles, uint32_t ntiles, hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  // two workgroups per CU (LDS), a multiple of 8 (the XCD-major run order)
  uint32_t grid = (uint32_t)(2 * ncu + 7) & ~7u;
  if (ntiles < grid) grid = (ntiles + 7u) & ~7u;
  hipLaunchKernelGGL(staged_kernel, dim3(grid), dim3(kNT), 0, stream, d_tiles, ntiles);
  return hipGetLastError();
}

bool staged_fits(uint32_t np, int dtype, int m) {
  return np <= (uint32_t)kMaxNp && dtype == 0 && m == 1;
}

}  // namespace psg
