// psg_snappy.hip -- snappy raw-format decompression of wire payloads on the
// device: SArray::uncompressFrom (src/base/shared_array_inl.h:232-240) as
// Van::recv applies it to every key/value part of a message
// (src/system/van.cc:204-214).  snappy itself is a third-party library the
// reference links (google/snappy; absent from the reference tree): its
// published raw format -- a varint length, then literal and copy elements
// (tag & 3: literal / copy with a 1-, 2- or 4-byte offset) -- is decoded
// here.
//
// One wave per message (grid-stride over messages).  The element stream is
// sequential, so every lane parses the same tag: the wave holds 64 bytes of
// lookahead in a register (filled from a 4 KB LDS window over the
// compressed stream, itself refilled with coalesced loads) and takes tag and
// offset bytes from it with readlane; the bytes of an element are moved by
// all 64 lanes.  The
// last 8 KB of output live in an LDS ring: a copy reads its source bytes
// there.  A copy's source is output[o - off + (l mod off)] for byte l, which
// lies before o for every l, so even overlapping (run-length) copies move in
// one step; copies are <= 64 bytes, so the step's reads precede its writes.
// Offsets beyond the ring read the output in global memory after a flush
// and a fence (slower per element, rare in the payloads here: sorted keys
// and float values match their recent neighbours).
//
// The parse is latency-bound per element, so the throughput is the number
// of parts in flight: the ring is 8 KB (r04: 64 KB, two parts per CU) and a
// part keeps up to 256 deferred pieces, ~15 KB of LDS per wave, ten parts
// per CU -- 2048 element-dense 64 KB parts decode 3.3x faster (28.5 ->
// 93 GB/s, profiles/r05_ab_snappy_ring.txt).
//
// Long literals (>= kBigLit bytes: what incompressible data becomes -- the
// cfg2 key and value parts are one 64 KB literal per snappy block) are not
// moved by the parsing wave: it records (source, destination, length) and
// skips them, and a second, chip-wide kernel copies every recorded piece
// 16 B per lane.  The part's deferred pieces are listed in LDS by output
// position; a copy element whose source lies wholly inside one of them is
// itself deferred as a piece of the compressed input (no bytes move in the
// parse), and one that straddles reads the deferred bytes from the input.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/psg.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))
#ifndef PSG_SNAPPY_IR
#define PSG_SNAPPY_IR 2  // few-part launches: 2 = the table form, 1 = the streamed form (A/B), 0 = snappy_kernel
#endif
#ifndef PSG_SNAPPY_PREFETCH
#define PSG_SNAPPY_PREFETCH 1  // A/B: 0 = no L2 prefetch of the parts
#endif

namespace psg {

namespace {

#ifdef PSG_SNAPPY_PROF
// diagnostic build only (tools/snappy_prof.py): per part, shader clocks in
// [0] window refills, [1] copies' piece lookups, [2] the whole part,
// [5] literals moved in the parse, [7] the part's end (flush, hand-off), and
// counts [3] refills, [4] deferred pieces, [6] elements
__device__ unsigned long long g_sprof[4096][8];
#define SP_T0() const unsigned long long _sp0 = clock64()
#define SP_ADD(i) (sp[i] += clock64() - _sp0)
#else
#define SP_T0() do { } while (0)
#define SP_ADD(i) do { } while (0)
#endif

#ifndef PSG_SNAPPY_RING
#define PSG_SNAPPY_RING 8192  // A/B builds: 16384, 65536 (r04's)
#endif
#ifndef PSG_SNAPPY_MAXDEF
#define PSG_SNAPPY_MAXDEF 256  // r04: 768
#endif
constexpr uint32_t kRing = PSG_SNAPPY_RING;
static_assert((kRing & (kRing - 1)) == 0 && kRing >= 4096, "ring: a power of two >= the window");
constexpr uint32_t kWin = 4096;

constexpr uint32_t kBigLit = 2048;   // literals deferred to the copy kernel
constexpr uint32_t kMaxDef = PSG_SNAPPY_MAXDEF;  // deferred pieces per part (LDS list)
constexpr uint32_t kLitUnits = 256;  // 16-B units per copy-kernel chunk (4 KB)
constexpr uint64_t kPrefetchParts = 64;         // parts per launch that are prefetched into L2
constexpr uint64_t kPrefetchMax = 2ull << 20;   // largest part prefetched

// This workgroup's earlier global stores visible to its own later loads (the
// decoders read back output they wrote): its waves share the CU's L1, so a
// workgroup-scope fence after the stores drain is enough.  __threadfence()
// (agent scope) would write back and invalidate the XCD's L2 -- ~3.5 us each
// (MI355X_MICROARCH.md), which r06 measured dominating the table form's
// in-order step.
__device__ __forceinline__ void own_stores_visible() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

__global__ __launch_bounds__(64) void snappy_kernel(const uint8_t* __restrict__ src,
                                                    const uint64_t* __restrict__ soff,
                                                    uint8_t* __restrict__ dst,
                                                    const uint64_t* __restrict__ doff,
                                                    const uint64_t* __restrict__ dcap,
                                                    uint64_t nmsg, int32_t* __restrict__ status,
                                                    SnappyLit* __restrict__ lits,
                                                    uint32_t* __restrict__ nlits,
                                                    uint32_t lit_cap,
                                                    unsigned long long* __restrict__ nbad,
                                                    int pairs, int prefetch) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
  __shared__ __attribute__((aligned(4))) uint8_t win[kWin];
  // deferred pieces of the current part, in output order: output start,
  // input start, length
  __shared__ uint32_t tdst[kMaxDef], tsrc[kMaxDef], tlen[kMaxDef];
  const uint32_t lane = threadIdx.x;
  for (uint64_t msg = blockIdx.x; msg < nmsg; msg += gridDim.x) {
    // pairs: soff holds (begin, end) device addresses per part
    // global (not flat) pointers: a flat load also counts on lgkmcnt, so every
    // LDS wait of the parse would wait for the loads in flight as well
    const AS1 uint8_t* const s0 =
        (const AS1 uint8_t*)(pairs ? (const uint8_t*)soff[2 * msg] : src + soff[msg]);
    const uint64_t slen = pairs ? soff[2 * msg + 1] - soff[2 * msg] : soff[msg + 1] - soff[msg];
    AS1 uint8_t* const out = (AS1 uint8_t*)(dst + doff[msg]);
    const uint64_t cap = dcap ? dcap[msg] : doff[msg + 1] - doff[msg];
    // an empty part is an empty array (uncompressFrom of 0 bytes clears, :233)
    if (slen == 0) {
      if (lane == 0) status[msg] = cap == 0 ? 0 : PSG_ERR_SIZE;
      continue;
    }
    if (slen >= (1ull << 31)) {  // a compressed part of 2 GB or more is refused
      if (lane == 0) status[msg] = PSG_ERR_ARG;
      continue;
    }
    // all positions are 32-bit offsets into the part (the parse is
    // instruction-bound at one wave per part; 64-bit pointer arithmetic
    // doubled it)
    const uint32_t e = (uint32_t)slen;
    int32_t st = 0;
    // A launch of few parts (a message's: the compressed-push path) pulls
    // each part into its XCD's L2 first -- one byte load per 128-B line, all
    // in flight at once -- so the walk's window refills, one after each
    // skipped literal and each a dependent round trip, hit L2 instead of
    // HBM.  Many parts at once would evict each other: no prefetch there.
    uint32_t pfx = 0;
    if (prefetch && slen <= kPrefetchMax)
      for (uint32_t x = lane * 128u; x < e; x += 64u * 128u) pfx ^= s0[x];
    // the element stream is read from an LDS window (4 KB, refilled with
    // coalesced 4-byte loads), and from it into a 64-byte register
    // lookahead (lane j holds byte lp + j) whose bytes the parse takes with
    // a scalar readlane: one LDS read serves several tags
    const uintptr_t mis = (uintptr_t)s0 & 3u;
    int32_t wb = -(int32_t)kWin - 64;  // part offset of win[0]; nothing loaded
    // an aligned in-range word for the refill's out-of-range lanes (parts
    // of at least 8 bytes; shorter ones are read byte by byte)
    const int64_t gs = (int64_t)((4u - (uint32_t)mis) & 3u);
#ifdef PSG_SNAPPY_PROF
    unsigned long long sp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long sp_part = clock64();
#endif
    auto refill = [&](uint32_t q) {
      SP_T0();
#ifdef PSG_SNAPPY_PROF
      sp[3] += 1;
#endif
      wb = (int32_t)((q + mis) & ~3u) - (int32_t)mis;  // 4-byte aligned in memory
      // all 16 loads in flight before the first LDS store (one HBM round
      // trip per refill, not 16: a refill follows every skipped literal)
      constexpr int kR = (int)(kWin / 256u);
      // The in-range words load from their address and the others from the
      // window's first in-range word (gs, the result dropped): no branch
      // around the loads, so all 16 issue back to back (a per-word branch
      // made the compiler wait after each, 16 round trips per refill).
      // Words that straddle the part's ends (at most two per refill) are
      // assembled byte by byte afterwards.
      uint32_t v[kR];
      bool edge = false;
      if (e >= 8u) {  // a part of fewer than 8 bytes may hold no aligned word: bytes only
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          const int64_t g = (int64_t)wb + lane * 4u + 256u * r;
          const bool inb = g >= 0 && g + 4 <= (int64_t)e;
          edge |= !inb;
          v[r] = *(const AS1 uint32_t*)(s0 + (inb ? g : gs));  // no select on the result
        }
      } else {
        edge = true;
#pragma unroll
        for (int r = 0; r < kR; ++r) v[r] = 0;
      }
      if (__ballot(edge)) {
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          const int64_t g = (int64_t)wb + lane * 4u + 256u * r;
          if (e < 8u || !(g >= 0 && g + 4 <= (int64_t)e)) {
            v[r] = 0;
            for (uint32_t b = 0; b < 4; ++b)
              if (g + b >= 0 && g + b < (int64_t)e) v[r] |= (uint32_t)s0[g + b] << (8 * b);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < kR; ++r) *(uint32_t*)&win[lane * 4u + 256u * r] = v[r];
      __builtin_amdgcn_wave_barrier();
#ifdef PSG_SNAPPY_PROF
      (void)__builtin_amdgcn_readfirstlane((int)win[lane]);  // wait for the window
#endif
      SP_ADD(0);
    };
    uint32_t lp = 0xffffffffu - 64u, la = 0;
    auto ub = [&](uint32_t q) -> uint32_t {
      if (q - lp >= 64u) {
        if ((uint32_t)((int32_t)q - wb) + 64u > kWin) refill(q);
        lp = q;
        la = win[(int32_t)q - wb + (int32_t)lane];
      }
      return (uint32_t)__builtin_amdgcn_readlane((int)la, (int)(q - lp));
    };
    // preamble: uncompressed length, little-endian varint
    uint64_t ulen = 0;
    bool done = false;
    uint32_t p = 0;
    while (p < 5 && p < e && !done) {
      const uint32_t b = ub(p);
      ulen |= (uint64_t)(b & 0x7f) << (7 * p);
      done = !(b & 0x80);
      ++p;
    }
    if (!done || ulen > 0xffffffffull) st = PSG_ERR_ARG;
    if (!st && ulen != cap) st = PSG_ERR_SIZE;
    const uint32_t ucap = (uint32_t)ulen;
    uint32_t o = 0;
    // this part's deferred pieces (LDS list); [dlo, dhi) spans them all
    uint32_t nd = 0, dlo = 0xffffffffu, dhi = 0;
    // Output bytes below fl are in memory or in deferred pieces; the rest
    // live only in the ring until a flush, which happens only when a ring
    // write would overwrite an unflushed byte (ofs: the first ring position
    // written since the last flush), before a read of memory, and at the
    // end -- so the element loop issues almost no global stores (on gfx9 a
    // store holds vmcnt, which the next window refill would wait for).
    // A flush skips the deferred pieces (the copy kernel writes them).
    uint32_t fl = 0, ofs = 0xffffffffu, fk = 0;
    // ring bytes [a, b) to the output: 16 B per lane where the output is
    // 16-B aligned (ring and output agree mod 16 then), four 1-KB steps in
    // flight at once; bytes at the ends one per lane
    const bool out16 = ((uintptr_t)out & 15u) == 0u;
    auto flush_range = [&](uint32_t a, uint32_t b) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      uint32_t a16 = a, b16 = a;
      if (out16 && b - a >= 256u) {
        a16 = (a + 15u) & ~15u;
        b16 = b & ~15u;
      }
      for (uint32_t y = a + lane; y < a16; y += 64) out[y] = ring[y & (kRing - 1)];
      for (uint32_t y0 = a16; y0 < b16; y0 += 4096u) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t y = y0 + 16u * (64u * k + lane);
          if (y < b16) v[k] = *(const u32x4*)&ring[y & (kRing - 1)];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t y = y0 + 16u * (64u * k + lane);
          if (y < b16) *(AS1 u32x4*)(out + y) = v[k];
        }
      }
      for (uint32_t y = b16 + lane; y < b; y += 64) out[y] = ring[y & (kRing - 1)];
    };
    auto flush = [&](uint32_t to) {
      __builtin_amdgcn_wave_barrier();
      uint32_t x = fl;
      while (x < to) {
        while (fk < nd && tdst[fk] + tlen[fk] <= x) ++fk;
        if (fk < nd && tdst[fk] <= x) {  // x inside a deferred piece
          x = tdst[fk] + tlen[fk];
          ++fk;
          continue;
        }
        const uint32_t end = fk < nd && tdst[fk] < to ? tdst[fk] : to;
        flush_range(x, end);
        x = end;
      }
      fl = to;
      ofs = 0xffffffffu;
    };
    // before ring writes of [o, o + n): keep every unflushed byte's slot
    auto room = [&](uint32_t n) {
      if (ofs != 0xffffffffu && o + n > ofs + kRing) flush(o);
      if (ofs == 0xffffffffu) ofs = o;
    };
    // last piece starting at or before output position x (-1: none)
    auto find = [&](uint32_t x) -> int {
      int lo = -1, hi = (int)nd;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tdst[mid] <= x) lo = mid; else hi = mid;
      }
      return lo;
    };
    // append a piece of input bytes [in, in + len) at output o (the caller
    // checked nd < kMaxDef); the list goes to the copy kernel when the part
    // ends (one reservation per part: no global round trip per piece)
    auto defer = [&](uint32_t len, uint32_t in) {
#ifdef PSG_SNAPPY_PROF
      sp[4] += 1;
#endif
      if (lane == 0) {
        tdst[nd] = o;
        tsrc[nd] = in;
        tlen[nd] = len;
      }
      __builtin_amdgcn_wave_barrier();
      ++nd;
      dlo = dlo < o ? dlo : o;
      o += len;
      dhi = o;  // its bytes never enter the ring
    };
    while (!st && p < e) {
#ifdef PSG_SNAPPY_PROF
      sp[6] += 1;
#endif
      const uint32_t tag = ub(p++);
      uint32_t len, off;
      if ((tag & 3u) == 0u) {  // literal
        len = (tag >> 2) + 1u;
        if (len > 60u) {
          const uint32_t n = len - 60u;
          if (e - p < n) { st = PSG_ERR_ARG; break; }
          len = 0;
          for (uint32_t b = 0; b < n; ++b) len |= ub(p + b) << (8 * b);
          p += n;
          if (len == 0xffffffffu) { st = PSG_ERR_ARG; break; }
          len += 1u;
        }
        if (e - p < len || ucap - o < len) { st = PSG_ERR_ARG; break; }
        if (lits && len >= kBigLit && nd < kMaxDef) {
          defer(len, p);
          p += len;
          continue;
        }
        SP_T0();
        if ((int32_t)p >= wb && (int64_t)p + len <= (int64_t)wb + kWin) {
          room(len);  // len <= kWin < kRing
          const uint32_t w0 = (uint32_t)((int32_t)p - wb);
          for (uint32_t l = lane; l < len; l += 64) ring[(o + l) & (kRing - 1)] = win[w0 + l];
          o += len;
        } else {
          for (uint32_t c = 0; c < len; c += 64) {  // wave-uniform steps
            room(64);
            if (c + lane < len) ring[(o + lane) & (kRing - 1)] = s0[p + c + lane];
            o += len - c < 64u ? len - c : 64u;
          }
        }
        SP_ADD(5);
        p += len;
        continue;
      }
      if ((tag & 3u) == 1u) {
        if (e - p < 1) { st = PSG_ERR_ARG; break; }
        len = 4u + ((tag >> 2) & 7u);
        off = (tag >> 5) << 8 | ub(p);
        p += 1;
      } else if ((tag & 3u) == 2u) {
        if (e - p < 2) { st = PSG_ERR_ARG; break; }
        len = 1u + (tag >> 2);
        off = ub(p) | ub(p + 1) << 8;
        p += 2;
      } else {
        if (e - p < 4) { st = PSG_ERR_ARG; break; }
        len = 1u + (tag >> 2);
        off = ub(p) | ub(p + 1) << 8 | ub(p + 2) << 16 | ub(p + 3) << 24;
        p += 4;
      }
      if (off == 0 || off > o || ucap - o < len) { st = PSG_ERR_ARG; break; }
      // len <= 64: one step; every source byte precedes o
      const uint32_t li = off >= 64u ? lane : lane % off;  // uniform branch on off
      const uint32_t slo = o - off, shi = slo + (len < off ? len : off);
      if (nd && slo < dhi && shi > dlo) {
        // wholly inside one deferred piece (and clear of its own output):
        // deferred too, as that piece's input bytes
        SP_T0();
        const int j = find(slo);
        SP_ADD(1);
        if (j >= 0 && off >= len && slo - tdst[j] + len <= tlen[j] && nd < kMaxDef) {
          defer(len, tsrc[j] + (slo - tdst[j]));
          continue;
        }
        // else: bytes in deferred pieces come from the compressed input,
        // the rest from the ring (or, past it, memory)
        const uint32_t pos = slo + li;
        uint32_t from = 0xffffffffu;
        const int jj = find(pos);
        if (jj >= 0 && pos - tdst[jj] < tlen[jj]) from = tsrc[jj] + (pos - tdst[jj]);
        if (off > kRing) {
          flush(o);
          own_stores_visible();
        }
        const uint8_t b = lane < len ? (from != 0xffffffffu ? s0[from]
                                        : off <= kRing ? ring[pos & (kRing - 1)] : out[pos])
                                     : 0;
        room(len);
        if (lane < len) ring[(o + lane) & (kRing - 1)] = b;
      } else if (off <= kRing) {
        room(len);
        if (lane < len) ring[(o + lane) & (kRing - 1)] = ring[(o - off + li) & (kRing - 1)];
      } else {
        // the source was flushed: read it back after this wave's stores land
        flush(o);
        own_stores_visible();
        room(len);
        if (lane < len) ring[(o + lane) & (kRing - 1)] = out[o - off + li];
      }
      o += len;
    }
#ifdef PSG_SNAPPY_PROF
    const unsigned long long sp_end = clock64();
#endif
    if (!st && o != ucap) st = PSG_ERR_ARG;
    if (!st) flush(o);
    if (!st && nd) {
      // hand the part's pieces to the copy kernel; past the launch's room,
      // move them here (reads of them took the input bytes, so late is fine)
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(nlits, nd);
      base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
      for (uint32_t i = lane; i < nd; i += 64)
        if (base + i < lit_cap) lits[base + i] = SnappyLit{(const uint8_t*)(s0 + tsrc[i]), (uint8_t*)(out + tdst[i]), tlen[i]};
      for (uint32_t i = (base < lit_cap ? lit_cap - base : 0u); i < nd; ++i)
        for (uint32_t b = lane; b < tlen[i]; b += 64) out[tdst[i] + b] = s0[tsrc[i] + b];
    }
    if (lane == 0) {
      status[msg] = st;
      if (st && nbad) atomicAdd(nbad, 1ull);
    }
    asm volatile("" ::"v"(pfx));  // the prefetch loads are kept
#ifdef PSG_SNAPPY_PROF
    sp[2] = clock64() - sp_part;
    sp[7] = clock64() - sp_end;
    if (lane == 0 && msg < 4096)
      for (int i = 0; i < 8; ++i) g_sprof[msg][i] = sp[i];
#endif
    __builtin_amdgcn_wave_barrier();  // the next part rewrites the piece list
  }
}

// ---------------------------------------------------------------------------
// The streamed form (launches of few parts: a message's, the compressed-push
// path).  r06 parse clocks of one cfg2 value part (512 KB, 176 elements,
// profiles/r06_snappy_parse_clocks.json): ~540 K clocks per part, the parse
// waiting on a global round trip per element -- its window refills, its
// inline literals read 64 B at a time from memory, copies whose source lies
// in deferred literals read byte by byte from memory, and the output ring
// (indexed by output position) flushed every few KB of output even though
// the deferred literals put almost no bytes in it: each flush's stores then
// hold vmcnt for the next load.  Here:
//   * the part's compressed bytes stream into a 128 KB LDS ring by LDS-DMA
//     (1 KB per wave instruction, up to 63 KB ahead of the parse; counted
//     vmcnt waits), so tags, inline literals and the input bytes behind
//     deferred pieces are LDS reads;
//   * the output bytes the parse produces itself (short literals, copies)
//     are APPENDED to a 16 KB LDS stage with a map (output position, stage
//     offset, length), written out only when the stage fills and at the
//     part's end -- a long-literal part flushes once;
//   * a copy's source byte comes from the input ring (inside a deferred
//     piece), the stage, or (rare: written out already) memory.
// One part per workgroup, one workgroup per CU (LDS); deferral and the
// copy kernel as in snappy_kernel.
constexpr uint32_t kIRB = 128u << 10;   // input ring bytes
constexpr uint32_t kIRC = kIRB >> 10;   // input ring chunks (1 KB each)
constexpr uint32_t kLA = 48;            // chunks issued ahead of the parse position's chunk
constexpr uint32_t kSkip = 4;           // a tag this many chunks past the issued front restarts the stream
constexpr uint32_t kRestart = 16u << 10;  // a deferred literal this long restarts the stream past it
constexpr uint32_t kSB = 16u << 10;     // output stage bytes
constexpr uint32_t kMaxSt = 512;        // staged elements
constexpr uint32_t kIRBigLit = 512;     // literals deferred to the copy kernel

typedef __attribute__((address_space(3))) void* LdsPtr;
// 16 B per lane from global memory into LDS: lane l writes lds + 16 l (M0
// saved and restored; the compiler does not see the load, every reader
// waits for it explicitly)
__device__ __forceinline__ void ir_dma16(const void* g, const void* lds) {
  const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LdsPtr)lds);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(la)
      : "memory");
}
// wait until at most ~n of this wave's vector-memory operations are
// outstanding (n rounded down to a step: waiting for more is safe, they
// complete in issue order); returns the step
#define IRW(k) else if (n >= k##u) { asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); return k##u; }
__device__ __forceinline__ uint32_t ir_wait(uint32_t n) {
  if (n >= 63u) { asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); return 63u; }
  IRW(60) IRW(56) IRW(52) IRW(48) IRW(44) IRW(40) IRW(36) IRW(32) IRW(28) IRW(24) IRW(20)
  IRW(16) IRW(14) IRW(12) IRW(10) IRW(8) IRW(7) IRW(6) IRW(5) IRW(4) IRW(3) IRW(2) IRW(1)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return 0u;
}
#undef IRW

// LDS of the streamed decoder (one part per workgroup): the input ring, the
// output stage and its map, the deferred pieces
struct IrLds {
  __attribute__((aligned(16))) uint8_t ir[kIRB];
  __attribute__((aligned(16))) uint8_t sb[kSB];
  uint32_t so[kMaxSt], ss[kMaxSt], sl[kMaxSt];  // staged: output pos, stage offset, length
  uint32_t tdst[kMaxDef], tsrc[kMaxDef], tlen[kMaxDef];  // deferred pieces
};

// one part (slen in [1, 2^31)) by one wave, lanes 0..63 of the workgroup
__device__ __forceinline__ void ir_part(IrLds& S, uint64_t msg, const AS1 uint8_t* const s0,
                                        const uint64_t slen, AS1 uint8_t* const out,
                                        const uint64_t cap, int32_t* __restrict__ status,
                                        SnappyLit* __restrict__ lits,
                                        uint32_t* __restrict__ nlits, uint32_t lit_cap,
                                        unsigned long long* __restrict__ nbad) {
    uint8_t* const ir = S.ir;
    uint8_t* const sb = S.sb;
    uint32_t* const so = S.so;
    uint32_t* const ss = S.ss;
    uint32_t* const sl = S.sl;
    uint32_t* const tdst = S.tdst;
    uint32_t* const tsrc = S.tsrc;
    uint32_t* const tlen = S.tlen;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t e = (uint32_t)slen;
    int32_t st = 0;
#ifdef PSG_SNAPPY_PROF
    unsigned long long sp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long sp_part = clock64();
#endif
    // ---- the input ring: input position q is byte q + mis of the 16-B
    // aligned stream, in chunk (q + mis) >> 10
    const uint32_t mis = (uint32_t)((uintptr_t)s0 & 15u);
    const AS1 uint8_t* const A = s0 - mis;
    const uint32_t nch = (e + mis + 1023u) >> 10;
    uint32_t lo = 0, iss = 0, wt = 0;  // chunks [lo, iss) issued since a restart, [lo, wt) landed
    auto issue = [&](uint32_t c) {
      const uint32_t u = 64u * c + lane;  // 16-B unit of the aligned stream
      if (16u * u < e + mis) ir_dma16((const void*)(A + 16u * u), &ir[(c << 10) & (kIRB - 1u)]);
    };
    // issue up to `ahead` chunks past the parse chunk pc: kLA while the
    // elements are short (value parts of floats: ~3 KB literals), 2 after a
    // deferred literal of >= kRestart bytes (key parts, incompressible
    // parts: the stream restarts past each one instead of carrying its
    // bytes through the ring)
    uint32_t ahead = kLA;
    auto topup = [&](uint32_t pc) {
      const uint32_t capc = pc + ahead + 1u < nch ? pc + ahead + 1u : nch;
#ifdef PSG_SNAPPY_PROF
      const unsigned long long _t0 = clock64();
#endif
      while (iss < capc) issue(iss++);
#ifdef PSG_SNAPPY_PROF
      sp[5] += clock64() - _t0;  // (r06 diagnostic: issue clocks in the literal slot)
#endif
    };
    auto land = [&](uint32_t c) {
      if (c < wt) return;
      SP_T0();
#ifdef PSG_SNAPPY_PROF
      sp[3] += 1;
#endif
      wt = iss - ir_wait(iss - 1u - c);
      SP_ADD(0);
    };
    auto resident = [&](uint32_t c) -> bool { return c >= lo && c < iss && c + kIRC >= iss; };
    // input bytes [a, b] (b - a < 63 KB) resident and landed; the stream
    // restarts at a's chunk when it lies far past the issued front (a long
    // deferred literal skipped).  false: read them from memory
    // the stream restarted at chunk ca (past a long deferred literal: its
    // bytes are not streamed through the ring).  The old stream's DMAs still
    // in flight hold the slots of chunks iss-63 .. iss-1: the new chunks
    // ca .. ca+kLA reuse none of them unless the jump is long
    auto restart = [&](uint32_t ca) {
      if (ca - iss + kLA + 64u > kIRC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lo = iss = wt = ca;
    };
    auto ensure = [&](uint32_t a, uint32_t b) -> bool {
      const uint32_t ca = (a + mis) >> 10, cb = (b + mis) >> 10;
      if (ca < lo) return false;
      if (cb >= iss + kSkip) restart(ca);
      topup(ca);
      if (!resident(ca) || !resident(cb)) return false;
      land(cb);
      return true;
    };
    auto irb = [&](uint32_t q) -> uint32_t { return ir[(q + mis) & (kIRB - 1u)]; };
    // one input byte q behind the parse (deferred-piece sources)
    auto inb = [&](uint32_t q) -> uint32_t {
      const uint32_t c = (q + mis) >> 10;
      return resident(c) && c < wt ? irb(q) : (uint32_t)s0[q];
    };
    uint32_t lp = 0xffffffffu - 64u, la = 0;
    auto ub = [&](uint32_t q) -> uint32_t {
      if (q - lp >= 64u) {
#ifdef PSG_SNAPPY_PROF
        const unsigned long long _u0 = clock64();
#endif
        const uint32_t q1 = q + 63u < e ? q + 63u : e - 1u;
        lp = q;
        la = ensure(q, q1) ? irb(q + lane) : (q + lane < e ? (uint32_t)s0[q + lane] : 0u);
#ifdef PSG_SNAPPY_PROF
        (void)__builtin_amdgcn_readfirstlane((int)la);
        sp[7] += clock64() - _u0;  // r06 diagnostic: lookahead loads in the end slot
#endif
      }
      return (uint32_t)__builtin_amdgcn_readlane((int)la, (int)(q - lp));
    };
    uint64_t ulen = 0;
    bool done = false;
    uint32_t p = 0;
    while (p < 5 && p < e && !done) {
      const uint32_t b = ub(p);
      ulen |= (uint64_t)(b & 0x7f) << (7 * p);
      done = !(b & 0x80);
      ++p;
    }
    if (!done || ulen > 0xffffffffull) st = PSG_ERR_ARG;
    if (!st && ulen != cap) st = PSG_ERR_SIZE;
    const uint32_t ucap = (uint32_t)ulen;
    uint32_t o = 0;
    // deferred pieces (output order); [dlo, dhi) spans them all
    uint32_t nd = 0, dlo = 0xffffffffu, dhi = 0;
    // the stage: nst elements, nsb bytes; output below fo that is neither
    // staged nor deferred is in memory
    uint32_t nst = 0, nsb = 0, fo = 0;
    bool wrote = false;  // stores since the last fence (a read of memory waits for them)
    auto flush_stage = [&]() {
      __builtin_amdgcn_wave_barrier();
      for (uint32_t i = 0; i < nst; ++i) {
        const uint32_t d = so[i], s = ss[i], n = sl[i];
        for (uint32_t l = lane; l < n; l += 64) out[d + l] = sb[s + l];
      }
      wrote = wrote || nst > 0;
      nst = 0;
      nsb = 0;
      fo = o;
      __builtin_amdgcn_wave_barrier();
    };
    // room in the stage for n bytes (n <= kSB) and one element
    auto room = [&](uint32_t n) {
      if (nsb + n > kSB || nst == kMaxSt) flush_stage();
    };
    auto add_stage = [&](uint32_t n) {  // the n bytes just written at sb[nsb]
      if (lane == 0) {
        so[nst] = o;
        ss[nst] = nsb;
        sl[nst] = n;
      }
      __builtin_amdgcn_wave_barrier();
      ++nst;
      nsb += n;
      o += n;
    };
    // last deferred piece / staged element starting at or before x (-1: none)
    auto find_def = [&](uint32_t x) -> int {
      if (nd && tdst[nd - 1] <= x) return (int)nd - 1;
      int l0 = -1, hi = (int)nd;
      while (hi - l0 > 1) {
        const int mid = (l0 + hi) >> 1;
        if (tdst[mid] <= x) l0 = mid; else hi = mid;
      }
      return l0;
    };
    auto find_st = [&](uint32_t x) -> int {
      if (nst && so[nst - 1] <= x) return (int)nst - 1;
      int l0 = -1, hi = (int)nst;
      while (hi - l0 > 1) {
        const int mid = (l0 + hi) >> 1;
        if (so[mid] <= x) l0 = mid; else hi = mid;
      }
      return l0;
    };
    auto defer = [&](uint32_t len, uint32_t in) {
#ifdef PSG_SNAPPY_PROF
      sp[4] += 1;
#endif
      if (lane == 0) {
        tdst[nd] = o;
        tsrc[nd] = in;
        tlen[nd] = len;
      }
      __builtin_amdgcn_wave_barrier();
      ++nd;
      dlo = dlo < o ? dlo : o;
      o += len;
      dhi = o;
    };
    while (!st && p < e) {
#ifdef PSG_SNAPPY_PROF
      sp[6] += 1;
#endif
      topup((p + mis) >> 10);  // keep the stream kLA chunks ahead
      const uint32_t tag = ub(p++);
      uint32_t len, off;
      if ((tag & 3u) == 0u) {  // literal
        len = (tag >> 2) + 1u;
        if (len > 60u) {
          const uint32_t n = len - 60u;
          if (e - p < n) { st = PSG_ERR_ARG; break; }
          len = 0;
          for (uint32_t b = 0; b < n; ++b) len |= ub(p + b) << (8 * b);
          p += n;
          if (len == 0xffffffffu) { st = PSG_ERR_ARG; break; }
          len += 1u;
        }
        if (e - p < len || ucap - o < len) { st = PSG_ERR_ARG; break; }
        if (lits && len >= kIRBigLit && nd < kMaxDef) {
          defer(len, p);
          p += len;
          if (len >= kRestart) {
            ahead = 2u;
            if (((p + mis) >> 10) >= iss && p < e) restart((p + mis) >> 10);
          } else {
            ahead = kLA;
          }
          continue;
        }
        ahead = kLA;
        // staged in pieces of <= 4 KB (from the input ring, or memory)
        for (uint32_t c = 0; c < len; c += 4096u) {
          const uint32_t n = len - c < 4096u ? len - c : 4096u;
          const bool inr = ensure(p + c, p + c + n - 1u);
          room(n);
          if (inr) {
            for (uint32_t l = lane; l < n; l += 64) sb[nsb + l] = (uint8_t)irb(p + c + l);
          } else {
            for (uint32_t l = lane; l < n; l += 64) sb[nsb + l] = s0[p + c + l];
          }
          add_stage(n);
        }
        p += len;
        continue;
      }
      if ((tag & 3u) == 1u) {
        if (e - p < 1) { st = PSG_ERR_ARG; break; }
        len = 4u + ((tag >> 2) & 7u);
        off = (tag >> 5) << 8 | ub(p);
        p += 1;
      } else if ((tag & 3u) == 2u) {
        if (e - p < 2) { st = PSG_ERR_ARG; break; }
        len = 1u + (tag >> 2);
        off = ub(p) | ub(p + 1) << 8;
        p += 2;
      } else {
        if (e - p < 4) { st = PSG_ERR_ARG; break; }
        len = 1u + (tag >> 2);
        off = ub(p) | ub(p + 1) << 8 | ub(p + 2) << 16 | ub(p + 3) << 24;
        p += 4;
      }
      if (off == 0 || off > o || ucap - o < len) { st = PSG_ERR_ARG; break; }
      // len <= 64: one step; source byte of lane l is output o - off + (l mod off)
      const uint32_t slo = o - off;
      SP_T0();
      if (nd && slo < dhi && slo + (len < off ? len : off) > dlo) {
        // wholly inside one deferred piece (and clear of its own output):
        // deferred too, as that piece's input bytes
        const int j = find_def(slo);
        if (j >= 0 && off >= len && slo - tdst[j] + len <= tlen[j] && nd < kMaxDef) {
          SP_ADD(1);
          defer(len, tsrc[j] + (slo - tdst[j]));
          continue;
        }
      }
      const uint32_t li = off >= 64u ? lane : lane % off;
      const uint32_t pos = slo + li;
      // where this lane's source byte is: 0 deferred piece (input), 1 the
      // stage, 2 memory (written out).  Usually the whole source span
      // [slo, shi) lies in one staged element or one deferred piece: one
      // uniform lookup then
      const uint32_t shi = slo + (len < off ? len : off);
      uint32_t where = 2u, at = 0u;
      bool one = false;
      {
        const int js = nst && slo >= fo ? find_st(slo) : -1;
        if (js >= 0 && shi - so[js] <= sl[js]) {
          one = true;
          where = 1u;
          at = ss[js] + (pos - so[js]);
        } else if (nd && slo >= dlo && slo < dhi) {
          const int jd = find_def(slo);
          if (jd >= 0 && shi - tdst[jd] <= tlen[jd]) {
            one = true;
            where = 0u;
            at = tsrc[jd] + (pos - tdst[jd]);
          }
        }
      }
      if (!one && lane < len) {
        const int jd = nd && pos < dhi && pos >= dlo ? find_def(pos) : -1;
        if (jd >= 0 && pos - tdst[jd] < tlen[jd]) {
          where = 0u;
          at = tsrc[jd] + (pos - tdst[jd]);
        } else {
          const int js = nst && pos >= fo ? find_st(pos) : -1;
          if (js >= 0 && pos - so[js] < sl[js]) {
            where = 1u;
            at = ss[js] + (pos - so[js]);
          } else {
            at = pos;
          }
        }
      }
      if (wrote && __ballot(lane < len && where == 2u)) {
        // bytes written out earlier by this wave: visible to its loads
        own_stores_visible();
        wrote = false;
      }
      const uint32_t b = lane < len ? (where == 0u ? inb(at) : where == 1u ? (uint32_t)sb[at]
                                                                         : (uint32_t)out[at])
                                    : 0u;
      SP_ADD(1);
      room(len);
      if (lane < len) sb[nsb + lane] = (uint8_t)b;
      add_stage(len);
    }
#ifdef PSG_SNAPPY_PROF
    const unsigned long long sp_end = clock64();
#endif
    if (!st && o != ucap) st = PSG_ERR_ARG;
    if (!st) flush_stage();
    if (!st && nd) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(nlits, nd);
      base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
      for (uint32_t i = lane; i < nd; i += 64)
        if (base + i < lit_cap)
          lits[base + i] = SnappyLit{(const uint8_t*)(s0 + tsrc[i]), (uint8_t*)(out + tdst[i]), tlen[i]};
      for (uint32_t i = (base < lit_cap ? lit_cap - base : 0u); i < nd; ++i)
        for (uint32_t b = lane; b < tlen[i]; b += 64) out[tdst[i] + b] = s0[tsrc[i] + b];
    }
    if (lane == 0) {
      status[msg] = st;
      if (st && nbad) atomicAdd(nbad, 1ull);
    }
    // every DMA of this part has landed before the next part reuses the ring
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef PSG_SNAPPY_PROF
    sp[2] = clock64() - sp_part;
    (void)sp_end;
    if (lane == 0 && msg < 4096)
      for (int i = 0; i < 8; ++i) g_sprof[msg][i] = sp[i];
#endif
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64) void snappy_ir_kernel(const uint8_t* __restrict__ src,
                                                       const uint64_t* __restrict__ soff,
                                                       uint8_t* __restrict__ dst,
                                                       const uint64_t* __restrict__ doff,
                                                       const uint64_t* __restrict__ dcap,
                                                       uint64_t nmsg, int32_t* __restrict__ status,
                                                       SnappyLit* __restrict__ lits,
                                                       uint32_t* __restrict__ nlits,
                                                       uint32_t lit_cap,
                                                       unsigned long long* __restrict__ nbad,
                                                       int pairs) {
  __shared__ IrLds S;
  const uint32_t lane = threadIdx.x;
  for (uint64_t msg = blockIdx.x; msg < nmsg; msg += gridDim.x) {
    const AS1 uint8_t* const s0 =
        (const AS1 uint8_t*)(pairs ? (const uint8_t*)soff[2 * msg] : src + soff[msg]);
    const uint64_t slen = pairs ? soff[2 * msg + 1] - soff[2 * msg] : soff[msg + 1] - soff[msg];
    AS1 uint8_t* const out = (AS1 uint8_t*)(dst + doff[msg]);
    const uint64_t cap = dcap ? dcap[msg] : doff[msg + 1] - doff[msg];
    if (slen == 0) {
      if (lane == 0) status[msg] = cap == 0 ? 0 : PSG_ERR_SIZE;
      continue;
    }
    if (slen >= (1ull << 31)) {
      if (lane == 0) status[msg] = PSG_ERR_ARG;
      continue;
    }
    ir_part(S, msg, s0, slen, out, cap, status, lits, nlits, lit_cap, nbad);
  }
}

// ---------------------------------------------------------------------------
// The table form (launches of few parts; PSG_SNAPPY_IR == 2, the default).
// r06 measured the streamed decoder above bound by its per-element chain on
// one wave (~2.8 K clocks per element of a cfg2 value part: the copy-source
// lookups among the deferred pieces, the stream's DMA issue, the stage's
// map, profiles/r06_ab_snappy_stream.txt), while the parts of a compressed
// push hold few elements (incompressible data: long literals and spurious
// 4-byte matches).  Here one workgroup (4 waves) per part:
//   1. wave 0 walks the TAGS only -- one dependent 64-byte lookahead load
//      per element past the window (L2 hits: waves 1-3 pull the part into
//      L2 meanwhile) -- into an LDS table (output position, input position
//      or offset, length), with the streamed form's format checks in the
//      same order (the same status for a corrupt part);
//   2. all waves move the elements at once: short literals from the input,
//      long ones (>= kTabBigLit) handed to the chip-wide copy kernel, and
//      every byte of a copy resolved on its own lane through the table to
//      the literal byte it repeats (copies of copies followed up to
//      kTabDepth times), read from the input -- no output is read back, and
//      no element waits for another;
//   3. wave 0 writes the copies that did not resolve (chains deeper than
//      kTabDepth: runs), in element order, from the output written so far.
// A part of more than kTabMax elements, or of more than kTabPend unresolved
// copies (compressible data: the streamed form's LDS-resident output serves
// it better), runs ir_part instead, in the same workgroup.
constexpr uint32_t kTabMax = 4096;
constexpr uint32_t kTabPend = 64;
constexpr uint32_t kTabBigLit = 512;
constexpr int kTabDepth = 4;
constexpr uint32_t kCopyBit = 0x80000000u;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
struct TabLds {
  // element i: x = output position (rec[nel].x = the part's length), y =
  // literal: input position / copy: offset, z = length (| kCopyBit for a
  // copy), w = literal: deferred index (~0: moved in step 2) / copy: 1 =
  // unresolved
  u32x4_t rec[kTabMax + 1];
  uint32_t nel, verdict, base, npend;
};
union SnappyTabLds {
  IrLds ir;
  TabLds tab;
};

__global__ __launch_bounds__(256) void snappy_tab_kernel(const uint8_t* __restrict__ src,
                                                        const uint64_t* __restrict__ soff,
                                                        uint8_t* __restrict__ dst,
                                                        const uint64_t* __restrict__ doff,
                                                        const uint64_t* __restrict__ dcap,
                                                        uint64_t nmsg, int32_t* __restrict__ status,
                                                        SnappyLit* __restrict__ lits,
                                                        uint32_t* __restrict__ nlits,
                                                        uint32_t lit_cap,
                                                        unsigned long long* __restrict__ nbad,
                                                        int pairs) {
  __shared__ SnappyTabLds U;
  TabLds& T = U.tab;
  // the wave index as a wave-uniform (scalar) value: branches on it are not
  // divergent, so the walk's state stays in SGPRs
  const uint32_t tid = threadIdx.x, lane = tid & 63u,
                 w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
  for (uint64_t msg = blockIdx.x; msg < nmsg; msg += gridDim.x) {
    const AS1 uint8_t* const s0 =
        (const AS1 uint8_t*)(pairs ? (const uint8_t*)soff[2 * msg] : src + soff[msg]);
    const uint64_t slen = pairs ? soff[2 * msg + 1] - soff[2 * msg] : soff[msg + 1] - soff[msg];
    AS1 uint8_t* const out = (AS1 uint8_t*)(dst + doff[msg]);
    const uint64_t cap = dcap ? dcap[msg] : doff[msg + 1] - doff[msg];
    if (slen == 0 || slen >= (1ull << 31)) {  // the workgroup agrees: no barrier skipped
      if (tid == 0) status[msg] = slen ? PSG_ERR_ARG : cap == 0 ? 0 : PSG_ERR_SIZE;
      continue;
    }
    const uint32_t e = (uint32_t)slen;
#ifdef PSG_SNAPPY_PROF
    // [0] step 1 clocks, [1] step 2 (wave 0's share), [2] the part, [3] window
    // loads, [4] unresolved copies, [5] step 3, [6] elements, [7] clocks in
    // the window loads' round trips
    unsigned long long sp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long sp_part = clock64();
#endif
    // ---- 1. the tags (wave 0); the part into L2 (waves 1-3)
    if (w == 0) {
      int32_t st = 0;
      bool full = false;
      // a 256-byte window of the part in the wave's registers (lane l: the
      // dword at wb + 4 l of the 4-B aligned stream, clamped to the dword
      // holding the last byte: never past it, so never into another page),
      // its bytes taken by readlane.  Every branch here is on wave-uniform
      // values: r06's first form loaded the window under a per-lane bound
      // test, which made every byte read a divergent branch with exec-mask
      // saves (~1.4 K clocks per element)
      const uint32_t mis4 = (uint32_t)((uintptr_t)s0 & 3u);
      const AS1 uint32_t* const s4 = (const AS1 uint32_t*)(s0 - mis4);
      const uint32_t lastw = (e - 1u + mis4) >> 2;  // dword holding the last byte
      uint32_t wb = 0xffffffffu - 1024u, la = 0;     // window start (dword index)
      auto ub = [&](uint32_t q) -> uint32_t {
        const uint32_t a = __builtin_amdgcn_readfirstlane(q + mis4);
        if ((a >> 2) - wb >= 64u) {
          wb = a >> 2;
          const uint32_t d = wb + lane;
          la = s4[d < lastw ? d : lastw];
#ifdef PSG_SNAPPY_PROF
          sp[3] += 1;
#endif
        }
        const uint32_t k = a - 4u * wb;
        return ((uint32_t)__builtin_amdgcn_readlane((int)la, (int)(k >> 2)) >> (8u * (k & 3u))) & 0xffu;
      };
      uint64_t ulen = 0;
      bool done = false;
      uint32_t p = 0;
      while (p < 5 && p < e && !done) {
        const uint32_t b = ub(p);
        ulen |= (uint64_t)(b & 0x7f) << (7 * p);
        done = !(b & 0x80);
        ++p;
      }
      if (!done || ulen > 0xffffffffull) st = PSG_ERR_ARG;
      if (!st && ulen != cap) st = PSG_ERR_SIZE;
      const uint32_t ucap = (uint32_t)ulen;
      // eight bytes at input position q in one 64-bit value (the tag and
      // every length / offset byte of an element): three readlanes from the
      // window instead of a window test and a readlane per byte; bytes past
      // the part's end are garbage, and the header checks below never use
      // them
      auto u8x8 = [&](uint32_t q) -> uint64_t {
        const uint32_t a = __builtin_amdgcn_readfirstlane(q + mis4);
        const uint32_t d0 = a >> 2;
        if (d0 - wb > 61u) {  // dwords d0 .. d0 + 2 in the window
          wb = d0;
          const uint32_t d = wb + lane;
#ifdef PSG_SNAPPY_PROF
          const unsigned long long t_ld = clock64();
#endif
          la = s4[d < lastw ? d : lastw];
#ifdef PSG_SNAPPY_PROF
          sp[3] += 1;
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the load's latency, in sp[7]
          sp[7] += clock64() - t_ld;
#endif
        }
        const uint32_t k = d0 - wb;
        const uint64_t x01 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)la, (int)k) |
                             (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)la, (int)k + 1) << 32;
        const uint32_t sh = 8u * (a & 3u);
        if (!sh) return x01;
        const uint64_t x2 = (uint32_t)__builtin_amdgcn_readlane((int)la, (int)k + 2);
        return (x01 >> sh) | (x2 << (64u - sh));
      };
      uint32_t o = 0, n = 0, nd = 0;
      // one element per iteration, with no divergent code in the loop (the
      // walk is issue-bound on its one wave: r06 measured ~1 K clocks per
      // element while a lane-0 LDS store made the compiler keep the loop's
      // state in VGPRs under exec masks): records collect in registers, lane
      // k of rx..rw holding element n0 + k (a per-lane select), and go to LDS
      // 64 at a time
      uint32_t rx = 0, ry = 0, rz = 0, rw = 0;
      auto flush_recs = [&](uint32_t n0, uint32_t cnt) {
        if (lane < cnt) *(u32x4_t*)&T.rec[n0 + lane] = u32x4_t{rx, ry, rz, rw};
      };
      while (!st && p < e) {
        if (n == kTabMax) {
          full = true;
          break;
        }
        const uint64_t hv = u8x8(p);
        const uint32_t tag = (uint32_t)hv & 0xffu, t3 = tag & 3u, l6 = tag >> 2;
        const uint32_t rem = e - p;  // >= 1
        const uint32_t b32 = (uint32_t)(hv >> 8);  // the bytes after the tag
        const bool lit = t3 == 0u;
        uint32_t len, a, x, adv;
        bool bad;
        if (lit) {  // 0..4 length bytes after the tag
          const uint32_t nb = __builtin_elementwise_max(l6, 59u) - 59u;
          const uint32_t hdr = 1u + nb;
          const uint32_t field = nb >= 4u ? b32 : b32 & ((1u << (8u * nb)) - 1u);
          len = nb ? field + 1u : l6 + 1u;  // a length field of 2^32 - 1 is corrupt
          bad = rem < hdr || (nb && field == 0xffffffffu) || rem - hdr < len || ucap - o < len;
          a = p + hdr;
          const bool dfr = lits && len >= kTabBigLit;
          x = dfr ? nd : 0xffffffffu;
          nd += dfr ? 1u : 0u;
          adv = hdr + len;
        } else {  // 1, 2 or 4 offset bytes
          const uint32_t nb = t3 + (t3 >> 1 & t3);  // 1, 2, 4
          len = t3 == 1u ? 4u + (l6 & 7u) : l6 + 1u;
          const uint32_t field = nb >= 4u ? b32 : b32 & ((1u << (8u * nb)) - 1u);
          a = t3 == 1u ? ((tag >> 5) << 8 | field) : field;  // the offset
          bad = rem < 1u + nb || a == 0u || a > o || ucap - o < len;
          x = 0u;
          adv = 1u + nb;
        }
        if (bad) {
          st = PSG_ERR_ARG;
          break;
        }
        const uint32_t k = n & 63u;
        const bool mine = lane == k;  // a select per lane, not a branch
        rx = mine ? o : rx;
        ry = mine ? a : ry;
        rz = mine ? (lit ? len : len | kCopyBit) : rz;
        rw = mine ? x : rw;
        if (k == 63u) flush_recs(n - 63u, 64u);
        p += adv;
        o += len;
        ++n;
      }
      if (n & 63u) flush_recs(n & ~63u, n & 63u);
      if (!st && !full && o != ucap) st = PSG_ERR_ARG;
#ifdef PSG_SNAPPY_PROF
      sp[0] = clock64() - sp_part;
      sp[6] = n;
#endif
      if (lane == 0) {
        T.rec[n].x = o;
        T.nel = n;
        T.verdict = st ? 1u : full ? 2u : 0u;
        T.npend = 0;
        uint32_t base = 0;
        if (st) {
          status[msg] = st;
          if (nbad) atomicAdd(nbad, 1ull);
        } else if (!full && nd) {
          base = atomicAdd(nlits, nd);
        }
        T.base = base;
      }
    } else {
      // one load per 128-B line, eight in flight per lane
      uint32_t acc = 0;
      for (uint32_t x0 = (tid - 64u) * 128u; x0 < e; x0 += 8u * 192u * 128u) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t x = x0 + (uint32_t)k * 192u * 128u;
          v[k] = x < e ? (uint32_t)s0[x] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k];
      }
      asm volatile("" ::"v"(acc));

    }
    __syncthreads();  // (1) the table
    const uint32_t verdict = T.verdict, nel = T.nel, base = T.base;
    __syncthreads();  // (1b) read by every wave before the LDS may be reused
    if (verdict == 1u) continue;  // corrupt: reported in step 1
    if (verdict == 2u) {          // too many elements: the streamed form
      if (w == 0) ir_part(U.ir, msg, s0, slen, out, cap, status, lits, nlits, lit_cap, nbad);
      __syncthreads();
      continue;
    }
    // last element starting at or before output position x (< the part's length)
    auto find = [&](uint32_t x) -> uint32_t {
      uint32_t lo = 0, hi = nel;  // to[lo] <= x < to[hi]
      while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (T.rec[mid].x <= x) lo = mid;
        else hi = mid;
      }
      return lo;
    };
    // ---- 2. the elements, round robin over the waves
#ifdef PSG_SNAPPY_PROF
    const unsigned long long sp_2 = clock64();
#endif
    // a copy byte at output position q (< the copy's own position), followed
    // through the table to the literal byte it repeats: its input position,
    // or ~0 past kTabDepth copies.  jc caches the last element found (the
    // bytes of one copy mostly lie in one element)
    auto resolve = [&](uint32_t q, uint32_t& jc) -> uint32_t {
      for (int d = 0; d < kTabDepth; ++d) {
        uint32_t j = jc;
        if (!(T.rec[j].x <= q && q < T.rec[j + 1].x)) j = find(q);
        if (d == 0) jc = j;
        const uint32_t lj = T.rec[j].z, dq = q - T.rec[j].x, aj = T.rec[j].y;
        if (!(lj & kCopyBit)) return aj + dq;
        q = T.rec[j].x - aj + dq % aj;  // byte dq of copy j repeats this one
      }
      return 0xffffffffu;
    };
    constexpr uint32_t kLaneCopy = 8;  // copies this short: one lane each, below
    for (uint32_t i = w; i < nel; i += 4u) {
      const uint32_t oo = T.rec[i].x, a = T.rec[i].y, lk = T.rec[i].z, x = T.rec[i].w;
      const uint32_t len = lk & ~kCopyBit;
      if (!(lk & kCopyBit)) {
        if (x != 0xffffffffu && base + x < lit_cap) {
          if (lane == 0)
            lits[base + x] = SnappyLit{(const uint8_t*)(s0 + a), (uint8_t*)(out + oo), len};
        } else {
          for (uint32_t l = lane; l < len; l += 64u) out[oo + l] = s0[a + l];
        }
        continue;
      }
      if (len <= kLaneCopy) continue;
      // a longer copy, one byte per lane: byte l is output[o - off + (l mod
      // off)] (run-length copies included)
      uint32_t from = 0;
      if (lane < len) {
        uint32_t jc = 0;
        from = resolve(oo - a + (a >= 64u ? lane : lane % a), jc);
      }
      if (__ballot(lane < len && from == 0xffffffffu)) {
        if (lane == 0) {
          T.rec[i].w = 1u;
          atomicAdd(&T.npend, 1u);
        }
      } else if (lane < len) {
        out[oo + lane] = s0[from];
      }
    }
    // short copies (incompressible data: spurious 4-byte matches), one lane
    // each: a wave resolves 64 of them at once instead of one
    for (uint32_t i = tid; i < nel; i += 256u) {
      const uint32_t lk = T.rec[i].z;
      const uint32_t len = lk & ~kCopyBit;
      if (!(lk & kCopyBit) || len > kLaneCopy) continue;
      const uint32_t oo = T.rec[i].x, a = T.rec[i].y;
      uint32_t src[kLaneCopy];
      uint32_t jc = 0;
      bool ok = true;
      for (uint32_t l = 0; l < len; ++l) {
        src[l] = resolve(oo - a + (l < a ? l : l % a), jc);
        ok = ok && src[l] != 0xffffffffu;
      }
      if (!ok) {
        T.rec[i].w = 1u;
        atomicAdd(&T.npend, 1u);
        continue;
      }
      uint8_t b[kLaneCopy];
      for (uint32_t l = 0; l < len; ++l) b[l] = s0[src[l]];
      for (uint32_t l = 0; l < len; ++l) out[oo + l] = b[l];
    }
    // step 2's stores visible to step 3's loads (and to ir_part's reads)
    own_stores_visible();
    __syncthreads();  // (2)
    const uint32_t npend = T.npend;
#ifdef PSG_SNAPPY_PROF
    sp[1] = clock64() - sp_2;
    sp[4] = npend;
    const unsigned long long sp_3 = clock64();
#endif
    if (npend > kTabPend) {  // compressible: the streamed form rewrites the whole part
      __syncthreads();
      if (w == 0) ir_part(U.ir, msg, s0, slen, out, cap, status, lits, nlits, lit_cap, nbad);
      __syncthreads();
      continue;
    }
    // ---- 3. the unresolved copies in element order (wave 0): a source byte
    // of a literal from the input, of a copy from the output (written in step
    // 2, or earlier in this step)
    if (w == 0) {
      for (uint32_t i0 = 0; npend && i0 < nel; i0 += 64u) {
        const uint32_t ii = i0 + lane;
        unsigned long long m = __ballot(ii < nel && (T.rec[ii].z & kCopyBit) && T.rec[ii].w == 1u);
        while (m) {
          const uint32_t i = i0 + (uint32_t)__builtin_ctzll(m);
          m &= m - 1;
          const uint32_t oo = T.rec[i].x, off = T.rec[i].y, len = T.rec[i].z & ~kCopyBit;
          if (lane < len) {
            const uint32_t q = oo - off + (off >= 64u ? lane : lane % off);
            const uint32_t j = find(q);
            const uint32_t b = (T.rec[j].z & kCopyBit) ? (uint32_t)out[q]
                                                     : (uint32_t)s0[T.rec[j].y + (q - T.rec[j].x)];
            out[oo + lane] = (uint8_t)b;
          }
          own_stores_visible();
        }
      }
      if (lane == 0) status[msg] = 0;
#ifdef PSG_SNAPPY_PROF
      sp[5] = clock64() - sp_3;
      sp[2] = clock64() - sp_part;
      if (lane == 0 && msg < 4096)
        for (int i = 0; i < 8; ++i) g_sprof[msg][i] = sp[i];
#endif
    }
    __syncthreads();  // (3) before the next part's table
  }
}

// The deferred literals, chip-wide: a literal is cut into 16-B units
// aligned to its destination; a workgroup moves 256 units (4 KB) per chunk,
// chunks numbered across literals and dealt round-robin to the grid (the
// literals' chunk counts are scanned in LDS, 256 literals at a time, and a
// chunk finds its literal by binary search there).  Each lane loads the 5
// aligned source dwords around its unit and shifts them into place
// (v_alignbyte): aligned 16-B stores whatever the source offset.  Units at
// a literal's ends, and ones whose source window would pass the dword
// holding the literal's last byte, move byte by byte.
__global__ __launch_bounds__(256) void snappy_lit_kernel(const SnappyLit* __restrict__ lits,
                                                         const uint32_t* __restrict__ nlits,
                                                         uint32_t lit_cap) {
  __shared__ uint32_t pre[257];  // chunks before literal i of the batch
  __shared__ uint32_t wsum[4];
  const uint32_t n = *nlits < lit_cap ? *nlits : lit_cap;
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint64_t base = 0;  // chunks of the batches before
  for (uint32_t b0 = 0; b0 < n; b0 += 256) {
    uint32_t nch = 0;
    if (b0 + t < n) {
      const SnappyLit L = lits[b0 + t];
      const uintptr_t A = (uintptr_t)L.dst & ~(uintptr_t)15;
      const uint64_t units = ((uintptr_t)L.dst + L.len - A + 15) / 16;
      nch = (uint32_t)((units + kLitUnits - 1) / kLitUnits);
    }
    // block exclusive scan of nch
    uint32_t x = nch;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t v = 0; v < w; ++v) off += wsum[v];
    pre[t + 1] = off + x;
    if (t == 0) pre[0] = 0;
    __syncthreads();
    const uint32_t nb = n - b0 < 256u ? n - b0 : 256u;
    const uint32_t tot = pre[nb];
    // this block's chunks g = base + c, c = 0..tot-1, g = blockIdx.x mod grid
    for (uint32_t c = (uint32_t)((blockIdx.x + gridDim.x - base % gridDim.x) % gridDim.x); c < tot;
         c += gridDim.x) {
      uint32_t lo = 0, hi = nb;  // last literal with pre[i] <= c
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= c) lo = mid; else hi = mid;
      }
      const SnappyLit L = lits[b0 + lo];
      const uintptr_t A = (uintptr_t)L.dst & ~(uintptr_t)15;
      const uint64_t units = ((uintptr_t)L.dst + L.len - A + 15) / 16;
      const uint64_t u = (uint64_t)(c - pre[lo]) * kLitUnits + t;
      if (u >= units) continue;
      const uintptr_t ua = A + 16 * u;
      const uintptr_t b0b = ua > (uintptr_t)L.dst ? ua : (uintptr_t)L.dst;
      const uintptr_t b1 = ua + 16 < (uintptr_t)L.dst + L.len ? ua + 16 : (uintptr_t)L.dst + L.len;
      const uintptr_t sa = (uintptr_t)L.src + (ua - (uintptr_t)L.dst);  // source of byte ua
      const uintptr_t a0 = sa & ~(uintptr_t)3;
      const uintptr_t slast = ((uintptr_t)L.src + L.len - 1) & ~(uintptr_t)3;
      if (b0b == ua && b1 == ua + 16 && a0 + 16 <= slast) {
        const uint32_t* wp = (const uint32_t*)a0;
        const uint32_t sh = (uint32_t)(sa & 3u);
        uint32_t xw[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) xw[i] = wp[i];
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 v;
        v.x = __builtin_amdgcn_alignbyte(xw[1], xw[0], sh);
        v.y = __builtin_amdgcn_alignbyte(xw[2], xw[1], sh);
        v.z = __builtin_amdgcn_alignbyte(xw[3], xw[2], sh);
        v.w = __builtin_amdgcn_alignbyte(xw[4], xw[3], sh);
        *(u4*)ua = v;
      } else {
        for (uintptr_t b = b0b; b < b1; ++b) *(uint8_t*)b = L.src[b - (uintptr_t)L.dst];
      }
    }
    base += tot;
    __syncthreads();  // pre[] is rewritten by the next batch
  }
}

}  // namespace

// room for 256 deferred pieces per part on average (shared by the launch;
// past it pieces move in the parse)
constexpr uint32_t kAvgDef = 256;
#ifdef PSG_SNAPPY_PROF
extern "C" int psg_debug_snappy_prof(unsigned long long* out, uint32_t nmsg) {
  if (nmsg > 4096) nmsg = 4096;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sprof), (size_t)nmsg * 64) == hipSuccess ? 0 : -1;
}
#endif

size_t snappy_scratch_bytes(uint64_t nmsg) {
  return 256 + (size_t)nmsg * kAvgDef * sizeof(SnappyLit);
}

hipError_t launch_snappy(const uint8_t* src, const uint64_t* soff, uint64_t nmsg, uint8_t* dst,
                         const uint64_t* doff, const uint64_t* dcap, int32_t* status,
                         void* scratch, hipStream_t stream, unsigned long long* nbad,
                         bool pairs) {
  if (nmsg == 0) return hipSuccess;
  uint32_t* nlits = (uint32_t*)scratch;
  SnappyLit* lits = (SnappyLit*)((char*)scratch + 256);
  const uint64_t cap64 = nmsg * kAvgDef;
  const uint32_t cap = cap64 < 0xffffffffull ? (uint32_t)cap64 : 0xffffffffu;
  if (nlits) {
    const hipError_t e = hipMemsetAsync(nlits, 0, 4, stream);
    if (e != hipSuccess) return e;
  }
  // one wave per part, as many resident per CU as the LDS allows (the ring,
  // the window and the piece list): the parse is latency-bound per part, so
  // resident parts are the throughput
  constexpr uint64_t kLdsPerPart = kRing + kWin + 12ull * kMaxDef + 64;
  constexpr uint64_t kPerCU = 163840ull / kLdsPerPart > 0 ? 163840ull / kLdsPerPart : 1;
  const uint64_t grid_cap = 256ull * kPerCU;
  const uint64_t blocks = nmsg < grid_cap ? nmsg : grid_cap;
  if (PSG_SNAPPY_IR == 2 && nmsg <= kPrefetchParts)
    // few parts (a message's): the table form, one part per CU
    hipLaunchKernelGGL(snappy_tab_kernel, dim3((uint32_t)nmsg), dim3(256), 0, stream, src, soff,
                       dst, doff, dcap, nmsg, status, nlits ? lits : nullptr, nlits, cap, nbad,
                       pairs ? 1 : 0);
  else if (PSG_SNAPPY_IR && nmsg <= kPrefetchParts)
    // the streamed form alone (A/B builds: PSG_SNAPPY_IR=1)
    hipLaunchKernelGGL(snappy_ir_kernel, dim3((uint32_t)nmsg), dim3(64), 0, stream, src, soff, dst,
                       doff, dcap, nmsg, status, nlits ? lits : nullptr, nlits, cap, nbad,
                       pairs ? 1 : 0);
  else
    hipLaunchKernelGGL(snappy_kernel, dim3((uint32_t)blocks), dim3(64), 0, stream, src, soff, dst,
                       doff, dcap, nmsg, status, nlits ? lits : nullptr, nlits, cap, nbad,
                       pairs ? 1 : 0, nmsg <= kPrefetchParts ? PSG_SNAPPY_PREFETCH : 0);
  if (!nlits) return hipGetLastError();
  hipLaunchKernelGGL(snappy_lit_kernel, dim3(1024), dim3(256), 0, stream, lits, nlits, cap);
  return hipGetLastError();
}

}  // namespace psg
