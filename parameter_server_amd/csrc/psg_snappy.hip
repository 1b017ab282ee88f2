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
// last 64 KB of output live in an LDS ring: a copy reads its source bytes
// there.  A copy's source is output[o - off + (l mod off)] for byte l, which
// lies before o for every l, so even overlapping (run-length) copies move in
// one step; copies are <= 64 bytes, so the step's reads precede its writes.
// Offsets beyond the ring (possible only for 4-byte-offset copies, which
// snappy's own compressor never emits across its 64 KB blocks) read the
// output in global memory after a fence.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/psg.h"
#include "psg_internal.h"

namespace psg {

namespace {

constexpr uint32_t kRing = 65536;
constexpr uint32_t kWin = 4096;
constexpr uint32_t kFlush = 4096;  // output burst size  // LDS window over the compressed stream (tags, offsets)

__global__ __launch_bounds__(64) void snappy_kernel(const uint8_t* __restrict__ src,
                                                    const uint64_t* __restrict__ soff,
                                                    uint8_t* __restrict__ dst,
                                                    const uint64_t* __restrict__ doff,
                                                    const uint64_t* __restrict__ dcap,
                                                    uint64_t nmsg, int32_t* __restrict__ status) {
  __shared__ uint8_t ring[kRing];
  __shared__ __attribute__((aligned(4))) uint8_t win[kWin];
  const uint32_t lane = threadIdx.x;
  for (uint64_t msg = blockIdx.x; msg < nmsg; msg += gridDim.x) {
    const uint8_t* const s0 = src + soff[msg];
    const uint64_t slen = soff[msg + 1] - soff[msg];
    uint8_t* const out = dst + doff[msg];
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
    // the element stream is read from an LDS window (4 KB, refilled with
    // coalesced 4-byte loads), and from it into a 64-byte register
    // lookahead (lane j holds byte lp + j) whose bytes the parse takes with
    // a scalar readlane: one LDS read serves several tags
    const uintptr_t mis = (uintptr_t)s0 & 3u;
    int32_t wb = -(int32_t)kWin - 64;  // part offset of win[0]; nothing loaded
    auto refill = [&](uint32_t q) {
      wb = (int32_t)((q + mis) & ~3u) - (int32_t)mis;  // 4-byte aligned in memory
      for (uint32_t o4 = lane * 4u; o4 < kWin; o4 += 256u) {
        const int64_t g = (int64_t)wb + o4;
        uint32_t v = 0;
        if (g >= 0 && g + 4 <= (int64_t)e) {
          v = *(const uint32_t*)(s0 + g);
        } else {
          for (uint32_t b = 0; b < 4; ++b)
            if (g + b >= 0 && g + b < (int64_t)e) v |= (uint32_t)s0[g + b] << (8 * b);
        }
        *(uint32_t*)&win[o4] = v;
      }
      __builtin_amdgcn_wave_barrier();
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
    // output bytes [fl, o) live only in the ring; they reach global memory
    // in kFlush-sized bursts, so the element loop issues no global stores
    // (on gfx9 a store holds vmcnt, which the next dependent wait drains)
    uint32_t fl = 0;
    auto flush = [&](uint32_t to) {
      __builtin_amdgcn_wave_barrier();
      for (uint32_t x = fl + lane; x < to; x += 64) out[x] = ring[x & (kRing - 1)];
      fl = to;
    };
    while (!st && p < e) {
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
        if ((int32_t)p >= wb && (int64_t)p + len <= (int64_t)wb + kWin) {
          const uint32_t w0 = (uint32_t)((int32_t)p - wb);
          for (uint32_t l = lane; l < len; l += 64) ring[(o + l) & (kRing - 1)] = win[w0 + l];
        } else {
          for (uint32_t c = 0; c < len; c += 64) {  // wave-uniform steps
            if (o + c - fl >= kRing - kFlush) flush(o + c);  // a long literal
            if (c + lane < len) ring[(o + c + lane) & (kRing - 1)] = s0[p + c + lane];
          }
        }
        p += len;
        o += len;
        if (o - fl >= kFlush) flush(o);
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
      if (off <= kRing) {
        if (lane < len) ring[(o + lane) & (kRing - 1)] = ring[(o - off + li) & (kRing - 1)];
      } else {
        // the source was flushed: read it back after this wave's stores land
        flush(o);
        __threadfence();
        if (lane < len) ring[(o + lane) & (kRing - 1)] = out[o - off + li];
      }
      o += len;
      if (o - fl >= kFlush) flush(o);
    }
    if (!st && o != ucap) st = PSG_ERR_ARG;
    if (!st) flush(o);
    if (lane == 0) status[msg] = st;
  }
}

}  // namespace

hipError_t launch_snappy(const uint8_t* src, const uint64_t* soff, uint64_t nmsg, uint8_t* dst,
                         const uint64_t* doff, const uint64_t* dcap, int32_t* status,
                         hipStream_t stream) {
  if (nmsg == 0) return hipSuccess;
  // 64 KB of LDS per workgroup: two resident per CU
  const uint64_t blocks = nmsg < 512 ? nmsg : 512;
  hipLaunchKernelGGL(snappy_kernel, dim3((uint32_t)blocks), dim3(64), 0, stream, src, soff, dst,
                     doff, dcap, nmsg, status);
  return hipGetLastError();
}

}  // namespace psg
