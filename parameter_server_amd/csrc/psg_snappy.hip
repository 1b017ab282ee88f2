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
// sequential, so every lane parses the same tag (uniform loads from the
// scalar cache); the bytes of an element are moved by all 64 lanes.  The
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

__device__ __forceinline__ uint32_t ub(const uint8_t* p) { return *p; }

__global__ __launch_bounds__(64) void snappy_kernel(const uint8_t* __restrict__ src,
                                                    const uint64_t* __restrict__ soff,
                                                    uint8_t* __restrict__ dst,
                                                    const uint64_t* __restrict__ doff,
                                                    const uint64_t* __restrict__ dcap,
                                                    uint64_t nmsg, int32_t* __restrict__ status) {
  __shared__ uint8_t ring[kRing];
  const uint32_t lane = threadIdx.x;
  for (uint64_t msg = blockIdx.x; msg < nmsg; msg += gridDim.x) {
    const uint8_t* p = src + soff[msg];
    const uint8_t* const e = src + soff[msg + 1];
    uint8_t* const out = dst + doff[msg];
    const uint64_t cap = dcap ? dcap[msg] : doff[msg + 1] - doff[msg];
    int32_t st = 0;
    // preamble: uncompressed length, little-endian varint.  An empty part
    // is an empty array (uncompressFrom of 0 bytes clears, :233).
    if (p == e) {
      if (lane == 0) status[msg] = cap == 0 ? 0 : PSG_ERR_SIZE;
      continue;
    }
    uint64_t ulen = 0;
    bool done = false;
    int nb = 0;
    while (nb < 5 && p + nb < e && !done) {
      const uint32_t b = ub(p + nb);
      ulen |= (uint64_t)(b & 0x7f) << (7 * nb);
      done = !(b & 0x80);
      ++nb;
    }
    if (!done || ulen > 0xffffffffull) st = PSG_ERR_ARG;
    p += nb;
    if (!st && ulen != cap) st = PSG_ERR_SIZE;
    uint64_t o = 0;
    while (!st && p < e) {
      const uint32_t tag = ub(p++);
      uint32_t len, off = 0;
      if ((tag & 3u) == 0u) {  // literal
        len = (tag >> 2) + 1u;
        if (len > 60u) {
          const uint32_t n = len - 60u;
          if (p + n > e) { st = PSG_ERR_ARG; break; }
          len = 0;
          for (uint32_t b = 0; b < n; ++b) len |= ub(p + b) << (8 * b);
          len += 1u;
          p += n;
        }
        if (p + len > e || o + len > cap) { st = PSG_ERR_ARG; break; }
        for (uint32_t l = lane; l < len; l += 64) {
          const uint8_t b = p[l];
          ring[(o + l) & (kRing - 1)] = b;
          out[o + l] = b;
        }
        p += len;
        o += len;
        continue;
      }
      if ((tag & 3u) == 1u) {
        if (p + 1 > e) { st = PSG_ERR_ARG; break; }
        len = 4u + ((tag >> 2) & 7u);
        off = (tag >> 5) << 8 | ub(p);
        p += 1;
      } else if ((tag & 3u) == 2u) {
        if (p + 2 > e) { st = PSG_ERR_ARG; break; }
        len = 1u + (tag >> 2);
        off = ub(p) | ub(p + 1) << 8;
        p += 2;
      } else {
        if (p + 4 > e) { st = PSG_ERR_ARG; break; }
        len = 1u + (tag >> 2);
        off = ub(p) | ub(p + 1) << 8 | ub(p + 2) << 16 | ub(p + 3) << 24;
        p += 4;
      }
      if (off == 0 || off > o || o + len > cap) { st = PSG_ERR_ARG; break; }
      // len <= 64: one step; every source byte precedes o
      uint8_t b = 0;
      if (off <= kRing) {
        if (lane < len) b = ring[(o - off + lane % off) & (kRing - 1)];
      } else {
        __threadfence();  // this wave's earlier output stores, visible to its loads
        if (lane < len) b = out[o - off + lane % off];
      }
      if (lane < len) {
        ring[(o + lane) & (kRing - 1)] = b;
        out[o + lane] = b;
      }
      o += len;
    }
    if (!st && o != cap) st = PSG_ERR_ARG;
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
