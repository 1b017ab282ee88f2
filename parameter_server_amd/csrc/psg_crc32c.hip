// psg_crc32c.hip -- CRC-32C (Castagnoli) of byte segments resident in HBM:
// the key signature of the wire-ingress key cache.
//
// Reference: RNode::cacheKeySender / cacheKeyRecver (src/system/
// remote_node.cc:96-184) sign a message's key bytes with
// crc32c::Value(key.data(), min(key.size(), max_sig_len_ = 2048))
// (remote_node.cc:108,163; remote_node.h:96); crc32c::Extend
// (src/util/crc32c.cc:283-330) is LevelDB's slicing-by-4 table CRC with
// init/final inversion.  Known answers: src/test/crc32c_test.cc:13-65
// (RFC 3720 B.4).
//
// GPU form.  CRC is linear over GF(2): with raw(M) the CRC register after M
// from state 0 and no inversion,
//   raw(A || B) = raw(A) * x^(8|B|) mod P  XOR  raw(B),
//   Extend(init, M) = ~(raw(M) ^ (~init) * x^(8|M|) mod P).
// A wave takes chunks of up to kChunk bytes of one segment; lane l reads
// the 16-byte blocks at l*16 + i*1024 (coalesced 1 KB per wave load) and
// folds them Horner-style: its register is advanced over the 1008 bytes
// between two of its blocks by one linear map (4 table lookups), then over
// its next block by slicing-by-16 (16 lookups).  At the end each lane's
// register is shifted over the bytes after its last block and the 64
// registers are XOR-reduced.  A segment longer than one chunk is the XOR of
// its chunks' partials, each shifted over the bytes after it
// (square-and-multiply by x^(8*2^k)), accumulated with atomic XOR.
// All tables are built at compile time (constexpr) and staged into LDS once
// per workgroup; waves then loop over chunk items (grid-stride).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_internal.h"

namespace psg {

namespace {

constexpr uint32_t kPoly = 0x82f63b78u;  // reflected Castagnoli polynomial
constexpr uint32_t kChunk = 65536;       // bytes per wave item
constexpr int kNT = 256;

// a * b mod P, both reflected (bit 31 = x^0)
constexpr __host__ __device__ uint32_t mulmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

struct Tables {
  uint32_t t[16][256];  // t[k][b]: byte b followed by k zero bytes
  uint32_t sh[4][256];  // c -> c * x^(8*1008): byte j of c
  uint32_t x8[1024];    // x^(8d) mod P, d < 1024
  uint32_t p2[64];      // x^(8 * 2^k) mod P
};

constexpr Tables make_tables() {
  Tables T{};
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int i = 0; i < 8; ++i) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
    T.t[0][b] = c;
  }
  for (int k = 1; k < 16; ++k)
    for (int b = 0; b < 256; ++b)
      T.t[k][b] = (T.t[k - 1][b] >> 8) ^ T.t[0][T.t[k - 1][b] & 0xffu];
  uint32_t x = 1u << 31;  // x^0
  for (int d = 0; d < 1024; ++d) {
    T.x8[d] = x;
    for (int i = 0; i < 8; ++i) x = (x & 1u) ? (x >> 1) ^ kPoly : x >> 1;
  }
  const uint32_t k1008 = T.x8[1008];
  for (int j = 0; j < 4; ++j)
    for (uint32_t b = 0; b < 256; ++b) T.sh[j][b] = mulmodp(k1008, b << (8 * j));
  uint32_t q = T.x8[1];  // x^8
  for (int k = 0; k < 64; ++k) {
    T.p2[k] = q;
    q = mulmodp(q, q);
  }
  return T;
}

__constant__ const Tables kTab = make_tables();

// c * x^(8n) mod P for any n (square-and-multiply over kTab.p2)
__device__ uint32_t shift_bytes(uint32_t c, uint64_t n) {
  for (int k = 0; n; ++k, n >>= 1)
    if (n & 1u) c = mulmodp(kTab.p2[k], c);
  return c;
}

// raw CRC (state 0, no inversion) of one chunk of <= kChunk bytes, the
// whole wave (every lane gets the result)
__device__ __forceinline__ uint32_t chunk_raw(const uint8_t* p, uint32_t clen, uint32_t lane,
                                              const uint32_t (*t)[256], const uint32_t (*sh)[256],
                                              const uint32_t* x8) {
  const bool a16 = ((uintptr_t)p & 15u) == 0;
  uint32_t r = 0;     // this lane's register
  uint32_t last = 0;  // end of this lane's last block (0: none)
  for (uint32_t base = 0; base < clen; base += 1024u) {
    const uint32_t bs = base + lane * 16u;
    if (bs >= clen) break;  // this lane has no block here (nor later)
    // advance over the 1008 bytes since this lane's previous block
    if (base)
      r = sh[0][r & 255u] ^ sh[1][(r >> 8) & 255u] ^ sh[2][(r >> 16) & 255u] ^ sh[3][r >> 24];
    const uint32_t bl = clen - bs < 16u ? clen - bs : 16u;
    if (bl == 16u) {
      uint32_t w0, w1, w2, w3;
      if (a16) {
        const uint4 v = *(const uint4*)(p + bs);
        w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w;
      } else {
        const uint8_t* q = p + bs;
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          w[j] = (uint32_t)q[4 * j] | (uint32_t)q[4 * j + 1] << 8 |
                 (uint32_t)q[4 * j + 2] << 16 | (uint32_t)q[4 * j + 3] << 24;
        w0 = w[0]; w1 = w[1]; w2 = w[2]; w3 = w[3];
      }
      w0 ^= r;
      r = t[15][w0 & 255u] ^ t[14][(w0 >> 8) & 255u] ^ t[13][(w0 >> 16) & 255u] ^ t[12][w0 >> 24] ^
          t[11][w1 & 255u] ^ t[10][(w1 >> 8) & 255u] ^ t[9][(w1 >> 16) & 255u] ^ t[8][w1 >> 24] ^
          t[7][w2 & 255u] ^ t[6][(w2 >> 8) & 255u] ^ t[5][(w2 >> 16) & 255u] ^ t[4][w2 >> 24] ^
          t[3][w3 & 255u] ^ t[2][(w3 >> 8) & 255u] ^ t[1][(w3 >> 16) & 255u] ^ t[0][w3 >> 24];
    } else {  // the segment's last, partial block
      for (uint32_t j = 0; j < bl; ++j) r = t[0][(r ^ p[bs + j]) & 255u] ^ (r >> 8);
    }
    last = bs + bl;
  }
  // shift over the bytes after this lane's last block (< 1024), reduce
  uint32_t v = last ? mulmodp(x8[clen - last], r) : 0u;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d, 64);
  return v;
}

__global__ __launch_bounds__(kNT) void crc_kernel(const uint8_t* __restrict__ data,
                                                  const uint64_t* __restrict__ off,
                                                  uint64_t nseg, uint64_t max_len,
                                                  uint64_t per_seg,
                                                  const uint32_t* __restrict__ init,
                                                  uint32_t* __restrict__ out) {
  __shared__ uint32_t t[16][256];
  __shared__ uint32_t sh[4][256];
  __shared__ uint32_t x8[1024];
  for (int i = threadIdx.x; i < 16 * 256; i += kNT) (&t[0][0])[i] = (&kTab.t[0][0])[i];
  for (int i = threadIdx.x; i < 4 * 256; i += kNT) (&sh[0][0])[i] = (&kTab.sh[0][0])[i];
  for (int i = threadIdx.x; i < 1024; i += kNT) x8[i] = kTab.x8[i];
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nitems = nseg * per_seg;
  const uint64_t wstride = (uint64_t)gridDim.x * (kNT / 64);
  for (uint64_t it = (uint64_t)blockIdx.x * (kNT / 64) + (threadIdx.x >> 6); it < nitems;
       it += wstride) {
    // item (s, c): chunks c, c + per_seg, ... of segment s
    const uint64_t s = it / per_seg, c = it - s * per_seg;
    const uint64_t b0 = off[s];
    uint64_t len = off[s + 1] - b0;
    len = len < max_len ? len : max_len;
    if (c * kChunk >= len && !(c == 0 && len == 0)) continue;
    uint32_t acc = 0;  // this item's chunks, each shifted to the segment's end
    for (uint64_t cb = c * kChunk; cb < len; cb += per_seg * kChunk) {
      const uint32_t clen = (uint32_t)(len - cb < kChunk ? len - cb : kChunk);
      acc ^= shift_bytes(chunk_raw(data + b0 + cb, clen, lane, t, sh, x8), len - cb - clen);
    }
    if (lane == 0) {
      // ~(raw ^ (~init) x^(8 len)): the init term and the final inversion
      // (both linear) are added once, by chunk 0's item
      if (c == 0) acc ^= ~shift_bytes(~(init ? init[s] : 0u), len);
      if (per_seg == 1)
        out[s] = acc;
      else
        __hip_atomic_fetch_xor(out + s, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// the key signature check of a message that carries keys (cacheKeyRecver,
// remote_node.cc:161-163): crc32c::Value of the first min(len, max) bytes
// against the carried signature; a mismatch counts into *bad (reported by
// psg_received), so the host does not wait for it.  One wave.
__global__ __launch_bounds__(64) void sig_kernel(const uint8_t* __restrict__ data, uint32_t len,
                                                 uint32_t want, unsigned long long* bad,
                                                 unsigned long long* bad2) {
  __shared__ uint32_t t[16][256];
  __shared__ uint32_t sh[4][256];
  __shared__ uint32_t x8[1024];
  for (int i = threadIdx.x; i < 16 * 256; i += 64) (&t[0][0])[i] = (&kTab.t[0][0])[i];
  for (int i = threadIdx.x; i < 4 * 256; i += 64) (&sh[0][0])[i] = (&kTab.sh[0][0])[i];
  for (int i = threadIdx.x; i < 1024; i += 64) x8[i] = kTab.x8[i];
  __syncthreads();
  const uint32_t raw = chunk_raw(data, len, threadIdx.x, t, sh, x8);
  const uint32_t got = raw ^ ~shift_bytes(~0u, len);  // Extend(0, data, len)
  if (threadIdx.x == 0 && got != want) {
    atomicAdd(bad, 1ull);
    if (bad2) atomicAdd(bad2, 1ull);
  }
}

}  // namespace

hipError_t launch_sig_check(const uint8_t* data, uint64_t len, uint64_t max_len, uint32_t want,
                            unsigned long long* bad, hipStream_t s, unsigned long long* bad2) {
  const uint64_t l = len < max_len ? len : max_len;
  if (l > kChunk) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sig_kernel, dim3(1), dim3(64), 0, s, data, (uint32_t)l, want, bad, bad2);
  return hipGetLastError();
}

// items per segment: one per 64 KB chunk up to kMaxPer (an item then takes
// every kMaxPer-th chunk), so any max_len gives a bounded grid
uint64_t crc32c_chunks_per_segment(uint64_t max_len) {
  constexpr uint64_t kMaxPer = 4096;
  const uint64_t c = max_len <= kChunk ? 1 : (max_len - 1) / kChunk + 1;
  return c < kMaxPer ? c : kMaxPer;
}

hipError_t launch_crc32c(const uint8_t* data, const uint64_t* off, uint64_t nseg,
                         uint64_t max_len, const uint32_t* init, uint32_t* out,
                         hipStream_t s) {
  if (nseg == 0) return hipSuccess;
  const uint64_t per = crc32c_chunks_per_segment(max_len);
  if (per > 1) {
    hipError_t e = hipMemsetAsync(out, 0, 4 * nseg, s);
    if (e != hipSuccess) return e;
  }
  const uint64_t waves = nseg * per;
  uint64_t blocks = (waves + kNT / 64 - 1) / (kNT / 64);
  // persistent grid: the 24 KB of tables are staged once per workgroup
  blocks = blocks < 2048 ? blocks : 2048;
  hipLaunchKernelGGL(crc_kernel, dim3((uint32_t)blocks), dim3(kNT), 0, s, data, off, nseg,
                     max_len, per, init, out);
  return hipGetLastError();
}

}  // namespace psg
