// psg_countmin.hip -- the server's tail-feature filter on the device:
// FreqencyFilter<uint64>::insertKeys / queryKeys
// (src/parameter/frequency_filter.h:27-43) over CountMin<uint64, uint8>
// (src/base/countmin.h:14-67), called from SharedParameter::process for
// insert_key_freq / query_key_freq tasks (shared_parameter.h:114-133).
//
// CountMin<K, uint8>: n_ byte counters, k_ probes per key; probe j of key x
// is data_[h_j % n_] with h_0 = hash(x), h_{j+1} = h_j + rotr(h_0, 17)
// (uint32 wrap).  insert adds (uint8)count to each probe (byte wrap);
// query = min over probes, starting from 255; queryKeys keeps, in input
// order, the keys whose query is > freqency.
//
// Insert, binned (the default when the filter's scratch holds the records):
// the table is cut into 32 KB regions.  A bin pass gives each block of KB
// keys one workgroup: it reads the keys and counts once, counts their probes
// per region in LDS, lays the probes out region-sorted in LDS as 4-byte
// records (offset in the region, count) and writes them as one contiguous
// run per block, with the block's region starts (u16; transposed to
// region-major by a small pass).  An apply pass gives each region one
// workgroup that adds the records of every block's run for the region into
// u32 LDS counters (native LDS adds: a counter's low byte is its sum mod 2^8)
// and then adds those sums into the region's bytes -- each table byte is
// read and written once, the keys are read once, and there are no global
// atomics per probe (the CAS form below makes one device-scope atomic per
// probe, the bound of its rate).  r04's form counted, reserved and
// scattered in three passes over the keys (1.65 GB per 16.8 M-key insert).
//
// GPU form.  The table is the reference's: n_ bytes (countmin.h:69,
// SArray<uint8>), 64 MB for 2^26 counters, so it stays resident in the
// 256 MB Infinity Cache while keys stream past.  There is no byte-wide
// global atomic, and a 32-bit add would carry out of the byte: a probe is a
// compare-and-swap of the aligned dword that holds its byte, the byte
// replaced by (byte + count) mod 2^8 and the other three kept.  A key's k
// probes are independent: their dword loads go out together, then rounds of
// CAS over the probes still pending (a failed CAS returns the current word,
// the next round retries with it).  Addition mod 2^8 does not depend on
// order, so any interleaving of inserts gives the reference's table
// byte for byte.
//
// Query, binned (queryKeys over many keys): a probe read straight from the
// table pulls a whole line for one byte, and the table (64 MB) is 16 times an
// XCD's L2, so every probe misses it (26.7 x the algorithmic bytes measured
// in r04).  The binned form moves the probes to the table instead:
//   bin    one workgroup per block of KB keys: each key's k probes are
//          counted per 128 KB table region, laid out region-sorted in LDS and
//          written out as one contiguous run per block (4-byte records:
//          offset in the region, key index in the block), with the block's
//          region starts (u16);
//   look   one workgroup per region: the region's 128 KB of table into LDS
//          (read once), then every block's run of records for the region;
//          each record becomes a 2-byte result (key index, probe <= freq) at
//          the same position;
//   keep   one workgroup per block: a key is dropped iff one of its probes
//          is <= freq (min over the probes > freq <=> every probe > freq);
//          the keep bits and per-tile counts the compaction below reads.
// Then, as in the direct form, the order-preserving compaction: one scan of
// the tile counts and a scatter of the kept keys.  Bytes per key: keys read
// twice (16 B), records 12 k B (written, read; results written, read), plus
// the table once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "psg_device.h"
#include "psg_internal.h"

namespace psg {

namespace {

constexpr int kNT = 256;
constexpr int kIPT = 8;                 // keys per thread in the query passes
constexpr int kQTile = kNT * kIPT;      // keys per workgroup

// CountMin::hash (countmin.h:53-64)
__device__ __forceinline__ uint32_t cm_hash(uint64_t key) {
  const uint32_t seed = 0xbc9f1d34u, m = 0xc6a4a793u, n = 8;
  uint32_t h = seed ^ (n * m);
  uint32_t w = (uint32_t)key;
  h += w;
  h *= m;
  h ^= (h >> 16);
  w = (uint32_t)(key >> 32);
  h += w;
  h *= m;
  h ^= (h >> 16);
  return h;
}

__device__ __forceinline__ uint32_t cm_query(const uint8_t* __restrict__ t, uint32_t n, int k,
                                             uint64_t key) {
  uint32_t res = 255u;  // (uint8)kuint64max
  uint32_t h = cm_hash(key);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int j = 0; j < k; ++j) {
    const uint32_t v = t[h % n];
    res = v < res ? v : res;
    h += delta;
  }
  return res;
}

constexpr int kProbeRegs = 8;  // probes held in registers (k <= 8: every app's k)

// ---- binned insert ----
constexpr uint32_t kRegShift = 15;                 // 32 KB of table per region
constexpr uint32_t kRegBytes = 1u << kRegShift;
constexpr uint32_t kMaxRegions = 4096;             // tables up to 128 MB binned

// probes of key i (count c != 0) -> fn(region, offset in region, c)
template <typename F>
__device__ __forceinline__ void probes(uint64_t key, uint32_t n, int k, F fn) {
  uint32_t h = cm_hash(key);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int j = 0; j < k; ++j) {
    const uint32_t idx = h % n;
    fn(idx >> kRegShift, idx & (kRegBytes - 1u));
    h += delta;
  }
}

constexpr int kBlkNT = 1024;
constexpr uint32_t kBlkRecs = 32768;               // records per block (LDS: 128 KB)

// keys per insert block: a power of two with KB * k <= kBlkRecs
__host__ __device__ constexpr uint32_t ins_block_keys(int k) {
  return k <= 4 ? 8192u : k <= 8 ? 4096u : k <= 16 ? 2048u : 1024u;
}

// XCD-contiguous runs of consecutive indices (blocks b and b + 8 share an
// XCD: observed dispatch, speed only): neighbouring regions' record runs
// share lines, read once per XCD this way
__device__ __forceinline__ uint32_t xcd_index(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + j;
}

// bin: block b's keys [b*KB, ...): their probes' records (offset | count
// << 15) region-sorted at R[b*KB*k ...), region starts S[b*(nreg+1) + r]
__global__ __launch_bounds__(kBlkNT) void cm_ibin_kernel(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ counts,
                                                         uint64_t nk, uint32_t n, int k,
                                                         uint32_t kb, uint32_t nreg,
                                                         uint16_t* __restrict__ S,
                                                         uint32_t* __restrict__ R) {
  __shared__ uint32_t stg[kBlkRecs];
  __shared__ uint32_t cur[kMaxRegions + 1];
  __shared__ uint32_t ws[kBlkNT / 64];
  const uint32_t t = threadIdx.x, b = blockIdx.x;
  const uint64_t k0 = (uint64_t)b * kb;
  const uint32_t nkb = (uint32_t)(nk - k0 < kb ? nk - k0 : kb);
  constexpr int kKPT = 8192 / kBlkNT;
  uint64_t key[kKPT];
  uint32_t cnt[kKPT];
#pragma unroll
  for (int i = 0; i < kKPT; ++i) {
    const uint32_t x = t + (uint32_t)i * kBlkNT;
    key[i] = x < nkb ? keys[k0 + x] : 0ull;
    cnt[i] = x < nkb ? counts[k0 + x] & 0xffu : 0u;  // insert(key, (uint8)count)
  }
  for (uint32_t r = t; r <= nreg; r += kBlkNT) cur[r] = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kKPT; ++i)
    if (cnt[i]) probes(key[i], n, k, [&](uint32_t r, uint32_t) { atomicAdd(&cur[r], 1u); });
  __syncthreads();
  // exclusive scan over the regions, 4 per thread (nreg <= 4 * kBlkNT)
  {
    uint32_t v[4], tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t r = 4 * t + j;
      v[j] = r < nreg ? cur[r] : 0u;
      tot += v[j];
    }
    uint32_t all;
    uint32_t ex = dev::block_excl_scan<kBlkNT>(tot, ws, &all);
    __syncthreads();
    uint16_t* Sb = S + (size_t)b * (nreg + 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t r = 4 * t + j;
      if (r < nreg) {
        cur[r] = ex;
        Sb[r] = (uint16_t)ex;
      }
      ex += v[j];
    }
    if (t == 0) Sb[nreg] = (uint16_t)all;  // <= KB * k <= 32768
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kKPT; ++i) {
    const uint32_t c = cnt[i];
    if (c)
      probes(key[i], n, k, [&](uint32_t r, uint32_t o) {
        stg[atomicAdd(&cur[r], 1u)] = o | c << kRegShift;
      });
  }
  __syncthreads();
  const uint32_t nrec = cur[nreg - 1];  // the last region's end = the block's records
  uint32_t* o = R + (size_t)b * kb * (uint32_t)k;
  for (uint32_t i = t; i < nrec; i += kBlkNT) o[i] = stg[i];
}

// S [nb][nreg + 1] -> ST [nreg + 1][nb] (64 x 64 tiles through LDS)
__global__ __launch_bounds__(256) void cm_transpose_kernel(const uint16_t* __restrict__ S,
                                                           uint32_t nb, uint32_t nc,
                                                           uint16_t* __restrict__ ST) {
  __shared__ uint16_t tl[64][65];
  const uint32_t c0 = blockIdx.x * 64u, b0 = blockIdx.y * 64u;
  const uint32_t tx = threadIdx.x & 63u, ty = threadIdx.x >> 6;
  for (uint32_t y = ty; y < 64u; y += 4u)
    if (b0 + y < nb && c0 + tx < nc) tl[y][tx] = S[(size_t)(b0 + y) * nc + c0 + tx];
  __syncthreads();
  for (uint32_t y = ty; y < 64u; y += 4u)
    if (c0 + y < nc && b0 + tx < nb) ST[(size_t)(c0 + y) * nb + b0 + tx] = tl[tx][y];
}

// apply: one workgroup per region (XCD-contiguous): every block's run of
// records for the region into u32 LDS sums, then the region's bytes += sum
// (mod 2^8); bytes past the table untouched.  A wave takes 64 blocks at a
// time: their runs' lengths scanned across the lanes, then the lanes walk
// the concatenated records (a 6-step LDS search finds each one's block)
__global__ __launch_bounds__(kBlkNT) void cm_iapply_kernel(uint8_t* __restrict__ t,
                                                           uint32_t tbytes, uint32_t nb,
                                                           uint32_t nreg, uint32_t rb,
                                                           const uint16_t* __restrict__ ST,
                                                           const uint32_t* __restrict__ R) {
  __shared__ uint32_t acc[kRegBytes];
  __shared__ uint32_t wpre[kBlkNT / 64][65];
  __shared__ uint32_t wst[kBlkNT / 64][64];
  const uint32_t r = xcd_index(blockIdx.x, gridDim.x);
  const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
  for (uint32_t i = tid; i < kRegBytes; i += kBlkNT) acc[i] = 0;
  __syncthreads();
  const uint16_t* s0 = ST + (size_t)r * nb;
  const uint16_t* s1 = ST + (size_t)(r + 1) * nb;
  for (uint32_t b0 = w * 64u; b0 < nb; b0 += kBlkNT) {
    const uint32_t bb = b0 + lane;
    const uint32_t a = bb < nb ? s0[bb] : 0u, e = bb < nb ? s1[bb] : 0u;
    uint32_t x = e - a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
      if ((int)lane >= d) x += y;
    }
    const uint32_t tot = (uint32_t)__shfl((int)x, 63, 64);
    wpre[w][lane + 1] = x;
    if (lane == 0) wpre[w][0] = 0;
    wst[w][lane] = bb * rb + a;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // kApU records per lane in flight: their loads issued together, then
    // their adds (one record at a time waited ~a memory trip per 64)
    constexpr int kApU = 8;
    for (uint32_t i0 = lane; i0 < tot; i0 += 64u * kApU) {
      uint32_t v[kApU];
#pragma unroll
      for (int q = 0; q < kApU; ++q) {
        const uint32_t i = i0 + 64u * q;
        v[q] = 0xffffffffu;
        if (i < tot) {
          uint32_t u = 0;
#pragma unroll
          for (uint32_t st = 32; st > 0; st >>= 1)
            if (wpre[w][u + st] <= i) u += st;
          v[q] = R[wst[w][u] + (i - wpre[w][u])];
        }
      }
#pragma unroll
      for (int q = 0; q < kApU; ++q)
        if (i0 + 64u * q < tot)
          __hip_atomic_fetch_add(&acc[v[q] & (kRegBytes - 1u)], v[q] >> kRegShift,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __syncthreads();
  // dwords of the region (the table is a whole number of dwords)
  uint32_t* tw = (uint32_t*)(t + (size_t)r * kRegBytes);
  const uint32_t nw = (tbytes - r * kRegBytes < kRegBytes ? tbytes - r * kRegBytes : kRegBytes) / 4u;
  for (uint32_t i = tid; i < nw; i += kBlkNT) {
    const uint32_t wd = tw[i];
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o |= ((((wd >> (8 * j)) & 0xffu) + acc[4 * i + j]) & 0xffu) << (8 * j);
    tw[i] = o;
  }
}

__device__ __forceinline__ uint32_t byte_add(uint32_t w, uint32_t sh, uint32_t c) {
  const uint32_t nb = ((w >> sh) + c) & 0xffu;
  return (w & ~(0xffu << sh)) | (nb << sh);
}

__global__ __launch_bounds__(kNT) void cm_insert_kernel(const uint64_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ counts,
                                                        uint64_t nk, uint8_t* __restrict__ t,
                                                        uint32_t n, int k) {
  const uint64_t i = (uint64_t)blockIdx.x * kNT + threadIdx.x;
  if (i >= nk) return;
  const uint32_t c = counts[i] & 0xffu;  // insert(key, (uint8)count)
  if (!c) return;
  uint32_t h = cm_hash(keys[i]);
  const uint32_t delta = (h >> 17) | (h << 15);
  if (k <= kProbeRegs) {
    uint32_t* wp[kProbeRegs];
    uint32_t sh[kProbeRegs], old[kProbeRegs];
#pragma unroll
    for (int j = 0; j < kProbeRegs; ++j) {
      if (j < k) {
        const uint32_t idx = h % n;
        wp[j] = (uint32_t*)(t + (idx & ~3u));
        sh[j] = 8u * (idx & 3u);
        old[j] = __hip_atomic_load(wp[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h += delta;
      }
    }
    uint32_t pend = (1u << k) - 1u;
    while (pend) {
#pragma unroll
      for (int j = 0; j < kProbeRegs; ++j) {
        if ((pend >> j) & 1u) {
          const uint32_t seen = atomicCAS(wp[j], old[j], byte_add(old[j], sh[j], c));
          if (seen == old[j]) pend &= ~(1u << j);
          else old[j] = seen;
        }
      }
    }
    return;
  }
  for (int j = 0; j < k; ++j) {
    const uint32_t idx = h % n;
    uint32_t* w = (uint32_t*)(t + (idx & ~3u));
    const uint32_t s8 = 8u * (idx & 3u);
    uint32_t o = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      const uint32_t seen = atomicCAS(w, o, byte_add(o, s8, c));
      if (seen == o) break;
      o = seen;
    }
    h += delta;
  }
}

// pass 1: the query of every key (each probe a random 4-byte read of the
// table: the cost of queryKeys), its keep bit, and the keys kept per
// workgroup tile.  Thread-contiguous runs of kIPT keys, so the bits are in
// input order; pass 3 reads the bits instead of querying the table again.
__global__ __launch_bounds__(kNT) void cm_count_kernel(const uint64_t* __restrict__ keys,
                                                       uint64_t nk, const uint8_t* __restrict__ t,
                                                       uint32_t n, int k, int freq,
                                                       uint32_t* __restrict__ tile_cnt,
                                                       uint8_t* __restrict__ keep_bits) {
  __shared__ uint32_t ws[kNT / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kQTile + (uint64_t)threadIdx.x * kIPT;
  uint32_t keep = 0;
#pragma unroll
  for (int r = 0; r < kIPT; ++r) {
    const uint64_t i = base + r;
    if (i < nk && (int)cm_query(t, n, k, keys[i]) > freq) keep |= 1u << r;
  }
  keep_bits[(uint64_t)blockIdx.x * kNT + threadIdx.x] = (uint8_t)keep;
  uint32_t c = (uint32_t)__popc(keep);
  for (int s = 32; s >= 1; s >>= 1) c += (uint32_t)__shfl_xor((int)c, s, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int w = 0; w < kNT / 64; ++w) tot += ws[w];
    tile_cnt[blockIdx.x] = tot;
  }
}

// pass 2: exclusive scan of the tile counts (one workgroup, sequential chunks)
__global__ __launch_bounds__(kNT) void cm_scan_kernel(uint32_t* __restrict__ tile_cnt,
                                                      uint32_t ntiles,
                                                      unsigned long long* __restrict__ total) {
  __shared__ uint32_t ws[kNT / 64];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < ntiles; b += kNT) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? tile_cnt[i] : 0u;
    uint32_t tot;
    const uint32_t ex = dev::block_excl_scan<kNT>(v, ws, &tot);
    const uint32_t c0 = carry;
    if (i < ntiles) tile_cnt[i] = c0 + ex;
    __syncthreads();
    if (threadIdx.x == 0) carry = c0 + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// pass 3: scatter the kept keys in input order (from pass 1's bits)
__global__ __launch_bounds__(kNT) void cm_scatter_kernel(const uint64_t* __restrict__ keys,
                                                         uint64_t nk,
                                                         const uint8_t* __restrict__ keep_bits,
                                                         const uint32_t* __restrict__ tile_off,
                                                         uint64_t* __restrict__ out) {
  __shared__ uint32_t ws[kNT / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kQTile + (uint64_t)threadIdx.x * kIPT;
  const uint32_t keep = keep_bits[(uint64_t)blockIdx.x * kNT + threadIdx.x];
  uint32_t tot;
  uint32_t pos = tile_off[blockIdx.x] + dev::block_excl_scan<kNT>(__popc(keep), ws, &tot);
#pragma unroll
  for (int r = 0; r < kIPT; ++r)
    if (((keep >> r) & 1u) && base + r < nk) out[pos++] = keys[base + r];
}

// ---- binned query (see the header) ----
constexpr uint32_t kQRegShift = 17;                  // 128 KB of table per region
constexpr uint32_t kQRegBytes = 1u << kQRegShift;
constexpr uint32_t kQMaxReg = 1024;                  // tables up to 128 MB binned
constexpr int kQMaxK = 8;                            // probes per key (every app's k)
constexpr int kQNT = 1024;
constexpr uint32_t kQMaxRecs = 32768;                // records per block (LDS: 128 KB)
constexpr uint32_t kQMaxBlocks = 4096;               // blocks per chunk (their starts in LDS)
constexpr uint64_t kQChunkKeys = 8ull << 20;         // keys per chunk at k = 8

// keys per block: a power of two, at most 8192 (13-bit key index in a
// result), with KB * k <= kQMaxRecs; a multiple of the compaction tile
__host__ __device__ constexpr uint32_t q_block_keys(int k) {
  return k <= 4 ? 8192u : 4096u;
}
// record slots of the scratch: whole blocks of the largest k
inline uint64_t q_record_cap(uint64_t nk) {
  const uint64_t keys = nk < kQChunkKeys ? nk : kQChunkKeys;
  const uint64_t r = keys * (uint64_t)kQMaxK;
  return (r + kQMaxRecs - 1) / kQMaxRecs * kQMaxRecs;
}
// region starts: (kQMaxReg + 1) u16 per block, for as many blocks as fit rcap
inline uint64_t q_starts_bytes(uint64_t rcap) {
  const uint64_t nb = std::min<uint64_t>(rcap / 8192u + 1, kQMaxBlocks);
  return (nb * (kQMaxReg + 1) * 2 + 255) / 256 * 256;
}
static_assert(kQTile == 2048 && q_block_keys(8) % kQTile == 0, "blocks of whole tiles");

// bin: block b's keys [b*KB, ...) of this chunk; their probes' records
// region-sorted at R1[b*KB*k ...), region starts S[b*(nreg+1) + r]
__global__ __launch_bounds__(kQNT) void cm_qbin_kernel(const uint64_t* __restrict__ keys,
                                                       uint64_t nk, uint32_t n, int k,
                                                       uint32_t kb, uint32_t nreg,
                                                       uint16_t* __restrict__ S,
                                                       uint32_t* __restrict__ R1) {
  __shared__ uint32_t stg[kQMaxRecs];
  __shared__ uint32_t cur[kQMaxReg + 1];
  __shared__ uint32_t ws[kQNT / 64];
  const uint32_t t = threadIdx.x, b = blockIdx.x;
  const uint64_t k0 = (uint64_t)b * kb;
  const uint32_t nkb = (uint32_t)(nk - k0 < kb ? nk - k0 : kb);
  constexpr int kKPT = 8192 / kQNT;  // keys per thread (at most)
  uint64_t key[kKPT];
#pragma unroll
  for (int i = 0; i < kKPT; ++i) {
    const uint32_t x = t + (uint32_t)i * kQNT;
    key[i] = x < nkb ? keys[k0 + x] : 0ull;
  }
  for (uint32_t r = t; r <= nreg; r += kQNT) cur[r] = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kKPT; ++i) {
    const uint32_t x = t + (uint32_t)i * kQNT;
    if (x < nkb) {
      uint32_t h = cm_hash(key[i]);
      const uint32_t delta = (h >> 17) | (h << 15);
      for (int j = 0; j < k; ++j) {
        atomicAdd(&cur[(h % n) >> kQRegShift], 1u);
        h += delta;
      }
    }
  }
  __syncthreads();
  // exclusive scan over the regions (one per thread: nreg <= kQNT)
  {
    const uint32_t v = t < nreg ? cur[t] : 0u;
    uint32_t tot;
    const uint32_t ex = dev::block_excl_scan<kQNT>(v, ws, &tot);
    __syncthreads();
    uint16_t* Sb = S + (size_t)b * (nreg + 1);
    if (t < nreg) {
      cur[t] = ex;
      Sb[t] = (uint16_t)ex;
    }
    if (t == 0) Sb[nreg] = (uint16_t)tot;  // < 2^16: tot <= KB * k <= 32768
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kKPT; ++i) {
    const uint32_t x = t + (uint32_t)i * kQNT;
    if (x < nkb) {
      uint32_t h = cm_hash(key[i]);
      const uint32_t delta = (h >> 17) | (h << 15);
      for (int j = 0; j < k; ++j) {
        const uint32_t idx = h % n;
        const uint32_t p = atomicAdd(&cur[idx >> kQRegShift], 1u);
        stg[p] = (idx & (kQRegBytes - 1u)) | x << kQRegShift;
        h += delta;
      }
    }
  }
  __syncthreads();
  const uint32_t nrec = nkb * (uint32_t)k;
  uint32_t* o = R1 + (size_t)b * kb * (uint32_t)k;
  for (uint32_t i = t; i < nrec; i += kQNT) o[i] = stg[i];
}

// look: region r's bytes into LDS, then every block's run of records for
// the region; result = key index | (probe <= freq) << 15, same position
__global__ __launch_bounds__(kQNT) void cm_qlook_kernel(const uint8_t* __restrict__ table,
                                                        uint32_t tb, uint32_t nb, uint32_t nreg,
                                                        uint32_t kb, int k, int freq,
                                                        const uint16_t* __restrict__ S,
                                                        const uint32_t* __restrict__ R1,
                                                        uint16_t* __restrict__ R2) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[kQRegBytes / 4];
  __shared__ uint32_t seg[kQMaxBlocks];  // block b's run: start | length << 16
  // XCD-contiguous regions (as the insert's apply pass): a block's runs for
  // neighbouring regions share their edge lines, read once per XCD's L2
  // instead of once per region's workgroup
  const uint32_t r = xcd_index(blockIdx.x, gridDim.x), t = threadIdx.x;
  const uint32_t lane = t & 63, w = t >> 6;
  const uint32_t r0 = r * kQRegBytes;
  const uint32_t rbytes = tb - r0 < kQRegBytes ? tb - r0 : kQRegBytes;  // a multiple of 4
  {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t nq = rbytes / 16u;
    const u32x4* src = (const u32x4*)(table + r0);
    for (uint32_t i = t; i < nq; i += kQNT) *(u32x4*)&tab[4 * i] = __builtin_nontemporal_load(src + i);
    for (uint32_t i = nq * 4u + t; i < rbytes / 4u; i += kQNT)
      tab[i] = ((const uint32_t*)(table + r0))[i];
  }
  for (uint32_t b = t; b < nb; b += kQNT) {
    const uint16_t* Sb = S + (size_t)b * (nreg + 1);
    const uint32_t a = Sb[r], e = Sb[r + 1];
    seg[b] = a | (e - a) << 16;
  }
  __syncthreads();
  const uint8_t* tab8 = (const uint8_t*)tab;
  const uint32_t rb = kb * (uint32_t)k;
  // one block's run per wave step (about k * KB / nreg records): lanes over
  // the run; kQLU runs' loads issued before their lookups
#ifndef PSG_QLU
#define PSG_QLU 16  // runs per wave in flight (r06: 16 vs 8, query -4 %, profiles/r06_ab_countmin_look.txt)
#endif
  constexpr int kQLU = PSG_QLU;
  for (uint32_t b0 = w * (uint32_t)kQLU; b0 < nb; b0 += (kQNT / 64) * (uint32_t)kQLU) {
    uint32_t rec[kQLU], at[kQLU];
    bool have[kQLU];
#pragma unroll
    for (int u = 0; u < kQLU; ++u) {
      const uint32_t b = b0 + (uint32_t)u;
      const uint32_t sg = b < nb ? seg[b] : 0u;
      const uint32_t len = sg >> 16;
      at[u] = b * rb + (sg & 0xffffu) + lane;
      have[u] = lane < len;
      rec[u] = have[u] ? R1[at[u]] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kQLU; ++u) {
      if (have[u]) {
        const uint32_t v = tab8[rec[u] & (kQRegBytes - 1u)];
        R2[at[u]] = (uint16_t)((rec[u] >> kQRegShift) | ((int)v <= freq ? 0x8000u : 0u));
      }
    }
    // runs longer than a wave (rare: about 64 records per run at k = 4)
#pragma unroll
    for (int u = 0; u < kQLU; ++u) {
      const uint32_t b = b0 + (uint32_t)u;
      const uint32_t sg = b < nb ? seg[b] : 0u;
      const uint32_t len = sg >> 16;
      for (uint32_t i = 64u + lane; i < len; i += 64u) {
        const uint32_t q = b * rb + (sg & 0xffffu) + i;
        const uint32_t x = R1[q];
        const uint32_t v = tab8[x & (kQRegBytes - 1u)];
        R2[q] = (uint16_t)((x >> kQRegShift) | ((int)v <= freq ? 0x8000u : 0u));
      }
    }
  }
}

// keep: block b's results -> drop bits in LDS -> the direct form's keep
// bytes (8 keys each, thread-major per kQTile tile) and tile counts
__global__ __launch_bounds__(kQNT) void cm_qkeep_kernel(uint64_t nk, uint32_t kb, int k,
                                                        uint32_t nreg,
                                                        const uint16_t* __restrict__ S,
                                                        const uint16_t* __restrict__ R2,
                                                        uint32_t tile0,
                                                        uint32_t* __restrict__ tile_cnt,
                                                        uint8_t* __restrict__ keep_bits) {
  __shared__ uint32_t drop[8192 / 32];
  __shared__ uint32_t ws[kQNT / 64];
  const uint32_t t = threadIdx.x, b = blockIdx.x;
  const uint64_t k0 = (uint64_t)b * kb;
  const uint32_t nkb = (uint32_t)(nk - k0 < kb ? nk - k0 : kb);
  if (t < kb / 32u) drop[t] = 0;
  __syncthreads();
  const uint32_t nrec = S[(size_t)b * (nreg + 1) + nreg];
  const uint16_t* in = R2 + (size_t)b * kb * (uint32_t)k;
  constexpr int kKU = 8;  // results per thread in flight
  for (uint32_t i0 = t; i0 < nrec; i0 += kQNT * kKU) {
    uint32_t v[kKU];
#pragma unroll
    for (int q = 0; q < kKU; ++q) v[q] = i0 + kQNT * q < nrec ? in[i0 + kQNT * q] : 0u;
#pragma unroll
    for (int q = 0; q < kKU; ++q)
      if (v[q] & 0x8000u) atomicOr(&drop[(v[q] & 0x1fffu) >> 5], 1u << (v[q] & 31u));
  }
  __syncthreads();
  // tile tt of the block, keep byte j (keys tt*kQTile + 8j .. +8)
  const uint32_t tt = t / (uint32_t)kNT, j = t % (uint32_t)kNT;
  const uint32_t ntb = kb / (uint32_t)kQTile;
  uint32_t keep = 0;
  if (tt < ntb) {
    const uint32_t x = tt * (uint32_t)kQTile + 8u * j;  // first key of the byte (block-local)
    keep = ~(drop[x >> 5] >> (x & 31u)) & 0xffu;
    const uint32_t valid = x >= nkb ? 0u : (nkb - x >= 8u ? 8u : nkb - x);
    keep &= (1u << valid) - 1u;
    if (k0 + tt * (uint32_t)kQTile < nk)  // every byte of a tile holding keys (0 past nk)
      keep_bits[((uint64_t)tile0 + (k0 / kQTile) + tt) * kNT + j] = (uint8_t)keep;
  }
  uint32_t c = (uint32_t)__popc(keep);
  for (int s2 = 32; s2 >= 1; s2 >>= 1) c += (uint32_t)__shfl_xor((int)c, s2, 64);
  if ((t & 63) == 0) ws[t >> 6] = c;
  __syncthreads();
  if (j == 0 && tt < ntb && k0 + tt * (uint32_t)kQTile < nk) {
    uint32_t tot = 0;
    for (uint32_t q = 0; q < (uint32_t)kNT / 64u; ++q) tot += ws[tt * ((uint32_t)kNT / 64u) + q];
    tile_cnt[tile0 + (k0 / kQTile) + tt] = tot;
  }
}

}  // namespace

// region starts (block-major and region-major, u16) then the records
size_t cm_insert_scratch_bytes(uint64_t nk, uint32_t n, int k) {
  const uint64_t nreg = (cm_table_bytes(n) + kRegBytes - 1) / kRegBytes;
  if (nreg > kMaxRegions || nk * (uint64_t)k >= (1ull << 32)) return 0;  // CAS form
  const uint64_t kb = ins_block_keys(k), nb = (nk + kb - 1) / kb;
  const uint64_t sb = (nb * (nreg + 1) * 2 + 255) / 256 * 256;
  return 2 * sb + 4 * nb * kb * (uint64_t)k + 256;
}

hipError_t launch_cm_insert(const uint64_t* keys, const uint32_t* counts, uint64_t nk,
                            uint8_t* table, uint32_t n, int k, void* bins, size_t bins_bytes,
                            hipStream_t s) {
  if (nk == 0) return hipSuccess;
  const size_t need = cm_insert_scratch_bytes(nk, n, k);
  if (need && bins && bins_bytes >= need) {
    const uint32_t tb = (uint32_t)cm_table_bytes(n);
    const uint32_t nreg = (tb + kRegBytes - 1) / kRegBytes;
    const uint32_t kb = ins_block_keys(k);
    const uint32_t nb = (uint32_t)((nk + kb - 1) / kb);
    const size_t sb = ((size_t)nb * (nreg + 1) * 2 + 255) / 256 * 256;
    uint16_t* S = (uint16_t*)bins;
    uint16_t* ST = (uint16_t*)((char*)bins + sb);
    uint32_t* R = (uint32_t*)((char*)bins + 2 * sb);
    hipLaunchKernelGGL(cm_ibin_kernel, dim3(nb), dim3(kBlkNT), 0, s, keys, counts, nk, n, k, kb,
                       nreg, S, R);
    hipLaunchKernelGGL(cm_transpose_kernel, dim3((nreg + 1 + 63) / 64, (nb + 63) / 64), dim3(256),
                       0, s, (const uint16_t*)S, nb, nreg + 1, ST);
    hipLaunchKernelGGL(cm_iapply_kernel, dim3(nreg), dim3(kBlkNT), 0, s, table, tb, nb, nreg,
                       kb * (uint32_t)k, (const uint16_t*)ST, (const uint32_t*)R);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(cm_insert_kernel, dim3((uint32_t)((nk + kNT - 1) / kNT)), dim3(kNT), 0, s,
                     keys, counts, nk, table, n, k);
  return hipGetLastError();
}

// tile counts (u32 per tile), the keep bits (a byte per thread), then the
// binned form's region starts and records (sized for k <= kQMaxK whatever
// the filter's k: the device entry point's scratch does not know it)
size_t cm_query_scratch_bytes(uint64_t nk) {
  const uint64_t ntiles = (nk + kQTile - 1) / kQTile;
  const uint64_t rcap = q_record_cap(nk);
  return ((4 * ntiles + 255) / 256) * 256 + (ntiles * kNT + 255) / 256 * 256 +
         q_starts_bytes(rcap) + 6 * rcap + 64;
}

hipError_t launch_cm_query(const uint64_t* keys, uint64_t nk, const uint8_t* table, uint32_t n,
                           int k, int freq, uint64_t* out, unsigned long long* nout,
                           void* scratch, hipStream_t s) {
  const uint32_t ntiles = (uint32_t)((nk + kQTile - 1) / kQTile);
  uint32_t* cnt = (uint32_t*)scratch;
  uint8_t* bits = (uint8_t*)scratch + ((4 * (uint64_t)ntiles + 255) / 256) * 256;
  const uint32_t tb = (uint32_t)cm_table_bytes(n);
  const uint32_t nreg = (tb + kQRegBytes - 1) / kQRegBytes;
  // binned when the probes' lines would exceed the table (each probe of the
  // direct form pulls a 64-B line; the binned form reads the table once)
  const bool binned = k <= kQMaxK && nreg <= kQMaxReg && nk * (uint64_t)k * 64u > (uint64_t)tb;
  if (ntiles && binned) {
    char* qs = (char*)bits + ((uint64_t)ntiles * kNT + 255) / 256 * 256;
    const uint64_t rcap = q_record_cap(nk);
    const uint32_t kb = q_block_keys(k);
    const uint32_t rb = kb * (uint32_t)k;  // record slots per block
    // keys per chunk: whole blocks (a multiple of kQTile), records within rcap
    uint64_t chunk = std::min<uint64_t>(rcap / rb, kQMaxBlocks) * kb;
    uint16_t* S = (uint16_t*)qs;
    uint32_t* R1 = (uint32_t*)(qs + q_starts_bytes(rcap));
    uint16_t* R2 = (uint16_t*)((char*)R1 + 4 * rcap);
    for (uint64_t c0 = 0; c0 < nk; c0 += chunk) {
      const uint64_t cn = std::min<uint64_t>(chunk, nk - c0);
      const uint32_t nb = (uint32_t)((cn + kb - 1) / kb);
      hipLaunchKernelGGL(cm_qbin_kernel, dim3(nb), dim3(kQNT), 0, s, keys + c0, cn, n, k, kb,
                         nreg, S, R1);
      hipLaunchKernelGGL(cm_qlook_kernel, dim3(nreg), dim3(kQNT), 0, s, table, tb, nb, nreg, kb,
                         k, freq, (const uint16_t*)S, (const uint32_t*)R1, R2);
      hipLaunchKernelGGL(cm_qkeep_kernel, dim3(nb), dim3(kQNT), 0, s, cn, kb, k, nreg,
                         (const uint16_t*)S, (const uint16_t*)R2, (uint32_t)(c0 / kQTile), cnt,
                         bits);
    }
  } else if (ntiles) {
    hipLaunchKernelGGL(cm_count_kernel, dim3(ntiles), dim3(kNT), 0, s, keys, nk, table, n, k,
                       freq, cnt, bits);
  }
  hipLaunchKernelGGL(cm_scan_kernel, dim3(1), dim3(kNT), 0, s, cnt, ntiles, nout);
  if (ntiles)
    hipLaunchKernelGGL(cm_scatter_kernel, dim3(ntiles), dim3(kNT), 0, s, keys, nk, bits, cnt,
                       out);
  return hipGetLastError();
}

}  // namespace psg
