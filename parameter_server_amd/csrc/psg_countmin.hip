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
// the table is cut into 32 KB regions; a counting pass finds how many probes
// land in each region, a scatter pass writes every probe as a 4-byte record
// (offset in the region, count) into its region's list, and an apply pass
// gives each region one workgroup that adds its records into u32 LDS
// counters (native LDS adds: a counter's low byte is its sum mod 2^8) and
// then adds those sums into the region's bytes -- each table byte is read
// and written once, with no global atomics per probe (the CAS form below
// makes one device-scope atomic per probe, the bound of its rate).
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
// byte for byte.  queryKeys is a query pass that keeps one bit per key and an
// order-preserving compaction of those bits (workgroup scan + one scan of
// block totals): the table is read once.
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
constexpr int kBinNT = 256;
constexpr int kBinKPT = 64;                        // keys per thread: 16 K keys per workgroup
constexpr int kApplyNT = 1024;

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

// pass 1: probes per region (an LDS histogram per workgroup, then one
// global add per region)
__global__ __launch_bounds__(kBinNT) void cm_bin_count_kernel(const uint64_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ counts,
                                                              uint64_t nk, uint32_t n, int k,
                                                              uint32_t nreg,
                                                              uint32_t* __restrict__ rcount) {
  __shared__ uint32_t hst[kMaxRegions];
  for (uint32_t r = threadIdx.x; r < nreg; r += kBinNT) hst[r] = 0;
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * kBinNT * kBinKPT + threadIdx.x;
  for (int i = 0; i < kBinKPT; ++i) {
    const uint64_t x = b0 + (uint64_t)i * kBinNT;
    if (x < nk && (counts[x] & 0xffu))
      probes(keys[x], n, k, [&](uint32_t r, uint32_t) { atomicAdd(&hst[r], 1u); });
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < nreg; r += kBinNT)
    if (hst[r]) atomicAdd(rcount + r, hst[r]);
}

// pass 2: exclusive scan of the region counts (one workgroup) into rbase,
// and the reservation cursors rcur = rbase
__global__ __launch_bounds__(kBinNT) void cm_bin_scan_kernel(const uint32_t* __restrict__ rcount,
                                                             uint32_t nreg,
                                                             uint32_t* __restrict__ rbase,
                                                             uint32_t* __restrict__ rcur) {
  __shared__ uint32_t ws[kBinNT / 64];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < nreg; b += kBinNT) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < nreg ? rcount[i] : 0u;
    uint32_t tot;
    const uint32_t ex = dev::block_excl_scan<kBinNT>(v, ws, &tot);
    const uint32_t c0 = carry;
    if (i < nreg) {
      rbase[i] = c0 + ex;
      rcur[i] = c0 + ex;
    }
    __syncthreads();
    if (threadIdx.x == 0) carry = c0 + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) rbase[nreg] = carry;
}

// pass 3: the records, region by region.  A workgroup (1024 threads)
// reserves its space in every region with one atomic per region, then takes
// its keys in sub-chunks whose records fit LDS: counts them per region, lays
// them out region-major in LDS (a scan and LDS positions), and writes each
// region's run of records with consecutive stores of one thread, so the
// lines of the record lists are written whole instead of 4 bytes at a time
constexpr int kScNT = 1024;
constexpr uint32_t kScRecs = 24576;  // staged records per sub-chunk (96 KB)
__global__ __launch_bounds__(kScNT) void cm_bin_scatter_kernel(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ counts, uint64_t nk,
    uint32_t n, int k, uint32_t nreg, uint32_t sub, uint32_t* __restrict__ rcur,
    uint32_t* __restrict__ recs) {
  __shared__ uint32_t stg[kScRecs];
  __shared__ uint32_t start[kMaxRegions + 1];
  __shared__ uint32_t pos[kMaxRegions];
  __shared__ uint32_t base[kMaxRegions];
  __shared__ uint32_t ws[kScNT / 64];
  const uint32_t t = threadIdx.x;
  const uint64_t c0 = (uint64_t)blockIdx.x * kBinNT * kBinKPT;  // this workgroup's keys
  const uint64_t c1 = c0 + kBinNT * kBinKPT < nk ? c0 + kBinNT * kBinKPT : nk;
  // this workgroup's records per region, then its reservation in each list
  for (uint32_t r = t; r < nreg; r += kScNT) pos[r] = 0;
  __syncthreads();
  for (uint64_t x = c0 + t; x < c1; x += kScNT)
    if (counts[x] & 0xffu)
      probes(keys[x], n, k, [&](uint32_t r, uint32_t) { atomicAdd(&pos[r], 1u); });
  __syncthreads();
  for (uint32_t r = t; r < nreg; r += kScNT) base[r] = pos[r] ? atomicAdd(rcur + r, pos[r]) : 0u;
  for (uint64_t s0 = c0; s0 < c1; s0 += sub) {
    const uint64_t s1 = s0 + sub < c1 ? s0 + sub : c1;
    __syncthreads();  // the previous sub-chunk's writes have read stg / start
    for (uint32_t r = t; r < nreg; r += kScNT) pos[r] = 0;
    __syncthreads();
    for (uint64_t x = s0 + t; x < s1; x += kScNT)
      if (counts[x] & 0xffu)
        probes(keys[x], n, k, [&](uint32_t r, uint32_t) { atomicAdd(&pos[r], 1u); });
    __syncthreads();
    // exclusive scan of the counts over the regions (4 per thread)
    {
      uint32_t v[4], tot = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t r = 4 * t + j;
        v[j] = r < nreg ? pos[r] : 0u;
        tot += v[j];
      }
      uint32_t all;
      uint32_t ex = dev::block_excl_scan<kScNT>(tot, ws, &all);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t r = 4 * t + j;
        if (r < nreg) {
          start[r] = ex;
          pos[r] = ex;
        }
        ex += v[j];
      }
      if (t == 0) start[nreg] = all;
    }
    __syncthreads();
    for (uint64_t x = s0 + t; x < s1; x += kScNT) {
      const uint32_t c = counts[x] & 0xffu;
      if (c)
        probes(keys[x], n, k, [&](uint32_t r, uint32_t o) {
          stg[atomicAdd(&pos[r], 1u)] = o | c << kRegShift;
        });
    }
    __syncthreads();
    // each thread writes its regions' runs (consecutive stores per run)
    for (uint32_t r = t; r < nreg; r += kScNT) {
      const uint32_t a = start[r], e = start[r + 1];
      uint32_t* dst = recs + base[r];
      for (uint32_t i = a; i < e; ++i) dst[i - a] = stg[i];
      base[r] += e - a;
    }
  }
}

// pass 4: one workgroup per region: the records into u32 LDS sums, then the
// region's bytes += sum (mod 2^8); bytes past the table untouched
__global__ __launch_bounds__(kApplyNT) void cm_bin_apply_kernel(
    uint8_t* __restrict__ t, uint32_t tbytes, const uint32_t* __restrict__ rbase,
    const uint32_t* __restrict__ recs) {
  __shared__ uint32_t acc[kRegBytes];
  const uint32_t r = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < kRegBytes; i += kApplyNT) acc[i] = 0;
  __syncthreads();
  const uint32_t a = rbase[r], b = rbase[r + 1];
  for (uint32_t i = a + threadIdx.x; i < b; i += kApplyNT) {
    const uint32_t v = recs[i];
    __hip_atomic_fetch_add(&acc[v & (kRegBytes - 1u)], v >> kRegShift, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  // dwords of the region (the table is a whole number of dwords)
  uint32_t* tw = (uint32_t*)(t + (size_t)r * kRegBytes);
  const uint32_t nw = (tbytes - r * kRegBytes < kRegBytes ? tbytes - r * kRegBytes : kRegBytes) / 4u;
  for (uint32_t i = threadIdx.x; i < nw; i += kApplyNT) {
    const uint32_t w = tw[i];
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o |= ((((w >> (8 * j)) & 0xffu) + acc[4 * i + j]) & 0xffu) << (8 * j);
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

}  // namespace

size_t cm_insert_scratch_bytes(uint64_t nk, uint32_t n, int k) {
  const uint64_t nreg = (cm_table_bytes(n) + kRegBytes - 1) / kRegBytes;
  if (nreg > kMaxRegions || nk * (uint64_t)k >= (1ull << 32)) return 0;  // CAS form
  return 256 + 4 * 3 * (nreg + 1) + 4 * nk * (uint64_t)k;
}

hipError_t launch_cm_insert(const uint64_t* keys, const uint32_t* counts, uint64_t nk,
                            uint8_t* table, uint32_t n, int k, void* bins, size_t bins_bytes,
                            hipStream_t s) {
  if (nk == 0) return hipSuccess;
  const size_t need = cm_insert_scratch_bytes(nk, n, k);
  if (need && bins && bins_bytes >= need) {
    const uint32_t tb = (uint32_t)cm_table_bytes(n);
    const uint32_t nreg = (tb + kRegBytes - 1) / kRegBytes;
    uint32_t* rcount = (uint32_t*)bins;
    uint32_t* rbase = rcount + (nreg + 1);
    uint32_t* rcur = rbase + (nreg + 1);
    uint32_t* recs = (uint32_t*)((char*)bins + ((4 * 3 * (size_t)(nreg + 1) + 255) / 256) * 256);
    const uint64_t chunks = (nk + kBinNT * kBinKPT - 1) / (kBinNT * kBinKPT);
    hipError_t e = hipMemsetAsync(rcount, 0, 4 * (size_t)nreg, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cm_bin_count_kernel, dim3((uint32_t)chunks), dim3(kBinNT), 0, s, keys,
                       counts, nk, n, k, nreg, rcount);
    hipLaunchKernelGGL(cm_bin_scan_kernel, dim3(1), dim3(kBinNT), 0, s, rcount, nreg, rbase, rcur);
    // keys per staged sub-chunk: their records fit the LDS staging area
    const uint32_t sub = std::max<uint32_t>(1, kScRecs / (uint32_t)k);
    hipLaunchKernelGGL(cm_bin_scatter_kernel, dim3((uint32_t)chunks), dim3(kScNT), 0, s, keys,
                       counts, nk, n, k, nreg, sub, rcur, recs);
    hipLaunchKernelGGL(cm_bin_apply_kernel, dim3(nreg), dim3(kApplyNT), 0, s, table, tb, rbase,
                       recs);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(cm_insert_kernel, dim3((uint32_t)((nk + kNT - 1) / kNT)), dim3(kNT), 0, s,
                     keys, counts, nk, table, n, k);
  return hipGetLastError();
}

// tile counts (u32 per tile) then the keep bits (a byte per thread)
size_t cm_query_scratch_bytes(uint64_t nk) {
  const uint64_t ntiles = (nk + kQTile - 1) / kQTile;
  return ((4 * ntiles + 255) / 256) * 256 + ntiles * kNT + 64;
}

hipError_t launch_cm_query(const uint64_t* keys, uint64_t nk, const uint8_t* table, uint32_t n,
                           int k, int freq, uint64_t* out, unsigned long long* nout,
                           void* scratch, hipStream_t s) {
  const uint32_t ntiles = (uint32_t)((nk + kQTile - 1) / kQTile);
  uint32_t* cnt = (uint32_t*)scratch;
  uint8_t* bits = (uint8_t*)scratch + ((4 * (uint64_t)ntiles + 255) / 256) * 256;
  if (ntiles)
    hipLaunchKernelGGL(cm_count_kernel, dim3(ntiles), dim3(kNT), 0, s, keys, nk, table, n, k,
                       freq, cnt, bits);
  hipLaunchKernelGGL(cm_scan_kernel, dim3(1), dim3(kNT), 0, s, cnt, ntiles, nout);
  if (ntiles)
    hipLaunchKernelGGL(cm_scatter_kernel, dim3(ntiles), dim3(kNT), 0, s, keys, nk, bits, cnt,
                       out);
  return hipGetLastError();
}

}  // namespace psg
