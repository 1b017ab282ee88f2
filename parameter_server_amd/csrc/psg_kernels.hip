// psg_kernels.hip -- hand-written gfx950 (CDNA4) kernels of the server-side
// push aggregation path.  No MFMA: this is an integer merge + float
// segmented sum, bound by HBM bandwidth (DESIGN.md "Kernels").
//
// Reference semantics restated here (wakensky/parameter_server):
//   aggregate  <- KVVector::serialSetValue / parallelSetValue
//                 (src/parameter/kv_vector.h:84-137, 171-204) built on
//                 oldMatch / match (src/system/message.h:134-267)
//   partition  <- SArray::findRange + sliceKeyOrderedMsg lower_bounds
//                 (src/base/shared_array_inl.h:164-171, message.h:96-99)
//   gather     <- KVVector::serialGetValue (kv_vector.h:215-227)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_internal.h"
#include "psg_device.h"

namespace psg {

using namespace dev;

namespace {

// ----------------------------------------------------------------------
// gather (pull reply): out[i] = W[pos(req[i])], 0 where absent or where
// req[i] repeats req[i-1] (the reference merge walk advances past a match,
// message.h:256-260, so a repeated request key reads 0).
//
// A workgroup takes kGR consecutive (sorted) requests, four consecutive ones
// per thread, loaded first so they arrive while two 64-ary wave searches
// bound their server positions, [lower_bound(first), upper_bound(last));
// when that span fits kGS keys (a dense pull) it is staged in LDS with one
// batch of coalesced reads and every request searches there, otherwise (a
// sparse pull) each searches the span in global memory.  The repeat test
// takes the previous request from a register (the thread's own, its lane
// neighbour's, or the previous wave's last through LDS), not from memory.
// ----------------------------------------------------------------------
constexpr int kGR = 1024;  // requests per workgroup
constexpr int kGS = 4096;  // server keys staged in LDS (32 KB)

template <typename V>
__global__ __launch_bounds__(256) void gather_kernel(
    const uint64_t* __restrict__ D, uint64_t nd, const V* __restrict__ W,
    const uint64_t* __restrict__ req, uint64_t nreq, V* __restrict__ out,
    unsigned long long* __restrict__ matched) {
  constexpr int kI = kGR / 256;
  __shared__ uint64_t t[kGS];
  __shared__ uint64_t rg[2];
  __shared__ uint64_t wlast[4];  // each wave's last request
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t r0 = (uint64_t)blockIdx.x * kGR;
  const uint64_t r1 = nreq - r0 < (uint64_t)kGR ? nreq : r0 + kGR;
  const uint64_t ib = r0 + (uint64_t)kI * threadIdx.x;
  uint64_t k[kI];
#pragma unroll
  for (int q = 0; q < kI; ++q) k[q] = ib + q < r1 ? req[ib + q] : 0;
  const uint64_t before = r0 > 0 ? req[r0 - 1] : 0;  // the request before the block's first
  if (w < 2) {
    const uint64_t r = wave_search(D, nd, req[w == 0 ? r0 : r1 - 1], w == 1, lane);
    if (lane == 0) rg[w] = r;
  }
  if (lane == 63) wlast[w] = k[kI - 1];
  __syncthreads();
  const uint64_t lo = rg[0], hi = rg[1] > rg[0] ? rg[1] : rg[0];
  const uint64_t n = hi - lo;
  const bool staged = n <= (uint64_t)kGS;
  if (staged) {
    uint64_t x[kGS / 256];
#pragma unroll
    for (int j = 0; j < kGS / 256; ++j) {
      const uint64_t e = (uint64_t)j * 256 + threadIdx.x;
      if (e < n) x[j] = __builtin_nontemporal_load(D + lo + e);
    }
#pragma unroll
    for (int j = 0; j < kGS / 256; ++j) {
      const uint64_t e = (uint64_t)j * 256 + threadIdx.x;
      if (e < n) t[e] = x[j];
    }
    __syncthreads();
  }
  // the request before each of this thread's: its own previous one, lane
  // - 1's last, or the previous wave's last (the block's first: `before`)
  const uint64_t up = (uint64_t)__shfl_up((long long)k[kI - 1], 1, 64);
  const uint64_t prev0 = lane > 0 ? up : (w > 0 ? wlast[w - 1] : before);
  uint64_t pos[kI];
  bool ok[kI];
#pragma unroll
  for (int q = 0; q < kI; ++q) {
    const uint64_t i = ib + q;
    uint64_t p;
    bool hit;
    if (staged) {
      const int lp = lds_lower_bound<kGS>(t, (int)n, k[q]);
      p = lo + (uint64_t)lp;
      hit = (uint64_t)lp < n && t[lp] == k[q];
    } else {
      p = lo + gl_lower_bound(D + lo, n, k[q]);
      hit = p < hi && D[p] == k[q];
    }
    const uint64_t prev = q == 0 ? prev0 : k[q > 0 ? q - 1 : 0];
    const bool rep = i > 0 && i < r1 && prev == k[q];
    ok[q] = i < r1 && hit && !rep;
    pos[q] = ok[q] ? p : 0;
  }
  V x[kI];
#pragma unroll
  for (int q = 0; q < kI; ++q) x[q] = nd && ok[q] ? W[pos[q]] : V(0);
  int found = 0;
#pragma unroll
  for (int q = 0; q < kI; ++q) {
    if (ib + q < r1) {
      out[ib + q] = x[q];
      found += ok[q];
    }
  }
  // the workgroup's total, one atomic per workgroup: every wave's atomic on
  // the one counter serialised at one L2 channel (r05: 4,096 atomics took
  // most of a 1 M-request gather's 59 us)
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) found += __shfl_xor(found, d, 64);
  __shared__ int wfound[4];
  if (lane == 0) wfound[w] = found;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = wfound[0] + wfound[1] + wfound[2] + wfound[3];
    if (tot) atomicAdd(matched, (unsigned long long)tot);
  }
}

// pinned host <-> device copies by the GPU itself (zero-copy access over
// PCIe): 16-B loads, 4 in flight per thread, every block walking each
// buffer of the batch in turn.  For the 0.5-4 MB buffers of a push it beats
// a DMA copy's fixed cost (tools/calib/hostbw.py: 1 MB 47 vs 38 GB/s,
// 512 KB 40 vs 28 GB/s), and one launch carries a flush's worth of them.
// Both ends 16-B aligned (the runtime checks).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void host_copy_kernel(HostCopyBatch b) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  for (uint32_t c = 0; c < b.n; ++c) {
    const u32x4_t* __restrict__ s = (const u32x4_t*)b.d[c].src;
    u32x4_t* __restrict__ d = (u32x4_t*)b.d[c].dst;
    const uint64_t n16 = b.d[c].len / 16;
    for (uint64_t u = (uint64_t)blockIdx.x * 256u + threadIdx.x; u < n16; u += 4 * stride) {
      u32x4_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (u + j * stride < n16) v[j] = __builtin_nontemporal_load(s + u + j * stride);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (u + j * stride < n16) d[u + j * stride] = v[j];
    }
    const uint32_t tail = (uint32_t)(b.d[c].len % 16);
    if (blockIdx.x == 0 && threadIdx.x < tail)
      ((uint8_t*)(d + n16))[threadIdx.x] = ((const uint8_t*)(s + n16))[threadIdx.x];
  }
}

__global__ __launch_bounds__(256) void check_sorted_kernel(
    const uint64_t* __restrict__ k, uint64_t n, unsigned long long* bad, bool strict) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const bool b = (i > 0 && i < n) && (strict ? !(k[i - 1] < k[i]) : k[i] < k[i - 1]);
  const unsigned long long m = __ballot(b);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, (unsigned long long)__popcll(m));
}

// Strictly-increasing check of keys in pinned HOST memory, read by the GPU
// itself (zero-copy, 16 B per lane per load) -- a dense push's keys are
// needed for nothing else, so they are never staged in HBM.  Lane l of a
// wave holds keys 2u, 2u+1 (u = unit index); key 2u-1 comes from lane l-1,
// or, for lane 0, from one 8-B load.  Keys 16-B aligned (the runtime checks).
__global__ __launch_bounds__(256) void check_sorted_host_kernel(
    const uint64_t* __restrict__ k, uint64_t n, unsigned long long* bad) {
  typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
  const uint64_t n2 = n / 2;  // whole units
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  const int lane = threadIdx.x & 63;
  uint32_t cnt = 0;
  // every lane of a wave runs the same iterations (u0 is wave-uniform)
  for (uint64_t u0 = (uint64_t)blockIdx.x * 256u + (threadIdx.x & ~63u); u0 < n2; u0 += stride) {
    const uint64_t u = u0 + (uint64_t)lane;
    u64x2_t v = {0ull, 0ull};
    if (u < n2) v = __builtin_nontemporal_load((const u64x2_t*)k + u);
    uint64_t prev = (uint64_t)__shfl_up((long long)v.y, 1, 64);
    if (lane == 0 && u > 0) prev = k[2 * u - 1];
    if (u < n2) cnt += (v.x < v.y ? 0u : 1u) + ((u > 0 && !(prev < v.x)) ? 1u : 0u);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1u) && n > 1)
    cnt += k[n - 2] < k[n - 1] ? 0u : 1u;
  for (int o = 32; o > 0; o >>= 1) cnt += (uint32_t)__shfl_down((int)cnt, o, 64);
  if (lane == 0 && cnt) atomicAdd(bad, (unsigned long long)cnt);
}

// sliceKeyOrderedMsg positions: one wave per separator (message.h:96-99)
__global__ __launch_bounds__(256) void slice_kernel(
    const uint64_t* __restrict__ keys, uint64_t n, uint64_t kb, uint64_t ke,
    const uint64_t* __restrict__ sep, int nsep, uint64_t* __restrict__ pos) {
  const int s = (int)((blockIdx.x * 256u + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= nsep) return;
  uint64_t k = sep[s];
  if (k > ke) k = ke;
  if (k < kb) k = kb;
  const uint64_t r = wave_search(keys, n, k, false, lane);
  if (lane == 0) pos[s] = r;
}

// keys of a job's pushes that were not matched, summed into *bad: push p
// covered seg(p, last) - seg(p, 0) positions of which fail[p] failed
// (the count the reference CHECKs per push, kv_vector.h:134,192)
__global__ __launch_bounds__(256) void unmatched_kernel(const JobDev* __restrict__ jobs,
                                                        uint32_t j,
                                                        unsigned long long* __restrict__ bad) {
  const JobDev& J = jobs[j];
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  uint64_t miss = 0;
  if (p < J.npush) {
    const uint64_t n = J.pn[p];
    uint64_t matched = 0;
    if (J.ntiles) {
      const uint32_t a = J.seg[(size_t)p * J.segq];
      const uint32_t b = J.seg[(size_t)p * J.segq + (size_t)J.ntiles * J.segb];
      const uint64_t covered = b >= a ? b - a : 0;
      const uint64_t f = J.fail[p];
      matched = covered >= f ? covered - f : 0;
    }
    miss = n - (matched < n ? matched : n);
  }
  // one atomic per wave
  for (int d = 32; d >= 1; d >>= 1) miss += (uint64_t)__shfl_xor((long long)miss, d, 64);
  if ((threadIdx.x & 63) == 0 && miss)
    __hip_atomic_fetch_add(bad, (unsigned long long)miss, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace
// ----------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------
hipError_t launch_gather(int dtype, const uint64_t* dkeys, uint64_t nd,
                         const void* dvals, const uint64_t* req, uint64_t nreq,
                         void* out, unsigned long long* matched,
                         hipStream_t stream) {
  if (nreq == 0) return hipSuccess;
  const uint64_t blocks = (nreq + kGR - 1) / kGR;
  if (dtype == 0)
    hipLaunchKernelGGL(gather_kernel<float>, dim3((uint32_t)blocks), dim3(256), 0,
                       stream, dkeys, nd, (const float*)dvals, req, nreq,
                       (float*)out, matched);
  else
    hipLaunchKernelGGL(gather_kernel<double>, dim3((uint32_t)blocks), dim3(256), 0,
                       stream, dkeys, nd, (const double*)dvals, req, nreq,
                       (double*)out, matched);
  return hipGetLastError();
}

hipError_t launch_host_copy_batch(const HostCopyBatch& b, hipStream_t stream) {
  uint64_t units = 0;
  for (uint32_t c = 0; c < b.n; ++c) units += b.d[c].len / 16;
  if (b.n == 0) return hipSuccess;
  uint64_t blocks = (units + 1023) / 1024;  // 4 units per thread per pass
  blocks = blocks < 1 ? 1 : (blocks > 128 ? 128 : blocks);
  hipLaunchKernelGGL(host_copy_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, b);
  return hipGetLastError();
}

hipError_t launch_host_copy(void* dst, const void* src, size_t len, hipStream_t stream) {
  if (len == 0) return hipSuccess;
  HostCopyBatch b;
  b.n = 1;
  b.d[0] = HostCopyDesc{src, dst, (uint64_t)len};
  return launch_host_copy_batch(b, stream);
}

hipError_t launch_check_sorted(const uint64_t* keys, uint64_t n,
                               unsigned long long* bad, hipStream_t stream, bool strict) {
  if (n < 2) return hipSuccess;
  hipLaunchKernelGGL(check_sorted_kernel, dim3((uint32_t)((n + 255) / 256)),
                     dim3(256), 0, stream, keys, n, bad, strict);
  return hipGetLastError();
}

hipError_t launch_check_sorted_host(const uint64_t* keys, uint64_t n,
                                    unsigned long long* bad, hipStream_t stream) {
  if (n < 2) return hipSuccess;
  uint64_t blocks = (n / 2 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 512 ? 512 : blocks);
  hipLaunchKernelGGL(check_sorted_host_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream,
                     keys, n, bad);
  return hipGetLastError();
}

hipError_t launch_slice(const uint64_t* keys, uint64_t n, uint64_t kb,
                        uint64_t ke, const uint64_t* sep, int nsep,
                        uint64_t* pos, hipStream_t stream) {
  if (nsep <= 0) return hipSuccess;
  hipLaunchKernelGGL(slice_kernel, dim3((uint32_t)((nsep + 3) / 4)), dim3(256), 0,
                     stream, keys, n, kb, ke, sep, nsep, pos);
  return hipGetLastError();
}

hipError_t launch_unmatched(const JobDev* jobs, uint32_t job, uint32_t npush,
                            unsigned long long* bad, hipStream_t stream) {
  if (npush == 0) return hipSuccess;
  hipLaunchKernelGGL(unmatched_kernel, dim3((npush + 255) / 256), dim3(256), 0, stream, jobs, job,
                     bad);
  return hipGetLastError();
}

}  // namespace psg
