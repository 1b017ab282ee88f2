// psg_tile_dense.hip -- the dense fast path: jobs whose
// every push is a contiguous slice of the server keys, D[a, a + n) -- e.g.
// cfg4, all workers pushing the whole dense key range.
//
// Such a push needs no key reads and no search: element i of the push lands
// on slot a + i.  Whether a push is such a slice is checked once, when a
// plan is made (psg_plan_create; the plan contract fixes the push keys for
// the plan's lifetime, the guarantee the key cache gives a server,
// remote_node.cc:139-184): dense_check_kernel compares the push with D at
// its lower_bound.  A run then reads only the values and writes the sums --
// SURVEY 8d's dense form, sum(n)*s_V + U*s_V bytes.
//
// Fold: exactly the tile kernel's (psg_tile.hip): pushes in arrival order,
// the first push assigns, serial mode adds one +0.0 per gap of absent pushes
// and a trailing one (kv_vector.h:171-204).  A workgroup owns 1024 slots,
// 4 per thread (16-B loads and stores); the pushes' pieces of the tile come
// from the host-computed seg table, so the loop over pushes is wave-uniform.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_device.h"
#include "psg_internal.h"

#define AS1 __attribute__((address_space(1)))

namespace psg {

namespace {

constexpr int kNT = 256;

template <typename T>
__device__ __forceinline__ const AS1 T* G(const T* p) {
  return (const AS1 T*)p;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + j;
}

template <typename V, int M>
__global__ __launch_bounds__(kNT) void dense_kernel(const TileDesc* __restrict__ tiles,
                                                    uint32_t ntiles) {
  const uint32_t ti = xcd_tile(blockIdx.x, gridDim.x);
  if (ti >= ntiles) return;
  const TileDesc& T = tiles[ti];
  const uint32_t np = T.np, nt = T.nt;
  const bool parallel = (T.flags & kFlagParallel) != 0;
  const bool cont = (T.flags & kFlagCont) != 0;
  const uint32_t s0 = 4u * threadIdx.x;
  V acc[M][4];
  int last[4] = {-1, -1, -1, -1};
#pragma unroll
  for (int mi = 0; mi < M; ++mi)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[mi][j] = (cont && s0 + j < nt) ? G((const V*)T.out[mi] + T.slot0)[s0 + j] : V(0);
  // pushes in batches of kB: all of a batch's value loads are issued before
  // its fold, so kB loads per thread are in flight instead of one
  constexpr int kB = (int)(32 / (M * sizeof(V))) > 0 ? (int)(32 / (M * sizeof(V))) : 1;
  for (uint32_t q0 = 0; q0 < np; q0 += kB) {
    int64_t ps[kB], pe[kB];
    V v[kB][M][4];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const uint32_t q = q0 + u;
      ps[u] = 0;
      pe[u] = 0;  // empty: no slot
      if (q < np) {
        // piece [a, b) of push q in this tile; its first element sits on
        // slot dpos[q] + a (job positions), i.e. tile slot ps
        const uint32_t* sg = T.seg + (size_t)q * T.stride;
        const uint32_t a = uni(G(sg)[0]), b = uni(G(sg)[T.segb]);
        if (b > a) {
          ps[u] = (int64_t)(G(T.dpos)[q] + a) - (int64_t)T.slot0;
          pe[u] = ps[u] + (int64_t)(b - a);
        }
#pragma unroll
        for (int mi = 0; mi < M; ++mi) {
          const V* vp = (const V*)G(T.pvals)[(size_t)q * M + mi] + a;  // element of slot ps
          const int64_t e0 = (int64_t)s0 - ps[u];  // element index of this thread's first slot
          if (e0 >= 0 && (int64_t)s0 + 3 < pe[u] &&
              (((uintptr_t)(vp + e0)) & (4 * sizeof(V) - 1)) == 0) {
            // read once: nontemporal (the measured copy ceiling is with them)
            if constexpr (sizeof(V) == 4) {
              typedef float f4 __attribute__((ext_vector_type(4)));
              const f4 x = __builtin_nontemporal_load((const AS1 f4*)(vp + e0));
              v[u][mi][0] = x.x; v[u][mi][1] = x.y; v[u][mi][2] = x.z; v[u][mi][3] = x.w;
            } else {
              typedef double d2 __attribute__((ext_vector_type(2)));
              const d2 x0 = __builtin_nontemporal_load((const AS1 d2*)(vp + e0));
              const d2 x1 = __builtin_nontemporal_load((const AS1 d2*)(vp + e0) + 1);
              v[u][mi][0] = x0.x; v[u][mi][1] = x0.y; v[u][mi][2] = x1.x; v[u][mi][3] = x1.y;
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int64_t sl = (int64_t)s0 + j;
              v[u][mi][j] = (sl >= ps[u] && sl < pe[u]) ? G(vp)[sl - ps[u]] : V(0);
            }
          }
        }
      }
    }
    // fold the batch in push order
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int q = (int)(q0 + u);
      const bool first = q == 0 && !cont;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t sl = (int64_t)s0 + j;
        if (sl >= ps[u] && sl < pe[u]) {
          const bool gap = !parallel && last[j] < q - 1;
#pragma unroll
          for (int mi = 0; mi < M; ++mi) {
            const V ag = gap ? acc[mi][j] + V(0) : acc[mi][j];
            acc[mi][j] = first ? v[u][mi][j] : ag + v[u][mi][j];
          }
          last[j] = q;
        }
      }
    }
  }
  // trailing "+0.0" of absent last pushes (serial), stores
#pragma unroll
  for (int mi = 0; mi < M; ++mi) {
    V r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool gap = !parallel && last[j] < (int)np - 1;
      r[j] = gap ? acc[mi][j] + V(0) : acc[mi][j];
    }
    V* o = (V*)T.out[mi] + T.slot0 + s0;
    if (s0 + 3u < nt && ((uintptr_t)o & 15u) == 0u) {
      if constexpr (sizeof(V) == 4) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        *(AS1 f4*)o = f4{r[0], r[1], r[2], r[3]};
      } else {
        typedef double d2 __attribute__((ext_vector_type(2)));
        ((AS1 d2*)o)[0] = d2{r[0], r[1]};
        ((AS1 d2*)o)[1] = d2{r[2], r[3]};
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (s0 + j < nt) ((AS1 V*)o)[j] = r[j];
    }
  }
}

// one push against the server keys: start = lower_bound(D, keys[0]); the
// push is dense iff start + n <= nd and keys[i] == D[start + i] for all i.
// One wave per push finds start (and rejects at once when the last key is
// not n - 1 slots on); then every 4096-key chunk is compared.
__global__ __launch_bounds__(kNT) void dense_start_kernel(const DenseCheck* __restrict__ c,
                                                          uint32_t nc) {
  const uint32_t w = (blockIdx.x * kNT + threadIdx.x) >> 6;
  if (w >= nc) return;
  const DenseCheck& d = c[w];
  const uint64_t k0 = d.n ? d.keys[0] : 0;
  const uint64_t st = d.n ? dev::wave_search(d.D, d.nd, k0, false, threadIdx.x & 63) : 0;
  if ((threadIdx.x & 63) == 0) {
    d.out[0] = st;
    // the last key must sit n - 1 slots after the first (a cheap reject)
    if (d.n == 0 || st + d.n > d.nd || d.D[st + d.n - 1] != d.keys[d.n - 1]) d.out[1] = 1;
  }
}

__global__ __launch_bounds__(kNT) void dense_cmp_kernel(const DenseCheck* __restrict__ c,
                                                        const uint64_t* __restrict__ items,
                                                        uint64_t nitems) {
  for (uint64_t it = blockIdx.x; it < nitems; it += gridDim.x) {
    const uint64_t e = items[it];
    const DenseCheck& d = c[e >> 32];
    const uint64_t st = d.out[0];
    if (d.out[1]) continue;  // rejected already
    const uint64_t b0 = (e & 0xffffffffull) * 4096;
    bool bad = false;
    for (uint64_t i = b0 + threadIdx.x; i < b0 + 4096 && i < d.n; i += kNT)
      bad |= d.keys[i] != d.D[st + i];
    if (__ballot(bad) && (threadIdx.x & 63) == 0)
      __hip_atomic_fetch_or(d.out + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename V, int M>
hipError_t go(const TileDesc* t, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL((dense_kernel<V, M>), dim3(n), dim3(kNT), 0, s, t, n);
  return hipGetLastError();
}

template <typename V>
hipError_t launch_m(int m, const TileDesc* t, uint32_t n, hipStream_t s) {
  switch (m) {
    case 1: return go<V, 1>(t, n, s);
    case 2: return go<V, 2>(t, n, s);
    case 3: return go<V, 3>(t, n, s);
    case 4: return go<V, 4>(t, n, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_aggregate_dense(int dtype, int m, const TileDesc* d_tiles, uint32_t ntiles,
                                  hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  return dtype == 0 ? launch_m<float>(m, d_tiles, ntiles, stream)
                    : launch_m<double>(m, d_tiles, ntiles, stream);
}

hipError_t launch_dense_check(const DenseCheck* checks, uint32_t nchecks, const uint64_t* items,
                              uint64_t nitems, hipStream_t stream) {
  if (nchecks == 0) return hipSuccess;
  hipLaunchKernelGGL(dense_start_kernel, dim3((nchecks + 3) / 4), dim3(kNT), 0, stream, checks,
                     nchecks);
  if (nitems) {
    const uint64_t blocks = nitems < 8192 ? nitems : 8192;
    hipLaunchKernelGGL(dense_cmp_kernel, dim3((uint32_t)blocks), dim3(kNT), 0, stream, checks,
                       items, nitems);
  }
  return hipGetLastError();
}

}  // namespace psg
