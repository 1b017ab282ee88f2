// psg_partition.hip -- where every push of a (channel, time) aggregate is
// cut at every tile of server slots: SArray::findRange restated per tile
// (reference src/base/shared_array_inl.h:164-171, and the per-separator
// lower_bound of sliceKeyOrderedMsg, src/system/message.h:96-99).
//
// Output, per job: seg[p*segq + b*segb] = first index of push p whose key is
// >= D[b*tile] (b < ntiles), or > D[nslots-1] (b == ntiles); push-major for
// kStream jobs, tile-major for kSearch jobs (psg_internal.h JobDev).  The
// aggregate kernel (psg_tile.hip) reads push p's piece of tile t as
// [seg(p, t), seg(p, t + 1)).
//
// Two ways to fill it (JobDev::mode, chosen per job by the host from the
// mean piece length):
//   kSearch: one lane per (push, boundary); interpolation probes (pushes of
//            murmur-hashed keys are near-uniform over their range), then a
//            bisection, then one batch of 15 independent loads.  Costs a few
//            random lines per boundary: the right choice for long pieces.
//   kStream: one wave per 512 consecutive keys of one push; every key is
//            mapped to its tile through the job's splitter array
//            split[t] = D[t*tile] (split[ntiles] = D[nslots-1] + 1), and the
//            tile transitions between consecutive keys write seg.  Costs
//            8 B per pushed key: the right choice for many short pieces.
// Items are u64: job << 37 | push << 24 | (boundary group or chunk).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "psg_device.h"
#include "psg_internal.h"

namespace psg {

namespace {

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

// ---- kStream jobs: splitters and the reset of the job's fail counters ----
__global__ __launch_bounds__(256) void splitter_kernel(const JobDev* __restrict__ jobs,
                                                       const uint32_t* __restrict__ item_job,
                                                       uint32_t nitems) {
  const uint32_t item = blockIdx.x;
  if (item >= nitems) return;
  const uint32_t j = uni(item_job[item]);
  const JobDev& J = jobs[j];
  // this job's splitter blocks are consecutive items
  const uint32_t first = uni(J.split_begin);
  const uint64_t t = (uint64_t)(item - first) * 256u + threadIdx.x;
  if (t < J.ntiles) J.split[t] = J.dkeys[t * J.tile];
  if (t == J.ntiles) J.split[t] = J.dkeys[J.nslots - 1] + 1ull;  // D never holds 2^64-1
  if (t < J.npush) J.fail[t] = 0ull;
}

// ---- kSearch: one lane per (push, tile boundary) ----
// (dev::bracket_lower_bound: interpolation probes, bisection, one batch of
// the last <= 15 candidates)
using dev::bracket_lower_bound;

// A wave holds 64 consecutive boundaries of one push.  Every 16th lane and
// the last search the whole push; the lanes between start from the bracket
// their neighbours' answers give (about 16 tiles' worth of the push instead
// of all of it), which saves probe lines per boundary (the partition is
// bound by the random lines it reads).  A bracket that does
// not hold (an unsorted push) falls back to the whole push.
__device__ __forceinline__ void search_item(const JobDev& J, uint32_t p, uint32_t g, int lane) {
  const uint32_t b = (g << 6) + (uint32_t)lane;
  const bool valid = b <= J.ntiles;
  const uint64_t* S = J.pkeys[p];
  const uint64_t n = J.pn[p];
  const uint32_t bc = valid ? b : J.ntiles;
  const bool up = bc == J.ntiles;
  // boundary key: lower_bound(D[bc * tile]); past the last tile
  // upper_bound(D[nslots - 1]) == lower_bound(D[nslots - 1] + 1) (D never
  // holds 2^64-1) -- exactly the splitter array a plan writes once
  const uint64_t xl = J.split ? J.split[bc]
                      : up ? J.dkeys[J.nslots - 1] + 1ull : J.dkeys[(uint64_t)bc * J.tile];
  const uint64_t k0 = S[0], kn = S[n - 1];
  // the wave's last valid lane (invalid lanes repeat boundary ntiles)
  const int last = (int)((J.ntiles - (g << 6)) < 63u ? (J.ntiles - (g << 6)) : 63u);
  // bracketing lanes: every 16th and the last valid one
  const bool edge = (lane & 15) == 0 || lane == last;
  const int lo_l = lane & ~15;
  const int hi_l = lo_l + 16 < last ? lo_l + 16 : last;
  uint64_t res = 0;
  if (edge) {
    res = xl <= k0 ? 0 : (xl > kn ? n : bracket_lower_bound(S, xl, 0, n - 1, k0, kn));
  }
  const uint64_t r0 = (uint64_t)__shfl((long long)res, lo_l, 64);
  const uint64_t r1 = (uint64_t)__shfl((long long)res, hi_l, 64);
  if (!edge) {
    if (xl <= k0) {
      res = 0;
    } else if (xl > kn) {
      res = n;
    } else {
      uint64_t a = r0 > 0 ? r0 - 1 : 0, c = r1 < n ? r1 : n - 1;
      uint64_t ka = 0, kc = 0;
      bool ok = a < c;
      if (ok) {
        ka = S[a];
        kc = S[c];
        ok = ka < xl && xl <= kc;
      }
      res = ok ? bracket_lower_bound(S, xl, a, c, ka, kc) : bracket_lower_bound(S, xl, 0, n - 1, k0, kn);
    }
  }
  if (valid) {
    J.seg[(size_t)p * J.segq + (size_t)b * J.segb] = (uint32_t)res;
    if (b == 0) J.fail[p] = 0ull;  // the aggregate launch follows in-stream
  }
}

// ---- kStream: one wave per kStreamChunk consecutive keys of one push ----
constexpr uint32_t kKPL = kStreamChunk / 64;  // keys per lane
// seg[p][t] = lower_bound(S_p, split[t]).  A chunk [i0, i0 + cl) owns the
// splitters whose lower bound falls inside it (the push's last chunk also
// those past its last key): split[t] > S[i0-1] and split[t] <= S[i0+cl-1].
// One lane per splitter, 64 consecutive splitters per window; each lane
// binary-searches its splitter in the chunk's keys, staged in LDS.
__device__ __forceinline__ void stream_item(const JobDev& J, uint32_t p, uint32_t c, int lane,
                                            uint64_t* ck /* LDS: this wave's chunk keys */) {
  const uint64_t* S = J.pkeys[p];
  const uint64_t n = J.pn[p];
  const uint32_t nt = J.ntiles;
  // global (not flat) accesses: a flat load also counts on lgkmcnt, so the
  // LDS searches would wait for the splitter and key loads in flight too
  const __attribute__((address_space(1))) uint64_t* sp =
      (const __attribute__((address_space(1))) uint64_t*)J.split;
  __attribute__((address_space(1))) uint32_t* seg =
      (__attribute__((address_space(1))) uint32_t*)(J.seg + (size_t)p * J.segq);  // push-major, segb = 1
  const uint64_t i0 = (uint64_t)c * kStreamChunk;
  const uint32_t cl = (uint32_t)(n - i0 < kStreamChunk ? n - i0 : kStreamChunk);
  const bool last = i0 + cl == n;
  // the chunk's keys (kKPL per lane, element j*64 + lane: every load is one
  // coalesced 512-B wave access), then into LDS in order; +inf past the end
  uint64_t k[kKPL];
  const __attribute__((address_space(1))) uint64_t* Sg =
      (const __attribute__((address_space(1))) uint64_t*)(S + i0);
#pragma unroll
  for (int j = 0; j < kKPL; ++j) {
    const uint32_t x = 64u * j + (uint32_t)lane;
    k[j] = x < cl ? Sg[x] : ~0ull;
  }
  // T0 = (splitters <= S[i0-1]) - 1: an interpolated guess checked against a
  // window of 64 splitters around it (murmur-hashed keys and D are near-
  // uniform, so the guess is a few tiles off), else a 64-ary search
  // The guess's window is 128 splitters (two per lane) starting a little
  // below the guess, so the splitters the chunk's first window pass needs
  // (T0 + 1 onwards) are usually already in registers: one dependent round
  // trip fewer per chunk.  win = index of splitter T0 + 1 in that window.
  int64_t T0 = -1;
  int64_t g = 0;
  uint64_t w0 = ~0ull, w1 = ~0ull;
  int32_t win = -1;
  if (i0 > 0) {
    // a first window guessed from the chunk's position in the push (pushes
    // of hashed keys spread over the job's key range like D does), loaded
    // together with the chunk's keys and S[i0-1]: when it brackets S[i0-1]
    // (most chunks) the interpolated window below, which waits for
    // S[i0-1], is not needed
    int64_t gq = (int64_t)((double)i0 / (double)n * (double)nt) - 32;
    gq = gq + 128 > (int64_t)nt + 1 ? (int64_t)nt + 1 - 128 : gq;
    gq = gq < 0 ? 0 : gq;
    const int64_t tq = gq + lane;
    const uint64_t q0 = tq <= (int64_t)nt ? sp[tq] : ~0ull;
    const uint64_t q1 = tq + 64 <= (int64_t)nt ? sp[tq + 64] : ~0ull;
    const uint64_t kp = uni64(((const __attribute__((address_space(1))) uint64_t*)S)[i0 - 1]);
    const uint64_t s0 = uni64(sp[0]), sn = uni64(sp[nt]);
    uint32_t qc = 64;  // splitters <= kp in the guessed window (64+: not usable)
    if (kp >= s0 && kp < sn) {
      qc = (uint32_t)__popcll(__ballot(tq <= (int64_t)nt && q0 <= kp));
      if (qc == 64u) qc += (uint32_t)__popcll(__ballot(tq + 64 <= (int64_t)nt && q1 <= kp));
    }
    if (kp >= sn) {
      T0 = nt;
    } else if (kp >= s0 && (qc > 0 || gq == 0) && qc < 64u) {
      // T0 + 1 is the window's splitter qc (< 64): the first pass reads
      // splitters qc .. qc + 63 of the 128 in registers
      g = gq;
      w0 = q0;
      w1 = q1;
      T0 = g + (int64_t)qc - 1;
      win = (int32_t)qc;
    } else if (kp >= s0) {
      const double f = (double)(kp - s0) / (double)(sn - s0);
      g = (int64_t)(f * (double)nt) - 24;
      g = g < 0 ? 0 : (g + 64 > (int64_t)nt + 1 ? (int64_t)nt + 1 - 64 : g);
      g = g < 0 ? 0 : g;
      const int64_t t = g + lane;
      w0 = t <= (int64_t)nt ? sp[t] : ~0ull;
      w1 = t + 64 <= (int64_t)nt ? sp[t + 64] : ~0ull;
      const bool le = t <= (int64_t)nt && w0 <= kp;
      const uint32_t cnt = (uint32_t)__popcll(__ballot(le));
      const bool inside = (cnt > 0 || g == 0) && (cnt < 64 || g + 64 > (int64_t)nt);
      if (inside) {
        T0 = g + (int64_t)cnt - 1;
        win = (int32_t)cnt;
      } else {
        T0 = (int64_t)dev::wave_search(J.split, (uint64_t)nt + 1u, kp, true, lane) - 1;
      }
    }
  }
  // stores before the wave's reads of them: LDS accesses of one wave are
  // ordered; the fences keep the compiler from moving the reads up
#pragma unroll
  for (int j = 0; j < kKPL; ++j) ck[64 * j + lane] = k[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint64_t klast = uni64(ck[cl - 1]);
  for (int64_t t0 = T0 + 1; t0 <= (int64_t)nt; t0 += 64) {
    const int64_t t = t0 + lane;
    uint64_t sv;
    if (win >= 0) {  // first pass after an interpolated T0: from the window
      const int32_t x = win + lane;  // window index of splitter t (< 128)
      const uint64_t a0 = (uint64_t)__shfl((long long)w0, x & 63, 64);
      const uint64_t a1 = (uint64_t)__shfl((long long)w1, x & 63, 64);
      sv = t <= (int64_t)nt ? (x < 64 ? a0 : a1) : ~0ull;
      win = -1;
    } else {
      sv = t <= (int64_t)nt ? sp[t] : ~0ull;
    }
    // keys of the chunk below sv: lower_bound over ck[0, cl)
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t st = kStreamChunk / 2; st > 0; st >>= 1)
      if (pos + st <= cl && ck[pos + st - 1] < sv) pos += st;
    pos += (pos < cl && ck[pos] < sv) ? 1u : 0u;
    if (t <= (int64_t)nt && (pos < cl || last)) seg[t] = (uint32_t)(i0 + pos);
    // later windows own nothing once a splitter passes the chunk's last key
    // (the push's last chunk fills every remaining boundary with n)
    if (!last && uni64((uint64_t)__shfl((long long)sv, 63, 64)) > klast) break;
  }
  // No order check here (r05): the aggregate kernel finds an unsorted push
  // by itself -- every key must be found, at strictly increasing positions
  // inside its piece, and a piece whose bounds run backwards is an
  // overflow -- so the push's fail counter is only reset here, by its
  // first chunk, ahead of the aggregate launch that adds to it (plans then
  // need no per-run splitter pass, psg_runtime.hip run_stage)
  if (c == 0 && lane == 0) J.fail[p] = 0ull;
}

// blocks b and b+8 share an XCD (observed dispatch, speed only).  `xcd`: each
// XCD takes a contiguous run of items, so neighbouring boundary groups of one
// push, whose probes touch the same lines, share one L2 -- for launches of
// search-mode jobs only (r06: cfg2 / cfg3 partition -2..-4 %; stream-mode
// chunks read their keys once and lost 5 % that way,
// profiles/r06_ab_partition_xcd.txt)
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + j;
}

__global__ __launch_bounds__(256) void partition_kernel(const JobDev* __restrict__ jobs,
                                                        const uint64_t* __restrict__ items,
                                                        uint32_t nitems, int xcd) {
  __shared__ uint64_t ck[4][kStreamChunk];
  const uint32_t blk = xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t item = uni((blk * 256u + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (item >= nitems) return;
  const uint64_t it = uni64(items[item]);
  const uint32_t j = (uint32_t)(it >> 37);
  const uint32_t p = (uint32_t)(it >> 24) & 0x1fffu;
  const uint32_t x = (uint32_t)it & 0xffffffu;
  const JobDev& J = jobs[j];
  if (J.mode == kStream)
    stream_item(J, p, x, lane, ck[threadIdx.x >> 6]);
  else
    search_item(J, p, x, lane);
}

}  // namespace

hipError_t launch_partition(const JobDev* d_jobs, const uint32_t* d_split_item_job,
                            uint32_t nsplit_items, const uint64_t* d_items, uint32_t nitems,
                            hipStream_t stream, bool xcd) {
  if (nsplit_items)
    hipLaunchKernelGGL(splitter_kernel, dim3(nsplit_items), dim3(256), 0, stream, d_jobs,
                       d_split_item_job, nsplit_items);
  if (nitems)
    hipLaunchKernelGGL(partition_kernel, dim3((nitems + 3) / 4), dim3(256), 0, stream, d_jobs,
                       d_items, nitems, xcd ? 1 : 0);
  return hipGetLastError();
}

}  // namespace psg
