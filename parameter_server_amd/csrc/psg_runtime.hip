// psg_runtime.hip -- host side of the C ABI (include/psg.h).
//
// psg_ctx mirrors KVVector<uint64,V> (src/parameter/kv_vector.h:13-62): per
// channel sorted server keys key_[chl] and values val_[chl], and per time t
// the aggregate recved_val_[t].  Keys/values/aggregates live in the HBM of
// one device; a host mirror of key_[chl] serves findRange without a device
// round trip.  All device work is ordered on one HIP stream per context;
// a mutex gives the reference's threading contract (setValue on the
// executor thread, received() from the app thread, kv_vector.h:45,67).
#include <hip/hip_runtime.h>
#include <chrono>

#include <algorithm>
#include <cmath>
#include <iterator>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/psg.h"
#include "psg_host.h"
#include "psg_internal.h"

using psg::JobDev;

namespace {
thread_local std::string g_err;
}  // namespace

int psg::fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

namespace {

using psg::fail;

size_t vsize(int dtype) { return dtype == PSG_F32 ? 4 : 8; }

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// --------------------------------------------------------------------------
// Job table: device image of a batch of merge jobs (shared by psg_plan and
// the context's flushes).
// --------------------------------------------------------------------------
struct JobSpec {
  const uint64_t* keys;
  uint64_t nslots;
  std::vector<const uint64_t*> pkeys;
  std::vector<const void*> pvals;  // [p*m + i]
  std::vector<uint64_t> pn;
  std::vector<void*> out;
  uint32_t flags;
  // dense job: every non-empty push p is D[dpos[p], dpos[p] + pn[p])
  bool dense = false;
  std::vector<uint64_t> dpos;
};

// Mean piece length (keys per push per tile) below which a job's partition
// streams the push keys instead of searching every tile boundary
// (DESIGN.md 4.1): a bracketed boundary search reads ~3.5 random lines
// (~450 B), the stream 8 B per key, but the stream's chunks wait on more
// dependent round trips; measured on cfg3 (29.7 keys per piece) the search
// is 8 % faster, so the switch sits below it.
constexpr double kStreamBelow = 24.0;
// Mean piece length below which the aggregate kernel packs several pushes'
// pieces into one 64-lane round; above it rounds are
// push-uniform, which is faster while most rounds are full anyway.
constexpr double kPackBelow = 16.0;
// psg_push tests pushes of at least this many keys for a contiguous slice
constexpr size_t kDenseMinKeys = 1024;

// Kernel-form overrides come from explicit flags (psg.h PSG_FORM_*,
// PSG_PART_*, PSG_GROUP*, PSG_NO_DENSE, PSG_NO_ZERO_COPY), never from the
// environment: tests and A/B measurements pass them to psg_plan_create /
// psg_create; results are bit-identical either way.

// Marks the jobs whose every non-empty push is a contiguous slice of the
// job's server keys (psg_tile_dense.hip), with each push's start position.
// One synchronous check on the device per plan.
int detect_dense(std::vector<JobSpec>& specs) {
  std::vector<psg::DenseCheck> hc;
  std::vector<std::pair<size_t, size_t>> at;  // (job, push) of each check
  std::vector<uint64_t> items;
  for (size_t j = 0; j < specs.size(); ++j) {
    const JobSpec& s = specs[j];
    if (s.nslots == 0) continue;
    for (size_t p = 0; p < s.pn.size(); ++p) {
      if (s.pn[p] == 0) continue;
      if (s.pn[p] > s.nslots) goto next_job;  // cannot be a slice
      at.emplace_back(j, p);
      hc.push_back(psg::DenseCheck{s.pkeys[p], s.pn[p], s.keys, s.nslots, nullptr});
    }
  next_job:;
  }
  if (hc.empty()) return PSG_OK;
  for (size_t c = 0; c < hc.size(); ++c)
    for (uint64_t q = 0; q * 4096 < hc[c].n; ++q) items.push_back((uint64_t)c << 32 | q);
  const size_t ob = align_up(16 * hc.size(), 256), cb = align_up(sizeof(psg::DenseCheck) * hc.size(), 256);
  char* tmp = nullptr;
  HIP_TRY(hipMalloc((void**)&tmp, ob + cb + 8 * items.size()));
  unsigned long long* outs = (unsigned long long*)tmp;
  for (size_t c = 0; c < hc.size(); ++c) hc[c].out = outs + 2 * c;
  std::vector<unsigned long long> ho(2 * hc.size());
  hipError_t e = hipMemset(outs, 0, 16 * hc.size());
  if (e == hipSuccess) e = hipMemcpy(tmp + ob, hc.data(), sizeof(psg::DenseCheck) * hc.size(),
                                     hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(tmp + ob + cb, items.data(), 8 * items.size(),
                                     hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = psg::launch_dense_check((const psg::DenseCheck*)(tmp + ob), (uint32_t)hc.size(),
                                (const uint64_t*)(tmp + ob + cb), items.size(), nullptr);
  if (e == hipSuccess) e = hipMemcpy(ho.data(), outs, 16 * hc.size(), hipMemcpyDeviceToHost);
  (void)hipFree(tmp);
  if (e != hipSuccess) return fail(PSG_ERR_DEVICE, "dense check: %s", hipGetErrorString(e));
  std::vector<int> ok(specs.size(), -1);  // -1 unchecked, 1 dense so far, 0 not
  for (size_t c = 0; c < hc.size(); ++c) {
    const size_t j = at[c].first;
    if (ok[j] < 0) {
      ok[j] = 1;
      specs[j].dpos.assign(specs[j].pn.size(), 0);
    }
    if (ho[2 * c + 1]) ok[j] = 0;
    specs[j].dpos[at[c].second] = ho[2 * c];
  }
  for (size_t j = 0; j < specs.size(); ++j) {
    // every non-empty push was checked (none skipped by the size test)
    size_t nonempty = 0, checked = 0;
    for (uint64_t n : specs[j].pn) nonempty += n != 0;
    for (const auto& a : at) checked += a.first == j;
    specs[j].dense = ok[j] == 1 && checked == nonempty && nonempty > 0;
    if (!specs[j].dense) specs[j].dpos.clear();
  }
  return PSG_OK;
}

struct JobTable {
  int device = -1;
  int knob_part = -1, knob_pack = -1, knob_wide = -1;  // forced (read_knobs), -1 = chosen
  int knob_cursor = -1;
  void read_knobs(unsigned f) {
    knob_cursor = (f & PSG_FORM_CURSOR) ? 1 : (f & PSG_NO_CURSOR) ? 0 : -1;
    knob_part = (f & PSG_PART_SEARCH) ? (int)psg::kSearch
                : (f & PSG_PART_STREAM) ? (int)psg::kStream : -1;
    knob_pack = (f & PSG_FORM_PACKED) ? 1 : (f & PSG_FORM_UNIFORM) ? 0 : -1;
    knob_wide = (f & PSG_GROUP64) ? 1 : (f & PSG_GROUP32) ? 0 : -1;
    zero_copy = !(f & PSG_NO_ZERO_COPY);
  }
  bool pack = false;  // rounds may hold several pushes
  bool wide = false;  // push groups of 64 in the tile kernel (a job has > 32 pushes)
  bool dense = false;  // every job dense: psg_tile_dense.hip, no partition
  // cursor form (psg_tile_cursor.hip): plans of long pieces, no partition
  // pass; chunks of consecutive tiles, one workgroup each
  bool cursor = false;
  // packed cursor form (psg_tile_packed.hip CUR): short pieces of <= 256
  // pushes, no partition pass either
  bool pcursor = false;
  uint32_t bxs = 32;          // boundary words per chunk boundary (pushes per job at most)
  uint32_t nchunks = 0;
  psg::CursorJob* d_cjobs = nullptr;
  psg::CursorChunk* d_chunks = nullptr;
  uint32_t* d_bx = nullptr;   // chunk boundary words
  void* d_zero = nullptr;     // fail counters of every job + boundary words: zeroed per run
  size_t zero_bytes = 0;
  std::vector<uint32_t> chunk0;  // per job: its first chunk
  uint32_t ckr = 3;              // rounds per push per tile (max over the jobs)
  int dtype = 0, m = 1;
  std::vector<JobDev> h;
  // per job (host): pushes kept (non-empty) and where their matched counts go
  struct JobInfo {
    uint32_t np = 0, ntiles = 0;
    std::vector<uint64_t> pn;          // kept pushes
    std::vector<uint32_t> slot;        // kept push -> index in the caller's push list
    uint32_t ncaller = 0;              // caller's push count (empties included)
    uint32_t* seg = nullptr;
    uint32_t segq = 1;                 // seg stride between pushes
    unsigned long long* fail = nullptr;
    uint32_t kr = 0;                   // cursor form: rounds per push per tile
    uint32_t nch = 0;                  // cursor form: chunks
  };
  std::vector<JobInfo> info;
  uint32_t ntiles = 0, nitems = 0, nsplit = 0;
  // plans (D fixed for their lifetime): the stream jobs' splitters are
  // written once, at build, and a run launches only the partition proper
  bool split_once = false;
  bool all_search = false;  // every job's partition searches (launch_partition xcd)
  void* blob = nullptr;
  size_t blob_bytes = 0;
  JobDev* d_jobs = nullptr;
  psg::TileDesc* d_tiles = nullptr;
  uint32_t* d_split_items = nullptr;
  uint64_t* d_items = nullptr;
  // pinned host images of the blob, used alternately: a build fills one
  // while the previous build's copy may still be in flight
  char* himg[2] = {nullptr, nullptr};
  const void* himg_dev[2] = {nullptr, nullptr};  // their device-visible addresses
  bool zero_copy = true;  // the image moves by the zero-copy kernel, not a DMA copy
  size_t himg_cap[2] = {0, 0};
  hipEvent_t himg_ev[2] = {nullptr, nullptr};
  int himg_cur = 0;

  // the shape of the last build whose tile descriptors and work items are
  // on the device (flushes only): a flush of the same shape -- the usual
  // case, the same range of a channel merged time after time -- writes and
  // uploads only the job tables and the pushes' pointers (for a 16.8 M-slot
  // aggregate the descriptors are 1.4 MB)
  std::vector<uint64_t> last_shape;
  void release_blob() {
    if (blob) (void)hipFree(blob);
    blob = nullptr;
    blob_bytes = 0;
    last_shape.clear();
  }
  void release() {
    release_blob();
    for (int i = 0; i < 2; ++i) {
      if (himg_ev[i]) (void)hipEventSynchronize(himg_ev[i]);
      if (himg_ev[i]) (void)hipEventDestroy(himg_ev[i]);
      if (himg[i]) (void)hipHostFree(himg[i]);
      himg[i] = nullptr;
      himg_dev[i] = nullptr;
      himg_ev[i] = nullptr;
      himg_cap[i] = 0;
    }
  }

  // Builds (or rebuilds, reusing the allocation when it fits) the device image:
  // [JobDev x njobs][TileDesc x ntiles][split items u32][items u64] then per
  // job: pkeys, pvals, pn, out, fail, seg, split.  The image is copied on
  // stream `strm`, without a host wait when `async`; work enqueued on
  // `strm` afterwards sees it.
  // `index`: give the tile kernel's tiles a resident bucket table (built
  // here, once, from D: plans, whose D is fixed for their lifetime)
  int build(int dev, int dt, int mm, const std::vector<JobSpec>& jobs, hipStream_t strm = nullptr,
            bool async = false, bool index = false) {
    device = dev;
    dtype = dt;
    m = mm;
    const int forced = knob_part;
    h.assign(jobs.size(), JobDev{});
    info.assign(jobs.size(), JobInfo{});
    struct Offs { size_t pk, pv, pn, out, fail, seg, split, dpos; };
    std::vector<Offs> offs(jobs.size());
    uint64_t tiles = 0, items = 0, sitems = 0;
    dense = !jobs.empty();
    for (const JobSpec& s : jobs) dense = dense && s.dense;
    // the round form first (mean keys per push per 1024-slot tile) and the
    // push-group size: they fix the tile size, 2048 slots for the packed
    // kernel and for the tile kernel's 64-push form
    {
      const uint64_t t1 = psg::kTileSlots;
      double kv_all = 0, pieces_all = 0;
      uint32_t maxnp = 0;
      for (const JobSpec& s : jobs) {
        uint32_t np = 0;
        for (uint64_t n : s.pn) {
          kv_all += (double)n;
          np += n != 0;
        }
        maxnp = std::max(maxnp, np);
        pieces_all += (double)np * (double)((s.nslots + t1 - 1) / t1);
      }
      const int fp = knob_pack;
      pack = fp >= 0 ? fp == 1 : (pieces_all > 0 && kv_all / pieces_all < kPackBelow);
      wide = knob_wide >= 0 ? knob_wide == 1 : maxnp > 32;
    }
    const uint32_t tile = dense ? psg::kTileSlots
                          : pack ? psg::kPackTileSlots
                                 : wide ? psg::kWideSlots : psg::kTileSlots;
    for (size_t j = 0; j < jobs.size(); ++j) {
      const JobSpec& s = jobs[j];
      JobInfo& I = info[j];
      I.ncaller = (uint32_t)s.pn.size();
      if (s.pn.size() > (size_t)psg::kMaxPush)
        return fail(PSG_ERR_ARG, "job %zu: %zu pushes > max %d", j, s.pn.size(), psg::kMaxPush);
      uint64_t kv = 0;
      for (size_t p = 0; p < s.pn.size(); ++p) {
        if (s.pn[p] >= (1ull << 32))
          return fail(PSG_ERR_ARG, "push of %llu keys >= 2^32", (unsigned long long)s.pn[p]);
        // an empty push is ignored (kv_vector.h:90,177): the first NON-empty
        // push is the one that assigns
        if (s.pn[p] == 0) continue;
        I.pn.push_back(s.pn[p]);
        I.slot.push_back((uint32_t)p);
        kv += s.pn[p];
      }
      I.np = (uint32_t)I.pn.size();
      // no server keys: nothing can match (every pushed key is reported unmatched)
      I.ntiles = s.nslots ? (uint32_t)((s.nslots + tile - 1) / tile) : 0u;
      JobDev& d = h[j];
      d.nslots = s.nslots;
      d.npush = I.np;
      d.ntiles = I.ntiles;
      d.tile = tile;
      // keys per push per 1024 slots (the partition modes' calibration unit)
      const uint64_t nt1 = (s.nslots + psg::kTileSlots - 1) / psg::kTileSlots;
      const double piece = I.np && nt1 ? (double)kv / ((double)I.np * nt1) : 1e9;
      d.mode = s.dense ? psg::kSearch
                       : forced >= 0 ? (uint32_t)forced
                                     : (piece < kStreamBelow ? psg::kStream : psg::kSearch);
      d.segq = d.mode == psg::kStream ? I.ntiles + 1 : 1u;
      d.segb = d.mode == psg::kStream ? 1u : I.np;
      I.segq = d.segq;
      tiles += I.ntiles;
      if (I.ntiles && I.np && !s.dense) {  // dense: seg filled here, nothing to search
        if (d.mode == psg::kSearch) {
          items += (uint64_t)((I.ntiles + 64) / 64) * I.np;
          if (index) {  // plans: the boundary keys as a splitter array, written once
            d.split_begin = (uint32_t)sitems;
            sitems += (std::max<uint64_t>(I.ntiles + 1, I.np) + 255) / 256;
          }
        } else {
          d.split_begin = (uint32_t)sitems;
          sitems += (std::max<uint64_t>(I.ntiles + 1, I.np) + 255) / 256;
          for (uint64_t n : I.pn) items += (n + psg::kStreamChunk - 1) / psg::kStreamChunk;
        }
      }
      if (tiles >= (1ull << 31) || items >= (1ull << 31) || sitems >= (1ull << 31))
        return fail(PSG_ERR_ARG, "batch too large (%llu tiles)", (unsigned long long)tiles);
      if (j >= (1ull << 27)) return fail(PSG_ERR_ARG, "too many jobs");
    }
    // the cursor form: plans (resident index) of search-mode jobs of at most
    // kCursorPushes pushes; kr = the rounds of 64 keys loaded per push per
    // tile (mean + 4 sigma keys, at most 3: longer pieces finish round by
    // round in the fold step).  Opt-in only (PSG_FORM_CURSOR), with no size
    // gate: measured slower than partition + tile kernel on cfg2 (0.509 vs
    // 0.437 ms per step)
    cursor = index && !dense && !pack && !wide && knob_cursor == 1 && tiles > 0;
    for (size_t j = 0; cursor && j < jobs.size(); ++j) {
      const JobSpec& s = jobs[j];
      JobInfo& I = info[j];
      if (s.dense || h[j].mode != psg::kSearch || I.np > (uint32_t)psg::kCursorPushes) {
        cursor = false;
        break;
      }
      double kv = 0;
      for (uint64_t n : I.pn) kv += (double)n;
      const double piece = I.np && I.ntiles ? kv / ((double)I.np * I.ntiles) : 0.0;
      const double need = piece + 4.0 * std::sqrt(piece) + 1.0;
      I.kr = (uint32_t)std::min(3.0, std::max(1.0, std::ceil(need / 64.0)));
    }
    if (cursor) {  // one kernel instance: the jobs' largest round count
      ckr = 1;
      for (const JobInfo& I : info) ckr = std::max(ckr, I.kr);
      for (JobInfo& I : info) I.kr = ckr;
    }
    // the packed cursor form: plans (resident index) of packed-round jobs of
    // at most 256 pushes whose pointers leave the top 16 bits free (the
    // kernel keeps a piece's length there); tiles whose elements overflow one
    // pass take more groups.  Opt-in only (PSG_FORM_CURSOR), with no size
    // gate: measured slower than partition + packed kernel on cfg5 (1.34 vs
    // 0.77 ms per step)
    pcursor = index && !dense && pack && knob_cursor == 1 && tiles > 0;
    for (size_t j = 0; pcursor && j < jobs.size(); ++j) {
      const JobSpec& s = jobs[j];
      const JobInfo& I = info[j];
      if (s.dense || I.np > (uint32_t)psg::kPackCursorPushes) {
        pcursor = false;
        break;
      }
      for (size_t p = 0; p < s.pkeys.size(); ++p) {
        bool hi = ((uint64_t)s.pkeys[p] >> 48) != 0;
        for (int i = 0; i < m; ++i) hi |= ((uint64_t)s.pvals[p * m + i] >> 48) != 0;
        if (hi) pcursor = false;
      }
    }
    bxs = pcursor ? (uint32_t)psg::kPackCursorPushes : 32u;
    if (cursor || pcursor) {
      // about one chunk per workgroup slot of the chip (256 CUs x 8
      // workgroups of the cursor kernel, x 4 of the packed one)
      const uint64_t kChunkTarget = cursor ? 2048 : 1024;
      const uint64_t per = std::max<uint64_t>(1, (tiles + kChunkTarget - 1) / kChunkTarget);
      uint64_t nc = 0;
      for (JobInfo& I : info) {
        I.nch = (uint32_t)((I.ntiles + per - 1) / per);
        nc += I.nch;
      }
      nchunks = (uint32_t)nc;
    } else {
      nchunks = 0;
    }
    size_t off = align_up(sizeof(JobDev) * jobs.size(), 256);
    const size_t tiles_off = off;
    off = align_up(off + sizeof(psg::TileDesc) * tiles, 256);
    // one bucket per slot in every kernel (the same bucket map): the index
    // depends only on D and the tile size
    const bool use_index = index && !dense;
    const uint32_t iw = psg::bucket_index_words(tile);
    const size_t index_off = off;
    if (use_index) off = align_up(off + 4 * (size_t)iw * tiles, 256);
    const size_t sitems_off = off;
    off = align_up(off + 4 * sitems, 256);
    const size_t items_off = off;
    off = align_up(off + 8 * items, 256);
    // the cursor form's job and chunk tables
    const size_t cjobs_off = off;
    if (cursor) off = align_up(off + sizeof(psg::CursorJob) * jobs.size(), 256);
    const size_t chunks_off = off;
    if (cursor || pcursor) off = align_up(off + sizeof(psg::CursorChunk) * nchunks, 256);
    // one zeroed region: every job's fail counters, then the boundary words
    const size_t zero_off = off;
    size_t fail_cur = zero_off;
    {
      uint64_t npall = 0;
      for (const JobInfo& I : info) npall += I.np;
      off = align_up(off + 8 * npall, 256);
    }
    const size_t bx_off = off;
    if (cursor || pcursor) off = align_up(off + 4 * (size_t)bxs * ((size_t)nchunks + 1), 256);
    const size_t zero_end = off;
    for (size_t j = 0; j < jobs.size(); ++j) {
      const size_t np = info[j].np, nt = info[j].ntiles;
      Offs& o = offs[j];
      o.pk = off; off = align_up(off + 8 * np, 64);
      o.pv = off; off = align_up(off + 8 * np * m, 64);
      o.pn = off; off = align_up(off + 8 * np, 64);
      o.out = off; off = align_up(off + 8 * m, 64);
      o.fail = fail_cur; fail_cur += 8 * np;
      o.seg = off; off = align_up(off + 4 * (nt + 1) * np, 256);
      o.split = off;
      const bool has_split = h[j].mode == psg::kStream || (index && !jobs[j].dense && nt && np);
      if (has_split) off = align_up(off + 8 * (nt + 1), 256);
      o.dpos = off;
      if (jobs[j].dense) off = align_up(off + 8 * np, 256);
    }
    if (off > blob_bytes) {
      if (async) HIP_TRY(hipStreamSynchronize(strm));  // the old blob may be in use
      release_blob();
      HIP_TRY(hipMalloc(&blob, off));
      blob_bytes = off;
    }
    char* base = (char*)blob;
    // everything the tile descriptors and work items depend on (their
    // pointers into the blob follow from the offsets)
    std::vector<uint64_t> shape;
    const bool cacheable = !index && !cursor && !pcursor;
    if (cacheable) {
      shape = {(uint64_t)jobs.size(), tile, (uint64_t)m, (uint64_t)dtype, (uint64_t)pack,
               (uint64_t)wide, (uint64_t)(uintptr_t)blob, off, tiles_off, zero_off, items,
               sitems, tiles};
      for (size_t j = 0; j < jobs.size(); ++j) {
        const JobSpec& s = jobs[j];
        const JobDev& d = h[j];
        const Offs& o = offs[j];
        shape.insert(shape.end(), {(uint64_t)info[j].np, s.nslots, (uint64_t)(uintptr_t)s.keys,
                                   (uint64_t)s.flags, (uint64_t)s.dense, (uint64_t)d.mode,
                                   (uint64_t)d.segq, (uint64_t)d.segb, o.pk, o.pv, o.pn, o.out,
                                   o.fail, o.seg, o.split, o.dpos});
        if (d.mode == psg::kStream) shape.insert(shape.end(), info[j].pn.begin(), info[j].pn.end());
      }
    }
    const bool same = cacheable && shape == last_shape;
    const int ib = himg_cur;
    himg_cur ^= 1;
    if (himg_ev[ib]) HIP_TRY(hipEventSynchronize(himg_ev[ib]));
    else HIP_TRY(hipEventCreateWithFlags(&himg_ev[ib], hipEventDisableTiming));
    if (off > himg_cap[ib]) {
      if (himg[ib]) HIP_TRY(hipHostFree(himg[ib]));
      himg[ib] = nullptr;
      himg_cap[ib] = 0;
      HIP_TRY(hipHostMalloc((void**)&himg[ib], off));
      himg_cap[ib] = off;
      himg_dev[ib] = nullptr;
      void* dp = nullptr;
      if (hipHostGetDevicePointer(&dp, himg[ib], 0) == hipSuccess) himg_dev[ib] = dp;
      else (void)hipGetLastError();
    }
    char* img = himg[ib];
    // only the region the kernels expect zeroed (fail counters, cursor
    // boundary words): every other field of the image is written below, or
    // (seg, splitters, bucket index) by a kernel before any read.  Zeroing
    // the whole image cost ~0.1 ms per flush of a 16.8 M-slot aggregate
    memset(img + zero_off, 0, zero_end - zero_off);
    psg::TileDesc* htiles = (psg::TileDesc*)(img + tiles_off);
    uint32_t* hsitems = (uint32_t*)(img + sitems_off);
    uint64_t* hitems = (uint64_t*)(img + items_off);
    uint64_t tcur = 0, icur = 0, scur = 0;
    for (size_t j = 0; j < jobs.size(); ++j) {
      const JobSpec& s = jobs[j];
      JobInfo& I = info[j];
      const Offs& o = offs[j];
      const uint32_t np = I.np, nt = I.ntiles;
      uint64_t* hk = (uint64_t*)(img + o.pk);
      uint64_t* hv = (uint64_t*)(img + o.pv);
      for (uint32_t p = 0; p < np; ++p) {
        const uint32_t c = I.slot[p];
        hk[p] = (uint64_t)s.pkeys[c];
        for (int i = 0; i < m; ++i) hv[(size_t)p * m + i] = (uint64_t)s.pvals[(size_t)c * m + i];
      }
      memcpy(img + o.pn, I.pn.data(), 8 * np);
      if (s.dense) {
        // seg(p, t) = clamp(t * tile - dpos[p], 0, n_p), tile-major (segq 1, segb np)
        uint64_t* hd = (uint64_t*)(img + o.dpos);
        uint32_t* hs = (uint32_t*)(img + o.seg);
        for (uint32_t p = 0; p < np; ++p) {
          const uint64_t dp = s.dpos[I.slot[p]], n = I.pn[p];
          hd[p] = dp;
          for (uint32_t t = 0; t <= nt; ++t) {
            const uint64_t edge = (uint64_t)t * tile;
            const uint64_t v = edge <= dp ? 0 : std::min<uint64_t>(edge - dp, n);
            hs[(size_t)t * np + p] = (uint32_t)v;
          }
        }
      }
      memcpy(img + o.out, s.out.data(), 8 * m);
      JobDev& d = h[j];
      d.dkeys = s.keys;
      d.pkeys = (const uint64_t* const*)(base + o.pk);
      d.pn = (const uint64_t*)(base + o.pn);
      d.seg = (uint32_t*)(base + o.seg);
      d.fail = (unsigned long long*)(base + o.fail);
      // search-mode jobs of plans read their boundary keys from the splitter
      // array (64 consecutive boundaries: one coalesced read per wave instead
      // of one line of D per boundary)
      const bool has_split = d.mode == psg::kStream || (index && !s.dense && nt && np);
      d.split = has_split ? (uint64_t*)(base + o.split) : nullptr;
      I.seg = d.seg;
      I.fail = d.fail;
      if (same) continue;  // descriptors and items already on the device
      if (nt && np && !s.dense) {  // as counted above: dense jobs have no items
        if (d.mode == psg::kSearch) {
          if (index) {
            const uint64_t ns = (std::max<uint64_t>(nt + 1, np) + 255) / 256;
            for (uint64_t b = 0; b < ns; ++b) hsitems[scur++] = (uint32_t)j;
          }
          const uint64_t ng = (nt + 64) / 64;
          for (uint64_t g = 0; g < ng; ++g)  // group-major: a boundary group's pushes adjacent
            for (uint32_t p = 0; p < np; ++p)
              hitems[icur++] = (uint64_t)j << 37 | (uint64_t)p << 24 | g;
        } else {
          const uint64_t ns = (std::max<uint64_t>(nt + 1, np) + 255) / 256;
          for (uint64_t b = 0; b < ns; ++b) hsitems[scur++] = (uint32_t)j;
          for (uint32_t p = 0; p < np; ++p) {
            const uint64_t nc = (I.pn[p] + psg::kStreamChunk - 1) / psg::kStreamChunk;
            for (uint64_t c = 0; c < nc; ++c)
              hitems[icur++] = (uint64_t)j << 37 | (uint64_t)p << 24 | c;
          }
        }
      }
      for (uint32_t t = 0; t < nt; ++t) {
        psg::TileDesc& T = htiles[tcur++];
        const uint64_t slot0 = (uint64_t)t * tile;
        T.dk = s.keys + slot0;
        T.seg = d.seg + (size_t)t * d.segb;
        T.pkeys = d.pkeys;
        T.pvals = (const void* const*)(base + o.pv);
        T.pn = d.pn;
        T.out = (void* const*)(base + o.out);
        T.fail = d.fail;
        T.slot0 = slot0;
        T.nt = (uint32_t)std::min<uint64_t>(tile, s.nslots - slot0);
        T.np = np;
        T.stride = d.segq;
        T.segb = d.segb;
        T.flags = s.flags | (t + 1 == nt ? psg::kFlagLastTile : 0u);
        T.dpos = s.dense ? (const uint64_t*)(base + o.dpos) : nullptr;
        T.bt = use_index ? (const uint32_t*)(base + index_off) + (size_t)(tcur - 1) * iw : nullptr;
      }
    }
    if (cursor) {
      psg::CursorJob* hcj = (psg::CursorJob*)(img + cjobs_off);
      psg::CursorChunk* hch = (psg::CursorChunk*)(img + chunks_off);
      chunk0.assign(jobs.size(), 0);
      uint64_t tbase = 0, ccur = 0;
      for (size_t j = 0; j < jobs.size(); ++j) {
        const JobInfo& I = info[j];
        const JobDev& d = h[j];
        psg::CursorJob& c = hcj[j];
        c.dkeys = jobs[j].keys;
        c.nslots = jobs[j].nslots;
        c.pkeys = d.pkeys;
        c.pvals = (const void* const*)(base + offs[j].pv);
        c.pn = d.pn;
        c.out = (void* const*)(base + offs[j].out);
        c.fail = d.fail;
        c.seg = d.seg;
        c.bt = (const uint32_t*)(base + index_off) + (size_t)tbase * iw;
        c.np = I.np;
        c.ntiles = I.ntiles;
        c.flags = jobs[j].flags;
        c.kr = I.kr;
        chunk0[j] = (uint32_t)ccur;
        for (uint32_t k = 0; k < I.nch; ++k) {
          psg::CursorChunk& ch = hch[ccur++];
          ch.job = (uint32_t)j;
          ch.t0 = (uint32_t)((uint64_t)k * I.ntiles / I.nch);
          ch.t1 = (uint32_t)((uint64_t)(k + 1) * I.ntiles / I.nch);
        }
        tbase += I.ntiles;
      }
      if (ccur != nchunks) return fail(PSG_ERR_DEVICE, "cursor chunks %llu/%u",
                                       (unsigned long long)ccur, nchunks);
    }
    if (pcursor) {  // chunks index the tile descriptors
      psg::CursorChunk* hch = (psg::CursorChunk*)(img + chunks_off);
      chunk0.assign(jobs.size(), 0);
      uint64_t tbase = 0, ccur = 0;
      for (size_t j = 0; j < jobs.size(); ++j) {
        const JobInfo& I = info[j];
        chunk0[j] = (uint32_t)ccur;
        for (uint32_t k = 0; k < I.nch; ++k) {
          psg::CursorChunk& ch = hch[ccur++];
          ch.job = (uint32_t)j;
          ch.t0 = (uint32_t)(tbase + (uint64_t)k * I.ntiles / I.nch);
          ch.t1 = (uint32_t)(tbase + (uint64_t)(k + 1) * I.ntiles / I.nch);
        }
        tbase += I.ntiles;
      }
      if (ccur != nchunks) return fail(PSG_ERR_DEVICE, "cursor chunks %llu/%u",
                                       (unsigned long long)ccur, nchunks);
    }
    if (same) {
      icur = items;
      scur = sitems;
      tcur = tiles;
    }
    // the fill must match the sizing pass exactly (the image regions are
    // packed back to back): a mismatch is a bug, never launched
    if (icur != items || scur != sitems || tcur != tiles)
      return fail(PSG_ERR_DEVICE, "job table: %llu/%llu items, %llu/%llu split items, "
                  "%llu/%llu tiles", (unsigned long long)icur, (unsigned long long)items,
                  (unsigned long long)scur, (unsigned long long)sitems,
                  (unsigned long long)tcur, (unsigned long long)tiles);
    memcpy(img, h.data(), sizeof(JobDev) * h.size());
    ntiles = (uint32_t)tiles;
    nitems = (uint32_t)items;
    nsplit = (uint32_t)scur;
    d_jobs = (JobDev*)blob;
    d_tiles = (psg::TileDesc*)(base + tiles_off);
    d_split_items = (uint32_t*)(base + sitems_off);
    d_items = (uint64_t*)(base + items_off);
    d_cjobs = cursor ? (psg::CursorJob*)(base + cjobs_off) : nullptr;
    d_chunks = cursor || pcursor ? (psg::CursorChunk*)(base + chunks_off) : nullptr;
    d_bx = cursor || pcursor ? (uint32_t*)(base + bx_off) : nullptr;
    d_zero = base + zero_off;
    zero_bytes = zero_end - zero_off;
    // the image is small: a DMA copy's fixed cost exceeds its transfer time.
    // Same shape: the job tables and the regions after the items only
    const bool zc_ok = zero_copy && himg_dev[ib] && (((uintptr_t)himg_dev[ib] | (uintptr_t)blob) & 15u) == 0;
    if (same && zc_ok) {
      psg::HostCopyBatch cb;
      cb.n = 2;
      cb.d[0] = psg::HostCopyDesc{himg_dev[ib], blob, (uint64_t)tiles_off};
      cb.d[1] = psg::HostCopyDesc{(const char*)himg_dev[ib] + zero_off, base + zero_off,
                                  (uint64_t)(off - zero_off)};
      HIP_TRY(psg::launch_host_copy_batch(cb, strm));
    } else if (same) {
      HIP_TRY(hipMemcpyAsync(blob, img, tiles_off, hipMemcpyHostToDevice, strm));
      HIP_TRY(hipMemcpyAsync(base + zero_off, img + zero_off, off - zero_off,
                             hipMemcpyHostToDevice, strm));
    } else if (zc_ok) {
      HIP_TRY(psg::launch_host_copy(blob, himg_dev[ib], off, strm));
    } else {
      HIP_TRY(hipMemcpyAsync(blob, img, off, hipMemcpyHostToDevice, strm));
    }
    if (cacheable) last_shape.swap(shape);
    else last_shape.clear();
    HIP_TRY(hipEventRecord(himg_ev[ib], strm));
    if (use_index)
      HIP_TRY(psg::launch_bucket_index(d_tiles, ntiles, tile,
                                       (uint32_t*)((char*)blob + index_off), strm));
    split_once = index && nsplit > 0 && !dense && !cursor && !pcursor;
    all_search = true;
    for (const JobDev& d : h) all_search = all_search && d.mode == psg::kSearch;
    if (split_once)  // the splitter pass alone (it also clears the fail counters once)
      HIP_TRY(psg::launch_partition(d_jobs, d_split_items, nsplit, nullptr, 0, strm));
    if (!async) HIP_TRY(hipStreamSynchronize(strm));
    return PSG_OK;
  }

  int run_stage(int stage, hipStream_t s) const {
    if (h.empty()) return PSG_OK;
    if (stage == 0) {
      if (cursor || pcursor)  // fail counters, boundaries
        HIP_TRY(hipMemsetAsync(d_zero, 0, zero_bytes, s));
      else if (!dense)
        HIP_TRY(psg::launch_partition(d_jobs, d_split_items, split_once ? 0u : nsplit, d_items,
                                      nitems, s, all_search));
    } else if (cursor)
      HIP_TRY(psg::launch_aggregate_cursor(dtype, m, (int)ckr, d_cjobs, d_chunks, nchunks, d_bx, s));
    else if (dense)
      HIP_TRY(psg::launch_aggregate_dense(dtype, m, d_tiles, ntiles, s));
    else if (pack)
      HIP_TRY(psg::launch_aggregate_tile_packed(dtype, m, d_tiles, ntiles, s,
                                                pcursor ? d_chunks : nullptr, nchunks, d_bx));
    else
      HIP_TRY(psg::launch_aggregate_tile(dtype, m, d_tiles, ntiles, wide ? 1 : 0, s));
    return PSG_OK;
  }

  int run(hipStream_t s) const {
    if (int rc = run_stage(0, s)) return rc;
    return run_stage(1, s);
  }

  // matched[p] per caller push (empty pushes 0): covered elements minus
  // match failures; the stream must be idle.
  int matched(std::vector<uint64_t>& out) const {
    out.clear();
    for (size_t j = 0; j < h.size(); ++j) {
      const JobInfo& I = info[j];
      std::vector<uint64_t> mt(I.ncaller, 0);
      const uint32_t np = I.np, nt = I.ntiles;
      if (np && nt) {
        std::vector<unsigned long long> f(np);
        std::vector<uint32_t> first(np), last(np);
        const size_t pitch = 4 * (size_t)I.segq;
        const size_t segb = I.segq == 1 ? np : 1;  // tile-major / push-major
        HIP_TRY(hipMemcpy(f.data(), I.fail, 8 * np, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy2D(first.data(), 4, I.seg, pitch, 4, np, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy2D(last.data(), 4, I.seg + (size_t)nt * segb, pitch, 4, np,
                            hipMemcpyDeviceToHost));
        // cursor form: a chunk boundary where the chunks' cursors disagree
        // (start != the previous chunk's end) means an unsorted push
        std::vector<uint32_t> bxw;
        const bool cur = cursor || pcursor;
        if (cur && I.nch > 1) {
          bxw.resize((size_t)bxs * (I.nch - 1));
          HIP_TRY(hipMemcpy(bxw.data(), d_bx + (size_t)bxs * (chunk0[j] + 1), 4 * bxw.size(),
                            hipMemcpyDeviceToHost));
        }
        for (uint32_t p = 0; p < np; ++p) {
          const uint64_t covered = last[p] >= first[p] ? (uint64_t)(last[p] - first[p]) : 0;
          uint64_t v = covered >= f[p] ? covered - f[p] : 0;
          bool torn = false;
          for (size_t k = 0; k + 1 < I.nch && cur; ++k) torn |= bxw[(size_t)bxs * k + p] != 0;
          if (torn && v >= I.pn[p]) v = I.pn[p] - 1;
          mt[I.slot[p]] = v;
        }
      }
      out.insert(out.end(), mt.begin(), mt.end());
    }
    return PSG_OK;
  }
};

}  // namespace

// ==========================================================================
// plan API (device-resident batch)
// ==========================================================================
struct psg_plan {
  JobTable table;
  hipStream_t last = nullptr;
  uint64_t bytes = 0, kv = 0;
};

// ==========================================================================
// server context
// ==========================================================================
namespace {

// Device keys of one push.  Shared: a key-cache entry (RNode::key_cache_,
// remote_node.h:92-93) and every pending push that was restored from it
// hold the same resident copy; the last owner returns it to the pool.
struct KeyBuf {
  uint64_t* d = nullptr;
  size_t n = 0, bytes = 0;
  // a dense push's keys left in the caller's pinned memory (d null): the
  // device-visible address its order check reads
  const uint64_t* host = nullptr;
};
using KeyRef = std::shared_ptr<KeyBuf>;

struct Channel {
  uint64_t* d_keys = nullptr;
  size_t n = 0, kbytes = 0;
  // host mirror of key_[chl] (findRange, key copies, psg_push's dense
  // test): after a key union the device key set is copied into pinned
  // memory asynchronously; readers wait for that copy (mirror())
  uint64_t* hk = nullptr;
  size_t hcap = 0;
  hipEvent_t hev = nullptr;
  bool hpend = false;
  const uint64_t* mirror() {
    if (hpend) {
      (void)hipEventSynchronize(hev);
      hpend = false;
    }
    return hk;
  }
  void* d_vals = nullptr;
  size_t nvals = 0;
  // Darling server state (darling.h:38-39): delta_[grp], active_set_[grp]
  double* d_delta = nullptr;
  uint32_t* d_active = nullptr;
  size_t dn = 0;
};

struct PendingPush {
  KeyRef keys;
  void* vblock = nullptr;  // the m value arrays
  size_t vbytes = 0;
  void* d_vals[psg::kMaxM] = {};
  int m = 0;  // value arrays of this push (the aggregate's list grows to the largest)
  uint64_t n = 0;
  // a contiguous slice of the server keys (psg_push's dense test): the merge
  // reads D[dpos, dpos + n) of the aggregate's range in place of the keys
  bool dense = false;
  uint64_t dpos = 0;           // position of the first key in [lo, hi)
  const uint64_t* kd = nullptr;  // D + lo + dpos
  // a compressed push's staging block (its parts, decoded on `copy`): held
  // until the merge that follows the decode
  void* sblock = nullptr;
  size_t sbytes = 0;
  // its parts still to decode (device addresses): input [cbeg, cend),
  // output cdst of ccap bytes -- decoded together with the other pending
  // compressed pushes right before the merge that needs them
  int cparts = 0;
  uint64_t cbeg[psg::kMaxM + 1] = {}, cend[psg::kMaxM + 1] = {};
  uint64_t cdst[psg::kMaxM + 1] = {}, ccap[psg::kMaxM + 1] = {};
};

// recved_val_[t] (kv_vector.h:189-196, 110-129): a list of value arrays that
// grows when a push brings more arrays than the earlier ones; array i is
// assigned by the first push holding an i-th array and added to by the later
// ones that hold one (a push without it leaves it alone)
// an aggregate's device counters: unmatched keys, compressed parts that failed
// to decode, pushes whose keys do not match their carried signature
constexpr size_t kBadBytes = 32;

struct Aggregate {
  int chl = 0, m = 0;                // m: arrays so far (the largest push's)
  size_t lo = 0, hi = 0;
  void* d_out[psg::kMaxM] = {};
  std::vector<PendingPush> pending;
  uint64_t folded = 0;               // pushes already merged into d_out
  uint64_t folded_arr[psg::kMaxM] = {};  // of them, those holding array i
  uint64_t expected_total = 0;
  // device: [0] pushed keys not matched so far, [1] compressed parts that
  // failed to decode (psg_push_compressed reports them here, asynchronously),
  // [2] pushes whose keys do not match their carried signature
  unsigned long long* d_bad = nullptr;
};

// key_cache_ of remote node `sender`, index (key_channel, key_range)
// (remote_node.cc:98-99,141-142)
struct CacheKey {
  int sender, chl;
  uint64_t kb, ke;
  bool operator<(const CacheKey& o) const {
    if (sender != o.sender) return sender < o.sender;
    return chl != o.chl ? chl < o.chl : kb != o.kb ? kb < o.kb : ke < o.ke;
  }
};
// The device check of a carried signature (keys + values message): its
// counter and the event after it on `copy`.  The entry that stored those
// keys is restorable only once the check passed; the reference checks before
// it stores (remote_node.cc:161-165).
struct SigCheck {
  unsigned long long* d = nullptr;  // the device counter (a slot of a counter slab)
  unsigned long long* h = nullptr;  // its pinned host copy, landed before `ev`
  uint32_t slot = 0;
  hipEvent_t ev = nullptr;
};
using SigCheckRef = std::shared_ptr<SigCheck>;
struct CacheEntry {
  uint32_t sig = 0;
  KeyRef keys;
  SigCheckRef chk;  // null: checked (or stored by a key-only message, checked at once)
};

// pinned host memory, and the address the device reads it at
bool host_pinned(const void* p, const void** dev = nullptr) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error for us
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  if (dev) {
    // the attribute's device pointer is the allocation's base: offset it
    const char* hb = (const char*)a.hostPointer;
    const char* db = (const char*)a.devicePointer;
    *dev = (hb && db) ? (const void*)(db + ((const char*)p - hb)) : nullptr;
  }
  return true;
}


// FreqencyFilter<uint64> of one channel (CountMin n_, k_, table)
struct Filter {
  uint8_t* d_table = nullptr;  // n byte counters (countmin.h:69)
  uint32_t n = 0;
  int k = 1;
  // the binned insert's records (psg_countmin.hip), grown on demand; the
  // filter's inserts are ordered on one stream (the context's, or the
  // caller's of psg_freq_insert_dev)
  void* d_bins = nullptr;
  size_t bins_bytes = 0;
  // the caller's stream of the last psg_freq_*_dev call: the table is not
  // recycled (clear / resize) before the kernels enqueued there finished
  hipStream_t ext = nullptr;
  bool ext_used = false;
  void sync_ext() {
    if (ext_used) (void)hipStreamSynchronize(ext);
    ext_used = false;
  }
  // the filter's operations run in call order whatever streams they are
  // enqueued on (the reference's calls are sequential): each one waits for
  // the event recorded after the previous one when their streams differ.
  // The binned insert reuses d_bins and writes table dwords with plain
  // read-modify-write stores, so two inserts must never overlap.
  hipEvent_t last = nullptr;
  hipStream_t last_s = nullptr;
};

}  // namespace

#ifndef PSG_SPIN
#define PSG_SPIN 1
#endif
// the host waits for the end of a call's device work by polling its event
// for a bounded time: a pushing caller is blocked on it anyway, and the poll
// sees a short wait's completion sooner than a blocking wait's wake-up (the
// e2e pinned path waits once per push).  Past ~50 us it
// yields to a blocking wait, so threads waiting on long device work (the
// loopback exchange's ranks, several contexts) do not each burn a core
// (ADVICE r05).
static hipError_t spin_wait(hipEvent_t e) {
#if PSG_SPIN
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0;; ++i) {
    const hipError_t q = hipEventQuery(e);
    if (q != hipErrorNotReady) return q;
    if ((i & 15) == 15 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(50))
      break;
  }
  return hipEventSynchronize(e);
#else
  return hipEventSynchronize(e);
#endif
}

struct psg_ctx {
  int device = 0;
  int dtype = PSG_F32;
  unsigned flags = PSG_SERIAL_MATCH;
  hipStream_t stream = nullptr;  // kernels, D2H
  hipStream_t copy = nullptr;    // H2D of pushes / keys / values
  hipEvent_t copy_ev = nullptr;
  hipEvent_t done_ev = nullptr;  // end of a call's work on `stream` (spin_wait)

  std::mutex mu;
  std::unordered_map<int, Channel> ch;
  std::map<int, Aggregate> agg;
  std::map<CacheKey, CacheEntry> kcache;
  std::unordered_map<int, Filter> ff;
  JobTable table;
  unsigned long long* d_small = nullptr;  // 32 device words: counters, crc args
  unsigned long long* d_vio_slots = nullptr;  // psg::kVioSlots x 64 B, zero between updates
  unsigned long long* h_small = nullptr;  // 32 pinned host words
  // signature-check counters, pooled: slabs of kCtrSlab device
  // words and as many pinned host words their results are copied back into;
  // slot i lives in slab i / kCtrSlab
  static constexpr uint32_t kCtrSlab = 256;
  std::vector<unsigned long long*> ctr_d, ctr_h;
  std::vector<uint32_t> ctr_free;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  size_t flush_pushes = psg::kMaxPush;  // pushes per aggregate launch

  // ---- device block pool.  Freed push, key and aggregate blocks, by size: a
  // server sees the same shapes every iteration, so after the first one no
  // push allocates.  A block is returned with an event recorded on `stream`
  // (the kernels that read it were enqueued there before); a writer on
  // another stream waits for that event before reusing it.
  struct Pooled {
    void* p;
    hipEvent_t ev;
  };
  std::multimap<size_t, Pooled> pool;
  size_t pool_bytes = 0;
  // the real size of every block this pool made (carved or allocated): a
  // reused block may be up to twice the size asked for, and the counts of
  // the pool and the slabs add and subtract that same size
  std::unordered_map<const void*, size_t> bsize;
  size_t real_size(const void* p, size_t b) const {
    auto it = bsize.find(p);
    return it == bsize.end() ? b : it->second;
  }
  std::vector<hipEvent_t> free_ev;
  static constexpr size_t kPoolCap = size_t(8) << 30;
  // ---- slabs: blocks up to kSlabBlock bytes (staged pushes, cached keys,
  // aggregates of a shard's range) are carved from kSlab-byte allocations
  // by a bump pointer and then cycle through the pool (never freed on their
  // own), so an aggregate's pushes sit back to back in a few large mappings
  // instead of one allocation each: the sparse kernel's tiles, which read a
  // few keys of each of hundreds of pushes, then touch far fewer address
  // translations (cfg5: 0.99 -> 0.74 ms for the same kernel, DESIGN.md 4.3;
  // bench.py --layout arena is this layout for the plan API)
#ifndef PSG_SLAB_BLOCK
#define PSG_SLAB_BLOCK (size_t(16) << 20)  // A/B builds: 0 = no slabs
#endif
  static constexpr size_t kSlab = size_t(256) << 20, kSlabBlock = PSG_SLAB_BLOCK;
  // carved: bytes handed out by the bump pointer; back: bytes of those
  // returned (in the pool, or dropped after a failed event).  A slab with
  // back == carved holds no live block and can be freed whole (reclaim_slabs:
  // when an allocation fails, or when idle carved bytes pass kPoolCap), so
  // blocks stranded by drifting sizes do not hold HBM for the context's life
  struct Slab {
    char* p;
    size_t size, carved, back;
  };
  std::vector<Slab> slabs;
  char* slab_cur = nullptr;
  size_t slab_left = 0;
  size_t slab_idle = 0;  // sum of back over the slabs
  int slab_of(const void* p) const {
    for (size_t i = 0; i < slabs.size(); ++i)
      if ((const char*)p >= slabs[i].p && (const char*)p < slabs[i].p + slabs[i].size)
        return (int)i;
    return -1;
  }
  bool in_slab(const void* p) const { return slab_of(p) >= 0; }
  // frees every slab none of whose blocks is live; returns the bytes freed
  size_t reclaim_slabs() {
    bool any = false;
    for (const Slab& s : slabs) any |= s.carved && s.back == s.carved;
    if (!any) return 0;
    // pooled blocks carry events on `stream`: once it is idle none is read
    (void)hipStreamSynchronize(stream);
    (void)hipStreamSynchronize(copy);
    size_t freed = 0;
    for (size_t i = 0; i < slabs.size();) {
      Slab& s = slabs[i];
      if (!(s.carved && s.back == s.carved)) {
        ++i;
        continue;
      }
      for (auto it = pool.begin(); it != pool.end();) {
        const char* q = (const char*)it->second.p;
        if (q >= s.p && q < s.p + s.size) {
          free_ev.push_back(it->second.ev);
          it = pool.erase(it);
        } else {
          ++it;
        }
      }
      for (auto it = bsize.begin(); it != bsize.end();) {
        const char* q = (const char*)it->first;
        it = (q >= s.p && q < s.p + s.size) ? bsize.erase(it) : std::next(it);
      }
      if (slab_cur >= s.p && slab_cur <= s.p + s.size) {
        slab_cur = nullptr;
        slab_left = 0;
      }
      slab_idle -= s.back;
      freed += s.size;
      (void)hipFree(s.p);
      slabs.erase(slabs.begin() + (ptrdiff_t)i);
    }
    return freed;
  }

  int event(hipEvent_t* e) {
    if (!free_ev.empty()) {
      *e = free_ev.back();
      free_ev.pop_back();
      return PSG_OK;
    }
    HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return PSG_OK;
  }

  int dev_get(size_t b, void** p, hipStream_t writer) {
    b = align_up(b ? b : 1, 4096);
    auto it = pool.lower_bound(b);
    if (it != pool.end() && it->first <= 2 * b) {
      *p = it->second.p;
      if (writer != stream) HIP_TRY(hipStreamWaitEvent(writer, it->second.ev, 0));
      free_ev.push_back(it->second.ev);
      const int si = slab_of(*p);
      if (si < 0) {
        pool_bytes -= it->first;
      } else {
        slabs[si].back -= it->first;
        slab_idle -= it->first;
      }
      pool.erase(it);
      return PSG_OK;
    }
    if (b <= kSlabBlock) {
      if (slab_left < b) {
        char* sp = nullptr;
        if (hipMalloc((void**)&sp, kSlab) != hipSuccess) {
          (void)hipGetLastError();
          if (reclaim_slabs() && hipMalloc((void**)&sp, kSlab) != hipSuccess) {
            (void)hipGetLastError();
            sp = nullptr;
          }
        }
        if (sp) {
          slabs.push_back(Slab{sp, kSlab, 0, 0});
          slab_cur = sp;
          slab_left = kSlab;
        }  // else no room for a slab: an allocation of its own
      }
      if (slab_left >= b) {
        *p = slab_cur;
        slab_cur += b;
        slab_left -= b;
        slabs[(size_t)slab_of(*p)].carved += b;
        bsize[*p] = b;
        return PSG_OK;
      }
    }
    if (hipMalloc(p, b) != hipSuccess) {
      (void)hipGetLastError();
      // idle slabs (blocks stranded by sizes that drifted) go back first
      if (!reclaim_slabs()) return fail(PSG_ERR_OOM, "device allocation of %zu bytes", b);
      HIP_TRY(hipMalloc(p, b));
    }
    bsize[*p] = b;
    return PSG_OK;
  }
  void dev_put(void* p, size_t b) {
    if (!p) return;
    // a deferred copy may target the block: issue it and order it before
    // the block's release event on `stream`
    if (zc.n) (void)join_copy();
    b = real_size(p, align_up(b ? b : 1, 4096));
    const int si = slab_of(p);  // a carved block is pooled (or counted back) always
    const bool carved = si >= 0;
    if (carved) {
      slabs[si].back += b;
      slab_idle += b;
    }
    hipEvent_t e = nullptr;
    if ((!carved && pool_bytes + b > kPoolCap) || event(&e) != PSG_OK ||
        hipEventRecord(e, stream) != hipSuccess) {
      if (e) free_ev.push_back(e);
      (void)hipStreamSynchronize(stream);
      if (!carved) {  // a carved block goes with its slab
        (void)hipFree(p);
        bsize.erase(p);
      }
      return;
    }
    pool.emplace(b, Pooled{p, e});
    if (!carved) pool_bytes += b;
    // idle carved bytes are bounded like the pool: whole idle slabs go back
    if (carved && slab_idle > kPoolCap) (void)reclaim_slabs();
  }
  void pool_release() {
    for (auto& kv : pool) {
      if (!in_slab(kv.second.p)) (void)hipFree(kv.second.p);
      (void)hipEventDestroy(kv.second.ev);
    }
    pool.clear();
    pool_bytes = 0;
    bsize.clear();
    for (auto& sl : slabs) (void)hipFree(sl.p);
    slabs.clear();
    slab_cur = nullptr;
    slab_left = 0;
    slab_idle = 0;
    for (hipEvent_t e : free_ev) (void)hipEventDestroy(e);
    free_ev.clear();
  }

  // the carried signature of resident keys checked on `copy` into a counter
  // of its own (the entry's), after the key copy, and -- one CRC for both
  //  -- into the aggregate's signature counter `agg` when given
  int ctr_get(uint32_t* slot) {
    if (ctr_free.empty()) {
      unsigned long long *d = nullptr, *h = nullptr;
      HIP_TRY(hipMalloc((void**)&d, 8 * kCtrSlab));
      if (hipHostMalloc((void**)&h, 8 * kCtrSlab) != hipSuccess) {
        (void)hipFree(d);
        return fail(PSG_ERR_DEVICE, "signature counter slab");
      }
      const uint32_t base = (uint32_t)ctr_d.size() * kCtrSlab;
      ctr_d.push_back(d);
      ctr_h.push_back(h);
      for (uint32_t i = kCtrSlab; i-- > 0;) ctr_free.push_back(base + i);
    }
    *slot = ctr_free.back();
    ctr_free.pop_back();
    return PSG_OK;
  }
  void ctr_release() {
    for (auto* d : ctr_d) (void)hipFree(d);
    for (auto* h : ctr_h) (void)hipHostFree(h);
    ctr_d.clear();
    ctr_h.clear();
    ctr_free.clear();
  }
  int sig_check_pending(const KeyRef& k, uint32_t sig, SigCheckRef* out,
                        unsigned long long* agg = nullptr) {
    SigCheck* s = new SigCheck();
    if (int rc = ctr_get(&s->slot)) {
      delete s;
      return rc;
    }
    s->d = ctr_d[s->slot / kCtrSlab] + s->slot % kCtrSlab;
    s->h = ctr_h[s->slot / kCtrSlab] + s->slot % kCtrSlab;
    int rc = event(&s->ev);
    if (rc == PSG_OK && (hipMemsetAsync(s->d, 0, 8, copy) != hipSuccess ||
                         psg::launch_sig_check((const uint8_t*)k->d, 8 * k->n, PSG_MAX_SIG_LEN,
                                               sig, s->d, copy, agg) != hipSuccess ||
                         hipMemcpyAsync(s->h, s->d, 8, hipMemcpyDeviceToHost, copy) != hipSuccess ||
                         hipEventRecord(s->ev, copy) != hipSuccess))
      rc = fail(PSG_ERR_DEVICE, "signature check launch");
    if (rc != PSG_OK) {
      (void)hipStreamSynchronize(copy);
      if (s->ev) free_ev.push_back(s->ev);
      ctr_free.push_back(s->slot);
      delete s;
      return rc;
    }
    *out = SigCheckRef(s, [this](SigCheck* q) {
      (void)hipEventSynchronize(q->ev);  // the counter slot is not reused under the check
      free_ev.push_back(q->ev);
      ctr_free.push_back(q->slot);
      delete q;
    });
    return PSG_OK;
  }
  // the result of a pending check: a wait for its event (once per stored
  // entry); the count is already in pinned host memory
  int sig_check_result(const SigCheckRef& s, bool* ok) {
    HIP_TRY(hipEventSynchronize(s->ev));
    *ok = *(volatile unsigned long long*)s->h == 0;
    return PSG_OK;
  }

  int new_keys(size_t n, KeyRef* out) {
    KeyBuf* k = new KeyBuf();
    k->n = n;
    k->bytes = 8 * n;
    if (int rc = dev_get(k->bytes, (void**)&k->d, copy)) {
      delete k;
      return rc;
    }
    *out = KeyRef(k, [this](KeyBuf* q) {
      dev_put(q->d, q->bytes);
      delete q;
    });
    return PSG_OK;
  }

  // ---- host -> device on `copy`.  The caller's buffer is free on return:
  // pinned memory is copied directly and waited for; pageable memory is
  // copied by the CPU into a pinned staging ring whose DMA runs on while
  // the caller goes on (no wait).
  char* ring = nullptr;
  size_t ring_cap = 0, ring_head = 0;
  struct Flight {
    size_t off, len;
    hipEvent_t ev;
  };
  std::deque<Flight> fly;
  static constexpr size_t kRingBytes = size_t(64) << 20;
  static constexpr size_t kRingPiece = size_t(4) << 20;

  int ring_reserve(size_t len, size_t* off) {
    if (!ring) {
      HIP_TRY(hipHostMalloc((void**)&ring, kRingBytes));
      ring_cap = kRingBytes;
    }
    if (ring_head + len > ring_cap) ring_head = 0;
    int last = -1;
    for (size_t i = 0; i < fly.size(); ++i)
      if (fly[i].off < ring_head + len && ring_head < fly[i].off + fly[i].len) last = (int)i;
    if (last >= 0) {  // events complete in order on `copy`
      HIP_TRY(hipEventSynchronize(fly[last].ev));
      for (int i = 0; i <= last; ++i) {
        free_ev.push_back(fly.front().ev);
        fly.pop_front();
      }
    }
    *off = ring_head;
    ring_head += len;
    return PSG_OK;
  }

  bool pinned_wait = false;  // a pinned copy of this call is still in flight
  bool zero_copy = true;     // pinned buffers read by a kernel, not a DMA copy
  // held pushes' pinned buffers (PSG_HOLD_BUFFERS: valid until received):
  // copied by one zero-copy launch when the merge needs them (join_copy)
  psg::HostCopyBatch zc;
  // a group of copies the caller flushes as one zero-copy launch (a
  // compressed push's parts), held buffers or not
  bool zc_group = false;
  int zc_flush() {
    if (zc.n == 0) return PSG_OK;
    const hipError_t e = psg::launch_host_copy_batch(zc, copy);
    zc.n = 0;
    HIP_TRY(e);
    return PSG_OK;
  }
  // `defer`: a push's keys or values, read by nothing before the merge
  int h2d(void* dst, const void* src, size_t len, bool defer = false) {
    if (!len) return PSG_OK;
    const void* sdev = nullptr;
    if (host_pinned(src, &sdev)) {
      // the GPU reads the caller's pinned buffer itself when both ends are
      // 16-B aligned (a DMA copy's fixed cost dominates at push sizes)
      const bool zok = zero_copy && sdev && (((uintptr_t)sdev | (uintptr_t)dst) & 15u) == 0;
      if (zok && ((defer && (flags & PSG_HOLD_BUFFERS)) || zc_group)) {
        if (zc.n == (uint32_t)psg::kHostCopyBatch)
          if (int rc = zc_flush()) return rc;
        zc.d[zc.n++] = psg::HostCopyDesc{sdev, dst, (uint64_t)len};
        if (!(flags & PSG_HOLD_BUFFERS)) pinned_wait = true;
        return PSG_OK;
      }
      if (zok)
        HIP_TRY(psg::launch_host_copy(dst, sdev, len, copy));
      else
        HIP_TRY(hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, copy));
      pinned_wait = !(flags & PSG_HOLD_BUFFERS);
      return PSG_OK;
    }
    for (size_t done = 0; done < len;) {
      const size_t piece = std::min(len - done, kRingPiece);
      size_t off;
      if (int rc = ring_reserve(piece, &off)) return rc;
      memcpy(ring + off, (const char*)src + done, piece);
      HIP_TRY(hipMemcpyAsync((char*)dst + done, ring + off, piece, hipMemcpyHostToDevice, copy));
      hipEvent_t e;
      if (int rc = event(&e)) return rc;
      HIP_TRY(hipEventRecord(e, copy));
      fly.push_back(Flight{off, piece, e});
      done += piece;
    }
    return PSG_OK;
  }

  // device -> host on `stream`: into pinned memory the GPU writes itself
  // (zero-copy kernel, no DMA fixed cost), else a DMA copy
  int d2h(void* dst, const void* src, size_t len) {
    if (!len) return PSG_OK;
    const void* ddev = nullptr;
    if (zero_copy && host_pinned(dst, &ddev) && ddev &&
        (((uintptr_t)ddev | (uintptr_t)src) & 15u) == 0)
      HIP_TRY(psg::launch_host_copy((void*)ddev, src, len, stream));
    else
      HIP_TRY(hipMemcpyAsync(dst, src, len, hipMemcpyDeviceToHost, stream));
    return PSG_OK;
  }

  // end of an API call that staged caller buffers: they must be free on
  // return unless the caller holds them (PSG_HOLD_BUFFERS)
  int h2d_finish() {
    if (!pinned_wait) return PSG_OK;
    pinned_wait = false;
    HIP_TRY(hipEventRecord(copy_ev, copy));
    HIP_TRY(spin_wait(copy_ev));
    return PSG_OK;
  }

  // work enqueued on `stream` from now on sees every H2D issued so far
  int join_copy() {
    if (int rc = zc_flush()) return rc;
    HIP_TRY(hipEventRecord(copy_ev, copy));
    HIP_TRY(hipStreamWaitEvent(stream, copy_ev, 0));
    return PSG_OK;
  }

  int ensure_scratch(size_t b) {
    if (b <= scratch_bytes) return PSG_OK;
    HIP_TRY(hipStreamSynchronize(stream));
    if (scratch) HIP_TRY(hipFree(scratch));
    scratch = nullptr;
    scratch_bytes = 0;
    HIP_TRY(hipMalloc(&scratch, b));
    scratch_bytes = b;
    return PSG_OK;
  }

  void release_push(PendingPush& pp) {
    pp.keys.reset();
    dev_put(pp.vblock, pp.vbytes);
    pp.vblock = nullptr;
    // its decode (on `copy`) must be ordered before the release event
    // dev_put records on `stream`
    if (pp.sblock) (void)join_copy();
    dev_put(pp.sblock, pp.sbytes);
    pp.sblock = nullptr;
  }

  // Enqueue the merge of every pending push of `a` into its device output;
  // unmatched keys accumulate in a.d_bad.  No host wait.
  // `outs`: write the sums there instead of a.d_out (device-visible caller
  // arrays; only for a single launch that starts the aggregate).
  // `bad_host`: read a.d_bad back there right after the last launch, ahead
  // of the host-side release work (psg_received waits for it)
  int flush(Aggregate& a, void* const* outs = nullptr, void* bad_host = nullptr) {
    if (a.pending.empty()) return PSG_OK;
    while (!a.pending.empty()) {
      const size_t take = std::min(a.pending.size(), flush_pushes);
      // compressed pushes of this launch: all their parts decode in one
      // launch on `copy` (one wave per part, side by side), then the join
      void* dblk = nullptr;
      size_t dbytes = 0;
      if (int rc = decode_pending(a, take, &dblk, &dbytes)) return rc;
      if (int rc = join_copy()) return rc;
      // one job over every push and all arrays when each push holds all of
      // them and every array has the same history (the reference's apps:
      // always); otherwise one single-array job per array over the pushes
      // holding it (kv_vector.h:189-196).  Job 0 holds every push either way
      // (each has array 0): its unmatched count is the launch's
      bool uniform = true;
      for (size_t p = 0; p < take; ++p) uniform = uniform && a.pending[p].m == a.m;
      for (int i = 1; i < a.m; ++i)
        uniform = uniform && (a.folded_arr[i] > 0) == (a.folded_arr[0] > 0);
      const int jm = uniform ? a.m : 1;
      std::vector<JobSpec> jobs;
      for (int i = 0; i < (uniform ? 1 : a.m); ++i) {
        JobSpec js;
        js.keys = ch[a.chl].d_keys + a.lo;
        js.nslots = a.hi - a.lo;
        js.flags = (flags & PSG_PARALLEL_MATCH ? psg::kFlagParallel : 0u) |
                   (a.folded_arr[i] > 0 ? psg::kFlagCont : 0u);
        bool dense = true;
        for (size_t p = 0; p < take; ++p) {
          const PendingPush& pp = a.pending[p];
          if (pp.m <= i) continue;
          js.pkeys.push_back(pp.kd ? pp.kd : pp.keys->d);
          for (int k = 0; k < jm; ++k) js.pvals.push_back(pp.d_vals[i + k]);
          js.pn.push_back(pp.n);
          js.dpos.push_back(pp.dpos);
          dense = dense && pp.dense;
        }
        if (js.pn.empty()) continue;  // no push of this launch holds array i
        // every push a contiguous slice: the dense kernel (no key reads)
        js.dense = dense;
        if (!dense) js.dpos.clear();
        for (int k = 0; k < jm; ++k) js.out.push_back(outs ? outs[i + k] : a.d_out[i + k]);
        jobs.push_back(std::move(js));
      }
      if (int rc = table.build(device, dtype, jm, jobs, stream, true)) return rc;
      if (int rc = table.run(stream)) return rc;
      HIP_TRY(psg::launch_unmatched(table.d_jobs, 0, table.info[0].np, a.d_bad, stream));
      if (bad_host && take == a.pending.size())
        if (int rc = d2h(bad_host, a.d_bad, kBadBytes)) return rc;
      for (size_t p = 0; p < take; ++p) {
        for (int i = 0; i < a.pending[p].m; ++i) ++a.folded_arr[i];
        release_push(a.pending[p]);
      }
      a.pending.erase(a.pending.begin(), a.pending.begin() + take);
      a.folded += take;
      dev_put(dblk, dbytes);  // after the join: `stream` is past the decode
    }
    return PSG_OK;
  }

  void drop(Aggregate& a) {
    const size_t sv = vsize(dtype);
    for (auto& pp : a.pending) release_push(pp);
    a.pending.clear();
    for (int i = 0; i < a.m; ++i) dev_put(a.d_out[i], (a.hi - a.lo) * sv);
    dev_put(a.d_bad, kBadBytes);
  }

  // the value push behind psg_push / psg_push_cached / psg_push_compressed:
  // keys already resident; values staged from the host, or (vblock) already
  // resident in a pool block of m arrays of align_up(n * s_V, 256) bytes
  // `slice`: the push is D[*slice, *slice + n) (absolute positions) by its
  // end keys; its staged keys are checked strictly increasing on `copy`
  // (the order check that completes the proof, psg_push) into the
  // aggregate's unmatched counter
  int push_values(int chl, int time, uint64_t kb, uint64_t ke, const KeyRef& keys, int m,
                  const void* const* vals, void* vblock = nullptr,
                  const size_t* slice = nullptr, void* sblock = nullptr, size_t sbytes = 0,
                  const PendingPush* comp = nullptr);
  int decode_pending(Aggregate& a, size_t take, void** blk, size_t* bytes);
  // the aggregate of `time` (created on first use) over [kb, ke) of chl
  int aggregate_for(int chl, int time, uint64_t kb, uint64_t ke, int m, Aggregate** out);
};

namespace {

int set_dev(int d) {
  HIP_TRY(hipSetDevice(d));
  return PSG_OK;
}

}  // namespace

extern "C" {

int psg_abi_version(void) { return PSG_ABI_VERSION; }

const char* psg_status_string(int s) {
  switch (s) {
    case PSG_OK: return "ok";
    case PSG_ERR_ARG: return "invalid argument";
    case PSG_ERR_UNMATCHED: return "pushed key not matched";
    case PSG_ERR_RANGE: return "position range mismatch";
    case PSG_ERR_NO_TIME: return "no data received at time";
    case PSG_ERR_OOM: return "out of device memory";
    case PSG_ERR_DEVICE: return "device error";
    case PSG_ERR_UNSORTED: return "keys not strictly increasing";
    case PSG_ERR_SIZE: return "value/key size mismatch";
    case PSG_ERR_CHANNEL: return "channel mismatch";
    case PSG_ERR_EMPTY_KEYS: return "channel has no server keys";
    case PSG_ERR_SIGNATURE: return "key signature mismatch";
    default: return "unknown status";
  }
}

const char* psg_last_error(void) { return g_err.c_str(); }

int psg_device_count(int* n) {
  if (!n) return fail(PSG_ERR_ARG, "null");
  HIP_TRY(hipGetDeviceCount(n));
  return PSG_OK;
}

int psg_plan_max_push(void) { return psg::kMaxPush; }

// ---------------------------------------------------------------- plans --
int psg_plan_create(int device, int dtype, int m, unsigned flags,
                    const psg_merge_job* jobs, int njobs, psg_plan** out) {
  if (!out || (njobs > 0 && !jobs)) return fail(PSG_ERR_ARG, "null argument");
  if (dtype != PSG_F32 && dtype != PSG_F64) return fail(PSG_ERR_ARG, "dtype %d", dtype);
  if (m < 1 || m > PSG_MAX_VALUE_ARRAYS) return fail(PSG_ERR_ARG, "m=%d", m);
  if (int rc = set_dev(device)) return rc;
  std::vector<JobSpec> specs(njobs);
  uint64_t bytes = 0, kv = 0;
  const uint64_t sv = vsize(dtype);
  for (int j = 0; j < njobs; ++j) {
    const psg_merge_job& J = jobs[j];
    if (J.npush < 0 || (J.npush > 0 && (!J.push_keys || !J.push_vals || !J.push_n)) ||
        !J.out || (J.nslots > 0 && !J.keys))
      return fail(PSG_ERR_ARG, "job %d: null pointer", j);
    JobSpec& s = specs[j];
    s.keys = J.keys;
    s.nslots = J.nslots;
    s.flags = (flags & PSG_PARALLEL_MATCH) ? psg::kFlagParallel : 0u;
    for (int p = 0; p < J.npush; ++p) {
      s.pkeys.push_back(J.push_keys[p]);
      for (int i = 0; i < m; ++i) s.pvals.push_back(J.push_vals[(size_t)p * m + i]);
      s.pn.push_back(J.push_n[p]);
      bytes += J.push_n[p] * (8 + m * sv);
      kv += J.push_n[p];
    }
    for (int i = 0; i < m; ++i) s.out.push_back(J.out[i]);
    bytes += J.nslots * (8 + m * sv);
  }
  // the dense kernel reads no push keys: only for keys the caller fixed
  // (PSG_STATIC_KEYS, psg.h); otherwise every run re-checks them
  if ((flags & PSG_STATIC_KEYS) && !(flags & PSG_NO_DENSE))
    if (int rc = detect_dense(specs)) return rc;
  psg_plan* p = new psg_plan();
  p->table.read_knobs(flags);
  int rc = p->table.build(device, dtype, m, specs, nullptr, false, !(flags & PSG_NO_INDEX));
  if (rc) {
    p->table.release();
    delete p;
    return rc;
  }
  p->bytes = bytes;
  p->kv = kv;
  *out = p;
  return PSG_OK;
}

int psg_plan_run(psg_plan* plan, void* stream) {
  if (!plan) return fail(PSG_ERR_ARG, "null plan");
  plan->last = (hipStream_t)stream;
  return plan->table.run((hipStream_t)stream);
}

int psg_plan_run_stage(psg_plan* plan, int stage, void* stream) {
  if (!plan || stage < 0 || stage > 1) return fail(PSG_ERR_ARG, "bad plan/stage");
  plan->last = (hipStream_t)stream;
  return plan->table.run_stage(stage, (hipStream_t)stream);
}

int psg_plan_matched(psg_plan* plan, uint64_t* matched) {
  if (!plan || !matched) return fail(PSG_ERR_ARG, "null argument");
  if (int rc = set_dev(plan->table.device)) return rc;
  HIP_TRY(hipStreamSynchronize(plan->last));
  std::vector<uint64_t> mt;
  if (int rc = plan->table.matched(mt)) return rc;
  std::copy(mt.begin(), mt.end(), matched);
  return PSG_OK;
}

int psg_plan_form(psg_plan* plan, int* form) {
  if (!plan || !form) return fail(PSG_ERR_ARG, "null argument");
  const JobTable& T = plan->table;
  *form = T.cursor ? PSG_KERNEL_CURSOR
          : T.pcursor ? PSG_KERNEL_PACKED_CURSOR
          : T.dense ? PSG_KERNEL_DENSE
          : T.pack  ? PSG_KERNEL_PACKED
          : T.wide  ? PSG_KERNEL_TILE64
                    : PSG_KERNEL_TILE;
  return PSG_OK;
}

int psg_plan_bytes(psg_plan* plan, uint64_t* bytes, uint64_t* kv) {
  if (!plan) return fail(PSG_ERR_ARG, "null plan");
  if (bytes) *bytes = plan->bytes;
  if (kv) *kv = plan->kv;
  return PSG_OK;
}

int psg_plan_destroy(psg_plan* plan) {
  if (!plan) return PSG_OK;
  (void)hipSetDevice(plan->table.device);
  plan->table.release();
  delete plan;
  return PSG_OK;
}

// -------------------------------------------------------- device helpers --
int psg_gather_dev(int dtype, const uint64_t* dkeys, uint64_t nd,
                   const void* dvals, const uint64_t* req, uint64_t nreq,
                   void* out, unsigned long long* matched, void* stream) {
  if (dtype != PSG_F32 && dtype != PSG_F64) return fail(PSG_ERR_ARG, "dtype");
  HIP_TRY(psg::launch_gather(dtype, dkeys, nd, dvals, req, nreq, out, matched,
                             (hipStream_t)stream));
  return PSG_OK;
}

int psg_key_union_dev(const uint64_t* a, uint64_t na, const uint64_t* b,
                      uint64_t nb, uint64_t* out, uint64_t* nout, void* stream) {
  if (!out || !nout || (na && !a) || (nb && !b)) return fail(PSG_ERR_ARG, "null");
  if (na + nb >= (1ull << 32)) return fail(PSG_ERR_ARG, "na + nb >= 2^32");
  hipStream_t s = (hipStream_t)stream;
  std::vector<const uint64_t*> pk;
  std::vector<uint64_t> pn;
  if (na) { pk.push_back(a); pn.push_back(na); }
  if (nb) { pk.push_back(b); pn.push_back(nb); }
  void* scratch = nullptr;
  HIP_TRY(hipMalloc(&scratch, psg::nway_scratch_bytes((uint32_t)pk.size(), pn.data())));
  unsigned long long* d_bad = nullptr;
  unsigned long long h[2] = {0, 0};
  hipError_t e = psg::nway_union_enqueue((uint32_t)pk.size(), pk.data(), pn.data(), out, scratch,
                                         &d_bad, s);
  if (e == hipSuccess) e = hipMemcpyAsync(h, d_bad, 16, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(scratch);
  if (e != hipSuccess) return fail(PSG_ERR_DEVICE, "key union: %s", hipGetErrorString(e));
  // high bits: tile overflow (1 << 32) / look-back timeout (1 << 40) of the
  // N-way kernels, a device fault and not an order violation
  if (h[0] >> 32) return fail(PSG_ERR_DEVICE, "key union: device fault (%llx)", h[0]);
  if (h[0]) return fail(PSG_ERR_UNSORTED, "%llu order violations", h[0]);
  *nout = h[1];
  return PSG_OK;
}

int psg_shard_bounds(size_t n, uint64_t* bounds) {
  if (n == 0 || !bounds) return fail(PSG_ERR_ARG, "n == 0");
  // Range<uint64>::all() = [0, 2^64-1)  (range.h:75-78); evenDivide (:85-98)
  const uint64_t b = 0, e = ~0ull;
  const long double itv = (long double)(e - b) / (long double)n;
  for (size_t i = 0; i < n; ++i) bounds[i] = (uint64_t)(b + itv * (long double)i);
  bounds[n] = e;
  return PSG_OK;
}

int psg_slice_dev(const uint64_t* keys, uint64_t n, uint64_t kb, uint64_t ke,
                  const uint64_t* sep, int nsep, uint64_t* pos, void* stream) {
  if (nsep < 0 || (nsep > 0 && (!sep || !pos))) return fail(PSG_ERR_ARG, "null");
  HIP_TRY(psg::launch_slice(keys, n, kb, ke, sep, nsep, pos, (hipStream_t)stream));
  return PSG_OK;
}

int psg_crc32c_dev(const void* data, const uint64_t* off, uint64_t nseg, uint64_t max_len,
                   const uint32_t* init, uint32_t* out, void* stream) {
  if (nseg == 0) return PSG_OK;
  if (!data || !off || !out) return fail(PSG_ERR_ARG, "null argument");
  HIP_TRY(psg::launch_crc32c((const uint8_t*)data, off, nseg, max_len, init, out,
                             (hipStream_t)stream));
  return PSG_OK;
}

int psg_snappy_uncompress_dev(const uint8_t* src, const uint64_t* soff, uint64_t nmsg,
                              uint8_t* dst, const uint64_t* doff, int32_t* status,
                              void* stream) {
  if (nmsg == 0) return PSG_OK;
  if (!src || !soff || !dst || !doff || !status) return fail(PSG_ERR_ARG, "null argument");
  // the deferred-literal list, stream-ordered (freed behind the kernels)
  hipStream_t st = (hipStream_t)stream;
  void* scratch = nullptr;
  HIP_TRY(hipMallocAsync(&scratch, psg::snappy_scratch_bytes(nmsg), st));
  const hipError_t e =
      psg::launch_snappy(src, soff, nmsg, dst, doff, nullptr, status, scratch, st, nullptr);
  HIP_TRY(hipFreeAsync(scratch, st));
  HIP_TRY(e);
  return PSG_OK;
}

int psg_snappy_uncompressed_length(const void* src, size_t n, size_t* len) {
  if (!len || (n && !src)) return fail(PSG_ERR_ARG, "null argument");
  // the preamble: a little-endian base-128 varint of at most 32 bits
  const uint8_t* p = (const uint8_t*)src;
  uint64_t v = 0;
  for (size_t i = 0; i < n && i < 5; ++i) {
    v |= (uint64_t)(p[i] & 0x7f) << (7 * i);
    if (!(p[i] & 0x80)) {
      if (v > 0xffffffffull) break;
      *len = (size_t)v;
      return PSG_OK;
    }
  }
  return fail(PSG_ERR_ARG, "snappy: bad length preamble");
}

// --------------------------------------------------------------- context --
int psg_create(int device, int dtype, unsigned flags, psg_ctx** out) {
  if (!out) return fail(PSG_ERR_ARG, "null out");
  if (dtype != PSG_F32 && dtype != PSG_F64) return fail(PSG_ERR_ARG, "dtype %d", dtype);
  if (int rc = set_dev(device)) return rc;
  psg_ctx* c = new psg_ctx();
  c->device = device;
  c->dtype = dtype;
  c->flags = flags;
  c->table.read_knobs(flags);
  c->zero_copy = !(flags & PSG_NO_ZERO_COPY);
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->copy_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_small, 256);
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_vio_slots, 64 * psg::kVioSlots);
  if (e == hipSuccess) e = hipMemsetAsync(c->d_vio_slots, 0, 64 * psg::kVioSlots, c->stream);
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_small, 256);
  if (e != hipSuccess) {
    psg_destroy(c);
    return fail(PSG_ERR_DEVICE, "psg_create: %s", hipGetErrorString(e));
  }
  *out = c;
  return PSG_OK;
}

namespace {
void filter_release(psg_ctx* c, Filter& F);
}  // namespace

int psg_destroy(psg_ctx* c) {
  if (!c) return PSG_OK;
  (void)hipSetDevice(c->device);
  c->zc.n = 0;  // held buffers of pushes never merged: not read any more
  if (c->copy) (void)hipStreamSynchronize(c->copy);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& kv : c->agg) c->drop(kv.second);
  c->agg.clear();
  c->kcache.clear();
  for (auto& kv : c->ch) {
    c->dev_put(kv.second.d_keys, kv.second.kbytes);
    c->dev_put(kv.second.d_vals, kv.second.nvals * vsize(c->dtype));
    c->dev_put(kv.second.d_delta, 8 * kv.second.dn);
    c->dev_put(kv.second.d_active, 4 * ((kv.second.dn + 31) / 32));
    (void)kv.second.mirror();
    if (kv.second.hk) (void)hipHostFree(kv.second.hk);
    if (kv.second.hev) (void)hipEventDestroy(kv.second.hev);
  }
  c->ch.clear();
  for (auto& kv : c->ff) filter_release(c, kv.second);
  c->ff.clear();
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& f : c->fly) c->free_ev.push_back(f.ev);
  c->fly.clear();
  c->table.release();
  c->pool_release();
  c->ctr_release();
  if (c->ring) (void)hipHostFree(c->ring);
  (void)hipFree(c->d_small);
  (void)hipFree(c->d_vio_slots);
  if (c->h_small) (void)hipHostFree(c->h_small);
  (void)hipFree(c->scratch);
  if (c->copy_ev) (void)hipEventDestroy(c->copy_ev);
  if (c->done_ev) (void)hipEventDestroy(c->done_ev);
  if (c->copy) (void)hipStreamDestroy(c->copy);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return PSG_OK;
}

int psg_set_match_flags(psg_ctx* c, unsigned flags) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  if (c->zc.n) HIP_TRY(hipSetDevice(c->device));
  if (int rc = c->zc_flush()) return rc;  // held copies were queued under the old mode
  c->flags = flags;
  c->table.read_knobs(flags);
  c->zero_copy = !(flags & PSG_NO_ZERO_COPY);
  return PSG_OK;
}

int psg_set_flush_pushes(psg_ctx* c, int n) {
  if (!c || n < 1 || n > psg::kMaxPush) return fail(PSG_ERR_ARG, "flush pushes %d", n);
  std::lock_guard<std::mutex> l(c->mu);
  c->flush_pushes = (size_t)n;
  return PSG_OK;
}

namespace {

// The host mirror of a changed key set: one asynchronous device-to-host copy
// into pinned memory on `stream`, waited for by the first reader.
int refresh_mirror(psg_ctx* c, Channel& C) {
  (void)C.mirror();  // the previous copy may still target the buffer
  if (C.n > C.hcap) {
    if (C.hk) HIP_TRY(hipHostFree(C.hk));
    C.hk = nullptr;
    C.hcap = 0;
    const size_t cap = std::max(C.n, C.n + C.n / 2);
    HIP_TRY(hipHostMalloc((void**)&C.hk, 8 * cap));
    C.hcap = cap;
  }
  if (!C.hev) HIP_TRY(hipEventCreateWithFlags(&C.hev, hipEventDisableTiming));
  if (C.n) HIP_TRY(hipMemcpyAsync(C.hk, C.d_keys, 8 * C.n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(C.hev, c->stream));
  C.hpend = true;
  return PSG_OK;
}

// key_[chl] = key_[chl].setUnion(keys_0).setUnion(keys_1)...; val_[chl].clear()
// (kv_vector.h:177-182, shared_array_inl.h:155-162) for resident key-only
// pushes d_push[i] (n[i] keys): one N-way merge on the device (psg_nway.hip)
// of the server keys and up to 63 pushes at a time; the host mirror is then
// refreshed from the device result by an asynchronous copy (no CPU union).
int key_union_impl(psg_ctx* c, int chl, const std::vector<const uint64_t*>& d_push,
                   const std::vector<uint64_t>& n) {
  Channel& C = c->ch[chl];
  // Pending value pushes of this channel were matched against the current
  // key_[chl] in the reference (setValue matches at arrival,
  // kv_vector.h:171-204): enqueue their merge before the key set (and so
  // every position) changes.  The old key array goes back to the pool after
  // those kernels.
  for (auto& kv : c->agg)
    if (kv.second.chl == chl && !kv.second.pending.empty())
      if (int rc = c->flush(kv.second)) return rc;
  if (int rc = c->join_copy()) return rc;
  bool changed = false;
  // once a merge applied, the key set (so every position) changed: the
  // mirror is refreshed and val_[chl] cleared (kv_vector.h:180) on every
  // way out, an error in a later chunk of pushes included
  auto settle = [&](int rc) -> int {
    if (!changed) return rc;
    const int mr = refresh_mirror(c, C);
    c->dev_put(C.d_vals, C.nvals * vsize(c->dtype));
    C.d_vals = nullptr;
    C.nvals = 0;
    return rc != PSG_OK ? rc : mr;
  };
  for (size_t i = 0; i < d_push.size();) {
    std::vector<const uint64_t*> pk;
    std::vector<uint64_t> pn;
    if (C.n) {
      pk.push_back(C.d_keys);
      pn.push_back(C.n);
    }
    const size_t base = pk.size();
    for (; i < d_push.size() && pk.size() < (size_t)psg_nway_max_push(); ++i)
      if (n[i]) {
        pk.push_back(d_push[i]);
        pn.push_back(n[i]);
      }
    if (pk.size() == base) continue;  // only empty pushes: ignored (kv_vector.h:177)
    uint64_t cap = 0;
    for (uint64_t x : pn) cap += x;
    if (cap >= (1ull << 32))
      return settle(fail(PSG_ERR_ARG, "key union of %llu keys >= 2^32", (unsigned long long)cap));
    const uint32_t K = (uint32_t)pk.size();
    if (int rc = c->ensure_scratch(psg::nway_scratch_bytes(K, pn.data()))) return settle(rc);
    uint64_t* d_out = nullptr;
    if (int rc = c->dev_get(8 * cap, (void**)&d_out, c->stream)) return settle(rc);
    unsigned long long* d_bad = nullptr;
    hipError_t e = psg::nway_union_enqueue(K, pk.data(), pn.data(), d_out, c->scratch, &d_bad,
                                           c->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(c->h_small, d_bad, 16, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      c->dev_put(d_out, 8 * cap);
      return settle(fail(PSG_ERR_DEVICE, "key union: %s", hipGetErrorString(e)));
    }
    const unsigned long long bad = c->h_small[0], nu = c->h_small[1];
    if (bad) {  // the pushes of this merge are not applied; earlier ones are
      c->dev_put(d_out, 8 * cap);
      return settle(fail(bad >> 32 ? PSG_ERR_DEVICE : PSG_ERR_UNSORTED,
                         "key-only push: %llu order violations", bad));
    }
    c->dev_put(C.d_keys, C.kbytes);
    C.d_keys = d_out;
    C.kbytes = 8 * cap;
    C.n = (size_t)nu;
    changed = true;
  }
  return settle(PSG_OK);
}

// findRange of a push and the consistency checks of setValue, before any
// data is staged
int check_push(psg_ctx* c, int chl, int time, uint64_t kb, uint64_t ke, size_t n, int m,
               size_t* lo, size_t* hi) {
  if (m < 1 || m > PSG_MAX_VALUE_ARRAYS) return fail(PSG_ERR_ARG, "m=%d", m);
  if (ke < kb) return fail(PSG_ERR_ARG, "invalid key range");
  auto cit = c->ch.find(chl);
  if (cit == c->ch.end() || cit->second.n == 0)
    return fail(PSG_ERR_EMPTY_KEYS, "channel %d has no server keys", chl);
  Channel& C = cit->second;
  const uint64_t* h = C.mirror();
  *lo = std::lower_bound(h, h + C.n, kb) - h;
  *hi = std::lower_bound(h, h + C.n, ke) - h;
  if (*hi - *lo < n)  // pigeonhole: some key cannot match (CHECK_GE, kv_vector.h:121,191)
    return fail(PSG_ERR_UNMATCHED, "push of %zu keys into a range of %zu server keys", n,
                *hi - *lo);
  auto ait = c->agg.find(time);
  if (ait != c->agg.end()) {
    const Aggregate& A = ait->second;
    if (A.chl != chl) return fail(PSG_ERR_CHANNEL, "time %d: channel %d != %d", time, chl, A.chl);
    if (A.lo != *lo || A.hi != *hi)  // CHECK_EQ(aligned.first, stored) kv_vector.h:199
      return fail(PSG_ERR_RANGE, "time %d: range [%zu,%zu) != [%zu,%zu)", time, *lo, *hi,
                  A.lo, A.hi);
  }
  return PSG_OK;
}

}  // namespace

int psg_ctx::decode_pending(Aggregate& a, size_t take, void** blk, size_t* bytes) {
  *blk = nullptr;
  *bytes = 0;
  std::vector<uint64_t> pr, dst, cap;
  for (size_t p = 0; p < take; ++p) {
    PendingPush& pp = a.pending[p];
    for (int i = 0; i < pp.cparts; ++i) {
      pr.push_back(pp.cbeg[i]);
      pr.push_back(pp.cend[i]);
      dst.push_back(pp.cdst[i]);
      cap.push_back(pp.ccap[i]);
    }
    pp.cparts = 0;
  }
  const size_t n = dst.size();
  if (n == 0) return PSG_OK;
  // held pushes' parts may still sit in the zero-copy batch: issue it first
  if (int rc = zc_flush()) return rc;
  // [pairs 16n][dst 8n][cap 8n] | [status 4n] | decoder scratch
  const size_t hb = 32 * n, sb = align_up(hb + 4 * n, 256);
  const size_t total = sb + psg::snappy_scratch_bytes(n);
  void* b = nullptr;
  if (int rc = dev_get(total, &b, copy)) return rc;
  std::vector<uint64_t> img(4 * n);
  std::copy(pr.begin(), pr.end(), img.begin());
  std::copy(dst.begin(), dst.end(), img.begin() + 2 * n);
  std::copy(cap.begin(), cap.end(), img.begin() + 3 * n);
  int rc = h2d(b, img.data(), hb);
  if (rc == PSG_OK) {
    const uint64_t* d = (const uint64_t*)b;
    const hipError_t e = psg::launch_snappy(nullptr, d, n, nullptr, d + 2 * n, d + 3 * n,
                                            (int32_t*)(d + 4 * n), (char*)b + sb, copy,
                                            a.d_bad + 1, true);
    if (e != hipSuccess) rc = fail(PSG_ERR_DEVICE, "snappy: %s", hipGetErrorString(e));
  }
  if (rc != PSG_OK) {
    (void)hipStreamSynchronize(copy);
    dev_put(b, total);
    return rc;
  }
  *blk = b;
  *bytes = total;
  return PSG_OK;
}

int psg_ctx::aggregate_for(int chl, int time, uint64_t kb, uint64_t ke, int m,
                           Aggregate** out) {
  auto ait = agg.find(time);
  if (ait == agg.end()) {
    // (re-derived: the caller checked the push against the range)
    Channel& C = ch[chl];
    const uint64_t* h = C.mirror();
    const size_t lo = std::lower_bound(h, h + C.n, kb) - h;
    const size_t hi = std::lower_bound(h, h + C.n, ke) - h;
    Aggregate A;
    A.chl = chl;
    A.lo = lo;
    A.hi = hi;
    // zeroed on `copy`: the dense pushes' order checks and the compressed
    // pushes' decodes add to it there; every reader on `stream` runs after
    // a join_copy
    if (int rc = dev_get(kBadBytes, (void**)&A.d_bad, copy)) return rc;
    HIP_TRY(hipMemsetAsync(A.d_bad, 0, kBadBytes, copy));
    ait = agg.emplace(time, A).first;
  }
  Aggregate& A = ait->second;
  // a push with more value arrays than the earlier ones extends the list
  // (recved_val_[t].push_back, kv_vector.h:118-125,193-194)
  for (; A.m < m; ++A.m)
    if (int rc = dev_get((A.hi - A.lo) * vsize(dtype), &A.d_out[A.m], stream)) return rc;
  *out = &A;
  return PSG_OK;
}

int psg_ctx::push_values(int chl, int time, uint64_t kb, uint64_t ke, const KeyRef& keys, int m,
                         const void* const* vals, void* vblock, const size_t* slice,
                         void* sblock, size_t sbytes, const PendingPush* comp) {
  const size_t sv = vsize(dtype), n = keys->n;
  PendingPush pp;
  if (comp) pp = *comp;  // the compressed parts to decode
  pp.n = n;
  pp.m = m;
  pp.keys = keys;
  pp.sblock = sblock;
  pp.sbytes = sbytes;
  const size_t vb = align_up(sv * n, 256);
  pp.vbytes = m * vb;
  if (vblock) {
    pp.vblock = vblock;
    for (int i = 0; i < m; ++i) pp.d_vals[i] = (char*)pp.vblock + i * vb;
  } else {
    if (int rc = dev_get(pp.vbytes, &pp.vblock, copy)) return rc;
    for (int i = 0; i < m; ++i) {
      pp.d_vals[i] = (char*)pp.vblock + i * vb;
      if (int rc = h2d(pp.d_vals[i], vals[i], sv * n, true)) {
        release_push(pp);
        return rc;
      }
    }
  }
  Aggregate* Ap = nullptr;
  if (int rc = aggregate_for(chl, time, kb, ke, m, &Ap)) {
    release_push(pp);
    return rc;
  }
  Aggregate& A = *Ap;
  if (slice) {
    pp.dense = true;
    pp.dpos = *slice - A.lo;
    pp.kd = ch[chl].d_keys + *slice;
    if (keys->d) {
      HIP_TRY(psg::launch_check_sorted(keys->d, n, A.d_bad, copy, true));
    } else {
      HIP_TRY(psg::launch_check_sorted_host(keys->host, n, A.d_bad, copy));
      pinned_wait = pinned_wait || !(flags & PSG_HOLD_BUFFERS);
    }
  }
  A.pending.push_back(pp);
  A.expected_total += n;
  if (A.pending.size() >= flush_pushes) return flush(A);
  return PSG_OK;
}

int psg_key_union(psg_ctx* c, int chl, const uint64_t* keys, size_t n) {
  if (!c || (n && !keys)) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  if (n == 0) return PSG_OK;  // kv_vector.h:177: empty key list is ignored
  if (int rc = set_dev(c->device)) return rc;
  KeyRef k;
  if (int rc = c->new_keys(n, &k)) return rc;
  int rc = c->h2d(k->d, keys, 8 * n);
  if (rc == PSG_OK) rc = key_union_impl(c, chl, {k->d}, {(uint64_t)n});
  const int rf = c->h2d_finish();
  return rc ? rc : rf;
}

int psg_key_union_batch(psg_ctx* c, int chl, const uint64_t* const* keys, const size_t* n,
                        int npush) {
  if (!c || npush < 0 || (npush && (!keys || !n))) return fail(PSG_ERR_ARG, "null argument");
  for (int p = 0; p < npush; ++p)
    if (n[p] && !keys[p]) return fail(PSG_ERR_ARG, "push %d: null keys", p);
  std::lock_guard<std::mutex> l(c->mu);
  if (int rc = set_dev(c->device)) return rc;
  std::vector<KeyRef> staged;
  std::vector<const uint64_t*> dp;
  std::vector<uint64_t> dn;
  int rc = PSG_OK;
  for (int p = 0; rc == PSG_OK && p < npush; ++p) {
    if (!n[p]) continue;
    KeyRef k;
    rc = c->new_keys(n[p], &k);
    if (rc == PSG_OK) rc = c->h2d(k->d, keys[p], 8 * n[p]);
    if (rc == PSG_OK) {
      staged.push_back(k);
      dp.push_back(k->d);
      dn.push_back(n[p]);
    }
  }
  if (rc == PSG_OK && !dp.empty()) rc = key_union_impl(c, chl, dp, dn);
  const int rf = c->h2d_finish();
  return rc ? rc : rf;
}

int psg_key_size(psg_ctx* c, int chl, size_t* n) {
  if (!c || !n) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ch.find(chl);
  *n = it == c->ch.end() ? 0 : it->second.n;
  return PSG_OK;
}

int psg_key_copy(psg_ctx* c, int chl, size_t off, size_t n, uint64_t* out) {
  if (!c || (n && !out)) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ch.find(chl);
  const size_t have = it == c->ch.end() ? 0 : it->second.n;
  if (off + n > have) return fail(PSG_ERR_ARG, "key copy out of range");
  if (n) memcpy(out, it->second.mirror() + off, 8 * n);
  return PSG_OK;
}

int psg_find_range(psg_ctx* c, int chl, uint64_t kb, uint64_t ke, size_t* lo,
                   size_t* hi) {
  if (!c || !lo || !hi) return fail(PSG_ERR_ARG, "null argument");
  if (ke < kb) return fail(PSG_ERR_ARG, "invalid key range");  // CHECK(bound.valid())
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ch.find(chl);
  if (it == c->ch.end() || it->second.n == 0) {
    *lo = *hi = 0;
    return PSG_OK;
  }
  const uint64_t* k = it->second.mirror();
  *lo = std::lower_bound(k, k + it->second.n, kb) - k;
  *hi = std::lower_bound(k, k + it->second.n, ke) - k;
  return PSG_OK;
}

int psg_value_assign(psg_ctx* c, int chl, const void* vals, size_t n) {
  if (!c || (n && !vals)) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  if (int rc = set_dev(c->device)) return rc;
  Channel& C = c->ch[chl];
  const size_t sv = vsize(c->dtype);
  // the old array goes back to the pool (after any kernel reading it); the
  // new one is written on the copy stream once it is free
  c->dev_put(C.d_vals, C.nvals * sv);
  C.d_vals = nullptr;
  C.nvals = 0;
  if (n) {
    if (int rc = c->dev_get(n * sv, &C.d_vals, c->copy)) return rc;
    C.nvals = n;
    if (int rc = c->h2d(C.d_vals, vals, n * sv)) return rc;
  }
  return c->h2d_finish();
}

int psg_value_size(psg_ctx* c, int chl, size_t* n) {
  if (!c || !n) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ch.find(chl);
  *n = it == c->ch.end() ? 0 : it->second.nvals;
  return PSG_OK;
}

int psg_value_copy(psg_ctx* c, int chl, size_t off, size_t n, void* out) {
  if (!c || (n && !out)) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ch.find(chl);
  const size_t have = it == c->ch.end() ? 0 : it->second.nvals;
  if (off + n > have) return fail(PSG_ERR_ARG, "value copy out of range");
  if (int rc = set_dev(c->device)) return rc;
  if (int rc = c->join_copy()) return rc;
  const size_t sv = vsize(c->dtype);
  if (n)
    HIP_TRY(hipMemcpyAsync(out, (char*)it->second.d_vals + off * sv, n * sv,
                           hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PSG_OK;
}

int psg_push(psg_ctx* c, int chl, int time, uint64_t kb, uint64_t ke,
             const uint64_t* keys, size_t n, int m, const void* const* vals) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  if (n == 0) return PSG_OK;  // kv_vector.h:90,177 -- empty push ignored
  if (!keys || !vals) return fail(PSG_ERR_ARG, "null keys/values");
  for (int i = 0; i < m && i < PSG_MAX_VALUE_ARRAYS; ++i)
    if (!vals[i]) return fail(PSG_ERR_ARG, "null value array %d", i);
  std::lock_guard<std::mutex> l(c->mu);
  if (int rc = set_dev(c->device)) return rc;
  size_t lo, hi;
  if (int rc = check_push(c, chl, time, kb, ke, n, m, &lo, &hi)) return rc;
  // Dense test ("back - front + 1 == n"): the push's first
  // key is server key a, its last is server key a + n - 1, and those n
  // server keys are n consecutive integers.  Then n strictly increasing
  // keys between them can only be exactly D[a, a + n): the merge reads no
  // keys (dense kernel, D's slice stands in for them) and the staged keys
  // are only checked strictly increasing, on the copy stream, into the
  // unmatched count psg_received reports -- the reference's
  // CHECK_EQ(matched, n) (kv_vector.h:192) in full.
  size_t a = 0;
  bool dense = false;
  if (n >= kDenseMinKeys) {
    const uint64_t* h = c->ch[chl].mirror();
    a = std::lower_bound(h + lo, h + hi, keys[0]) - h;
    dense = a + n <= hi && h[a] == keys[0] && h[a + n - 1] == keys[n - 1] &&
            h[a + n - 1] - h[a] == n - 1;
  }
  KeyRef k;
  int rc = PSG_OK;
  const void* kdev = nullptr;
  if (dense && c->zero_copy && host_pinned(keys, &kdev) && kdev && ((uintptr_t)kdev & 15u) == 0) {
    // pinned keys of a dense push: its order check reads them where they
    // are; nothing else needs them on the device (no HBM copy)
    k = std::make_shared<KeyBuf>();
    k->n = n;
    k->host = (const uint64_t*)kdev;
  } else {
    rc = c->new_keys(n, &k);
    // the keys and values of a pinned push in one zero-copy launch (a dense
    // push's keys are read by its check right away: not deferred)
    c->zc_group = !dense;
    if (rc == PSG_OK) rc = c->h2d(k->d, keys, 8 * n, !dense);
  }
  if (rc == PSG_OK) rc = c->push_values(chl, time, kb, ke, k, m, vals, nullptr, dense ? &a : nullptr);
  c->zc_group = false;
  if (!(c->flags & PSG_HOLD_BUFFERS)) {
    if (rc == PSG_OK) rc = c->zc_flush();
    else c->zc.n = 0;  // this push's queued copies only (its blocks went back)
  }
  const int rf = c->h2d_finish();
  return rc ? rc : rf;
}

namespace {
int push_cached_impl(psg_ctx* c, int sender, int chl, int time, uint64_t kb, uint64_t ke,
                     unsigned kc, uint32_t sig, const uint64_t* keys, size_t nkeys, int m,
                     const void* const* vals, size_t nvals);
}

int psg_push_compressed(psg_ctx* c, int chl, int time, uint64_t kb, uint64_t ke,
                        const void* ckeys, size_t ckeys_bytes, int m, const void* const* cvals,
                        const size_t* cvals_bytes) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  if (m < 1 || m > PSG_MAX_VALUE_ARRAYS || !cvals || !cvals_bytes || (ckeys_bytes && !ckeys))
    return fail(PSG_ERR_ARG, "bad compressed push arguments");
  if (ckeys_bytes == 0) return PSG_OK;  // an empty key part: empty push, ignored
  // declared lengths (GetUncompressedLength); whole elements (:236)
  size_t klen = 0;
  if (int rc = psg_snappy_uncompressed_length(ckeys, ckeys_bytes, &klen)) return rc;
  if (klen % 8) return fail(PSG_ERR_SIZE, "key part of %zu bytes", klen);
  const size_t n = klen / 8;
  if (n == 0) return PSG_OK;
  const size_t sv = vsize(c->dtype);
  for (int i = 0; i < m; ++i) {
    size_t vl = 0;
    if (!cvals[i] || !cvals_bytes[i]) return fail(PSG_ERR_SIZE, "empty value part %d", i);
    if (int rc = psg_snappy_uncompressed_length(cvals[i], cvals_bytes[i], &vl)) return rc;
    if (vl != n * sv)  // CHECK_EQ(recv_data.size(), recv_key.size()) kv_vector.h:187
      return fail(PSG_ERR_SIZE, "value part %d: %zu bytes for %zu keys", i, vl, n);
  }
  std::lock_guard<std::mutex> l(c->mu);
  if (int rc = set_dev(c->device)) return rc;
  size_t lo, hi;
  if (int rc = check_push(c, chl, time, kb, ke, n, m, &lo, &hi)) return rc;
  // staging block: the m + 1 compressed parts back to back; they are
  // decoded right before the merge that needs them (psg_ctx::flush), with
  // every other compressed push pending then, in one launch
  const int np = m + 1;
  // part i at soff[i], 16-B aligned (the zero-copy read needs both ends
  // aligned), plen[i] bytes
  std::vector<uint64_t> soff(np + 1, 0), plen(np, 0);
  plen[0] = ckeys_bytes;
  for (int i = 0; i < m; ++i) plen[i + 1] = cvals_bytes[i];
  for (int i = 0; i < np; ++i) soff[i + 1] = align_up(soff[i] + plen[i], 16);
  const size_t tb = align_up(soff[np], 256);
  void* blk = nullptr;
  if (int rc = c->dev_get(tb, &blk, c->copy)) return rc;
  KeyRef k;
  void* vblock = nullptr;
  const size_t vb = align_up(sv * n, 256);
  int rc = c->new_keys(n, &k);
  if (rc == PSG_OK) rc = c->dev_get(m * vb, &vblock, c->copy);
  char* b = (char*)blk;
  // the parts in one zero-copy launch when the caller's buffers are pinned
  c->zc_group = true;
  if (rc == PSG_OK) rc = c->h2d(b, ckeys, ckeys_bytes, true);
  for (int i = 0; rc == PSG_OK && i < m; ++i) rc = c->h2d(b + soff[i + 1], cvals[i], cvals_bytes[i], true);
  c->zc_group = false;
  if (rc == PSG_OK && !(c->flags & PSG_HOLD_BUFFERS)) rc = c->zc_flush();
  // the caller's buffers are free once their copies land (unless held)
  if (rc == PSG_OK) rc = c->h2d_finish();
  if (rc != PSG_OK) {
    if (!(c->flags & PSG_HOLD_BUFFERS)) c->zc.n = 0;  // this push's queued copies only
    (void)hipStreamSynchronize(c->copy);
    c->dev_put(blk, tb);
    c->dev_put(vblock, m * vb);
    return rc;
  }
  PendingPush cp;
  cp.cparts = np;
  for (int i = 0; i < np; ++i) {
    cp.cbeg[i] = (uint64_t)(b + soff[i]);
    cp.cend[i] = (uint64_t)(b + soff[i] + plen[i]);
    cp.cdst[i] = i == 0 ? (uint64_t)k->d : (uint64_t)((char*)vblock + (i - 1) * vb);
    cp.ccap[i] = i == 0 ? (uint64_t)klen : (uint64_t)(n * sv);
  }
  return c->push_values(chl, time, kb, ke, k, m, nullptr, vblock, nullptr, blk, tb, &cp);
}

int psg_push_cached(psg_ctx* c, int sender, int chl, int time, uint64_t kb, uint64_t ke,
                    unsigned kc, uint32_t sig, const uint64_t* keys, size_t nkeys, int m,
                    const void* const* vals, size_t nvals) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  const int rc = push_cached_impl(c, sender, chl, time, kb, ke, kc, sig, keys, nkeys, m, vals,
                                  nvals);
  const int rf = c->h2d_finish();
  return rc ? rc : rf;
}

namespace {
int push_cached_impl(psg_ctx* c, int sender, int chl, int time, uint64_t kb, uint64_t ke,
                     unsigned kc, uint32_t sig, const uint64_t* keys, size_t nkeys, int m,
                     const void* const* vals, size_t nvals) {
  if ((kc & PSG_KC_KEYS) && nkeys && !keys) return fail(PSG_ERR_ARG, "null keys");
  if (m < 0 || m > PSG_MAX_VALUE_ARRAYS || (m > 0 && !vals)) return fail(PSG_ERR_ARG, "m=%d", m);
  for (int i = 0; i < m; ++i)
    if (nvals && !vals[i]) return fail(PSG_ERR_ARG, "null value array %d", i);
  if (int rc = set_dev(c->device)) return rc;
  const CacheKey ck{sender, chl, kb, ke};
  KeyRef k;  // the message's keys, resident
  bool sigcheck = false;  // the carried signature checked on the device
  if (!(kc & PSG_KC_SIG)) {
    // no signature: the cache entry of (channel, range) is dropped
    // (remote_node.cc:143-156) and the message's own keys are used
    c->kcache.erase(ck);
    if ((kc & PSG_KC_KEYS) && nkeys) {
      if (int rc = c->new_keys(nkeys, &k)) return rc;
      if (int rc = c->h2d(k->d, keys, 8 * nkeys)) return rc;
    }
  } else if (kc & PSG_KC_KEYS) {
    // keys carried: check the signature, store them (remote_node.cc:161-171)
    if (nkeys) {
      if (int rc = c->new_keys(nkeys, &k)) return rc;
      if (int rc = c->h2d(k->d, keys, 8 * nkeys)) return rc;
    }
    uint32_t got = 0;  // crc32c::Value of no bytes
    // with values (m > 0) the check runs on the device and a mismatch is
    // reported by psg_received (no host wait); the entry stores the keys as
    // pending on that check: a restore waits for its result and fails (and
    // drops the entry) if it failed.  A key-only message merges into the
    // channel's keys at once, so it is checked before that
    if (nkeys && m > 0) {
      sigcheck = true;  // launched below, into the entry's and the aggregate's counters
      got = sig;
    } else if (nkeys) {
      c->h_small[8] = 0;
      c->h_small[9] = 8 * nkeys;
      HIP_TRY(hipMemcpyAsync(c->d_small + 8, c->h_small + 8, 16, hipMemcpyHostToDevice, c->copy));
      HIP_TRY(psg::launch_crc32c((const uint8_t*)k->d, (const uint64_t*)(c->d_small + 8), 1,
                                 PSG_MAX_SIG_LEN, nullptr, (uint32_t*)(c->d_small + 10), c->copy));
      HIP_TRY(hipMemcpyAsync(c->h_small + 10, c->d_small + 10, 8, hipMemcpyDeviceToHost, c->copy));
      HIP_TRY(hipStreamSynchronize(c->copy));
      got = (uint32_t)c->h_small[10];
    }
    if (got != sig)  // CHECK_EQ(crc32c(key), sig) remote_node.cc:163
      return fail(PSG_ERR_SIGNATURE, "key signature %08x != carried %08x", got, sig);
    CacheEntry& e = c->kcache[ck];
    e.sig = sig;
    e.keys = k;
    e.chk.reset();
  } else {
    // keys restored from the cache (remote_node.cc:172-176)
    auto it = c->kcache.find(ck);
    if (it != c->kcache.end() && it->second.chk) {
      // stored by a keyed message whose device check has not been read yet
      bool ok = false;
      if (int rc = c->sig_check_result(it->second.chk, &ok)) return rc;
      if (!ok) {
        const uint32_t bad = it->second.sig;
        c->kcache.erase(it);
        return fail(PSG_ERR_SIGNATURE,
                    "key cache of channel %d [%llu,%llu): the stored keys did not match their "
                    "signature %08x",
                    chl, (unsigned long long)kb, (unsigned long long)ke, bad);
      }
      it->second.chk.reset();
    }
    const uint32_t have = it == c->kcache.end() ? 0u : it->second.sig;
    if (sig != have)  // CHECK_EQ(sig, cache.first)
      return fail(PSG_ERR_SIGNATURE, "key cache of channel %d [%llu,%llu): signature %08x != %08x",
                  chl, (unsigned long long)kb, (unsigned long long)ke, sig, have);
    if (it != c->kcache.end()) k = it->second.keys;
  }
  // the stored entry's pending check (keys carried with values): ONE device
  // CRC of the keys, counted into the entry's counter (a later restore waits
  // for it) and into the aggregate's (psg_received reports a mismatch).  If
  // the message is refused before its aggregate exists, the check still
  // runs, into the entry's counter alone: the entry is never restorable
  // unchecked
  auto store_check = [&](unsigned long long* agg) -> int {
    auto it = c->kcache.find(ck);
    if (it == c->kcache.end() || it->second.keys != k) return PSG_OK;  // erased meanwhile
    SigCheckRef pend;
    if (int rc = c->sig_check_pending(k, sig, &pend, agg)) return rc;
    it->second.chk = pend;
    return PSG_OK;
  };
  if (kc & PSG_KC_ERASE) c->kcache.erase(ck);  // remote_node.cc:183
  const size_t n = k ? k->n : 0;
  if (n == 0) return PSG_OK;  // kv_vector.h:90,177: no keys, message ignored
  if (m == 0) {
    // key-only message: setUnion with the (possibly restored) keys, on the device
    return key_union_impl(c, chl, {k->d}, {(uint64_t)n});
  }
  if (nvals != n) {  // CHECK_EQ(recv_data.size(), recv_key.size()) kv_vector.h:108,187
    if (sigcheck) (void)store_check(nullptr);
    return fail(PSG_ERR_SIZE, "%zu values for %zu keys", nvals, n);
  }
  size_t lo, hi;
  if (int rc = check_push(c, chl, time, kb, ke, n, m, &lo, &hi)) {
    if (sigcheck) (void)store_check(nullptr);
    return rc;
  }
  if (sigcheck) {  // on `copy` after the key copy
    Aggregate* A = nullptr;
    if (int rc = c->aggregate_for(chl, time, kb, ke, m, &A)) {
      (void)store_check(nullptr);
      return rc;
    }
    if (int rc = store_check(A->d_bad + 2)) return rc;
    if (!c->kcache.count(ck))  // the entry was erased (PSG_KC_ERASE): the aggregate's check alone
      HIP_TRY(psg::launch_sig_check((const uint8_t*)k->d, 8 * n, PSG_MAX_SIG_LEN, sig,
                                    A->d_bad + 2, c->copy));
  }
  return c->push_values(chl, time, kb, ke, k, m, vals);
}

}  // namespace

int psg_key_cache_clear(psg_ctx* c, int sender) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  for (auto it = c->kcache.begin(); it != c->kcache.end();)
    it = (sender < 0 || it->first.sender == sender) ? c->kcache.erase(it) : std::next(it);
  return PSG_OK;
}

int psg_key_cache_bytes(psg_ctx* c, int sender, size_t* bytes) {
  if (!c || !bytes) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  size_t b = 0;
  for (const auto& kv : c->kcache)
    if ((sender < 0 || kv.first.sender == sender) && kv.second.keys) b += kv.second.keys->bytes;
  *bytes = b;
  return PSG_OK;
}

int psg_received_shape(psg_ctx* c, int time, int* m, size_t* lo, size_t* hi) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->agg.find(time);
  if (it == c->agg.end()) return fail(PSG_ERR_NO_TIME, "no data received at time %d", time);
  if (m) *m = it->second.m;
  if (lo) *lo = it->second.lo;
  if (hi) *hi = it->second.hi;
  return PSG_OK;
}

int psg_received(psg_ctx* c, int time, int m, void* const* out) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->agg.find(time);
  if (it == c->agg.end()) return fail(PSG_ERR_NO_TIME, "no data received at time %d", time);
  if (int rc = set_dev(c->device)) return rc;
  Aggregate& A = it->second;
  if (m != A.m || !out) return fail(PSG_ERR_ARG, "expected %d output arrays", A.m);
  const size_t len = A.hi - A.lo, sv = vsize(c->dtype);
  // the whole aggregate in one launch into pinned caller arrays: the merge
  // kernel writes the sums there itself (no separate readback)
  bool direct = c->zero_copy && A.folded == 0 && !A.pending.empty() &&
                A.pending.size() <= c->flush_pushes && len > 0;
  void* dev_out[psg::kMaxM] = {};
  for (int i = 0; direct && i < A.m; ++i) {
    const void* d = nullptr;
    direct = host_pinned(out[i], &d) && d && ((uintptr_t)d & 15u) == 0;
    dev_out[i] = (void*)d;
  }
  const bool pend = !A.pending.empty();
  int rc = c->flush(A, direct ? dev_out : nullptr, direct ? c->h_small : nullptr);
  for (int i = 0; !direct && rc == PSG_OK && i < A.m && len; ++i)
    rc = c->d2h(out[i], A.d_out[i], len * sv);
  unsigned long long bad = 0;
  unsigned long long corrupt = 0, badsig = 0;
  if (rc == PSG_OK && !(direct && pend)) rc = c->d2h(c->h_small, A.d_bad, kBadBytes);
  if (rc == PSG_OK) {
    hipError_t e = hipEventRecord(c->done_ev, c->stream);
    if (e == hipSuccess) e = spin_wait(c->done_ev);
    if (e != hipSuccess) rc = fail(PSG_ERR_DEVICE, "received: %s", hipGetErrorString(e));
    bad = c->h_small[0];
    corrupt = c->h_small[1];
    badsig = c->h_small[2];
  }
  const unsigned long long want = A.expected_total;
  c->drop(A);
  c->agg.erase(it);
  if (rc) return rc;
  if (corrupt)  // Van::recv's CHECK on uncompressFrom (shared_array_inl.h:236)
    return fail(PSG_ERR_ARG, "time %d: %llu compressed parts failed to decode", time, corrupt);
  if (badsig)  // cacheKeyRecver's CHECK_EQ(crc32c(key), sig) (remote_node.cc:163)
    return fail(PSG_ERR_SIGNATURE, "time %d: %llu pushes' keys do not match their signature",
                time, badsig);
  if (bad)
    return fail(PSG_ERR_UNMATCHED, "time %d: matched %llu of %llu pushed keys", time,
                want - bad, want);
  return PSG_OK;
}

int psg_darling_init(psg_ctx* c, int chl, double delta_init) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  if (c->dtype != PSG_F64) return fail(PSG_ERR_ARG, "Darling needs a PSG_F64 context");
  if (int rc = set_dev(c->device)) return rc;
  Channel& C = c->ch[chl];
  if (C.dn != C.n) {
    c->dev_put(C.d_delta, 8 * C.dn);
    c->dev_put(C.d_active, 4 * ((C.dn + 31) / 32));
    C.d_delta = nullptr;
    C.d_active = nullptr;
    C.dn = 0;
    if (C.n) {
      if (int rc = c->dev_get(8 * C.n, (void**)&C.d_delta, c->stream)) return rc;
      if (int rc = c->dev_get(4 * ((C.n + 31) / 32), (void**)&C.d_active, c->stream)) return rc;
    }
    C.dn = C.n;
  }
  HIP_TRY(psg::launch_darling_init(C.d_delta, C.d_active, C.dn, delta_init, c->stream));
  return PSG_OK;
}

int psg_darling_reset_active(psg_ctx* c, int chl) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ch.find(chl);
  if (it == c->ch.end() || !it->second.d_active)
    return fail(PSG_ERR_ARG, "channel %d: no Darling state (psg_darling_init)", chl);
  if (int rc = set_dev(c->device)) return rc;
  HIP_TRY(psg::launch_bitmap_fill(it->second.d_active, it->second.dn, c->stream));
  return PSG_OK;
}

int psg_darling_update(psg_ctx* c, int chl, int time, const psg_darling_param* p,
                       double* violation) {
  if (!c || !p) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->agg.find(time);
  if (it == c->agg.end()) return fail(PSG_ERR_NO_TIME, "no data received at time %d", time);
  if (int rc = set_dev(c->device)) return rc;
  Aggregate& A = it->second;
  if (A.chl != chl) return fail(PSG_ERR_CHANNEL, "time %d: channel %d != %d", time, A.chl, chl);
  if (A.m != 2) return fail(PSG_ERR_ARG, "Darling needs 2 aggregates (G, U), time %d has %d",
                            time, A.m);  // CHECK_EQ(data.size(), 2) darling.cc:253
  Channel& C = c->ch[chl];
  if (C.nvals != C.n || C.dn != C.n)
    return fail(PSG_ERR_SIZE, "channel %d: %zu keys, %zu values, Darling state of %zu", chl,
                C.n, C.nvals, C.dn);
  int rc = c->flush(A);
  if (rc == PSG_OK) {
    const psg::DarlingParam P{p->eta, p->lambda, p->kkt_filter_threshold, p->delta_max};
    unsigned long long* dv = c->d_small + 4;
    hipError_t e = psg::launch_darling((const double*)A.d_out[0], (const double*)A.d_out[1],
                                       (double*)C.d_vals, C.d_delta, C.d_active, A.lo,
                                       A.hi - A.lo, P, A.d_bad, c->d_vio_slots, dv, c->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(c->h_small + 4, dv, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(c->h_small + 5, A.d_bad, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) rc = fail(PSG_ERR_DEVICE, "darling update: %s", hipGetErrorString(e));
  }
  const unsigned long long bad = rc == PSG_OK ? c->h_small[5] : 0, want = A.expected_total;
  if (rc == PSG_OK && violation) memcpy(violation, c->h_small + 4, 8);
  c->drop(A);
  c->agg.erase(it);
  if (rc) return rc;
  if (bad)
    return fail(PSG_ERR_UNMATCHED, "time %d: matched %llu of %llu pushed keys", time,
                want - bad, want);
  return PSG_OK;
}

int psg_darling_state(psg_ctx* c, int chl, size_t off, size_t n, double* delta, uint8_t* active,
                      size_t* nnz_active) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ch.find(chl);
  if (it == c->ch.end() || !it->second.d_active)
    return fail(PSG_ERR_ARG, "channel %d: no Darling state (psg_darling_init)", chl);
  const Channel& C = it->second;
  if (off + n > C.dn) return fail(PSG_ERR_ARG, "Darling state copy out of range");
  if (int rc = set_dev(c->device)) return rc;
  std::vector<uint32_t> bits;
  if (active && n) bits.resize((off + n + 31) / 32 - off / 32);
  if (delta && n)
    HIP_TRY(hipMemcpyAsync(delta, C.d_delta + off, 8 * n, hipMemcpyDeviceToHost, c->stream));
  if (!bits.empty())
    HIP_TRY(hipMemcpyAsync(bits.data(), C.d_active + off / 32, 4 * bits.size(),
                           hipMemcpyDeviceToHost, c->stream));
  if (nnz_active) {
    HIP_TRY(hipMemsetAsync(c->d_small + 6, 0, 8, c->stream));
    HIP_TRY(psg::launch_popcount(C.d_active, (C.dn + 31) / 32, c->d_small + 6, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_small + 6, c->d_small + 6, 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (size_t i = 0; active && i < n; ++i) {
    const size_t k = off + i;
    active[i] = (uint8_t)((bits[k / 32 - off / 32] >> (k % 32)) & 1u);
  }
  if (nnz_active) *nnz_active = (size_t)c->h_small[6];
  return PSG_OK;
}

// ------------------------------------------------------ frequency filter --
namespace {
int filter_order(Filter* F, hipStream_t s);
int filter_mark(psg_ctx* c, Filter* F, hipStream_t s);
}  // namespace

int psg_freq_resize(psg_ctx* c, int chl, int n, int k) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  if (int rc = set_dev(c->device)) return rc;
  Filter& F = c->ff[chl];
  const uint32_t nn = (uint32_t)std::max(n, 64);  // countmin.h:15
  F.sync_ext();
  if (nn != F.n) {
    c->dev_put(F.d_table, psg::cm_table_bytes(F.n));
    F.d_table = nullptr;
    F.n = 0;
    if (int rc = c->dev_get(psg::cm_table_bytes(nn), (void**)&F.d_table, c->stream)) return rc;
    F.n = nn;
  }
  F.k = std::min(30, std::max(1, k));  // countmin.h:18
  // the clear joins the filter's call order: after the filter's
  // previous operation on any stream, and before the next one on any stream
  // (a caller stream, the null stream included, does not wait for the
  // non-blocking context stream by itself)
  if (int rc = filter_order(&F, c->stream)) return rc;
  HIP_TRY(hipMemsetAsync(F.d_table, 0, psg::cm_table_bytes(F.n), c->stream));
  return filter_mark(c, &F, c->stream);
}

int psg_freq_clear(psg_ctx* c, int chl) {
  if (!c) return fail(PSG_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ff.find(chl);
  if (it != c->ff.end()) {
    filter_release(c, it->second);
    c->ff.erase(it);
  }
  return PSG_OK;
}

int psg_freq_empty(psg_ctx* c, int chl, int* empty) {
  if (!c || !empty) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  auto it = c->ff.find(chl);
  *empty = it == c->ff.end() || it->second.n == 0;
  return PSG_OK;
}

namespace {
int filter_of(psg_ctx* c, int chl, Filter** F) {
  auto it = c->ff.find(chl);
  if (it == c->ff.end() || it->second.n == 0)
    return fail(PSG_ERR_ARG, "channel %d: frequency filter is empty (psg_freq_resize)", chl);
  *F = &it->second;
  return PSG_OK;
}

// the binned insert's scratch for n keys (stream s: where the insert runs);
// a filter too large to bin gets none (the CAS form runs)
int filter_bins(psg_ctx* c, Filter* F, size_t n, hipStream_t s) {
  const size_t need = psg::cm_insert_scratch_bytes(n, F->n, F->k);
  if (need == 0 || need <= F->bins_bytes) return PSG_OK;
  F->sync_ext();
  c->dev_put(F->d_bins, F->bins_bytes);
  F->d_bins = nullptr;
  F->bins_bytes = 0;
  if (int rc = c->dev_get(need, &F->d_bins, s)) return rc;
  F->bins_bytes = need;
  return PSG_OK;
}

// order an operation on stream s after the filter's previous one
int filter_order(Filter* F, hipStream_t s) {
  if (F->last && F->last_s != s) HIP_TRY(hipStreamWaitEvent(s, F->last, 0));
  return PSG_OK;
}
// ... and mark it as the filter's last
int filter_mark(psg_ctx* c, Filter* F, hipStream_t s) {
  if (!F->last)
    if (int rc = c->event(&F->last)) return rc;
  HIP_TRY(hipEventRecord(F->last, s));
  F->last_s = s;
  return PSG_OK;
}
void filter_release(psg_ctx* c, Filter& F) {
  F.sync_ext();
  if (F.last) {
    (void)hipEventSynchronize(F.last);
    c->free_ev.push_back(F.last);
    F.last = nullptr;
  }
  c->dev_put(F.d_table, psg::cm_table_bytes(F.n));
  c->dev_put(F.d_bins, F.bins_bytes);
  F.d_table = nullptr;
  F.d_bins = nullptr;
}
}  // namespace

int psg_freq_insert_dev(psg_ctx* c, int chl, const uint64_t* keys, const uint32_t* counts,
                        size_t n, void* stream) {
  if (!c || (n && (!keys || !counts))) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  Filter* F;
  if (int rc = filter_of(c, chl, &F)) return rc;
  if (int rc = filter_order(F, (hipStream_t)stream)) return rc;
  if (int rc = filter_bins(c, F, n, (hipStream_t)stream)) return rc;
  HIP_TRY(psg::launch_cm_insert(keys, counts, n, F->d_table, F->n, F->k, F->d_bins,
                                F->bins_bytes, (hipStream_t)stream));
  F->ext = (hipStream_t)stream;
  F->ext_used = true;
  return filter_mark(c, F, (hipStream_t)stream);
}

size_t psg_freq_query_scratch_bytes(size_t n) { return psg::cm_query_scratch_bytes(n); }

int psg_freq_query_dev(psg_ctx* c, int chl, const uint64_t* keys, size_t n, int freq,
                       uint64_t* out, unsigned long long* nout, void* scratch, void* stream) {
  if (!c || !nout || !scratch || (n && (!keys || !out))) return fail(PSG_ERR_ARG, "null argument");
  if (freq >= 255) return fail(PSG_ERR_ARG, "freqency %d >= kuint8max", freq);  // :29
  std::lock_guard<std::mutex> l(c->mu);
  Filter* F;
  if (int rc = filter_of(c, chl, &F)) return rc;
  if (int rc = filter_order(F, (hipStream_t)stream)) return rc;
  HIP_TRY(psg::launch_cm_query(keys, n, F->d_table, F->n, F->k, freq, out, nout, scratch,
                               (hipStream_t)stream));
  F->ext = (hipStream_t)stream;
  F->ext_used = true;
  return filter_mark(c, F, (hipStream_t)stream);
}

int psg_freq_insert(psg_ctx* c, int chl, const uint64_t* keys, const uint32_t* counts,
                    size_t n) {
  if (!c || (n && (!keys || !counts))) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  Filter* F;
  if (int rc = filter_of(c, chl, &F)) return rc;
  if (n == 0) return PSG_OK;
  if (int rc = set_dev(c->device)) return rc;
  // one staging block for keys + counts, back to the pool after the kernel
  const size_t kb = align_up(8 * n, 256), b = kb + 4 * n;
  void* blk = nullptr;
  if (int rc = c->dev_get(b, &blk, c->copy)) return rc;
  int rc = c->h2d(blk, keys, 8 * n);
  if (rc == PSG_OK) rc = c->h2d((char*)blk + kb, counts, 4 * n);
  if (rc == PSG_OK) rc = c->join_copy();
  if (rc == PSG_OK) rc = filter_order(F, c->stream);
  if (rc == PSG_OK) rc = filter_bins(c, F, n, c->stream);
  if (rc == PSG_OK) {
    hipError_t e = psg::launch_cm_insert((const uint64_t*)blk, (const uint32_t*)((char*)blk + kb),
                                         n, F->d_table, F->n, F->k, F->d_bins, F->bins_bytes,
                                         c->stream);
    if (e != hipSuccess) rc = fail(PSG_ERR_DEVICE, "freq insert: %s", hipGetErrorString(e));
  }
  if (rc == PSG_OK) rc = filter_mark(c, F, c->stream);
  c->dev_put(blk, b);
  const int rf = c->h2d_finish();
  return rc ? rc : rf;
}

int psg_freq_query(psg_ctx* c, int chl, const uint64_t* keys, size_t n, int freq, uint64_t* out,
                   size_t* nout) {
  if (!c || !nout || (n && (!keys || !out))) return fail(PSG_ERR_ARG, "null argument");
  if (freq >= 255) return fail(PSG_ERR_ARG, "freqency %d >= kuint8max", freq);
  std::lock_guard<std::mutex> l(c->mu);
  Filter* F;
  if (int rc = filter_of(c, chl, &F)) return rc;
  *nout = 0;
  if (n == 0) return PSG_OK;
  if (int rc = set_dev(c->device)) return rc;
  const size_t kb = align_up(8 * n, 256), sb = psg::cm_query_scratch_bytes(n);
  if (int rc = c->ensure_scratch(2 * kb + sb)) return rc;
  uint64_t* d_keys = (uint64_t*)c->scratch;
  uint64_t* d_out = (uint64_t*)((char*)c->scratch + kb);
  void* d_s = (char*)c->scratch + 2 * kb;
  if (int rc = c->h2d(d_keys, keys, 8 * n)) return rc;
  if (int rc = c->join_copy()) return rc;
  if (int rc = filter_order(F, c->stream)) return rc;
  HIP_TRY(psg::launch_cm_query(d_keys, n, F->d_table, F->n, F->k, freq, d_out, c->d_small + 7,
                               d_s, c->stream));
  if (int rc = filter_mark(c, F, c->stream)) return rc;
  HIP_TRY(hipMemcpyAsync(c->h_small + 7, c->d_small + 7, 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t m = (size_t)c->h_small[7];
  if (m) HIP_TRY(hipMemcpy(out, d_out, 8 * m, hipMemcpyDeviceToHost));
  *nout = m;
  return c->h2d_finish();
}

int psg_freq_table(psg_ctx* c, int chl, uint8_t* out, size_t n) {
  if (!c || (n && !out)) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  Filter* F;
  if (int rc = filter_of(c, chl, &F)) return rc;
  if (n > F->n) return fail(PSG_ERR_ARG, "table copy of %zu > %u counters", n, F->n);
  if (int rc = set_dev(c->device)) return rc;
  if (int rc = filter_order(F, c->stream)) return rc;
  if (n) HIP_TRY(hipMemcpyAsync(out, F->d_table, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PSG_OK;
}

int psg_gather(psg_ctx* c, int chl, const uint64_t* keys, size_t n, void* out,
               size_t* matched) {
  if (!c || (n && (!keys || !out))) return fail(PSG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> l(c->mu);
  if (matched) *matched = 0;
  if (n == 0) return PSG_OK;  // kv_vector.h:218
  if (int rc = set_dev(c->device)) return rc;
  Channel& C = c->ch[chl];
  if (C.n != C.nvals)  // CHECK_EQ(key_[ch].size(), val_[ch].size()) kv_vector.h:220
    return fail(PSG_ERR_SIZE, "channel %d: %zu keys but %zu values", chl, C.n, C.nvals);
  const size_t sv = vsize(c->dtype);
  if (int rc = c->ensure_scratch(align_up(8 * n, 256) + n * sv)) return rc;
  uint64_t* d_req = (uint64_t*)c->scratch;
  void* d_out = (char*)c->scratch + align_up(8 * n, 256);
  if (int rc = c->h2d(d_req, keys, 8 * n)) return rc;
  if (int rc = c->join_copy()) return rc;
  HIP_TRY(hipMemsetAsync(c->d_small, 0, 16, c->stream));
  HIP_TRY(psg::launch_check_sorted(d_req, n, c->d_small + 1, c->stream, false));
  HIP_TRY(psg::launch_gather(c->dtype, C.d_keys, C.n, C.d_vals, d_req, n, d_out,
                             c->d_small, c->stream));
  HIP_TRY(hipMemcpyAsync(out, d_out, n * sv, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(c->h_small, c->d_small, 16, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  // getValue walks the request with the merge of oldMatch (kv_vector.h:
  // 222-224), whose contract is a sorted request (message.h:248-264)
  if (int rc = c->h2d_finish()) return rc;
  if (c->h_small[1]) return fail(PSG_ERR_UNSORTED, "gather: request keys not sorted");
  if (matched) *matched = (size_t)c->h_small[0];
  return PSG_OK;
}

}  // extern "C"
