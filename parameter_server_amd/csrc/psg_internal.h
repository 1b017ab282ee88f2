// psg_internal.h -- shared between the gfx950 kernels and the host runtime
// behind the C ABI (psg_runtime.hip).  Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psg {

constexpr int kMaxPush = 4096;  // pushes per job per launch
constexpr int kMaxM = 4;        // value arrays per push
constexpr int kTileSlots = 1024;  // server slots per aggregate-kernel tile
// sparse (packed-round) plans use tiles twice as large: each push's piece
// per tile doubles, so a round's element loads touch half as many pushes
// (pages) per element
#ifndef PSG_PACK_TS
#define PSG_PACK_TS 2048  // A/B builds: 4096
#endif
constexpr int kPackTileSlots = PSG_PACK_TS;
// and so do tile-kernel plans with more than 32 pushes (psg_tile.hip)
constexpr int kWideSlots = 2048;

constexpr uint32_t kFlagParallel = 1u;  // PSG_PARALLEL_MATCH
constexpr uint32_t kFlagCont = 2u;      // continue an aggregate of an earlier launch
constexpr uint32_t kFlagLastTile = 4u;  // TileDesc: the job's last tile

// How the partition finds a job's (push, tile) pieces:
// kSearch: one lane per (push, tile boundary), interpolation search -- cost
//          per boundary, right when pieces are long (cfg2: ~140 keys);
// kStream: every push key read once and mapped to its tile through the
//          job's splitter array -- cost per key, right when pieces are
//          short (many sparse pushes: cfg5 ~4 keys).
enum PartMode : uint32_t { kSearch = 0, kStream = 1 };
constexpr uint32_t kStreamChunk = 512;  // push keys per streaming-partition wave

// One (channel, time) aggregate as the partition kernels see it.  All
// pointers are device pointers.  seg[p*segq + b*segb] = first index of push
// p whose key is >= D[b*tile] (b < ntiles) or > D[nslots-1] (b == ntiles):
// SArray::findRange restated per tile.  kStream jobs store it push-major
// (segq = ntiles + 1, segb = 1: a chunk's boundaries are contiguous), kSearch
// jobs tile-major (segq = 1, segb = npush: a tile's bounds of every push share
// one cache line).
struct JobDev {
  const uint64_t* dkeys;          // D + lo
  uint64_t nslots;                // hi - lo
  const uint64_t* const* pkeys;   // [npush]
  const uint64_t* pn;             // [npush]
  uint32_t* seg;                  // [npush * (ntiles + 1)], strides segq / segb
  unsigned long long* fail;       // [npush] match failures
  uint64_t* split;                // kStream: [ntiles + 1] tile splitters
  uint32_t npush;
  uint32_t ntiles;
  uint32_t split_begin;           // kStream: first splitter item of this job
  uint32_t mode;                  // PartMode
  uint32_t tile;                  // slots per tile
  uint32_t segq, segb;
};

// One workgroup tile of the aggregate kernel.
struct TileDesc {
  const uint64_t* dk;             // D + lo + slot0
  const uint32_t* seg;            // &job.seg[t*segb]; push q's bounds: seg[q*stride], seg[q*stride+segb]
  const uint64_t* const* pkeys;   // job push key pointers [npush]
  const void* const* pvals;       // job push value pointers [npush * m]
  const uint64_t* pn;             // job push lengths [npush]
  void* const* out;               // job output pointers [m]
  unsigned long long* fail;       // job fail counters [npush]
  uint64_t slot0;                 // first slot of the tile in the job
  uint32_t nt;                    // slots in this tile (<= kTileSlots)
  uint32_t np;                    // pushes of the job
  uint32_t stride;                // the job's segq
  uint32_t flags;
  uint32_t segb;                  // the job's segb
  const uint64_t* dpos;           // dense jobs: job position of each push's first key
  // tile kernel: the tile's bucket table built once with D (a plan's resident
  // bucket index, launch_bucket_index), or null: built in the kernel
  const uint32_t* bt;
};

// Cursor form (psg_tile_cursor.hip): one job of a plan as the cursor kernel
// sees it (no partition pass: pieces are found by the element loads), and a
// chunk = a run of consecutive tiles of one job walked by one workgroup.
struct CursorJob {
  const uint64_t* dkeys;          // D + lo
  uint64_t nslots;
  const uint64_t* const* pkeys;   // [np]
  const void* const* pvals;       // [np * m]
  const uint64_t* pn;             // [np]
  void* const* out;               // [m]
  unsigned long long* fail;       // [np] match failures
  uint32_t* seg;                  // tile-major rows: row 0 / row ntiles = covered range
  const uint32_t* bt;             // the resident bucket index of the job's tile 0
  uint32_t np, ntiles, flags;
  uint32_t kr;                    // rounds of 64 keys per push per tile (1..3, the plan's)
};
struct CursorChunk {
  uint32_t job, t0, t1;           // tiles [t0, t1) of job
};
constexpr int kCursorPushes = 32;  // pushes per job in the cursor form (LDS cursors)
// boundary words: (nchunks + 1) x 32 u32, zeroed before each run
// kr: rounds per push per tile, one value for every job of the launch
hipError_t launch_aggregate_cursor(int dtype, int m, int kr, const CursorJob* d_jobs,
                                   const CursorChunk* d_chunks, uint32_t nchunks, uint32_t* bx,
                                   hipStream_t stream);

// dense check of one push against the server keys (psg_tile_dense.hip):
// out[0] = lower_bound(D, keys[0]), out[1] != 0 unless keys == D[out0, +n)
struct DenseCheck {
  const uint64_t* keys;
  uint64_t n;
  const uint64_t* D;
  uint64_t nd;
  unsigned long long* out;
};

// ---- kernel launchers; all enqueue on `stream` only ----
// partition: splitters + fail reset of kStream jobs (one block of 256
// splitters per split item; entry = job index), then the search / stream
// items (u64: job << 37 | push << 24 | boundary group or chunk)
// xcd: deal the items to the XCDs in contiguous runs (launches whose jobs are
// all search mode)
hipError_t launch_partition(const JobDev* d_jobs, const uint32_t* d_split_item_job,
                            uint32_t nsplit_items, const uint64_t* d_items,
                            uint32_t nitems, hipStream_t stream, bool xcd = false);
// aggregate: one workgroup per tile of kTileSlots slots.  psg_tile.hip:
// every round holds one push (long pieces); psg_tile_packed.hip: rounds may
// hold several pushes (many short pieces)
// form: 0 = groups of 32 pushes (1024-slot tiles), 1 = groups of 64 (2048-slot
// tiles)
hipError_t launch_aggregate_tile(int dtype, int m, const TileDesc* d_tiles, uint32_t ntiles,
                                 int form, hipStream_t stream);
// the bucket tables of the tile kernel's tiles (psg_tile.hip), built from D
// alone: bucket_index_words(wide) u32 per tile at out + tile * words
uint32_t bucket_index_words(uint32_t tile_slots);
hipError_t launch_bucket_index(const TileDesc* d_tiles, uint32_t ntiles, uint32_t tile_slots,
                               uint32_t* out,
                               hipStream_t stream);
// cursor form (d_chunks non-null): one workgroup per chunk of consecutive
// tiles (t0, t1 index d_tiles), boundary words (nchunks + 1) x kPackCursorPushes
// u32, zeroed before each run
constexpr int kPackCursorPushes = 256;
hipError_t launch_aggregate_tile_packed(int dtype, int m, const TileDesc* d_tiles,
                                        uint32_t ntiles, hipStream_t stream,
                                        const CursorChunk* d_chunks = nullptr,
                                        uint32_t nchunks = 0, uint32_t* bx = nullptr);
// psg_tile_dense.hip: every push of every job a contiguous slice of D
hipError_t launch_aggregate_dense(int dtype, int m, const TileDesc* d_tiles, uint32_t ntiles,
                                  hipStream_t stream);
// items: check index << 32 | 4096-key chunk
hipError_t launch_dense_check(const DenseCheck* checks, uint32_t nchecks, const uint64_t* items,
                              uint64_t nitems, hipStream_t stream);
hipError_t launch_gather(int dtype, const uint64_t* dkeys, uint64_t nd,
                         const void* dvals, const uint64_t* req, uint64_t nreq,
                         void* out, unsigned long long* matched,
                         hipStream_t stream);
// keys strictly increasing?  *bad (device) += number of violations.
// copies between pinned host memory and the device made by the GPU itself
// (zero-copy; src/dst are device-visible addresses, 16-B aligned)
struct HostCopyDesc {
  const void* src;
  void* dst;
  uint64_t len;
};
constexpr int kHostCopyBatch = 32;  // buffers per launch (kernel arguments)
struct HostCopyBatch {
  HostCopyDesc d[kHostCopyBatch];
  uint32_t n = 0;
};
hipError_t launch_host_copy(void* dst, const void* src, size_t len, hipStream_t stream);
hipError_t launch_host_copy_batch(const HostCopyBatch& b, hipStream_t stream);
hipError_t launch_check_sorted(const uint64_t* keys, uint64_t n,
                               unsigned long long* bad, hipStream_t stream,
                               bool strict = true);
// strictly increasing, keys in pinned host memory (device-visible address,
// 16-B aligned), read by the GPU over the link
hipError_t launch_check_sorted_host(const uint64_t* keys, uint64_t n,
                                    unsigned long long* bad, hipStream_t stream);
// keys-only N-way union of K (<= 64) non-empty sorted device arrays into
// out_keys (psg_nway.hip); scratch >= nway_scratch_bytes(K, n).  Uploads its
// tables with a synchronous copy on `stream`, then enqueues the merge;
// (*d_bad)[0] = order violations, (*d_bad)[1] = |union| after the stream ran.
size_t nway_scratch_bytes(uint32_t K, const uint64_t* n);
hipError_t nway_union_enqueue(uint32_t K, const uint64_t* const* keys, const uint64_t* n,
                              uint64_t* out_keys, void* scratch, unsigned long long** d_bad,
                              hipStream_t stream);
hipError_t launch_slice(const uint64_t* keys, uint64_t n, uint64_t kb,
                        uint64_t ke, const uint64_t* sep, int nsep,
                        uint64_t* pos, hipStream_t stream);

// sum over job `job`'s pushes of (keys - matched keys) into *bad (after the
// aggregate of that job's table ran on the same stream)
hipError_t launch_unmatched(const JobDev* jobs, uint32_t job, uint32_t npush,
                            unsigned long long* bad, hipStream_t stream);

// Darling::updateWeight fused on the resident aggregate (psg_darling.hip)
struct DarlingParam {
  double eta, lambda, kkt, delta_max;
};
// slots: kVioSlots x 64 B of zeroed device memory (left zeroed); *vio is
// written by the launch (the violation's bit pattern, 0 if none)
constexpr int kVioSlots = 256;
hipError_t launch_darling(const double* G, const double* U, double* w, double* delta,
                          uint32_t* active, uint64_t lo, uint64_t n, const DarlingParam& P,
                          const unsigned long long* bad, unsigned long long* slots,
                          unsigned long long* vio, hipStream_t stream);
hipError_t launch_darling_init(double* delta, uint32_t* active, uint64_t n, double delta_init,
                               hipStream_t stream);
hipError_t launch_bitmap_fill(uint32_t* active, uint64_t n, hipStream_t stream);
hipError_t launch_popcount(const uint32_t* a, uint64_t nw, unsigned long long* out,
                           hipStream_t stream);

// FreqencyFilter / CountMin<uint64, uint8> (psg_countmin.hip); the table is
// n byte counters (allocated to a multiple of 4 bytes: dword CAS)
inline size_t cm_table_bytes(uint32_t n) { return ((size_t)n + 3) & ~(size_t)3; }
// binned insert scratch (0: the table is too large, the CAS form runs)
size_t cm_insert_scratch_bytes(uint64_t nk, uint32_t n, int k);
// bins (nullable): scratch of >= cm_insert_scratch_bytes for the binned form
hipError_t launch_cm_insert(const uint64_t* keys, const uint32_t* counts, uint64_t nk,
                            uint8_t* table, uint32_t n, int k, void* bins, size_t bins_bytes,
                            hipStream_t stream);
size_t cm_query_scratch_bytes(uint64_t nk);
hipError_t launch_cm_query(const uint64_t* keys, uint64_t nk, const uint8_t* table, uint32_t n,
                           int k, int freq, uint64_t* out, unsigned long long* nout,
                           void* scratch, hipStream_t stream);

// snappy raw-format decompression (psg_snappy.hip), one wave per message:
// part i -> dst + doff[i], of dcap[i] bytes (dcap NULL: doff[i+1] - doff[i]).
// scratch (snappy_scratch_bytes(nmsg), device; NULL: no deferral) holds the
// long literals the parse defers to the chip-wide copy kernel.
struct SnappyLit {
  const uint8_t* src;
  uint8_t* dst;
  uint64_t len;
};
size_t snappy_scratch_bytes(uint64_t nmsg);
// nbad (nullable): incremented once per part that fails.  pairs: soff holds
// each part's (begin, end) device addresses (src unused), so the parts of
// several staging blocks decode in one launch.
hipError_t launch_snappy(const uint8_t* src, const uint64_t* soff, uint64_t nmsg, uint8_t* dst,
                         const uint64_t* doff, const uint64_t* dcap, int32_t* status,
                         void* scratch, hipStream_t stream, unsigned long long* nbad,
                         bool pairs = false);

// CRC-32C (psg_crc32c.hip): out[i] = crc32c::Extend(init ? init[i] : 0,
// data + off[i], min(off[i+1] - off[i], max_len)); all pointers device
uint64_t crc32c_chunks_per_segment(uint64_t max_len);
hipError_t launch_crc32c(const uint8_t* data, const uint64_t* off, uint64_t nseg,
                         uint64_t max_len, const uint32_t* init, uint32_t* out,
                         hipStream_t stream);
// *bad += 1 (and *bad2, when given) unless crc32c::Value(data,
// min(len, max_len)) == want (one wave; max_len <= 64 KB)
hipError_t launch_sig_check(const uint8_t* data, uint64_t len, uint64_t max_len, uint32_t want,
                            unsigned long long* bad, hipStream_t stream,
                            unsigned long long* bad2 = nullptr);

}  // namespace psg
