// psg_internal.h -- shared between the gfx950 kernels (psg_kernels.hip) and
// the host runtime behind the C ABI (psg_runtime.hip).  Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psg {

// ---- aggregate kernel geometry (see DESIGN.md "Kernels") ----
constexpr int kEPT = 8;          // push elements per thread per chunk
constexpr int kGroup = 64;       // pushes per chunk (one mask bit each)
constexpr int kMaxPush = 4096;   // pushes per job per launch
constexpr int kMaxM = 4;         // value arrays per push

// Tile geometries: server slots per workgroup tile / threads per workgroup
// (4 slots per thread in every geometry).
enum Geometry { kGeoS = 0, kGeoM = 1, kGeoL = 2, kNumGeo = 3 };
constexpr int geo_tile(int g) { return g == kGeoS ? 512 : g == kGeoM ? 1024 : 2048; }
constexpr int geo_threads(int g) { return geo_tile(g) / 4; }

constexpr uint32_t kFlagParallel = 1u;  // PSG_PARALLEL_MATCH
constexpr uint32_t kFlagCont = 2u;      // continue an aggregate of an earlier launch

// One (channel, time) aggregate as the partition kernel sees it.  All
// pointers are device pointers.  seg[b*npush + p] = first index of push p
// whose key is >= D[b*tile] (b < ntiles) or > D[nslots-1] (b == ntiles).
struct JobDev {
  const uint64_t* dkeys;          // D + lo
  uint64_t nslots;                // hi - lo
  const uint64_t* const* pkeys;   // [npush]
  const uint64_t* pn;             // [npush]
  uint32_t* seg;                  // [(ntiles + 1) * npush]
  unsigned long long* fail;       // [npush] in-tile match failures
  uint32_t npush;
  uint32_t ntiles;
  uint32_t part_begin;            // first global partition item of this job
  uint32_t tile;                  // slots per tile
};

// One workgroup tile of the aggregate kernel: everything it needs is one
// scalar-load round trip away.
struct TileDesc {
  const uint64_t* dk;             // D + lo + slot0
  const uint32_t* seg;            // &job.seg[t * npush]; row t+1 follows
  const uint64_t* const* pkeys;   // job push key pointers [npush]
  const void* const* pvals;       // job push value pointers [npush * m]
  void* const* out;               // job output pointers [m]
  unsigned long long* fail;       // job fail counters [npush]
  uint64_t slot0;                 // first slot of the tile in the job
  uint32_t nt;                    // slots in this tile (<= tile)
  uint32_t np;                    // pushes of the job
  uint32_t flags;
  // rows kernel: this tile's slot offset inside its partition range (low
  // 16 bits) and that range's slot count (high 16 bits); the tile's own
  // push boundaries are searched inside the range's segments
  uint32_t sub;
};

// Kernel launchers (psg_kernels.hip).  All enqueue on `stream` only.
hipError_t launch_partition(const JobDev* d_jobs, const uint32_t* d_item_job,
                            uint32_t nitems, hipStream_t stream);
size_t aggregate_lds_bytes(int geo, int dtype, int m, uint32_t maxnp);
hipError_t launch_aggregate(int dtype, int m, int geo, const TileDesc* d_tiles,
                            uint32_t ntiles, uint32_t maxnp, hipStream_t stream);
hipError_t launch_aggregate_v4(int dtype, int m, int geo, const TileDesc* d_tiles,
                               uint32_t ntiles, uint32_t maxnp, hipStream_t stream);
hipError_t launch_aggregate_v5(int dtype, int m, int geo, const TileDesc* d_tiles,
                               uint32_t ntiles, uint32_t maxnp, hipStream_t stream);
// streaming kernel: one wave per coarse tile of kStreamTile slots, np <= 64
constexpr int kStreamTile = 4096;
constexpr int kStreamMaxPush = 64;
hipError_t launch_aggregate_stream(int dtype, int m, const TileDesc* d_tiles,
                                   uint32_t ncoarse, hipStream_t stream);
hipError_t launch_aggregate_stream2(int dtype, int m, const TileDesc* d_tiles,
                                    uint32_t ncoarse, hipStream_t stream);
hipError_t launch_aggregate_stream3(int dtype, int m, const TileDesc* d_tiles,
                                    uint32_t ncoarse, hipStream_t stream);
hipError_t launch_aggregate_stream4(int dtype, int m, const TileDesc* d_tiles,
                                    uint32_t ncoarse, uint32_t maxnp, hipStream_t stream);
// rows kernel (v10): one wave per coarse tile of rows_tile() slots, np <= 64
int rows_tile();
constexpr int kRowsInlinePush = 8;  // pushes whose sub-tile boundaries the rows kernel searches
constexpr int kRowsMaxSub = 4;      // sub-tiles per rows-kernel wave (span)
hipError_t launch_aggregate_rows(int dtype, int m, const TileDesc* d_tiles, uint32_t ncoarse,
                                 hipStream_t stream);
// tile kernel (v13, psg_tile.hip): one workgroup per tile of `tile` slots
// (1024 or 2048), any number of pushes; the partition cuts pushes at every tile
constexpr int kTileSlots = 1024;
bool tile_size_ok(int tile);
hipError_t launch_aggregate_tile(int dtype, int m, int tile, const TileDesc* d_tiles,
                                 uint32_t ntiles, hipStream_t stream);
hipError_t launch_gather(int dtype, const uint64_t* dkeys, uint64_t nd,
                         const void* dvals, const uint64_t* req, uint64_t nreq,
                         void* out, unsigned long long* matched,
                         hipStream_t stream);
// keys strictly increasing?  *bad (device) += number of violations.
hipError_t launch_check_sorted(const uint64_t* keys, uint64_t n,
                               unsigned long long* bad, hipStream_t stream);
// out = a U b (strictly increasing inputs).  scratch: >= union_scratch_bytes(nb).
size_t union_scratch_bytes(uint64_t nb);
hipError_t launch_union(const uint64_t* a, uint64_t na, const uint64_t* b,
                        uint64_t nb, uint64_t* out, void* scratch,
                        uint64_t* d_nout, hipStream_t stream);
hipError_t launch_slice(const uint64_t* keys, uint64_t n, uint64_t kb,
                        uint64_t ke, const uint64_t* sep, int nsep,
                        uint64_t* pos, hipStream_t stream);

}  // namespace psg
