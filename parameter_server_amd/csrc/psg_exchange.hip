// psg_exchange.hip -- re-homing of pushes to the key-range shards over RCCL
// ("mode B" ingress): what RNode::submit does per push on the
// worker side (src/system/remote_node.cc:39-60) -- KVVector::slice ->
// sliceKeyOrderedMsg (src/system/message.h:89-123) at the server key ranges
// Range<uint64>::all().evenDivide(nranks, s) (src/base/range.h:85-98,
// linear_method.cc:137-145) and one message per server -- done for a batch
// of device-resident pushes by one rank per GPU.
//
// Set-up (psg_exchange_create, synchronous): one wave per (push, boundary)
// finds the cut positions (a sorted push's piece for shard s is the
// contiguous run [lower_bound(b_s), lower_bound(b_s+1))); the piece counts
// go to their shards with one grouped ncclSend/ncclRecv round (plus an error
// word, so a rank that cannot build its layout still takes part and every
// rank fails together); the send and receive buffers are sized from them.
// A step (psg_exchange_run, on a stream, no host wait): the cut is redone
// on the device and compared with the layout (a push whose keys changed
// since set-up is counted, psg_exchange_status), one gather kernel packs
// every piece into destination-major send buffers (2048-element chunks, all
// of a thread's loads before its stores; this rank's own pieces straight
// into its receive buffers, so they never cross the transport), then per
// peer one ncclSend/ncclRecv of the keys and one per value array in a
// single group.  After a step, shard `rank` holds, for
// each source rank src and push p, the piece at recv offset off[src][p]
// with cnt[src][p] keys (the layout a psg_plan job points at directly).
//
// psg_exchange_create_local builds the same layout for S virtual shards on
// one device with no communicator: a step re-cuts and packs, and
// psg_exchange_send_layout hands out the packed buffers (tests of the
// multi-shard layout on one GPU, SURVEY 4 "8 shards on 1 device").
//
// Transport.  Both rounds (counts at create, payload per run) are one group
// of point-to-point sends and receives (xport_group).  A communicator from
// psg_comm_init runs the group over RCCL (ncclGroupStart / ncclSend /
// ncclRecv / ncclGroupEnd on the caller's stream); one from
// psg_comm_init_loopback is one of S ranks living in this process on one
// device (one host thread per rank, as RCCL ranks are one process each): a
// rank's sends and receives are matched in posting order per (source,
// destination) pair, exactly RCCL's pairing rule, and each matched pair is
// a device copy on the receiver's stream ordered after the sender's stream.
// The count round, the layout and the pairing code are the same for both,
// so the multi-rank path runs on one GPU before it meets xGMI (RCCL itself
// refuses two ranks on one device).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "psg_device.h"
#include "psg_host.h"
#include "psg_internal.h"

using psg::fail;

#define NCCL_TRY(expr)                                                           \
  do {                                                                           \
    ncclResult_t _r = (expr);                                                    \
    if (_r != ncclSuccess)                                                       \
      return fail(PSG_ERR_DEVICE, "%s: %s (%s:%d)", #expr, ncclGetErrorString(_r), \
                  __FILE__, __LINE__);                                           \
  } while (0)

namespace {

// pos[p * (S+1) + s] = lower_bound(push p, bounds[s]); one wave each.
// Verify mode (expect != null): count the positions that differ from the
// layout built at set-up instead of writing them.
__global__ __launch_bounds__(256) void cut_kernel(const uint64_t* const* __restrict__ keys,
                                                  const uint64_t* __restrict__ n,
                                                  const uint64_t* __restrict__ bounds, int S1,
                                                  int P, uint64_t* __restrict__ pos,
                                                  const uint64_t* __restrict__ expect,
                                                  unsigned long long* __restrict__ bad) {
  const int w = (int)((blockIdx.x * 256u + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= P * S1) return;
  const int p = w / S1, s = w - p * S1;
  // every separator, the last (2^64-1, the end of Range::all()) included:
  // the reference's cut (message.h:96-99) leaves a key 2^64-1 in no shard
  const uint64_t r = psg::dev::wave_search(keys[p], n[p], bounds[s], false, lane);
  if (lane == 0) {
    if (expect) {
      if (r != expect[w]) atomicAdd(bad, 1ull);
    } else {
      pos[w] = r;
    }
  }
}

// one piece of the send layout
struct Piece {
  uint64_t src;  // element offset inside push p
  uint64_t dst;  // element offset in the send buffers (tgt 0) or receive buffers (tgt 1)
  uint64_t len;
  uint32_t p;
  uint32_t tgt;  // 1: this rank's own piece, packed straight into its receive buffers
};

constexpr uint32_t kChunk = 2048;  // elements per pack workgroup: 8 per thread

// elements [0, n <= kChunk) from s to d: every thread issues its 8 loads
// (coalesced wave accesses of consecutive elements) before any store
template <typename T>
__device__ __forceinline__ void copy_chunk(T* __restrict__ d, const T* __restrict__ s, uint32_t n) {
  T r[kChunk / 256];
#pragma unroll
  for (int j = 0; j < (int)(kChunk / 256); ++j) {
    const uint32_t i = 256u * j + threadIdx.x;
    if (i < n) r[j] = __builtin_nontemporal_load(s + i);
  }
#pragma unroll
  for (int j = 0; j < (int)(kChunk / 256); ++j) {
    const uint32_t i = 256u * j + threadIdx.x;
    if (i < n) d[i] = r[j];
  }
}

// every piece into the destination-major send buffers (this rank's own
// pieces into its receive buffers: no transport copy for them): keys (8 B)
// and m value arrays of `vb` bytes per element; a workgroup per chunk
__global__ __launch_bounds__(256) void pack_kernel(const Piece* __restrict__ pieces,
                                                   const uint64_t* __restrict__ chunk_piece,
                                                   uint64_t nchunks,
                                                   const uint64_t* const* __restrict__ keys,
                                                   const void* const* __restrict__ vals, int m,
                                                   int vb, uint64_t* __restrict__ skeys,
                                                   void* const* __restrict__ svals,
                                                   uint64_t* __restrict__ rkeys,
                                                   void* const* __restrict__ rvals) {
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uint64_t e = chunk_piece[c];
    const Piece pc = pieces[e >> 24];
    const uint64_t c0 = (e & 0xffffffull) * kChunk;
    const uint32_t len = (uint32_t)(pc.len - c0 < kChunk ? pc.len - c0 : kChunk);
    uint64_t* const dk = pc.tgt ? rkeys : skeys;
    void* const* const dv = pc.tgt ? rvals : svals;
    copy_chunk(dk + pc.dst + c0, keys[pc.p] + pc.src + c0, len);
    for (int a = 0; a < m; ++a) {
      const uint64_t o = pc.src + c0, q = pc.dst + c0;
      if (vb == 4)
        copy_chunk((uint32_t*)dv[a] + q, (const uint32_t*)vals[(size_t)pc.p * m + a] + o, len);
      else
        copy_chunk((uint64_t*)dv[a] + q, (const uint64_t*)vals[(size_t)pc.p * m + a] + o, len);
    }
  }
}

}  // namespace

namespace {

// One point-to-point operation of a transport group.
struct XOp {
  bool send;
  int peer;
  void* buf;
  size_t bytes;
};

// ---- loopback hub: S ranks of one process on one device.  Sends and
// receives queue per ordered (source, destination) pair; the k-th send of
// src to dst pairs with the k-th receive of dst from src (RCCL's rule within
// and across groups).  Whoever completes a pair issues its copy: the
// receiver's stream waits for the sender's "data ready" event, copies, and
// records the pair's "copied" event, which the sender's stream then waits
// for before it may overwrite the send buffer (no host wait on the data).
struct LoopPair {
  // send side
  const void* src = nullptr;
  size_t sbytes = 0;
  hipEvent_t ready = nullptr;  // recorded on the sender's stream at group end
  // receive side
  void* dst = nullptr;
  size_t rbytes = 0;
  hipStream_t rstream = nullptr;
  // result
  bool have_send = false, have_recv = false, done = false;
  // one side gave up waiting (timeout): the other side completes the pair
  // with an error and no copy (the buffers of the side that left may be gone)
  bool cancelled = false;
  int status = PSG_OK;
  hipEvent_t copied = nullptr;
  int users = 2;  // sender + receiver; the last one to leave frees the events
};

struct LoopHub {
  int S = 0, device = 0;
  std::mutex mu;
  std::condition_variable cv;
  // per ordered pair src * S + dst: pairs in posting order not yet completed
  std::vector<std::deque<std::shared_ptr<LoopPair>>> q;
  int refs = 0;

  void complete(LoopPair& P) {  // with mu held; both sides present
    P.done = true;
    if (P.cancelled) {
      P.status = PSG_ERR_DEVICE;
      return;
    }
    if (P.sbytes != P.rbytes) {
      P.status = PSG_ERR_SIZE;
      return;
    }
    hipError_t e = hipEventCreateWithFlags(&P.copied, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamWaitEvent(P.rstream, P.ready, 0);
    if (e == hipSuccess && P.sbytes)
      e = hipMemcpyAsync(P.dst, P.src, P.sbytes, hipMemcpyDeviceToDevice, P.rstream);
    if (e == hipSuccess) e = hipEventRecord(P.copied, P.rstream);
    if (e != hipSuccess) P.status = PSG_ERR_DEVICE;
  }
  static void leave(LoopPair& P) {  // with mu held
    if (--P.users == 0) {
      if (P.ready) (void)hipEventDestroy(P.ready);
      if (P.copied) (void)hipEventDestroy(P.copied);
      P.ready = P.copied = nullptr;
    }
  }
};

}  // namespace

struct psg_comm {
  ncclComm_t nccl = nullptr;
  LoopHub* loop = nullptr;  // loopback rank (psg_comm_init_loopback)
  int device = 0, nranks = 1, rank = 0;
};

namespace {

// seconds a loopback rank waits for its peers to post their side of a group
constexpr int kLoopTimeoutS = 120;

int loop_group(psg_comm* c, hipStream_t st, const std::vector<XOp>& ops) {
  LoopHub& H = *c->loop;
  const int S = H.S, me = c->rank;
  for (const XOp& o : ops)
    if (o.peer < 0 || o.peer >= S) return fail(PSG_ERR_ARG, "loopback peer %d", o.peer);
  // a "data ready" event per send: everything enqueued on `st` so far
  std::vector<hipEvent_t> ready(ops.size(), nullptr);
  for (size_t i = 0; i < ops.size(); ++i)
    if (ops[i].send) {
      hipError_t e = hipEventCreateWithFlags(&ready[i], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventRecord(ready[i], st);
      if (e != hipSuccess) {
        for (hipEvent_t x : ready)
          if (x) (void)hipEventDestroy(x);
        return fail(PSG_ERR_DEVICE, "loopback event: %s", hipGetErrorString(e));
      }
    }
  std::vector<std::shared_ptr<LoopPair>> mine;
  std::unique_lock<std::mutex> lk(H.mu);
  for (size_t i = 0; i < ops.size(); ++i) {
    const XOp& o = ops[i];
    auto& qq = o.send ? H.q[(size_t)me * S + o.peer] : H.q[(size_t)o.peer * S + me];
    // the oldest pair of this direction still missing this side
    std::shared_ptr<LoopPair> P;
    for (auto& x : qq)
      if (o.send ? !x->have_send : !x->have_recv) {
        P = x;
        break;
      }
    if (!P) {
      P = std::make_shared<LoopPair>();
      qq.push_back(P);
    }
    if (o.send) {
      P->have_send = true;
      P->src = o.buf;
      P->sbytes = o.bytes;
      P->ready = ready[i];
    } else {
      P->have_recv = true;
      P->dst = o.buf;
      P->rbytes = o.bytes;
      P->rstream = st;
    }
    if (P->have_send && P->have_recv) {
      H.complete(*P);
      while (!qq.empty() && qq.front()->done) qq.pop_front();
      H.cv.notify_all();
    }
    mine.push_back(P);
  }
  const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(kLoopTimeoutS);
  int rc = PSG_OK;
  for (auto& P : mine) {
    if (!H.cv.wait_until(lk, until, [&] { return P->done; })) {
      rc = fail(PSG_ERR_DEVICE, "loopback rank %d: a peer did not join the group", me);
      break;
    }
    if (P->status != PSG_OK && rc == PSG_OK)
      rc = fail(P->status, "loopback rank %d: %s", me,
                P->status == PSG_ERR_SIZE ? "send and receive sizes differ"
                : P->cancelled            ? "the peer left the group (timeout)"
                                          : "device copy failed");
  }
  // pairs still missing their peer: cancelled, so a peer that joins later
  // fails them instead of copying from or into this rank's buffers
  for (auto& P : mine)
    if (!P->done) P->cancelled = true;
  // a send buffer is reusable once its copy ran: later work on `st` waits
  for (size_t i = 0; rc == PSG_OK && i < ops.size(); ++i)
    if (ops[i].send && mine[i]->copied && hipStreamWaitEvent(st, mine[i]->copied, 0) != hipSuccess)
      rc = fail(PSG_ERR_DEVICE, "loopback: stream wait");
  for (auto& P : mine) LoopHub::leave(*P);
  return rc;
}

// One transport group: every op of `ops` on stream `st`.
int xport_group(psg_comm* c, hipStream_t st, const std::vector<XOp>& ops) {
  if (c->loop) return loop_group(c, st, ops);
  ncclResult_t r = ncclGroupStart();
  for (size_t i = 0; r == ncclSuccess && i < ops.size(); ++i) {
    const XOp& o = ops[i];
    r = o.send ? ncclSend(o.buf, o.bytes, ncclUint8, o.peer, c->nccl, st)
               : ncclRecv(o.buf, o.bytes, ncclUint8, o.peer, c->nccl, st);
  }
  const ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return fail(PSG_ERR_DEVICE, "RCCL group: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
  return PSG_OK;
}

}  // namespace

struct psg_exchange {
  psg_comm* comm = nullptr;  // null: a local exchange (S virtual shards, no transport)
  int device = 0;
  int dtype = 0, m = 1, P = 0, S = 1;
  std::vector<uint64_t> send_cnt;   // [s][p]
  std::vector<uint64_t> recv_cnt;   // [src][p]
  std::vector<uint64_t> send_tot, send_off, recv_tot, recv_off;  // per peer
  void* dev = nullptr;              // one device block for everything below
  uint64_t* skeys = nullptr;
  void* svals[psg::kMaxM] = {};
  uint64_t* rkeys = nullptr;
  void* rvals[psg::kMaxM] = {};
  const uint64_t* const* d_keys = nullptr;
  const void* const* d_vals = nullptr;
  void* const* d_svals = nullptr;
  void* const* d_rvals = nullptr;
  Piece* d_pieces = nullptr;
  uint64_t* d_chunks = nullptr;
  const uint64_t* d_n = nullptr;       // push lengths
  const uint64_t* d_bounds = nullptr;  // the S + 1 shard boundaries
  const uint64_t* d_pos = nullptr;     // the layout's cut positions [p][S + 1]
  unsigned long long* d_bad = nullptr; // positions that differed in a run's re-cut
  uint64_t nchunks = 0, nsend = 0, nrecv = 0;
  // direct mode (psg_exchange_set_direct): peer-bound pieces go to the
  // transport straight from the push arrays (one send per piece and array),
  // only this rank's own pieces are packed
  bool direct = false;
  std::vector<const uint64_t*> hkeys;  // the pushes (host copies of the tables)
  std::vector<const void*> hvals;
  std::vector<uint64_t> hpos;          // cut positions [p][S + 1]
  uint64_t* d_chunks_own = nullptr;    // chunks of the own pieces
  uint64_t nchunks_own = 0;
  hipStream_t last = nullptr;          // stream of the last run
};

namespace {
size_t al(size_t x) { return (x + 255) / 256 * 256; }
}  // namespace

extern "C" {

int psg_comm_unique_id(uint8_t* id) {
  if (!id) return fail(PSG_ERR_ARG, "null id");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, u.internal, PSG_COMM_ID_BYTES);
  return PSG_OK;
}

int psg_comm_init(int device, int nranks, const uint8_t* id, int rank, psg_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(PSG_ERR_ARG, "bad communicator arguments");
  HIP_TRY(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(u.internal, id, PSG_COMM_ID_BYTES);
  psg_comm* c = new psg_comm();
  c->device = device;
  c->nranks = nranks;
  c->rank = rank;
  ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(PSG_ERR_DEVICE, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  *out = c;
  return PSG_OK;
}

int psg_comm_init_loopback(int device, int nranks, psg_comm** out) {
  if (!out || nranks < 1) return fail(PSG_ERR_ARG, "bad loopback arguments");
  HIP_TRY(hipSetDevice(device));
  LoopHub* H = new LoopHub();
  H->S = nranks;
  H->device = device;
  H->q.resize((size_t)nranks * nranks);
  H->refs = nranks;
  for (int r = 0; r < nranks; ++r) {
    psg_comm* c = new psg_comm();
    c->device = device;
    c->nranks = nranks;
    c->rank = r;
    c->loop = H;
    out[r] = c;
  }
  return PSG_OK;
}

int psg_comm_destroy(psg_comm* c) {
  if (!c) return PSG_OK;
  if (c->nccl) (void)ncclCommDestroy(c->nccl);
  if (c->loop) {
    LoopHub* H = c->loop;
    bool last;
    {
      std::lock_guard<std::mutex> lk(H->mu);
      last = --H->refs == 0;
    }
    if (last) {
      (void)hipSetDevice(H->device);
      (void)hipDeviceSynchronize();
      for (auto& qq : H->q)
        for (auto& P : qq) {
          if (P->ready) (void)hipEventDestroy(P->ready);
          if (P->copied) (void)hipEventDestroy(P->copied);
        }
      delete H;
    }
  }
  delete c;
  return PSG_OK;
}

namespace {

// psg_exchange_create / psg_exchange_create_local.  comm == null: S local
// shards, no count exchange, no receive buffers.
int exchange_create(psg_comm* comm, int device, int S, int dtype, int m, int npush,
                    const uint64_t* const* push_keys, const uint64_t* push_n,
                    const void* const* push_vals, psg_exchange** out) {
  int err = PSG_OK;  // a local argument error; collective callers still exchange counts
  if (!out || npush < 0 || (npush && (!push_keys || !push_n || !push_vals)))
    err = fail(PSG_ERR_ARG, "null argument");
  else if (dtype != PSG_F32 && dtype != PSG_F64)
    err = fail(PSG_ERR_ARG, "dtype %d", dtype);
  else if (m < 1 || m > PSG_MAX_VALUE_ARRAYS)
    err = fail(PSG_ERR_ARG, "m=%d", m);
  if (err && !comm) return err;
  HIP_TRY(hipSetDevice(device));
  // an erring rank still takes part in the header round (its npush and an
  // error word), so every rank fails together instead of waiting on it
  const int P = npush < 0 ? 0 : npush, S1 = S + 1;
  const int vb = dtype == PSG_F32 ? 4 : 8;
  std::vector<uint64_t> bounds(S1);
  if (int rc = psg_shard_bounds((size_t)S, bounds.data())) return rc;
  hipStream_t st;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // ---- set-up block: bounds, push tables, cut positions, headers {npush,
  // error} to and from every peer, counts [s][p] to and from every peer
  const size_t o_b = 0, o_k = al(8 * S1), o_n = o_k + al(8 * P), o_pos = o_n + al(8 * P),
               o_hs = o_pos + al(8 * (size_t)P * S1), o_hr = o_hs + al(16 * (size_t)S),
               o_sc = o_hr + al(16 * (size_t)S), o_rc = o_sc + al(8 * (size_t)P * S),
               tot = o_rc + al(8 * (size_t)P * S);
  char* setup = nullptr;
  if (hipMalloc((void**)&setup, tot) != hipSuccess) {
    (void)hipStreamDestroy(st);
    return fail(PSG_ERR_OOM, "exchange set-up: %zu bytes", tot);
  }
  std::vector<uint64_t> pos((size_t)P * S1);
  psg_exchange* x = new psg_exchange();
  x->comm = comm;
  x->device = device;
  x->dtype = dtype;
  x->m = m;
  x->P = P;
  x->S = S;
  auto done = [&](int r) {
    (void)hipStreamSynchronize(st);
    (void)hipFree(setup);
    (void)hipStreamDestroy(st);
    if (r != PSG_OK) psg_exchange_destroy(x);
    return r;
  };
#define X_TRY(expr)                                                                  \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess)                                                            \
      return done(fail(PSG_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(_e)));   \
  } while (0)
  if (P && !err) {
    X_TRY(hipMemcpyAsync(setup + o_b, bounds.data(), 8 * S1, hipMemcpyHostToDevice, st));
    X_TRY(hipMemcpyAsync(setup + o_k, push_keys, 8 * (size_t)P, hipMemcpyHostToDevice, st));
    X_TRY(hipMemcpyAsync(setup + o_n, push_n, 8 * (size_t)P, hipMemcpyHostToDevice, st));
    const uint64_t waves = (uint64_t)P * S1;
    hipLaunchKernelGGL(cut_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, st,
                       (const uint64_t* const*)(setup + o_k), (const uint64_t*)(setup + o_n),
                       (const uint64_t*)(setup + o_b), S1, P, (uint64_t*)(setup + o_pos),
                       nullptr, nullptr);
    X_TRY(hipGetLastError());
    X_TRY(hipMemcpyAsync(pos.data(), setup + o_pos, 8 * pos.size(), hipMemcpyDeviceToHost, st));
    X_TRY(hipStreamSynchronize(st));
  }
  // send counts [s][p] (+ this rank's error word per peer); pieces in
  // destination-major, push order
  x->send_cnt.assign((size_t)S * P, 0);
  x->send_tot.assign(S, 0);
  x->send_off.assign(S, 0);
  std::vector<Piece> pieces;
  std::vector<uint64_t> chunks, chunks_own;
  uint64_t off = 0;
  // this rank's own pieces (a communicator's rank) go straight to the
  // receive buffers: their offsets there (push order, from recv_off[rank])
  // are fixed once the counts are known
  const int self = comm ? comm->rank : -1;
  uint64_t own = 0;  // elements of this rank's own pieces so far
  for (int s = 0; s < S; ++s) {
    x->send_off[s] = off;
    for (int p = 0; p < P; ++p) {
      const uint64_t a = pos[(size_t)p * S1 + s], b = pos[(size_t)p * S1 + s + 1];
      const uint64_t c = b > a ? b - a : 0;
      x->send_cnt[(size_t)s * P + p] = c;
      if (c && !err) {
        if (pieces.size() >= (1u << 24)) {
          err = fail(PSG_ERR_ARG, "too many pieces (> 2^24)");
          break;
        }
        const bool mine = s == self;
        for (uint64_t q = 0; q * kChunk < c; ++q) {
          chunks.push_back((uint64_t)pieces.size() << 24 | q);
          if (mine) chunks_own.push_back((uint64_t)pieces.size() << 24 | q);
        }
        pieces.push_back(Piece{a, mine ? own : off, c, (uint32_t)p, mine ? 1u : 0u});
      }
      if (s == self) own += c;  // own pieces take no send-buffer space
      else off += c;
    }
    x->send_tot[s] = off - x->send_off[s];
  }
  x->nsend = off;
  if (!comm) {
    if (err) return done(err);
  } else {
    // header round: {npush, error} to and from every peer.  Every rank
    // sees every header, so all decide alike: any error or a differing npush
    // fails every rank before the count round (whose sizes rest on npush)
    std::vector<uint64_t> hs(2 * (size_t)S), hr(2 * (size_t)S);
    for (int s = 0; s < S; ++s) {
      hs[2 * (size_t)s] = (uint64_t)P;
      hs[2 * (size_t)s + 1] = err ? 1u : 0u;
    }
    X_TRY(hipMemcpyAsync(setup + o_hs, hs.data(), 16 * (size_t)S, hipMemcpyHostToDevice, st));
    std::vector<XOp> ops;
    for (int s = 0; s < S; ++s) {
      ops.push_back(XOp{true, s, setup + o_hs + 16 * (size_t)s, 16});
      ops.push_back(XOp{false, s, setup + o_hr + 16 * (size_t)s, 16});
    }
    if (int rc = xport_group(comm, st, ops)) return done(rc);
    X_TRY(hipMemcpyAsync(hr.data(), setup + o_hr, 16 * (size_t)S, hipMemcpyDeviceToHost, st));
    X_TRY(hipStreamSynchronize(st));
    if (err) return done(err);
    for (int s = 0; s < S; ++s) {
      if (hr[2 * (size_t)s + 1])
        return done(fail(PSG_ERR_ARG, "exchange set-up failed on rank %d", s));
      if (hr[2 * (size_t)s] != (uint64_t)P)
        return done(fail(PSG_ERR_ARG, "rank %d has %llu pushes, this rank %d (every rank passes "
                         "the same npush)", s, (unsigned long long)hr[2 * (size_t)s], P));
    }
    // counts to their shards: P words to and from every peer
    std::vector<uint64_t> rc((size_t)P * S);
    if (P) {
      X_TRY(hipMemcpyAsync(setup + o_sc, x->send_cnt.data(), 8 * (size_t)P * S,
                           hipMemcpyHostToDevice, st));
      ops.clear();
      for (int s = 0; s < S; ++s) {
        ops.push_back(XOp{true, s, setup + o_sc + 8 * (size_t)s * P, 8 * (size_t)P});
        ops.push_back(XOp{false, s, setup + o_rc + 8 * (size_t)s * P, 8 * (size_t)P});
      }
      if (int r = xport_group(comm, st, ops)) return done(r);
      X_TRY(hipMemcpyAsync(rc.data(), setup + o_rc, 8 * rc.size(), hipMemcpyDeviceToHost, st));
      X_TRY(hipStreamSynchronize(st));
    }
    x->recv_cnt = rc;
  }
  x->recv_tot.assign(S, 0);
  x->recv_off.assign(S, 0);
  uint64_t roff = 0;
  for (int s = 0; comm && s < S; ++s) {
    x->recv_off[s] = roff;
    for (int p = 0; p < P; ++p) roff += x->recv_cnt[(size_t)s * P + p];
    x->recv_tot[s] = roff - x->recv_off[s];
  }
  x->nrecv = roff;
  x->nchunks = chunks.size();
  for (Piece& pc : pieces)
    if (pc.tgt) pc.dst += x->recv_off[self];
  // ---- the step's device block: send / receive buffers and the tables
  size_t b = 0;
  const size_t b_sk = b; b += al(8 * x->nsend);
  size_t b_sv[psg::kMaxM];
  for (int a = 0; a < m; ++a) { b_sv[a] = b; b += al((size_t)vb * x->nsend); }
  const size_t b_rk = b; b += al(8 * x->nrecv);
  size_t b_rv[psg::kMaxM];
  for (int a = 0; a < m; ++a) { b_rv[a] = b; b += al((size_t)vb * x->nrecv); }
  const size_t b_keys = b; b += al(8 * (size_t)P);
  const size_t b_vals = b; b += al(8 * (size_t)P * m);
  const size_t b_svp = b; b += al(8 * (size_t)m);
  const size_t b_rvp = b; b += al(8 * (size_t)m);
  const size_t b_pc = b; b += al(sizeof(Piece) * pieces.size());
  const size_t b_ch = b; b += al(8 * chunks.size());
  const size_t b_cho = b; b += al(8 * chunks_own.size());
  const size_t b_n = b; b += al(8 * (size_t)P);
  const size_t b_bd = b; b += al(8 * (size_t)S1);
  const size_t b_pos = b; b += al(8 * (size_t)P * S1);
  const size_t b_bad = b; b += al(8);
  X_TRY(hipMalloc(&x->dev, b));
  char* d = (char*)x->dev;
  x->skeys = (uint64_t*)(d + b_sk);
  x->rkeys = (uint64_t*)(d + b_rk);
  std::vector<uint64_t> svp(m), rvp(m);
  for (int a = 0; a < m; ++a) {
    x->svals[a] = d + b_sv[a];
    x->rvals[a] = d + b_rv[a];
    svp[a] = (uint64_t)x->svals[a];
    rvp[a] = (uint64_t)x->rvals[a];
  }
  x->d_keys = (const uint64_t* const*)(d + b_keys);
  x->d_vals = (const void* const*)(d + b_vals);
  x->d_svals = (void* const*)(d + b_svp);
  x->d_rvals = (void* const*)(d + b_rvp);
  x->d_pieces = (Piece*)(d + b_pc);
  x->d_chunks = (uint64_t*)(d + b_ch);
  x->d_chunks_own = (uint64_t*)(d + b_cho);
  x->nchunks_own = chunks_own.size();
  x->hkeys.assign(push_keys, push_keys + P);
  x->hvals.assign(push_vals, push_vals + (size_t)P * m);
  x->hpos = pos;
  x->d_n = (const uint64_t*)(d + b_n);
  x->d_bounds = (const uint64_t*)(d + b_bd);
  x->d_pos = (const uint64_t*)(d + b_pos);
  x->d_bad = (unsigned long long*)(d + b_bad);
  if (P) {
    X_TRY(hipMemcpyAsync(d + b_keys, push_keys, 8 * (size_t)P, hipMemcpyHostToDevice, st));
    X_TRY(hipMemcpyAsync(d + b_vals, push_vals, 8 * (size_t)P * m, hipMemcpyHostToDevice, st));
    X_TRY(hipMemcpyAsync(d + b_n, push_n, 8 * (size_t)P, hipMemcpyHostToDevice, st));
    X_TRY(hipMemcpyAsync(d + b_pos, pos.data(), 8 * pos.size(), hipMemcpyHostToDevice, st));
  }
  X_TRY(hipMemcpyAsync(d + b_bd, bounds.data(), 8 * (size_t)S1, hipMemcpyHostToDevice, st));
  X_TRY(hipMemsetAsync(d + b_bad, 0, 8, st));
  X_TRY(hipMemcpyAsync(d + b_svp, svp.data(), 8 * (size_t)m, hipMemcpyHostToDevice, st));
  X_TRY(hipMemcpyAsync(d + b_rvp, rvp.data(), 8 * (size_t)m, hipMemcpyHostToDevice, st));
  if (!pieces.empty())
    X_TRY(hipMemcpyAsync(d + b_pc, pieces.data(), sizeof(Piece) * pieces.size(),
                         hipMemcpyHostToDevice, st));
  if (!chunks.empty())
    X_TRY(hipMemcpyAsync(d + b_ch, chunks.data(), 8 * chunks.size(), hipMemcpyHostToDevice, st));
  if (!chunks_own.empty())
    X_TRY(hipMemcpyAsync(d + b_cho, chunks_own.data(), 8 * chunks_own.size(),
                         hipMemcpyHostToDevice, st));
#undef X_TRY
  *out = x;
  return done(PSG_OK);
}

}  // namespace

int psg_exchange_create(psg_comm* comm, int dtype, int m, int npush,
                        const uint64_t* const* push_keys, const uint64_t* push_n,
                        const void* const* push_vals, psg_exchange** out) {
  if (!comm) return fail(PSG_ERR_ARG, "null communicator");
  return exchange_create(comm, comm->device, comm->nranks, dtype, m, npush, push_keys, push_n,
                         push_vals, out);
}

int psg_exchange_create_local(int device, int nshards, int dtype, int m, int npush,
                              const uint64_t* const* push_keys, const uint64_t* push_n,
                              const void* const* push_vals, psg_exchange** out) {
  if (nshards < 1) return fail(PSG_ERR_ARG, "nshards=%d", nshards);
  return exchange_create(nullptr, device, nshards, dtype, m, npush, push_keys, push_n, push_vals,
                         out);
}

int psg_exchange_run(psg_exchange* x, void* stream) {
  if (!x) return fail(PSG_ERR_ARG, "null exchange");
  HIP_TRY(hipSetDevice(x->device));
  hipStream_t st = (hipStream_t)stream;
  x->last = st;
  const int vb = x->dtype == PSG_F32 ? 4 : 8;
  if (x->P) {
    // the cut of this step's pushes, checked against the layout (no host wait)
    const int S1 = x->S + 1;
    const uint64_t waves = (uint64_t)x->P * S1;
    hipLaunchKernelGGL(cut_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, st, x->d_keys,
                       x->d_n, x->d_bounds, S1, x->P, nullptr, x->d_pos, x->d_bad);
    HIP_TRY(hipGetLastError());
  }
  const bool direct = x->direct && x->comm;
  const uint64_t nch = direct ? x->nchunks_own : x->nchunks;
  if (nch) {
    const uint64_t blocks = nch < 4096 ? nch : 4096;
    hipLaunchKernelGGL(pack_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, x->d_pieces,
                       direct ? x->d_chunks_own : x->d_chunks, nch, x->d_keys, x->d_vals, x->m,
                       vb, x->skeys, x->d_svals, x->rkeys, x->d_rvals);
    HIP_TRY(hipGetLastError());
  }
  if (!x->comm) return PSG_OK;  // local shards: the packed buffers are the result
  std::vector<XOp> ops;
  const int S1 = x->S + 1;
  for (int s = 0; s < x->S; ++s) {
    if (s == x->comm->rank) continue;  // own pieces were packed into the receive buffers
    if (direct) {
      // per push in order: its keys, then its m value arrays -- the
      // receiver posts the same sequence (the count round told it the
      // sizes), so RCCL pairs them one to one
      for (int p = 0; p < x->P; ++p) {
        const uint64_t a = x->hpos[(size_t)p * S1 + s], c = x->send_cnt[(size_t)s * x->P + p];
        if (!c) continue;
        ops.push_back(XOp{true, s, (void*)(x->hkeys[p] + a), 8 * c});
        for (int i = 0; i < x->m; ++i)
          ops.push_back(XOp{true, s, (char*)x->hvals[(size_t)p * x->m + i] + a * vb, (size_t)vb * c});
      }
      uint64_t o = x->recv_off[s];
      for (int p = 0; p < x->P; ++p) {
        const uint64_t c = x->recv_cnt[(size_t)s * x->P + p];
        if (!c) continue;
        ops.push_back(XOp{false, s, x->rkeys + o, 8 * c});
        for (int i = 0; i < x->m; ++i)
          ops.push_back(XOp{false, s, (char*)x->rvals[i] + o * vb, (size_t)vb * c});
        o += c;
      }
      continue;
    }
    if (x->send_tot[s]) {
      ops.push_back(XOp{true, s, x->skeys + x->send_off[s], 8 * x->send_tot[s]});
      for (int a = 0; a < x->m; ++a)
        ops.push_back(XOp{true, s, (char*)x->svals[a] + x->send_off[s] * vb,
                          (size_t)vb * x->send_tot[s]});
    }
    if (x->recv_tot[s]) {
      ops.push_back(XOp{false, s, x->rkeys + x->recv_off[s], 8 * x->recv_tot[s]});
      for (int a = 0; a < x->m; ++a)
        ops.push_back(XOp{false, s, (char*)x->rvals[a] + x->recv_off[s] * vb,
                          (size_t)vb * x->recv_tot[s]});
    }
  }
  return xport_group(x->comm, st, ops);
}

int psg_exchange_set_direct(psg_exchange* x, int on) {
  if (!x) return fail(PSG_ERR_ARG, "null exchange");
  if (!x->comm) return fail(PSG_ERR_ARG, "direct mode needs a communicator");
  x->direct = on != 0;
  return PSG_OK;
}

int psg_exchange_status(psg_exchange* x, uint64_t* changed) {
  if (!x) return fail(PSG_ERR_ARG, "null exchange");
  HIP_TRY(hipSetDevice(x->device));
  if (x->last) HIP_TRY(hipStreamSynchronize(x->last));
  unsigned long long bad = 0;
  HIP_TRY(hipMemcpy(&bad, x->d_bad, 8, hipMemcpyDeviceToHost));
  if (changed) *changed = bad;
  if (bad)
    return fail(PSG_ERR_SIZE, "exchange: %llu cut positions differ from the set-up layout", bad);
  return PSG_OK;
}

int psg_exchange_send_layout(psg_exchange* x, const uint64_t** keys, void** vals,
                             uint64_t* send_cnt) {
  if (!x) return fail(PSG_ERR_ARG, "null exchange");
  if (keys) *keys = x->skeys;
  for (int a = 0; vals && a < x->m; ++a) vals[a] = x->svals[a];
  if (send_cnt && !x->send_cnt.empty())
    memcpy(send_cnt, x->send_cnt.data(), 8 * x->send_cnt.size());
  return PSG_OK;
}

int psg_exchange_recv(psg_exchange* x, const uint64_t** keys, void** vals, uint64_t* nrecv,
                      uint64_t* recv_cnt, uint64_t* sent) {
  if (!x) return fail(PSG_ERR_ARG, "null exchange");
  if (keys) *keys = x->rkeys;
  for (int a = 0; vals && a < x->m; ++a) vals[a] = x->rvals[a];
  if (nrecv) *nrecv = x->nrecv;
  if (recv_cnt) memcpy(recv_cnt, x->recv_cnt.data(), 8 * x->recv_cnt.size());
  if (sent) *sent = x->nsend;
  return PSG_OK;
}

int psg_exchange_destroy(psg_exchange* x) {
  if (!x) return PSG_OK;
  if (x->dev) {
    (void)hipSetDevice(x->device);
    (void)hipDeviceSynchronize();
    (void)hipFree(x->dev);
  }
  delete x;
  return PSG_OK;
}

}  // extern "C"
