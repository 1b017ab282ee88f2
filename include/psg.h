/*
 * psg.h -- C ABI of the MI355X-native server-side push aggregation path.
 *
 * This is the drop-in boundary that replaces the host-side hot path of
 * wakensky/parameter_server:
 *
 *   KVVector<uint64,V>::setValue / serialSetValue / parallelSetValue
 *       src/parameter/kv_vector.h:75-82, 84-137, 171-204
 *   KVVector<uint64,V>::received          src/parameter/kv_vector.h:65-73
 *   KVVector<uint64,V>::getValue (pull)   src/parameter/kv_vector.h:206-227
 *   match / oldMatch merge kernels        src/system/message.h:134-267
 *   SArray::setUnion / findRange          src/base/shared_array_inl.h:155-171
 *   sliceKeyOrderedMsg / Range::evenDivide src/system/message.h:89-123,
 *                                          src/base/range.h:85-98
 *
 * The reference calls these from SharedParameter<K>::process on the
 * customer's executor thread (src/parameter/shared_parameter.h:91-149).
 * Every entry point here takes plain pointers and sizes; none retains a
 * caller pointer past the call (host data is staged before return), and
 * every failure the reference turns into a glog CHECK abort is returned as
 * a negative psg_status instead (the C++ adapter converts it back to an
 * abort, see parameter_server_amd/csrc/kv_vector.h).
 *
 * Keys are uint64 (the reference's PS::Key); values are float or double
 * (KVVector<Key,double> in linear_method/batch_solver.h:32).
 */
#ifndef PSG_H_
#define PSG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSG_ABI_VERSION 1
#define PSG_MAX_VALUE_ARRAYS 4   /* m: value arrays per push (Darling: 2) */

typedef enum psg_status {
  PSG_OK = 0,
  PSG_ERR_ARG = -1,        /* bad argument (null pointer, m out of range ...) */
  PSG_ERR_UNMATCHED = -2,  /* CHECK_EQ(recv_key.size(), n)  kv_vector.h:134,192 */
  PSG_ERR_RANGE = -3,      /* CHECK_EQ(range, stored range) kv_vector.h:128,199 */
  PSG_ERR_NO_TIME = -4,    /* CHECK(it != recved_val_.end()) kv_vector.h:69 */
  PSG_ERR_OOM = -5,
  PSG_ERR_DEVICE = -6,     /* HIP runtime error / no device */
  PSG_ERR_UNSORTED = -7,   /* key-only push not strictly increasing */
  PSG_ERR_SIZE = -8,       /* CHECK_EQ(recv_data.size(), recv_key.size()) :108,187 */
  PSG_ERR_CHANNEL = -9,    /* pushes of one time t name different channels */
  PSG_ERR_EMPTY_KEYS = -10, /* value push to a channel with no server keys */
  PSG_ERR_SIGNATURE = -11   /* key signature / key cache mismatch
                               CHECK_EQ remote_node.cc:163,174 */
} psg_status;

typedef enum psg_dtype { PSG_F32 = 0, PSG_F64 = 1 } psg_dtype;

/* Aggregation semantics (FLAGS_parallel_match, system/postoffice.cc:24).
 * SERIAL (the shipped default, script/local.sh:35) adds an explicit +0.0 for
 * keys absent from a later push (kv_vector.h:200), so a -0.0 can become
 * +0.0; PARALLEL touches only matched keys (message.h:195-198).  Both are
 * reproduced bit-exactly. */
#define PSG_SERIAL_MATCH 0u
#define PSG_PARALLEL_MATCH 1u
/* Context option (psg_create / psg_set_match_flags flags): the caller keeps
 * the key and value buffers of psg_push / psg_push_cached valid and
 * unmodified until psg_received of that time returns -- as the reference's
 * MessagePtr keeps a message's SArrays alive -- so pinned buffers are DMA'd
 * without a wait per push.  Without it every push returns with the caller's
 * buffers free. */
#define PSG_HOLD_BUFFERS 0x100u
/* Kernel-form overrides, for tests and A/B measurements (flags of
 * psg_plan_create, psg_create and psg_set_match_flags).  By default the
 * runtime picks each form from the shape of the pushes; the results are
 * bit-identical whichever form runs.  No environment variable changes the
 * path. */
#define PSG_FORM_PACKED 0x1000u   /* rounds that pack several pushes (short pieces) */
#define PSG_FORM_UNIFORM 0x2000u  /* rounds of one push each (long pieces) */
#define PSG_PART_SEARCH 0x4000u   /* partition: one search per (push, tile boundary) */
#define PSG_PART_STREAM 0x8000u   /* partition: every push key read once */
#define PSG_GROUP32 0x10000u      /* uniform rounds: groups of 32 pushes, 1024-slot tiles */
#define PSG_GROUP64 0x20000u      /* uniform rounds: groups of 64 pushes, 2048-slot tiles */
#define PSG_NO_DENSE 0x40000u     /* never the dense (contiguous-slice) kernel */
#define PSG_NO_ZERO_COPY 0x80000u /* context: DMA copies instead of GPU reads of pinned memory */
#define PSG_NO_INDEX 0x100000u    /* plan: no resident bucket index (tables built per run) */
#define PSG_FORM_CURSOR 0x400000u /* plan: a cursor form (no partition pass) where it applies */
#define PSG_NO_CURSOR 0x800000u   /* plan: never a cursor form (the default) */
/* Plan option (psg_plan_create): the caller promises that the push KEYS at
 * the job's device pointers stay as they were at creation for the plan's
 * lifetime (values may change between runs).  Only then may the plan take
 * the dense kernel for pushes that are contiguous slices of D: that kernel
 * reads no push keys, so it cannot see a key that changed.  Without this
 * flag every run partitions and order-checks the keys it merges, and a
 * changed key is reported through psg_plan_matched.  (D itself is always
 * fixed for a plan's lifetime: its bucket index is built at creation.) */
#define PSG_STATIC_KEYS 0x200000u

int psg_abi_version(void);
const char* psg_status_string(int status);
/* Thread-local text of the last error returned on this thread. */
const char* psg_last_error(void);
int psg_device_count(int* n);

/* ------------------------------------------------------------------ */
/* Server context: one KVVector<uint64,V> whose keys, values and      */
/* per-time aggregates are resident in the HBM of one device.         */
/* ------------------------------------------------------------------ */
typedef struct psg_ctx psg_ctx;

int psg_create(int device, int dtype, unsigned flags, psg_ctx** out);
int psg_destroy(psg_ctx* ctx);
int psg_set_match_flags(psg_ctx* ctx, unsigned flags);
/* Pushes of one time merged per launch (default and maximum
 * psg_plan_max_push()); an aggregate of more pushes continues across
 * launches with the same bits.  Lower values force launch seams (tests). */
int psg_set_flush_pushes(psg_ctx* ctx, int n);

/* Key-only push: key_[chl] = key_[chl].setUnion(keys); val_[chl].clear()
 * (kv_vector.h:177-182).  keys must be strictly increasing. */
int psg_key_union(psg_ctx* ctx, int chl, const uint64_t* keys, size_t n);
/* npush key-only pushes at once: the same key set as psg_key_union of each
 * in order (the union is order-free), merged on the device in one N-way
 * pass per psg_nway_max_push() - 1 pushes (BatchSolver::preprocessData's
 * key pushes, batch_solver.cc:318-323).  Empty pushes are ignored. */
int psg_key_union_batch(psg_ctx* ctx, int chl, const uint64_t* const* keys, const size_t* n,
                        int npush);
/* key(chl).size() / copy of key(chl)[off, off+n) (kv_vector.h:17). */
int psg_key_size(psg_ctx* ctx, int chl, size_t* n);
int psg_key_copy(psg_ctx* ctx, int chl, size_t off, size_t n, uint64_t* out);
/* find(chl, [kb,ke)) = key_[chl].findRange (kv_vector.h:21-23). */
int psg_find_range(psg_ctx* ctx, int chl, uint64_t kb, uint64_t ke,
                   size_t* lo, size_t* hi);
/* value(chl) (kv_vector.h:18): replace / read the server values. */
int psg_value_assign(psg_ctx* ctx, int chl, const void* vals, size_t n);
int psg_value_size(psg_ctx* ctx, int chl, size_t* n);
int psg_value_copy(psg_ctx* ctx, int chl, size_t off, size_t n, void* out);

/* Value push: setValue(msg) for msg->value of m arrays, each n entries,
 * msg->task.key_range() = [kb, ke), msg->task.time() = time,
 * msg->task.key_channel() = chl.  vals[i] points to array i.  The caller's
 * buffers are free on return: pinned host memory (hipHostMalloc /
 * hipHostRegister) is DMA'd directly, pageable memory is copied into a
 * pinned staging ring whose DMA continues after return.  The merge runs
 * asynchronously on the context's stream and its match check is reported
 * by psg_received for `time`.  Pushes of one `time` may carry different m:
 * the aggregate's list of arrays grows to the largest (recved_val_[t],
 * kv_vector.h:110-129,189-196); array i is assigned by the first push
 * holding an i-th array and added to by the later pushes holding one. */
int psg_push(psg_ctx* ctx, int chl, int time, uint64_t kb, uint64_t ke,
             const uint64_t* keys, size_t n, int m, const void* const* vals);

/* Value push of snappy-compressed parts, as they arrive off the wire
 * (Van::recv with task.uncompressed_size set, van.cc:204-214): the key part
 * (uint64 keys) and m value parts are DMA'd compressed and decompressed on
 * the device (psg_snappy_uncompress_dev), then pushed like psg_push.
 * Parts of inconsistent declared sizes are PSG_ERR_SIZE here (the
 * reference's CHECKs).  The decode runs asynchronously (the caller's
 * buffers are free on return, as for psg_push): a part that fails to decode
 * is reported by psg_received(time) as PSG_ERR_ARG, for the whole aggregate. */
int psg_push_compressed(psg_ctx* ctx, int chl, int time, uint64_t kb, uint64_t ke,
                        const void* ckeys, size_t ckeys_bytes, int m,
                        const void* const* cvals, const size_t* cvals_bytes);

/* Value or key push through the receiver's key cache: RNode::cacheKeyRecver
 * (src/system/remote_node.cc:139-184) followed by setValue.  The server
 * keeps one cache per remote node (RNode::key_cache_, remote_node.h:92-93):
 * `sender` names it (any caller-chosen id, e.g. the worker's rank).  `kc` carries
 * the task's key-cache fields:
 *   PSG_KC_SIG   task.has_key_signature(), signature `sig`;
 *   PSG_KC_KEYS  task.has_key(): the message carries keys[nkeys];
 *   PSG_KC_ERASE task.erase_key_cache().
 * Each cache is indexed by (chl, [kb, ke)).  No signature: the entry is
 * dropped and the message's keys are used.  Signature + keys: the keys'
 * crc32c over their first PSG_MAX_SIG_LEN bytes (computed on the GPU) must
 * equal `sig`, and the resident copy is cached under `sig`.  With values
 * (m > 0) the check runs on the device without a host wait and a mismatch
 * is reported by psg_received for `time` (PSG_ERR_SIGNATURE); a key-only
 * message (m == 0) is checked before its union and fails here.
 * Signature without keys: the cached keys are used in place (no key bytes
 * cross PCIe); a missing entry or another signature is PSG_ERR_SIGNATURE
 * (sig 0 against a missing entry restores no keys: the message is
 * ignored, as the reference's empty key list is).  m == 0 is a key-only
 * message (setUnion, merged on the device); otherwise nvals must equal the
 * key count (PSG_ERR_SIZE, nvals == 0 included: kv_vector.h:108,187). */
#define PSG_KC_SIG 1u
#define PSG_KC_KEYS 2u
#define PSG_KC_ERASE 4u
int psg_push_cached(psg_ctx* ctx, int sender, int chl, int time, uint64_t kb,
                    uint64_t ke, unsigned kc, uint32_t sig, const uint64_t* keys, size_t nkeys,
                    int m, const void* const* vals, size_t nvals);
/* RNode::clearCache (remote_node.h:54) / memSize (remote_node.cc:186-195)
 * of one sender's cache (sender < 0: every sender). */
int psg_key_cache_clear(psg_ctx* ctx, int sender);
int psg_key_cache_bytes(psg_ctx* ctx, int sender, size_t* bytes);
/* Shape of the aggregate of `time`: m arrays over server positions
 * [lo, hi) of key(chl).  PSG_ERR_NO_TIME if nothing was pushed. */
int psg_received_shape(psg_ctx* ctx, int time, int* m, size_t* lo,
                       size_t* hi);
/* received(t): copies the m aggregates (hi-lo entries each) into out[i] and
 * erases them.  Returns PSG_ERR_UNMATCHED if any push of `time` had a key
 * that is not a server key of its range (or was unsorted / duplicated). */
int psg_received(psg_ctx* ctx, int time, int m, void* const* out);

/* Pull reply: getValue(msg) (kv_vector.h:206-227): out[i] = value(chl) at
 * keys[i], 0 where keys[i] is not a server key.  keys sorted (repeats
 * allowed); PSG_ERR_UNSORTED otherwise. */
int psg_gather(psg_ctx* ctx, int chl, const uint64_t* keys, size_t n,
               void* out, size_t* matched);

/* ------------------------------------------------------------------ */
/* Device-resident batched merge: the hot path with every buffer      */
/* already in HBM (benchmarks, multi-GPU shards, graph capture).      */
/* ------------------------------------------------------------------ */
typedef struct psg_merge_job {
  const uint64_t* keys;      /* device: server keys D[lo, hi) (sorted unique) */
  uint64_t nslots;           /* hi - lo */
  int npush;                 /* pushes of this (channel, time), arrival order */
  const uint64_t* const* push_keys; /* host array[npush] of device pointers */
  const void* const* push_vals;     /* host array[npush*m], [p*m + i] */
  const uint64_t* push_n;           /* host array[npush] */
  void* const* out;          /* host array[m] of device pointers, nslots each */
} psg_merge_job;

typedef struct psg_plan psg_plan;

/* All jobs share dtype, m and flags; npush <= psg_plan_max_push() per job.
 * CONTRACT: each job's server keys (the `keys` array, D) must keep their
 * contents for the plan's lifetime.  The plan builds a bucket index of D at
 * creation and every run searches with it; if D changes between runs, keys
 * are misplaced and show up as unmatched in psg_plan_matched.  To merge
 * against a different D, create a new plan (or pass PSG_NO_INDEX, which
 * rebuilds the tables from D in every run).  Push keys and values may
 * change between runs (see PSG_STATIC_KEYS for the one exception). */
int psg_plan_create(int device, int dtype, int m, unsigned flags,
                    const psg_merge_job* jobs, int njobs, psg_plan** out);
int psg_plan_max_push(void);
/* Enqueue the merge on `stream` (a hipStream_t; NULL = default stream).
 * No allocation, no synchronisation: capturable into a hipGraph. */
int psg_plan_run(psg_plan* plan, void* stream);
/* One stage of psg_plan_run: 0 = partition (findRange / slice lower
 * bounds), 1 = aggregate.  Lets a caller bracket the dominant kernel with
 * its own events on `stream`. */
int psg_plan_run_stage(psg_plan* plan, int stage, void* stream);
/* Synchronises the plan's last run and returns per-push matched counts,
 * jobs in order, pushes in order (sum of npush entries). */
int psg_plan_matched(psg_plan* plan, uint64_t* matched);
/* The aggregate kernel a plan runs (its form, chosen at creation from the
 * shape of the jobs or by the PSG_FORM_* flags): */
#define PSG_KERNEL_TILE 0    /* partition + push-uniform rounds, 1024-slot tiles */
#define PSG_KERNEL_TILE64 1  /* partition + push-uniform rounds, 64-push groups */
#define PSG_KERNEL_PACKED 2  /* partition + rounds packing several pushes */
#define PSG_KERNEL_DENSE 3   /* contiguous slices: no key reads */
#define PSG_KERNEL_CURSOR 4  /* no partition: per-push cursors across tile chunks */
#define PSG_KERNEL_PACKED_CURSOR 5  /* no partition: packed rounds, cursors across tile chunks */
int psg_plan_form(psg_plan* plan, int* form);
/* Algorithmic HBM bytes of one run (SURVEY.md 8d general form). */
int psg_plan_bytes(psg_plan* plan, uint64_t* bytes, uint64_t* kv_pairs);
int psg_plan_destroy(psg_plan* plan);

/* Device-resident gather (pull reply) over resident keys/values. */
int psg_gather_dev(int dtype, const uint64_t* dkeys, uint64_t nd,
                   const void* dvals, const uint64_t* req, uint64_t nreq,
                   void* out, unsigned long long* matched, void* stream);

/* Device-resident key union: out = a U b (both strictly increasing, else
 * PSG_ERR_UNSORTED); out must hold na+nb; *nout (host) receives |a U b|.
 * The N-way merge of psg_nway_* with two pushes.  Synchronises. */
int psg_key_union_dev(const uint64_t* a, uint64_t na, const uint64_t* b,
                      uint64_t nb, uint64_t* out, uint64_t* nout,
                      void* stream);

/* ------------------------------------------------------------------ */
/* N-way merge of sorted pushes into their merged key set  */
/* ------------------------------------------------------------------ */
/* out_keys = the union of the npush pushes' keys (SArray::setUnion applied
 * push after push, shared_array_inl.h:155-162), sorted; with m > 0 value
 * arrays, out_vals[i][j] = the sum over the pushes holding out_keys[j] in
 * arrival order -- KVVector::serialSetValue / parallelSetValue over that
 * key set (kv_vector.h:84-204; flags PSG_SERIAL_MATCH / PSG_PARALLEL_MATCH).
 * Empty pushes are ignored (kv_vector.h:90,177); at most psg_nway_max_push()
 * non-empty pushes and < 2^32 keys in total.  All pointers are device
 * pointers except the host arrays keys[npush], n[npush], vals[npush * m]
 * and out_vals[m]; out_keys / out_vals hold sum(n) entries.  The pushes'
 * buffers are read again by every run (a prepared merge, like psg_plan).
 * Run: no host wait, capturable; the merged count is a device word
 * (psg_nway_count_dev).  psg_nway_result synchronises and returns
 * PSG_ERR_UNSORTED if a push was not strictly increasing (the reference's
 * std::set_union precondition; the output is then unspecified). */
typedef struct psg_nway psg_nway;
int psg_nway_max_push(void);
int psg_nway_create(int device, int dtype, int m, unsigned flags, int npush,
                    const uint64_t* const* keys, const uint64_t* n, const void* const* vals,
                    uint64_t* out_keys, void* const* out_vals, psg_nway** out);
/* A batch of nmerge independent merges run as one pipeline (one launch per
 * stage over all of them: e.g. the 64 aggregates of a bench step).  Merge j
 * has npush[j] pushes; keys / n / vals list the merges' pushes back to back
 * (vals: m per push); out_keys[j] and out_vals[j * m + i] are merge j's
 * outputs.  psg_nway_create is the batch of one. */
int psg_nway_create_batch(int device, int dtype, int m, unsigned flags, int nmerge,
                          const int* npush, const uint64_t* const* keys, const uint64_t* n,
                          const void* const* vals, uint64_t* const* out_keys,
                          void* const* out_vals, psg_nway** out);
int psg_nway_run(psg_nway* u, void* stream);
/* the first merge's merged-count word (device) */
int psg_nway_count_dev(psg_nway* u, unsigned long long** nout);
/* nout (host, nullable): one merged count per merge */
int psg_nway_result(psg_nway* u, uint64_t* nout);
/* Algorithmic bytes read by a run (sum(n) * (8 + m s_V)) and keys read;
 * the merged output adds |union| * (8 + m s_V). */
int psg_nway_bytes(psg_nway* u, uint64_t* bytes, uint64_t* kv_pairs);
int psg_nway_destroy(psg_nway* u);

/* ------------------------------------------------------------------ */
/* Shard exchange over RCCL ("unsliced" ingress)          */
/* ------------------------------------------------------------------ */
/* One communicator per rank and GPU (RCCL = NCCL API over xGMI).  Rank 0
 * makes the id and the caller broadcasts it (any channel). */
#define PSG_COMM_ID_BYTES 128
typedef struct psg_comm psg_comm;
int psg_comm_unique_id(uint8_t* id);
int psg_comm_init(int device, int nranks, const uint8_t* id, int rank,
                  psg_comm** out);
int psg_comm_destroy(psg_comm* comm);
/* nranks loopback communicators of ONE process on one device (out[r] is
 * rank r): the exchange's collective rounds run with the same pairing rule
 * as RCCL's grouped send/recv, each matched pair a device copy.  Each rank
 * must call the collective functions from its own host thread, all ranks
 * concurrently (as RCCL ranks do from their own processes); a rank whose
 * peers do not join within 120 s gets PSG_ERR_DEVICE.  For tests of the
 * multi-rank path on one GPU (RCCL refuses two ranks on one device).
 * Destroy every rank's communicator. */
int psg_comm_init_loopback(int device, int nranks, psg_comm** out);

/* RNode::submit's slice-and-send (remote_node.cc:39-60: KVVector::slice ->
 * sliceKeyOrderedMsg, message.h:89-123) for a batch of npush sorted
 * device-resident pushes held by this rank, at the server ranges
 * Range<uint64>::all().evenDivide(nranks, s) (linear_method.cc:137-145).
 * Every rank passes the same npush, dtype and m.  Create (synchronous,
 * collective): cut positions, piece counts exchanged, buffers sized.
 * Run (collective, enqueued on `stream`): pack + one grouped send/recv per
 * peer.  Afterwards psg_exchange_recv gives the received keys / m value
 * arrays (device) and recv_cnt[src * npush + p] (host, may be NULL): the
 * piece of push p of rank src starts after all earlier (src, p) pieces;
 * *nsent = keys this rank sends to the other ranks (its own pieces are
 * packed straight into its receive buffers and never cross the transport). */
typedef struct psg_exchange psg_exchange;
int psg_exchange_create(psg_comm* comm, int dtype, int m, int npush,
                        const uint64_t* const* push_keys, const uint64_t* push_n,
                        const void* const* push_vals, psg_exchange** out);
int psg_exchange_run(psg_exchange* x, void* stream);
int psg_exchange_recv(psg_exchange* x, const uint64_t** keys, void** vals,
                      uint64_t* nrecv, uint64_t* recv_cnt, uint64_t* nsent);
int psg_exchange_destroy(psg_exchange* x);
/* The layout is fixed at create (the pushes' device buffers are read again
 * by every run, like a psg_plan's).  Each run also redoes the cut on the
 * device and counts the positions that differ from the layout (pushes whose
 * keys changed since create); psg_exchange_status synchronises the last
 * run's stream and returns PSG_ERR_SIZE (*changed = that count) if any run
 * saw one.  The run's pieces are then those of the create-time cut. */
int psg_exchange_status(psg_exchange* x, uint64_t* changed);
/* Direct mode (on != 0; communicator exchanges only): a run sends every
 * peer-bound piece straight from the push arrays (one send per piece and
 * array, the receiver posts the matching receives in the same order) instead
 * of packing them into the send buffer first; own pieces are still packed
 * into the receive buffers.  Same received layout and bytes either way. */
int psg_exchange_set_direct(psg_exchange* x, int on);
/* The same slice-and-pack for nshards virtual shards on one device with no
 * communicator ("8 shards on 1 device"): a run re-cuts and packs
 * only; psg_exchange_send_layout gives the packed buffers (device) and
 * send_cnt[s * npush + p] (host, may be NULL): shard s's piece of push p
 * starts after all earlier (s, p) pieces.  Works on either kind. */
int psg_exchange_create_local(int device, int nshards, int dtype, int m, int npush,
                              const uint64_t* const* push_keys, const uint64_t* push_n,
                              const void* const* push_vals, psg_exchange** out);
int psg_exchange_send_layout(psg_exchange* x, const uint64_t** keys, void** vals,
                             uint64_t* send_cnt);

/* Server shard boundaries: Range<uint64>::all().evenDivide(n, i)
 * (range.h:75-98, linear_method.cc:137-145); bounds[n+1]. */
int psg_shard_bounds(size_t n, uint64_t* bounds);
/* sliceKeyOrderedMsg positions (message.h:89-123) of a device-resident
 * sorted push: pos[nsep] device array, computed on `stream`. */
int psg_slice_dev(const uint64_t* keys, uint64_t n, uint64_t kb, uint64_t ke,
                  const uint64_t* sep, int nsep, uint64_t* pos, void* stream);

/* ------------------------------------------------------------------ */
/* Server model update fused on the resident aggregate (Darling, L1-LR */
/* block coordinate descent; src/linear_method/darling.cc)             */
/* ------------------------------------------------------------------ */
typedef struct psg_darling_param {
  double eta;                  /* conf_.learning_rate().eta() */
  double lambda;               /* conf_.penalty().lambda(0) */
  double kkt_filter_threshold; /* Darling::KKT_filter_threshold_ */
  double delta_max;            /* conf_.darling().delta_max_value() */
} psg_darling_param;

/* Darling::preprocessData server state of channel grp (darling.cc:
 * 111-117): active_set all true, delta = delta_init, sized to key(chl).
 * Requires a PSG_F64 context (KVVector<Key,double>). */
int psg_darling_init(psg_ctx* ctx, int chl, double delta_init);
/* kkt_filter_reset: active_set.fill(true) (darling.cc:167-169). */
int psg_darling_reset_active(psg_ctx* ctx, int chl);
/* The server's UPDATE_MODEL step (darling.cc:251-262): received(time) must
 * hold m = 2 aggregates (G, U) of channel chl; updateWeight
 * (darling.cc:437-477) runs on the device over value(chl), delta and the
 * active set at the aggregate's positions, and the aggregate is erased.
 * Nothing crosses PCIe but *violation = max vio of this block (the caller
 * folds it into violation_ with std::max).  PSG_ERR_UNMATCHED leaves the
 * model untouched. */
int psg_darling_update(psg_ctx* ctx, int chl, int time, const psg_darling_param* p,
                       double* violation);
/* Copies of delta[off, off+n) and the active bits (one byte each, 0/1);
 * *nnz_active = active_set.nnz() (darling.cc:549).  Any output may be NULL. */
int psg_darling_state(psg_ctx* ctx, int chl, size_t off, size_t n, double* delta,
                      uint8_t* active, size_t* nnz_active);

/* ------------------------------------------------------------------ */
/* Tail-feature filter: FreqencyFilter<uint64> of channel chl          */
/* (SharedParameter::key_filter_, shared_parameter.h:82,114-133) over  */
/* CountMin<uint64, uint8> (src/base/countmin.h), resident in HBM.     */
/* ------------------------------------------------------------------ */
/* CountMin::resize (countmin.h:14-19): n_ = max(n, 64) byte counters,
 * k_ = min(30, max(1, k)) probes, all zero. */
int psg_freq_resize(psg_ctx* ctx, int chl, int n, int k);
int psg_freq_clear(psg_ctx* ctx, int chl);                 /* clear() */
int psg_freq_empty(psg_ctx* ctx, int chl, int* empty);     /* empty() */
/* insertKeys (frequency_filter.h:36-43): counts[i] is added as uint8 to
 * every probe of keys[i] (byte arithmetic wraps).  Host arrays; async. */
int psg_freq_insert(psg_ctx* ctx, int chl, const uint64_t* keys,
                    const uint32_t* counts, size_t n);
/* queryKeys (frequency_filter.h:27-34): out[0, *nout) = the keys whose
 * count estimate is > freq, in input order (out holds n).  freq < 255. */
int psg_freq_query(psg_ctx* ctx, int chl, const uint64_t* keys, size_t n,
                   int freq, uint64_t* out, size_t* nout);
/* Device-resident forms on `stream`: *nout is a device word; scratch holds
 * psg_freq_query_scratch_bytes(n) device bytes (the binned query's records:
 * about 50 B per key up to 8 M keys, then constant -- longer queries take
 * several chunks).  A filter's operations run in call order whatever streams
 * they are enqueued on (each waits for the previous one's event). */
int psg_freq_insert_dev(psg_ctx* ctx, int chl, const uint64_t* keys,
                        const uint32_t* counts, size_t n, void* stream);
size_t psg_freq_query_scratch_bytes(size_t n);
int psg_freq_query_dev(psg_ctx* ctx, int chl, const uint64_t* keys, size_t n,
                       int freq, uint64_t* out, unsigned long long* nout,
                       void* scratch, void* stream);
/* The n_ counters as CountMin's uint8 data_ (tests, checkpoints). */
int psg_freq_table(psg_ctx* ctx, int chl, uint8_t* out, size_t n);

/* ------------------------------------------------------------------ */
/* Wire ingress: key signatures of the key cache                       */
/* ------------------------------------------------------------------ */
/* CRC-32C of device-resident byte segments: out[i] = crc32c::Extend(
 * init ? init[i] : 0, data + off[i], min(off[i+1] - off[i], max_len))
 * (src/util/crc32c.cc:283-330; crc32c::Value = init 0).  The key signature
 * of RNode::cacheKeySender/cacheKeyRecver (src/system/remote_node.cc:108,
 * 163) is max_len = PSG_MAX_SIG_LEN over the key bytes.  off[nseg+1], init
 * (nullable) and out[nseg] are device arrays; enqueued on `stream`. */
#define PSG_MAX_SIG_LEN 2048 /* RNode::max_sig_len_, remote_node.h:96 */

/* snappy raw-format decompression of device-resident message parts: what
 * Van::recv does per key/value part (van.cc:204-214,
 * SArray::uncompressFrom, shared_array_inl.h:232-240), for nmsg parts in
 * one launch.  Part i is src[soff[i], soff[i+1]) and decompresses into
 * dst[doff[i], doff[i+1]), which must be its declared length
 * (snappy::GetUncompressedLength; psg_snappy_uncompressed_length reads it
 * from a host copy of the first bytes).  status[i] = 0, PSG_ERR_SIZE (the
 * declared length differs) or PSG_ERR_ARG (corrupt stream: the reference's
 * CHECK).  soff, doff, status: device arrays; enqueued on `stream`. */
int psg_snappy_uncompress_dev(const uint8_t* src, const uint64_t* soff, uint64_t nmsg,
                              uint8_t* dst, const uint64_t* doff, int32_t* status,
                              void* stream);
int psg_snappy_uncompressed_length(const void* src, size_t n, size_t* len);
int psg_crc32c_dev(const void* data, const uint64_t* off, uint64_t nseg,
                   uint64_t max_len, const uint32_t* init, uint32_t* out,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PSG_H_ */
