/*
 * psg_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference parameter server's server-side push
 * aggregation path (wakensky/parameter_server, src/parameter + src/system +
 * src/base).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path
 * (parameter_server_amd/, include/psg.h) never links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - set ops / findRange: known answers of src/test/shared_array_test.cc:43-69;
 *   - aggregate / gather / evenDivide / murmur key shuffle: the known-answer
 *     constants that SURVEY.md Appendix C records from the reference's own
 *     code; murmur additionally against oracle/_ref (the reference's
 *     src/util/MurmurHash3.cc compiled in place).
 *   The reference's message.h / kv_vector.h cannot be compiled here without
 *   glog/gflags/protobuf/Eigen, so there is no oracle/_ref build of them.
 *
 * Reference quirks are given defined behaviour here:
 *   - a pushed key that is not among the server keys of the position range
 *     is "unmatched" (the caller reports an error); oldMatch's overrun past
 *     range.end() (message.h:251) is not reproduced;
 *   - empty server keys / empty push: no matches, empty range.
 */
#ifndef PSG_ORACLE_H_
#define PSG_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SArray<uint64>::setUnion -- std::set_union (shared_array_inl.h:155-162).
 * out must hold na+nb; returns size of the union. */
size_t orc_set_union_u64(const uint64_t* a, size_t na, const uint64_t* b,
                         size_t nb, uint64_t* out);
/* SArray<uint64>::setIntersection (shared_array_inl.h:145-153). */
size_t orc_set_intersection_u64(const uint64_t* a, size_t na,
                                const uint64_t* b, size_t nb, uint64_t* out);
/* SArray::findRange (shared_array_inl.h:164-171): [lower_bound(kb),
 * lower_bound(ke)). */
void orc_find_range_u64(const uint64_t* a, size_t n, uint64_t kb, uint64_t ke,
                        size_t* lo, size_t* hi);
/* Range<uint64>::evenDivide (range.h:85-98), long double arithmetic. */
void orc_even_divide_u64(uint64_t begin, uint64_t end, size_t n, size_t i,
                         uint64_t* out_begin, uint64_t* out_end);
/* sliceKeyOrderedMsg<uint64> (message.h:89-123): pos[nsep] split positions,
 * valid[nsep-1] piece validity. */
void orc_slice_key_ordered(const uint64_t* keys, size_t n, uint64_t rb,
                           uint64_t re, const uint64_t* sep, size_t nsep,
                           size_t* pos, int* valid);

/* oldMatch (message.h:228-267): out[0..hi-lo) = zeros, matched src values
 * assigned at their server positions.  Returns 0. */
int orc_old_match_f32(const uint64_t* dst_key, size_t ndst,
                      const uint64_t* src_key, size_t nsrc,
                      const float* src_val, uint64_t kb, uint64_t ke,
                      float* out, size_t* lo, size_t* hi, size_t* matched);
int orc_old_match_f64(const uint64_t* dst_key, size_t ndst,
                      const uint64_t* src_key, size_t nsrc,
                      const double* src_val, uint64_t kb, uint64_t ke,
                      double* out, size_t* lo, size_t* hi, size_t* matched);

/* match (message.h:134-226): op 0 = ASSIGN, 1 = ADD; dst positions [lo,hi)
 * split over nthreads threads created for this call (as the reference's
 * per-call ThreadPool). */
void orc_match_f32(size_t lo, size_t hi, const uint64_t* dst_key,
                   float* dst_val, const uint64_t* src_key, size_t nsrc,
                   const float* src_val, int op, int nthreads,
                   size_t* matched);
void orc_match_f64(size_t lo, size_t hi, const uint64_t* dst_key,
                   double* dst_val, const uint64_t* src_key, size_t nsrc,
                   const double* src_val, int op, int nthreads,
                   size_t* matched);

/* KVVector::serialSetValue (parallel = 0, kv_vector.h:171-204) or
 * parallelSetValue (parallel = 1, kv_vector.h:84-137) applied to npush
 * value-carrying pushes of one time t, in arrival order.
 *   vals[p*m + i] = push p's i-th value array (n[p] entries);
 *   out[i]        = aggregate i, (hi-lo) entries.
 * Returns 0, or -1 if D is empty while pushes are non-empty (the
 * reference CHECK-fails there).  matched[p] = matched count of push p. */
int orc_aggregate_f32(const uint64_t* D, size_t nD, uint64_t kb, uint64_t ke,
                      int npush, const uint64_t* const* keys, const size_t* n,
                      int m, const float* const* vals, int parallel,
                      int nthreads, float* const* out, size_t* lo, size_t* hi,
                      size_t* matched);
int orc_aggregate_f64(const uint64_t* D, size_t nD, uint64_t kb, uint64_t ke,
                      int npush, const uint64_t* const* keys, const size_t* n,
                      int m, const double* const* vals, int parallel,
                      int nthreads, double* const* out, size_t* lo,
                      size_t* hi, size_t* matched);
/* parallelSetValue in O(sum n log |D|) (large checks; see psg_oracle.c) */
int orc_aggregate_scatter_f32(const uint64_t* D, size_t nD, uint64_t kb, uint64_t ke, int npush,
                              const uint64_t* const* keys, const size_t* n, int m,
                              const float* const* vals, float* const* out, size_t* lo, size_t* hi,
                              size_t* matched);
int orc_aggregate_scatter_f64(const uint64_t* D, size_t nD, uint64_t kb, uint64_t ke, int npush,
                              const uint64_t* const* keys, const size_t* n, int m,
                              const double* const* vals, double* const* out, size_t* lo,
                              size_t* hi, size_t* matched);
/* serialSetValue in the same form, strictly increasing pushes only */
int orc_aggregate_scatter_serial_f32(const uint64_t* D, size_t nD, uint64_t kb, uint64_t ke,
                                     int npush, const uint64_t* const* keys, const size_t* n,
                                     int m, const float* const* vals, float* const* out,
                                     size_t* lo, size_t* hi, size_t* matched);
int orc_aggregate_scatter_serial_f64(const uint64_t* D, size_t nD, uint64_t kb, uint64_t ke,
                                     int npush, const uint64_t* const* keys, const size_t* n,
                                     int m, const double* const* vals, double* const* out,
                                     size_t* lo, size_t* hi, size_t* matched);

/* KVVector::serialGetValue (kv_vector.h:215-227): out[i] = W[pos(req[i])]
 * or 0 when req[i] is not a server key. */
void orc_gather_f32(const uint64_t* D, size_t nD, const float* W,
                    const uint64_t* req, size_t nreq, float* out,
                    size_t* matched);
void orc_gather_f64(const uint64_t* D, size_t nD, const double* W,
                    const uint64_t* req, size_t nreq, double* out,
                    size_t* matched);

/* MurmurHash3_x64_128 (util/MurmurHash3.cc:255), restated; the CTR key
 * shuffle folds o[0]^o[1] (data/example_parser.cc:205-208). */
void orc_murmur3_x64_128(const void* key, int len, uint32_t seed,
                         uint64_t out[2]);
void orc_shuffle_keys(const uint64_t* ids, size_t n, uint32_t seed,
                      uint64_t* out);

/* crc32c::Extend / Mask / Unmask (util/crc32c.cc:283-330, crc32c.h:29-38);
 * Value(data, n) = Extend(0, data, n).  The key-cache signature is
 * Value(keys, min(bytes, 2048)) (system/remote_node.cc:108,163). */
uint32_t orc_crc32c_extend(uint32_t init, const void* data, size_t n);
uint32_t orc_crc32c_mask(uint32_t crc);
uint32_t orc_crc32c_unmask(uint32_t masked);

/* Darling::updateWeight (linear_method/darling.cc:437-477), parity
 * unpinned (no reference test; darling.cc not buildable here).  active is
 * one byte per position (0/1); *violation is folded with std::max. */
void orc_darling_update_weight(double* value, double* delta, uint8_t* active,
                               size_t lo, size_t n, const double* G,
                               const double* U, double eta, double lambda,
                               double kkt, double delta_max,
                               double* violation);

/* CountMin<uint64,uint8> insert/query and FreqencyFilter::queryKeys
 * (countmin.h:33-51, frequency_filter.h:27-34), parity unpinned. */
void orc_cm_insert(uint8_t* data, uint32_t n, int k, const uint64_t* keys,
                   const uint32_t* counts, size_t nk);
uint8_t orc_cm_query(const uint8_t* data, uint32_t n, int k, uint64_t key);
size_t orc_ff_query(const uint8_t* data, uint32_t n, int k, const uint64_t* keys,
                    size_t nk, int freq, uint64_t* out);

/* snappy raw format (google/snappy, absent from the reference tree; the
 * published format restated), parity unpinned.  uncompressed_length
 * returns the preamble size or -1; uncompress returns 0 or -1; compress is
 * a test-input generator (dst holds 32 + n + n / 6 bytes). */
int orc_snappy_uncompressed_length(const uint8_t* src, size_t n, size_t* out);
int orc_snappy_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap);
size_t orc_snappy_compress(const uint8_t* src, size_t n, uint8_t* dst);

#ifdef __cplusplus
}
#endif
#endif /* PSG_ORACLE_H_ */
