/*
 * psg_oracle.c -- TEST INFRASTRUCTURE ONLY (see psg_oracle.h).
 *
 * Plain-C restatement of the reference's CPU push-aggregation path.  Every
 * function cites the reference file:line it restates.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 */
#include "psg_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* std::lower_bound / upper_bound over uint64 */
static size_t lb_u64(const uint64_t* a, size_t n, uint64_t k) {
  size_t lo = 0, len = n;
  while (len > 0) {
    size_t half = len >> 1;
    if (a[lo + half] < k) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo;
}
static size_t ub_u64(const uint64_t* a, size_t n, uint64_t k) {
  size_t lo = 0, len = n;
  while (len > 0) {
    size_t half = len >> 1;
    if (!(k < a[lo + half])) {
      lo += half + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  return lo;
}

/* shared_array_inl.h:155-162 -> std::set_union (multiset semantics: an
 * element present c_a times in a and c_b times in b appears max(c_a,c_b)
 * times). */
size_t orc_set_union_u64(const uint64_t* a, size_t na, const uint64_t* b,
                         size_t nb, uint64_t* out) {
  size_t i = 0, j = 0, k = 0;
  while (i < na) {
    if (j == nb) {
      while (i < na) out[k++] = a[i++];
      return k;
    }
    if (b[j] < a[i]) {
      out[k++] = b[j++];
    } else {
      out[k++] = a[i];
      if (!(a[i] < b[j])) ++j;
      ++i;
    }
  }
  while (j < nb) out[k++] = b[j++];
  return k;
}

/* shared_array_inl.h:145-153 -> std::set_intersection */
size_t orc_set_intersection_u64(const uint64_t* a, size_t na,
                                const uint64_t* b, size_t nb, uint64_t* out) {
  size_t i = 0, j = 0, k = 0;
  while (i < na && j < nb) {
    if (a[i] < b[j]) {
      ++i;
    } else {
      if (!(b[j] < a[i])) out[k++] = a[i++];
      ++j;
    }
  }
  return k;
}

/* shared_array_inl.h:164-171 */
void orc_find_range_u64(const uint64_t* a, size_t n, uint64_t kb, uint64_t ke,
                        size_t* lo, size_t* hi) {
  if (n == 0) {
    *lo = *hi = 0;
    return;
  }
  *lo = lb_u64(a, n, kb);
  *hi = lb_u64(a, n, ke);
}

/* range.h:85-98: itv = (long double)(end-begin)/n; [begin+itv*i,
 * begin+itv*(i+1)) with the last piece ending at end. */
void orc_even_divide_u64(uint64_t begin, uint64_t end, size_t n, size_t i,
                         uint64_t* out_begin, uint64_t* out_end) {
  long double itv = (long double)(end - begin) / (long double)n;
  uint64_t new_end = (uint64_t)(begin + itv * (long double)(i + 1));
  if (i + 1 == n) new_end = end;
  *out_begin = (uint64_t)(begin + itv * (long double)i);
  *out_end = new_end;
}

/* message.h:89-123 (positions + validity only; the pieces are zero-copy
 * segments [pos[i], pos[i+1]) of keys and, proportionally, of values). */
void orc_slice_key_ordered(const uint64_t* keys, size_t n, uint64_t rb,
                           uint64_t re, const uint64_t* sep, size_t nsep,
                           size_t* pos, int* valid) {
  for (size_t s = 0; s < nsep; ++s) {
    uint64_t p = sep[s];
    uint64_t k = p < re ? p : re;       /* std::min(range.end, p) */
    if (k < rb) k = rb;                 /* std::max(range.begin, .) */
    pos[s] = lb_u64(keys, n, k);
  }
  for (size_t s = 0; s + 1 < nsep; ++s) {
    uint64_t ib = sep[s] > rb ? sep[s] : rb;
    uint64_t ie = sep[s + 1] < re ? sep[s + 1] : re;
    valid[s] = !(ib >= ie);             /* Range::setIntersection().empty() */
  }
}

/* ---------------------------------------------------------------------- */
/* oldMatch (message.h:228-267) and match (message.h:134-226), per V.      */
/* ---------------------------------------------------------------------- */

#define DEFINE_OLD_MATCH(SUF, V)                                               \
  int orc_old_match_##SUF(const uint64_t* dst_key, size_t ndst,               \
                          const uint64_t* src_key, size_t nsrc,               \
                          const V* src_val, uint64_t kb, uint64_t ke, V* out, \
                          size_t* lo, size_t* hi, size_t* matched) {          \
    *matched = 0;                                                              \
    *lo = *hi = 0;                                                             \
    if (ndst == 0 || nsrc == 0) return 0; /* message.h:236-238 */              \
    orc_find_range_u64(dst_key, ndst, kb, ke, lo, hi); /* :240 */              \
    size_t len = *hi - *lo;                                                    \
    memset(out, 0, sizeof(V) * len); /* :242-244 */                            \
    if (len == 0) return 0;                                                    \
    /* :247-249 binary search the start point */                               \
    const uint64_t* d = dst_key + *lo;                                         \
    const uint64_t* dend = dst_key + *hi; /* defined: stop at range end */     \
    size_t s = lb_u64(src_key, nsrc, *d);                                      \
    V* o = out;                                                                \
    while (d != dend && s != nsrc) { /* :251-265 merge walk */                 \
      if (src_key[s] < *d) {                                                   \
        ++s;                                                                   \
      } else {                                                                 \
        if (!(*d < src_key[s])) {                                              \
          *o = src_val[s];                                                     \
          ++s;                                                                 \
          ++*matched;                                                          \
        }                                                                      \
        ++d;                                                                   \
        ++o;                                                                   \
      }                                                                        \
    }                                                                          \
    return 0;                                                                  \
  }

DEFINE_OLD_MATCH(f32, float)
DEFINE_OLD_MATCH(f64, double)

#define DEFINE_MATCH(SUF, V)                                                   \
  typedef struct {                                                             \
    size_t b, e, lo;                                                           \
    const uint64_t* dst_key;                                                   \
    V* dst_val;                                                                \
    const uint64_t* src_key;                                                   \
    size_t nsrc;                                                               \
    const V* src_val;                                                          \
    int op;                                                                    \
    size_t matched;                                                            \
  } match_arg_##SUF;                                                           \
  static void* match_worker_##SUF(void* p) {                                   \
    match_arg_##SUF* a = (match_arg_##SUF*)p;                                  \
    a->matched = 0;                                                            \
    if (a->e <= a->b) return NULL; /* Appendix B #5: empty slice */            \
    const uint64_t* d = a->dst_key + a->b;                                     \
    const uint64_t* dend = a->dst_key + a->e;                                  \
    V* o = a->dst_val + (a->b - a->lo);                                        \
    /* message.h:177-179 */                                                    \
    size_t s = lb_u64(a->src_key, a->nsrc, *d);                                \
    size_t send = ub_u64(a->src_key, a->nsrc, *(dend - 1));                    \
    if (a->op == 0) memset(o, 0, sizeof(V) * (size_t)(dend - d)); /* :182 */   \
    while (d != dend && s != send) { /* :187-214 */                            \
      if (a->src_key[s] < *d) {                                                \
        ++s;                                                                   \
      } else {                                                                 \
        if (!(*d < a->src_key[s])) {                                           \
          if (a->op == 0)                                                      \
            *o = a->src_val[s];                                                \
          else                                                                 \
            *o += a->src_val[s];                                               \
          ++s;                                                                 \
          ++a->matched;                                                        \
        }                                                                      \
        ++d;                                                                   \
        ++o;                                                                   \
      }                                                                        \
    }                                                                          \
    return NULL;                                                               \
  }                                                                            \
  void orc_match_##SUF(size_t lo, size_t hi, const uint64_t* dst_key,         \
                       V* dst_val, const uint64_t* src_key, size_t nsrc,      \
                       const V* src_val, int op, int nthreads,                \
                       size_t* matched) {                                      \
    *matched = 0;                                                              \
    if (hi <= lo || nsrc == 0) return; /* message.h:145-147 */                 \
    if (nthreads < 1) nthreads = 1;                                            \
    match_arg_##SUF* args =                                                    \
        (match_arg_##SUF*)calloc((size_t)nthreads, sizeof(match_arg_##SUF));   \
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));   \
    for (int t = 0; t < nthreads; ++t) {                                       \
      /* message.h:160-166: SizeR::evenDivide, last thread takes the rest */   \
      uint64_t b, e;                                                           \
      orc_even_divide_u64(lo, hi, (size_t)nthreads, (size_t)t, &b, &e);       \
      if (t == nthreads - 1) e = hi;                                           \
      match_arg_##SUF a = {b, e, lo, dst_key, dst_val, src_key,               \
                           nsrc, src_val, op, 0};                              \
      args[t] = a;                                                             \
    }                                                                          \
    if (nthreads == 1) {                                                       \
      match_worker_##SUF(&args[0]);                                            \
    } else {                                                                   \
      /* a pool is created and joined on every call (message.h:152-218) */    \
      for (int t = 0; t < nthreads; ++t)                                       \
        pthread_create(&th[t], NULL, match_worker_##SUF, &args[t]);            \
      for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);            \
    }                                                                          \
    for (int t = 0; t < nthreads; ++t) *matched += args[t].matched;           \
    free(args);                                                                \
    free(th);                                                                  \
  }

DEFINE_MATCH(f32, float)
DEFINE_MATCH(f64, double)

/* ---------------------------------------------------------------------- */
/* KVVector::serialSetValue / parallelSetValue over one time t.            */
/* ---------------------------------------------------------------------- */

#define DEFINE_AGGREGATE(SUF, V)                                               \
  int orc_aggregate_##SUF(const uint64_t* D, size_t nD, uint64_t kb,          \
                          uint64_t ke, int npush,                              \
                          const uint64_t* const* keys, const size_t* n, int m, \
                          const V* const* vals, int parallel, int nthreads,   \
                          V* const* out, size_t* lo, size_t* hi,               \
                          size_t* matched) {                                   \
    *lo = *hi = 0;                                                             \
    int have = 0; /* recved_val_[t] exists */                                  \
    for (int p = 0; p < npush; ++p) {                                          \
      matched[p] = 0;                                                          \
      if (n[p] == 0) continue; /* kv_vector.h:90,177: empty push ignored */    \
      if (nD == 0) return -1;  /* CHECK_GE / range CHECK fails */              \
      size_t plo, phi;                                                         \
      orc_find_range_u64(D, nD, kb, ke, &plo, &phi);                           \
      if (have && (plo != *lo || phi != *hi)) return -2; /* CHECK_EQ range */  \
      size_t len = phi - plo;                                                  \
      for (int i = 0; i < m; ++i) {                                            \
        const V* v = vals[(size_t)p * m + i];                                  \
        size_t mt = 0;                                                         \
        if (!parallel) {                                                       \
          /* kv_vector.h:190: aligned = oldMatch(...) (new + memset) */       \
          size_t alo, ahi;                                                     \
          if (!have) { /* :195-196 the first aligned array is stored */        \
            orc_old_match_##SUF(D, nD, keys[p], n[p], v, kb, ke, out[i], &alo, \
                                &ahi, &mt);                                    \
          } else {                                                             \
            V* aligned = (V*)malloc(sizeof(V) * (len ? len : 1));              \
            orc_old_match_##SUF(D, nD, keys[p], n[p], v, kb, ke, aligned,     \
                                &alo, &ahi, &mt);                              \
            V* acc = out[i]; /* :200 eigenArray() += */                        \
            for (size_t j = 0; j < len; ++j) acc[j] += aligned[j];             \
            free(aligned);                                                     \
          }                                                                    \
        } else {                                                               \
          /* kv_vector.h:114-131: first push ASSIGN, later ADD */              \
          orc_match_##SUF(plo, phi, D, out[i], keys[p], n[p], v,              \
                          have ? 1 : 0, nthreads, &mt);                        \
        }                                                                      \
        matched[p] = mt;                                                       \
      }                                                                        \
      if (!have) {                                                             \
        *lo = plo;                                                             \
        *hi = phi;                                                             \
        have = 1;                                                              \
      }                                                                        \
    }                                                                          \
    return 0;                                                                  \
  }

DEFINE_AGGREGATE(f32, float)
DEFINE_AGGREGATE(f64, double)

/* parallelSetValue (kv_vector.h:84-137) restated in O(sum n log |D|) for
 * large checks: match() (message.h:134-226) sets (ASSIGN, first push, after
 * zero-filling the range, :182) or adds (ADD) src_val at the dst position of
 * every src key that equals a dst key and touches no other position, so one
 * push's effect is a scatter of its matched values; the merge walk skips an
 * unmatched src key (matched < n) -- here a key that lower_bound does not
 * find, or a repeated key, which the walk never revisits.  For
 * non-decreasing pushes (unsorted ones take orc_aggregate); cross-checked
 * against orc_aggregate (parallel) in tests/test_oracle.py. */
#define DEFINE_AGGREGATE_SCATTER(SUF, V)                                       \
  int orc_aggregate_scatter_##SUF(const uint64_t* D, size_t nD, uint64_t kb,  \
                                  uint64_t ke, int npush,                      \
                                  const uint64_t* const* keys, const size_t* n,\
                                  int m, const V* const* vals, V* const* out,  \
                                  size_t* lo, size_t* hi, size_t* matched) {   \
    *lo = *hi = 0;                                                             \
    int have = 0;                                                              \
    for (int p = 0; p < npush; ++p) {                                          \
      matched[p] = 0;                                                          \
      if (n[p] == 0) continue;                                                 \
      if (nD == 0) return -1;                                                  \
      size_t plo, phi;                                                         \
      orc_find_range_u64(D, nD, kb, ke, &plo, &phi);                           \
      if (have && (plo != *lo || phi != *hi)) return -2;                       \
      if (!have)                                                               \
        for (int i = 0; i < m; ++i) memset(out[i], 0, sizeof(V) * (phi - plo));\
      size_t mt = 0, prev = (size_t)-1;                                        \
      for (size_t k = 0; k < n[p]; ++k) {                                      \
        const size_t pos = plo + lb_u64(D + plo, phi - plo, keys[p][k]);       \
        if (pos >= phi || D[pos] != keys[p][k]) continue;                      \
        if (prev != (size_t)-1 && pos <= prev) continue; /* walk never backs */\
        prev = pos;                                                            \
        ++mt;                                                                  \
        for (int i = 0; i < m; ++i) {                                          \
          V* o = out[i] + (pos - plo);                                         \
          const V v = vals[(size_t)p * m + i][k];                              \
          *o = have ? *o + v : v;                                              \
        }                                                                      \
      }                                                                        \
      matched[p] = mt;                                                         \
      if (!have) {                                                             \
        *lo = plo;                                                             \
        *hi = phi;                                                             \
        have = 1;                                                              \
      }                                                                        \
    }                                                                          \
    return 0;                                                                  \
  }

DEFINE_AGGREGATE_SCATTER(f32, float)
DEFINE_AGGREGATE_SCATTER(f64, double)

/* serialSetValue (kv_vector.h:171-204) in the same O(sum n log |D|) form, for
 * strictly increasing pushes (returns -3 on any other): oldMatch
 * (message.h:229-267) zero-fills an aligned array and writes each matched
 * value, the first non-empty push's array is stored (:195-196) and every
 * later one is added element-wise (:200).  A later push lacking the key
 * therefore adds +0.0; x + 0.0 is x except on -0.0 (-> +0.0) and a
 * signalling NaN (quieted), and after either happened further adds keep
 * it, so the dense fold equals the fold of the present values followed by
 * ONE +0.0 iff some non-empty push lacked the key (a push before the first
 * contribution leaves +0.0 + v, which that +0.0 does not change).
 * Cross-checked against orc_aggregate (serial) in tests/test_oracle.py. */
#define DEFINE_AGGREGATE_SCATTER_SERIAL(SUF, V)                                \
  int orc_aggregate_scatter_serial_##SUF(                                      \
      const uint64_t* D, size_t nD, uint64_t kb, uint64_t ke, int npush,       \
      const uint64_t* const* keys, const size_t* n, int m, const V* const* vals,\
      V* const* out, size_t* lo, size_t* hi, size_t* matched) {                \
    *lo = *hi = 0;                                                             \
    int have = 0;                                                              \
    uint32_t nne = 0;   /* non-empty pushes */                                 \
    uint32_t* cnt = 0;  /* pushes holding each slot */                         \
    for (int p = 0; p < npush; ++p) {                                          \
      matched[p] = 0;                                                          \
      if (n[p] == 0) continue; /* kv_vector.h:177: empty push ignored */       \
      if (nD == 0) { free(cnt); return -1; }                                   \
      size_t plo, phi;                                                         \
      orc_find_range_u64(D, nD, kb, ke, &plo, &phi);                           \
      if (have && (plo != *lo || phi != *hi)) { free(cnt); return -2; }        \
      if (!have) {                                                             \
        for (int i = 0; i < m; ++i) memset(out[i], 0, sizeof(V) * (phi - plo));\
        cnt = (uint32_t*)calloc(phi - plo ? phi - plo : 1, sizeof(uint32_t));  \
      }                                                                        \
      size_t mt = 0;                                                           \
      for (size_t k = 0; k < n[p]; ++k) {                                      \
        if (k > 0 && keys[p][k] <= keys[p][k - 1]) { free(cnt); return -3; }  \
        const size_t pos = plo + lb_u64(D + plo, phi - plo, keys[p][k]);       \
        if (pos >= phi || D[pos] != keys[p][k]) continue;                      \
        ++mt;                                                                  \
        ++cnt[pos - plo];                                                      \
        for (int i = 0; i < m; ++i) {                                          \
          V* o = out[i] + (pos - plo);                                         \
          const V v = vals[(size_t)p * m + i][k];                              \
          *o = have ? *o + v : v;                                              \
        }                                                                      \
      }                                                                        \
      matched[p] = mt;                                                         \
      if (!have) {                                                             \
        *lo = plo;                                                             \
        *hi = phi;                                                             \
        have = 1;                                                              \
      }                                                                        \
      ++nne;                                                                   \
    }                                                                          \
    if (have)                                                                  \
      for (size_t j = 0; j < *hi - *lo; ++j)                                   \
        if (cnt[j] < nne)                                                      \
          for (int i = 0; i < m; ++i) out[i][j] = out[i][j] + (V)0;            \
    free(cnt);                                                                 \
    return 0;                                                                  \
  }

DEFINE_AGGREGATE_SCATTER_SERIAL(f32, float)
DEFINE_AGGREGATE_SCATTER_SERIAL(f64, double)

/* kv_vector.h:215-227: oldMatch(recv_key, key_[ch], val_[ch], union range)
 * -- a gather aligned to the request keys, zero where absent. */
#define DEFINE_GATHER(SUF, V)                                                  \
  void orc_gather_##SUF(const uint64_t* D, size_t nD, const V* W,             \
                        const uint64_t* req, size_t nreq, V* out,             \
                        size_t* matched) {                                     \
    *matched = 0;                                                              \
    memset(out, 0, sizeof(V) * nreq);                                          \
    if (nD == 0 || nreq == 0) return;                                          \
    size_t i = 0, j = lb_u64(D, nD, req[0]);                                   \
    while (i < nreq && j < nD) {                                               \
      if (D[j] < req[i]) {                                                     \
        ++j;                                                                   \
      } else {                                                                 \
        if (!(req[i] < D[j])) {                                                \
          out[i] = W[j];                                                       \
          ++j;                                                                 \
          ++*matched;                                                          \
        }                                                                      \
        ++i;                                                                   \
      }                                                                        \
    }                                                                          \
  }

DEFINE_GATHER(f32, float)
DEFINE_GATHER(f64, double)

/* ---------------------------------------------------------------------- */
/* MurmurHash3_x64_128 (util/MurmurHash3.cc:255-331), restated.            */
/* ---------------------------------------------------------------------- */
static inline uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
static inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

void orc_murmur3_x64_128(const void* key, int len, uint32_t seed,
                         uint64_t out[2]) {
  const uint8_t* data = (const uint8_t*)key;
  const int nblocks = len / 16;
  uint64_t h1 = seed, h2 = seed;
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  for (int i = 0; i < nblocks; i++) {
    uint64_t k1, k2;
    memcpy(&k1, data + 16 * i, 8);
    memcpy(&k2, data + 16 * i + 8, 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = data + nblocks * 16;
  uint64_t k1 = 0, k2 = 0;
  int rem = len & 15;
  for (int t = rem - 1; t >= 8; --t) k2 ^= ((uint64_t)tail[t]) << (8 * (t - 8));
  if (rem > 8) {
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
  }
  for (int t = (rem < 8 ? rem : 8) - 1; t >= 0; --t)
    k1 ^= ((uint64_t)tail[t]) << (8 * t);
  if (rem > 0) {
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)len;
  h2 ^= (uint64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
  out[0] = h1;
  out[1] = h2;
}

/* data/example_parser.cc:205-208 */
void orc_shuffle_keys(const uint64_t* ids, size_t n, uint32_t seed,
                      uint64_t* out) {
  for (size_t i = 0; i < n; ++i) {
    uint64_t o[2];
    orc_murmur3_x64_128(&ids[i], 8, seed, o);
    out[i] = o[0] ^ o[1];
  }
}

/* ---------------------------------------------------------------------- */
/* crc32c::Extend (util/crc32c.cc:283-330), restated bit by bit: reflected */
/* Castagnoli polynomial 0x82f63b78, register inverted on entry and exit.  */
/* The reference's slicing-by-4 table walk computes the same function.     */
/* ---------------------------------------------------------------------- */
uint32_t orc_crc32c_extend(uint32_t init, const void* data, size_t n) {
  const uint8_t* p = (const uint8_t*)data;
  uint32_t l = init ^ 0xffffffffu;
  for (size_t i = 0; i < n; ++i) {
    l ^= p[i];
    for (int b = 0; b < 8; ++b) l = (l & 1u) ? (l >> 1) ^ 0x82f63b78u : l >> 1;
  }
  return l ^ 0xffffffffu;
}

/* crc32c::Mask / Unmask (util/crc32c.h:29-38) */
uint32_t orc_crc32c_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}
uint32_t orc_crc32c_unmask(uint32_t masked) {
  const uint32_t rot = masked - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

/* ---------------------------------------------------------------------- */
/* Darling::updateWeight (linear_method/darling.cc:437-477) with newDelta  */
/* (darling.h:31-33) and kInactiveValue_ = all-ones bits (darling.cc:13-15)*/
/* over positions [lo, lo+n) of the server weights.  *violation is folded  */
/* with std::max as violation_ is (darling.cc:466).  PARITY UNPINNED: the  */
/* reference ships no test of this function and darling.cc cannot be      */
/* built here (protobuf/glog/Eigen); this is a line-by-line restatement.   */
/* ---------------------------------------------------------------------- */
static double std_min_d(double a, double b) { return b < a ? b : a; }
static double std_max_d(double a, double b) { return a < b ? b : a; }

void orc_darling_update_weight(double* value, double* delta, uint8_t* active,
                               size_t lo, size_t n, const double* G,
                               const double* U, double eta, double lambda,
                               double kkt, double delta_max,
                               double* violation) {
  double inactive_value;
  const uint64_t ones = ~(uint64_t)0;
  memcpy(&inactive_value, &ones, sizeof(double));
  for (size_t i = 0; i < n; ++i) {
    const size_t k = i + lo;
    if (!active[k]) continue;
    double g = G[i], u = U[i] / eta + 1e-10;
    double g_pos = g + lambda, g_neg = g - lambda;
    double* w = &value[k];
    double d = -*w, vio = 0;
    if (*w == 0) {
      if (g_pos < 0) {
        vio = -g_pos;
      } else if (g_neg > 0) {
        vio = g_neg;
      } else if (g_pos > kkt && g_neg < -kkt) {
        active[k] = 0;
        *w = inactive_value;
        continue;
      }
    }
    *violation = std_max_d(*violation, vio);
    if (g_pos <= u * *w) {
      d = -g_pos / u;
    } else if (g_neg >= u * *w) {
      d = -g_neg / u;
    }
    d = std_min_d(delta[k], std_max_d(-delta[k], d));
    delta[k] = std_min_d(delta_max, 2 * fabs(d) + .1);
    *w += d;
  }
}

/* ---------------------------------------------------------------------- */
/* CountMin<uint64, uint8> (base/countmin.h:14-67) and FreqencyFilter      */
/* insertKeys / queryKeys (parameter/frequency_filter.h:27-43), restated   */
/* on a caller-held table of n uint8 counters (n = max(n, 64) and          */
/* k = min(30, max(1, k)) already applied by the caller, as resize() does).*/
/* PARITY UNPINNED: src/test/countmin_test.cc is entirely commented out    */
/* and countmin.h cannot be compiled here (glog via shared_array_inl.h).   */
/* ---------------------------------------------------------------------- */
static uint32_t cm_hash(uint64_t key) {
  const uint32_t seed = 0xbc9f1d34u, m = 0xc6a4a793u, n = 8;
  uint32_t h = seed ^ (n * m);
  uint32_t w = (uint32_t)key;
  h += w; h *= m; h ^= (h >> 16);
  w = (uint32_t)(key >> 32);
  h += w; h *= m; h ^= (h >> 16);
  return h;
}

void orc_cm_insert(uint8_t* data, uint32_t n, int k, const uint64_t* keys,
                   const uint32_t* counts, size_t nk) {
  for (size_t i = 0; i < nk; ++i) {
    const uint8_t c = (uint8_t)counts[i]; /* insert(key, V count): uint32 -> uint8 */
    uint32_t h = cm_hash(keys[i]);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (int j = 0; j < k; ++j) {
      data[h % n] = (uint8_t)(data[h % n] + c);
      h += delta;
    }
  }
}

uint8_t orc_cm_query(const uint8_t* data, uint32_t n, int k, uint64_t key) {
  uint8_t res = (uint8_t)0xff;
  uint32_t h = cm_hash(key);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int j = 0; j < k; ++j) {
    if (data[h % n] < res) res = data[h % n];
    h += delta;
  }
  return res;
}

size_t orc_ff_query(const uint8_t* data, uint32_t n, int k, const uint64_t* keys,
                    size_t nk, int freq, uint64_t* out) {
  size_t m = 0;
  for (size_t i = 0; i < nk; ++i)
    if ((int)orc_cm_query(data, n, k, keys[i]) > freq) out[m++] = keys[i];
  return m;
}

/* ---------------------------------------------------------------------- */
/* snappy raw format (third-party dependency of the reference, absent from */
/* /root/reference: google/snappy, used by SArray::uncompressFrom /        */
/* compressTo, base/shared_array_inl.h:232-254, on Van payloads,           */
/* system/van.cc:204-214).  Restated from snappy's published format        */
/* description (format_description.txt): a little-endian varint of the     */
/* uncompressed length, then elements -- tag & 3: 0 literal (length-1 in   */
/* tag >> 2, or in 1..4 following bytes when that is 60..63), 1 copy of    */
/* 4 + ((tag >> 2) & 7) bytes at offset (tag >> 5) << 8 | next byte, 2 / 3  */
/* copy of 1 + (tag >> 2) bytes at a 2 / 4-byte little-endian offset.      */
/* PARITY UNPINNED: no snappy test vectors ship in /root/reference; the    */
/* tests use spec-derived hand-made streams and this file's compressor.    */
/* ---------------------------------------------------------------------- */
int orc_snappy_uncompressed_length(const uint8_t* src, size_t n, size_t* out) {
  uint64_t v = 0;
  for (size_t i = 0; i < n && i < 5; ++i) {
    v |= (uint64_t)(src[i] & 0x7f) << (7 * i);
    if (!(src[i] & 0x80)) {
      if (v > 0xffffffffull) return -1;
      *out = (size_t)v;
      return (int)(i + 1);  /* preamble bytes */
    }
  }
  return -1;
}

/* RawUncompress: 0, or -1 for a corrupt stream / length mismatch. */
int orc_snappy_uncompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  size_t ulen;
  const int pre = orc_snappy_uncompressed_length(src, n, &ulen);
  if (pre < 0 || ulen != cap) return -1;
  size_t p = (size_t)pre, o = 0;
  while (p < n) {
    const uint32_t tag = src[p++];
    size_t len, off = 0;
    if ((tag & 3) == 0) {
      len = (tag >> 2) + 1;
      if (len > 60) {
        const size_t nb = len - 60;
        if (p + nb > n) return -1;
        len = 0;
        for (size_t b = 0; b < nb; ++b) len |= (size_t)src[p + b] << (8 * b);
        len += 1;
        p += nb;
      }
      if (p + len > n || o + len > cap) return -1;
      memcpy(dst + o, src + p, len);
      p += len;
      o += len;
      continue;
    }
    if ((tag & 3) == 1) {
      if (p + 1 > n) return -1;
      len = 4 + ((tag >> 2) & 7);
      off = ((size_t)(tag >> 5) << 8) | src[p];
      p += 1;
    } else if ((tag & 3) == 2) {
      if (p + 2 > n) return -1;
      len = 1 + (tag >> 2);
      off = (size_t)src[p] | (size_t)src[p + 1] << 8;
      p += 2;
    } else {
      if (p + 4 > n) return -1;
      len = 1 + (tag >> 2);
      off = (size_t)src[p] | (size_t)src[p + 1] << 8 | (size_t)src[p + 2] << 16 |
            (size_t)src[p + 3] << 24;
      p += 4;
    }
    if (off == 0 || off > o || o + len > cap) return -1;
    for (size_t i = 0; i < len; ++i) dst[o + i] = dst[o - off + i]; /* overlap: byte order */
    o += len;
  }
  return o == cap ? 0 : -1;
}

/* A greedy compressor producing a valid raw stream (test input only; not
 * the reference's RawCompress, whose exact bytes differ): 64 KB blocks,
 * 4-byte hash matches, copies of <= 64 bytes with 2-byte offsets, literals
 * with every length encoding.  dst holds 32 + n + n / 6 bytes. */
size_t orc_snappy_compress(const uint8_t* src, size_t n, uint8_t* dst) {
  size_t o = 0;
  size_t v = n;
  do { uint8_t b = v & 0x7f; v >>= 7; dst[o++] = (uint8_t)(b | (v ? 0x80 : 0)); } while (v);
  static int table[1 << 14];
  for (size_t blk = 0; blk < n; blk += 65536) {
    const size_t end = blk + 65536 < n ? blk + 65536 : n;
    for (int i = 0; i < (1 << 14); ++i) table[i] = -1;
    size_t lit = blk, i = blk;
#define EMIT_LIT(from, to)                                                   \
    do {                                                                     \
      size_t L = (to) - (from);                                              \
      if (L) {                                                               \
        if (L <= 60) dst[o++] = (uint8_t)((L - 1) << 2);                     \
        else {                                                               \
          size_t x = L - 1, nb = x < 256 ? 1 : x < 65536 ? 2 : x < (1u << 24) ? 3 : 4; \
          dst[o++] = (uint8_t)((59 + nb) << 2);                              \
          for (size_t b = 0; b < nb; ++b) dst[o++] = (uint8_t)(x >> (8 * b)); \
        }                                                                    \
        memcpy(dst + o, src + (from), L);                                    \
        o += L;                                                              \
      }                                                                      \
    } while (0)
    while (i + 4 <= end) {
      uint32_t w;
      memcpy(&w, src + i, 4);
      const uint32_t h = (w * 0x1e35a7bdu) >> 18;
      const int c = table[h];
      table[h] = (int)(i - blk);
      if (c >= 0 && memcmp(src + blk + c, src + i, 4) == 0) {
        size_t m = 4;
        while (i + m < end && m < 64 && src[blk + c + m] == src[i + m]) ++m;
        EMIT_LIT(lit, i);
        const size_t off = i - (blk + (size_t)c);
        dst[o++] = (uint8_t)(2 | ((m - 1) << 2));
        dst[o++] = (uint8_t)off;
        dst[o++] = (uint8_t)(off >> 8);
        i += m;
        lit = i;
      } else {
        ++i;
      }
    }
    EMIT_LIT(lit, end);
#undef EMIT_LIT
  }
  return o;
}
