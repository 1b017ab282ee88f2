// MEASUREMENT AID (not product code): the PCIe-inclusive host path of one
// aggregate driven through the C ABI from C++, as the reference's C++ server
// would call it (SharedParameter::process -> setValue per push ->
// received(t), src/parameter/shared_parameter.h:91-149), without Python in
// the loop.  bench.py loads this library with ctypes and passes the host
// buffers (pageable or pinned).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/psg.h"

extern "C" int psg_e2e(int device, int dtype, unsigned flags, const uint64_t* D, size_t nd,
                       int npush, const uint64_t* const* keys, const size_t* n,
                       const void* const* vals, const uint32_t* sigs, void* out, int reps,
                       double* ms) {
  psg_ctx* c = nullptr;
  int rc = psg_create(device, dtype, flags, &c);
  if (rc) return rc;
  rc = psg_key_union(c, 0, D, nd);
  const uint64_t all = ~0ull;
  for (int r = 0; rc == 0 && r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; rc == 0 && p < npush; ++p) {
      const void* v[1] = {vals[p]};
      if (sigs) {  // each worker's keys ride the key cache after the first time
        const bool carry = r == 0;
        rc = psg_push_cached(c, p, 0, r, 0, all, PSG_KC_SIG | (carry ? PSG_KC_KEYS : 0u),
                             sigs[p], carry ? keys[p] : nullptr, carry ? n[p] : 0, 1, v, n[p]);
      } else {
        rc = psg_push(c, 0, r, 0, all, keys[p], n[p], 1, v);
      }
    }
    void* o[1] = {out};
    if (rc == 0) rc = psg_received(c, r, 1, o);
    ms[r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                .count();
  }
  if (rc) fprintf(stderr, "psg_e2e: %s\n", psg_last_error());
  psg_destroy(c);
  return rc;
}

// The Darling server step (darling.cc:245-262) for one feature block:
// npush workers push (G, U) for their keys of the block (keys from the key
// cache after the first time), then the fused updateWeight runs on the
// device over the resident aggregate -- no aggregate D2H, no host update,
// no value re-upload.  f64, m = 2.
extern "C" int psg_e2e_darling(int device, unsigned flags, const uint64_t* D, size_t nd,
                               int npush, const uint64_t* const* keys, const size_t* n,
                               const double* const* G, const double* const* U,
                               const uint32_t* sigs, int reps, double* ms, double* vio_out) {
  psg_ctx* c = nullptr;
  int rc = psg_create(device, PSG_F64, flags, &c);
  if (rc) return rc;
  rc = psg_key_union(c, 0, D, nd);
  std::vector<double> w(nd, 0.0);
  if (rc == 0) rc = psg_value_assign(c, 0, w.data(), nd);
  if (rc == 0) rc = psg_darling_init(c, 0, 1.0);
  const psg_darling_param P = {1.0, 0.1, 1e20, 5.0};
  const uint64_t all = ~0ull;
  for (int r = 0; rc == 0 && r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; rc == 0 && p < npush; ++p) {
      const void* v[2] = {G[p], U[p]};
      const bool carry = r == 0;
      rc = psg_push_cached(c, p, 0, r, 0, all, PSG_KC_SIG | (carry ? PSG_KC_KEYS : 0u), sigs[p],
                           carry ? keys[p] : nullptr, carry ? n[p] : 0, 2, v, n[p]);
    }
    double vio = 0;
    if (rc == 0) rc = psg_darling_update(c, 0, r, &P, &vio);
    if (vio_out) *vio_out = vio;
    ms[r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                .count();
  }
  if (rc) fprintf(stderr, "psg_e2e_darling: %s\n", psg_last_error());
  psg_destroy(c);
  return rc;
}

// The worker's side of a compressed message (SArray::compressTo,
// shared_array_inl.h:222-230, as Van::send applies it): a raw snappy stream
// -- varint length, then per 64 KB block greedy 4-byte hash matches as
// 2-byte-offset copies (<= 64 bytes) and literals between them.  Harness
// code: it only has to produce valid streams of the usual shape.
extern "C" size_t psg_e2e_compress(const uint8_t* src, size_t n, uint8_t* dst) {
  size_t o = 0;
  for (size_t v = n;;) {
    const uint8_t b = v & 0x7f;
    v >>= 7;
    dst[o++] = (uint8_t)(b | (v ? 0x80 : 0));
    if (!v) break;
  }
  std::vector<int32_t> h(1 << 14);
  auto lit = [&](size_t a, size_t b) {
    if (a == b) return;
    const size_t x = b - a - 1;
    if (x < 60) {
      dst[o++] = (uint8_t)(x << 2);
    } else {
      const int nb = x < 256 ? 1 : x < 65536 ? 2 : x < (1u << 24) ? 3 : 4;
      dst[o++] = (uint8_t)((59 + nb) << 2);
      for (int i = 0; i < nb; ++i) dst[o++] = (uint8_t)(x >> (8 * i));
    }
    memcpy(dst + o, src + a, b - a);
    o += b - a;
  };
  for (size_t blk = 0; blk < n; blk += 65536) {
    const size_t end = blk + 65536 < n ? blk + 65536 : n;
    std::fill(h.begin(), h.end(), -1);
    size_t i = blk, pend = blk;
    while (i + 4 <= end) {
      uint32_t w;
      memcpy(&w, src + i, 4);
      const uint32_t k = (w * 0x1e35a7bdu) >> 18;
      const int32_t c = h[k];
      h[k] = (int32_t)(i - blk);
      if (c >= 0 && memcmp(src + blk + c, src + i, 4) == 0) {
        size_t m = 4;
        while (i + m < end && m < 64 && src[blk + c + m] == src[i + m]) ++m;
        lit(pend, i);
        const size_t off = i - blk - (size_t)c;
        dst[o++] = (uint8_t)(2 | ((m - 1) << 2));
        dst[o++] = (uint8_t)off;
        dst[o++] = (uint8_t)(off >> 8);
        i += m;
        pend = i;
      } else {
        ++i;
      }
    }
    lit(pend, end);
  }
  return o;
}

// The aggregate from compressed messages (Van::recv's uncompressFrom,
// van.cc:204-214, then setValue): each push's key part and value part,
// pinned, through psg_push_compressed, then received(t).
extern "C" int psg_e2e_compressed(int device, int dtype, unsigned flags, const uint64_t* D,
                                  size_t nd, int npush, const void* const* ckeys,
                                  const size_t* ckn, const void* const* cvals, const size_t* cvn,
                                  void* out, int reps, double* ms) {
  psg_ctx* c = nullptr;
  int rc = psg_create(device, dtype, flags, &c);
  if (rc) return rc;
  rc = psg_key_union(c, 0, D, nd);
  const uint64_t all = ~0ull;
  for (int r = 0; rc == 0 && r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; rc == 0 && p < npush; ++p) {
      const void* v[1] = {cvals[p]};
      const size_t vn[1] = {cvn[p]};
      rc = psg_push_compressed(c, 0, r, 0, all, ckeys[p], ckn[p], 1, v, vn);
    }
    void* o[1] = {out};
    if (rc == 0) rc = psg_received(c, r, 1, o);
    ms[r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
                .count();
  }
  if (rc) fprintf(stderr, "psg_e2e_compressed: %s\n", psg_last_error());
  psg_destroy(c);
  return rc;
}
