// MEASUREMENT AID (not product code): the PCIe-inclusive host path of one
// aggregate driven through the C ABI from C++, as the reference's C++ server
// would call it (SharedParameter::process -> setValue per push ->
// received(t), src/parameter/shared_parameter.h:91-149), without Python in
// the loop.  bench.py loads this library with ctypes and passes the host
// buffers (pageable or pinned).
#include <chrono>
#include <cstdint>
#include <cstdio>
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
