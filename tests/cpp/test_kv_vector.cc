// C++ driver for the KVVector adapter (parameter_server_amd/csrc/kv_vector.h).
// Reads like the reference's own usage: a server KVVector receives
// key-only pushes (the key union), value pushes (setValue) for a time, then
// takes received(t); pull requests go through getValue.  Results are
// compared bit-for-bit with the C oracle (oracle/psg_oracle.h, test-only).
//
//   test_kv_vector host   -- slice / shard bounds (no GPU)
//   test_kv_vector gpu    -- the merge path on device 0
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>

#include "../../oracle/psg_oracle.h"
#include "../../parameter_server_amd/csrc/kv_vector.h"

using psg::Key;
using psg::KVVector;
using psg::Message;
using psg::MessagePtr;

static int failures = 0;
#define EXPECT(c)                                                  \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "%s:%d: EXPECT(%s)\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

template <typename V>
static bool same_bits(const std::vector<V>& a, const std::vector<V>& b) {
  return a.size() == b.size() &&
         (a.empty() || std::memcmp(a.data(), b.data(), a.size() * sizeof(V)) == 0);
}

static MessagePtr key_msg(const std::vector<Key>& k, int chl = 0) {
  MessagePtr m(new Message());
  m->task.key_channel = chl;
  m->key = k;
  return m;
}

// ---- host-only: sliceKeyOrderedMsg (message.h:89-123) and evenDivide ----
static void host_tests() {
  // shard bounds of Range::all().evenDivide(4, i)
  auto b = psg::shardBounds(4);
  EXPECT(b.size() == 5 && b[0] == 0 && b[4] == ~0ull);
  EXPECT(b[1] == 4611686018427387903ull && b[2] == 9223372036854775807ull);

  MessagePtr m = key_msg({1, 4, 7, 9, 12});
  m->addValue(std::vector<float>{1, 2, 3, 4, 5});
  m->task.key_range = psg::Range<Key>(0, 10);
  auto pieces = KVVector<float>::slice(m, {0, 5, 10, 20});
  EXPECT(pieces.size() == 3);
  EXPECT(pieces[0]->valid && (pieces[0]->key == std::vector<Key>{1, 4}));
  EXPECT(same_bits(pieces[0]->valueAs<float>(0), std::vector<float>{1, 2}));
  EXPECT(pieces[1]->valid && (pieces[1]->key == std::vector<Key>{7, 9}));
  EXPECT(same_bits(pieces[1]->valueAs<float>(0), std::vector<float>{3, 4}));
  EXPECT(!pieces[2]->valid);  // [10, 20) is outside key_range [0, 10)
}

// ---- GPU: SURVEY.md Appendix C worked example, both match modes ----
static void appendix_c(bool parallel) {
  KVVector<float> kv(0, parallel);
  kv.setValue(key_msg({3, 5, 8, 9, 10, 11}));
  EXPECT((kv.key(0) == std::vector<Key>{3, 5, 8, 9, 10, 11}));
  MessagePtr p0 = key_msg({5, 9}), p1 = key_msg({3, 5, 11});
  p0->task.time = p1->task.time = 7;
  p0->addValue(std::vector<float>{1.5f, 2.5f});
  p1->addValue(std::vector<float>{0.25f, 1.0f, 4.0f});
  kv.setValue(p0);
  kv.setValue(p1);
  auto r = kv.received(7);
  EXPECT(r.size() == 1 && r[0].first == psg::SizeR(0, 6));
  EXPECT(same_bits(r[0].second, std::vector<float>{0.25f, 2.5f, 0.0f, 2.5f, 0.0f, 4.0f}));
  bool threw = false;
  try {
    kv.received(7);  // erased after the first call (kv_vector.h:69-72)
  } catch (const psg::Error& e) {
    threw = e.status() == PSG_ERR_NO_TIME;
  }
  EXPECT(threw);

  // pull (getValue): W = {10..60}, request {5, 6, 11} -> {20, 0, 60}
  kv.setValueArray(0, {10, 20, 30, 40, 50, 60});
  MessagePtr pull = key_msg({5, 6, 11});
  kv.getValue(pull);
  EXPECT(same_bits(pull->valueAs<float>(0), std::vector<float>{20, 0, 60}));

  // sub-range push (key_range [4, 11) -> positions [1, 5))
  MessagePtr q0 = key_msg({5, 9}), q1 = key_msg({5});
  q0->task.time = q1->task.time = 8;
  q0->task.key_range = q1->task.key_range = psg::Range<Key>(4, 11);
  q0->addValue(std::vector<float>{1.5f, 2.5f});
  q1->addValue(std::vector<float>{1.0f});
  kv.setValue(q0);
  kv.setValue(q1);
  auto s = kv.received(8);
  EXPECT(s.size() == 1 && s[0].first == psg::SizeR(1, 5));
  EXPECT(same_bits(s[0].second, std::vector<float>{2.5f, 0.0f, 2.5f, 0.0f}));
  EXPECT(kv.find(0, psg::Range<Key>(4, 11)) == psg::SizeR(1, 5));
}

// ---- GPU: random pushes (m = 2, Darling's layout) vs the oracle ----
template <typename V>
static void random_vs_oracle(bool parallel, unsigned seed) {
  std::mt19937_64 rng(seed);
  std::set<Key> ks;
  while (ks.size() < 20000) ks.insert(rng() >> 20);
  std::vector<Key> D(ks.begin(), ks.end());
  KVVector<V> kv(0, parallel);
  kv.setValue(key_msg(D));

  const int npush = 9, m = 2, t = 3;
  std::vector<std::vector<Key>> pk(npush);
  std::vector<std::vector<V>> pv(npush * m);
  std::uniform_real_distribution<double> U(-1, 1);
  for (int p = 0; p < npush; ++p) {
    for (Key k : D)
      if ((rng() % 100) < (unsigned)(10 + 10 * p)) pk[p].push_back(k);
    MessagePtr msg = key_msg(pk[p]);
    msg->task.time = t;
    for (int i = 0; i < m; ++i) {
      for (size_t j = 0; j < pk[p].size(); ++j) pv[p * m + i].push_back((V)U(rng));
      if (p == 2 && i == 0 && !pv[p * m].empty()) pv[p * m][0] = (V)-0.0;
      msg->addValue(pv[p * m + i]);
    }
    kv.setValue(msg);
  }
  auto r = kv.received(t);

  std::vector<const Key*> kp(npush);
  std::vector<size_t> n(npush), matched(npush);
  std::vector<const V*> vp(npush * m);
  for (int p = 0; p < npush; ++p) {
    kp[p] = pk[p].data();
    n[p] = pk[p].size();
    for (int i = 0; i < m; ++i) vp[p * m + i] = pv[p * m + i].data();
  }
  std::vector<std::vector<V>> want(m, std::vector<V>(D.size()));
  std::vector<V*> wp = {want[0].data(), want[1].data()};
  size_t lo = 0, hi = 0;
  int rc;
  if (sizeof(V) == 4)
    rc = orc_aggregate_f32(D.data(), D.size(), 0, ~0ull, npush, kp.data(), n.data(), m,
                           (const float* const*)vp.data(), parallel, 1, (float* const*)wp.data(),
                           &lo, &hi, matched.data());
  else
    rc = orc_aggregate_f64(D.data(), D.size(), 0, ~0ull, npush, kp.data(), n.data(), m,
                           (const double* const*)vp.data(), parallel, 1,
                           (double* const*)wp.data(), &lo, &hi, matched.data());
  EXPECT(rc == 0 && lo == 0 && hi == D.size());
  EXPECT(r.size() == (size_t)m);
  for (int i = 0; i < m && i < (int)r.size(); ++i) EXPECT(same_bits(r[i].second, want[i]));

  // a push carrying a key the server does not hold -> CHECK failure
  MessagePtr bad = key_msg({D[0], D[1] + 1 == D[2] ? D[2] + 1 : D[1] + 1});
  bad->task.time = t + 1;
  bad->addValue(std::vector<V>{1, 2});
  int status = PSG_OK;
  try {
    kv.setValue(bad);
    kv.received(t + 1);
  } catch (const psg::Error& e) {
    status = e.status();
  }
  EXPECT(status == PSG_ERR_UNMATCHED);
}

// ---- GPU: the rows around the merge, through the adapter ----
// the receiver's key cache: iteration 1 carries keys + signature, iteration
// 2 only the signature; both merges equal plain pushes (oracle)
static void key_cache_and_filter() {
  std::mt19937_64 rng(7);
  std::set<Key> ks;
  while (ks.size() < 6000) ks.insert(rng() >> 20);
  std::vector<Key> D(ks.begin(), ks.end());
  KVVector<float> kv;
  kv.setValue(key_msg(D));
  std::vector<std::vector<Key>> pk;
  std::vector<std::vector<float>> pv;
  for (int w = 0; w < 3; ++w) {
    std::vector<Key> k;
    for (size_t i = w; i < D.size(); i += 2 + w) k.push_back(D[i]);
    std::vector<float> v(k.size());
    for (auto& x : v) x = (float)((int)(rng() % 2001) - 1000) / 256.0f;
    pk.push_back(k);
    pv.push_back(v);
  }
  for (int t = 1; t <= 2; ++t) {
    for (int w = 0; w < 3; ++w) {
      MessagePtr m(new Message());
      m->task.time = t;
      m->sender = w;
      m->task.has_key_signature = true;
      m->task.key_signature = orc_crc32c_extend(0, pk[w].data(),
                                                std::min<size_t>(8 * pk[w].size(), 2048));
      m->task.has_key = t == 1;
      if (t == 1) m->key = pk[w];
      m->addValue(pv[w]);
      kv.setValue(m);
    }
    auto got = kv.received(t);
    std::vector<float> want(D.size());
    const uint64_t* keys[3] = {pk[0].data(), pk[1].data(), pk[2].data()};
    const size_t n[3] = {pk[0].size(), pk[1].size(), pk[2].size()};
    const float* vals[3] = {pv[0].data(), pv[1].data(), pv[2].data()};
    float* out[1] = {want.data()};
    size_t lo, hi, matched[3];
    orc_aggregate_f32(D.data(), D.size(), 0, ~0ull, 3, keys, n, 1, vals, 0, 1, out, &lo, &hi,
                      matched);
    EXPECT(got.size() == 1 && same_bits(got[0].second, want));
  }
  // FreqencyFilter: insertKeys then queryKeys against the oracle's CountMin
  kv.keyFilterResize(0, 5000, 3);
  EXPECT(!kv.keyFilterEmpty(0));
  std::vector<uint32_t> cnt(D.size());
  for (auto& c : cnt) c = (uint32_t)(rng() % 700);
  kv.keyFilterInsert(0, D, cnt);
  std::vector<uint8_t> table(5000, 0);
  orc_cm_insert(table.data(), 5000, 3, D.data(), cnt.data(), D.size());
  std::vector<Key> want(D.size());
  want.resize(orc_ff_query(table.data(), 5000, 3, D.data(), D.size(), 100, want.data()));
  EXPECT(kv.keyFilterQuery(0, D, 100) == want);
}

// Darling's fused server update against the oracle's updateWeight
static void darling() {
  std::mt19937_64 rng(11);
  std::vector<Key> D;
  for (Key k = 0; k < 3000; ++k) D.push_back(k * 977 + 5);
  KVVector<double> kv;
  kv.setValue(key_msg(D));
  std::vector<double> w(D.size(), 0.0), delta(D.size(), 1.0);
  std::vector<uint8_t> act(D.size(), 1);
  kv.setValueArray(0, w);
  kv.darlingInit(0, 1.0);
  const psg_darling_param P = {0.7, 0.2, 1e20, 4.0};
  for (int t = 1; t <= 3; ++t) {
    std::vector<Key> k;
    for (size_t i = t; i < D.size(); i += 3) k.push_back(D[i]);
    std::vector<double> g(k.size()), u(k.size());
    for (size_t i = 0; i < k.size(); ++i) {
      g[i] = (double)((int)(rng() % 2001) - 1000) / 300.0;
      u[i] = (double)(rng() % 1000) / 400.0;
    }
    MessagePtr m = key_msg(k);
    m->task.time = t;
    m->addValue(g);
    m->addValue(u);
    kv.setValue(m);
    const double vio = kv.darlingUpdate(0, t, P);
    // the oracle: aggregate (m = 2) then updateWeight over [0, n)
    std::vector<double> G(D.size()), U(D.size());
    const uint64_t* keys[1] = {k.data()};
    const size_t n[1] = {k.size()};
    const double* vals[2] = {g.data(), u.data()};
    double* out[2] = {G.data(), U.data()};
    size_t lo, hi, matched[1];
    orc_aggregate_f64(D.data(), D.size(), 0, ~0ull, 1, keys, n, 2, vals, 0, 1, out, &lo, &hi,
                      matched);
    double want_vio = 0;
    orc_darling_update_weight(w.data(), delta.data(), act.data(), 0, D.size(), G.data(),
                              U.data(), P.eta, P.lambda, P.kkt_filter_threshold, P.delta_max,
                              &want_vio);
    EXPECT(std::memcmp(&vio, &want_vio, sizeof(double)) == 0);
  }
  EXPECT(same_bits(kv.value(0), w));
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "host";
  try {
    host_tests();
    if (mode == "gpu") {
      appendix_c(false);
      appendix_c(true);
      random_vs_oracle<float>(false, 1);
      random_vs_oracle<float>(true, 2);
      random_vs_oracle<double>(false, 3);
      key_cache_and_filter();
      darling();
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "uncaught: %s\n", e.what());
    return 2;
  }
  std::printf("%s: %d failure(s)\n", mode.c_str(), failures);
  return failures ? 1 : 0;
}
