// kv_vector.h -- host C++ mirror of PS::KVVector<Key, V> over the psg C ABI.
//
// Reference: wakensky/parameter_server src/parameter/kv_vector.h:13-62 (the
// class), :65-73 (received), :75-82 (setValue), :206-213 (getValue),
// :230-235 (slice); message fields from src/system/message.h:17-87 and
// src/proto/task.proto:12-62.  The method names and argument meaning are
// the reference's; the storage behind them (keys, values, per-time
// aggregates) is resident in the HBM of one MI355X, and every hot-path
// operation is a libpsg call (include/psg.h).  Header-only, plain C++11 +
// the C ABI: a server built with g++ links libpsg.so and nothing else.
//
// Where the reference aborts through glog CHECK, this adapter throws
// psg::Error carrying the psg_status (let it escape to get the reference's
// abort).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/psg.h"

namespace psg {

typedef uint64_t Key;

class Error : public std::runtime_error {
 public:
  Error(int status, const std::string& what) : std::runtime_error(what), status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

inline void check(int rc) {
  if (rc != PSG_OK)
    throw Error(rc, std::string(psg_status_string(rc)) + ": " + psg_last_error());
}

// Range<T> (reference src/base/range.h:10-82): half-open [begin, end).
template <class T>
struct Range {
  T b = 0, e = 0;
  Range() {}
  Range(T begin, T end) : b(begin), e(end) {}
  T begin() const { return b; }
  T end() const { return e; }
  size_t size() const { return (size_t)(e - b); }
  bool empty() const { return b >= e; }
  bool operator==(const Range& o) const { return b == o.b && e == o.e; }
  static Range all() { return Range(0, (T)-1); }  // range.h:75-78
};
typedef Range<size_t> SizeR;

// The Task fields the aggregation path reads (task.proto:12-62).
struct Task {
  int time = 0;
  int key_channel = 0;
  Range<Key> key_range = Range<Key>::all();
  bool request = true;
  bool push = true;  // CallSharedPara::PUSH vs PULL
  // key cache fields (task.proto; RNode::cacheKeyRecver, remote_node.cc:139-184)
  bool has_key_signature = false;
  uint32_t key_signature = 0;
  bool has_key = true;
  bool erase_key_cache = false;
};

// PS::Message (message.h:17-87): task header + key bytes + value arrays.
struct Message {
  Task task;
  int sender = 0;  // the remote node (one key cache per node)
  std::vector<Key> key;
  std::vector<std::vector<char>> value;  // each: n * sizeof(V) bytes
  bool valid = true;

  template <typename V>
  void addValue(const std::vector<V>& v) {
    std::vector<char> b(v.size() * sizeof(V));
    if (!v.empty()) std::memcpy(b.data(), v.data(), b.size());
    value.push_back(std::move(b));
  }
  template <typename V>
  std::vector<V> valueAs(size_t i) const {
    std::vector<V> out(value[i].size() / sizeof(V));
    if (!out.empty()) std::memcpy(out.data(), value[i].data(), value[i].size());
    return out;
  }
};
typedef std::shared_ptr<Message> MessagePtr;
typedef std::vector<MessagePtr> MessagePtrList;

template <typename V>
using AlignedArray = std::pair<SizeR, std::vector<V>>;  // message.h:125
template <typename V>
using AlignedArrayList = std::vector<AlignedArray<V>>;  // message.h:126

template <typename V>
struct DType;
template <>
struct DType<float> {
  static const int value = PSG_F32;
};
template <>
struct DType<double> {
  static const int value = PSG_F64;
};

template <typename V>
class KVVector {
 public:
  explicit KVVector(int device = 0, bool parallel_match = false) {
    psg_ctx* c = nullptr;
    check(psg_create(device, DType<V>::value,
                     parallel_match ? PSG_PARALLEL_MATCH : PSG_SERIAL_MATCH, &c));
    ctx_.reset(c, [](psg_ctx* p) { psg_destroy(p); });
  }

  // FLAGS_parallel_match (system/postoffice.cc:24)
  void setParallelMatch(bool on) {
    check(psg_set_match_flags(ctx_.get(), on ? PSG_PARALLEL_MATCH : PSG_SERIAL_MATCH));
  }

  // key(channel) / value(channel) (kv_vector.h:17-18): host copies
  std::vector<Key> key(int channel) const {
    size_t n = 0;
    check(psg_key_size(ctx_.get(), channel, &n));
    std::vector<Key> k(n);
    if (n) check(psg_key_copy(ctx_.get(), channel, 0, n, k.data()));
    return k;
  }
  std::vector<V> value(int channel) const {
    size_t n = 0;
    check(psg_value_size(ctx_.get(), channel, &n));
    std::vector<V> v(n);
    if (n) check(psg_value_copy(ctx_.get(), channel, 0, n, v.data()));
    return v;
  }
  // the app writes value(channel) (e.g. Darling::updateWeight, darling.cc:437-477)
  void setValueArray(int channel, const std::vector<V>& v) {
    check(psg_value_assign(ctx_.get(), channel, v.data(), v.size()));
  }

  // find (kv_vector.h:21-23)
  SizeR find(int channel, const Range<Key>& key_range) const {
    size_t lo = 0, hi = 0;
    check(psg_find_range(ctx_.get(), channel, key_range.begin(), key_range.end(), &lo, &hi));
    return SizeR(lo, hi);
  }

  // received(t) (kv_vector.h:65-73): the aggregate of time t, then erased
  AlignedArrayList<V> received(int t) {
    int m = 0;
    size_t lo = 0, hi = 0;
    check(psg_received_shape(ctx_.get(), t, &m, &lo, &hi));
    AlignedArrayList<V> out(m);
    std::vector<void*> ptrs(m);
    for (int i = 0; i < m; ++i) {
      out[i].first = SizeR(lo, hi);
      out[i].second.resize(hi - lo);
      ptrs[i] = out[i].second.data();
    }
    check(psg_received(ctx_.get(), t, m, ptrs.data()));
    return out;
  }

  // setValue (kv_vector.h:75-82 -> serialSetValue / parallelSetValue); a
  // message with key-cache fields goes through the receiver's key cache
  // first (RNode::cacheKeyRecver): without keys it uses the resident copy
  void setValue(const MessagePtr& msg) {
    const Task& t = msg->task;
    if (t.has_key_signature || !t.has_key || t.erase_key_cache) {
      const unsigned kc = (t.has_key_signature ? PSG_KC_SIG : 0u) |
                          (t.has_key ? PSG_KC_KEYS : 0u) | (t.erase_key_cache ? PSG_KC_ERASE : 0u);
      std::vector<const void*> vals;
      size_t nv = 0;
      for (const auto& v : msg->value) {
        vals.push_back(v.data());
        nv = v.size() / sizeof(V);
      }
      check(psg_push_cached(ctx_.get(), msg->sender, t.key_channel, t.time, t.key_range.begin(),
                            t.key_range.end(), kc, t.key_signature,
                            t.has_key ? msg->key.data() : nullptr, t.has_key ? msg->key.size() : 0,
                            (int)vals.size(), vals.data(), nv));
      return;
    }
    const auto& k = msg->key;
    if (k.empty()) return;                                   // :90, :177
    if (msg->value.empty()) {                                // key-only push :178-182
      check(psg_key_union(ctx_.get(), msg->task.key_channel, k.data(), k.size()));
      return;
    }
    std::vector<const void*> vals;
    for (const auto& v : msg->value) {
      if (v.size() != k.size() * sizeof(V))                  // CHECK_EQ :108, :187
        throw Error(PSG_ERR_SIZE, "value array size != key count");
      vals.push_back(v.data());
    }
    check(psg_push(ctx_.get(), msg->task.key_channel, msg->task.time,
                   msg->task.key_range.begin(), msg->task.key_range.end(), k.data(),
                   k.size(), (int)vals.size(), vals.data()));
  }

  // getValue (kv_vector.h:206-227): a pull request's reply values
  void getValue(const MessagePtr& msg) {
    const auto& k = msg->key;
    if (k.empty()) return;
    std::vector<V> out(k.size());
    size_t matched = 0;
    check(psg_gather(ctx_.get(), msg->task.key_channel, k.data(), k.size(), out.data(),
                     &matched));
    msg->addValue(out);
  }

  // snappy-compressed parts off the wire (Van::recv, van.cc:204-214)
  void setValueCompressed(const Task& t, const std::vector<char>& ckeys,
                          const std::vector<std::vector<char>>& cvals) {
    std::vector<const void*> p;
    std::vector<size_t> n;
    for (const auto& v : cvals) {
      p.push_back(v.data());
      n.push_back(v.size());
    }
    check(psg_push_compressed(ctx_.get(), t.key_channel, t.time, t.key_range.begin(),
                              t.key_range.end(), ckeys.data(), ckeys.size(), (int)p.size(),
                              p.data(), n.data()));
  }

  // tail-feature filter of a channel (SharedParameter::key_filter_,
  // shared_parameter.h:114-133; FreqencyFilter / CountMin)
  bool keyFilterEmpty(int channel) const {
    int e = 1;
    check(psg_freq_empty(ctx_.get(), channel, &e));
    return e != 0;
  }
  void keyFilterResize(int channel, int n, int k) {
    check(psg_freq_resize(ctx_.get(), channel, n, k));
  }
  void keyFilterInsert(int channel, const std::vector<Key>& key,
                       const std::vector<uint32_t>& count) {
    if (key.size() != count.size()) throw Error(PSG_ERR_SIZE, "key/count sizes");  // :37
    check(psg_freq_insert(ctx_.get(), channel, key.data(), count.data(), key.size()));
  }
  std::vector<Key> keyFilterQuery(int channel, const std::vector<Key>& key, int freq) {
    std::vector<Key> out(key.size());
    size_t n = 0;
    check(psg_freq_query(ctx_.get(), channel, key.data(), key.size(), freq, out.data(), &n));
    out.resize(n);
    return out;
  }

  // Darling's server update on the resident aggregate (darling.cc:245-262,
  // 437-477); value arrays are double (KVVector<Key,double>)
  void darlingInit(int channel, double delta_init) {
    check(psg_darling_init(ctx_.get(), channel, delta_init));
  }
  double darlingUpdate(int channel, int time, const psg_darling_param& p) {
    double vio = 0;
    check(psg_darling_update(ctx_.get(), channel, time, &p, &vio));
    return vio;
  }

  // slice (kv_vector.h:230-235 -> sliceKeyOrderedMsg, message.h:89-123):
  // zero-copy in the reference; pieces own their (host) arrays here.
  static MessagePtrList slice(const MessagePtr& msg, const std::vector<Key>& sep) {
    const size_t n = sep.size();
    std::vector<size_t> pos;
    const auto& key = msg->key;
    const Range<Key> kr = msg->task.key_range;
    for (Key p : sep) {
      Key k = std::max(kr.begin(), std::min(kr.end(), p));
      pos.push_back(std::lower_bound(key.begin(), key.end(), k) - key.begin());
    }
    MessagePtrList ret(n - 1);
    for (size_t i = 0; i + 1 < n; ++i) {
      MessagePtr piece(new Message(*msg));
      const Key ib = std::max(sep[i], kr.begin()), ie = std::min(sep[i + 1], kr.end());
      if (ib >= ie) {
        piece->valid = false;  // the remote node does not own this range
      } else {
        piece->valid = true;
        piece->key.assign(key.begin() + pos[i], key.begin() + pos[i + 1]);
        piece->value.clear();
        for (const auto& v : msg->value) {
          const size_t w = key.empty() ? 0 : v.size() / key.size();  // bytes per key
          piece->value.emplace_back(v.begin() + pos[i] * w, v.begin() + pos[i + 1] * w);
        }
      }
      ret[i] = piece;
    }
    return ret;
  }

 private:
  std::shared_ptr<psg_ctx> ctx_;
};

// Server shard boundaries: Range<Key>::all().evenDivide(n, i)
// (range.h:85-98, linear_method.cc:137-145)
inline std::vector<Key> shardBounds(size_t n) {
  std::vector<Key> b(n + 1);
  check(psg_shard_bounds(n, b.data()));
  return b;
}

}  // namespace psg
