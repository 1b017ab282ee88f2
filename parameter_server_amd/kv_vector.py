"""Python mirror of the reference's server-side KV surface over the C ABI.

``KVVector`` follows ``PS::KVVector<Key,V>`` (reference
src/parameter/kv_vector.h:13-62) method for method -- ``key``, ``value``,
``find``, ``received``, ``setValue``, ``getValue`` -- with the message
fields of ``PS::Message``/``Task`` that the path reads
(src/system/message.h:17-87, src/proto/task.proto:12-62).  Every call goes
to libpsg.so; a failing reference ``CHECK`` surfaces as :class:`PSGError`.

``MergePlan`` is the device-resident batched form used by bench.py and the
multi-GPU shards: every buffer is a device pointer (e.g. a torch tensor's
``data_ptr()``), and a run is two kernel launches on a caller stream.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import PSG_F32, PSG_F64, PSG_PARALLEL_MATCH, PSG_SERIAL_MATCH

KEY_ALL = (0, (1 << 64) - 1)  # Range<uint64>::all() (range.h:75-78)


def _np_dtype(dtype: int):
    return np.float32 if dtype == PSG_F32 else np.float64


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


@dataclass
class Message:
    """The fields of PS::Message / Task the aggregation path reads."""

    time: int = 0
    key_channel: int = 0
    key_range: tuple = KEY_ALL
    push: bool = True
    request: bool = True
    key: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    value: List[np.ndarray] = field(default_factory=list)
    # key cache fields (task.proto: key_signature, has_key, erase_key_cache;
    # system/remote_node.cc:96-184); key_signature None = not set
    key_signature: Optional[int] = None
    has_key: bool = True
    erase_key_cache: bool = False
    sender: int = 0  # the remote node (each has its own key cache)


class KVVector:
    """KVVector<uint64, V> with keys, values and aggregates resident in HBM."""

    def __init__(self, device: int = 0, dtype: int = PSG_F32,
                 parallel_match: bool = False, flags: int = 0):
        """flags: context options of psg_create (PSG_HOLD_BUFFERS and the
        kernel-form overrides of include/psg.h, tests only)."""
        self._L = _lib.lib()
        self.dtype = dtype
        self.np_dtype = _np_dtype(dtype)
        h = C.c_void_p()
        self._opts = flags & ~PSG_PARALLEL_MATCH
        flags = self._opts | (PSG_PARALLEL_MATCH if parallel_match else PSG_SERIAL_MATCH)
        _lib.check(self._L.psg_create(device, dtype, flags, C.byref(h)))
        self._h = h

    def union_keys(self, channel: int, key_lists) -> None:
        """Several key-only pushes at once (psg_key_union_batch): the key set
        setUnion of each in turn gives (kv_vector.h:177-182), merged on the
        device in one N-way pass."""
        ks = [np.ascontiguousarray(k, np.uint64) for k in key_lists]
        arr = _lib.ptr_array([_ptr(k) if k.size else 0 for k in ks])
        ns = (C.c_size_t * max(1, len(ks)))(*[k.size for k in ks])
        _lib.check(self._L.psg_key_union_batch(self._h, channel, arr, ns, len(ks)))

    def set_flush_pushes(self, n: int) -> None:
        """Pushes merged per launch (launch seams; psg_set_flush_pushes)."""
        _lib.check(self._L.psg_set_flush_pushes(self._h, n))

    def close(self):
        if getattr(self, "_h", None):
            self._L.psg_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_parallel_match(self, on: bool):
        """FLAGS_parallel_match (system/postoffice.cc:24)."""
        _lib.check(self._L.psg_set_match_flags(
            self._h, self._opts | (PSG_PARALLEL_MATCH if on else PSG_SERIAL_MATCH)))

    # -- key(ch) / value(ch) / find(ch, range): kv_vector.h:17-23 ---------
    def key(self, channel: int) -> np.ndarray:
        n = C.c_size_t()
        _lib.check(self._L.psg_key_size(self._h, channel, C.byref(n)))
        out = np.empty(n.value, np.uint64)
        _lib.check(self._L.psg_key_copy(self._h, channel, 0, n.value, _ptr(out)))
        return out

    def value(self, channel: int) -> np.ndarray:
        n = C.c_size_t()
        _lib.check(self._L.psg_value_size(self._h, channel, C.byref(n)))
        out = np.empty(n.value, self.np_dtype)
        _lib.check(self._L.psg_value_copy(self._h, channel, 0, n.value, _ptr(out)))
        return out

    def set_value_array(self, channel: int, vals) -> None:
        """Assign value(channel) (the app side writes it, e.g. Darling
        updateWeight, darling.cc:437-477)."""
        v = np.ascontiguousarray(vals, dtype=self.np_dtype)
        _lib.check(self._L.psg_value_assign(self._h, channel, _ptr(v), v.size))

    def find(self, channel: int, key_range) -> tuple:
        lo, hi = C.c_size_t(), C.c_size_t()
        _lib.check(self._L.psg_find_range(self._h, channel, int(key_range[0]),
                                          int(key_range[1]), C.byref(lo),
                                          C.byref(hi)))
        return lo.value, hi.value

    # -- setValue: kv_vector.h:75-82 ---------------------------------------
    def setValue(self, msg: Message) -> None:
        if msg.key_signature is not None or not msg.has_key or msg.erase_key_cache:
            return self._set_value_cached(msg)
        keys = np.ascontiguousarray(msg.key, dtype=np.uint64)
        if keys.size == 0:
            return
        if not msg.value:  # key-only push: key_ = key_.setUnion(recv) (:177-182)
            _lib.check(self._L.psg_key_union(self._h, msg.key_channel, _ptr(keys),
                                             keys.size))
            return
        vals = []
        for v in msg.value:
            a = np.ascontiguousarray(v, dtype=self.np_dtype)
            if a.size != keys.size:  # CHECK_EQ(recv_data.size(), recv_key.size())
                raise _lib.PSGError(_lib.PSG_ERR_SIZE,
                                    f"{a.size} values for {keys.size} keys")
            vals.append(a)
        arr = _lib.ptr_array([_ptr(a) for a in vals])
        _lib.check(self._L.psg_push(self._h, msg.key_channel, msg.time,
                                    int(msg.key_range[0]), int(msg.key_range[1]),
                                    _ptr(keys), keys.size, len(vals), arr))

    def _set_value_cached(self, msg: Message) -> None:
        """RNode::cacheKeyRecver (remote_node.cc:139-184), then setValue: the
        keys of a message without them are the resident cached copy."""
        from ._lib import PSG_KC_ERASE, PSG_KC_KEYS, PSG_KC_SIG
        kc = (PSG_KC_SIG if msg.key_signature is not None else 0) | \
             (PSG_KC_KEYS if msg.has_key else 0) | (PSG_KC_ERASE if msg.erase_key_cache else 0)
        keys = np.ascontiguousarray(msg.key if msg.has_key else np.zeros(0), dtype=np.uint64)
        vals = [np.ascontiguousarray(v, dtype=self.np_dtype) for v in msg.value]
        nv = vals[0].size if vals else 0
        if any(v.size != nv for v in vals):
            raise _lib.PSGError(_lib.PSG_ERR_SIZE, "value arrays of different sizes")
        arr = _lib.ptr_array([_ptr(a) for a in vals]) if vals else None
        _lib.check(self._L.psg_push_cached(
            self._h, msg.sender, msg.key_channel, msg.time, int(msg.key_range[0]), int(msg.key_range[1]),
            kc, int(msg.key_signature or 0) & 0xffffffff, _ptr(keys) if keys.size else None,
            keys.size, len(vals), arr, nv))

    def key_cache_bytes(self, sender: int = -1) -> int:
        """RNode::memSize (remote_node.cc:186-195); -1: all senders."""
        n = C.c_size_t()
        _lib.check(self._L.psg_key_cache_bytes(self._h, sender, C.byref(n)))
        return n.value

    def clear_key_cache(self, sender: int = -1) -> None:
        """RNode::clearCache (remote_node.h:54); -1: all senders."""
        _lib.check(self._L.psg_key_cache_clear(self._h, sender))

    # -- received(t): kv_vector.h:65-73 ------------------------------------
    def received(self, t: int, out: Optional[List[np.ndarray]] = None):
        """Returns [((lo, hi), values_i) for each value array], then erases t.
        `out`: caller arrays (e.g. pinned) of at least hi - lo entries."""
        m, lo, hi = C.c_int(), C.c_size_t(), C.c_size_t()
        _lib.check(self._L.psg_received_shape(self._h, t, C.byref(m), C.byref(lo),
                                              C.byref(hi)))
        n = hi.value - lo.value
        if out is not None and len(out) == m.value and all(
                o.dtype == self.np_dtype and o.size >= n and o.flags.c_contiguous for o in out):
            outs = [o[:n] for o in out]
        else:
            outs = [np.empty(n, self.np_dtype) for _ in range(m.value)]
        arr = _lib.ptr_array([_ptr(o) for o in outs])
        _lib.check(self._L.psg_received(self._h, t, m.value, arr))
        return [((lo.value, hi.value), o) for o in outs]

    # -- getValue (pull request): kv_vector.h:206-227 ----------------------
    def getValue(self, msg: Message) -> int:
        """Fills msg.value with value(channel) gathered at msg.key; returns
        the matched count."""
        keys = np.ascontiguousarray(msg.key, dtype=np.uint64)
        if keys.size == 0:
            return 0
        out = np.empty(keys.size, self.np_dtype)
        matched = C.c_size_t()
        _lib.check(self._L.psg_gather(self._h, msg.key_channel, _ptr(keys), keys.size,
                                      _ptr(out), C.byref(matched)))
        msg.value.append(out)
        return matched.value


class MergePlan:
    """A prepared device-resident batch of (channel, time) merges.

    jobs: list of dicts with device pointers
        {"keys": int, "nslots": int, "push_keys": [int], "push_vals": [[int]*m],
         "push_n": [int], "out": [int]*m}
    """

    def __init__(self, device: int, dtype: int, m: int, jobs: Sequence[dict],
                 parallel_match: bool = False, flags: int = 0):
        """flags: kernel-form overrides of include/psg.h (tests, A/B only)."""
        self._L = _lib.lib()
        self._keep = []
        cj = (_lib.MergeJob * max(1, len(jobs)))()
        for j, J in enumerate(jobs):
            npush = len(J["push_keys"])
            pk = _lib.ptr_array(J["push_keys"])
            pv = _lib.ptr_array([v for vs in J["push_vals"] for v in vs])
            pn = (C.c_uint64 * max(1, npush))(*J["push_n"])
            out = _lib.ptr_array(J["out"])
            self._keep += [pk, pv, pn, out]
            cj[j].keys = J["keys"]
            cj[j].nslots = J["nslots"]
            cj[j].npush = npush
            cj[j].push_keys = C.cast(pk, C.POINTER(C.c_void_p))
            cj[j].push_vals = C.cast(pv, C.POINTER(C.c_void_p))
            cj[j].push_n = C.cast(pn, C.POINTER(C.c_uint64))
            cj[j].out = C.cast(out, C.POINTER(C.c_void_p))
        h = C.c_void_p()
        flags = (flags & ~PSG_PARALLEL_MATCH) | (PSG_PARALLEL_MATCH if parallel_match
                                                 else PSG_SERIAL_MATCH)
        _lib.check(self._L.psg_plan_create(device, dtype, m, flags, cj, len(jobs),
                                           C.byref(h)))
        self._h = h
        self.npush_total = sum(len(J["push_keys"]) for J in jobs)
        b, kv = C.c_uint64(), C.c_uint64()
        _lib.check(self._L.psg_plan_bytes(h, C.byref(b), C.byref(kv)))
        self.bytes, self.kv_pairs = b.value, kv.value
        f = C.c_int()
        _lib.check(self._L.psg_plan_form(h, C.byref(f)))
        self.form = f.value  # _lib.PSG_KERNEL_*

    def run(self, stream: Optional[int] = None) -> None:
        _lib.check(self._L.psg_plan_run(self._h, stream or None))

    def run_stage(self, stage: int, stream: Optional[int] = None) -> None:
        """0 = partition, 1 = aggregate (the dominant kernel)."""
        _lib.check(self._L.psg_plan_run_stage(self._h, stage, stream or None))

    def matched(self) -> np.ndarray:
        out = np.zeros(max(1, self.npush_total), np.uint64)
        _lib.check(self._L.psg_plan_matched(
            self._h, out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out[: self.npush_total]

    def close(self):
        if getattr(self, "_h", None):
            self._L.psg_plan_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class NWayMergeBatch:
    """A batch of independent N-way merges run as one pipeline
    (psg_nway_create_batch: one launch per stage over every merge).

    merges: [dict(push_keys=[ptr], push_n=[n], push_vals=[[ptr] * m],
    out_keys=ptr, out_vals=[ptr] * m)]; all device pointers."""

    def __init__(self, device: int, dtype: int, merges, parallel_match: bool = False):
        self._L = _lib.lib()
        m = len(merges[0]["out_vals"]) if merges else 0
        npush = [len(x["push_keys"]) for x in merges]
        keys = [k for x in merges for k in x["push_keys"]]
        ns = [n for x in merges for n in x["push_n"]]
        vals = [v for x in merges for vs in x["push_vals"] for v in vs]
        np_ = (C.c_int * max(1, len(npush)))(*npush)
        pk = _lib.ptr_array(keys) if keys else None
        pn = (C.c_uint64 * max(1, len(ns)))(*ns)
        pv = _lib.ptr_array(vals) if m and vals else None
        ok = _lib.ptr_array([x["out_keys"] for x in merges])
        ov = _lib.ptr_array([v for x in merges for v in x["out_vals"]]) if m else None
        self._keep = [np_, pk, pn, pv, ok, ov]
        self.nmerge = len(merges)
        h = C.c_void_p()
        flags = PSG_PARALLEL_MATCH if parallel_match else PSG_SERIAL_MATCH
        _lib.check(self._L.psg_nway_create_batch(device, dtype, m, flags, len(merges), np_, pk, pn,
                                                 pv, ok, ov, C.byref(h)))
        self._h = h
        b, kv = C.c_uint64(), C.c_uint64()
        _lib.check(self._L.psg_nway_bytes(h, C.byref(b), C.byref(kv)))
        self.bytes_in, self.kv_pairs = b.value, kv.value

    def run(self, stream: Optional[int] = None) -> None:
        _lib.check(self._L.psg_nway_run(self._h, stream or None))

    def result(self) -> List[int]:
        """Synchronises; the merged key count of each merge."""
        n = (C.c_uint64 * self.nmerge)()
        _lib.check(self._L.psg_nway_result(self._h, n))
        return list(n)

    def close(self):
        if getattr(self, "_h", None):
            self._L.psg_nway_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class NWayMerge:
    """A prepared N-way merge (psg_nway_*): the union of sorted device
    pushes and, with values, their per-key sums in arrival order.

    push_keys / push_n: device pointers / lengths; push_vals: [[ptr] * m]
    per push (m = 0: keys only); out_keys / out_vals: device pointers of
    sum(n) entries each."""

    def __init__(self, device: int, dtype: int, push_keys, push_n, push_vals, out_keys,
                 out_vals=(), parallel_match: bool = False):
        self._L = _lib.lib()
        m = len(out_vals)
        P = len(push_keys)
        pk = _lib.ptr_array(push_keys)
        pn = (C.c_uint64 * max(1, P))(*push_n)
        pv = _lib.ptr_array([v for vs in push_vals for v in vs]) if m else None
        ov = _lib.ptr_array(list(out_vals)) if m else None
        self._keep = [pk, pn, pv, ov]
        h = C.c_void_p()
        flags = PSG_PARALLEL_MATCH if parallel_match else PSG_SERIAL_MATCH
        _lib.check(self._L.psg_nway_create(device, dtype, m, flags, P, pk, pn, pv, out_keys, ov,
                                           C.byref(h)))
        self._h = h
        b, kv = C.c_uint64(), C.c_uint64()
        _lib.check(self._L.psg_nway_bytes(h, C.byref(b), C.byref(kv)))
        self.bytes_in, self.kv_pairs = b.value, kv.value

    def run(self, stream: Optional[int] = None) -> None:
        _lib.check(self._L.psg_nway_run(self._h, stream or None))

    def result(self) -> int:
        """Synchronises; the merged key count (PSGError if a push was unsorted)."""
        n = C.c_uint64()
        _lib.check(self._L.psg_nway_result(self._h, C.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "_h", None):
            self._L.psg_nway_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def shard_bounds(n: int) -> np.ndarray:
    """Range<uint64>::all().evenDivide(n, i) boundaries (range.h:85-98)."""
    L = _lib.lib()
    out = np.zeros(n + 1, np.uint64)
    _lib.check(L.psg_shard_bounds(n, out.ctypes.data_as(C.POINTER(C.c_uint64))))
    return out
