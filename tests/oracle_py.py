"""TEST INFRASTRUCTURE: numpy-facing ctypes binding of oracle/liborc.so (the
plain-C restatement of the reference CPU path, oracle/psg_oracle.c) and of
oracle/_ref/libref_murmur3.so (the reference's own MurmurHash3.cc).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
this module; the product path never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_PATH = os.path.join(ROOT, "oracle", "liborc.so")
REF_MURMUR_PATH = os.path.join(ROOT, "oracle", "_ref", "libref_murmur3.so")
REF_CRC_PATH = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")

_p = C.c_void_p
_sz = C.c_size_t
_u64 = C.c_uint64
_psz = C.POINTER(C.c_size_t)
_orc = None


def orc() -> C.CDLL:
    global _orc
    if _orc is None:
        if not os.path.exists(ORC_PATH):
            raise ImportError(f"{ORC_PATH} missing: run `make -C oracle`")
        L = C.CDLL(ORC_PATH)
        sig = {
            "orc_set_union_u64": (_sz, [_p, _sz, _p, _sz, _p]),
            "orc_set_intersection_u64": (_sz, [_p, _sz, _p, _sz, _p]),
            "orc_find_range_u64": (None, [_p, _sz, _u64, _u64, _psz, _psz]),
            "orc_even_divide_u64": (None, [_u64, _u64, _sz, _sz,
                                           C.POINTER(_u64), C.POINTER(_u64)]),
            "orc_slice_key_ordered": (None, [_p, _sz, _u64, _u64, _p, _sz, _p, _p]),
            "orc_gather_f32": (None, [_p, _sz, _p, _p, _sz, _p, _psz]),
            "orc_gather_f64": (None, [_p, _sz, _p, _p, _sz, _p, _psz]),
            "orc_aggregate_f32": (C.c_int, [_p, _sz, _u64, _u64, C.c_int, _p, _p,
                                            C.c_int, _p, C.c_int, C.c_int, _p,
                                            _psz, _psz, _p]),
            "orc_aggregate_f64": (C.c_int, [_p, _sz, _u64, _u64, C.c_int, _p, _p,
                                            C.c_int, _p, C.c_int, C.c_int, _p,
                                            _psz, _psz, _p]),
            "orc_aggregate_scatter_f32": (C.c_int, [_p, _sz, _u64, _u64, C.c_int, _p, _p,
                                                    C.c_int, _p, _p, _psz, _psz, _p]),
            "orc_aggregate_scatter_f64": (C.c_int, [_p, _sz, _u64, _u64, C.c_int, _p, _p,
                                                    C.c_int, _p, _p, _psz, _psz, _p]),
            "orc_aggregate_scatter_serial_f32": (C.c_int, [_p, _sz, _u64, _u64, C.c_int, _p,
                                                           _p, C.c_int, _p, _p, _psz, _psz,
                                                           _p]),
            "orc_aggregate_scatter_serial_f64": (C.c_int, [_p, _sz, _u64, _u64, C.c_int, _p,
                                                           _p, C.c_int, _p, _p, _psz, _psz,
                                                           _p]),
            "orc_old_match_f32": (C.c_int, [_p, _sz, _p, _sz, _p, _u64, _u64, _p,
                                            _psz, _psz, _psz]),
            "orc_murmur3_x64_128": (None, [_p, C.c_int, C.c_uint32, _p]),
            "orc_shuffle_keys": (None, [_p, _sz, C.c_uint32, _p]),
            "orc_darling_update_weight": (None, [_p, _p, _p, _sz, _sz, _p, _p, C.c_double,
                                                 C.c_double, C.c_double, C.c_double, _p]),
            "orc_cm_insert": (None, [_p, C.c_uint32, C.c_int, _p, _p, _sz]),
            "orc_cm_query": (C.c_uint8, [_p, C.c_uint32, C.c_int, _u64]),
            "orc_ff_query": (_sz, [_p, C.c_uint32, C.c_int, _p, _sz, C.c_int, _p]),
            "orc_snappy_uncompressed_length": (C.c_int, [_p, _sz, _psz]),
            "orc_snappy_uncompress": (C.c_int, [_p, _sz, _p, _sz]),
            "orc_snappy_compress": (_sz, [_p, _sz, _p]),
            "orc_crc32c_extend": (C.c_uint32, [C.c_uint32, _p, _sz]),
            "orc_crc32c_mask": (C.c_uint32, [C.c_uint32]),
            "orc_crc32c_unmask": (C.c_uint32, [C.c_uint32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _orc = L
    return _orc


def _a(x):
    return x.ctypes.data


def u64(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint64))


def set_union(a, b) -> np.ndarray:
    a, b = u64(a), u64(b)
    out = np.empty(a.size + b.size + 1, np.uint64)
    n = orc().orc_set_union_u64(_a(a), a.size, _a(b), b.size, _a(out))
    return out[:n]


def set_intersection(a, b) -> np.ndarray:
    a, b = u64(a), u64(b)
    out = np.empty(min(a.size, b.size) + 1, np.uint64)
    n = orc().orc_set_intersection_u64(_a(a), a.size, _a(b), b.size, _a(out))
    return out[:n]


def find_range(a, kb, ke):
    a = u64(a)
    lo, hi = C.c_size_t(), C.c_size_t()
    orc().orc_find_range_u64(_a(a), a.size, int(kb), int(ke), C.byref(lo), C.byref(hi))
    return lo.value, hi.value


def even_divide(b, e, n, i):
    ob, oe = C.c_uint64(), C.c_uint64()
    orc().orc_even_divide_u64(int(b), int(e), n, i, C.byref(ob), C.byref(oe))
    return ob.value, oe.value


def slice_key_ordered(keys, rb, re, sep):
    keys, sep = u64(keys), u64(sep)
    pos = np.zeros(sep.size, np.uint64)
    valid = np.zeros(max(1, sep.size - 1), np.int32)
    orc().orc_slice_key_ordered(_a(keys), keys.size, int(rb), int(re), _a(sep),
                                sep.size, _a(pos), _a(valid))
    return pos, valid[: sep.size - 1]


def aggregate(D, kb, ke, pushes, parallel=False, nthreads=1, dtype=np.float32):
    """pushes: [(keys, [vals]*m)].  Returns (rc, lo, hi, [out]*m, matched)."""
    D = u64(D)
    dtype = np.dtype(dtype)
    npush = len(pushes)
    m = len(pushes[0][1]) if npush else 1
    keys = [u64(k) for k, _ in pushes]
    vals = [np.ascontiguousarray(v, dtype=dtype) for _, vs in pushes for v in vs]
    kp = (C.c_void_p * max(1, npush))(*[_a(k) for k in keys])
    ns = (C.c_size_t * max(1, npush))(*[k.size for k in keys])
    vp = (C.c_void_p * max(1, len(vals)))(*[_a(v) for v in vals])
    lo0, hi0 = find_range(D, kb, ke)
    outs = [np.zeros(max(1, hi0 - lo0), dtype) for _ in range(m)]
    op = (C.c_void_p * m)(*[_a(o) for o in outs])
    lo, hi = C.c_size_t(), C.c_size_t()
    matched = np.zeros(max(1, npush), np.uint64)
    f = orc().orc_aggregate_f32 if dtype == np.float32 else orc().orc_aggregate_f64
    rc = f(_a(D), D.size, int(kb), int(ke), npush, kp, ns, m, vp, int(parallel),
           nthreads, op, C.byref(lo), C.byref(hi), _a(matched))
    n = hi.value - lo.value
    return rc, lo.value, hi.value, [o[:n] for o in outs], matched[:npush]


def aggregate_scatter(D, kb, ke, pushes, dtype=np.float32, parallel=True):
    """parallelSetValue (or, parallel=False, serialSetValue over strictly
    increasing pushes) in O(sum n log |D|) (orc_aggregate_scatter[_serial]):
    results for checks too large for the merge-walk oracle."""
    D = u64(D)
    dtype = np.dtype(dtype)
    npush = len(pushes)
    m = len(pushes[0][1]) if npush else 1
    keys = [u64(k) for k, _ in pushes]
    vals = [np.ascontiguousarray(v, dtype=dtype) for _, vs in pushes for v in vs]
    kp = (C.c_void_p * max(1, npush))(*[_a(k) for k in keys])
    ns = (C.c_size_t * max(1, npush))(*[k.size for k in keys])
    vp = (C.c_void_p * max(1, len(vals)))(*[_a(v) for v in vals])
    lo0, hi0 = find_range(D, kb, ke)
    outs = [np.zeros(max(1, hi0 - lo0), dtype) for _ in range(m)]
    op = (C.c_void_p * m)(*[_a(o) for o in outs])
    lo, hi = C.c_size_t(), C.c_size_t()
    matched = np.zeros(max(1, npush), np.uint64)
    sfx = ("" if parallel else "_serial") + ("_f32" if dtype == np.float32 else "_f64")
    f = getattr(orc(), "orc_aggregate_scatter" + sfx)
    rc = f(_a(D), D.size, int(kb), int(ke), npush, kp, ns, m, vp, op, C.byref(lo), C.byref(hi),
           _a(matched))
    n = hi.value - lo.value
    return rc, lo.value, hi.value, [o[:n] for o in outs], matched[:npush]


def gather(D, W, req, dtype=np.float32):
    D, req = u64(D), u64(req)
    W = np.ascontiguousarray(W, dtype=dtype)
    out = np.zeros(max(1, req.size), dtype)
    mt = C.c_size_t()
    f = orc().orc_gather_f32 if np.dtype(dtype) == np.float32 else orc().orc_gather_f64
    f(_a(D), D.size, _a(W), _a(req), req.size, _a(out), C.byref(mt))
    return out[: req.size], mt.value


def shuffle_keys(ids, seed=512927377):
    ids = u64(ids)
    out = np.empty(ids.size, np.uint64)
    orc().orc_shuffle_keys(_a(ids), ids.size, seed, _a(out))
    return out


def ref_murmur_available() -> bool:
    return os.path.exists(REF_MURMUR_PATH)


def ref_shuffle_keys(ids, seed=512927377):
    """The reference's own MurmurHash3_x64_128 (compiled in place)."""
    L = C.CDLL(REF_MURMUR_PATH)
    f = L.ref_murmur3_x64_128
    f.restype = None
    f.argtypes = [_p, C.c_int, C.c_uint, _p]
    ids = u64(ids)
    out = np.empty(ids.size, np.uint64)
    o = np.zeros(2, np.uint64)
    for i in range(ids.size):
        x = ids[i: i + 1].copy()
        f(_a(x), 8, seed, _a(o))
        out[i] = o[0] ^ o[1]
    return out


# ---- crc32c (util/crc32c.cc:283-330): the key-cache signature ------------
def crc32c(data, init: int = 0) -> int:
    """crc32c::Extend(init, data, len(data)); Value = init 0."""
    b = bytes(memoryview(np.ascontiguousarray(data)).cast("B")) if not isinstance(data, bytes) else data
    return int(orc().orc_crc32c_extend(init, b, len(b)))


def crc32c_mask(c: int) -> int:
    return int(orc().orc_crc32c_mask(c))


def crc32c_unmask(c: int) -> int:
    return int(orc().orc_crc32c_unmask(c))


def key_signature(keys, max_sig_len: int = 2048) -> int:
    """RNode::cacheKeySender/Recver signature (remote_node.cc:108,163):
    Value(key bytes, min(key bytes, max_sig_len_))."""
    b = u64(keys).tobytes()
    return crc32c(b[:max_sig_len])


def ref_crc_available() -> bool:
    return os.path.exists(REF_CRC_PATH)


def ref_crc32c(data: bytes, init: int = 0) -> int:
    """The reference's own crc32c::Extend (src/util/crc32c.cc compiled in place)."""
    L = C.CDLL(REF_CRC_PATH)
    L.ref_crc32c_extend.restype = C.c_uint
    L.ref_crc32c_extend.argtypes = [C.c_uint, C.c_char_p, _sz]
    return int(L.ref_crc32c_extend(init, data, len(data)))


# ---- Darling::updateWeight (linear_method/darling.cc:437-477) ------------
def darling_update_weight(value, delta, active, lo, G, U, eta, lam, kkt, delta_max,
                          violation=0.0):
    """In-place on copies: returns (value, delta, active, violation)."""
    value = np.array(value, np.float64)
    delta = np.array(delta, np.float64)
    active = np.array(active, np.uint8)
    G = np.ascontiguousarray(G, np.float64)
    U = np.ascontiguousarray(U, np.float64)
    vio = np.array([violation], np.float64)
    orc().orc_darling_update_weight(_a(value), _a(delta), _a(active), lo, G.size, _a(G), _a(U),
                                    eta, lam, kkt, delta_max, _a(vio))
    return value, delta, active, float(vio[0])


# ---- CountMin<uint64,uint8> / FreqencyFilter (countmin.h, frequency_filter.h)
def cm_resize(n, k):
    """CountMin::resize (countmin.h:14-19): (table, n_, k_)."""
    n = max(int(n), 64)
    return np.zeros(n, np.uint8), n, min(30, max(1, int(k)))


def cm_insert(table, n, k, keys, counts):
    keys, counts = u64(keys), np.ascontiguousarray(counts, np.uint32)
    orc().orc_cm_insert(_a(table), n, k, _a(keys), _a(counts), keys.size)


def ff_query(table, n, k, keys, freq):
    keys = u64(keys)
    out = np.empty(max(1, keys.size), np.uint64)
    m = orc().orc_ff_query(_a(table), n, k, _a(keys), keys.size, freq, _a(out))
    return out[:m].copy()


# ---- snappy raw format (google/snappy; absent from the reference tree) -----
def snappy_compress(data: bytes) -> bytes:
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    out = np.zeros(32 + len(data) + len(data) // 6, np.uint8)
    n = orc().orc_snappy_compress(_a(src), len(data), _a(out))
    return out[:n].tobytes()


def snappy_uncompress(data: bytes):
    """bytes, or None for a corrupt stream (RawUncompress false)."""
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    ln = C.c_size_t()
    if orc().orc_snappy_uncompressed_length(_a(src), len(data), C.byref(ln)) < 0:
        return None
    out = np.zeros(max(1, ln.value), np.uint8)
    if orc().orc_snappy_uncompress(_a(src), len(data), _a(out), ln.value) != 0:
        return None
    return out[: ln.value].tobytes()
