"""Tail-feature filter: FreqencyFilter<uint64> over
CountMin<uint64, uint8> (src/parameter/frequency_filter.h:27-43,
src/base/countmin.h:14-67), as SharedParameter::process drives it
(shared_parameter.h:114-133).

The oracle (oracle/psg_oracle.c orc_cm_*) is a restatement, PARITY
UNPINNED: the reference's countmin_test.cc is entirely commented out and
countmin.h cannot be compiled here (glog through shared_array_inl.h); it is
checked against an independent pure-Python restatement.  The GPU table is
compared byte for byte and the filtered keys in order.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O

M32 = 0xFFFFFFFF


def py_hash(key):
    seed, m, n = 0xbc9f1d34, 0xc6a4a793, 8
    h = (seed ^ (n * m)) & M32
    w = key & M32
    h = ((h + w) * m) & M32
    h ^= h >> 16
    w = (key >> 32) & M32
    h = ((h + w) * m) & M32
    h ^= h >> 16
    return h


def py_probes(key, n, k):
    h = py_hash(int(key))
    delta = ((h >> 17) | (h << 15)) & M32
    for _ in range(k):
        yield h % n
        h = (h + delta) & M32


def py_insert(table, n, k, keys, counts):
    for key, c in zip(keys, counts):
        c = int(c) & 0xFF
        for p in py_probes(key, n, k):
            table[p] = (int(table[p]) + c) & 0xFF


def py_query(table, n, k, keys, freq):
    out = []
    for key in keys:
        res = 255
        for p in py_probes(key, n, k):
            res = min(res, int(table[p]))
        if res > freq:
            out.append(key)
    return np.asarray(out, np.uint64)


def zipf_keys(rng, n, a=1.1, space=1 << 40):
    ranks = rng.zipf(a, n).astype(np.uint64) % np.uint64(space)
    return O.shuffle_keys(ranks)


@pytest.mark.parametrize("n,k", [(10, 3), (1000, 1), (777, 40)])
def test_countmin_oracle_vs_python(n, k):
    rng = np.random.default_rng(n + k)
    t, nn, kk = O.cm_resize(n, k)
    assert nn == max(n, 64) and kk == min(30, max(1, k))
    tp = t.copy()
    for _ in range(3):
        keys = np.unique(zipf_keys(rng, 2000))
        counts = rng.integers(0, 700, keys.size).astype(np.uint32)  # > 255: uint8 truncation
        O.cm_insert(t, nn, kk, keys, counts)
        py_insert(tp, nn, kk, keys, counts)
    assert np.array_equal(t, tp)
    q = zipf_keys(rng, 3000)
    for freq in (0, 3, 100, 254):
        assert np.array_equal(O.ff_query(t, nn, kk, q, freq), py_query(tp, nn, kk, q, freq))


# ------------------------------------------------------------------ GPU --
def _ctx():
    from parameter_server_amd.kv_vector import KVVector
    return KVVector(0)


def _table(v, ch, n):
    from parameter_server_amd import _lib
    out = np.empty(n, np.uint8)
    _lib.check(v._L.psg_freq_table(v._h, ch, out.ctypes.data, n))
    return out


def _query(v, ch, keys, freq):
    import ctypes as C
    from parameter_server_amd import _lib
    keys = np.ascontiguousarray(keys, np.uint64)
    out = np.empty(max(1, keys.size), np.uint64)
    m = C.c_size_t()
    _lib.check(v._L.psg_freq_query(v._h, ch, keys.ctypes.data, keys.size, freq, out.ctypes.data,
                                   C.byref(m)))
    return out[: m.value]


@pytest.mark.gpu
def test_gpu_freq_filter_vs_oracle():
    """The filter as the server sizes it (shared_parameter.h:118-122: n =
    max(w * countmin_n / log(w + 1), 64)), several insertKeys batches of
    unique Zipf keys with uint32 counts (byte wrap), then queryKeys at
    several thresholds: table bytes and kept keys (in order) exact."""
    import math
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(5)
    w = 16.0
    n = max(int(w * 2_000_000 / math.log(w + 1)), 64)
    k = 4
    v = _ctx()
    e = __import__("ctypes").c_int()
    _lib.check(v._L.psg_freq_empty(v._h, 2, __import__("ctypes").byref(e)))
    assert e.value == 1
    _lib.check(v._L.psg_freq_resize(v._h, 2, n, k))
    t, nn, kk = O.cm_resize(n, k)
    for b in range(4):
        keys = np.unique(zipf_keys(rng, 400_000))
        counts = rng.integers(1, 600, keys.size).astype(np.uint32)
        _lib.check(v._L.psg_freq_insert(v._h, 2, keys.ctypes.data, counts.ctypes.data, keys.size))
        O.cm_insert(t, nn, kk, keys, counts)
    assert np.array_equal(_table(v, 2, nn), t)
    q = zipf_keys(rng, 300_001)
    for freq in (0, 1, 7, 200, 254):
        assert np.array_equal(_query(v, 2, q, freq), O.ff_query(t, nn, kk, q, freq))
    with pytest.raises(_lib.PSGError):
        _query(v, 2, q, 255)  # CHECK_LT(freqency, kuint8max)
    with pytest.raises(_lib.PSGError):
        _query(v, 3, q, 1)  # a channel whose filter was never sized
    _lib.check(v._L.psg_freq_clear(v._h, 2))
    _lib.check(v._L.psg_freq_empty(v._h, 2, __import__("ctypes").byref(e)))
    assert e.value == 1
    v.close()


@pytest.mark.gpu
def test_gpu_freq_filter_device_entry_points_and_k_clamp():
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(6)
    v = _ctx()
    _lib.check(v._L.psg_freq_resize(v._h, 0, 10, 99))  # n -> 64, k -> 30
    t, nn, kk = O.cm_resize(10, 99)
    keys = np.unique(rng.integers(0, 1 << 62, 50_000, dtype=np.uint64))
    counts = rng.integers(0, 1 << 32, keys.size, dtype=np.uint64).astype(np.uint32)
    dk = torch.from_numpy(keys.view(np.int64)).cuda()
    dc = torch.from_numpy(counts.view(np.int32)).cuda()
    _lib.check(v._L.psg_freq_insert_dev(v._h, 0, dk.data_ptr(), dc.data_ptr(), keys.size, None))
    O.cm_insert(t, nn, kk, keys, counts)
    torch.cuda.synchronize()
    assert np.array_equal(_table(v, 0, nn), t)
    n = keys.size
    sb = v._L.psg_freq_query_scratch_bytes(n)
    scratch = torch.empty(sb, dtype=torch.uint8, device="cuda")
    dout = torch.empty(n, dtype=torch.int64, device="cuda")
    dn = torch.zeros(1, dtype=torch.int64, device="cuda")
    for freq in (0, 128):
        _lib.check(v._L.psg_freq_query_dev(v._h, 0, dk.data_ptr(), n, freq, dout.data_ptr(),
                                           dn.data_ptr(), scratch.data_ptr(), None))
        m = int(dn.item())
        got = dout[:m].cpu().numpy().view(np.uint64)
        assert np.array_equal(got, O.ff_query(t, nn, kk, keys, freq))
    v.close()


@pytest.mark.gpu
def test_gpu_freq_filter_large_table_cas_form():
    """A table past the binned insert's 128 MB (2^27 + 4,096 counters): the
    per-probe CAS form runs; bytes exact against the oracle, including
    counters hit by many keys (repeated keys, byte wrap)."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(8)
    v = _ctx()
    n = (1 << 27) + 4096
    _lib.check(v._L.psg_freq_resize(v._h, 1, n, 3))
    t, nn, kk = O.cm_resize(n, 3)
    keys = np.concatenate([rng.integers(0, 1 << 62, 60_000, dtype=np.uint64),
                           np.full(700, 12345, np.uint64)])
    counts = rng.integers(1, 300, keys.size).astype(np.uint32)
    _lib.check(v._L.psg_freq_insert(v._h, 1, keys.ctypes.data, counts.ctypes.data, keys.size))
    O.cm_insert(t, nn, kk, keys, counts)
    assert np.array_equal(_table(v, 1, nn), t)
    v.close()


@pytest.mark.gpu
def test_gpu_freq_filter_inserts_on_two_streams_in_call_order():
    """Binned inserts share the filter's record scratch and write table dwords
    with plain stores: an insert on a caller stream, then inserts on the
    context stream and on a second caller stream, issued back to back with no
    host wait, must land exactly as sequential calls (the reference's
    insertKeys calls are sequential, frequency_filter.h:37-43)."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(9)
    v = _ctx()
    n = 1 << 22
    _lib.check(v._L.psg_freq_resize(v._h, 4, n, 4))
    t, nn, kk = O.cm_resize(n, 4)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    batches = []
    for b in range(3):
        keys = np.unique(zipf_keys(rng, 300_000))
        counts = rng.integers(1, 400, keys.size).astype(np.uint32)
        batches.append((keys, counts))
    dev = [(torch.from_numpy(k.view(np.int64)).cuda(), torch.from_numpy(c.view(np.int32)).cuda())
           for k, c in batches]
    torch.cuda.synchronize()
    k0, c0 = dev[0]
    _lib.check(v._L.psg_freq_insert_dev(v._h, 4, k0.data_ptr(), c0.data_ptr(), batches[0][0].size,
                                        C.c_void_p(s1.cuda_stream)))
    _lib.check(v._L.psg_freq_insert(v._h, 4, batches[1][0].ctypes.data, batches[1][1].ctypes.data,
                                    batches[1][0].size))
    k2, c2 = dev[2]
    _lib.check(v._L.psg_freq_insert_dev(v._h, 4, k2.data_ptr(), c2.data_ptr(), batches[2][0].size,
                                        C.c_void_p(s2.cuda_stream)))
    for keys, counts in batches:
        O.cm_insert(t, nn, kk, keys, counts)
    assert np.array_equal(_table(v, 4, nn), t)
    v.close()


@pytest.mark.gpu
def test_gpu_freq_filter_resize_then_insert_on_side_stream():
    """psg_freq_resize clears the table on the context stream; an insert on a
    caller stream enqueued right after it (no host wait) must see the cleared
    table (the clear joins the filter's call order).  A second
    resize of an already filled filter, then an insert on the same side
    stream, must also start from zero."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(19)
    v = _ctx()
    n = 1 << 22
    s1 = torch.cuda.Stream()
    for rep in range(2):  # a new filter, then a resize of a filled one
        keys = np.unique(zipf_keys(rng, 400_000))
        counts = rng.integers(1, 300, keys.size).astype(np.uint32)
        dk = torch.from_numpy(keys.view(np.int64)).cuda()
        dc = torch.from_numpy(counts.view(np.int32)).cuda()
        torch.cuda.synchronize()
        _lib.check(v._L.psg_freq_resize(v._h, 6, n, 3))
        _lib.check(v._L.psg_freq_insert_dev(v._h, 6, dk.data_ptr(), dc.data_ptr(), keys.size,
                                            C.c_void_p(s1.cuda_stream)))
        t, nn, kk = O.cm_resize(n, 3)
        O.cm_insert(t, nn, kk, keys, counts)
        assert np.array_equal(_table(v, 6, nn), t)
    v.close()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("k,nq", [(1, 400_000), (3, 1_000_003), (4, 2_000_000), (5, 700_001),
                                  (8, 9_000_000)])
def test_gpu_freq_query_binned_vs_oracle(k, nq):
    """queryKeys (frequency_filter.h:27-34, countmin.h:42-51) through the
    binned query (probes moved to 128 KB table regions, the region read once
    into LDS, results binned back per key block): kept keys, in input order,
    exact against the oracle for k = 1..8, table sizes with a partial last
    region, thresholds around the table's counts, repeated and unsorted
    query keys, and at k = 8 / 9 M keys two chunks of the key stream (the
    scratch holds 8 M keys' records at k = 8).  The device entry point runs
    the same form with caller scratch."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(100 + k)
    v = _ctx()
    n = 3_000_017 if k != 8 else (1 << 24) + 12
    _lib.check(v._L.psg_freq_resize(v._h, 5, n, k))
    t, nn, kk = O.cm_resize(n, k)
    keys = np.unique(zipf_keys(rng, 600_000))
    counts = rng.integers(1, 40, keys.size).astype(np.uint32)
    _lib.check(v._L.psg_freq_insert(v._h, 5, keys.ctypes.data, counts.ctypes.data, keys.size))
    O.cm_insert(t, nn, kk, keys, counts)
    q = np.concatenate([zipf_keys(rng, nq - 1000), keys[:1000]])
    for freq in (0, 3, 20):
        assert np.array_equal(_query(v, 5, q, freq), O.ff_query(t, nn, kk, q, freq)), freq
    if k == 4:
        m = 500_000
        dq = torch.from_numpy(q[:m].view(np.int64)).cuda()
        sb = v._L.psg_freq_query_scratch_bytes(m)
        scratch = torch.empty(sb, dtype=torch.uint8, device="cuda")
        dout = torch.empty(m, dtype=torch.int64, device="cuda")
        dn = torch.zeros(1, dtype=torch.int64, device="cuda")
        _lib.check(v._L.psg_freq_query_dev(v._h, 5, dq.data_ptr(), m, 3, dout.data_ptr(),
                                           dn.data_ptr(), scratch.data_ptr(), None))
        got = dout[:int(dn.item())].cpu().numpy().view(np.uint64)
        assert np.array_equal(got, O.ff_query(t, nn, kk, q[:m], 3))
    v.close()
