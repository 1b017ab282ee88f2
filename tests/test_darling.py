"""Fused server update: Darling::updateWeight
(src/linear_method/darling.cc:437-477) on the resident (G, U) aggregate.

The oracle (oracle/psg_oracle.c orc_darling_update_weight) is a line-by-line
restatement, PARITY UNPINNED: the reference ships no test of updateWeight
and darling.cc cannot be built here (protobuf/glog/Eigen), so it is checked
against an independent pure-Python restatement and hand-derived cases.  The
GPU path is compared with the oracle bit for bit, NaN sentinel included
(kInactiveValue_ = all-ones bits, darling.cc:13-15).
"""
import math
import struct

import numpy as np
import pytest

import oracle_py as O

NAN1 = struct.unpack("<d", b"\xff" * 8)[0]


def py_update_weight(value, delta, active, lo, G, U, eta, lam, kkt, dmax, violation=0.0):
    """Independent restatement of darling.cc:437-477 (Python floats are IEEE
    doubles; std::min/std::max written as their definitions)."""
    value, delta, active = list(value), list(delta), list(active)
    smin = lambda a, b: b if b < a else a  # noqa: E731
    smax = lambda a, b: b if a < b else a  # noqa: E731
    for i in range(len(G)):
        k = i + lo
        if not active[k]:
            continue
        g, u = G[i], U[i] / eta + 1e-10
        gp, gn = g + lam, g - lam
        w = value[k]
        d, vio = -w, 0.0
        if w == 0:
            if gp < 0:
                vio = -gp
            elif gn > 0:
                vio = gn
            elif gp > kkt and gn < -kkt:
                active[k] = 0
                value[k] = NAN1
                continue
        violation = smax(violation, vio)
        if gp <= u * w:
            d = -gp / u
        elif gn >= u * w:
            d = -gn / u
        d = smin(delta[k], smax(-delta[k], d))
        delta[k] = smin(dmax, 2 * math.fabs(d) + .1)
        value[k] = w + d
    return value, delta, active, violation


def bits64(a):
    return np.asarray(a, np.float64).view(np.uint64)


def darling_case(seed, n=3000, lo=100, m=1500):
    rng = np.random.default_rng(seed)
    value = rng.standard_normal(n) * (rng.random(n) < 0.5)  # half exactly zero
    value[::17] = -0.0
    delta = rng.random(n) * 2 + 0.05
    active = (rng.random(n) < 0.9).astype(np.uint8)
    G = rng.standard_normal(m) * 2
    U = rng.random(m) * 3
    U[::31] = 0.0
    G[::53] = 1e-3  # inside [-lambda, lambda]: the KKT filter branch
    return value, delta, active, lo, G, U


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_darling_oracle_vs_python_restatement(seed):
    value, delta, active, lo, G, U = darling_case(seed)
    for kkt in (1e20, 0.0):
        a = O.darling_update_weight(value, delta, active, lo, G, U, 0.7, 0.5, kkt, 3.0, 0.25)
        b = py_update_weight(value, delta, active, lo, G, U, 0.7, 0.5, kkt, 3.0, 0.25)
        assert np.array_equal(bits64(a[0]), bits64(b[0]))
        assert np.array_equal(bits64(a[1]), bits64(b[1]))
        assert np.array_equal(a[2], np.asarray(b[2], np.uint8))
        assert a[3] == b[3]


def test_darling_hand_cases():
    """w = 0 with g_pos < 0 (violation -g_pos, step -g_pos/u clipped to
    delta); w = 0 inside the KKT band (deactivated, all-ones NaN); an
    inactive position untouched."""
    value = np.array([0.0, 0.0, 1.0])
    delta = np.array([0.5, 0.5, 0.5])
    active = np.array([1, 1, 0], np.uint8)
    G = np.array([-2.0, 0.1, 5.0])
    U = np.array([1.0, 1.0, 1.0])
    v, d, a, vio = O.darling_update_weight(value, delta, active, 0, G, U, 1.0, 1.0, 0.5, 10.0)
    # k=0: g_pos = -1 < 0: vio 1, d = 1/(1+1e-10) clipped to 0.5, delta = 2*.5+.1
    assert vio == 1.0 and v[0] == 0.5 and d[0] == 1.1 and a[0] == 1
    # k=1: g_pos = 1.1 > .5, g_neg = -0.9 < -.5: deactivated
    assert a[1] == 0 and bits64(v[1:2])[0] == np.uint64(0xFFFFFFFFFFFFFFFF) and d[1] == 0.5
    assert v[2] == 1.0 and d[2] == 0.5 and a[2] == 0


# ------------------------------------------------------------------ GPU --
def _ctx():
    from parameter_server_amd.kv_vector import KVVector
    from parameter_server_amd._lib import PSG_F64
    return KVVector(0, PSG_F64)


def _msg(keys, vals=None, t=0, rng=(0, (1 << 64) - 1), ch=0):
    from parameter_server_amd.kv_vector import Message
    return Message(time=t, key_channel=ch, key_range=rng, key=np.asarray(keys, np.uint64),
                   value=[] if vals is None else [np.asarray(v, np.float64) for v in vals])


def darling_call(v, ch, t, eta, lam, kkt, dmax):
    import ctypes as C
    from parameter_server_amd import _lib
    P = (C.c_double * 4)(eta, lam, kkt, dmax)
    vio = C.c_double(-1.0)
    rc = v._L.psg_darling_update(v._h, ch, t, C.cast(P, C.c_void_p), C.byref(vio))
    return rc, vio.value


def darling_state(v, ch, n):
    import ctypes as C
    from parameter_server_amd import _lib
    delta = np.empty(n, np.float64)
    act = np.empty(n, np.uint8)
    nnz = C.c_size_t()
    _lib.check(v._L.psg_darling_state(v._h, ch, 0, n, delta.ctypes.data, act.ctypes.data,
                                      C.byref(nnz)))
    return delta, act, nnz.value


@pytest.mark.gpu
def test_gpu_darling_rcv1_shape_blocks():
    """rcv1 shape (cfg1): 47,236 server keys, feature blocks of ~4k keys,
    2 workers push (G, U) (m = 2, f64) for about 150-key pieces of each
    block; the fused update over several blocks and iterations, with the
    KKT filter on for the last iteration; w / delta / active / violation
    bit-exact against the oracle, then the workers' pull (gather) of w with
    the NaN sentinel's bits."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(47)
    D = np.unique(rng.integers(1, 1 << 48, 47236 + 64, dtype=np.uint64))[:47236]
    n = D.size
    v = _ctx()
    v.setValue(_msg(D, t=0))
    w = np.zeros(n)
    v.set_value_array(0, w)
    delta0 = 1.0
    _lib.check(v._L.psg_darling_init(v._h, 0, delta0))
    delta = np.full(n, delta0)
    active = np.ones(n, np.uint8)
    bounds = np.linspace(0, n, 12).astype(int)
    t = 10
    for it in range(3):
        kkt = 1e20 if it < 2 else 0.05
        for b in range(len(bounds) - 1):
            lo, hi = int(bounds[b]), int(bounds[b + 1])
            kb, ke = int(D[lo]), int(D[hi]) if hi < n else (1 << 64) - 1
            pushes = []
            for wk in range(2):
                pos = np.sort(rng.choice(np.arange(lo, hi), 150, replace=False))
                g = rng.standard_normal(pos.size) * (0.3 + it)
                u = rng.random(pos.size) * 2
                pushes.append((D[pos], [g, u]))
                v.setValue(_msg(D[pos], [g, u], t=t, rng=(kb, ke)))
            rc, lo2, hi2, (G, U), _ = O.aggregate(D, kb, ke, pushes, dtype=np.float64)
            assert rc == 0 and (lo2, hi2) == (lo, hi)
            rc, vio = darling_call(v, 0, t, 0.8, 0.1, kkt, 5.0)
            _lib.check(rc)
            w, delta, active, vio_o = O.darling_update_weight(w, delta, active, lo, G, U, 0.8,
                                                              0.1, kkt, 5.0, 0.0)
            assert vio == vio_o
            t += 3
    got_w = v.value(0)
    got_d, got_a, nnz = darling_state(v, 0, n)
    assert np.array_equal(bits64(got_w), bits64(w))
    assert np.array_equal(bits64(got_d), bits64(delta))
    assert np.array_equal(got_a, active)
    assert nnz == int(active.sum()) and nnz < n  # the KKT filter deactivated some
    # the pull of the updated model (darling.cc:224-229): NaN sentinels bit-exact
    req = np.sort(rng.choice(D, 3000, replace=False))
    from parameter_server_amd.kv_vector import Message
    m = Message(key=req)
    v.getValue(m)
    want, _ = O.gather(D, w, req, dtype=np.float64)
    assert np.array_equal(bits64(m.value[0]), bits64(want))
    assert np.any(bits64(m.value[0]) == np.uint64(0xFFFFFFFFFFFFFFFF))
    # kkt_filter_reset: every position active again
    _lib.check(v._L.psg_darling_reset_active(v._h, 0))
    assert darling_state(v, 0, n)[2] == n
    v.close()


@pytest.mark.gpu
def test_gpu_darling_unmatched_leaves_model():
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(3)
    D = np.unique(rng.integers(1, 1 << 40, 5000, dtype=np.uint64))
    v = _ctx()
    v.setValue(_msg(D))
    w0 = rng.standard_normal(D.size)
    v.set_value_array(0, w0)
    _lib.check(v._L.psg_darling_init(v._h, 0, 0.5))
    bad = np.sort(np.concatenate([D[:100], [np.uint64((1 << 41) + 5)]]))  # one key not a server key
    g = rng.standard_normal(bad.size)
    v.setValue(_msg(bad, [g, np.abs(g)], t=4))
    rc, _ = darling_call(v, 0, 4, 1.0, 0.1, 1e20, 5.0)
    assert rc == _lib.PSG_ERR_UNMATCHED
    assert np.array_equal(bits64(v.value(0)), bits64(w0))
    d, a, nnz = darling_state(v, 0, D.size)
    assert np.all(d == 0.5) and nnz == D.size
    # a block with one aggregate (m = 1) is not a Darling block
    v.setValue(_msg(D[:10], [np.ones(10)], t=5))
    rc, _ = darling_call(v, 0, 5, 1.0, 0.1, 1e20, 5.0)
    assert rc == _lib.PSG_ERR_ARG
    v.close()


@pytest.mark.gpu
def test_gpu_darling_large_block_grid_stride():
    """One feature block of ~1.2 M positions (more than the 2,048 workgroups
    x 256 positions one pass of the launch covers, so every workgroup loops),
    starting at an unaligned bitmap word: two iterations, the second with the
    KKT filter on; w / delta / active / violation bit-exact against the
    oracle (the violation is one max over every workgroup's)."""
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import _lib
    rng = np.random.default_rng(1202)
    n = 1_300_000
    D = np.unique(rng.integers(1, 1 << 50, n + 4096, dtype=np.uint64))[:n]
    v = _ctx()
    v.setValue(_msg(D, t=0))
    w = np.zeros(n)
    v.set_value_array(0, w)
    _lib.check(v._L.psg_darling_init(v._h, 0, 1.0))
    delta = np.full(n, 1.0)
    active = np.ones(n, np.uint8)
    lo, hi = 1007, n - 5
    kb, ke = int(D[lo]), int(D[hi])
    t = 3
    for it in range(2):
        kkt = 1e20 if it == 0 else 0.05
        pushes = []
        for wk in range(2):
            pos = np.sort(rng.choice(np.arange(lo, hi), (hi - lo) * 3 // 4, replace=False))
            g = rng.standard_normal(pos.size) * (0.3 + it)
            u = rng.random(pos.size) * 2
            pushes.append((D[pos], [g, u]))
            v.setValue(_msg(D[pos], [g, u], t=t, rng=(kb, ke)))
        rc, lo2, hi2, (G, U), _ = O.aggregate(D, kb, ke, pushes, dtype=np.float64)
        assert rc == 0 and (lo2, hi2) == (lo, hi)
        rc, vio = darling_call(v, 0, t, 0.8, 0.1, kkt, 5.0)
        _lib.check(rc)
        w, delta, active, vio_o = O.darling_update_weight(w, delta, active, lo, G, U, 0.8,
                                                          0.1, kkt, 5.0, 0.0)
        assert vio == vio_o and vio > 0
        t += 1
    got_d, got_a, nnz = darling_state(v, 0, n)
    assert np.array_equal(bits64(v.value(0)), bits64(w))
    assert np.array_equal(bits64(got_d), bits64(delta))
    assert np.array_equal(got_a, active)
    assert nnz == int(active.sum()) and nnz < n
    v.close()
