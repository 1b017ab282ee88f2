"""CPU: pin the oracle (oracle/psg_oracle.c) to the reference's known answers
and to an independent pure-Python restatement on small random cases."""
import json
import os
import struct

import numpy as np
import pytest

import oracle_py as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
ALL = (0, (1 << 64) - 1)


def test_shared_array_known_answers():
    sa = GOLD["shared_array_test"]
    i = sa["intersection"]
    assert O.set_intersection(i["a"], i["b"]).tolist() == i["c"]
    assert O.set_intersection(i["b"], i["a"]).tolist() == i["c"]
    assert O.set_intersection(i["a"], []).tolist() == []
    u = sa["union"]
    assert O.set_union(u["a"], u["b"]).tolist() == u["c"]
    assert O.set_union(u["b"], u["a"]).tolist() == u["c"]
    assert O.set_union(u["a"], []).tolist() == u["a"]
    assert O.set_union([], u["a"]).tolist() == u["a"]
    r = sa["range"]
    lo, hi = O.find_range(r["a"], *r["bound"])
    assert r["a"][lo:hi] == r["segment"]


@pytest.mark.parametrize("parallel", [0, 1])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_appendix_c_aggregate(parallel, dtype):
    g = GOLD["aggregate"]
    pushes = [(p["keys"], [p["vals"]]) for p in g["pushes"]]
    rc, lo, hi, outs, matched = O.aggregate(g["D"], *ALL, pushes, parallel, 3, dtype)
    assert rc == 0 and [lo, hi] == g["positions"]
    assert matched.tolist() == g["matched"]
    assert outs[0].tolist() == g["A"]


def test_appendix_c_subrange_and_gather():
    g = GOLD["aggregate_subrange"]
    pushes = [(p["keys"], [p["vals"]]) for p in g["pushes"]]
    rc, lo, hi, outs, _ = O.aggregate(g["D"], *g["key_range"], pushes)
    assert [lo, hi] == g["positions"] and outs[0].tolist() == g["A"]
    g = GOLD["gather"]
    out, mt = O.gather(g["D"], g["W"], g["R"])
    assert mt == g["matched"] and out.tolist() == g["out"]


@pytest.mark.parametrize("n", ["2", "4", "8"])
def test_shard_boundaries(n):
    want = [int(x) for x in GOLD["shards"][n]]
    k = int(n)
    got = [O.even_divide(*ALL, k, i)[0] for i in range(k)] + [O.even_divide(*ALL, k, k - 1)[1]]
    assert got == want


def test_murmur_shuffle_known_and_reference():
    s = GOLD["shuffle"]
    got = O.shuffle_keys(s["ids"])
    assert [int(x) for x in got] == [int(x) for x in s["keys"]]
    if O.ref_murmur_available():
        ids = np.arange(0, 2000, 7, dtype=np.uint64)
        assert np.array_equal(O.shuffle_keys(ids), O.ref_shuffle_keys(ids))
    # the product's numpy generator restates the same hash
    from parameter_server_amd import synth
    ids = np.random.default_rng(0).integers(0, 10 ** 9, 5000, dtype=np.uint64)
    assert np.array_equal(synth.murmur_shuffle(ids), O.shuffle_keys(ids))


def test_slice_key_ordered():
    keys = np.array([1, 5, 9, 20, 33, 40], np.uint64)
    sep = np.array([0, 6, 21, 100], np.uint64)
    pos, valid = O.slice_key_ordered(keys, 0, 100, sep)
    assert pos.tolist() == [0, 2, 4, 6] and valid.tolist() == [1, 1, 1]
    pos, valid = O.slice_key_ordered(keys, 7, 30, sep)
    assert pos.tolist() == [2, 2, 4, 4] and valid.tolist() == [0, 1, 1]


# ---------------------------------------------------------------------------
# independent restatement: a dict fold in push order (SURVEY 8a contract)
# ---------------------------------------------------------------------------
def py_aggregate(D, kb, ke, pushes, parallel, dtype):
    D = [int(x) for x in D]
    lo = sum(1 for x in D if x < kb)
    hi = sum(1 for x in D if x < ke)
    pos = {k: i - lo for i, k in enumerate(D[lo:hi], start=lo)}
    cast = np.float32 if dtype == np.float32 else np.float64
    m = len(pushes[0][1])
    outs = [[cast(0.0)] * (hi - lo) for _ in range(m)]
    matched = []
    first = True
    for keys, vals in pushes:
        keys = [int(k) for k in keys]
        if not keys:
            matched.append(0)
            continue
        mt = 0
        seen = {}
        last = -1
        for idx, k in enumerate(keys):  # merge walk: strictly increasing keys only
            if k in pos and k > last:
                seen[pos[k]] = idx
                mt += 1
                last = k
        matched.append(mt)
        for i in range(m):
            o = outs[i]
            for j in range(hi - lo):
                v = cast(vals[i][seen[j]]) if j in seen else None
                if first:
                    o[j] = v if v is not None else cast(0.0)
                elif v is not None:
                    o[j] = cast(o[j] + v)
                elif not parallel:
                    o[j] = cast(o[j] + cast(0.0))
        first = False
    return lo, hi, [np.array(o, dtype) for o in outs], matched


def _bits(a):
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("parallel", [0, 1])
def test_oracle_vs_python_restatement(seed, parallel):
    rng = np.random.default_rng(seed)
    dtype = np.float32 if seed % 2 == 0 else np.float64
    D = np.unique(rng.integers(0, 500, 120).astype(np.uint64))
    pushes = []
    for p in range(5):
        k = np.sort(rng.choice(D, rng.integers(0, 40), replace=False))
        v = rng.standard_normal(k.size).astype(dtype)
        v[rng.random(k.size) < 0.2] = -0.0  # exercise the sign of zero
        pushes.append((k, [v, -v]))
    kb, ke = (int(D[5]), int(D[-3])) if seed % 3 == 0 else ALL
    pushes = [(k[(k >= kb) & (k < ke)], [v[(k >= kb) & (k < ke)] for v in vs]) for k, vs in pushes]
    rc, lo, hi, outs, matched = O.aggregate(D, kb, ke, pushes, parallel, 2, dtype)
    plo, phi, pouts, pm = py_aggregate(D, kb, ke, pushes, parallel, dtype)
    assert rc == 0 and (lo, hi) == (plo, phi)
    assert matched.tolist() == pm
    for a, b in zip(outs, pouts):
        assert np.array_equal(_bits(a), _bits(b))


def test_serial_parallel_differ_only_in_zero_sign():
    D = np.array([1, 2, 3], np.uint64)
    pushes = [([1, 2], [np.array([-0.0, 1.0], np.float32)]),
              ([2], [np.array([1.0], np.float32)])]
    _, _, _, s, _ = O.aggregate(D, *ALL, pushes, parallel=0)
    _, _, _, p, _ = O.aggregate(D, *ALL, pushes, parallel=1)
    assert struct.pack("<f", s[0][0]) == struct.pack("<f", 0.0)   # -0 + +0 = +0
    assert struct.pack("<f", p[0][0]) == struct.pack("<f", -0.0)  # untouched
    assert s[0][1:].tolist() == p[0][1:].tolist() == [2.0, 0.0]


def test_unmatched_and_duplicates_are_counted():
    D = np.array([10, 20, 30], np.uint64)
    for keys in ([10, 25], [20, 20], [30, 10]):
        _, _, _, _, m = O.aggregate(D, *ALL, [(keys, [np.ones(2, np.float32)])])
        assert m[0] < 2
    rc, *_ = O.aggregate([], *ALL, [([1], [np.ones(1, np.float32)])])
    assert rc == -1


@pytest.mark.parametrize("seed", range(6))
def test_scatter_serial_form_equals_serial_fold(seed):
    """orc_aggregate_scatter_serial (serialSetValue with ONE trailing +0.0
    where a non-empty push lacked the key; the whole-cfg5 serial GPU check)
    equals the dense oldMatch fold (orc_aggregate, serial) bit for bit:
    -0.0 and signalling / quiet NaN payloads, empty pushes (the first one
    too), keys absent from D, sub-ranges, f32 and f64, m = 1..2."""
    rng = np.random.default_rng(300 + seed)
    dtype = np.float32 if seed % 2 == 0 else np.float64
    ity = np.uint32 if dtype == np.float32 else np.uint64
    snan = ity(0x7F800001) if dtype == np.float32 else ity(0x7FF0000000000001)
    m = 1 + seed % 2
    D = np.unique(rng.integers(0, 1 << 40, 2000, dtype=np.uint64))
    pushes = []
    for p in range(6):
        cnt = 0 if p == (seed % 3) * 2 else int(rng.integers(1, 1500))
        k = np.unique(np.concatenate([rng.choice(D, cnt, replace=False),
                                      rng.integers(0, 1 << 40, 10 if cnt else 0,
                                                   dtype=np.uint64)]))
        vs = []
        for _ in range(m):
            v = rng.standard_normal(k.size).astype(dtype)
            v[rng.random(k.size) < 0.2] = -0.0
            bits = v.view(ity)
            bits[rng.random(k.size) < 0.02] = snan
            v[rng.random(k.size) < 0.02] = np.nan
            vs.append(v)
        pushes.append((k, vs))
    for kb, ke in [(0, (1 << 64) - 1), (int(D[50]), int(D[1700]))]:
        a = O.aggregate(D, kb, ke, pushes, False, 1, dtype)
        b = O.aggregate_scatter(D, kb, ke, pushes, dtype, parallel=False)
        assert a[0] == b[0] == 0 and a[1:3] == b[1:3]
        assert np.array_equal(a[4], b[4])
        for x, y in zip(a[3], b[3]):
            assert x.tobytes() == y.tobytes()


def test_scatter_serial_form_rejects_unsorted_push():
    D = np.arange(10, dtype=np.uint64)
    pushes = [(np.array([1, 3, 2], np.uint64), [np.ones(3, np.float32)])]
    assert O.aggregate_scatter(D, 0, (1 << 64) - 1, pushes, parallel=False)[0] == -3


def test_gather_repeated_request_reads_zero():
    out, mt = O.gather([5, 7], [1.0, 2.0], [5, 5, 7])
    assert out.tolist() == [1.0, 0.0, 2.0] and mt == 2


@pytest.mark.parametrize("seed", range(4))
def test_scatter_form_equals_parallel_merge_walk(seed):
    """orc_aggregate_scatter (the O(sum n log U) parallelSetValue used for
    the whole-cfg5 GPU check) equals the merge-walk restatement of match()
    bit for bit: sub-ranges, keys outside the range or absent from D,
    repeated keys, -0.0, empty pushes, f32 and f64, m = 1..2."""
    rng = np.random.default_rng(100 + seed)
    dtype = np.float32 if seed % 2 == 0 else np.float64
    m = 1 + seed % 2
    D = np.unique(rng.integers(0, 1 << 40, 3000, dtype=np.uint64))
    pushes = []
    for p in range(7):
        k = np.sort(np.concatenate([rng.choice(D, int(rng.integers(0, 900)), replace=False),
                                    rng.integers(0, 1 << 40, 20, dtype=np.uint64)]))
        if p == 3 and k.size > 10:
            k[5] = k[4]  # a repeated key
        vs = [rng.standard_normal(k.size).astype(dtype) for _ in range(m)]
        for v in vs:
            v[rng.random(k.size) < 0.1] = -0.0
        pushes.append((k, vs))
    for kb, ke in [(0, (1 << 64) - 1), (int(D[100]), int(D[2500]))]:
        a = O.aggregate(D, kb, ke, pushes, True, 3, dtype)
        b = O.aggregate_scatter(D, kb, ke, pushes, dtype)
        assert a[0] == b[0] == 0 and a[1:3] == b[1:3]
        assert np.array_equal(a[4], b[4])
        for x, y in zip(a[3], b[3]):
            assert x.tobytes() == y.tobytes()
