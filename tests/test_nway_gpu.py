"""N-way merge of sorted pushes (psg_nway_*) against the
oracle: the merged key set equals the reference's setUnion applied push
after push (shared_array_inl.h:155-162), and the sums equal the oracle's
serialSetValue / parallelSetValue over that key set (kv_vector.h:84-204),
bit for bit, NaN payloads included where one push carries the NaN."""
import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu

ALL = (0, (1 << 64) - 1)


def _run(pushes, dtype=np.float32, m=1, parallel=False):
    import torch
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    from parameter_server_amd.kv_vector import NWayMerge
    dev = torch.device("cuda", 0)
    tdt = torch.float32 if dtype == np.float32 else torch.float64
    dk = [torch.from_numpy(np.ascontiguousarray(k).view(np.int64)).to(dev) for k, _ in pushes]
    dv = [[torch.from_numpy(np.ascontiguousarray(v, dtype)).to(dev) for v in vs[:m]]
          for _, vs in pushes]
    tot = max(1, sum(k.size for k, _ in pushes))
    ok = torch.full((tot,), -1, dtype=torch.int64, device=dev)
    ov = [torch.empty(tot, dtype=tdt, device=dev) for _ in range(m)]
    u = NWayMerge(0, PSG_F32 if dtype == np.float32 else PSG_F64,
                  [t.data_ptr() for t in dk], [k.size for k, _ in pushes],
                  [[t.data_ptr() for t in vs] for vs in dv], ok.data_ptr(),
                  [t.data_ptr() for t in ov], parallel)
    outs = []
    for _ in range(2):  # a second run lands in the same buffers
        u.run()
        n = u.result()
        outs.append((ok.cpu().numpy()[:n].view(np.uint64).copy(),
                     [t.cpu().numpy()[:n].copy() for t in ov]))
    u.close()
    assert outs[0][0].tobytes() == outs[1][0].tobytes()
    return outs[1]


def _union(pushes):
    D = np.zeros(0, np.uint64)
    for k, _ in pushes:
        D = O.set_union(D, k)
    return D


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def _check(pushes, dtype=np.float32, m=1, parallel=False):
    keys, vals = _run(pushes, dtype, m, parallel)
    D = _union(pushes)
    assert np.array_equal(keys, D)
    if m and D.size:
        # Range::all() = [0, 2^64 - 1) (range.h:75-78): a key 2^64 - 1 is in
        # the union but outside the oracle's aligned range; compare [lo, hi)
        rc, lo, hi, want, _ = O.aggregate(D, *ALL, [(k, vs[:m]) for k, vs in pushes],
                                          parallel, 1, dtype)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(_bits(vals[i][lo:hi]), _bits(np.asarray(want[i], dtype)))


@pytest.mark.parametrize("parallel", [False, True])
def test_nway_cfg2_union_and_sums(parallel):
    """cfg2's 8 pushes x 131,072 keys (10 % shared): union = U = 956,827."""
    from parameter_server_amd import synth
    D, pushes = synth.overlap_pushes(1)
    keys, vals = _run(pushes, parallel=parallel)
    assert keys.size == D.size == 956827 and np.array_equal(keys, D)
    rc, _, _, want, _ = O.aggregate(D, *ALL, pushes, parallel, 1, np.float32)
    assert np.array_equal(_bits(vals[0]), _bits(want[0]))


def test_nway_keys_only_union():
    from parameter_server_amd import synth
    _, pushes = synth.uniform_pushes(seed=7, npush=12, n=30000, union=False)
    keys, _ = _run(pushes, m=0)
    assert np.array_equal(keys, _union(pushes))


@pytest.mark.parametrize("dtype,m", [(np.float64, 2), (np.float32, 3), (np.float64, 4)])
@pytest.mark.parametrize("parallel", [False, True])
def test_nway_value_types(dtype, m, parallel):
    rng = np.random.default_rng(5 + m)
    base = np.unique(rng.integers(0, 1 << 63, 60000, dtype=np.uint64))
    pushes = []
    for p in range(9):
        k = np.sort(rng.choice(base, int(rng.integers(1, 20000)), replace=False))
        vs = [rng.standard_normal(k.size).astype(dtype) for _ in range(m)]
        for v in vs:
            v[rng.random(k.size) < 0.05] = -0.0
        pushes.append((k, vs))
    _check(pushes, dtype, m, parallel)


def test_nway_edge_shapes():
    """Empty pushes (ignored: the first non-empty one assigns), one push,
    64 pushes, every push the same keys, keys 0 and 2^64 - 1, and a
    clustered distribution (most keys in a narrow range) that would
    overflow an interpolation bucketing."""
    rng = np.random.default_rng(9)
    e = (np.zeros(0, np.uint64), [np.zeros(0, np.float32)])
    one = np.sort(rng.choice(1 << 40, 5000, replace=False).astype(np.uint64))
    v = lambda n: [rng.standard_normal(n).astype(np.float32)]  # noqa: E731
    _check([e, (one, v(one.size)), e])
    _check([(one, v(one.size))])
    many = [(np.sort(rng.choice(1 << 20, int(rng.integers(1, 3000)), replace=False)
                     ).astype(np.uint64), None) for _ in range(64)]
    _check([(k, v(k.size)) for k, _ in many])
    same = np.arange(7000, dtype=np.uint64) * np.uint64(3)
    _check([(same, v(same.size)) for _ in range(10)])
    edge = np.array([0, 1, (1 << 63), (1 << 64) - 2, (1 << 64) - 1], np.uint64)
    _check([(edge, v(5)), (edge[[0, 4]], v(2)), (edge[1:4], v(3))])
    clustered = np.unique(np.concatenate([
        np.arange(1 << 40, (1 << 40) + 50000, dtype=np.uint64),
        rng.integers(0, 1 << 63, 100, dtype=np.uint64)]))
    _check([(np.sort(rng.choice(clustered, 30000, replace=False)), v(30000)) for _ in range(5)])
    _check([(e[0], e[1])])  # all empty: nothing merged


def test_nway_nan_payloads():
    """A NaN carried by one push keeps its payload (quieted) through the
    run's fold, as the reference's IEEE adds give it."""
    k = np.arange(100, dtype=np.uint64)
    a = np.ones(100, np.float32)
    a.view(np.uint32)[::7] = 0x7fc12345
    a.view(np.uint32)[3::7] = 0x7f800001  # signalling: quieted by the add
    b = np.full(100, 0.5, np.float32)
    for parallel in (False, True):
        _check([(k, [a]), (k[::2], [b[::2]])], parallel=parallel)
        _check([(k[::3], [b[::3]]), (k, [a])], parallel=parallel)


def test_nway_unsorted_push_is_reported():
    from parameter_server_amd._lib import PSGError, PSG_ERR_UNSORTED
    k = np.arange(10000, dtype=np.uint64) * np.uint64(2)
    bad = k.copy()
    bad[500], bad[501] = bad[501], bad[500]
    with pytest.raises(PSGError) as e:
        _run([(k, [np.ones(k.size, np.float32)]), (bad, [np.ones(k.size, np.float32)])])
    assert e.value.status == PSG_ERR_UNSORTED


def test_context_key_union_on_device():
    """The server's key-only pushes (kv_vector.h:177-182) go through the
    N-way merge: one at a time and batched (psg_key_union_batch) they give
    the oracle's successive setUnion; findRange, key copies and a value
    push afterwards read the refreshed host mirror; an unsorted key-only
    push is PSG_ERR_UNSORTED and leaves the key set unchanged."""
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSGError, PSG_ERR_UNSORTED
    from parameter_server_amd.kv_vector import KVVector, Message
    D, pushes = synth.overlap_pushes(3, npush=8, n=20000)
    keys = [k for k, _ in pushes]
    v1, v2 = KVVector(0), KVVector(0)
    for k in keys:
        v1.setValue(Message(key=k))
    v2.union_keys(0, keys[:3] + [np.zeros(0, np.uint64)] + keys[3:])
    want = _union(pushes)
    assert np.array_equal(v1.key(0), want) and np.array_equal(v2.key(0), want)
    assert v2.find(0, (int(want[100]), int(want[5000]))) == tuple(O.find_range(want, int(want[100]), int(want[5000])))
    # growing the key set again: more keys than the mirror held
    extra = np.unique(np.random.default_rng(4).integers(0, 1 << 63, 300000, dtype=np.uint64))
    v2.union_keys(0, [extra])
    want2 = O.set_union(want, extra)
    assert np.array_equal(v2.key(0), want2)
    # a value push matched against the new key set
    v2.setValue(Message(time=1, key=keys[0], value=[pushes[0][1][0]]))
    (rng, got), = v2.received(1)
    rc, lo, hi, w, _ = O.aggregate(want2, *ALL, [pushes[0]])
    assert rc == 0 and tuple(rng) == (lo, hi) and np.array_equal(_bits(got), _bits(w[0]))
    bad = keys[1].copy()
    bad[10], bad[11] = bad[11], bad[10]
    with pytest.raises(PSGError) as e:
        v2.setValue(Message(key=bad))
    assert e.value.status == PSG_ERR_UNSORTED
    assert np.array_equal(v2.key(0), want2)
    v1.close()
    v2.close()


def test_key_union_batch_fails_in_later_chunk():
    """A batched key union of more pushes than one N-way merge takes
    (psg_nway_max_push() - 1 besides the resident keys) whose bad push sits
    in the second chunk: the first chunk is applied, the error is
    PSG_ERR_UNSORTED, and since the key set changed the value array is
    cleared (kv_vector.h:180) -- no stale values stay attached to a new key
    set, even when the first chunk added no new key."""
    from parameter_server_amd._lib import PSGError, PSG_ERR_UNSORTED, lib
    from parameter_server_amd.kv_vector import KVVector, Message
    rng = np.random.default_rng(11)
    D = np.unique(rng.integers(0, 1 << 62, 50000, dtype=np.uint64))
    nmax = lib().psg_nway_max_push()
    npush = nmax + 6
    # every push a subset of D: the first chunk adds no new key
    pushes = [np.sort(rng.choice(D, 3000, replace=False)) for _ in range(npush)]
    bad_at = nmax + 2  # in the second chunk
    bad = pushes[bad_at].copy()
    bad[5], bad[6] = bad[6], bad[5]
    pushes[bad_at] = bad
    v = KVVector(0)
    v.setValue(Message(key=D))
    v.set_value_array(0, rng.standard_normal(D.size).astype(np.float32))
    assert v.value(0).size == D.size
    with pytest.raises(PSGError) as e:
        v.union_keys(0, pushes)
    assert e.value.status == PSG_ERR_UNSORTED
    assert np.array_equal(v.key(0), D)
    assert v.value(0).size == 0, "stale values survived a partially applied key union"
    # and with new keys in the first chunk: they are applied
    extra = np.unique(rng.integers(1 << 62, 1 << 63, 1000, dtype=np.uint64))
    pushes[0] = extra
    v.set_value_array(0, np.zeros(D.size, np.float32))
    with pytest.raises(PSGError):
        v.union_keys(0, pushes)
    assert np.array_equal(v.key(0), O.set_union(D, extra))
    assert v.value(0).size == 0
    v.close()


def test_nway_batch_of_merges_vs_oracle():
    """psg_nway_create_batch: independent merges as one pipeline (one
    launch per stage over all of them): cfg2-shaped merges of different
    sizes and push counts (8, 3, 64 pushes, one with an empty push, one of
    keys past 2^63), f64 m = 2, serial and parallel; every merge's union and
    sums bit-exact against the oracle, its count from psg_nway_result; an
    unsorted push in one merge of a batch is reported."""
    import torch
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_F64, PSGError, PSG_ERR_UNSORTED
    from parameter_server_amd.kv_vector import NWayMergeBatch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    cases = [synth.overlap_pushes(41, npush=8, n=40000, dtype=np.float64, m=2)[1],
             synth.overlap_pushes(42, npush=3, n=70000, overlap=0.5, dtype=np.float64, m=2)[1],
             synth.overlap_pushes(43, npush=64, n=3000, overlap=0.2, dtype=np.float64, m=2)[1]]
    hi = [(np.unique(rng.integers(1 << 63, (1 << 64) - 1, 20000, dtype=np.uint64)),) for _ in range(5)]
    cases.append([(k, [rng.standard_normal(k.size), rng.standard_normal(k.size)]) for (k,) in hi])
    cases[0][5] = (np.zeros(0, np.uint64), [np.zeros(0), np.zeros(0)])
    keep, merges = [], []
    for pushes in cases:
        dk = [torch.from_numpy(np.ascontiguousarray(k).view(np.int64)).to(dev) for k, _ in pushes]
        dv = [[torch.from_numpy(np.ascontiguousarray(v, np.float64)).to(dev) for v in vs]
              for _, vs in pushes]
        tot = max(1, sum(k.size for k, _ in pushes))
        ok = torch.full((tot,), -1, dtype=torch.int64, device=dev)
        ov = [torch.empty(tot, dtype=torch.float64, device=dev) for _ in range(2)]
        keep += [dk, dv, ok, ov]
        merges.append(dict(push_keys=[t.data_ptr() for t in dk], push_n=[k.size for k, _ in pushes],
                           push_vals=[[t.data_ptr() for t in vs] for vs in dv],
                           out_keys=ok.data_ptr(), out_vals=[t.data_ptr() for t in ov]))
    for parallel in (False, True):
        u = NWayMergeBatch(0, PSG_F64, merges, parallel)
        for _ in range(2):
            u.run()
            counts = u.result()
            for j, pushes in enumerate(cases):
                D = _union(pushes)
                assert counts[j] == D.size
                ok, ov = keep[4 * j + 2], keep[4 * j + 3]
                assert np.array_equal(ok.cpu().numpy()[: D.size].view(np.uint64), D)
                rc, lo, hi_, want, _ = O.aggregate(D, *ALL, pushes, parallel, 2, np.float64)
                assert rc == 0
                for i in range(2):
                    assert np.array_equal(_bits(ov[i].cpu().numpy()[lo:hi_]), _bits(want[i]))
        u.close()
    # one unsorted push in the second merge: reported by the batch's result
    bad = np.ascontiguousarray(cases[1][1][0].copy())
    bad[[10, 11]] = bad[[11, 10]]
    keep.append(torch.from_numpy(bad.view(np.int64)).to(dev))
    merges[1]["push_keys"][1] = keep[-1].data_ptr()
    u = NWayMergeBatch(0, PSG_F64, merges)
    u.run()
    with pytest.raises(PSGError) as e:
        u.result()
    assert e.value.status == PSG_ERR_UNSORTED
    u.close()


def test_nway_skewed_batch_vs_oracle():
    """A skewed batch (one cfg2-shaped merge of ~150 tiles and 40 one-tile
    merges of 1-3 short pushes): the tickets map one per tile instead of
    round-robin over the merges (maxT x nm would be ~40 x the
    tiles); unions and sums bit-exact against the oracle, both modes."""
    import torch
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_F32
    from parameter_server_amd.kv_vector import NWayMergeBatch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(23)
    cases = [synth.overlap_pushes(51, npush=8, n=40000)[1]]
    for j in range(40):
        ps = []
        for _ in range(int(rng.integers(1, 4))):
            k = np.unique(rng.integers(0, 1 << 40, int(rng.integers(1, 60)), dtype=np.uint64))
            ps.append((k, [rng.standard_normal(k.size).astype(np.float32)]))
        cases.append(ps)
    keep, merges = [], []
    for pushes in cases:
        dk = [torch.from_numpy(np.ascontiguousarray(k).view(np.int64)).to(dev) for k, _ in pushes]
        dv = [[torch.from_numpy(np.ascontiguousarray(v, np.float32)).to(dev) for v in vs[:1]]
              for _, vs in pushes]
        tot = max(1, sum(k.size for k, _ in pushes))
        ok = torch.full((tot,), -1, dtype=torch.int64, device=dev)
        ov = torch.empty(tot, dtype=torch.float32, device=dev)
        keep += [dk, dv, ok, ov]
        merges.append(dict(push_keys=[t.data_ptr() for t in dk], push_n=[k.size for k, _ in pushes],
                           push_vals=[[t.data_ptr() for t in vs] for vs in dv],
                           out_keys=ok.data_ptr(), out_vals=[ov.data_ptr()]))
    for parallel in (False, True):
        u = NWayMergeBatch(0, PSG_F32, merges, parallel)
        u.run()
        counts = u.result()
        for j, pushes in enumerate(cases):
            D = _union(pushes)
            assert counts[j] == D.size
            ok, ov = keep[4 * j + 2], keep[4 * j + 3]
            assert np.array_equal(ok.cpu().numpy()[: D.size].view(np.uint64), D)
            rc, lo, hi_, want, _ = O.aggregate(D, *ALL, [(k, vs[:1]) for k, vs in pushes],
                                               parallel, 1, np.float32)
            assert rc == 0
            assert np.array_equal(_bits(ov.cpu().numpy()[lo:hi_]), _bits(want[0]))
        u.close()
