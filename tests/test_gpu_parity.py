"""GPU parity: libpsg.so on an MI355X against the oracle (bit-exact).

Integer/key outputs and float sums are compared bit for bit (the kernels
fold in the reference's push order with IEEE adds, so the tolerance the
north star allows, 1e-6 relative, is not needed); NaN payloads are
compared bit for bit too (assert_bitexact).
"""
import json
import os

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
ALL = (0, (1 << 64) - 1)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    from parameter_server_amd import _lib
    _lib.lib()
    return torch


def kvv(dtype=np.float32, parallel=False, flags=0):
    from parameter_server_amd.kv_vector import KVVector
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    return KVVector(0, PSG_F32 if dtype == np.float32 else PSG_F64, parallel, flags)


def msg(keys, vals=None, t=0, ch=0, rng=ALL):
    from parameter_server_amd.kv_vector import Message
    return Message(time=t, key_channel=ch, key_range=rng,
                   key=np.asarray(keys, np.uint64),
                   value=[] if vals is None else [np.asarray(v) for v in vals])


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


def assert_bitexact(got, want):
    """Every bit, NaN payloads included (test_nan_payloads covers the one
    case where payloads may legitimately differ)."""
    got, want = np.asarray(got), np.asarray(want)
    assert got.shape == want.shape
    gn, wn = np.isnan(got), np.isnan(want)
    assert np.array_equal(gn, wn)
    assert np.array_equal(bits(got), bits(want))


def run_ctx(D, pushes, kb=0, ke=(1 << 64) - 1, dtype=np.float32, parallel=False, t=7,
            flags=0, flush=None):
    v = kvv(dtype, parallel, flags)
    if flush:
        v.set_flush_pushes(flush)
    v.setValue(msg(D))
    for k, vals in pushes:
        v.setValue(msg(k, [np.asarray(x, dtype) for x in vals], t=t, rng=(kb, ke)))
    out = v.received(t)
    v.close()
    return out


# ------------------------------------------------------------- known answers
@pytest.mark.parametrize("parallel", [False, True])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_appendix_c(torch_cuda, parallel, dtype):
    g = GOLD["aggregate"]
    out = run_ctx(g["D"], [(p["keys"], [p["vals"]]) for p in g["pushes"]],
                  dtype=dtype, parallel=parallel)
    (rng, a), = out
    assert list(rng) == g["positions"] and a.tolist() == g["A"]
    g = GOLD["aggregate_subrange"]
    out = run_ctx(g["D"], [(p["keys"], [p["vals"]]) for p in g["pushes"]],
                  *g["key_range"], dtype=dtype, parallel=parallel)
    assert list(out[0][0]) == g["positions"] and out[0][1].tolist() == g["A"]


def test_known_union_and_gather(torch_cuda):
    u = GOLD["shared_array_test"]["union"]
    v = kvv()
    v.setValue(msg(u["a"]))
    v.setValue(msg(u["b"]))
    assert v.key(0).tolist() == u["c"]
    v.setValue(msg([]))  # empty push is ignored
    assert v.key(0).tolist() == u["c"]
    g = GOLD["gather"]
    w = kvv()
    w.setValue(msg(g["D"]))
    w.set_value_array(0, g["W"])
    m = msg(g["R"])
    assert w.getValue(m) == g["matched"]
    assert m.value[0].tolist() == g["out"]
    r = msg([5, 5, 7, 8, 11, 12])
    w.getValue(r)
    assert r.value[0].tolist() == O.gather(g["D"], g["W"], [5, 5, 7, 8, 11, 12])[0].tolist()


# ---------------------------------------------------------- random vs oracle
def random_case(seed, dtype, m, npush, density, nD, special=True):
    rng = np.random.default_rng(seed)
    D = np.unique(rng.integers(0, 1 << 62, nD, dtype=np.uint64) * np.uint64(3))
    pushes = []
    for p in range(npush):
        k = np.sort(rng.choice(D, int(rng.binomial(D.size, density)), replace=False))
        vals = []
        for i in range(m):
            v = rng.standard_normal(k.size).astype(dtype)
            if special and k.size:
                sel = rng.random(k.size)
                v[sel < 0.05] = -0.0
                v[(sel >= 0.05) & (sel < 0.07)] = 0.0
                fin = np.finfo(dtype)
                v[(sel >= 0.07) & (sel < 0.08)] = fin.tiny * np.asarray(0.25, dtype)  # denormal
                v[(sel >= 0.08) & (sel < 0.081)] = np.nan
            vals.append(v)
        pushes.append((k, vals))
    return D, pushes


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("parallel", [False, True])
def test_random_vs_oracle(torch_cuda, seed, parallel):
    dtype = np.float32 if seed % 2 == 0 else np.float64
    m = 1 + seed % 3
    npush = [1, 2, 8, 13, 70, 3, 65, 9][seed]
    D, pushes = random_case(seed, dtype, m, npush, [0.3, 0.9, 0.05, 0.5, 0.02, 1.0, 0.01, 0.2][seed],
                            [5000, 3000, 20000, 4097, 9000, 2048, 12000, 1][seed])
    if seed in (2, 5):
        kb, ke = int(D[D.size // 5]), int(D[-(D.size // 7)])
    else:
        kb, ke = ALL
    pushes = [(k[(k >= kb) & (k < ke)], [v[(k >= kb) & (k < ke)] for v in vs]) for k, vs in pushes]
    pushes = [p for p in pushes if p[0].size]  # empty pushes are ignored by both
    if not pushes:
        pytest.skip("all pushes empty")
    out = run_ctx(D, pushes, kb, ke, dtype, parallel)
    rc, lo, hi, want, matched = O.aggregate(D, kb, ke, pushes, parallel, 1, dtype)
    assert rc == 0 and all(matched[i] == pushes[i][0].size for i in range(len(pushes)))
    assert len(out) == m
    for i in range(m):
        assert tuple(out[i][0]) == (lo, hi)
        assert_bitexact(out[i][1], want[i])


@pytest.mark.parametrize("per_launch", [7, 64, 4096])
def test_launch_seams(torch_cuda, per_launch):
    """600 pushes for one time split into launches of `per_launch` pushes
    (psg_set_flush_pushes), each continuing the aggregate (serial zero
    semantics across seams)."""
    D, pushes = random_case(11, np.float32, 1, 600, 0.02, 4000)
    pushes = [p for p in pushes if p[0].size]
    for parallel in (False, True):
        out = run_ctx(D, pushes, dtype=np.float32, parallel=parallel, flush=per_launch)
        _, lo, hi, want, _ = O.aggregate(D, *ALL, pushes, parallel, 1, np.float32)
        assert_bitexact(out[0][1], want[0])


def test_dense_and_crowded_tiles(torch_cuda):
    """Every push holds every key (dense fast path, 8 chunks per tile)."""
    D = np.arange(5000, dtype=np.uint64) * np.uint64(7)
    pushes = [(D, [np.random.default_rng(p).standard_normal(D.size).astype(np.float32)])
              for p in range(9)]
    out = run_ctx(D, pushes)
    _, _, _, want, _ = O.aggregate(D, *ALL, pushes)
    assert_bitexact(out[0][1], want[0])


@pytest.mark.parametrize("dtype,m", [(np.float64, 1), (np.float64, 2), (np.float32, 3),
                                     (np.float32, 4), (np.float64, 4)])
def test_packed_rounds_value_types(torch_cuda, dtype, m):
    """The packed kernel (2048-slot tiles) for every value type and array
    count it instantiates, sparse pushes spanning several tiles and push
    groups, serial and parallel, bit-exact against the oracle."""
    from parameter_server_amd._lib import PSG_FORM_PACKED
    D, pushes = random_case(31 + m, dtype, m, 150, 0.004, 30000)
    pushes = [p for p in pushes if p[0].size]
    for parallel in (False, True):
        out = run_ctx(D, pushes, dtype=dtype, parallel=parallel, flags=PSG_FORM_PACKED)
        rc, lo, hi, want, _ = O.aggregate(D, *ALL, pushes, parallel, 1, dtype)
        assert rc == 0 and len(out) == m
        for i in range(m):
            assert_bitexact(out[i][1], want[i])


@pytest.mark.parametrize("npush,density,nD", [(700, 0.002, 40000), (40, 0.6, 12000)])
def test_packed_push_groups(torch_cuda, npush, density, nD):
    """The packed kernel's push groups (up to 256 pushes whose elements fit
    one pass of 2,560): 700 sparse pushes (three groups per tile, the
    lastl rebase between them) and 40 dense pushes (~1,200 elements per push
    per tile: groups cut by the pass capacity, a piece per group at most
    2,048), serial and parallel, plan and context paths, bit-exact against
    the oracle; an unsorted push in the second case is reported."""
    torch = torch_cuda
    from parameter_server_amd._lib import PSG_FORM_PACKED
    D, pushes = random_case(900 + npush, np.float32, 1, npush, density, nD)
    pushes = [p for p in pushes if p[0].size]
    for parallel in (False, True):
        out = run_ctx(D, pushes, parallel=parallel, flags=PSG_FORM_PACKED)
        rc, lo, hi, want, _ = O.aggregate(D, *ALL, pushes, parallel, 1, np.float32)
        assert rc == 0
        assert_bitexact(out[0][1], want[0])
        plan, keep = plan_for(torch, [(D, pushes)], parallel=parallel, flags=PSG_FORM_PACKED)
        plan.run()
        assert plan.matched().tolist() == [k.size for k, _ in pushes]
        assert_bitexact(keep[3][0].cpu().numpy()[: D.size], want[0])
        plan.close()
    if npush == 40:
        bad = list(pushes)
        k = bad[7][0].copy()
        k[[100, 101]] = k[[101, 100]]  # two keys out of order
        bad[7] = (k, bad[7][1])
        plan, keep = plan_for(torch, [(D, bad)], flags=PSG_FORM_PACKED)
        plan.run()
        mt = plan.matched().tolist()
        assert mt[7] < k.size and all(mt[i] == bad[i][0].size for i in range(len(bad)) if i != 7)
        plan.close()


def extreme_range_keys():
    """5 tiles of 1024 server keys whose key ranges hit the bucket map's
    edges: 1023 wide; just under 2^32; exactly 2^32 (33 bits); one crowded
    bucket (1000 consecutive keys + 24 far ones); up to 2^64 - 2."""
    u = np.uint64
    seg0 = np.arange(1024, dtype=u)
    seg1 = u(1 << 20) + np.arange(1024, dtype=u) * u((2 ** 32 - 1) // 1023)
    seg2 = np.concatenate([u(1 << 40) + np.arange(1023, dtype=u),
                           np.array([(1 << 40) + (1 << 32)], u)])
    seg3 = np.concatenate([u(1 << 50) + np.arange(1000, dtype=u),
                           u(1 << 50) + u(1 << 30) + np.arange(24, dtype=u) * u(1 << 40)])
    step = (2 ** 64 - 2 - 2 ** 62) // 1023
    seg4 = np.array([2 ** 62 + i * step for i in range(1024)], u)
    D = np.concatenate([seg0, seg1, seg2, seg3, seg4])
    assert np.all(D[1:] > D[:-1]) and int(D[-1]) <= 2 ** 64 - 2
    return D


@pytest.mark.parametrize("pack", ["0", "1"])
def test_extreme_key_ranges(torch_cuda, pack):
    """Bucket scale (f32 reciprocal with a margin) at the key-range edges,
    crowded buckets, both round forms and both match modes, bit-exact."""
    from parameter_server_amd._lib import PSG_FORM_PACKED, PSG_FORM_UNIFORM
    flags = PSG_FORM_PACKED if pack == "1" else PSG_FORM_UNIFORM
    D = extreme_range_keys()
    rng = np.random.default_rng(77)
    pushes = []
    for p in range(6):
        k = np.sort(rng.choice(D, D.size // 2, replace=False))
        v = rng.standard_normal(k.size).astype(np.float32)
        v[rng.random(k.size) < 0.05] = -0.0
        pushes.append((k, [v]))
    for parallel in (False, True):
        out = run_ctx(D, pushes, parallel=parallel, flags=flags)
        rc, lo, hi, want, _ = O.aggregate(D, *ALL, pushes, parallel, 1, np.float32)
        assert rc == 0
        assert_bitexact(out[0][1], want[0])


# ------------------------------------------------------------------- errors
def test_defined_errors(torch_cuda):
    from parameter_server_amd._lib import (PSGError, PSG_ERR_UNMATCHED, PSG_ERR_RANGE,
                                           PSG_ERR_NO_TIME, PSG_ERR_EMPTY_KEYS,
                                           PSG_ERR_UNSORTED, PSG_ERR_CHANNEL)
    one = lambda n: [np.ones(n, np.float32)]  # noqa: E731
    v = kvv()
    with pytest.raises(PSGError) as e:
        v.setValue(msg([1], one(1)))
    assert e.value.status == PSG_ERR_EMPTY_KEYS
    v.setValue(msg([10, 20, 30, 40]))
    with pytest.raises(PSGError) as e:
        v.setValue(msg([40, 10]))  # unsorted key-only push
    assert e.value.status == PSG_ERR_UNSORTED
    for bad in ([10, 25], [20, 20], [30, 10], [5, 10], [10, 45]):
        v.setValue(msg(bad, one(2), t=1))
        with pytest.raises(PSGError) as e:
            v.received(1)
        assert e.value.status == PSG_ERR_UNMATCHED, bad
    with pytest.raises(PSGError) as e:
        v.received(1)
    assert e.value.status == PSG_ERR_NO_TIME
    v.setValue(msg([10], one(1), t=2, rng=(0, 25)))
    with pytest.raises(PSGError) as e:
        v.setValue(msg([30], one(1), t=2, rng=(25, 50)))
    assert e.value.status == PSG_ERR_RANGE
    v.setValue(msg([5, 6], t=0, ch=3))
    with pytest.raises(PSGError) as e:
        v.setValue(msg([5], one(1), t=2, ch=3, rng=(0, 25)))
    assert e.value.status == PSG_ERR_CHANNEL
    with pytest.raises(PSGError) as e:  # pigeonhole: 3 keys into 2 slots
        v.setValue(msg([10, 20, 30], one(3), t=3, rng=(0, 25)))
    assert e.value.status == PSG_ERR_UNMATCHED
    (rng, a), = v.received(2)
    assert a.tolist() == [1.0, 0.0]


# ------------------------------------------------------- union and gather
@pytest.mark.parametrize("seed", range(4))
def test_union_vs_oracle(torch_cuda, seed):
    rng = np.random.default_rng(100 + seed)
    v = kvv()
    acc = np.zeros(0, np.uint64)
    for step in range(4):
        n = [0, 1, 5000, 70000][(seed + step) % 4]
        k = np.unique(rng.integers(0, 1 << 40, n, dtype=np.uint64))
        v.setValue(msg(k))
        acc = O.set_union(acc, k)
        assert np.array_equal(v.key(0), acc)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_gather_vs_oracle(torch_cuda, dtype):
    rng = np.random.default_rng(5)
    D = np.unique(rng.integers(0, 1 << 50, 200000, dtype=np.uint64))
    W = rng.standard_normal(D.size).astype(dtype)
    req = np.sort(np.concatenate([rng.choice(D, 30000), rng.integers(0, 1 << 50, 3000, dtype=np.uint64)]))
    v = kvv(dtype)
    v.setValue(msg(D))
    v.set_value_array(0, W)
    m = msg(req)
    got_m = v.getValue(m)
    want, want_m = O.gather(D, W, req, dtype)
    assert got_m == want_m
    assert_bitexact(m.value[0], want)


def test_gather_tile_forms(torch_cuda):
    """Both gather forms (1024 requests per workgroup): chunks whose server
    span fits 4096 keys are staged in LDS, sparse chunks search global
    memory; requests repeated, on 4096-key boundaries and outside D's
    range."""
    rng = np.random.default_rng(21)
    D = np.unique(rng.integers(1 << 20, 1 << 44, 100000, dtype=np.uint64))
    W = rng.standard_normal(D.size).astype(np.float32)
    T = 4096
    edges = D[T::T]
    busy = D[3 * T:5 * T]  # two tiles with every key requested
    quiet = rng.choice(D, 40)
    req = np.sort(np.concatenate([
        busy, quiet, edges, edges, edges - np.uint64(1),
        np.array([0, 5, 1 << 60, (1 << 64) - 1], np.uint64),
        rng.integers(0, 1 << 44, 300, dtype=np.uint64)]))
    v = kvv(np.float32)
    v.setValue(msg(D))
    v.set_value_array(0, W)
    m = msg(req)
    got_m = v.getValue(m)
    want, want_m = O.gather(D, W, req)
    assert got_m == want_m
    assert_bitexact(m.value[0], want)


def test_flush_job_tables_reused_across_shapes(torch_cuda):
    """One context, received() after received() over shapes that repeat and
    change: the flush reuses its device tile descriptors and work items only
    when the shape repeats (range, push count, partition mode, the stream
    mode's push lengths, the continued-sum flag of a split flush); every
    result bit-exact against the oracle."""
    rng = np.random.default_rng(77)
    D = np.unique(rng.integers(1, 1 << 44, 60000, dtype=np.uint64))
    v = kvv(np.float32)
    v.setValue(msg(D))

    def dense_pushes(lo, hi, npush, frac):
        out = []
        for _ in range(npush):
            k = np.sort(rng.choice(D[lo:hi], int((hi - lo) * frac), replace=False))
            out.append((k, [rng.standard_normal(k.size).astype(np.float32)]))
        return out

    shapes = [(0, 60000, 8, 0.5), (0, 60000, 8, 0.5), (1000, 41000, 3, 0.7),
              (0, 60000, 8, 0.5), (0, 60000, 40, 0.002), (0, 60000, 40, 0.002),
              (0, 60000, 40, 0.003), (1000, 41000, 3, 0.7)]
    t = 3
    for i, (lo, hi, npush, frac) in enumerate(shapes):
        kb, ke = int(D[lo]), int(D[hi]) if hi < D.size else (1 << 64) - 1
        pushes = dense_pushes(lo, hi, npush, frac)
        v.set_flush_pushes(3 if i == 3 else 4096)  # one split flush: continued sums
        for k, vals in pushes:
            v.setValue(msg(k, vals, t=t, rng=(kb, ke)))
        (r, a), = v.received(t)
        rc, lo2, hi2, (want,), _ = O.aggregate(D, kb, ke, pushes)
        assert rc == 0 and tuple(r) == (lo2, hi2) == (lo, hi)
        assert_bitexact(a, want)
        t += 1
    v.close()


# ------------------------------------------- device-resident plans (bench path)
def to_dev(torch, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    return torch.from_numpy(a).cuda()


def plan_for(torch, cases, dtype=np.float32, parallel=False, flags=0):
    from parameter_server_amd.kv_vector import MergePlan
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    keep, jobs = [], []
    m = len(cases[0][1][0][1])
    for D, pushes in cases:
        dD = to_dev(torch, D)
        pk = [to_dev(torch, k) for k, _ in pushes]
        pv = [[to_dev(torch, np.asarray(x, dtype)) for x in vs] for _, vs in pushes]
        out = [torch.full((max(1, D.size),), float("nan"), dtype=torch.float32 if dtype == np.float32 else torch.float64, device="cuda") for _ in range(m)]
        keep += [dD, pk, pv, out]
        jobs.append({"keys": dD.data_ptr(), "nslots": D.size,
                     "push_keys": [t.data_ptr() for t in pk],
                     "push_vals": [[t.data_ptr() for t in vs] for vs in pv],
                     "push_n": [k.size for k, _ in pushes],
                     "out": [o.data_ptr() for o in out]})
    plan = MergePlan(0, PSG_F32 if dtype == np.float32 else PSG_F64, m, jobs, parallel, flags)
    return plan, keep


def test_plan_cfg2_full_size_bitexact(torch_cuda):
    torch = torch_cuda
    from parameter_server_amd import synth
    D, pushes = synth.overlap_pushes(1)
    assert D.size == GOLD["cfg2"]["U"]
    plan, keep = plan_for(torch, [(D, pushes)])
    plan.run()
    assert plan.matched().tolist() == [131072] * 8
    got = keep[3][0].cpu().numpy()[: D.size]
    _, _, _, want, _ = O.aggregate(D, *ALL, pushes)
    assert_bitexact(got, want[0])
    plan.run()  # idempotent re-run (bench loop)
    assert_bitexact(keep[3][0].cpu().numpy()[: D.size], want[0])


def test_plan_batched_jobs_and_dense(torch_cuda):
    torch = torch_cuda
    from parameter_server_amd import synth
    cases = [synth.overlap_pushes(3, npush=4, n=20000),
             synth.dense_pushes(npush=8, n=1 << 20),
             synth.overlap_pushes(4, npush=40, n=3000, overlap=0.5),
             synth.zipf_pushes(3, npush=16, n=8192)]
    from parameter_server_amd._lib import PSG_STATIC_KEYS
    for flags in (PSG_STATIC_KEYS, 0):  # dense job allowed / never
        plan, keep = plan_for(torch, cases, flags=flags)
        plan.run()
        mt = plan.matched()
        assert mt.tolist() == [k.size for _, ps in cases for k, _ in ps]
        outs = keep[3::4]
        for (D, pushes), out in zip(cases, outs):
            _, _, _, want, _ = O.aggregate(D, *ALL, pushes)
            assert_bitexact(out[0].cpu().numpy()[: D.size], want[0])
        plan.close()


def test_plan_changed_slice_keys_are_reported(torch_cuda):
    """a plan over contiguous-slice pushes created WITHOUT
    PSG_STATIC_KEYS re-checks the keys every run, so a push key changed
    after creation (here: one key of a slice moved off D) is reported
    unmatched by the next run instead of being folded silently."""
    torch = torch_cuda
    from parameter_server_amd import synth
    D, pushes = synth.dense_pushes(npush=4, n=1 << 16)
    plan, keep = plan_for(torch, [(D, pushes)])
    plan.run()
    assert plan.matched().tolist() == [1 << 16] * 4
    keep[1][2][777] = int(D[777]) * 1000 + 3  # not a server key any more
    plan.run()
    mt = plan.matched().tolist()
    assert mt[2] < (1 << 16) and mt[:2] == [1 << 16] * 2 and mt[3] == 1 << 16
    plan.close()


def test_plan_cfg4_full_dense(torch_cuda):
    """cfg4 at its full size: 8 pushes x 16 M contiguous keys."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_STATIC_KEYS
    D, pushes = synth.dense_pushes()
    plan, keep = plan_for(torch, [(D, pushes)], flags=PSG_STATIC_KEYS)
    plan.run()
    assert plan.matched().tolist() == [1 << 24] * 8
    _, _, _, want, _ = O.aggregate(D, *ALL, pushes)
    assert_bitexact(keep[3][0].cpu().numpy(), want[0])


@pytest.mark.parametrize("dtype,parallel", [(np.float32, False), (np.float64, True),
                                            (np.float64, False)])
def test_plan_dense_slices(torch_cuda, dtype, parallel):
    """The dense fast path (psg_tile_dense.hip): pushes that are contiguous
    slices of D (whole, inner, tail, single key, empty) fold without key
    reads, bit-exact with the oracle (m = 2, -0.0 values, pushes starting
    mid-tile); a job with one near-slice push (one key missing) and a mixed
    plan take the general kernels and agree too; a second run repeats."""
    torch = torch_cuda
    rng = np.random.default_rng(91)
    D = (np.arange(1, 100001, dtype=np.uint64) * np.uint64(3))
    sl = [(0, 100000), (500, 70000), (99000, 100000), (0, 0), (12345, 12346), (1023, 4097)]

    def vals(n):
        v = [rng.standard_normal(n).astype(dtype) for _ in range(2)]
        v[0][::7] = -0.0
        return v

    dense = (D, [(D[a:b], vals(b - a)) for a, b in sl])
    near_k = np.delete(D[200:5200], 77)
    near = (D, [(D[0:3000], vals(3000)), (near_k, vals(near_k.size))])
    from parameter_server_amd._lib import PSG_STATIC_KEYS
    for cases in ([dense], [dense, near]):
        plan, keep = plan_for(torch, cases, dtype=dtype, parallel=parallel, flags=PSG_STATIC_KEYS)
        for rep in range(2):
            plan.run()
            mt = plan.matched().tolist()
            want_mt = [k.size for _, ps in cases for k, _ in ps]
            assert mt == want_mt
            for j, (Dj, pushes) in enumerate(cases):
                _, _, _, want, _ = O.aggregate(Dj, *ALL, pushes, parallel=parallel, dtype=dtype)
                for i in range(2):
                    assert_bitexact(keep[4 * j + 3][i].cpu().numpy()[: Dj.size], want[i])
        plan.close()


@pytest.mark.parametrize("pack", ["0", "1"])
def test_plan_round_forms_agree(torch_cuda, pack):
    """Both aggregate kernels on the same jobs, forced with the plan flags
    PSG_FORM_PACKED / PSG_FORM_UNIFORM: push-uniform rounds (psg_tile.hip) and packed multi-push
    rounds (psg_tile_packed.hip), whose rounds hold several pushes that can
    hit one slot (heavy overlap: many same-slot lanes per round, resolved in
    push order) -- bit-exact either way, serial and parallel."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_FORM_PACKED, PSG_FORM_UNIFORM
    flags = PSG_FORM_PACKED if pack == "1" else PSG_FORM_UNIFORM
    rng = np.random.default_rng(5)
    D = np.unique(rng.integers(0, 1 << 50, 20000, dtype=np.uint64))
    tiny = [(np.sort(rng.choice(D, n, replace=False)),
             [rng.standard_normal(n).astype(np.float32)]) for n in
            [int(x) for x in rng.integers(1, 60, 150)]]
    for p_ in tiny[::7]:
        p_[1][0][::3] = -0.0
    cases = [(D, tiny), synth.overlap_pushes(8, npush=70, n=2000, overlap=0.9),
             synth.zipf_pushes(9, npush=24, n=3000)]
    for parallel in (False, True):
        plan, keep = plan_for(torch, cases, parallel=parallel, flags=flags)
        plan.run()
        assert plan.matched().tolist() == [k.size for _, ps in cases for k, _ in ps]
        for j, (Dj, pushes) in enumerate(cases):
            _, _, _, want, _ = O.aggregate(Dj, *ALL, pushes, parallel=parallel)
            assert_bitexact(keep[4 * j + 3][0].cpu().numpy()[: Dj.size], want[0])
        plan.close()


@pytest.mark.parametrize("mode", ["search", "stream"])
def test_plan_partition_modes_agree(torch_cuda, mode):
    """Both partition modes on dense and sparse jobs, forced
    with the plan flags PSG_PART_SEARCH / PSG_PART_STREAM: every (push, tile) piece must
    come out the same, so the merge is bit-exact either way, including
    pushes much sparser than the tiles (window fallback of the stream mode)
    and pushes with keys below D[0] or above D[-1] only in other tiles."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_PART_SEARCH, PSG_PART_STREAM
    flags = PSG_PART_SEARCH if mode == "search" else PSG_PART_STREAM
    rng = np.random.default_rng(77)
    D = np.unique(rng.integers(0, 1 << 60, 300000, dtype=np.uint64))
    sparse = [(np.sort(rng.choice(D, n, replace=False)),
               [rng.standard_normal(n).astype(np.float32)]) for n in (3, 40, 700, 5000, 1)]
    cases = [synth.overlap_pushes(21, npush=8, n=30000),
             (D, sparse),
             synth.zipf_pushes(22, npush=20, n=4000)]
    for parallel in (False, True):
        plan, keep = plan_for(torch, cases, parallel=parallel, flags=flags)
        plan.run()
        assert plan.matched().tolist() == [k.size for _, ps in cases for k, _ in ps]
        for (Dj, pushes), out in zip(cases, keep[3::4]):
            _, _, _, want, _ = O.aggregate(Dj, *ALL, pushes, parallel=parallel)
            assert_bitexact(out[0].cpu().numpy()[: Dj.size], want[0])


def test_plan_cfg3_full_size(torch_cuda):
    """cfg3 at its configured shape (BASELINE.json configs[2]): 64 pushes x
    131,072 unique murmur-shuffled Zipf(1.1) ranks in [1, 1e9]
    (synth.zipf_pushes defaults), f32, both match modes."""
    torch = torch_cuda
    from parameter_server_amd import synth
    D, pushes = synth.zipf_pushes()
    assert len(pushes) == 64 and all(k.size == 131072 for k, _ in pushes)
    for parallel in (False, True):
        plan, keep = plan_for(torch, [(D, pushes)], parallel=parallel)
        plan.run()
        assert plan.matched().tolist() == [131072] * 64
        _, _, _, want, _ = O.aggregate(D, *ALL, pushes, parallel=parallel)
        assert_bitexact(keep[3][0].cpu().numpy()[: D.size], want[0])


def test_plan_cfg5_shard(torch_cuda):
    """cfg5 (BASELINE.json configs[4]) as one GPU's shard: 256 pushes x
    262,144 unique murmur-shuffled uniform ranks in [0, 1e9), cut at the
    8-shard evenDivide bounds (range.h:85-98) by sliceKeyOrderedMsg's
    lower_bound rule (message.h:96-99); shard 0's pieces merged on the GPU
    against the oracle's merge of the same pieces over the shard's keys."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd.kv_vector import shard_bounds
    b = shard_bounds(8)
    D, pieces = synth.cfg5_shard(0, 8)
    assert len(pieces) == 256
    assert D.size > 0 and int(D[-1]) < int(b[1])
    plan, keep = plan_for(torch, [(D, pieces)])
    plan.run()
    assert plan.matched().tolist() == [k.size for k, _ in pieces]
    _, _, _, want, _ = O.aggregate(D, int(b[0]), int(b[1]), pieces)
    assert_bitexact(keep[3][0].cpu().numpy()[: D.size], want[0])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("parallel", [True, False])
def test_plan_cfg5_whole_workload(torch_cuda, parallel):
    """The whole 1-GPU cfg5 workload (the bench's cfg5 line): 256 pushes x
    262,144 keys over U = 64.9 M server slots, packed-round kernel and stream
    partition, both modes, bit-exact against the oracle's scatter forms:
    parallelSetValue (orc_aggregate_scatter, cross-checked against the
    merge-walk restatement of match) and serialSetValue
    (orc_aggregate_scatter_serial, cross-checked against the dense oldMatch
    fold) in tests/test_oracle.py."""
    torch = torch_cuda
    from parameter_server_amd import synth
    D, pushes = synth.uniform_pushes(seed=5)
    assert len(pushes) == 256 and D.size > 64_000_000
    plan, keep = plan_for(torch, [(D, pushes)], parallel=parallel)
    plan.run()
    assert plan.matched().tolist() == [k.size for k, _ in pushes]
    got = keep[3][0].cpu().numpy()[: D.size]
    del plan, keep
    torch.cuda.empty_cache()
    rc, lo, hi, want, matched = O.aggregate_scatter(D, *ALL, pushes, parallel=parallel)
    assert rc == 0 and (lo, hi) == (0, D.size)
    assert_bitexact(got, want[0])


def test_rcv1_shape_blocks(torch_cuda):
    """cfg1 (rcv1 L1-LR via Darling) shape through the host API: 47,236
    server keys in [1, 47237), feature blocks as key ranges, 2 workers
    pushing ~150 keys each per block with m = 2 f64 arrays (G and U,
    darling.cc:196-220); received(t) per block against the oracle, serial
    and parallel (the data itself cannot be fetched)."""
    rng = np.random.default_rng(1)
    D = np.arange(1, 47237, dtype=np.uint64)
    edges = np.linspace(1, 47237, 298).astype(np.uint64)  # 297 blocks per pass
    for parallel in (False, True):
        v = kvv(np.float64, parallel)
        v.setValue(msg(D))
        for t, blk in enumerate(range(0, 297, 15)):
            kb, ke = int(edges[blk]), int(edges[blk + 1])
            inr = D[(D >= kb) & (D < ke)]
            pushes = []
            for wkr in range(2):
                k = np.sort(rng.choice(inr, min(inr.size, 150), replace=False))
                pushes.append((k, [rng.standard_normal(k.size), rng.standard_normal(k.size)]))
                v.setValue(msg(k, pushes[-1][1], t=t, rng=(kb, ke)))
            out = v.received(t)
            rc, lo, hi, want, _ = O.aggregate(D, kb, ke, pushes, parallel, 1, np.float64)
            assert rc == 0 and len(out) == 2
            for i in range(2):
                assert tuple(out[i][0]) == (lo, hi)
                assert_bitexact(out[i][1], want[i])
        v.close()


def test_plan_empty_first_push_keeps_negative_zero(torch_cuda):
    """An empty push is ignored (kv_vector.h:90,177): when the caller's first
    push is empty, the first NON-empty push assigns, so its -0.0 stays -0.0
    where no later push holds the key (parallel), and the serial path's
    trailing +0.0 canonicalises it exactly as the reference's dense += does."""
    torch = torch_cuda
    D = np.array([2, 4, 6, 8], np.uint64)
    pushes = [(np.zeros(0, np.uint64), [np.zeros(0, np.float32)]),
              (np.array([2, 4], np.uint64), [np.array([-0.0, 1.5], np.float32)]),
              (np.array([4, 8], np.uint64), [np.array([2.0, -0.0], np.float32)])]
    for parallel in (False, True):
        plan, keep = plan_for(torch, [(D, pushes)], parallel=parallel)
        plan.run()
        assert plan.matched().tolist() == [0, 2, 2]
        _, _, _, want, _ = O.aggregate(D, *ALL, pushes[1:], parallel=parallel)
        got = keep[3][0].cpu().numpy()
        assert_bitexact(got, want[0])
        assert np.signbit(got[0]) == (parallel is True)  # -0.0 kept only by parallel


def test_key_union_between_push_and_received(torch_cuda):
    """A key-only push that lands between a value push at time t and
    received(t) (keys added below and inside the range): the pending push
    was matched against the key set it arrived with (kv_vector.h:171-204),
    so received(t) equals the oracle over the OLD keys and positions."""
    D = np.array([10, 20, 30, 40, 50], np.uint64)
    v = kvv()
    v.setValue(msg(D))
    k = np.array([20, 40], np.uint64)
    v.setValue(msg(k, [np.array([1.0, 2.0], np.float32)], t=3))
    v.setValue(msg(np.array([5, 25, 45], np.uint64)))  # union changes every position
    (rng, got), = v.received(3)
    _, lo, hi, want, _ = O.aggregate(D, *ALL, [(k, [np.array([1.0, 2.0], np.float32)])])
    assert tuple(rng) == (lo, hi) and got.tolist() == want[0].tolist()
    assert v.key(0).tolist() == [5, 10, 20, 25, 30, 40, 45, 50]
    v.close()


def test_device_entry_points(torch_cuda):
    """psg_gather_dev, psg_key_union_dev and psg_slice_dev on device buffers
    against the oracle's gather / setUnion / sliceKeyOrderedMsg."""
    torch = torch_cuda
    import ctypes as C
    from parameter_server_amd import _lib
    from parameter_server_amd.kv_vector import shard_bounds
    L = _lib.lib()
    rng = np.random.default_rng(9)
    D = np.unique(rng.integers(0, 1 << 62, 50000, dtype=np.uint64))
    W = rng.standard_normal(D.size).astype(np.float32)
    req = np.sort(np.concatenate([rng.choice(D, 4000, replace=False),
                                  rng.integers(0, 1 << 62, 500, dtype=np.uint64)]))
    dD, dW, dR = to_dev(torch, D), to_dev(torch, W), to_dev(torch, req)
    dout = torch.empty(req.size, dtype=torch.float32, device="cuda")
    dm = torch.zeros(1, dtype=torch.int64, device="cuda")
    _lib.check(L.psg_gather_dev(_lib.PSG_F32, dD.data_ptr(), D.size, dW.data_ptr(), dR.data_ptr(),
                                req.size, dout.data_ptr(), dm.data_ptr(), None))
    want, wm = O.gather(D, W, req)
    assert int(dm.item()) == wm
    assert_bitexact(dout.cpu().numpy(), want)
    a = np.unique(rng.integers(0, 1 << 40, 30000, dtype=np.uint64))
    bb = np.unique(rng.integers(0, 1 << 40, 20000, dtype=np.uint64))
    da, db = to_dev(torch, a), to_dev(torch, bb)
    du = torch.empty(a.size + bb.size, dtype=torch.int64, device="cuda")
    nout = C.c_uint64()
    _lib.check(L.psg_key_union_dev(da.data_ptr(), a.size, db.data_ptr(), bb.size, du.data_ptr(),
                                   C.byref(nout), None))
    assert np.array_equal(du.cpu().numpy().view(np.uint64)[: nout.value], O.set_union(a, bb))
    bad = to_dev(torch, np.array([5, 3], np.uint64))
    assert L.psg_key_union_dev(da.data_ptr(), a.size, bad.data_ptr(), 2, du.data_ptr(),
                               C.byref(nout), None) == _lib.PSG_ERR_UNSORTED
    sep = shard_bounds(8)
    for kb, ke in ((0, (1 << 64) - 1), (int(D[100]), int(D[-100]))):
        dsep = to_dev(torch, sep)
        dpos = torch.empty(sep.size, dtype=torch.int64, device="cuda")
        _lib.check(L.psg_slice_dev(dD.data_ptr(), D.size, kb, ke, dsep.data_ptr(), sep.size,
                                   dpos.data_ptr(), None))
        torch.cuda.synchronize()
        pos, _ = O.slice_key_ordered(D, kb, ke, sep)
        assert np.array_equal(dpos.cpu().numpy().view(np.uint64), pos)


# --------------------------------------------- dense slices through psg_push
@pytest.mark.parametrize("parallel", [False, True])
def test_push_dense_slices_server_api(torch_cuda, parallel):
    """psg_push's dense test: pushes that are contiguous
    slices of a contiguous key range take the dense kernel (no key reads;
    their keys are only checked strictly increasing on the copy stream);
    mixed with a sparse push they take the general kernels with D's slice
    standing in for the keys.  Bit-exact against the oracle either way, with
    launch seams, -0.0 and sub-ranges."""
    rng = np.random.default_rng(3)
    D = np.arange(1000, 1000 + 200000, dtype=np.uint64)
    pushes = []
    for a, n in [(0, 200000), (5000, 70000), (0, 200000), (150000, 50000), (1, 4096)]:
        v = rng.standard_normal(n).astype(np.float32)
        v[rng.random(n) < 0.03] = -0.0
        pushes.append((D[a:a + n].copy(), [v]))
    for flush in (None, 2):
        out = run_ctx(D, pushes, parallel=parallel, flush=flush)
        _, lo, hi, want, _ = O.aggregate(D, *ALL, pushes, parallel, 1, np.float32)
        assert_bitexact(out[0][1], want[0])
    # a sparse push among them: general kernels, same bits
    sp = np.sort(rng.choice(D, 3000, replace=False))
    mixed = pushes[:2] + [(sp, [rng.standard_normal(sp.size).astype(np.float32)])] + pushes[2:]
    out = run_ctx(D, mixed, parallel=parallel)
    _, lo, hi, want, _ = O.aggregate(D, *ALL, mixed, parallel, 1, np.float32)
    assert_bitexact(out[0][1], want[0])
    # a sub-range push (key_range [2000, 90000))
    kb, ke = 2000, 90000
    sub = [(np.arange(3000, 50000, dtype=np.uint64), [np.ones(47000, np.float32)])]
    out = run_ctx(D, sub, kb, ke, parallel=parallel)
    _, lo, hi, want, _ = O.aggregate(D, kb, ke, sub, parallel, 1, np.float32)
    assert tuple(out[0][0]) == (lo, hi)
    assert_bitexact(out[0][1], want[0])


def test_push_dense_slice_order_violation_is_unmatched(torch_cuda):
    """End keys of a slice but two interior keys swapped: the reference's
    merge walk matches fewer than n keys (CHECK_EQ, kv_vector.h:192); the
    dense path reports it through the copy-stream order check."""
    from parameter_server_amd._lib import PSGError, PSG_ERR_UNMATCHED
    D = np.arange(50000, dtype=np.uint64)
    k = D.copy()
    k[100], k[101] = k[101], k[100]
    v = kvv()
    v.setValue(msg(D))
    v.setValue(msg(k, [np.ones(k.size, np.float32)], t=3))
    with pytest.raises(PSGError) as e:
        v.received(3)
    assert e.value.status == PSG_ERR_UNMATCHED
    v.close()


@pytest.mark.parametrize("hold", [False, True])
def test_push_dense_pinned_keys_checked_in_place(torch_cuda, hold):
    """Pinned keys of a dense push are never staged: the order check reads
    them from host memory (16 B per lane, neighbour keys across lanes and
    waves).  Every kind of violation is reported -- swaps inside a lane's
    pair, across lanes, across a wave boundary, in an odd tail, and a
    duplicate -- and a clean push still merges bit-exact.  A pinned buffer
    that is not 16-B aligned takes the staged path."""
    torch = torch_cuda
    from parameter_server_amd._lib import PSGError, PSG_ERR_UNMATCHED, PSG_HOLD_BUFFERS
    n = 50001  # odd: a tail key past the last whole pair
    D = np.arange(7, 7 + n, dtype=np.uint64)

    def pinned(a, shift=0):
        t = torch.empty(a.size + 2, dtype=torch.int64).pin_memory()
        h = t.numpy().view(np.uint64)[shift:shift + a.size]
        h[:] = a
        return t, h

    def swap(i, j):
        k = D.copy()
        k[i], k[j] = k[j], k[i]
        return k
    dup = D.copy()
    dup[1001:20000] = D[1000:19999]  # keys 1000 twice, ends and count unchanged
    dup[20000:] = D[20000:]
    cases = [swap(100, 101), swap(101, 102), swap(127, 128), swap(255, 256),
             swap(n - 2, n - 1), dup]
    flags = PSG_HOLD_BUFFERS if hold else 0
    for shift in (0, 1):
        for k in cases:
            keep, hk = pinned(k, shift)
            v = kvv(flags=flags)
            v.setValue(msg(D))
            vals = np.ones(n, np.float32)
            v.setValue(msg(hk, [vals], t=3))
            with pytest.raises(PSGError) as e:
                v.received(3)
            assert e.value.status == PSG_ERR_UNMATCHED
            v.close()
            del keep
        keep, hk = pinned(D, shift)
        vals = np.random.default_rng(2).standard_normal(n).astype(np.float32)
        v = kvv(flags=flags)
        v.setValue(msg(D))
        v.setValue(msg(hk, [vals], t=4))
        v.setValue(msg(hk, [vals], t=4))
        (rng, got), = v.received(4)
        _, lo, hi, want, _ = O.aggregate(D, *ALL, [(D, [vals])] * 2, False, 1, np.float32)
        assert tuple(rng) == (lo, hi)
        assert_bitexact(got, want[0])
        v.close()
        del keep


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("parallel", [False, True])
def test_nan_payloads(torch_cuda, dtype, parallel):
    """NaN payload bits through the fold: quiet and signalling NaNs of both
    signs with distinct payloads.  A slot with ONE NaN contributor must come
    out as the reference's IEEE add gives it (the input NaN, quieted) bit
    for bit.  A slot with two or more NaN contributors is compared only as
    "one of the input NaNs, quieted": which operand's payload an add of two
    NaNs keeps is not fixed by IEEE 754 (x86 SSE keeps the first source,
    and the compiler may commute the reference's `+=`), so the reference
    itself does not pin it."""
    ut = np.uint32 if dtype == np.float32 else np.uint64
    if dtype == np.float32:
        pays = [0x7fc12345, 0xffc00001, 0x7f800001, 0xff812345, 0x7fffffff]
        quiet = 1 << 22
    else:
        pays = [0x7ff8000000012345, 0xfff8000000000001, 0x7ff0000000000001,
                0xfff0000000abcdef, 0x7fffffffffffffff]
        quiet = 1 << 51
    rng = np.random.default_rng(11)
    D = np.arange(4000, dtype=np.uint64) * np.uint64(5)
    pushes = []
    owner = rng.integers(0, 6, D.size)        # the push that carries a NaN at slot i
    second = rng.random(D.size) < 0.1          # ... and a second NaN from push owner+1
    for p in range(6):
        k = D.copy()
        v = rng.standard_normal(D.size).astype(dtype)
        b = v.view(ut)
        one = owner == p
        b[one] = np.array(pays, ut)[np.arange(D.size)[one] % len(pays)]
        two = second & ((owner + 1) % 6 == p)
        b[two] = np.array(pays, ut)[(np.arange(D.size)[two] + 2) % len(pays)]
        drop = rng.random(D.size) < 0.2
        drop[one | two] = False
        pushes.append((k[~drop], [v[~drop]]))
    out = run_ctx(D, pushes, dtype=dtype, parallel=parallel)
    _, _, _, want, _ = O.aggregate(D, *ALL, pushes, parallel, 1, dtype)
    got = np.asarray(out[0][1])
    gb, wb = bits(got), bits(np.asarray(want[0], dtype))
    assert np.array_equal(np.isnan(got), np.isnan(want[0]))
    single = ~second
    assert np.array_equal(gb[single], wb[single])
    # two NaN contributors: one of the two inputs' payloads, quieted
    idx = np.nonzero(second)[0]
    pa = np.array(pays, ut)
    cand = np.stack([pa[idx % len(pays)], pa[(idx + 2) % len(pays)]]) | ut(quiet)
    assert np.all((gb[idx] == cand[0]) | (gb[idx] == cand[1]))




def _corner_pushes(dtype, seed, npush=8, nkeys=6000, m=2):
    """Pushes whose values mix IEEE corner cases (denormals of both signs,
    +-0, +inf, the largest finite, round-to-even ties around 1.0 and 2^24 /
    2^53, values whose sums go denormal or overflow to +inf) with ordinary
    values.  No -inf and no large negatives: +inf + -inf makes the default
    NaN, whose sign differs between x86 (the oracle) and the GPU."""
    rng = np.random.default_rng(seed)
    if dtype == np.float32:
        ut, tiny = np.uint32, 2.0 ** -140
        pool = [0x00000001, 0x80000001, 0x007fffff, 0x807fffff, 0x00800000, 0x80800000,
                0x7f7fffff, 0x7f800000, 0x00000000, 0x80000000, 0x3f800000, 0x33800000,
                0x33800001, 0xb3800000, 0x4b800000, 0x3f800001, 0x00400000, 0x80400001]
    else:
        ut, tiny = np.uint64, 2.0 ** -1060
        pool = [0x1, 0x8000000000000001, 0x000fffffffffffff, 0x800fffffffffffff,
                0x0010000000000000, 0x8010000000000000, 0x7fefffffffffffff,
                0x7ff0000000000000, 0x0, 0x8000000000000000, 0x3ff0000000000000,
                0x3ca0000000000000, 0x3ca0000000000001, 0xbca0000000000000,
                0x4340000000000000, 0x3ff0000000000001, 0x0008000000000000]
    pool = np.array(pool, ut)
    D = np.unique(rng.integers(0, 1 << 40, nkeys).astype(np.uint64))
    pushes = []
    for _ in range(npush):
        keep = rng.random(D.size) < 0.7
        k = D[keep]
        vs = []
        for _ in range(m):
            v = rng.standard_normal(k.size).astype(dtype)
            sel = rng.random(k.size)
            v[sel < 0.4] = pool[rng.integers(0, pool.size, int((sel < 0.4).sum()))].view(dtype)
            small = (sel >= 0.4) & (sel < 0.6)
            v[small] = (rng.standard_normal(int(small.sum())) * tiny).astype(dtype)
            vs.append(v)
        pushes.append((k, vs))
    return D, pushes


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("parallel", [False, True])
def test_fold_ieee_corner_values(torch_cuda, dtype, parallel):
    """The tile kernel's fold adds by LDS float atomics (ds_add_f32 /
    ds_add_f64): bit-identical to the reference's `+=` on denormals,
    signed zeros, overflow and ties, through a plan (m = 2) and through the
    server context."""
    torch = torch_cuda
    D, pushes = _corner_pushes(dtype, 21)
    plan, keep = plan_for(torch, [(D, pushes)], dtype, parallel)
    plan.run()
    torch.cuda.synchronize()
    _, _, _, want, _ = O.aggregate(D, *ALL, pushes, parallel, 2, dtype)
    for i in range(2):
        assert_bitexact(keep[3][i].cpu().numpy()[:D.size], np.asarray(want[i], dtype))
    plan.close()
    out = run_ctx(D, [(k, vs) for k, vs in pushes], dtype=dtype, parallel=parallel)
    for i in range(2):
        assert_bitexact(np.asarray(out[i][1]), np.asarray(want[i], dtype))


# ------------------------------- a value-array list that grows within a time
@pytest.mark.parametrize("parallel", [False, True])
@pytest.mark.parametrize("flush", [None, 2])
def test_growing_value_array_list(torch_cuda, parallel, flush):
    """recved_val_[t] grows when a later push of the same time brings more
    value arrays (kv_vector.h:110-129 / 189-196): array i is assigned by the
    first push holding an i-th array and added to only by later pushes that
    hold one (serial: with the dense += over the range, so a push without
    the key adds +0.0; a push without array i adds nothing to it).  So array
    i is exactly the aggregate of the pushes holding it: checked bit for bit
    against the oracle run over that subset, with single-launch and
    continued (2 pushes per launch) flushes."""
    mseq = [1, 2, 1, 3, 2, 1, 3]
    dtype = np.float64 if parallel else np.float32
    D, full = random_case(77, dtype, 3, len(mseq), 0.3, 4000)
    pushes = [(k, vs[:mp]) for (k, vs), mp in zip(full, mseq)]
    out = run_ctx(D, pushes, dtype=dtype, parallel=parallel, flush=flush)
    assert len(out) == max(mseq)
    for i in range(max(mseq)):
        sub = [(k, [vs[i]]) for k, vs in pushes if len(vs) > i]
        rc, lo, hi, want, _ = O.aggregate(D, *ALL, sub, parallel, 1, dtype)
        assert rc == 0 and list(out[i][0]) == [lo, hi]
        assert_bitexact(out[i][1], want[0])


def _oracle_keys(Dj, pushes):
    """The oracle's aggregate takes Range::all() = [0, 2^64 - 1) (range.h:
    75-78); a case whose D ends at 2^64 - 1 (the open last tile) is handed
    to it with every key shifted down by one: same order, same matches,
    same fold."""
    if Dj.size and int(Dj[-1]) == (1 << 64) - 1:
        assert int(Dj[0]) > 0
        one = np.uint64(1)
        return Dj - one, [(k - one, vs) for k, vs in pushes]
    return Dj, pushes


def _cursor_check(torch, cases, parallel, flags=0, want_form=None, reps=2):
    from parameter_server_amd._lib import PSG_KERNEL_CURSOR
    plan, keep = plan_for(torch, cases, parallel=parallel, flags=flags)
    assert plan.form == (PSG_KERNEL_CURSOR if want_form is None else want_form)
    for _ in range(reps):  # a second run lands in the same buffers (bench loop)
        plan.run()
        mt = plan.matched().tolist()
        want_mt = []
        for j, (Dj, pushes) in enumerate(cases):
            rc, _, _, want, wm = O.aggregate(*_oracle_keys(Dj, pushes)[:1], *ALL,
                                             _oracle_keys(Dj, pushes)[1], parallel=parallel)
            want_mt += [int(x) for x in wm]
            assert_bitexact(keep[4 * j + 3][0].cpu().numpy()[: Dj.size], want[0])
        assert mt == want_mt
    plan.close()


@pytest.mark.parametrize("parallel", [False, True])
def test_plan_cursor_form(torch_cuda, parallel):
    """The cursor kernel (psg_tile_cursor.hip: no partition pass; each
    workgroup walks a chunk of tiles with one cursor per push and finds a
    piece's end with the element loads), PSG_FORM_CURSOR on plans of long
    pieces, bit-exact with the oracle's serialSetValue /
    parallelSetValue and matched counts, over 8, 3 and 20 pushes (groups of
    8, idle waves), 1-3 rounds per push, one- and many-tile chunks, D ending
    at 2^64 - 1 (the open last tile) and a second run."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_FORM_CURSOR
    rng = np.random.default_rng(123)
    Dh = np.unique(np.concatenate([rng.integers(1 << 63, (1 << 64) - 1, 30000, dtype=np.uint64),
                                   np.array([(1 << 64) - 1], np.uint64)]))
    hp = [(np.sort(rng.choice(Dh, 3000, replace=False)),
           [rng.standard_normal(3000).astype(np.float32)]) for _ in range(4)]
    # the last 3 tiles whole: ~1000-key pieces, the slow path
    hp.append((Dh[-3000:].copy(), [rng.standard_normal(3000).astype(np.float32)]))
    hp[2][1][0][::5] = -0.0
    cases = [synth.overlap_pushes(31, npush=8, n=40000),            # cfg2-like: 3 rounds
             synth.overlap_pushes(33, npush=20, n=12000, overlap=0.5),  # 3 groups
             (Dh, hp),                                                 # open end, 2^64 - 1
             synth.overlap_pushes(34, npush=8, n=2000)]                 # 15 tiles
    _cursor_check(torch, cases, parallel, flags=PSG_FORM_CURSOR)


def test_plan_cursor_long_pieces_and_unmatched(torch_cuda):
    """PSG_FORM_CURSOR on pieces longer than 3 rounds (3 pushes of ~365 keys
    per tile: every group takes the slow path, which merges push after push
    to each piece's end) and pushes holding keys outside D (below D[0],
    between server keys, above D[-1]): matched counts equal the oracle's,
    the sums too; PSG_NO_CURSOR gives the partition path the same bits."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_FORM_CURSOR, PSG_NO_CURSOR, PSG_KERNEL_TILE
    rng = np.random.default_rng(7)
    long_ = synth.overlap_pushes(32, npush=3, n=30000)
    D = np.unique(rng.integers(1000, 1 << 40, 60000, dtype=np.uint64))
    extra = np.array([1, 2, int(D[100]) + 1, int(D[-1]) + 5], np.uint64)
    ps = []
    for i in range(5):
        k = np.sort(rng.choice(D, 4000, replace=False))
        if i in (1, 3):
            k = np.unique(np.concatenate([k, extra if i == 1 else extra[2:]]))
        ps.append((k, [rng.standard_normal(k.size).astype(np.float32)]))
    for parallel in (False, True):
        _cursor_check(torch, [long_, (D, ps)], parallel, flags=PSG_FORM_CURSOR)
        _cursor_check(torch, [long_, (D, ps)], parallel, flags=PSG_NO_CURSOR,
                      want_form=PSG_KERNEL_TILE, reps=1)


def test_plan_cursor_unsorted_push_is_reported(torch_cuda):
    """An unsorted push through the cursor form: keys swapped inside one
    tile (the order check) and across tiles far apart (the chunks' cursors
    disagree at a chunk boundary: the boundary word reaches
    psg_plan_matched) are both reported (matched < n) while the sorted
    pushes of the same plan stay exact."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_FORM_CURSOR, PSG_KERNEL_CURSOR
    D, pushes = synth.overlap_pushes(35, npush=8, n=40000)
    for (i, j) in ((100, 101), (500, 39000)):
        bad = [(k.copy(), vs) for k, vs in pushes]
        k = bad[4][0]
        k[i], k[j] = k[j], k[i]
        plan, keep = plan_for(torch, [(D, bad)], flags=PSG_FORM_CURSOR)
        assert plan.form == PSG_KERNEL_CURSOR
        plan.run()
        mt = plan.matched().tolist()
        assert mt[4] < 40000 and mt[:4] == [40000] * 4 and mt[5:] == [40000] * 3
        plan.close()


def _pcursor_check(torch, cases, parallel, dtype=np.float32, flags=None, reps=2):
    """Plan over `cases` in the packed cursor form: every value array and
    matched count against the oracle, `reps` runs into the same buffers."""
    from parameter_server_amd._lib import PSG_KERNEL_PACKED_CURSOR, PSG_FORM_CURSOR
    flags = PSG_FORM_CURSOR if flags is None else flags
    m = len(cases[0][1][0][1])
    plan, keep = plan_for(torch, cases, dtype=dtype, parallel=parallel, flags=flags)
    assert plan.form == PSG_KERNEL_PACKED_CURSOR
    for _ in range(reps):
        plan.run()
        mt = plan.matched().tolist()
        want_mt = []
        for j, (Dj, pushes) in enumerate(cases):
            Do, po = _oracle_keys(Dj, pushes)
            _, _, _, want, wm = O.aggregate(Do, *ALL, po, parallel, m, dtype)
            want_mt += [int(x) for x in wm]
            for i in range(m):
                assert_bitexact(keep[4 * j + 3][i].cpu().numpy()[: Dj.size], want[i])
        assert mt == want_mt
    plan.close()


def _open_end_case(seed, npush, density, nD, dtype, m):
    """Sparse pushes over a D whose last key is 2^64 - 1 (the open last tile)."""
    rng = np.random.default_rng(seed)
    D = np.unique(np.concatenate([rng.integers(1 << 63, (1 << 64) - 1, nD, dtype=np.uint64),
                                  np.array([(1 << 64) - 1], np.uint64)]))
    pushes = []
    for p in range(npush):
        k = np.sort(rng.choice(D, int(rng.binomial(D.size, density)), replace=False))
        if p == 1:
            k = np.unique(np.concatenate([k, D[-3:]]))
        pushes.append((k, [rng.standard_normal(k.size).astype(dtype) for _ in range(m)]))
    return D, pushes


@pytest.mark.parametrize("parallel", [False, True])
@pytest.mark.parametrize("dtype,m", [(np.float32, 1), (np.float64, 2)])
def test_plan_packed_cursor_form(torch_cuda, parallel, dtype, m):
    """The packed kernel's cursor form (psg_tile_packed.hip, CUR: no
    partition pass; a workgroup walks a chunk of 2048-slot tiles and two
    lanes per push find each piece from the push's cursor), chosen by
    PSG_FORM_CURSOR on packed plans of <= 256 pushes: bit-exact with the oracle's
    serialSetValue / parallelSetValue and matched counts over three jobs of
    one plan (chunk seams inside and between jobs): 256 sparse pushes with
    one dense push among them (pieces past 16 keys: the 16-key steps) and
    an empty one; 20 pushes; a D ending at 2^64 - 1 (the open last tile);
    a second run into the same buffers."""
    torch = torch_cuda
    D1, p1 = random_case(4101, dtype, m, 256, 0.004, 300_000)
    rng = np.random.default_rng(5)
    k = np.sort(rng.choice(D1, D1.size // 20, replace=False))
    p1[17] = (k, [rng.standard_normal(k.size).astype(dtype) for _ in range(m)])
    p1[40] = (np.zeros(0, np.uint64), [np.zeros(0, dtype) for _ in range(m)])
    D2, p2 = random_case(4102, dtype, m, 20, 0.005, 120_000)
    D3, p3 = _open_end_case(4103, 12, 0.006, 50_000, dtype, m)
    _pcursor_check(torch_cuda, [(D1, p1), (D2, p2), (D3, p3)], parallel, dtype)


def test_plan_packed_cursor_groups_and_unmatched(torch_cuda):
    """PSG_FORM_PACKED | PSG_FORM_CURSOR on tiles whose elements exceed one
    pass (256 pushes x ~20 keys per tile: the cursor form's later groups
    read the piece lengths back from the piece words), and pushes holding
    keys outside D (below D[0], between server keys, above D[-1]): matched
    counts and sums equal the oracle's, serial and parallel."""
    from parameter_server_amd._lib import PSG_FORM_CURSOR, PSG_FORM_PACKED
    D, pushes = random_case(4104, np.float32, 1, 256, 0.01, 200_000)
    D2, p2 = random_case(4105, np.float32, 1, 30, 0.004, 150_000)
    extra = np.array([1, 2, int(D2[100]) + 1, int(D2[-1]) + 3], np.uint64)
    for i in (3, 11):
        k, vs = p2[i]
        k2 = np.unique(np.concatenate([k, extra if i == 3 else extra[2:]]))
        p2[i] = (k2, [np.random.default_rng(i).standard_normal(k2.size).astype(np.float32)])
    for parallel in (False, True):
        _pcursor_check(torch_cuda, [(D, pushes), (D2, p2)], parallel,
                       flags=PSG_FORM_PACKED | PSG_FORM_CURSOR, reps=1)


def test_plan_packed_cursor_unsorted_push_is_reported(torch_cuda):
    """An unsorted push through the packed cursor form: two keys swapped
    inside one tile (the order check) and across far-apart tiles (the
    chunks' cursors disagree at a seam) are both reported (matched < n)
    while the other pushes of the plan stay exact."""
    torch = torch_cuda
    from parameter_server_amd import synth
    from parameter_server_amd._lib import PSG_KERNEL_PACKED_CURSOR, PSG_FORM_CURSOR
    D, pushes = synth.cfg5_shard(1, 8)
    n = [k.size for k, _ in pushes]
    for (i, j) in ((100, 101), (50, n[9] - 50)):
        bad = list(pushes)
        k = bad[9][0].copy()
        k[i], k[j] = k[j], k[i]
        bad[9] = (k, bad[9][1])
        plan, keep = plan_for(torch, [(D, bad)], flags=PSG_FORM_CURSOR)
        assert plan.form == PSG_KERNEL_PACKED_CURSOR
        plan.run()
        mt = plan.matched().tolist()
        assert mt[9] < n[9] and mt[:9] == n[:9] and mt[10:] == n[10:]
        plan.close()


def _stream_case(seed):
    """Sparse pushes over a 2 M-slot D: ~10 keys per push per 1024 slots, so
    the partition runs in stream mode (512-key chunks of each push)."""
    rng = np.random.default_rng(seed)
    D = np.unique(rng.integers(0, 1 << 50, 2_100_000, dtype=np.uint64))
    pushes = []
    for p in range(24):
        k = np.sort(rng.choice(D, 20000, replace=False))
        pushes.append((k, [rng.standard_normal(k.size).astype(np.float32)]))
    return D, pushes


def _swap_blocks(k):
    """Two 4,096-key blocks swapped: unsorted across several 512-key chunks."""
    k = k.copy()
    a, b = slice(2048, 2048 + 4096), slice(12000, 12000 + 4096)
    k[a], k[b] = k[b].copy(), k[a].copy()
    return k


def test_stream_partition_unsorted_push_across_chunks_plan(torch_cuda):
    """the stream partition no longer order-checks; an unsorted
    push (4 K-key blocks swapped, across chunk boundaries) must still be
    reported by the aggregate kernel's order check and coverage.  The plan
    runs once sorted (seg and the descriptors written), then the same push's
    device keys are swapped in place and the plan re-runs on the stale seg
    image: that push reported, the others exact."""
    torch = torch_cuda
    from parameter_server_amd._lib import PSG_PART_STREAM
    D, pushes = _stream_case(61)
    for parallel in (False, True):
        plan, keep = plan_for(torch, [(D, pushes)], parallel=parallel, flags=PSG_PART_STREAM)
        plan.run()
        assert plan.matched().tolist() == [20000] * 24
        _, _, _, want, _ = O.aggregate(D, *ALL, pushes, parallel=parallel)
        assert_bitexact(keep[3][0].cpu().numpy()[: D.size], want[0])
        bad = _swap_blocks(pushes[5][0])
        keep[1][5].copy_(torch.from_numpy(bad.view(np.int64)).cuda())
        plan.run()
        mt = plan.matched().tolist()
        assert mt[5] < 20000 and mt[:5] + mt[6:] == [20000] * 23
        plan.close()


def test_stream_partition_unsorted_push_across_chunks_context(torch_cuda):
    """The same through the server API (context flushes, stream partition
    forced): time 1 sorted (the flush's job tables and seg written), time 2
    of the same shape with one push unsorted across chunks (the reused
    descriptors, stale seg words): reported PSG_ERR_UNMATCHED; time 3 sorted
    again is exact."""
    from parameter_server_amd._lib import PSGError, PSG_ERR_UNMATCHED, PSG_PART_STREAM
    D, pushes = _stream_case(62)
    v = kvv(flags=PSG_PART_STREAM)
    v.setValue(msg(D))
    _, _, _, want, _ = O.aggregate(D, *ALL, pushes)
    for t, unsorted in ((1, False), (2, True), (3, False)):
        for p, (k, vals) in enumerate(pushes):
            kk = _swap_blocks(k) if unsorted and p == 7 else k
            v.setValue(msg(kk, vals, t=t))
        if unsorted:
            with pytest.raises(PSGError) as e:
                v.received(t)
            assert e.value.status == PSG_ERR_UNMATCHED
        else:
            (rng, a), = v.received(t)
            assert_bitexact(a, want[0])
    v.close()
