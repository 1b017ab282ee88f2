"""Shard exchange through the C ABI (psg_comm_*, psg_exchange_*; RCCL) on one
GPU: a world-1 communicator, so every piece comes back to this rank through
RCCL's self send/recv.  The exchanged pieces are merged by the HIP plan and
compared bit for bit with the oracle's aggregate of the original pushes
(sliceKeyOrderedMsg, message.h:89-123, then setValue).  The multi-rank
layout logic is covered by the gloo tests in test_multi_rank.py."""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def d2h(ptr, nbytes):
    hip = C.CDLL("libamdhip64.so")
    out = np.empty(nbytes, np.uint8)
    assert hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(ptr), C.c_size_t(nbytes), 2) == 0
    return out


@pytest.mark.parametrize("dtype,m", [(np.float32, 1), (np.float64, 2)])
def test_world1_rccl_exchange_then_hip_merge(dtype, m):
    import torch
    assert torch.cuda.is_available()
    from parameter_server_amd import shard, synth
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    from parameter_server_amd.kv_vector import MergePlan, shard_bounds
    rng = np.random.default_rng(7)
    J, P = 3, 6
    aggs = []
    for j in range(J):
        D, pushes = synth.overlap_pushes(seed=31 + j, npush=P, n=40000)
        pushes = [(k, [np.asarray(v, dtype) for v in vs] +
                   [rng.standard_normal(k.size).astype(dtype) for _ in range(m - 1)])
                  for k, vs in pushes]
        aggs.append(pushes)
    ex = shard.UnslicedExchange(aggs, shard_bounds(1), None, torch.device("cuda", 0))
    assert ex.x is not None  # the RCCL path, not torch.distributed
    ex.run()
    torch.cuda.synchronize()
    x = ex.x
    sv = np.dtype(dtype).itemsize
    rkeys = d2h(x.recv_keys_ptr, 8 * x.nrecv).view(np.uint64)
    sent = np.concatenate([k for agg in aggs for k, _ in agg])
    assert np.array_equal(rkeys, sent)  # world 1: every piece back, push order
    # merge each aggregate's received pieces with the HIP plan
    jobs, outs, wants = [], [], []
    for j in range(J):
        pcs = [(ex.recv_off[0, j, p], ex.recv_cnt[0, j, p]) for p in range(P)]
        D = np.unique(np.concatenate([k for k, _ in aggs[j]]))
        dD = torch.from_numpy(D.view(np.int64)).cuda()
        o = [torch.empty(D.size, dtype=torch.float32 if dtype == np.float32 else torch.float64,
                         device="cuda") for _ in range(m)]
        outs.append((dD, o))
        jobs.append({"keys": dD.data_ptr(), "nslots": D.size,
                     "push_keys": [x.recv_keys_ptr + 8 * int(a) for a, _ in pcs],
                     "push_vals": [[x.recv_vals_ptr[i] + sv * int(a) for i in range(m)]
                                   for a, _ in pcs],
                     "push_n": [int(c) for _, c in pcs], "out": [t.data_ptr() for t in o]})
        rc, lo, hi, want, _ = O.aggregate(D, 0, (1 << 64) - 1, aggs[j], dtype=dtype)
        assert rc == 0
        wants.append(want)
    plan = MergePlan(0, PSG_F32 if dtype == np.float32 else PSG_F64, m, jobs)
    plan.run()
    torch.cuda.synchronize()
    for (dD, o), want in zip(outs, wants):
        for i in range(m):
            got = o[i].cpu().numpy()
            assert np.array_equal(got.view(np.uint8), np.asarray(want[i], dtype).view(np.uint8))
    plan.close()
    x.close()
    shard.destroy_comm(ex.comm)


def _dev_pushes(pushes, dev):
    import torch
    return [(torch.from_numpy(k.view(np.int64)).to(dev),
             [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in vs]) for k, vs in pushes]


@pytest.mark.parametrize("dtype,m", [(np.float32, 1), (np.float64, 2)])
def test_local_exchange_8_shards_layout_and_merge(dtype, m):
    """The exchange's cut + pack with 8 shards on one device (the RCCL path's
    multi-shard layout, psg_exchange_create_local): every shard's packed
    pieces equal the oracle's sliceKeyOrderedMsg cut (message.h:89-123) at
    evenDivide(8) (range.h:85-98), in push order; merging each shard's
    pieces with the HIP plan equals the oracle's aggregate of that shard's
    key range, bit for bit; a second run lands in the same buffers."""
    import torch
    from parameter_server_amd import shard, synth
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    from parameter_server_amd.kv_vector import MergePlan, shard_bounds
    S = 8
    _, pushes = synth.uniform_pushes(seed=41, npush=12, n=20000, dtype=dtype, m=m, union=False)
    pushes.append((np.zeros(0, np.uint64), [np.zeros(0, dtype)] * m))  # empty push
    # a push confined to one shard and one holding the edge keys of shard 3
    b = shard_bounds(S)
    pushes.append((np.arange(b[5] + 10, b[5] + 3000, dtype=np.uint64),
                   [np.full(2990, 0.5, dtype)] * m))
    edge = np.array([b[3] - 1, b[3], b[4] - 1, b[4]], np.uint64)
    pushes.append((edge, [np.arange(4, dtype=dtype) + 1] * m))
    dev = torch.device("cuda", 0)
    dp = _dev_pushes(pushes, dev)
    x = shard.LocalExchange(0, dp, S, PSG_F32 if dtype == np.float32 else PSG_F64)
    for _ in range(2):
        x.run()
    torch.cuda.synchronize()
    assert x.status() == 0
    sv = np.dtype(dtype).itemsize
    ntot = int(x.send_cnt.sum())
    assert ntot == sum(k.size for k, _ in pushes)
    keys = d2h(x.keys_ptr, 8 * ntot).view(np.uint64)
    vals = [d2h(p, sv * ntot).view(dtype) for p in x.vals_ptr]
    ALL = (0, (1 << 64) - 1)
    for p, (k, vs) in enumerate(pushes):
        pos, _ = O.slice_key_ordered(k, *ALL, b)
        for s in range(S):
            a, e = int(pos[s]), int(pos[s + 1])
            assert x.send_cnt[s, p] == e - a
            o = int(x.send_off[s, p])
            assert np.array_equal(keys[o:o + e - a], k[a:e])
            for i in range(m):
                assert vals[i][o:o + e - a].tobytes() == vs[i][a:e].tobytes()
    # each shard merged by the HIP plan = the oracle over that shard's range
    D = np.unique(np.concatenate([k for k, _ in pushes]))
    jobs, outs, wants = [], [], []
    for s in range(S):
        lo, hi = O.find_range(D, int(b[s]), int(b[s + 1]))
        Ds = D[lo:hi]
        dD = torch.from_numpy(Ds.view(np.int64)).to(dev)
        o = [torch.empty(max(1, Ds.size), dtype=torch.float32 if dtype == np.float32
                         else torch.float64, device=dev) for _ in range(m)]
        pcs = x.pieces(s)
        jobs.append({"keys": dD.data_ptr(), "nslots": int(Ds.size),
                     "push_keys": [x.keys_ptr + 8 * a for a, _ in pcs],
                     "push_vals": [[x.vals_ptr[i] + sv * a for i in range(m)] for a, _ in pcs],
                     "push_n": [c for _, c in pcs], "out": [t.data_ptr() for t in o]})
        outs.append((dD, o, Ds.size))
        pieces = [(keys[a:a + c], [v[a:a + c] for v in vals]) for a, c in pcs]
        rc, _, _, want, _ = O.aggregate(D, int(b[s]), int(b[s + 1]), pieces, dtype=dtype)
        assert rc == 0
        wants.append(want)
    plan = MergePlan(0, PSG_F32 if dtype == np.float32 else PSG_F64, m, jobs)
    plan.run()
    torch.cuda.synchronize()
    want_n = [c for s in range(S) for _, c in x.pieces(s)]
    assert list(plan.matched()) == want_n
    for (dD, o, n), want in zip(outs, wants):
        for i in range(m):
            got = o[i].cpu().numpy()[:n]
            assert got.tobytes() == np.asarray(want[i], dtype).tobytes()
    plan.close()
    x.close()


def test_local_exchange_detects_changed_keys():
    """A run re-cuts the pushes on the device: keys changed after set-up so
    that a piece boundary moves are reported by psg_exchange_status
    (PSG_ERR_SIZE) instead of being shipped silently with the old cut."""
    import torch
    from parameter_server_amd import shard, synth
    from parameter_server_amd._lib import PSG_F32, PSGError
    from parameter_server_amd.kv_vector import shard_bounds
    _, pushes = synth.uniform_pushes(seed=43, npush=4, n=5000, union=False)
    dp = _dev_pushes(pushes, torch.device("cuda", 0))
    x = shard.LocalExchange(0, dp, 8, PSG_F32)
    x.run()
    assert x.status() == 0
    # move push 2's first key of shard 5 below the shard 5 boundary
    k = pushes[2][0]
    b = shard_bounds(8)
    i = int(np.searchsorted(k, b[5]))
    newk = k.copy()
    newk[i] = np.uint64(b[5] - 1)
    assert newk[i - 1] < newk[i]
    dp[2][0].copy_(torch.from_numpy(newk.view(np.int64)))
    x.run()
    with pytest.raises(PSGError):
        x.status()
    x.close()


def _threads(fns):
    """Run fns[r]() for every rank r on its own thread (loopback ranks must
    enter the collective rounds concurrently); returns (results, errors)."""
    import threading
    res, err = [None] * len(fns), [None] * len(fns)

    def body(r):
        try:
            res[r] = fns[r]()
        except BaseException as e:  # noqa: BLE001 - reported per rank
            err[r] = e

    ts = [threading.Thread(target=body, args=(r,)) for r in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
        assert not t.is_alive(), "a loopback rank hung"
    return res, err


@pytest.mark.parametrize("dtype,m,direct", [(np.float32, 1, False), (np.float64, 2, False),
                                            (np.float32, 1, True)])
def test_loopback_8_ranks_exchange_then_hip_merge(dtype, m, direct):
    """The multi-rank exchange at S = 8 ranks (psg_comm_init_loopback: 8
    ranks of one process on one GPU, one host thread each), cfg5-shaped
    pushes (murmur-shuffled uniform ranks, 8 whole pushes per rank): the
    collective count round, the receive offsets and the pairing of sends and
    receives across peers run exactly as over RCCL.  Per rank, recv counts
    equal the oracle's sliceKeyOrderedMsg cut (message.h:89-123) at
    evenDivide(8) of every source's pushes, the received keys/values are
    those pieces in (source, push) order, and the HIP plan's merge of them
    equals the oracle's aggregate over the rank's key range, bit for bit.
    Two runs land in the same buffers.  `direct`: peer-bound pieces sent
    straight from the push arrays (psg_exchange_set_direct), one send per
    piece and array, received in the same layout."""
    import torch
    from parameter_server_amd import shard, synth
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    from parameter_server_amd.kv_vector import MergePlan, shard_bounds
    S, PR = 8, 8
    _, pushes = synth.uniform_pushes(seed=51, npush=S * PR, n=12000, dtype=dtype, m=m,
                                     union=False)
    b = shard_bounds(S)
    # a push holding the shard edges, one confined to shard 6, an empty one
    pushes[3] = (np.array([b[1] - 1, b[1], b[2], b[7] - 1, b[7]], np.uint64),
                 [np.arange(5, dtype=dtype) - 2 for _ in range(m)])
    pushes[20] = (np.arange(b[6] + 5, b[6] + 2005, dtype=np.uint64),
                  [np.full(2000, 0.25, dtype) for _ in range(m)])
    pushes[41] = (np.zeros(0, np.uint64), [np.zeros(0, dtype) for _ in range(m)])
    dev = torch.device("cuda", 0)
    comms = shard.loopback_comms(0, S)
    held = [_dev_pushes(pushes[r * PR:(r + 1) * PR], dev) for r in range(S)]
    vt = PSG_F32 if dtype == np.float32 else PSG_F64
    xs, err = _threads([lambda r=r: shard.RcclExchange(comms[r], held[r], S, vt)
                        for r in range(S)])
    assert not any(err), err
    for x in xs:
        x.set_direct(direct)
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    for _ in range(2):
        _, err = _threads([lambda r=r: xs[r].run(streams[r].cuda_stream) for r in range(S)])
        assert not any(err), err
    torch.cuda.synchronize()
    sv = np.dtype(dtype).itemsize
    ALL = (0, (1 << 64) - 1)
    cut = [O.slice_key_ordered(k, *ALL, b)[0].astype(np.int64) for k, _ in pushes]
    D = np.unique(np.concatenate([k for k, _ in pushes]))
    for r in range(S):
        x = xs[r]
        assert x.status() == 0
        want_cnt = np.array([[cut[src * PR + p][r + 1] - cut[src * PR + p][r] for p in range(PR)]
                             for src in range(S)], np.int64)
        assert np.array_equal(x.recv_cnt, want_cnt), f"rank {r} recv counts"
        assert x.nsent == sum(int(cut[r * PR + p][s + 1] - cut[r * PR + p][s])
                              for p in range(PR) for s in range(S) if s != r)
        rk = d2h(x.recv_keys_ptr, 8 * x.nrecv).view(np.uint64)
        rv = [d2h(p, sv * x.nrecv).view(dtype) for p in x.recv_vals_ptr]
        pieces = []
        for src in range(S):
            for p in range(PR):
                k, vs = pushes[src * PR + p]
                a, e = int(cut[src * PR + p][r]), int(cut[src * PR + p][r + 1])
                o = int(x.recv_off[src, p])
                assert np.array_equal(rk[o:o + e - a], k[a:e]), f"rank {r} keys of {src},{p}"
                for i in range(m):
                    assert rv[i][o:o + e - a].tobytes() == vs[i][a:e].tobytes()
                if e > a:
                    pieces.append((k[a:e], [v[a:e] for v in vs]))
        # the rank's merge of what it received (arrival order: source, push)
        lo, hi = O.find_range(D, int(b[r]), int(b[r + 1]))
        dD = torch.from_numpy(D[lo:hi].view(np.int64)).to(dev)
        o = [torch.empty(max(1, hi - lo), dtype=torch.float32 if dtype == np.float32
                         else torch.float64, device=dev) for _ in range(m)]
        pcs = x.pieces()
        plan = MergePlan(0, vt, m, [{
            "keys": dD.data_ptr(), "nslots": hi - lo,
            "push_keys": [x.recv_keys_ptr + 8 * a for a, _ in pcs],
            "push_vals": [[x.recv_vals_ptr[i] + sv * a for i in range(m)] for a, _ in pcs],
            "push_n": [c for _, c in pcs], "out": [t.data_ptr() for t in o]}])
        plan.run()
        torch.cuda.synchronize()
        assert list(plan.matched()) == [c for _, c in pcs]
        rc, _, _, want, _ = O.aggregate(D, int(b[r]), int(b[r + 1]), pieces, dtype=dtype)
        assert rc == 0
        for i in range(m):
            assert o[i].cpu().numpy()[:hi - lo].tobytes() == np.asarray(want[i], dtype).tobytes()
        plan.close()
    for x in xs:
        x.close()
    for c in comms:
        shard.destroy_comm(c)


def test_loopback_bad_rank_fails_everywhere_without_hang():
    """One rank of 8 passes a bad dtype to psg_exchange_create: it still
    takes part in the collective count round (with an error word), so every
    rank returns an error instead of waiting on it; the communicators are
    usable afterwards (a good exchange on the same ranks succeeds)."""
    import time
    import torch
    from parameter_server_amd import shard, synth
    from parameter_server_amd._lib import PSG_F32, PSGError
    S = 8
    _, pushes = synth.uniform_pushes(seed=53, npush=S, n=3000, union=False)
    dev = torch.device("cuda", 0)
    comms = shard.loopback_comms(0, S)
    held = [_dev_pushes(pushes[r:r + 1], dev) for r in range(S)]
    t0 = time.time()
    _, err = _threads([lambda r=r: shard.RcclExchange(comms[r], held[r], S,
                                                      99 if r == 3 else PSG_F32)
                       for r in range(S)])
    assert time.time() - t0 < 60
    assert all(isinstance(e, PSGError) for e in err), err
    xs, err = _threads([lambda r=r: shard.RcclExchange(comms[r], held[r], S, PSG_F32)
                        for r in range(S)])
    assert not any(err), err
    _, err = _threads([lambda r=r: xs[r].run(None) for r in range(S)])
    assert not any(err), err
    torch.cuda.synchronize()
    assert sum(x.nrecv for x in xs) == sum(k.size for k, _ in pushes)
    for x in xs:
        x.close()
    for c in comms:
        shard.destroy_comm(c)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("direct", [False, True])
def test_loopback_8_ranks_full_cfg5(direct):
    """BASELINE.json configs[4] at its real size through the 8-rank exchange:
    256 pushes x 262,144 murmur-shuffled uniform keys (1e9-rank space, f32),
    32 whole pushes held per rank (the bench's unsliced leg at N = 8; ranks
    are loopback ranks of one process on one GPU, psg_comm_init_loopback).
    Per rank: the received counts equal the oracle's sliceKeyOrderedMsg cut
    (message.h:89-123) at evenDivide(8) (range.h:85-98) of every source's
    pushes; the received keys and values are those pieces in (source, push)
    order, byte for byte; the HIP merge of the received buffers equals the
    HIP merge of the same pieces staged separately (the sliced leg) and the
    oracle's serialSetValue over the rank's range (orc_aggregate_scatter_serial),
    bit for bit.  Pack mode and direct mode."""
    import torch
    from parameter_server_amd import shard, synth
    from parameter_server_amd._lib import PSG_F32
    from parameter_server_amd.kv_vector import MergePlan, shard_bounds
    S = 8
    _, pushes = synth.uniform_pushes(seed=5, union=False)
    P = len(pushes)
    assert P == 256 and all(k.size == 262144 for k, _ in pushes)
    PR = P // S
    b = shard_bounds(S)
    dev = torch.device("cuda", 0)
    comms = shard.loopback_comms(0, S)
    held = [_dev_pushes(pushes[r * PR:(r + 1) * PR], dev) for r in range(S)]
    xs, err = _threads([lambda r=r: shard.RcclExchange(comms[r], held[r], S, PSG_F32)
                        for r in range(S)])
    assert not any(err), err
    try:
        for x in xs:
            x.set_direct(direct)
        streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
        for _ in range(2):
            _, err = _threads([lambda r=r: xs[r].run(streams[r].cuda_stream) for r in range(S)])
            assert not any(err), err
        torch.cuda.synchronize()
        ALL = (0, (1 << 64) - 1)
        cut = [O.slice_key_ordered(k, *ALL, b)[0].astype(np.int64) for k, _ in pushes]
        assert sum(x.nrecv for x in xs) == P * 262144
        for r in range(S):
            x = xs[r]
            assert x.status() == 0
            want_cnt = np.array([[cut[s * PR + p][r + 1] - cut[s * PR + p][r] for p in range(PR)]
                                 for s in range(S)], np.int64)
            assert np.array_equal(x.recv_cnt, want_cnt), f"rank {r} recv counts"
            pieces = []
            for s in range(S):
                for p in range(PR):
                    k, vs = pushes[s * PR + p]
                    a, e = int(cut[s * PR + p][r]), int(cut[s * PR + p][r + 1])
                    assert int(x.recv_off[s, p]) == sum(pc[0].size for pc in pieces)
                    pieces.append((k[a:e], [vs[0][a:e]]))
            rk = d2h(x.recv_keys_ptr, 8 * x.nrecv).view(np.uint64)
            rv = d2h(x.recv_vals_ptr[0], 4 * x.nrecv)
            assert np.array_equal(rk, np.concatenate([k for k, _ in pieces])), f"rank {r} keys"
            assert rv.tobytes() == np.concatenate([v[0] for _, v in pieces]).tobytes()
            del rk, rv
            # the rank's merge of the received buffers vs the same pieces staged apart
            Dr = np.unique(np.concatenate([k for k, _ in pieces]))
            dD = torch.from_numpy(Dr.view(np.int64)).to(dev)
            pcs = x.pieces()
            o_x = torch.empty(Dr.size, dtype=torch.float32, device=dev)
            plan_x = MergePlan(0, PSG_F32, 1, [{
                "keys": dD.data_ptr(), "nslots": int(Dr.size),
                "push_keys": [x.recv_keys_ptr + 8 * a for a, _ in pcs],
                "push_vals": [[x.recv_vals_ptr[0] + 4 * a] for a, _ in pcs],
                "push_n": [c for _, c in pcs], "out": [o_x.data_ptr()]}])
            sp = _dev_pushes(pieces, dev)
            o_s = torch.empty(Dr.size, dtype=torch.float32, device=dev)
            plan_s = MergePlan(0, PSG_F32, 1, [{
                "keys": dD.data_ptr(), "nslots": int(Dr.size),
                "push_keys": [k.data_ptr() for k, _ in sp],
                "push_vals": [[v[0].data_ptr()] for _, v in sp],
                "push_n": [int(k.size) for k, _ in pieces], "out": [o_s.data_ptr()]}])
            plan_x.run()
            plan_s.run()
            torch.cuda.synchronize()
            assert list(plan_x.matched()) == [c for _, c in pcs]
            assert torch.equal(o_x.view(torch.int32), o_s.view(torch.int32)), f"rank {r} merge"
            if r in (0, 5):  # the oracle on two ranks (one at each end of the key space)
                rc, lo, hi, want, _ = O.aggregate_scatter(Dr, int(b[r]), int(b[r + 1]), pieces,
                                                          parallel=False)
                assert rc == 0 and (lo, hi) == (0, Dr.size)
                assert o_x.cpu().numpy().tobytes() == np.asarray(want[0], np.float32).tobytes()
            plan_x.close()
            plan_s.close()
            del sp, dD, o_x, o_s
    finally:
        for x in xs:
            x.close()
        for c in comms:
            shard.destroy_comm(c)
