"""Multi-rank paths on CPU (gloo, world size 2) and the sharding rule.

Mode A (the reference's behaviour): workers slice pushes by server key range
(sliceKeyOrderedMsg, reference message.h:89-123; shard ranges
Range::all().evenDivide, range.h:85-98 / linear_method.cc:137-145), so
the per-shard aggregates concatenate to the unsharded one.  Mode B: whole
pushes are re-homed with one all-to-all (parameter_server_amd/shard.py) and
each rank merges the pieces it owns.  The merges here are the oracle's
(these tests check the partition/exchange logic, not the kernels; the GPU
merge is pinned to the oracle in test_gpu_parity.py).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_py as O  # noqa: E402
from parameter_server_amd import shard as S  # noqa: E402
from parameter_server_amd import synth  # noqa: E402
from parameter_server_amd.kv_vector import shard_bounds  # noqa: E402

ALL = (0, (1 << 64) - 1)


def _pushes(seed, npush=4, n=3000):
    return synth.overlap_pushes(seed, npush, n, 0.1)


def _merge(D, kb, ke, pushes, parallel=False):
    rc, lo, hi, outs, matched = O.aggregate(D, kb, ke, pushes, parallel, 1)
    assert rc == 0
    return lo, hi, outs, matched


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("parallel", [False, True])
def test_mode_a_shards_concatenate_to_unsharded(world, parallel):
    D, pushes = _pushes(11 + world)
    _, _, full, _ = _merge(D, *ALL, pushes, parallel)
    b = shard_bounds(world)
    got = []
    for s in range(world):
        pieces = []
        for k, vs in pushes:
            pos = S.slice_positions(k, b)
            a, e = int(pos[s]), int(pos[s + 1])
            pieces.append((k[a:e], [v[a:e] for v in vs]))
        # a shard's server keys: D restricted to its range (findRange)
        lo, hi, outs, matched = _merge(D, int(b[s]), int(b[s + 1]), pieces, parallel)
        assert list(matched) == [pc[0].size for pc in pieces]
        got.append(outs[0])
    cat = np.concatenate(got)
    assert cat.tobytes() == full[0].tobytes()  # bit-exact


def test_slice_positions_match_oracle_slice():
    D, pushes = _pushes(5)
    b = shard_bounds(8)
    for k, _ in pushes:
        pos, valid = O.slice_key_ordered(k, *ALL, b)
        assert np.array_equal(S.slice_positions(k, b).astype(np.uint64), pos)
        assert valid.all()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _exchange_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = shard_bounds(world)
        mine = _pushes(100 + rank)[1]
        per_src = S.exchange_pieces(mine, b, dist)
        # every source's pieces for my shard, in (source, push) arrival order
        src_pushes = [_pushes(100 + r)[1] for r in range(world)]
        for src in range(world):
            for p, (k, vs) in enumerate(src_pushes[src]):
                pos = S.slice_positions(k, b)
                a, e = int(pos[rank]), int(pos[rank + 1])
                gk, gv = per_src[src][p]
                assert np.array_equal(gk, k[a:e])
                assert gv[0].tobytes() == vs[0][a:e].tobytes()
        # merging the received pieces = the shard of the unsharded merge of
        # all sources' pushes in the same order
        allp = [pc for src in range(world) for pc in src_pushes[src]]
        D = np.unique(np.concatenate([k for k, _ in allp]))
        _, _, full, _ = _merge(D, *ALL, allp)
        lo, hi = O.find_range(D, int(b[rank]), int(b[rank + 1]))
        pieces = [pc for src in range(world) for pc in per_src[src]]
        _, _, outs, matched = _merge(D, int(b[rank]), int(b[rank + 1]), pieces)
        assert list(matched) == [pc[0].size for pc in pieces]
        assert outs[0].tobytes() == full[0][lo:hi].tobytes()
        # bench's whole-job reduction: max wall over ranks, sum of kv
        import bench
        wall, kv = bench.reduce_over_ranks(1.0 + rank, 10 * (rank + 1), dist,
                                           torch.device("cpu"))
        assert wall == float(world) and kv == 10.0 * world * (world + 1) / 2
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_mode_b_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res


def _timed_exchange_worker(rank, world, port, q):
    """UnslicedExchange (the timed mode-B step of bench.py): after run(),
    aggregate j's pieces for this shard are every source's pushes of j cut
    at the shard bounds, in (source, push) order, bit for bit."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = shard_bounds(world)
        J = 3
        aggs = {r: [_pushes(200 + 10 * r + j)[1] for j in range(J)] for r in range(world)}
        ex = S.UnslicedExchange(aggs[rank], b, dist, torch.device("cpu"))
        ex.run()
        ex.run()  # a second step lands in the same buffers
        rk = ex.recv_keys.numpy().view(np.uint64)
        rv = ex.recv_vals[0].numpy()
        for j in range(J):
            want = []
            for src in range(world):
                for k, vs in aggs[src][j]:
                    pos = S.slice_positions(k, b)
                    a, e = int(pos[rank]), int(pos[rank + 1])
                    if e > a:
                        want.append((k[a:e], vs[0][a:e]))
            got = ex.pieces(j)
            assert len(got) == len(want)
            for (off, c), (wk, wv) in zip(got, want):
                assert np.array_equal(rk[off:off + c], wk)
                assert rv[off:off + c].tobytes() == wv.tobytes()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_mode_b_timed_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timed_exchange_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res
