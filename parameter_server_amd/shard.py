"""Multi-GPU ingress modes for the key-range-sharded server.

Mode A ("sliced", the reference's behaviour): workers slice every push by
the server key ranges before sending (RNode::submit -> KVVector::slice ->
sliceKeyOrderedMsg, reference remote_node.cc:39-60, message.h:89-123), so
each GPU receives only its shard's pieces and the data path has no
collective.

Mode B ("unsliced"): every rank receives whole pushes; each push is cut at
the shard boundaries (the same lower_bound rule, message.h:96-99) and the
pieces are re-homed with one all-to-all of counts and one of payload
(RCCL over xGMI on GPUs, gloo in the CPU tests), after which every rank
merges the pieces it owns.
"""
from __future__ import annotations

import numpy as np


def slice_positions(keys: np.ndarray, bounds: np.ndarray) -> np.ndarray:
    """lower_bound of every shard boundary in a sorted push (message.h:96-99,
    with msg key_range = Range::all())."""
    return np.searchsorted(keys, bounds, side="left").astype(np.int64)


def exchange_pieces(pushes, bounds, dist, device=None):
    """All-to-all re-homing of the shard pieces of `pushes`.

    pushes: list of (keys uint64[n], [vals]) held by this rank.
    Returns, for this rank's shard, a list (per source rank) of lists (per
    push of that source) of (keys, [vals]) pieces, in push order.
    """
    import torch
    world = dist.get_world_size()
    m = len(pushes[0][1]) if pushes else 1
    vdt = pushes[0][1][0].dtype if pushes else np.float32
    npush = len(pushes)
    # counts[p, s] = keys of push p for shard s
    pos = [slice_positions(k, bounds) for k, _ in pushes]
    counts = np.array([np.diff(p) for p in pos], np.int64).reshape(npush, world)
    send_counts = torch.from_numpy(counts.T.copy().reshape(-1))  # [s, p]
    if device is not None:
        send_counts = send_counts.to(device)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts)
    rc = recv_counts.cpu().numpy().reshape(world, npush)  # [src, p]
    # payload: keys as int64, then each value array
    split_send = counts.sum(axis=0)  # per destination shard
    split_recv = rc.sum(axis=1)      # per source rank

    def pack(arrs_per_push, dtype):
        parts = []
        for s in range(world):
            for p in range(npush):
                a, b = pos[p][s], pos[p][s + 1]
                parts.append(arrs_per_push[p][a:b])
        return np.concatenate(parts).astype(dtype, copy=False) if parts else np.zeros(0, dtype)

    def a2a(flat_np):
        t = torch.from_numpy(np.ascontiguousarray(flat_np))
        if device is not None:
            t = t.to(device)
        out = torch.empty(int(split_recv.sum()), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t, output_split_sizes=split_recv.tolist(),
                               input_split_sizes=split_send.tolist())
        return out.cpu().numpy()

    keys = a2a(pack([k.view(np.int64) for k, _ in pushes], np.int64)).view(np.uint64)
    vals = [a2a(pack([vs[i] for _, vs in pushes], vdt)) for i in range(m)]
    result, off = [], 0
    for src in range(world):
        pieces = []
        for p in range(npush):
            c = int(rc[src, p])
            pieces.append((keys[off:off + c], [v[off:off + c] for v in vals]))
            off += c
        result.append(pieces)
    return result


def exchange_unsliced(args, rank, world, bounds, dist):
    """bench.py --ingress unsliced: each rank draws its pushes of `batch`
    aggregates (keys over the full key space), re-homes their pieces, and
    returns for each aggregate its shard's job (all sources' pieces)."""
    import torch
    from . import synth
    dev = torch.device("cuda", torch.cuda.current_device())
    jobs = []
    for j in range(args.batch):
        D, pushes = synth.overlap_pushes(1 + j + 1000 * rank, args.npush, args.n, args.overlap)
        per_src = exchange_pieces(pushes, bounds, dist, dev)
        # one aggregate per j: every source's pieces, in (source, push) order
        pieces = [pc for src in per_src for pc in src if pc[0].size]
        if pieces:
            Dsh = np.unique(np.concatenate([k for k, _ in pieces]))
            jobs.append((Dsh, pieces))
    return jobs
