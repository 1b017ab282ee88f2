"""Multi-GPU ingress modes for the key-range-sharded server.

Mode A ("sliced", the reference's behaviour): workers slice every push by
the server key ranges before sending (RNode::submit -> KVVector::slice ->
sliceKeyOrderedMsg, reference remote_node.cc:39-60, message.h:89-123), so
each GPU receives only its shard's pieces and the data path has no
collective.

Mode B ("unsliced"): every rank receives whole pushes; each push is cut at
the shard boundaries (the same lower_bound rule, message.h:96-99) and the
pieces are re-homed with one exchange of counts and one of payload, after
which every rank merges the pieces it owns.  On GPUs the exchange is the
C ABI's psg_exchange_* over a psg_comm (RCCL over xGMI, hand-written cut
and pack kernels; :class:`RcclExchange`); the torch.distributed forms below
(:func:`exchange_pieces`, :class:`UnslicedExchange` on CPU tensors) restate
the same layout for the gloo tests of the partition/exchange logic.
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


class UnslicedExchange:
    """Mode B inside a timed step (bench.py's cfg5 "unsliced" leg uses the
    RCCL form directly, :class:`RcclExchange`).

    The rank holds whole pushes of `len(aggs)` aggregates on its device
    (aggs[j] = [(keys, [vals])] per push).  A step re-homes them: one gather
    into destination-major order (shard s's pieces of every push are the
    contiguous runs [pos_s, pos_s+1) of the sorted push, message.h:96-99),
    then one all-to-all for the keys and one per value array (RCCL over
    xGMI on GPUs; gloo in the CPU tests; a plain copy at world size 1).
    The slice positions are computed once at set-up (a sorted push's cut
    is data-dependent but costs S binary searches, the partition kernel's
    work class).  After a step, source rank src's piece of aggregate j,
    push p starts at `recv_off[src, j, p]` with `recv_cnt[src, j, p]` keys:
    the layout the merge plan points at.  The received data is the tensors
    `recv_keys` / `recv_vals` (torch.distributed form), or device memory at
    `x.recv_keys_ptr` / `x.recv_vals_ptr` (the GPU form, `x` an
    :class:`RcclExchange`).  `bounds` must be evenDivide(world), the
    server ranges both forms cut at.
    """

    def __init__(self, aggs, bounds, dist, device):
        import torch
        self.dist = dist
        world = dist.get_world_size() if dist is not None else 1
        J, P = len(aggs), len(aggs[0])
        m = len(aggs[0][0][1])
        vdt = aggs[0][0][1][0].dtype
        self.x = None
        from .kv_vector import shard_bounds
        if not np.array_equal(np.asarray(bounds, np.uint64), shard_bounds(world)):
            raise ValueError("UnslicedExchange cuts at evenDivide(world) (linear_method.cc:"
                             "137-145); other bounds are not supported")
        if torch.device(device).type == "cuda":
            # GPUs: the C ABI's RCCL exchange (cut + pack kernels, grouped
            # send/recv per peer); bounds are evenDivide(world) there too
            from ._lib import PSG_F32, PSG_F64
            dev = torch.device(device)
            rank = dist.get_rank() if dist is not None else 0
            self._dev_pushes = [(torch.from_numpy(k.view(np.int64)).to(dev),
                                 [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in vs])
                                for agg in aggs for k, vs in agg]
            self.comm = make_comm(dev.index or 0, rank, world, dist)
            self.x = RcclExchange(self.comm, self._dev_pushes, world,
                                  PSG_F32 if vdt == np.float32 else PSG_F64)
            self.world, self.J, self.P, self.m = world, J, P, m
            self.recv_cnt = self.x.recv_cnt.reshape(world, J, P)
            self.recv_off = self.x.recv_off.reshape(world, J, P)
            self.sent_bytes = int(self.x.nsent) * (8 + m * np.dtype(vdt).itemsize)
            return
        flat_k, flat_v, perm_parts = [], [[] for _ in range(m)], []
        cnt = np.zeros((world, J, P), np.int64)  # send counts [dest, j, p]
        base = 0
        starts = np.zeros((J, P), np.int64)
        pos = {}
        for j in range(J):
            for p in range(P):
                k, vs = aggs[j][p]
                pos[j, p] = slice_positions(k, bounds)
                cnt[:, j, p] = np.diff(pos[j, p])
                starts[j, p] = base
                base += k.size
                flat_k.append(k.view(np.int64))
                for i in range(m):
                    flat_v[i].append(vs[i])
        for s in range(world):
            for j in range(J):
                for p in range(P):
                    a, e = int(pos[j, p][s]), int(pos[j, p][s + 1])
                    perm_parts.append(np.arange(starts[j, p] + a, starts[j, p] + e, dtype=np.int64))
        perm = np.concatenate(perm_parts) if perm_parts else np.zeros(0, np.int64)
        self.send_split = cnt.sum(axis=(1, 2)).tolist()
        send_cnt = torch.from_numpy(cnt.reshape(-1).copy()).to(device)
        if world > 1:
            recv_cnt = torch.empty_like(send_cnt)
            dist.all_to_all_single(recv_cnt, send_cnt)
        else:
            recv_cnt = send_cnt.clone()
        self.recv_cnt = recv_cnt.cpu().numpy().reshape(world, J, P)
        self.recv_split = self.recv_cnt.sum(axis=(1, 2)).tolist()
        self.recv_off = (np.cumsum(self.recv_cnt.reshape(-1)) - self.recv_cnt.reshape(-1)).reshape(
            world, J, P)
        self.world, self.J, self.P, self.m = world, J, P, m
        self.flat_keys = torch.from_numpy(np.concatenate(flat_k)).to(device)
        self.flat_vals = [torch.from_numpy(np.concatenate(v).astype(vdt, copy=False)).to(device)
                          for v in flat_v]
        # int32 gather indices when they fit (half the index traffic)
        self.perm = torch.from_numpy(perm.astype(np.int32) if base < 2 ** 31 else perm).to(device)
        nrecv = int(sum(self.recv_split))
        self.send_keys = torch.empty_like(self.flat_keys)
        self.send_vals = [torch.empty_like(v) for v in self.flat_vals]
        self.recv_keys = torch.empty(nrecv, dtype=torch.int64, device=device)
        self.recv_vals = [torch.empty(nrecv, dtype=v.dtype, device=device) for v in self.flat_vals]
        self.sent_bytes = int(self.flat_keys.numel()) * (8 + sum(v.element_size() for v in self.flat_vals))

    def run(self):
        """One step's re-homing (enqueued on the current stream)."""
        import torch
        if self.x is not None:
            self.x.run(torch.cuda.current_stream().cuda_stream)
            return
        if self.world == 1:  # one shard: the pushes are already in send order
            pairs = [(self.recv_keys, self.flat_keys)] + list(zip(self.recv_vals, self.flat_vals))
        else:
            torch.index_select(self.flat_keys, 0, self.perm, out=self.send_keys)
            for src, dst in zip(self.flat_vals, self.send_vals):
                torch.index_select(src, 0, self.perm, out=dst)
            pairs = [(self.recv_keys, self.send_keys)] + list(zip(self.recv_vals, self.send_vals))
        for out, inp in pairs:
            if self.world > 1:
                self.dist.all_to_all_single(out, inp, output_split_sizes=self.recv_split,
                                            input_split_sizes=self.send_split)
            else:
                out.copy_(inp)

    def pieces(self, j):
        """Aggregate j's received pieces in (source, push) arrival order:
        [(offset, count)] into recv_keys / recv_vals (empty pieces dropped)."""
        return [(int(self.recv_off[s, j, p]), int(self.recv_cnt[s, j, p]))
                for s in range(self.world) for p in range(self.P) if self.recv_cnt[s, j, p]]


# --------------------------------------------------------------------------
# RCCL through the C ABI (include/psg.h: psg_comm_*, psg_exchange_*)
# --------------------------------------------------------------------------
def make_comm(device: int, rank: int = 0, world: int = 1, dist=None):
    """A psg_comm for this rank: rank 0 makes the RCCL unique id and `dist`
    (any initialised torch.distributed group) carries it to the others."""
    import ctypes as C
    from . import _lib
    L = _lib.lib()
    idb = (C.c_uint8 * 128)()
    if rank == 0:
        _lib.check(L.psg_comm_unique_id(idb))
    if world > 1:
        obj = [bytes(idb)]
        dist.broadcast_object_list(obj, src=0)
        C.memmove(idb, obj[0], 128)
    h = C.c_void_p()
    _lib.check(L.psg_comm_init(device, world, idb, rank, C.byref(h)))
    return h


def destroy_comm(h) -> None:
    from . import _lib
    _lib.lib().psg_comm_destroy(h)


def loopback_comms(device: int, world: int):
    """`world` psg_comm ranks living in this process on one device
    (psg_comm_init_loopback): the exchange's collective rounds with RCCL's
    pairing rule, each matched send/recv a device copy.  Drive each rank
    from its own thread (ctypes releases the GIL), all ranks concurrently,
    as RCCL ranks run in their own processes."""
    import ctypes as C
    from . import _lib
    hs = (C.c_void_p * world)()
    _lib.check(_lib.lib().psg_comm_init_loopback(device, world, hs))
    return [C.c_void_p(hs[r]) for r in range(world)]


class RcclExchange:
    """Mode B re-homing of this rank's device-resident pushes through
    psg_exchange_* (one grouped RCCL send/recv per peer per step).

    pushes: [(keys, [vals] * m)] torch CUDA tensors (keys int64 holding the
    uint64 keys, sorted).  After run(), shard `rank` holds for each source
    src and push p the piece (offset, count) = pieces()[src][p] in
    recv_keys_ptr / recv_vals_ptr (device addresses)."""

    def __init__(self, comm, pushes, world: int, dtype: int):
        import ctypes as C
        from . import _lib
        self._L = _lib.lib()
        self.world, self.P = world, len(pushes)
        self.m = len(pushes[0][1]) if pushes else 1
        self._keep = pushes
        kp = (C.c_void_p * max(1, self.P))(*[k.data_ptr() for k, _ in pushes])
        ns = (C.c_uint64 * max(1, self.P))(*[k.numel() for k, _ in pushes])
        vp = (C.c_void_p * max(1, self.P * self.m))(*[v.data_ptr() for _, vs in pushes
                                                      for v in vs])
        h = C.c_void_p()
        _lib.check(self._L.psg_exchange_create(comm, dtype, self.m, self.P, kp, ns, vp,
                                               C.byref(h)))
        self._h = h
        keys = C.c_void_p()
        vals = (C.c_void_p * self.m)()
        nrecv, nsent = C.c_uint64(), C.c_uint64()
        cnt = np.zeros(max(1, world * self.P), np.uint64)
        _lib.check(self._L.psg_exchange_recv(h, C.byref(keys), vals, C.byref(nrecv),
                                             cnt.ctypes.data, C.byref(nsent)))
        self.recv_keys_ptr = keys.value
        self.recv_vals_ptr = [vals[i] for i in range(self.m)]
        self.nrecv, self.nsent = nrecv.value, nsent.value
        self.recv_cnt = cnt[: world * self.P].reshape(world, self.P).astype(np.int64)
        flat = self.recv_cnt.reshape(-1)
        self.recv_off = (np.cumsum(flat) - flat).reshape(world, self.P)

    def set_direct(self, on: bool = True) -> None:
        """psg_exchange_set_direct: peer-bound pieces sent straight from the
        push arrays (no pack copy)."""
        from . import _lib
        _lib.check(self._L.psg_exchange_set_direct(self._h, 1 if on else 0))

    def run(self, stream=None) -> None:
        from . import _lib
        _lib.check(self._L.psg_exchange_run(self._h, stream))

    def status(self) -> int:
        """Cut positions of any run that differed from the set-up layout
        (pushes changed since create); raises PSGError if nonzero."""
        import ctypes as C
        from . import _lib
        n = C.c_uint64()
        _lib.check(self._L.psg_exchange_status(self._h, C.byref(n)))
        return n.value

    def send_layout(self):
        """(keys_ptr, [vals_ptr], send_cnt[S, P]) of the packed send buffers."""
        return _send_layout(self._L, self._h, self.world, self.P, self.m)

    def pieces(self):
        """[(offset, count)] per (source, push), arrival order, empties dropped."""
        return [(int(self.recv_off[s, p]), int(self.recv_cnt[s, p]))
                for s in range(self.world) for p in range(self.P) if self.recv_cnt[s, p]]

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.psg_exchange_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def _send_layout(L, h, S, P, m):
    import ctypes as C
    from . import _lib
    keys = C.c_void_p()
    vals = (C.c_void_p * m)()
    cnt = np.zeros(max(1, S * P), np.uint64)
    _lib.check(L.psg_exchange_send_layout(h, C.byref(keys), vals, cnt.ctypes.data))
    return keys.value, [vals[i] for i in range(m)], cnt[: S * P].reshape(S, P).astype(np.int64)


class LocalExchange:
    """The exchange's slice-and-pack for `nshards` virtual shards on one
    device, no communicator (psg_exchange_create_local): each run re-cuts
    the pushes on the device (checked against the set-up layout) and packs
    shard s's pieces of every push destination-major.  Tests the multi-shard
    layout of the RCCL path on one GPU.

    pushes: [(keys, [vals] * m)] torch CUDA tensors (keys int64 holding the
    sorted uint64 keys)."""

    def __init__(self, device: int, pushes, nshards: int, dtype: int):
        import ctypes as C
        from . import _lib
        self._L = _lib.lib()
        self.S, self.P = nshards, len(pushes)
        self.m = len(pushes[0][1]) if pushes else 1
        self._keep = pushes
        kp = (C.c_void_p * max(1, self.P))(*[k.data_ptr() for k, _ in pushes])
        ns = (C.c_uint64 * max(1, self.P))(*[k.numel() for k, _ in pushes])
        vp = (C.c_void_p * max(1, self.P * self.m))(*[v.data_ptr() for _, vs in pushes
                                                      for v in vs])
        h = C.c_void_p()
        _lib.check(self._L.psg_exchange_create_local(device, nshards, dtype, self.m, self.P, kp,
                                                     ns, vp, C.byref(h)))
        self._h = h
        self.keys_ptr, self.vals_ptr, self.send_cnt = _send_layout(self._L, h, nshards, self.P,
                                                                   self.m)
        flat = self.send_cnt.reshape(-1)
        self.send_off = (np.cumsum(flat) - flat).reshape(nshards, self.P)

    def run(self, stream=None) -> None:
        from . import _lib
        _lib.check(self._L.psg_exchange_run(self._h, stream))

    def status(self) -> int:
        import ctypes as C
        from . import _lib
        n = C.c_uint64()
        _lib.check(self._L.psg_exchange_status(self._h, C.byref(n)))
        return n.value

    def pieces(self, s: int):
        """Shard s's [(offset, count)] per push, push order, empties dropped."""
        return [(int(self.send_off[s, p]), int(self.send_cnt[s, p]))
                for p in range(self.P) if self.send_cnt[s, p]]

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.psg_exchange_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
