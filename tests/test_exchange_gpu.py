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
