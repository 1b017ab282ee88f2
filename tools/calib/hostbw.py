"""MEASUREMENT AID: zero-copy kernel access to pinned host memory vs
hipMemcpyAsync, at the sizes of a cfg2 push (1 MB keys, 0.5 MB values) and
of a shard readback (3.8 MB).  usage: python tools/calib/hostbw.py"""
import ctypes as C
import json
import os

import torch

L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhostbw.so"))
L.hostbw_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


out = {}
st = torch.cuda.current_stream().cuda_stream
for nbytes in (1 << 16, 1 << 19, 1 << 20, 4 << 20, 16 << 20):
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    r = {}
    r["memcpy_h2d"] = nbytes / timed(lambda: d.copy_(h, non_blocking=True)) / 1e9
    r["memcpy_d2h"] = nbytes / timed(lambda: h.copy_(d, non_blocking=True)) / 1e9
    for blocks in (64, 256, 1024):
        r[f"kernel_read_{blocks}"] = nbytes / timed(
            lambda: L.hostbw_copy(h.data_ptr(), d.data_ptr(), nbytes, blocks, st)) / 1e9
        r[f"kernel_write_{blocks}"] = nbytes / timed(
            lambda: L.hostbw_copy(d.data_ptr(), h.data_ptr(), nbytes, blocks, st)) / 1e9
    # eight 1 MB pushes: eight copies vs one kernel per buffer (launch cost)
    out[nbytes] = {k: round(v, 1) for k, v in r.items()}
    print(nbytes, json.dumps(out[nbytes]), flush=True)
