"""MEASUREMENT AID: the batched N-way merge (psg_nway_create_batch) over
--batch cfg2 aggregates, run --reps times (for rocprofv3 --kernel-trace)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--prof", action="store_true",
                    help="read the phase clocks of a -DPSG_NWAY_PROF build (PSG_LIB_PATH)")
    a = ap.parse_args()
    import torch
    from parameter_server_amd import _lib, synth
    from parameter_server_amd.kv_vector import NWayMergeBatch
    dev = torch.device("cuda", 0)
    keep, merges, nb, sizes = [], [], 0, []
    for j in range(a.batch):
        D, ps = synth.overlap_pushes(1 + j)
        dk = [torch.from_numpy(k.view(np.int64)).to(dev) for k, _ in ps]
        dv = [torch.from_numpy(vs[0]).to(dev) for _, vs in ps]
        tot = sum(k.size for k, _ in ps)
        ok = torch.empty(tot, dtype=torch.int64, device=dev)
        ov = torch.empty(tot, dtype=torch.float32, device=dev)
        keep.append((dk, dv, ok, ov))
        merges.append(dict(push_keys=[t.data_ptr() for t in dk], push_n=[k.size for k, _ in ps],
                           push_vals=[[t.data_ptr()] for t in dv] if a.m else [[] for _ in dk],
                           out_keys=ok.data_ptr(), out_vals=[ov.data_ptr()] if a.m else []))
        nb += tot * (8 + 4 * a.m) + D.size * (8 + 4 * a.m)
        sizes.append(D.size)
    u = NWayMergeBatch(0, _lib.PSG_F32, merges)
    u.run()
    assert u.result() == sizes
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        u.run(st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(f"batch {a.batch} m {a.m}: {ms:.3f} ms, {nb / ms / 1e6:.1f} GB/s, frac {nb / ms / 1e6 / 8000:.3f}")
    u.close()
    if a.prof:
        import ctypes as C
        f = _lib.lib().psg_debug_nway_prof
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_uint32]
        buf = np.zeros((65536, 8), np.uint64)
        assert f(buf.ctypes.data, 65536) == 0
        rows = buf[buf[:, 7] > 0].astype(np.float64)
        d = np.diff(rows, axis=1)
        names = ["table", "load+check", "merge", "heads", "sums", "lookback", "store"]
        tot = rows[:, 7] - rows[:, 0]
        print(f"tiles {rows.shape[0]}, clocks per tile: total mean {tot.mean():.0f} p50 "
              f"{np.median(tot):.0f} p99 {np.percentile(tot, 99):.0f}")
        for i, n in enumerate(names):
            print(f"  {n:11s} mean {d[:, i].mean():9.0f}  p50 {np.median(d[:, i]):9.0f}  "
                  f"p99 {np.percentile(d[:, i], 99):9.0f}")
