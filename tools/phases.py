#!/usr/bin/env python3
"""Per-phase time split of the tile kernel (diagnostic build only).

Build: tools/ab_build.sh phases "-DPSG_PHASES"; run on the GPU box:
  PSG_LIB_PATH=$PWD/build/phases/libpsg.so python3 tools/phases.py [--workload cfg2]
Thread 0 of every workgroup stores the shader clocks between phase marks of
psg_tile.hip into its tile's row (no atomics, so the timing is not
disturbed); printed as a share of the summed clocks and as clocks per tile.  Phases:
  0 start -> barrier (1): descriptor, push tables, D into LDS
  1 -> element loads of the first pass issued
  2 -> bucket table (histogram, scan; barriers 2-4)
  3 -> searches of a pass + barrier (5) (waits for the element loads)
  4 -> order check + wave-ordered fold of a pass (4 barriers)
  5 -> after the last pass
  6 -> stores issued
  7 -> (persistent form) the end-of-tile barrier
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--plan-flags", type=lambda x: int(x, 0), default=0)
    a = ap.parse_args()
    import torch
    import bench
    bench.PLAN_FLAGS = a.plan_flags
    from parameter_server_amd import synth, _lib
    dev = torch.device("cuda", 0)
    if a.workload == "cfg2":
        insts = [synth.shard_instance(seed=1 + j, lo=0, hi=(1 << 64) - 1, npush=8, n=131072,
                                      overlap=0.1) for j in range(a.batch)]
    else:
        insts = [synth.zipf_pushes(seed=3 + j) for j in range(2)]
    plan, keep, jobs = bench.make_plan(insts, dev, 0)
    st = torch.cuda.current_stream()
    L = _lib.lib()
    f = L.psg_debug_phases
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_uint32]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    plan.run(st.cuda_stream)
    e0.record(st)
    for _ in range(a.reps):
        plan.run_stage(1, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ntiles = 1 << 17
    buf = np.zeros((ntiles, 8), np.uint32)
    assert f(buf.ctypes.data, ntiles) == 0
    rows = buf[buf.sum(axis=1) > 0].astype(np.float64)  # tiles of the last launch
    tot = rows.sum()
    out = {"workload": a.workload, "kernel_ms": e0.elapsed_time(e1) / a.reps,
           "tiles": int(rows.shape[0]), "clocks_per_tile": tot / max(rows.shape[0], 1),
           "share": {str(i): float(rows[:, i].sum() / tot) for i in range(8)},
           "clocks_per_tile_by_phase": {str(i): float(rows[:, i].mean()) for i in range(8)},
           "p90_by_phase": {str(i): float(np.percentile(rows[:, i], 90)) for i in range(8)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
