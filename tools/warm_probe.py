#!/usr/bin/env python3
"""MEASUREMENT AID (GPU box): does the cfg2 step time depend on how long the
GPU has been busy?  After the plan is built and checked, the GPU idles for
2 s (as it does in bench.py while the host generates data), then runs blocks
of 10 steps back to back, each block timed by wall clock (synchronize on
both sides), and prints every block's ms/step -- the first blocks show the
clock ramp, the last ones the steady state.
usage: tools/warm_probe.py [blocks]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from parameter_server_amd import synth  # noqa: E402

if __name__ == "__main__":
    import torch
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    bench.ARENA = True
    from parameter_server_amd.kv_vector import shard_bounds
    b1 = shard_bounds(1)
    insts = [synth.shard_instance(seed=1 + j, lo=int(b1[0]), hi=int(b1[1]), npush=8, n=131072,
                                  overlap=0.1, dtype=np.float32) for j in range(64)]
    plan, keep, _ = bench.make_plan(insts, dev, 0)
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    plan.run(sh)
    assert int(plan.matched().sum()) == 64 * 8 * 131072
    for trial in range(2):
        torch.cuda.synchronize()
        time.sleep(2.0)
        blocks = []
        t_start = time.perf_counter()
        for b in range(nb):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                plan.run(sh)
            torch.cuda.synchronize()
            blocks.append(((time.perf_counter() - t0) / 10 * 1e3, (t0 - t_start) * 1e3))
        print(f"trial {trial}: ms/step per block of 10 (ms since the first):", flush=True)
        print("  " + " ".join(f"{ms:.3f}@{at:.0f}" for ms, at in blocks), flush=True)
