#!/usr/bin/env python3
"""MEASUREMENT AID (GPU box): does the partition of the next aggregates run
beside the aggregate kernel of the current ones?  A step's aggregates are
split into P plans; serial = every plan's partition then aggregate on one
stream; pipelined = partitions on a second stream running ahead, each
aggregate launch waiting (event) for its own plan's partition.  Same plans,
same kernels, same bytes.  usage: tools/pipe_probe.py cfg2|cfg5 [P ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from parameter_server_amd import synth  # noqa: E402


def main():
    import torch
    wl = sys.argv[1]
    Ps = [int(x) for x in sys.argv[2:]] or [1, 2, 4]
    dev = torch.device("cuda", 0)
    if wl == "cfg2":
        insts = [synth.shard_instance(seed=1 + j, lo=0, hi=(1 << 64) - 1) for j in range(64)]
    else:
        insts = [synth.uniform_pushes(seed=5 + j) for j in range(2)]
    nbytes = 0
    for P in Ps:
        per = (len(insts) + P - 1) // P
        plans = [bench.make_plan(insts[i:i + per], dev, 0) for i in range(0, len(insts), per)]
        nbytes = sum(int(p.bytes) for p, _, _ in plans)
        s0 = torch.cuda.current_stream()
        s1 = torch.cuda.Stream()

        def serial():
            for p, _, _ in plans:
                p.run_stage(0, s0.cuda_stream)
                p.run_stage(1, s0.cuda_stream)

        def piped():
            s1.wait_stream(s0)  # the previous step's aggregates done before the partitions rewrite seg
            for p, _, _ in plans:
                p.run_stage(0, s1.cuda_stream)
                e = torch.cuda.Event()
                e.record(s1)
                s0.wait_event(e)
                p.run_stage(1, s0.cuda_stream)

        for name, fn in (("serial", serial), ("piped", piped)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            K = 20
            t0 = time.perf_counter()
            for _ in range(K):
                fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / K * 1e3
            print(f"{wl} P={P} {name}: {ms:.4f} ms/step  step_frac {nbytes / (ms * 1e-3) / 8e12:.3f}",
                  flush=True)
        # the pipelined run merges the same bits
        serial()
        torch.cuda.synchronize()
        ref = [k[0][3].clone() for _, k, _ in plans]
        for t in [k[0][3] for _, k, _ in plans]:
            t.zero_()
        piped()
        torch.cuda.synchronize()
        assert all(torch.equal(a.view(torch.int32), k[0][3].view(torch.int32))
                   for a, (_, k, _) in zip(ref, plans)), "pipelined result differs"
        del plans
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
