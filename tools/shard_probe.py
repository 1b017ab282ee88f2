#!/usr/bin/env python3
"""MEASUREMENT AID (GPU box): one evenDivide(8) shard of the cfg5 workload
(its pieces of all 256 pushes) as its rank merges it: partition and
aggregate times and the step, HIP events, K steps (tools/shard_probe.py [K])."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from parameter_server_amd import synth  # noqa: E402

if __name__ == "__main__":
    import torch
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    D, pieces = synth.cfg5_shard(0, 8)
    plan, keep, _ = bench.make_plan([(D, pieces)], dev, 0)
    st = torch.cuda.current_stream()
    plan.run(st.cuda_stream)
    assert np.array_equal(plan.matched(), np.array([k.size for k, _ in pieces], np.uint64))
    wall, (part_ms, agg_ms) = bench.timed_stages([lambda: plan.run_stage(0, st.cuda_stream),
                                                  lambda: plan.run_stage(1, st.cuda_stream)],
                                                 K, 3, st, None)
    print(f"shard0 step {wall / K * 1e3:.4f} ms partition {part_ms:.4f} kernel {agg_ms:.4f}",
          flush=True)
