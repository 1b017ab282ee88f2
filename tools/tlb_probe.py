#!/usr/bin/env python3
"""MEASUREMENT AID (GPU box): is the sparse (packed) aggregate bound by the
number of distinct pages a tile touches?  Same per-tile shape (256 pushes x
~4 keys per 1024-slot tile) two ways:
  A  cfg5: ONE job, 256 pushes x 262,144 keys (each push's arrays 2 MB + 1 MB:
     a tile reads 256 key pages and 256 value pages)
  B  16 jobs, 256 pushes x 16,384 keys each over a 1/16 key space (each
     push's arrays 128 KB + 64 KB, packed into shared 2 MB allocator blocks)
  C  shard 0 of cfg5 at 8 GPUs (evenDivide(8)): one rank's plan of the
     north star's 8-GPU run (its arrays are 1/8 the size)
Prints the aggregate kernel's mean time per tile for each."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from parameter_server_amd import synth  # noqa: E402


def run(name, insts):
    import torch
    dev = torch.device("cuda", 0)
    plan, keep, jobs = bench.make_plan(insts, dev, 0)
    stream = torch.cuda.current_stream()
    _, part, agg = bench.timed_steps(plan, 10, 2, stream, None)
    slots = sum(int(j["nslots"]) for j in jobs)
    kv = int(plan.kv_pairs)
    print(f"{name}: {len(jobs)} jobs, {slots} slots, {kv} kv: aggregate {agg:.3f} ms "
          f"({agg * 1e9 / kv:.2f} ps per kv), partition {part:.3f} ms", flush=True)
    del plan, keep
    torch.cuda.empty_cache()


def main():
    D, pushes = synth.uniform_pushes(seed=5)
    run("A cfg5", [(D, pushes)])
    insts = [synth.uniform_pushes(seed=50 + j, n=16384, rank_max=10 ** 9 // 16) for j in range(16)]
    run("B 16 small jobs", insts)
    from parameter_server_amd.kv_vector import shard_bounds
    pieces = synth.shard_pieces(pushes, shard_bounds(8), 0)
    Ds = np.unique(np.concatenate([k for k, _ in pieces]))
    run("C cfg5 shard 0 of 8", [(Ds, pieces)])


if __name__ == "__main__":
    main()
