#!/usr/bin/env python3
"""MEASUREMENT AID (GPU box): what a step costs beyond its two kernels.
For the cfg2 headline plan (64 aggregates), one evenDivide(8) cfg5 shard and
a one-tile plan, K steps (partition + aggregate) timed three ways:
  events  HIP events recorded between the stages (bench.timed_steps' form);
  plain   the K steps back to back, wall clock only;
  graph   one step captured into a hipGraph (torch.cuda.CUDAGraph around
          psg_plan_run on the capture stream), replayed K times.
Usage: tools/gap_probe.py [K] [events|plain]  (with a mode: the cfg2 plan only,
that mode only -- a rocprofv3 --kernel-trace of each shows whether the
kernels themselves or the gaps between them differ)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from parameter_server_amd import synth  # noqa: E402


def probe(name, plan, K):
    import torch
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    wall, part, agg = bench.timed_steps(plan, K, 3, st, None)
    ev_ms = wall / K * 1e3

    def plain():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            plan.run(sh)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e3

    plain()
    pl = min(plain() for _ in range(3))
    s = torch.cuda.Stream()
    s.wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        plan.run(s.cuda_stream)
    torch.cuda.synchronize()

    def graph():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e3

    graph()
    gr = min(graph() for _ in range(3))
    ok = plan.matched()
    print(f"{name:8s} events {ev_ms:.4f} (part {part:.4f} agg {agg:.4f})  plain {pl:.4f}  "
          f"graph {gr:.4f} ms/step  matched {int(ok.sum())}", flush=True)


def cfg2_plan(dev):
    from parameter_server_amd.kv_vector import shard_bounds
    b1 = shard_bounds(1)
    insts = [synth.shard_instance(seed=1 + j, lo=int(b1[0]), hi=int(b1[1]), npush=8, n=131072,
                                  overlap=0.1, dtype=np.float32) for j in range(64)]
    return bench.make_plan(insts, dev, 0)


def modes(K):
    """cfg2: the step timed several ways, wall clock of K steps (best of 3)."""
    import torch
    plan, keep, _ = cfg2_plan(torch.device("cuda", 0))
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    E = lambda: torch.cuda.Event(enable_timing=True)

    def run(body):
        for _ in range(3):
            body(-1)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                body(k)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / K * 1e3)
        return best

    ev = [[E() for _ in range(3)] for _ in range(K)]

    def ev3(k):
        if k >= 0:
            ev[k][0].record(st)
        plan.run_stage(0, sh)
        if k >= 0:
            ev[k][1].record(st)
        plan.run_stage(1, sh)
        if k >= 0:
            ev[k][2].record(st)

    def ev_agg(k):
        plan.run_stage(0, sh)
        if k >= 0:
            ev[k][1].record(st)
        plan.run_stage(1, sh)
        if k >= 0:
            ev[k][2].record(st)

    out = {"events3": run(ev3)}
    out["agg_by_events3"] = float(np.mean([ev[k][1].elapsed_time(ev[k][2]) for k in range(K)]))
    out["events_agg_only"] = run(ev_agg)
    out["agg_by_events2"] = float(np.mean([ev[k][1].elapsed_time(ev[k][2]) for k in range(K)]))
    out["plain"] = run(lambda k: plan.run(sh))
    out["partition_only"] = run(lambda k: plan.run_stage(0, sh))
    out["aggregate_only"] = run(lambda k: plan.run_stage(1, sh))
    out["plain_again"] = run(lambda k: plan.run(sh))
    ok = plan.matched()
    print("cfg2 " + " ".join(f"{k} {v:.4f}" for k, v in out.items()) + f" matched {int(ok.sum())}",
          flush=True)


def trace(mode, K):
    import torch
    plan, keep, _ = cfg2_plan(torch.device("cuda", 0))
    st = torch.cuda.current_stream()
    if mode == "events":
        wall, part, agg = bench.timed_steps(plan, K, 3, st, None)
    else:
        for _ in range(3):
            plan.run(st.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            plan.run(st.cuda_stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    print(f"{mode} {wall / K * 1e3:.4f} ms/step", flush=True)


if __name__ == "__main__":
    import torch
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    if len(sys.argv) > 2:
        bench.ARENA = True
        if sys.argv[2] == "modes":
            modes(K)
        else:
            trace(sys.argv[2], K)
        sys.exit(0)
    dev = torch.device("cuda", 0)
    bench.ARENA = True
    rng = np.random.default_rng(0)
    Dt = np.unique(rng.integers(0, 1 << 40, 2048, dtype=np.uint64))[:1024]
    tiny = [(np.sort(rng.choice(Dt, 64, replace=False)), [np.ones(64, np.float32)])
            for _ in range(8)]
    plan, keep, _ = bench.make_plan([(Dt, tiny)], dev, 0)
    probe("floor", plan, K)
    del plan, keep
    D, pieces = synth.cfg5_shard(0, 8)
    plan, keep, _ = bench.make_plan([(D, pieces)], dev, 0)
    probe("shard0", plan, K)
    del plan, keep
    from parameter_server_amd.kv_vector import shard_bounds
    b1 = shard_bounds(1)
    insts = [synth.shard_instance(seed=1 + j, lo=int(b1[0]), hi=int(b1[1]), npush=8, n=131072,
                                  overlap=0.1, dtype=np.float32) for j in range(64)]
    plan, keep, _ = bench.make_plan(insts, dev, 0)
    probe("cfg2", plan, K)
