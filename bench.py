#!/usr/bin/env python3
"""Benchmark of the device-resident server-side push aggregation.

Headline workload (BASELINE.json configs[1], "cfg2"): one (channel, time)
aggregate = 8 worker pushes x 131,072 sorted unique uint64 keys with f32
values, 10 % of the keys shared by all pushes, U = 956,827 server keys.
A step is one pass of the hot path (partition + aggregate kernels) over a
batch of --batch such aggregates per GPU (default 64: 1.54 GB of distinct
inputs/outputs, 6x the 256 MB Infinity Cache, so the rate is an HBM rate;
SURVEY 8d sizes one merge at ~4 us at the target, so a launch should carry
>= 64 of them to amortise launch and tail).

Multi-GPU (one process per GPU, torchrun): the key space is range-
partitioned with Range<uint64>::all().evenDivide(N, rank) (reference
linear_method.cc:137-145); each rank holds the shard of every aggregate
that its key range owns, exactly what the reference's worker-side
sliceKeyOrderedMsg delivers (message.h:89-123), so the data path has no
collective and per-GPU work is fixed ("scaling": "weak").  --ingress
unsliced instead hands every rank whole pushes and re-homes the pieces with
an RCCL all-to-all before merging (SURVEY 8e mode B).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "aggregated kv-pairs/s (device-resident), N-way sparse push merge at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="cfg2 aggregates per GPU per step")
    ap.add_argument("--npush", type=int, default=8)
    ap.add_argument("--n", type=int, default=131072)
    ap.add_argument("--overlap", type=float, default=0.1)
    ap.add_argument("--workload", choices=["cfg2", "cfg3", "cfg4"], default="cfg2",
                    help="cfg2 (default, the headline); cfg3 CTR shape (64 Zipf(1.1) "
                         "murmur-keyed pushes x 131072) and cfg4 dense (8 x 16 M contiguous "
                         "keys) are single-GPU side lines (BASELINE.json configs[2], [3])")
    ap.add_argument("--ingress", choices=["sliced", "unsliced"], default="sliced")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="only run warmup+steps (for rocprofv3); skip baselines")
    return ap.parse_args()


WORKLOADS = {
    "cfg2": ("cfg2: {a.npush} pushes x {a.n} sorted unique uint64 keys + f32 values, 10% shared "
             "keys (U={U:,}); {a.batch} such (channel,time) aggregates per GPU per step"),
    "cfg3": ("cfg3 (CTR shape): 64 pushes x 131072 unique murmur-shuffled Zipf(1.1) ranks in "
             "[1,1e9] + f32 values (U={U:,}); {a.batch} such aggregates per step"),
    "cfg4": ("cfg4 (dense-bucket limit): 8 pushes of all keys [0,16777216) + f32 values "
             "(U={U:,}); {a.batch} such aggregates per step"),
}


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        log(f"--gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from parameter_server_amd import synth
    from parameter_server_amd.kv_vector import MergePlan, shard_bounds
    from parameter_server_amd._lib import PSG_F32

    bounds = shard_bounds(world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])

    # ---- synthetic inputs (each rank: its shard of `batch` aggregates) ----
    t0 = time.time()
    if args.workload != "cfg2":
        if world > 1:
            raise SystemExit("--workload cfg3/cfg4 are single-GPU side lines")
        insts = [synth.zipf_pushes(seed=3 + j) if args.workload == "cfg3"
                 else synth.dense_pushes(seed=4 + j) for j in range(args.batch)]
    elif args.ingress == "sliced":
        insts = [synth.shard_instance(seed=1 + j + 1000 * rank, lo=lo, hi=hi,
                                      npush=args.npush, n=args.n, overlap=args.overlap)
                 for j in range(args.batch)]
    else:
        # mode B: this rank's workers push whole pushes; they are re-homed by
        # an all-to-all inside every timed step (shard.UnslicedExchange)
        aggs = [synth.overlap_pushes(1 + j + 1000 * rank, args.npush, args.n, args.overlap)[1]
                for j in range(args.batch)]
        insts = None
    log(f"rank {rank}: generated {args.batch} aggregates in {time.time() - t0:.1f}s")

    dev = torch.device("cuda", local)

    def to_dev(a):
        a = np.ascontiguousarray(a)
        return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)

    keep, jobs = [], []
    ex = None
    if insts is None:
        from parameter_server_amd import shard as S
        ex = S.UnslicedExchange(aggs, bounds, dist, dev)
        ex.run()
        torch.cuda.synchronize()
        rk = ex.recv_keys.cpu().numpy().view(np.uint64)
        for j in range(args.batch):
            pcs = ex.pieces(j)
            if not pcs:
                continue
            D = np.unique(np.concatenate([rk[o:o + c] for o, c in pcs]))
            dD = to_dev(D)
            out = torch.empty(max(1, D.size), dtype=torch.float32, device=dev)
            keep.append((dD, out))
            jobs.append({"keys": dD.data_ptr(), "nslots": int(D.size),
                         "push_keys": [ex.recv_keys.data_ptr() + 8 * o for o, _ in pcs],
                         "push_vals": [[ex.recv_vals[0].data_ptr() + 4 * o] for o, _ in pcs],
                         "push_n": [c for _, c in pcs],
                         "out": [out.data_ptr()]})
        del rk
    for D, pushes in insts or []:
        dD = to_dev(D)
        pk = [to_dev(k) for k, _ in pushes]
        pv = [[to_dev(v) for v in vs] for _, vs in pushes]
        out = torch.empty(max(1, D.size), dtype=torch.float32, device=dev)
        keep.append((dD, pk, pv, out))
        jobs.append({"keys": dD.data_ptr(), "nslots": int(D.size),
                     "push_keys": [t.data_ptr() for t in pk],
                     "push_vals": [[t.data_ptr() for t in vs] for vs in pv],
                     "push_n": [int(k.size) for k, _ in pushes],
                     "out": [out.data_ptr()]})
    plan = MergePlan(local, PSG_F32, 1, jobs)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    # correctness guard: every pushed key matched
    plan.run(sh)
    mt = plan.matched()
    want = np.array([n for jb in jobs for n in jb["push_n"]], np.uint64)
    assert np.array_equal(mt, want), "unmatched keys in the bench workload"

    for _ in range(args.warmup):
        if ex is not None:
            ex.run()
        plan.run(sh)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()

    K = args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
    t_start = time.perf_counter()
    for s in range(K):
        ev[s][3].record(stream)
        if ex is not None:
            ex.run()  # mode B: the RCCL all-to-all re-homing is part of the step
        ev[s][0].record(stream)
        plan.run_stage(0, sh)
        ev[s][1].record(stream)
        plan.run_stage(1, sh)
        ev[s][2].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start

    part_ms = float(np.mean([ev[s][0].elapsed_time(ev[s][1]) for s in range(K)]))
    agg_ms = float(np.mean([ev[s][1].elapsed_time(ev[s][2]) for s in range(K)]))
    xchg_ms = float(np.mean([ev[s][3].elapsed_time(ev[s][0]) for s in range(K)]))

    wall_max, kv_all = reduce_over_ranks(wall, plan.kv_pairs, dist, dev)
    value = kv_all * K / wall_max
    ms_per_step = wall_max / K * 1e3

    if args.profile_steps:
        if rank == 0:
            log(f"profile run: {ms_per_step:.3f} ms/step, aggregate {agg_ms:.3f} ms")
        if dist:
            dist.destroy_process_group()
        return

    # copy-kernel bandwidth in the same run (read + write bytes / time)
    nbytes = 1 << 30
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    for _ in range(3):
        dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(10):
        dst.copy_(src)
    e1.record(stream)
    torch.cuda.synchronize()
    copy_gbps = 2 * nbytes * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst

    achieved = plan.bytes / (agg_ms * 1e-3) / 1e9
    traffic = load_traffic(args, plan.bytes)

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "kv-pairs/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": WORKLOADS[args.workload].format(a=args, U=jobs[0]["nslots"] if jobs else 0),
            "global_batch": args.batch * world,
            "kv_per_step": kv_all,
            "parallelism": (f"key-range shards evenDivide({world}); "
                            + ("worker-sliced ingress, no data-path collective"
                               if ex is None else
                               "unsliced ingress, RCCL all-to-all re-homing in every step")),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "kernel": kernel_name(),
            "bytes_per_launch": plan.bytes,
            "bytes_formula": "sum_p n_p*(8+4) [pushes] + U*(8+4) [server keys + sums]",
            "kernel_ms": agg_ms,
            "partition_ms": part_ms,
            "measured_copy_GBps": copy_gbps,
            "frac_of_measured_copy": achieved / copy_gbps,
        },
    }
    if ex is not None:
        result["exchange"] = {"ms": xchg_ms, "bytes_sent_per_rank": ex.sent_bytes,
                              "scope": "gather into destination order + all-to-all of keys "
                                       "and values (RCCL), per step, rank 0's HIP events"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and ex is None:
        result["end_to_end"] = end_to_end(insts[0], local)
        result["cpu_baseline"] = cpu_baseline(insts[0], args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def reduce_over_ranks(wall, kv_rank, dist, dev):
    """Whole-job timing: the slowest rank's wall time and the kv-pairs all
    ranks merged (bench contract: value = all units / max-over-ranks time)."""
    import torch
    t = torch.tensor([wall, float(kv_rank)], dtype=torch.float64, device=dev)
    if dist:
        w = t[:1].clone()
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        k = t[1:].clone()
        dist.all_reduce(k)
        return float(w.item()), float(k.item())
    return float(t[0].item()), float(t[1].item())


def kernel_name():
    """The aggregate kernel (psg_tile.hip)."""
    return "tile_kernel<float,1>"


def end_to_end(inst, device, reps=5):
    """PCIe-inclusive rate of one cfg2 aggregate through the host API
    (KVVector.setValue per push from pageable host memory + received(t)
    D2H), the reference's own call pattern.  Reported beside `value`,
    never as it."""
    import ctypes
    from parameter_server_amd.kv_vector import KVVector, Message
    D, pushes = inst
    kv = sum(int(k.size) for k, _ in pushes)
    v = KVVector(device)
    v.setValue(Message(key=D))  # key-only push: the server key set
    times = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        for k, vs in pushes:
            v.setValue(Message(time=r, key=k, value=list(vs)))
        out = v.received(r)
        el = time.perf_counter() - t0
        if r:
            times.append(el)
    assert out[0][1].size == D.size
    v.close()
    t = float(np.median(times))
    return {"value": kv / t, "unit": "kv-pairs/s", "ms_per_aggregate": t * 1e3,
            "scope": ("one cfg2 aggregate: 8 x psg_push (H2D of keys+values from pageable "
                      "host memory, merge) + psg_received (D2H of the merged shard), "
                      f"median of {reps}")}


def load_traffic(args, bytes_per_launch):
    """HBM bytes per aggregate launch from the committed rocprofv3 PMC
    summary (profiles/pmc_summary.json, written by tools/pmc_traffic.py),
    when it was collected on this same workload; else null."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        d = json.load(open(p))
    except Exception:
        return None
    if d.get("bytes_per_launch") != bytes_per_launch:
        return None
    return d.get("hbm_bytes_per_launch")


def cpu_baseline(inst, seconds):
    """The oracle's restatement of the reference CPU path (serialSetValue:
    oldMatch + dense +=, the shipped default) on one cfg2 aggregate,
    repeated for ~`seconds` on this host; plus the threaded match path."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    D, pushes = inst
    kv = sum(int(k.size) for k, _ in pushes)
    ALL = (0, (1 << 64) - 1)

    def timed(parallel, nthreads):
        reps, t0 = 0, time.perf_counter()
        while True:
            rc, *_ = O.aggregate(D, *ALL, pushes, parallel, nthreads)
            assert rc == 0
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds / 2:
                return reps * kv / el, reps, el

    v, reps, el = timed(0, 1)
    # the threaded match path (FLAGS_parallel_match) at 4 threads (local.sh:25)
    # and at this job's CPU share (<= 16 on the GPU box)
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    par = {}
    for nt in sorted({4, max(1, min(16, share))}):
        vp, repsp, elp = timed(1, nt)
        par[str(nt)] = {"value": vp, "reps": repsp, "seconds": elp}
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {
        "value": v, "unit": "kv-pairs/s", "cores": 1, "kind": "port",
        "sample": (f"{reps} x one cfg2 aggregate (8 x 131072 kv, U={D.size}) through "
                   f"oracle serialSetValue restatement in {el:.1f}s, 1 thread, {model}"),
        "parallel_match_by_threads": par,
    }


if __name__ == "__main__":
    main()
