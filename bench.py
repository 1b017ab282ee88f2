#!/usr/bin/env python3
"""Benchmark of the device-resident server-side push aggregation.

Headline workload (BASELINE.json configs[1], "cfg2"): one (channel, time)
aggregate = 8 worker pushes x 131,072 sorted unique uint64 keys with f32
values, 10 % of the keys shared by all pushes, U = 956,827 server keys.
A step is one pass of the hot path (partition + aggregate kernels) over a
batch of --batch such aggregates per GPU (default 64: 1.54 GB of distinct
inputs/outputs, 6x the 256 MB Infinity Cache, so the rate is an HBM rate).

Multi-GPU (one process per GPU, torchrun): the key space is range-
partitioned with Range<uint64>::all().evenDivide(N, rank) (reference
linear_method.cc:137-145).  The headline line shards the units (aggregates'
key ranges) across ranks with no data-path collective: each rank holds the
shard of --batch aggregates that its key range owns, exactly what the
reference's worker-side sliceKeyOrderedMsg delivers (message.h:89-123);
per-GPU work is fixed ("scaling": "weak").

The line also carries a "cfg5" block (BASELINE.json configs[4], the
north star's 8-GPU target): ONE fixed global workload -- 256 worker pushes
x 262,144 murmur-shuffled uniform keys over a 1e9-rank (1 B-key) space --
range-partitioned over the N ranks (strong scaling), timed on all ranks
together, plus the same whole workload on ONE GPU (rank 0) in the same job,
so "speedup_vs_1gpu" is measured, not inferred.

--workload cfg3|cfg4|cfg5 runs a single-GPU side line of that config.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "aggregated kv-pairs/s (device-resident), N-way sparse push merge at 1/2/4/8 GPU"

WORKLOADS = {
    "cfg2": dict(batch=64, desc=(
        "cfg2: {a.npush} pushes x {a.n} sorted unique uint64 keys + {a.dtype} values, 10% shared "
        "keys (U={U:,}); {batch} such (channel,time) aggregates per GPU per step")),
    "cfg3": dict(batch=4, desc=(
        "cfg3 (CTR shape): 64 pushes x 131072 unique murmur-shuffled Zipf(1.1) ranks in "
        "[1,1e9] + f32 values (U={U:,}); {batch} such aggregates per step")),
    "cfg4": dict(batch=1, desc=(
        "cfg4 (dense-bucket limit): 8 pushes of all keys [0,16777216) + f32 values "
        "(U={U:,}); {batch} such aggregate per step")),
    "cfg5": dict(batch=1, desc=(
        "cfg5: 256 pushes x 262144 unique murmur-shuffled uniform ranks in [0,1e9) + f32 "
        "values (U={U:,}), the whole 1 B-key-space aggregate on one GPU")),
}


# the aggregate kernel a plan runs (the runtime picks the form: dense slices,
# sorted pushes on a resident index -> per-push cursors, short pieces ->
# packed rounds, > 32 pushes -> 64-push groups); names as rocprofv3 lists them
def kernel_name(plan, dtype="f32"):
    from parameter_server_amd import _lib
    v = "double" if dtype == "f64" else "float"
    return {_lib.PSG_KERNEL_TILE: f"tile_kernel<{v},1,32>",
            _lib.PSG_KERNEL_TILE64: f"tile_kernel<{v},1,64>",
            _lib.PSG_KERNEL_PACKED: f"tile_packed_kernel<{v},1>",
            _lib.PSG_KERNEL_DENSE: f"dense_kernel<{v},1>",
            _lib.PSG_KERNEL_CURSOR: f"cursor_kernel<{v},1,KR>",
            _lib.PSG_KERNEL_PACKED_CURSOR: f"tile_packed_kernel<{v},1,true>"}[plan.form]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm-ms", type=float, default=100.0,
                    help="untimed steps for this long before each timed region's warm-up "
                         "steps (the GPU's clock ramp after host-side phases; 0 = off)")
    ap.add_argument("--batch", type=int, default=0,
                    help="aggregates per GPU per step (default: 64 for cfg2, else 1-2)")
    ap.add_argument("--npush", type=int, default=8)
    ap.add_argument("--n", type=int, default=131072)
    ap.add_argument("--overlap", type=float, default=0.1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg2")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32",
                    help="value type of a side line (the reference's apps use double, "
                         "batch_solver.h:32); the headline is f32 (north star)")
    ap.add_argument("--no-cfg5", action="store_true",
                    help="skip the cfg5 strong-scaling block of the default line")
    ap.add_argument("--no-f64", action="store_true",
                    help="skip the f64 (the reference apps' double) cfg2 block of the default line")
    ap.add_argument("--cfg5-steps", type=int, default=10)
    ap.add_argument("--no-shard8", action="store_true",
                    help="skip the cfg5 block's one-GPU per-shard leg (shard_of_8)")
    ap.add_argument("--cfg5-unsliced-child", action="store_true",
                    help=argparse.SUPPRESS)  # internal: the unsliced leg in its own process
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--layout", choices=["arena", "separate"], default="arena",
                    help="where the pushes sit in HBM: 'arena' = each aggregate's push keys "
                         "back to back in one allocation and each value array likewise (a "
                         "server's receive buffer; the layout psg_exchange delivers), "
                         "'separate' = one allocation per push array")
    ap.add_argument("--arena-pushes", type=int, default=0,
                    help=argparse.SUPPRESS)  # A/B: pushes per arena allocation (0 = all)
    ap.add_argument("--plan-flags", type=lambda x: int(x, 0), default=0,
                    help="kernel-form overrides of include/psg.h (A/B measurements only)")
    ap.add_argument("--no-server-api", action="store_true",
                    help="cfg4: skip the server-API (psg_push + psg_received) leg")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the matched-count guard (ablation builds via PSG_LIB_PATH only)")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="only run warmup+steps (for rocprofv3); skip baselines and blocks")
    a = ap.parse_args()
    if not a.batch:
        a.batch = WORKLOADS[a.workload]["batch"]
    return a


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def to_dev(a, dev):
    import torch
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)


PLAN_FLAGS = 0  # --plan-flags
ROT = 3  # shard_of_8: copies of a shard rotated through (3 x ~200 MB > the 256 MB MALL)
ARENA = True    # --layout arena
ARENA_PUSHES = 0  # --arena-pushes


def make_plan(insts, dev, local):
    """MergePlan over [(D, pushes)] resident on `dev`; returns (plan, keep, jobs)."""
    import torch
    from parameter_server_amd.kv_vector import MergePlan
    from parameter_server_amd._lib import PSG_F32, PSG_F64
    keep, jobs = [], []
    f64 = bool(insts) and insts[0][1][0][1][0].dtype == np.float64
    for D, pushes in insts:
        dD = to_dev(D, dev)
        if ARENA:
            # the aggregate's pushes in one key arena and one value arena per
            # value array, back to back, as views: a server receives an
            # aggregate's pushes into one buffer (psg_exchange's receive
            # buffer has exactly this layout).  Same bytes and kernels as
            # --layout separate; sparse many-push tiles (cfg5) touch far fewer
            # translation entries this way
            m = len(pushes[0][1]) if pushes else 0
            step = ARENA_PUSHES or max(1, len(pushes))
            pk, pv = [], []
            for c0 in range(0, len(pushes), step):
                part = pushes[c0:c0 + step]
                ka = to_dev(np.concatenate([k for k, _ in part]), dev)
                va = [to_dev(np.concatenate([vs[i] for _, vs in part]), dev) for i in range(m)]
                offs = np.concatenate([[0], np.cumsum([k.size for k, _ in part])]).astype(np.int64)
                pk += [ka[offs[p]:offs[p + 1]] for p in range(len(part))]
                pv += [[a[offs[p]:offs[p + 1]] for a in va] for p in range(len(part))]
        else:
            pk = [to_dev(k, dev) for k, _ in pushes]
            pv = [[to_dev(v, dev) for v in vs] for _, vs in pushes]
        out = torch.empty(max(1, D.size), dtype=torch.float64 if f64 else torch.float32,
                          device=dev)
        keep.append((dD, pk, pv, out))
        jobs.append({"keys": dD.data_ptr(), "nslots": int(D.size),
                     "push_keys": [t.data_ptr() for t in pk],
                     "push_vals": [[t.data_ptr() for t in vs] for vs in pv],
                     "push_n": [int(k.size) for k, _ in pushes],
                     "out": [out.data_ptr()]})
    plan = MergePlan(local, PSG_F64 if f64 else PSG_F32, 1, jobs, flags=PLAN_FLAGS)
    return plan, keep, jobs


PREWARM_S = 0.1  # --prewarm-ms / 1000


def prewarm(step):
    """Untimed steps for PREWARM_S seconds of wall time before a timed
    region's W warm-up steps.  MI355X raises its clocks over ~25 ms of
    sustained work after an idle spell (here: the host generating the next
    block's data), so a timed region that starts on a cold GPU measures the
    ramp, not the kernel: cfg2 steps run 0.43 ms in the first ~10 ms and
    0.362 ms from ~25 ms on (tools/warm_probe.py,
    profiles/r06_warm_probe.txt).  The timed region itself is unchanged:
    exactly K whole steps.  Returns the steps run."""
    import torch
    if PREWARM_S <= 0:
        return 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while True:
        for _ in range(4):  # a few at a time: the host stays ahead of the GPU
            step()
            n += 1
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= PREWARM_S:
            return n


def timed_steps(plan, K, W, stream, dist):
    """W untimed warm-up steps (after the prewarm), then exactly K timed steps
    bracketed by a barrier + device synchronize on both sides.  Returns (wall
    s, mean partition ms, mean aggregate ms).  Inside the timed region two
    HIP events per step bracket the aggregate kernel on its launch stream
    (the roofline's kernel time); the partition's time comes from a second,
    untimed pass of K steps with events around the partition.  A third event
    per step between the stages cost ~6 us per step (1.6 %,
    profiles/r06_warm_probe.txt)."""
    import torch
    sh = stream.cuda_stream
    prewarm(lambda: plan.run(sh))
    for _ in range(W):
        plan.run(sh)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(K)]
    t0 = time.perf_counter()
    for s in range(K):
        plan.run_stage(0, sh)
        ev[s][0].record(stream)
        plan.run_stage(1, sh)
        ev[s][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    agg = float(np.mean([ev[s][0].elapsed_time(ev[s][1]) for s in range(K)]))
    # the partition, untimed: events around it in K more steps
    for s in range(K):
        ev[s][0].record(stream)
        plan.run_stage(0, sh)
        ev[s][1].record(stream)
        plan.run_stage(1, sh)
    torch.cuda.synchronize()
    part = float(np.mean([ev[s][0].elapsed_time(ev[s][1]) for s in range(K)]))
    return wall, part, agg


def main():
    global PLAN_FLAGS, ARENA, ARENA_PUSHES
    args = parse()
    PLAN_FLAGS = args.plan_flags
    global PREWARM_S
    PREWARM_S = args.prewarm_ms / 1000.0
    ARENA = args.layout == "arena"
    ARENA_PUSHES = args.arena_pushes
    if args.cfg5_unsliced_child:
        return unsliced_child_main(args)
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
    from parameter_server_amd.kv_vector import shard_bounds

    bounds = shard_bounds(world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    dev = torch.device("cuda", local)
    wl = args.workload

    # ---- synthetic inputs (each rank: its shard of `batch` aggregates) ----
    t0 = time.time()
    if wl != "cfg2" and world > 1:
        raise SystemExit("--workload cfg3/cfg4/cfg5 are single-GPU side lines; the default "
                         "line carries cfg5's multi-GPU strong-scaling block")
    vdt = np.float64 if args.dtype == "f64" else np.float32
    if args.dtype == "f64" and wl != "cfg2":
        raise SystemExit("--dtype f64 is a cfg2 side line")
    if wl == "cfg2":
        insts = [synth.shard_instance(seed=1 + j + 1000 * rank, lo=lo, hi=hi,
                                      npush=args.npush, n=args.n, overlap=args.overlap,
                                      dtype=vdt)
                 for j in range(args.batch)]
    elif wl == "cfg3":
        insts = [synth.zipf_pushes(seed=3 + j) for j in range(args.batch)]
    elif wl == "cfg4":
        insts = [synth.dense_pushes(seed=4 + j) for j in range(args.batch)]
    else:
        insts = [synth.uniform_pushes(seed=5 + j) for j in range(args.batch)]
    log(f"rank {rank}: generated {args.batch} {wl} aggregates in {time.time() - t0:.1f}s")

    if wl == "cfg4":
        # the bench's pushes are fixed for the plan's lifetime: the dense
        # kernel (no key reads) is allowed (include/psg.h PSG_STATIC_KEYS)
        from parameter_server_amd._lib import PSG_STATIC_KEYS
        PLAN_FLAGS |= PSG_STATIC_KEYS
    plan, keep, jobs = make_plan(insts, dev, local)
    stream = torch.cuda.current_stream()

    # correctness guard: every pushed key matched
    plan.run(stream.cuda_stream)
    want = np.array([n for jb in jobs for n in jb["push_n"]], np.uint64)
    assert args.no_check or np.array_equal(plan.matched(), want), \
        "unmatched keys in the bench workload"

    K = args.steps
    wall, part_ms, agg_ms = timed_steps(plan, K, args.warmup, stream, dist)
    wall_max, kv_all = reduce_over_ranks(wall, plan.kv_pairs, dist, dev)
    value = kv_all * K / wall_max
    ms_per_step = wall_max / K * 1e3

    if args.profile_steps:
        if rank == 0:
            log(f"profile run: {ms_per_step:.3f} ms/step, aggregate {agg_ms:.3f} ms, "
                f"partition {part_ms:.3f} ms")
        if dist:
            dist.destroy_process_group()
        return

    # roofline of the aggregate kernel: ALGORITHMIC bytes per launch (SURVEY
    # 8d) / its mean HIP-event duration; cfg4 is priced in the dense form
    U = sum(int(jb["nslots"]) for jb in jobs)
    sv = 8 if args.dtype == "f64" else 4
    if wl == "cfg4":
        nbytes = int(plan.kv_pairs) * 4 + U * 4
        formula = "dense form: sum_p n_p*4 [push values] + U*4 [sums] (keys implied, SURVEY 8d)"
    else:
        nbytes = int(plan.bytes)
        formula = (f"sum_p n_p*(8+{sv}) [pushes] + U*(8+{sv}) [server keys + sums] "
                   "(SURVEY 8d)")
    achieved = nbytes / (agg_ms * 1e-3) / 1e9
    step_gbps = nbytes / (ms_per_step * 1e-3) / 1e9
    copy_gbps = copy_bandwidth(dev, stream)
    traffic = load_traffic(nbytes, wl)

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "kv-pairs/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "prewarm_ms": args.prewarm_ms,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic",
        "config": {
            "workload": WORKLOADS[wl]["desc"].format(a=args, U=jobs[0]["nslots"] if jobs else 0,
                                                     batch=args.batch),
            "global_batch": args.batch * world,
            "kv_per_step": kv_all,
            "input_layout": args.layout,
            "parallelism": (f"key-range shards evenDivide({world}); worker-sliced ingress, "
                            "no data-path collective"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic.get("tile") if traffic else None,
            "kernel": kernel_name(plan, args.dtype),
            "bytes_per_launch": nbytes,
            "bytes_formula": formula,
            "kernel_ms": agg_ms,
            "partition_ms": part_ms,
            "step_achieved": step_gbps,
            "step_frac": step_gbps / HBM_PEAK_GBPS,
            "traffic_partition": traffic.get("partition") if traffic else None,
            "traffic_source": traffic.get("source") if traffic else None,
            "measured_copy_GBps": copy_gbps,
            "frac_of_measured_copy": achieved / copy_gbps if copy_gbps else None,
        },
    }
    if wl == "cfg4" and rank == 0 and not args.no_server_api:
        del plan, keep
        torch.cuda.empty_cache()
        result["server_api"] = {"pinned_out": cfg4_server_api(insts[0], local),
                                "pageable_out": cfg4_server_api(insts[0], local, pinned_out=False)}
    if wl == "cfg2" and not args.no_f64 and args.dtype == "f32":
        del plan, keep
        torch.cuda.empty_cache()
        result["f64"] = f64_block(args, insts, dist, dev, local, stream)
    if wl == "cfg2" and not args.no_cfg5 and args.dtype == "f32":
        plan = keep = None
        torch.cuda.empty_cache()
        result["cfg5"] = cfg5_block(args, rank, world, bounds, dist, dev, local, stream)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and wl == "cfg2" and \
            args.dtype == "f32":
        result["end_to_end"] = end_to_end(insts[0], local)
        result["rows"] = bench_rows(local, insts=insts)
        result["cpu_baseline"] = cpu_baseline(insts[0], args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def f64_block(args, insts, dist, dev, local, stream):
    """The headline workload in the reference apps' value type
    (KVVector<Key,double>, batch_solver.h:32): the same --batch cfg2
    aggregates (same keys; the f32 values widened to f64, exact), the same
    timed step (partition + aggregate, K steps, barrier + synchronize,
    max over ranks).  Bytes per launch use s_V = 8."""
    f64 = [(D, [(k, [np.asarray(v, np.float64) for v in vs]) for k, vs in pushes])
           for D, pushes in insts]
    plan, keep, jobs = make_plan(f64, dev, local)
    plan.run(stream.cuda_stream)
    want = np.array([n for jb in jobs for n in jb["push_n"]], np.uint64)
    assert args.no_check or np.array_equal(plan.matched(), want), "f64: unmatched keys"
    K = args.steps
    wall, part_ms, agg_ms = timed_steps(plan, K, args.warmup, stream, dist)
    wall_max, kv_all = reduce_over_ranks(wall, plan.kv_pairs, dist, dev)
    nbytes = int(plan.bytes)
    out = {
        "dtype": "f64",
        "value": kv_all * K / wall_max,
        "unit": "kv-pairs/s",
        "ms_per_step": wall_max / K * 1e3,
        "kernel": kernel_name(plan, "f64"),
        "kernel_ms": agg_ms,
        "partition_ms": part_ms,
        "bytes_per_launch": nbytes,
        "bytes_formula": "sum_p n_p*(8+8) [pushes] + U*(8+8) [server keys + sums] (SURVEY 8d)",
        "frac": nbytes / (agg_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
        "step_frac": nbytes / (wall_max / K) / 1e9 / HBM_PEAK_GBPS,
        "data": "the f32 line's aggregates, values widened to f64",
    }
    del plan, keep
    return out


def timed_stages(stages, K, W, stream, dist):
    """Like timed_steps for a step made of `stages` (callables enqueuing on
    `stream`): W warm-up steps, then K timed steps between barrier +
    synchronize pairs.  Returns (wall s, [mean ms per stage]).  As in
    timed_steps, the timed region holds two HIP events per step, around the
    last stage (the aggregate kernel); every stage's time comes from a
    second, untimed pass of K steps with an event between each."""
    import torch

    def step():
        for f in stages:
            f()

    prewarm(step)
    for _ in range(W):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(stages) + 1)] for _ in range(K)]
    t0 = time.perf_counter()
    for s in range(K):
        for f in stages[:-1]:
            f()
        ev[s][0].record(stream)
        stages[-1]()
        ev[s][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    last = float(np.mean([ev[s][0].elapsed_time(ev[s][1]) for s in range(K)]))
    for s in range(K):  # untimed: every stage between events
        ev[s][0].record(stream)
        for i, f in enumerate(stages):
            f()
            ev[s][i + 1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    ms = [float(np.mean([ev[s][i].elapsed_time(ev[s][i + 1]) for s in range(K)]))
          for i in range(len(stages) - 1)] + [last]
    return wall, ms


def timed_rotating(plans, K, W, stream):
    """timed_stages for a step that runs plans[s % R] (partition, then
    aggregate): R independent copies of one shard's inputs and outputs, so
    consecutive steps never re-read the same bytes and a working set larger
    than the 256 MB MALL (Infinity Cache) is read from HBM.  Returns (wall s,
    mean partition ms, mean aggregate ms)."""
    import torch
    sh = stream.cuda_stream
    R = len(plans)
    rot = [0]

    def step():
        plans[rot[0] % R].run_stage(0, sh)
        plans[rot[0] % R].run_stage(1, sh)
        rot[0] += 1

    prewarm(step)
    for s in range(W):
        plans[s % R].run_stage(0, sh)
        plans[s % R].run_stage(1, sh)
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    t0 = time.perf_counter()
    for s in range(K):  # two events per step, around the aggregate (timed_steps)
        plans[s % R].run_stage(0, sh)
        ev[s][1].record(stream)
        plans[s % R].run_stage(1, sh)
        ev[s][2].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    agg = float(np.mean([ev[s][1].elapsed_time(ev[s][2]) for s in range(K)]))
    for s in range(K):  # untimed: the partition between events
        ev[s][0].record(stream)
        plans[s % R].run_stage(0, sh)
        ev[s][1].record(stream)
        plans[s % R].run_stage(1, sh)
    torch.cuda.synchronize()
    part = float(np.mean([ev[s][0].elapsed_time(ev[s][1]) for s in range(K)]))
    return wall, part, agg


def cfg5_block(args, rank, world, bounds, dist, dev, local, stream):
    """BASELINE.json configs[4]: one fixed global workload (256 pushes x
    262,144 keys over a 1 B-key space) range-partitioned over the N ranks
    by evenDivide(N), two ingress modes:
      sliced    workers slice their pushes by the server ranges (the
                reference's RNode::submit -> sliceKeyOrderedMsg), so each
                rank receives only its shard's pieces of all 256 pushes: the
                step is the merge, no data-path collective;
      unsliced  rank r receives whole pushes (256/N of them); the step is
                psg_exchange_run (device re-cut + pack + one grouped RCCL
                send/recv per peer over xGMI) followed by the merge of the
                pieces this rank received (same arrival order: sources hold
                consecutive push blocks, so the sums are bit-identical to
                the sliced leg's, checked);
    plus the whole workload on rank 0's GPU alone in the same job
    (speedup_vs_1gpu)."""
    import torch
    from parameter_server_amd import shard, synth
    from parameter_server_amd._lib import PSG_F32
    from parameter_server_amd.kv_vector import MergePlan
    t0 = time.time()
    _, pushes = synth.uniform_pushes(seed=5, union=False)
    kv_total = sum(int(k.size) for k, _ in pushes)
    pieces = synth.shard_pieces(pushes, bounds, rank)
    D = np.unique(np.concatenate([k for k, _ in pieces]))
    log(f"rank {rank}: cfg5 shard {D.size:,} keys generated in {time.time() - t0:.1f}s")
    sh = stream.cuda_stream
    K = args.cfg5_steps
    # ---- sliced ingress (the reference's mode)
    plan, keep, jobs = make_plan([(D, pieces)], dev, local)
    plan.run(sh)
    assert args.no_check or np.array_equal(plan.matched(),
                                            np.array([k.size for k, _ in pieces], np.uint64))
    wall, (part_ms, agg_ms) = timed_stages([lambda: plan.run_stage(0, sh),
                                            lambda: plan.run_stage(1, sh)], K, 2, stream, dist)
    wall_max, kv_all = reduce_over_ranks(wall, plan.kv_pairs, dist, dev)
    assert int(kv_all) == kv_total
    nbytes = int(plan.bytes)
    sliced = {
        "value": kv_total * K / wall_max,
        "ms_per_step": wall_max / K * 1e3,
        "rank0": {"slots": int(D.size), "kernel_ms": agg_ms, "partition_ms": part_ms,
                  "bytes_per_launch": nbytes,
                  "frac": nbytes / (agg_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                  "step_frac": nbytes / (wall / K) / 1e9 / HBM_PEAK_GBPS},
    }
    out_sliced = keep[0][3].clone()
    del plan, keep
    torch.cuda.empty_cache()
    out = {
        "workload": ("256 pushes x 262144 murmur-shuffled uniform keys (1e9-rank space), "
                     f"f32; fixed global workload split by evenDivide({world})"),
        "scaling": "strong",
        "n_gpus": world,
        "value": sliced["value"],
        "unit": "kv-pairs/s",
        "ms_per_step": sliced["ms_per_step"],
        "rank0": sliced["rank0"],
        "modes": {"sliced": sliced},
    }
    log(f"rank {rank}: cfg5 sliced leg {sliced['ms_per_step']:.3f} ms/step")
    # ---- unsliced ingress: whole pushes per rank, RCCL exchange in the step,
    # run in a child process per rank (its own HIP context and RCCL world),
    # so a failure of that leg cannot take this line down
    del out_sliced
    torch.cuda.empty_cache()
    out["modes"]["unsliced"] = cfg5_unsliced_child(args, rank, world, dist)
    if world > 1:
        # the same whole workload on ONE GPU (rank 0), the others waiting
        t1 = None
        if rank == 0:
            Dall = np.unique(np.concatenate([k for k, _ in pushes]))
            p1, k1, _ = make_plan([(Dall, pushes)], dev, local)
            w1, _, _ = timed_steps(p1, K, 2, stream, None)
            t1 = w1 / K
            del p1, k1
            torch.cuda.empty_cache()
        dist.barrier()
        if rank == 0:
            out["one_gpu_ms_per_step"] = t1 * 1e3
            out["speedup_vs_1gpu"] = t1 / (wall_max / K)
    else:
        out["one_gpu_ms_per_step"] = out["ms_per_step"]
        out["speedup_vs_1gpu"] = 1.0
        if not args.no_shard8:
            out["shard_of_8"] = cfg5_shard_of_8(args, pushes, dev, local, stream,
                                                out["ms_per_step"])
    return out


def cfg5_shard_of_8(args, pushes, dev, local, stream, whole_ms):
    """One-GPU per-rank measurement (NOT a scaling result): each of the 8
    evenDivide(8) shards of the cfg5 workload (range.h:85-98,
    linear_method.cc:137-145) merged exactly as rank r of an 8-GPU job runs
    it in the sliced mode -- its pieces of all 256 pushes
    (sliceKeyOrderedMsg, message.h:89-123), partition + aggregate, K steps
    -- one shard after the other on this GPU.  The max per-shard step bounds
    what 8 GPUs can reach on this path: whole-workload step / max shard step
    is the speedup ceiling before any transport cost.  A shard's working set
    (~200 MB) fits the 256 MB MALL, so each shard is timed twice: repeated
    (the same buffers every step) and rotated over ROT independent copies of
    its inputs and outputs (>= 512 MB in flight: every step reads HBM); the
    rotated ceiling is the HBM-honest one.  `launch_floor_ms` is the same
    two-launch step on a one-tile plan: the fixed cost per step that does
    not shrink with the shard."""
    from parameter_server_amd import synth
    from parameter_server_amd.kv_vector import shard_bounds
    sh = stream.cuda_stream
    K = args.cfg5_steps
    b8 = shard_bounds(8)
    shards = []
    for r in range(8):
        pieces = synth.shard_pieces(pushes, b8, r)
        D = np.unique(np.concatenate([k for k, _ in pieces]))
        plan, keep, _ = make_plan([(D, pieces)], dev, local)
        plan.run(sh)
        assert args.no_check or np.array_equal(
            plan.matched(), np.array([k.size for k, _ in pieces], np.uint64))
        wall, (part_ms, agg_ms) = timed_stages([lambda: plan.run_stage(0, sh),
                                                lambda: plan.run_stage(1, sh)], K, 2, stream, None)
        nbytes = int(plan.bytes)
        # rotated: ROT copies of the shard (the first is this plan)
        copies = [plan] + [make_plan([(D, pieces)], dev, local)[:2] for _ in range(ROT - 1)]
        plans = [copies[0]] + [c[0] for c in copies[1:]]
        for p_ in plans[1:]:
            p_.run(sh)
        rwall, rpart, ragg = timed_rotating(plans, max(K, 2 * ROT), 2 * ROT, stream)
        rK = max(K, 2 * ROT)
        shards.append({"shard": r, "slots": int(D.size), "kv": int(plan.kv_pairs),
                       "ms_per_step": wall / K * 1e3, "partition_ms": part_ms,
                       "kernel_ms": agg_ms, "bytes_per_launch": nbytes,
                       "frac": nbytes / (agg_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                       "step_frac": nbytes / (wall / K) / 1e9 / HBM_PEAK_GBPS,
                       "rotated": {"copies": ROT, "ms_per_step": rwall / rK * 1e3,
                                   "partition_ms": rpart, "kernel_ms": ragg,
                                   "frac": nbytes / (ragg * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                                   "step_frac": nbytes / (rwall / rK) / 1e9 / HBM_PEAK_GBPS},
                       "form": kernel_name(plan)})
        del plan, keep, copies, plans
        import torch
        torch.cuda.empty_cache()
    # the fixed per-step cost: the same two launches on a one-tile plan
    rng = np.random.default_rng(0)
    Dt = np.unique(rng.integers(0, 1 << 40, 2048, dtype=np.uint64))[:1024]
    tiny = [(np.sort(rng.choice(Dt, 64, replace=False)), [np.ones(64, np.float32)])
            for _ in range(8)]
    plan, keep, _ = make_plan([(Dt, tiny)], dev, local)
    wall, (tp, ta) = timed_stages([lambda: plan.run_stage(0, sh),
                                   lambda: plan.run_stage(1, sh)], K, 2, stream, None)
    floor = {"ms_per_step": wall / K * 1e3, "partition_ms": tp, "kernel_ms": ta}
    del plan, keep
    steps = [x["ms_per_step"] for x in shards]
    rsteps = [x["rotated"]["ms_per_step"] for x in shards]
    rmax = max(rsteps)
    return {
        "what": "one-GPU per-rank measurement, not a scaling result: each evenDivide(8) shard "
                "of the cfg5 workload merged (sliced ingress) on this GPU as its rank would; "
                f"'rotated' = every step on the next of {ROT} copies of the shard (>= 512 MB "
                "in flight: HBM-resident), the plain fields = the same buffers every step "
                "(~200 MB, MALL-resident)",
        "max_ms_per_step": max(steps), "min_ms_per_step": min(steps),
        "max_kernel_ms": max(x["kernel_ms"] for x in shards),
        "max_partition_ms": max(x["partition_ms"] for x in shards),
        "whole_ms_per_step": whole_ms,
        "speedup_ceiling_8_repeated": whole_ms / max(steps),
        "rotated_max_ms_per_step": rmax, "rotated_min_ms_per_step": min(rsteps),
        "rotated_max_kernel_ms": max(x["rotated"]["kernel_ms"] for x in shards),
        "rotated_max_partition_ms": max(x["rotated"]["partition_ms"] for x in shards),
        "speedup_ceiling_8": whole_ms / rmax,
        "launch_floor": floor,
        "launch_floor_share": floor["ms_per_step"] / rmax,
        "shards": shards,
    }


def cfg5_unsliced_child(args, rank, world, dist):
    """Runs `bench.py --cfg5-unsliced-child` as a child process of this rank
    (rendezvous on MASTER_PORT + 1 for N > 1) and returns rank 0's result,
    or an error record if the child failed."""
    import subprocess
    env = dict(os.environ)
    if world > 1:
        env["MASTER_PORT"] = str(int(os.environ.get("MASTER_PORT", "29500")) + 1)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cfg5-unsliced-child",
           "--cfg5-steps", str(args.cfg5_steps), "--prewarm-ms", str(args.prewarm_ms)] + \
        (["--no-check"] if args.no_check else [])
    res = {"error": "child did not report"}
    try:
        p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=None, timeout=400,
                           text=True)
        lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
        if p.returncode == 0 and lines:
            res = json.loads(lines[-1])
        elif rank == 0:
            res = {"error": f"child exit {p.returncode}"}
    except Exception as e:  # noqa: BLE001 - reported in the line
        res = {"error": repr(e)}
    if dist:
        dist.barrier()
    return res


def unsliced_child_main(args):
    """The unsliced cfg5 leg alone (bench.py --cfg5-unsliced-child): its own
    torch.distributed world (gloo, for the RCCL id) when N > 1; prints rank
    0's JSON result."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    from parameter_server_amd import synth
    from parameter_server_amd.kv_vector import shard_bounds
    bounds = shard_bounds(world)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream()
    _, pushes = synth.uniform_pushes(seed=5, union=False)
    kv_total = sum(int(k.size) for k, _ in pushes)
    pieces = synth.shard_pieces(pushes, bounds, rank)
    D = np.unique(np.concatenate([k for k, _ in pieces]))
    # the sliced merge of the same pieces, once (the bit-exactness reference)
    ref = None
    if not args.no_check:
        plan, keep, _ = make_plan([(D, pieces)], dev, local)
        plan.run(stream.cuda_stream)
        torch.cuda.synchronize()
        ref = keep[0][3].clone()
        del plan, keep
        torch.cuda.empty_cache()
    r = cfg5_unsliced(args, rank, world, bounds, dist, dev, local, stream, pushes, D, ref,
                      kv_total)
    if rank == 0:
        print(json.dumps(r), flush=True)
    if dist:
        dist.destroy_process_group()


def cfg5_unsliced(args, rank, world, bounds, dist, dev, local, stream, pushes, D, out_sliced,
                  kv_total):
    """The cfg5 step with unsliced ingress (mode B): rank r holds pushes
    [r*P/N, (r+1)*P/N) whole; psg_exchange_run re-homes their pieces over
    RCCL, then the plan merges the pieces this rank received."""
    import torch
    from parameter_server_amd import shard
    from parameter_server_amd._lib import PSG_F32
    from parameter_server_amd.kv_vector import MergePlan
    P = len(pushes)
    a, b = rank * P // world, (rank + 1) * P // world
    sh = stream.cuda_stream
    dp = [(to_dev(k, dev), [to_dev(v, dev) for v in vs]) for k, vs in pushes[a:b]]
    log(f"rank {rank}: unsliced cfg5 leg: {b - a} whole pushes, RCCL communicator")
    comm = shard.make_comm(local, rank, world, dist)
    x = shard.RcclExchange(comm, dp, world, PSG_F32)
    log(f"rank {rank}: exchange set up: {x.nsent:,} keys to peers, {x.nrecv:,} received")
    try:
        pcs = x.pieces()  # (offset, count) per (source, push), arrival order
        dD = to_dev(D, dev)
        res = torch.empty(max(1, D.size), dtype=torch.float32, device=dev)
        job = {"keys": dD.data_ptr(), "nslots": int(D.size),
               "push_keys": [x.recv_keys_ptr + 8 * o for o, _ in pcs],
               "push_vals": [[x.recv_vals_ptr[0] + 4 * o] for o, _ in pcs],
               "push_n": [c for _, c in pcs], "out": [res.data_ptr()]}
        plan = MergePlan(local, PSG_F32, 1, [job])
        x.run(sh)
        plan.run(sh)
        ref_bits = res.view(torch.int32).clone()
        if not args.no_check:
            assert np.array_equal(plan.matched(), np.array([c for _, c in pcs], np.uint64))
            assert x.status() == 0
            # same pushes, same arrival order as the sliced leg: same bits
            assert out_sliced is None or torch.equal(res.view(torch.int32),
                                                     out_sliced.view(torch.int32)), \
                "unsliced cfg5 merge differs from the sliced one"
        K = args.cfg5_steps
        wall, (x_ms, part_ms, agg_ms) = timed_stages(
            [lambda: x.run(sh), lambda: plan.run_stage(0, sh), lambda: plan.run_stage(1, sh)],
            K, 2, stream, dist)
        wall_max, kv_all = reduce_over_ranks(wall, plan.kv_pairs, dist, dev)
        assert int(kv_all) == kv_total
        assert args.no_check or x.status() == 0
        # A/B of the transport: peer-bound pieces sent straight from the push
        # arrays (psg_exchange_set_direct) instead of packed first; the same
        # received bytes, checked against the packed run's merge
        x.set_direct(True)
        x.run(sh)
        plan.run(sh)
        if not args.no_check:
            assert torch.equal(res.view(torch.int32), ref_bits), "direct exchange differs"
        wall_d, (x_ms_direct,) = timed_stages([lambda: x.run(sh)], K, 2, stream, dist)
        x.set_direct(False)
        _, _, send_cnt = x.send_layout()
        per_dest = send_cnt.sum(axis=1) * 12  # keys + f32 values
        peers = [s for s in range(world) if s != rank]
        to_peers = int(sum(per_dest[s] for s in peers))
        peer_max = int(max((per_dest[s] for s in peers), default=0))
        xs = x_ms * 1e-3
        res_out = {
            "value": kv_total * K / wall_max,
            "ms_per_step": wall_max / K * 1e3,
            "rank0": {"exchange_ms": x_ms, "exchange_ms_direct": x_ms_direct,
                      "partition_ms": part_ms, "kernel_ms": agg_ms,
                      "pushes_held": b - a, "bytes_sent_to_peers": to_peers,
                      "bytes_kept_local": int(per_dest[rank]),
                      "max_bytes_to_one_peer": peer_max,
                      "GBps_to_peers": to_peers / xs / 1e9 if peers else None,
                      "GBps_per_peer_max": peer_max / xs / 1e9 if peers else None},
            "step": "psg_exchange_run (device re-cut + pack + grouped RCCL send/recv) + "
                    "partition + aggregate of the received pieces",
        }
        del plan, dD, res
        return res_out
    finally:
        x.close()
        shard.destroy_comm(comm)
        del dp


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


def copy_bandwidth(dev, stream):
    """HBM copy ceiling in the same run: tools/copybw (a hand-written 16-B
    per lane copy kernel), 1 GiB -> 1 GiB, read + write bytes / time."""
    import torch
    path = os.path.join(ROOT, "tools", "copybw", "libcopybw.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.copybw_copy.restype = ctypes.c_int
    L.copybw_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    nbytes = 1 << 30
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    sh = stream.cuda_stream
    for _ in range(3):
        L.copybw_copy(dst.data_ptr(), src.data_ptr(), nbytes, sh)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(10):
        L.copybw_copy(dst.data_ptr(), src.data_ptr(), nbytes, sh)
    e1.record(stream)
    torch.cuda.synchronize()
    gbps = 2 * nbytes * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    return gbps


def end_to_end(inst, device, reps=7, only=None):
    """PCIe-inclusive rate of one cfg2 aggregate through the host C ABI, the
    reference's own call pattern (setValue per push, then received(t) with
    the D2H of the merged shard), driven from C++ (tools/e2e/libe2e.so, no
    Python in the loop).  Caller setups:
      pageable       keys+values and output in pageable memory (CPU copy into
                     the pinned staging ring, DMA overlapped with the next push);
      pinned         pinned host memory, read by the GPU itself (zero-copy
                     kernel); each push waits for it (the caller's buffers
                     are free on return);
      pinned_hold    pinned, PSG_HOLD_BUFFERS (buffers held until received,
                     as a MessagePtr holds its SArrays): no wait per push;
      pinned_cached  pinned_hold, and each worker's keys come from the key
                     cache (RNode::cacheKeyRecver): only values cross PCIe;
      darling_fused  the Darling server step on the same keys: f64 (G, U)
                     pushes from the key cache, then the fused updateWeight
                     on the device (psg_darling_update): no aggregate D2H.
    Reported beside `value`, never as it."""
    import ctypes as C
    import torch
    from parameter_server_amd import _lib
    L = _lib.lib()
    E = C.CDLL(os.path.join(ROOT, "tools", "e2e", "libe2e.so"))
    E.psg_e2e.restype = C.c_int
    D, pushes = inst
    kv = sum(int(k.size) for k, _ in pushes)
    npush = len(pushes)
    # the senders' key signatures, on the device (psg_crc32c_dev)
    dev = "cuda:%d" % device
    keys = torch.from_numpy(np.concatenate([k for k, _ in pushes]).view(np.int64)).to(dev)
    off = np.concatenate([[0], np.cumsum([8 * k.size for k, _ in pushes])]).astype(np.uint64)
    doff = torch.from_numpy(off.view(np.int64)).to(dev)
    dsig = torch.zeros(npush, dtype=torch.int32, device=dev)
    _lib.check(L.psg_crc32c_dev(keys.data_ptr(), doff.data_ptr(), npush, _lib.PSG_MAX_SIG_LEN,
                                None, dsig.data_ptr(), None))
    sigs = np.ascontiguousarray(dsig.cpu().numpy().view(np.uint32))
    del keys, doff, dsig
    out = {}
    for mode in ("pageable", "pinned", "pinned_hold", "pinned_cached"):
        if only and mode not in only:
            continue
        pin = mode != "pageable"
        if pin:
            src = [(torch.from_numpy(k.view(np.int64)).pin_memory().numpy().view(np.uint64),
                    torch.from_numpy(vs[0]).pin_memory().numpy()) for k, vs in pushes]
            res = torch.empty(D.size, dtype=torch.float32, pin_memory=True).numpy()
        else:
            src = [(k, vs[0]) for k, vs in pushes]
            res = np.empty(D.size, np.float32)
        kp = (C.c_void_p * npush)(*[k.ctypes.data for k, _ in src])
        ns = (C.c_size_t * npush)(*[k.size for k, _ in src])
        vp = (C.c_void_p * npush)(*[v.ctypes.data for _, v in src])
        ms = np.zeros(reps + 1, np.float64)
        hold = mode in ("pinned_hold", "pinned_cached")
        flags = _lib.PSG_SERIAL_MATCH | (_lib.PSG_HOLD_BUFFERS if hold else 0)
        rc = E.psg_e2e(C.c_int(device), C.c_int(_lib.PSG_F32), C.c_uint(flags),
                       C.c_void_p(D.ctypes.data), C.c_size_t(D.size), C.c_int(npush), kp, ns, vp,
                       C.c_void_p(sigs.ctypes.data) if mode == "pinned_cached" else None,
                       C.c_void_p(res.ctypes.data), C.c_int(reps + 1),
                       C.c_void_p(ms.ctypes.data))
        _lib.check(rc)
        t = float(np.median(ms[1:])) * 1e-3
        out[mode] = {"value": kv / t, "ms_per_aggregate": t * 1e3}
    if not only or "compressed" in only:
        # compressed messages (the worker's compressTo, van.cc:204-214): each
        # push's key and value parts snappy-compressed by the harness, pinned,
        # through psg_push_compressed (decoded on the device), then received
        E.psg_e2e_compress.restype = C.c_size_t
        cparts = []
        for k, vs in pushes:
            pair = []
            for raw in (np.ascontiguousarray(k).view(np.uint8), np.ascontiguousarray(vs[0]).view(np.uint8)):
                buf = np.empty(32 + raw.size + raw.size // 6, np.uint8)
                nb = E.psg_e2e_compress(C.c_void_p(raw.ctypes.data), C.c_size_t(raw.size),
                                        C.c_void_p(buf.ctypes.data))
                pin = torch.empty(nb, dtype=torch.uint8, pin_memory=True).numpy()
                pin[:] = buf[:nb]
                pair.append(pin)
            cparts.append(pair)
        ck = (C.c_void_p * npush)(*[a.ctypes.data for a, _ in cparts])
        ckn = (C.c_size_t * npush)(*[a.size for a, _ in cparts])
        cv = (C.c_void_p * npush)(*[b.ctypes.data for _, b in cparts])
        cvn = (C.c_size_t * npush)(*[b.size for _, b in cparts])
        res = torch.empty(D.size, dtype=torch.float32, pin_memory=True).numpy()
        ms = np.zeros(reps + 1, np.float64)
        _lib.check(E.psg_e2e_compressed(C.c_int(device), C.c_int(_lib.PSG_F32),
                                        C.c_uint(_lib.PSG_SERIAL_MATCH), C.c_void_p(D.ctypes.data),
                                        C.c_size_t(D.size), C.c_int(npush), ck, ckn, cv, cvn,
                                        C.c_void_p(res.ctypes.data), C.c_int(reps + 1),
                                        C.c_void_p(ms.ctypes.data)))
        t = float(np.median(ms[1:])) * 1e-3
        cbytes = sum(a.size + b.size for a, b in cparts)
        out["compressed"] = {"value": kv / t, "ms_per_aggregate": t * 1e3,
                             "compressed_bytes": cbytes, "ratio": cbytes / (12 * kv)}
    if not only or "darling_fused" in only:
        # the Darling server step on the same keys (f64 G and U from pinned
        # memory, keys from the key cache, fused updateWeight: nothing D2H)
        rng = np.random.default_rng(77)
        GU = [(torch.from_numpy(rng.standard_normal(k.size)).pin_memory().numpy(),
               torch.from_numpy(rng.random(k.size)).pin_memory().numpy()) for k, _ in pushes]
        kp = (C.c_void_p * npush)(*[k.ctypes.data for k, _ in pushes])
        ns = (C.c_size_t * npush)(*[k.size for k, _ in pushes])
        gp = (C.c_void_p * npush)(*[g.ctypes.data for g, _ in GU])
        up = (C.c_void_p * npush)(*[u.ctypes.data for _, u in GU])
        ms = np.zeros(reps + 1, np.float64)
        vio = C.c_double()
        _lib.check(E.psg_e2e_darling(C.c_int(device), C.c_uint(_lib.PSG_HOLD_BUFFERS),
                                     C.c_void_p(D.ctypes.data), C.c_size_t(D.size), C.c_int(npush),
                                     kp, ns, gp, up, C.c_void_p(sigs.ctypes.data), C.c_int(reps + 1),
                                     C.c_void_p(ms.ctypes.data), C.byref(vio)))
        t = float(np.median(ms[1:])) * 1e-3
        out["darling_fused"] = {"value": kv / t, "ms_per_aggregate": t * 1e3, "dtype": "f64", "m": 2}
    # the link itself: pinned <-> device copies of 64 MB (torch, same streams)
    link = {}
    hbuf = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    for name, (dst, srcb) in (("h2d", (dbuf, hbuf)), ("d2h", (hbuf, dbuf))):
        dst.copy_(srcb, non_blocking=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            dst.copy_(srcb, non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        link[name + "_GBps"] = 10 * (64 << 20) / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del hbuf, dbuf
    # bytes that must cross the link per aggregate in each mode
    vb, kb, ob = 4 * kv, 8 * kv, 4 * D.size
    for mode, b, ob in (("pageable", kb + vb + ob, ob), ("pinned", kb + vb + ob, ob),
                        ("pinned_hold", kb + vb + ob, ob), ("pinned_cached", vb + ob, ob),
                        ("compressed", out.get("compressed", {}).get("compressed_bytes", 0) + ob,
                         ob),
                        ("darling_fused", 16 * kv, 0)):
        if mode not in out:
            continue
        bound = (b - ob) / (link["h2d_GBps"] * 1e9) + ob / (link["d2h_GBps"] * 1e9)
        out[mode]["link_bytes"] = b
        out[mode]["frac_of_link"] = bound * 1e3 / out[mode]["ms_per_aggregate"]
    return {"value": out.get("pinned_hold", {}).get("value"), "unit": "kv-pairs/s", "modes": out,
            "link": link,
            "scope": ("one cfg2 aggregate (8 pushes x 131,072 keys): 8 x psg_push (H2D, merge) "
                      "+ psg_received (D2H of the 956,827-slot shard), C++ caller, median of "
                      f"{reps}; value = the pinned_hold mode")}


def cfg4_server_api(inst, device, reps=5, pinned_out=True):
    """cfg4 through the server API, the reference's call pattern
    (KVVector::setValue per push, then received(t)): 8 x psg_push of pinned
    keys + values (PSG_HOLD_BUFFERS) + psg_received into pinned memory.
    psg_push's O(1) dense test routes every push to the dense kernel; the
    keys are order-checked where they lie (zero-copy, never staged).  Wall
    time per aggregate, PCIe included; the merge's device time is in the
    committed kernel trace (tools/run_cfg4_server.py under rocprofv3)."""
    import torch
    from parameter_server_amd import _lib
    from parameter_server_amd.kv_vector import KVVector, Message
    D, pushes = inst
    kv = sum(int(k.size) for k, _ in pushes)
    hk = [torch.from_numpy(k.view(np.int64)).pin_memory() for k, _ in pushes]
    hv = [torch.from_numpy(vs[0]).pin_memory() for _, vs in pushes]
    # pinned out: the merge kernel writes the sums straight into host memory
    # (its stores are the D2H); pageable out: sums in HBM, then a DMA copy
    res = (torch.empty(D.size, dtype=torch.float32, pin_memory=True).numpy() if pinned_out
           else np.empty(D.size, np.float32))
    v = KVVector(device, _lib.PSG_F32, flags=_lib.PSG_HOLD_BUFFERS)
    v.setValue(Message(key=D))
    times = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        for k, x in zip(hk, hv):
            v.setValue(Message(time=r, key=k.numpy().view(np.uint64), value=[x.numpy()]))
        v.received(r, out=[res])
        if r:
            times.append(time.perf_counter() - t0)
    v.close()
    t = float(np.median(times))
    link = kv * (4 + 8) + D.size * 4
    return {"value": kv / t, "unit": "kv-pairs/s", "ms_per_aggregate": t * 1e3,
            "link_bytes": link, "link_GBps": link / t / 1e9,
            "scope": ("8 x psg_push (pinned, held) + psg_received of one cfg4 aggregate "
                      f"(8 x 16,777,216 kv), median of {reps}: PCIe-inclusive, never `value`")}


def load_traffic(bytes_per_launch, workload):
    """HBM bytes per launch of the aggregate and partition kernels from the
    committed rocprofv3 PMC summary of this workload
    (profiles/pmc_summary_<workload>.json, or profiles/pmc_summary.json for
    cfg2; written by tools/pmc_traffic.py), when it was collected on this
    same workload and size; else null."""
    d = None
    for name in (f"pmc_summary_{workload}.json", "pmc_summary.json"):
        try:
            d = json.load(open(os.path.join(ROOT, "profiles", name)))
            break
        except Exception:
            continue
    if d is None:
        return None
    if d.get("bytes_per_launch") != bytes_per_launch or d.get("workload", "cfg2") != workload:
        return None
    return {"tile": d.get("hbm_bytes_per_launch"),
            "partition": d.get("partition_hbm_bytes_per_launch"),
            "source": d.get("source")}


def bench_rows(device, reps=5, insts=None, only=None):
    """The SURVEY 8(f) rows beside the merge, each on device-resident input
    with its own HBM roofline: algorithmic bytes / mean kernel time (HIP
    events on the stream the kernel runs on).  Shapes: the N-way merge of
    cfg2's pushes (keys only: the key union; with values: union + sums;
    a run is 5 small kernels), the pull of a cfg2
    shard, crc32c key signatures of 65,536 pushes and one 1 GiB stream,
    snappy parts of 64 KB, Darling over 16.8 M f64 positions, CountMin
    insert/query of 16.8 M keys into 2^26 counters."""
    import ctypes as C
    import torch
    from parameter_server_amd import _lib, synth
    from parameter_server_amd.kv_vector import KVVector, Message
    L = _lib.lib()
    dev = torch.device("cuda", device)
    st = torch.cuda.current_stream()
    out = {}

    def timed(fn):
        prewarm(fn)  # the clock ramp, as before every timed region (PREWARM_S)
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps  # ms

    def row(name, ms, nbytes, unit_count, unit):
        gbps = nbytes / (ms * 1e-3) / 1e9
        out[name] = {"ms": ms, "algorithmic_bytes": nbytes, "GBps": gbps,
                     "frac": gbps / HBM_PEAK_GBPS, "rate": unit_count / (ms * 1e-3),
                     "unit": unit}

    rng = np.random.default_rng(3)
    D, pushes = synth.overlap_pushes(1)
    if only is None or 'nway' in only:
        # N-way merge (psg_nway): cfg2's 8 key-only pushes ->
        # the merged key set (BatchSolver's key pushes, setUnion push after
        # push), and the same pushes with their f32 values -> union + sums
        from parameter_server_amd.kv_vector import NWayMerge
        dk = [torch.from_numpy(k.view(np.int64)).to(dev) for k, _ in pushes]
        dv = [torch.from_numpy(vs[0]).to(dev) for _, vs in pushes]
        tot = sum(k.size for k, _ in pushes)
        ok = torch.empty(tot, dtype=torch.int64, device=dev)
        ov = torch.empty(tot, dtype=torch.float32, device=dev)
        for name, m in (("key_union", 0), ("nway_merge_1agg", 1)):
            u = NWayMerge(device, _lib.PSG_F32, [t.data_ptr() for t in dk], [k.size for k, _ in pushes],
                          [[t.data_ptr()] for t in dv] if m else [[] for _ in dk], ok.data_ptr(),
                          [ov.data_ptr()] if m else [])
            u.run()
            nu = u.result()
            assert nu == D.size, "N-way union size"
            ms = timed(lambda: u.run(st.cuda_stream))
            assert u.result() == D.size
            u.close()
            row(name, ms, tot * (8 + 4 * m) + D.size * (8 + 4 * m), tot, "keys/s")
            out[name]["shape"] = ("8 pushes x 131,072 sorted keys (cfg2) -> U = 956,827 merged keys" +
                                  (" + f32 sums" if m else ""))
        assert np.array_equal(ok[:D.size].cpu().numpy().view(np.uint64), D)
        del dk, dv, ok, ov
        if insts:
            # the N-way merge at the headline's scale: its --batch cfg2
            # aggregates (keys + f32 values) as one pipeline (psg_nway_create_batch:
            # one launch per stage over every aggregate)
            from parameter_server_amd.kv_vector import NWayMergeBatch
            keepb, merges, nb, kvb = [], [], 0, 0
            for Dj, ps in insts:
                dkb = [torch.from_numpy(k.view(np.int64)).to(dev) for k, _ in ps]
                dvb = [torch.from_numpy(vs[0]).to(dev) for _, vs in ps]
                totb = sum(k.size for k, _ in ps)
                okb = torch.empty(totb, dtype=torch.int64, device=dev)
                ovb = torch.empty(totb, dtype=torch.float32, device=dev)
                keepb.append((dkb, dvb, okb, ovb))
                merges.append(dict(push_keys=[t.data_ptr() for t in dkb],
                                   push_n=[k.size for k, _ in ps],
                                   push_vals=[[t.data_ptr()] for t in dvb],
                                   out_keys=okb.data_ptr(), out_vals=[ovb.data_ptr()]))
                nb += totb * 12 + Dj.size * 12
                kvb += totb
            u = NWayMergeBatch(device, _lib.PSG_F32, merges)
            u.run()
            assert u.result() == [Dj.size for Dj, _ in insts], "batched N-way union sizes"
            ms = timed(lambda: u.run(st.cuda_stream))
            u.result()
            u.close()
            row("nway_merge", ms, nb, kvb, "keys/s")
            out["nway_merge"]["shape"] = (f"{len(insts)} cfg2 aggregates (8 pushes x 131,072 keys + "
                                          "f32 values each -> U = 956,827 keys + sums), one pipeline")
            del keepb, merges
    if only is None or 'gather' in only:
        # pull gather (getValue) of 1 M sorted request keys from a cfg2 shard
        req = np.sort(np.concatenate([k for k, _ in pushes[:8]]))[::1]
        dD = torch.from_numpy(D.view(np.int64)).to(dev)
        dW = torch.from_numpy(rng.standard_normal(D.size).astype(np.float32)).to(dev)
        dR = torch.from_numpy(req.view(np.int64)).to(dev)
        dO = torch.empty(req.size, dtype=torch.float32, device=dev)
        dM = torch.zeros(1, dtype=torch.int64, device=dev)
        ms = timed(lambda: _lib.check(L.psg_gather_dev(_lib.PSG_F32, dD.data_ptr(), D.size,
                                                       dW.data_ptr(), dR.data_ptr(), req.size,
                                                       dO.data_ptr(), dM.data_ptr(), None)))
        row("gather", ms, req.size * (8 + 4 + 4), req.size, "keys/s")
        del dD, dW, dR, dO
    if only is None or 'crc' in only:
        # crc32c: key signatures (2048 B of each of 65,536 pushes) and one 1 GiB stream
        nsig = 65536
        blob = torch.randint(0, 255, (nsig * 4096,), dtype=torch.uint8, device=dev)
        off = torch.arange(0, nsig + 1, dtype=torch.int64, device=dev) * 4096
        sig = torch.empty(nsig, dtype=torch.int32, device=dev)
        ms = timed(lambda: _lib.check(L.psg_crc32c_dev(blob.data_ptr(), off.data_ptr(), nsig,
                                                       _lib.PSG_MAX_SIG_LEN, None, sig.data_ptr(),
                                                       None)))
        row("crc32c_signatures", ms, nsig * 2048, nsig, "signatures/s")
        big = torch.randint(0, 255, (1 << 30,), dtype=torch.uint8, device=dev)
        off1 = torch.tensor([0, 1 << 30], dtype=torch.int64, device=dev)
        ms = timed(lambda: _lib.check(L.psg_crc32c_dev(big.data_ptr(), off1.data_ptr(), 1, 1 << 30,
                                                       None, sig.data_ptr(), None)))
        row("crc32c_stream", ms, 1 << 30, 1 << 30, "bytes/s")
        del blob, big
    if only is None or 'snappy' in only:
        # snappy: 2048 parts of 64 KB, each a synthetic raw stream of alternating
        # 16-byte literals and 16-byte copies (2-byte offsets): 4096 elements per
        # part, the element density of typical snappy output
        nparts, plen = 2048, 65536

        def part(seed):
            # per 32 output bytes: a literal of 16 (tag 15 << 2, 16 bytes),
            # then a copy of 16 (tag 2 | 15 << 2, 2-byte offset in [1, min(o, 4096)])
            r = np.random.default_rng(seed)
            npair = plen // 32
            o = 32 * np.arange(npair, dtype=np.int64) + 16
            off = r.integers(1, np.minimum(o, 4096) + 1)
            rec = np.empty((npair, 20), np.uint8)
            rec[:, 0] = 15 << 2
            rec[:, 1:17] = r.integers(0, 256, (npair, 16), dtype=np.uint8)
            rec[:, 17] = 2 | (15 << 2)
            rec[:, 18] = off & 0xff
            rec[:, 19] = off >> 8
            return bytes([0x80, 0x80, 0x04]) + rec.tobytes()  # varint 65536

        parts = [part(i % 16) for i in range(nparts)]
        soff = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.uint64)
        dsrc = torch.from_numpy(np.frombuffer(b"".join(parts), np.uint8).copy()).to(dev)
        dso = torch.from_numpy(soff.view(np.int64)).to(dev)
        ddo = torch.arange(0, nparts + 1, dtype=torch.int64, device=dev) * plen
        ddst = torch.empty(nparts * plen, dtype=torch.uint8, device=dev)
        dst_ = torch.empty(nparts, dtype=torch.int32, device=dev)
        ms = timed(lambda: _lib.check(L.psg_snappy_uncompress_dev(
            dsrc.data_ptr(), dso.data_ptr(), nparts, ddst.data_ptr(), ddo.data_ptr(),
            dst_.data_ptr(), None)))
        assert int(dst_.abs().sum().item()) == 0, "snappy row: a part failed to decode"
        row("snappy_uncompress", ms, int(soff[-1]) + nparts * plen, nparts * plen,
            "uncompressed bytes/s")
        del dsrc, ddst
        # snappy, incompressible 1 MB parts (a cfg2 push's key part: what snappy
        # emits for random data is one 65,536-byte literal per block), 16 parts:
        # the parse defers the literals, the copy kernel moves them chip-wide
        nbig, blen = 16, 1 << 20

        def lit_part(seed):
            r = np.random.default_rng(seed)
            b = bytearray([0x80, 0x80, 0x40])  # varint 1 MiB
            for _ in range(blen // 65536):
                b += bytes([61 << 2, 0xff, 0xff]) + r.integers(0, 256, 65536, dtype=np.uint8).tobytes()
            return bytes(b)

        parts = [lit_part(i) for i in range(nbig)]
        soff = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.uint64)
        dsrc = torch.from_numpy(np.frombuffer(b"".join(parts), np.uint8).copy()).to(dev)
        dso = torch.from_numpy(soff.view(np.int64)).to(dev)
        ddo = torch.arange(0, nbig + 1, dtype=torch.int64, device=dev) * blen
        ddst = torch.empty(nbig * blen, dtype=torch.uint8, device=dev)
        dst_ = torch.empty(nbig, dtype=torch.int32, device=dev)
        ms = timed(lambda: _lib.check(L.psg_snappy_uncompress_dev(
            dsrc.data_ptr(), dso.data_ptr(), nbig, ddst.data_ptr(), ddo.data_ptr(),
            dst_.data_ptr(), None)))
        assert int(dst_.abs().sum().item()) == 0, "snappy row: a large part failed to decode"
        row("snappy_uncompress_1MB_parts", ms, int(soff[-1]) + nbig * blen, nbig * blen,
            "uncompressed bytes/s")
        del dsrc, ddst
    if only is None or 'countmin' in only:
        # CountMin: insertKeys / queryKeys of 16.8 M keys, 2^26 counters, k = 4
        v = KVVector(device)
        nk = 1 << 24
        keys = torch.randint(0, 1 << 62, (nk,), dtype=torch.int64, device=dev)
        cnt = torch.randint(1, 100, (nk,), dtype=torch.int32, device=dev)
        _lib.check(L.psg_freq_resize(v._h, 0, 1 << 26, 4))
        ms = timed(lambda: _lib.check(L.psg_freq_insert_dev(v._h, 0, keys.data_ptr(),
                                                            cnt.data_ptr(), nk, None)))
        # keys + counts read; per probe one counter byte read and written
        # (countmin.h:69: uint8 counters, the table 64 MB)
        row("countmin_insert", ms, nk * (8 + 4) + nk * 4 * 2, nk, "keys/s")
        scratch = torch.empty(L.psg_freq_query_scratch_bytes(nk), dtype=torch.uint8, device=dev)
        qo = torch.empty(nk, dtype=torch.int64, device=dev)
        qn = torch.zeros(1, dtype=torch.int64, device=dev)
        ms = timed(lambda: _lib.check(L.psg_freq_query_dev(v._h, 0, keys.data_ptr(), nk, 200,
                                                           qo.data_ptr(), qn.data_ptr(),
                                                           scratch.data_ptr(), None)))
        kept = int(qn.item())
        # keys read by the count and the scatter pass, one byte per probe, kept keys written
        row("countmin_query", ms, nk * 8 * 2 + nk * 4 + kept * 8, nk, "keys/s")
        v.close()
        del keys, cnt, qo, scratch
    if only is None or 'darling' in only:
        # Darling's server step over 16.8 M f64 positions: the (G, U) aggregate of
        # one resident push plus the fused updateWeight (nothing crosses PCIe)
        n = 1 << 24
        Dk = np.arange(n, dtype=np.uint64) * np.uint64(3)
        v = KVVector(device, _lib.PSG_F64)
        v.setValue(Message(key=Dk))
        v.set_value_array(0, np.zeros(n))
        _lib.check(L.psg_darling_init(v._h, 0, 1.0))
        G = rng.standard_normal(n)
        U = rng.random(n)
        P = (C.c_double * 4)(1.0, 0.1, 1e20, 5.0)
        vio = C.c_double()
        times = []
        for r in range(reps + 1):
            v.setValue(Message(time=r, key=Dk, value=[G, U]))  # H2D here, untimed
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _lib.check(L.psg_darling_update(v._h, 0, r, C.cast(P, C.c_void_p), C.byref(vio)))
            if r:
                times.append(time.perf_counter() - t0)
        v.close()
        ms = float(np.median(times)) * 1e3
        # aggregate (dense: values in, sums out) + update (G, U, w, delta r/w)
        row("darling_server_step", ms, n * 16 + n * 16 + n * (16 + 16 + 16), n, "positions/s")
    return out


def cpu_baseline(inst, seconds):
    """The oracle's restatement of the reference CPU path (serialSetValue:
    oldMatch + dense +=, the shipped default) on one cfg2 aggregate,
    repeated for ~`seconds` on this host; plus the threaded match path."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    from parameter_server_amd import synth
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
    # 4 threads (local.sh:25) and nproc; plus this job's CPU
    # share (16 on the GPU box, whose cgroup quota also throttles nproc)
    nproc = os.cpu_count() or 1
    for nt in sorted({4, max(1, min(16, share)), nproc}):
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
    # the key union the reference's way: setUnion push after push
    # (shared_array_inl.h:155-162) on one core, beside rows.key_union
    _, kpushes = synth.overlap_pushes(1)
    ktot = sum(int(k.size) for k, _ in kpushes)
    t0, ureps = time.perf_counter(), 0
    while time.perf_counter() - t0 < 1.0:
        acc = np.zeros(0, np.uint64)
        for k, _ in kpushes:
            acc = O.set_union(acc, k)
        ureps += 1
    union_rate = ureps * ktot / (time.perf_counter() - t0)
    return {
        "value": v, "unit": "kv-pairs/s", "cores": 1, "kind": "port",
        "setUnion_keys_per_s": union_rate,
        "sample": (f"{reps} x one cfg2 aggregate (8 x 131072 kv, U={D.size}) through the "
                   f"oracle's serialSetValue restatement in {el:.1f}s on 1 thread of {model} "
                   f"(host: nproc {os.cpu_count()}, this job's affinity {share} CPUs); the "
                   "same 24 MB aggregate is re-run, so its inputs are warm in the host's L3"),
        "parallel_match_by_threads": par,
    }


if __name__ == "__main__":
    main()
