"""MEASUREMENT AID: pinned host <-> device copy time vs size (torch copies on
one stream, each synchronised), to see the per-copy overhead of the link."""
import json
import time

import torch

assert torch.cuda.is_available()
res = {}
for sz in (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
    h = torch.empty(sz, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(sz, dtype=torch.uint8, device="cuda")
    for name, (dst, src) in (("h2d", (d, h)), ("d2h", (h, d))):
        for _ in range(3):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        t0 = time.perf_counter()
        e0.record()
        for _ in range(n):
            dst.copy_(src, non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n
        gpu = e0.elapsed_time(e1) * 1e-3 / n
        res["%s_%dK" % (name, sz >> 10)] = {"us": round(gpu * 1e6, 1), "GBps": round(sz / gpu / 1e9, 1),
                                             "wall_us": round(wall * 1e6, 1)}
print(json.dumps(res, indent=0))
