"""MEASUREMENT AID: cfg5 (256 pushes x 262,144 sparse keys over a 1e9-rank
space, U = 64.9 M) through the server API -- KVVector::setValue per push,
then received(t) -- so a rocprofv3 kernel trace shows the merge kernel's
device time on the pushes as the context stages them (pool blocks carved
from slabs), to compare with the plan API's `--layout arena/separate`:
  rocprofv3 --kernel-trace --stats -d <dir> -o run -- python3 tools/run_cfg5_server.py
Pinned pushes with PSG_HOLD_BUFFERS; the sums stay in HBM (pageable out)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch
    from parameter_server_amd import _lib, synth
    from parameter_server_amd.kv_vector import KVVector, Message
    assert torch.cuda.is_available()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    D, pushes = synth.uniform_pushes(seed=5)
    hk = [torch.from_numpy(k.view(np.int64)).pin_memory().numpy().view(np.uint64) for k, _ in pushes]
    hv = [torch.from_numpy(vs[0]).pin_memory().numpy() for _, vs in pushes]
    v = KVVector(0, _lib.PSG_F32, flags=_lib.PSG_HOLD_BUFFERS)
    v.setValue(Message(key=D))
    res = np.empty(D.size, np.float32)
    times = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        for k, x in zip(hk, hv):
            v.setValue(Message(time=r, key=k, value=[x]))
        v.received(r, out=[res])
        times.append(time.perf_counter() - t0)
    v.close()
    kv = sum(int(k.size) for k, _ in pushes)
    print(json.dumps({"kv": kv, "U": int(D.size), "ms_per_aggregate": float(np.median(times[1:])) * 1e3,
                      "scope": "256 x psg_push (pinned, held) + psg_received (pageable out)"}))
