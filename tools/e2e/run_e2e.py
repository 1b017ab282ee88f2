"""MEASUREMENT AID: bench.py's end-to-end host-path measurement alone, for a
rocprofv3 timeline (--memory-copy-trace --kernel-trace --hip-runtime-trace).
usage: python tools/e2e/run_e2e.py [reps] [mode,...]  (modes: compressed only with
"compressed"; the uncompressed modes by name)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from parameter_server_amd import synth  # noqa: E402

if __name__ == "__main__":
    import torch
    assert torch.cuda.is_available()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    lo, hi = 0, (1 << 64) - 1
    inst = synth.shard_instance(seed=1, lo=lo, hi=hi)
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    print(json.dumps(bench.end_to_end(inst, 0, reps=reps, only=only)))
