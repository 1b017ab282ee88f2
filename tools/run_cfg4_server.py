"""MEASUREMENT AID: cfg4 through the server API alone (bench.cfg4_server_api),
for a rocprofv3 kernel trace of the merge's device time:
  rocprofv3 --kernel-trace --stats -d <dir> -o run -- python3 tools/run_cfg4_server.py [--pageable-out]
(--pageable-out: the sums stay in HBM and a DMA copy follows, so the merge
kernel's duration is the device merge alone)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    from parameter_server_amd import synth
    assert torch.cuda.is_available()
    pinned = "--pageable-out" not in sys.argv
    print(json.dumps(bench.cfg4_server_api(synth.dense_pushes(seed=4), 0, pinned_out=pinned)))
