"""MEASUREMENT AID: bench.py's 8(f)-row block alone (python tools/run_rows.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    assert torch.cuda.is_available()
    print(json.dumps(bench.bench_rows(0), indent=1))
