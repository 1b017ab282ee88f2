"""MEASUREMENT AID: bench.py's 8(f)-row block alone (python tools/run_rows.py
[group ...]; groups: nway gather crc snappy countmin darling, default all)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    assert torch.cuda.is_available()
    only = set(sys.argv[1:]) or None
    print(json.dumps(bench.bench_rows(0, only=only), indent=1))
