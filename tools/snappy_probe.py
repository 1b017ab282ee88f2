"""MEASUREMENT AID: snappy decode time vs part count and element mix."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from parameter_server_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    plen = 65536

    def part(seed, mode):
        r = np.random.default_rng(seed)
        b = bytearray([0x80, 0x80, 0x04])
        o = 0
        if mode == "literal":
            b += bytes([61 << 2, 0xff, 0xff])  # literal of 65536, 2-byte length
            b += r.integers(0, 256, plen, dtype=np.uint8).tobytes()
            return bytes(b)
        while o < plen:
            if mode != "copies":
                b.append(15 << 2)
                b += r.integers(0, 256, 16, dtype=np.uint8).tobytes()
                o += 16
            else:
                if o == 0:
                    b.append(15 << 2)
                    b += r.integers(0, 256, 16, dtype=np.uint8).tobytes()
                    o += 16
            off = int(r.integers(1, min(o, 4096) + 1))
            b += bytes([2 | (15 << 2), off & 0xff, off >> 8])
            o += 16
        return bytes(b)

    for mode in ("mixed", "copies", "literal"):
        for nparts in (256, 512, 1024, 2048):
            parts = [part(i % 16, mode) for i in range(nparts)]
            soff = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.uint64)
            dsrc = torch.from_numpy(np.frombuffer(b"".join(parts), np.uint8).copy()).to(dev)
            dso = torch.from_numpy(soff.view(np.int64)).to(dev)
            ddo = torch.arange(0, nparts + 1, dtype=torch.int64, device=dev) * plen
            ddst = torch.empty(nparts * plen, dtype=torch.uint8, device=dev)
            dst_ = torch.empty(nparts, dtype=torch.int32, device=dev)

            def fn():
                _lib.check(L.psg_snappy_uncompress_dev(
                    dsrc.data_ptr(), dso.data_ptr(), nparts, ddst.data_ptr(), ddo.data_ptr(),
                    dst_.data_ptr(), None))
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 5
            bad = int(dst_.abs().sum().item())
            print(f"{mode:8s} nparts={nparts:5d} ms={ms:8.3f} GB/s(out)={nparts * plen / ms / 1e6:8.1f}"
                  f" bad={bad}", flush=True)


if __name__ == "__main__":
    main()
