"""MEASUREMENT AID: device time of psg_snappy_uncompress_dev on one cfg2
aggregate's 16 key/value parts (compressed by the e2e harness, tools/e2e),
and on its first value part alone; bit-exact against the raw bytes."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from parameter_server_amd import _lib, synth
    L = _lib.lib()
    E = C.CDLL(os.path.join(ROOT, "tools", "e2e", "libe2e.so"))
    E.psg_e2e_compress.restype = C.c_size_t
    D, pushes = synth.shard_instance(seed=1, lo=0, hi=(1 << 64) - 1)
    raws, comps = [], []
    for k, vs in pushes:
        for raw in (np.ascontiguousarray(k).view(np.uint8), np.ascontiguousarray(vs[0]).view(np.uint8)):
            buf = np.empty(32 + raw.size + raw.size // 6, np.uint8)
            nb = E.psg_e2e_compress(C.c_void_p(raw.ctypes.data), C.c_size_t(raw.size),
                                    C.c_void_p(buf.ctypes.data))
            raws.append(raw)
            comps.append(buf[:nb].copy())
    soff = np.concatenate([[0], np.cumsum([c.size for c in comps])]).astype(np.uint64)
    doff = np.concatenate([[0], np.cumsum([r.size for r in raws])]).astype(np.uint64)
    dev = "cuda:0"
    ds = torch.from_numpy(np.concatenate(comps)).to(dev)
    dso = torch.from_numpy(soff.view(np.int64)).to(dev)
    ddo = torch.from_numpy(doff.view(np.int64)).to(dev)
    dd = torch.empty(int(doff[-1]), dtype=torch.uint8, device=dev)
    st = torch.zeros(len(comps), dtype=torch.int32, device=dev)
    out = {}
    for name, n, base in (("all16", len(comps), 0), ("one_value_part", 1, 1), ("one_key_part", 1, 0)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for rep in range(5):
            e0.record()
            _lib.check(L.psg_snappy_uncompress_dev(ds.data_ptr(), dso[base:].data_ptr(), n,
                                                   dd.data_ptr(), ddo[base:].data_ptr(),
                                                   st.data_ptr(), None))
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        assert int(st[:n].abs().sum()) == 0
        got = dd.cpu().numpy()
        for i in range(base, base + n):
            assert np.array_equal(got[int(doff[i]):int(doff[i + 1])], raws[i]), i
        out[name] = round(float(np.median(ts[1:])), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
