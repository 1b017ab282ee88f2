"""DIAGNOSTIC: where a snappy part's parse spends its clocks (build:
tools/ab_build.sh sprof "-DPSG_SNAPPY_PROF"; run on the GPU box with
PSG_LIB_PATH=$PWD/build/sprof/libpsg.so).  The parts are one cfg2 aggregate's
key and value parts, compressed by the e2e harness (tools/e2e)."""
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
    f = L.psg_debug_snappy_prof
    f.argtypes = [C.c_void_p, C.c_uint32]
    out = {}
    for name, n in (("all16", len(comps)), ("one_value_part", 1)):
        base = 1 if n == 1 else 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for rep in range(3):
            e0.record()
            _lib.check(L.psg_snappy_uncompress_dev(ds.data_ptr(), dso[base:].data_ptr(),
                                                   n, dd.data_ptr(), ddo[base:].data_ptr(),
                                                   st.data_ptr(), None))
            e1.record()
            torch.cuda.synchronize()
        assert int(st[:n].abs().sum()) == 0
        prof = np.zeros((n, 8), np.uint64)
        assert f(prof.ctypes.data, n) == 0
        out[name] = {"ms": e0.elapsed_time(e1),
                     "per_part": [{"refill_clk": int(r[0]), "lookup_clk": int(r[1]),
                                   "total_clk": int(r[2]), "refills": int(r[3]),
                                   "deferred": int(r[4]), "literal_clk": int(r[5]),
                                   "end_clk": int(r[7]),
                                   "elements": int(r[6]), "bytes_in": int(comps[base + i].size),
                                   # the table form's fields (psg_snappy.hip snappy_tab_kernel)
                                   "tab": {"walk_clk": int(r[0]), "move_clk": int(r[1]),
                                           "total_clk": int(r[2]), "window_loads": int(r[3]),
                                           "unresolved": int(r[4]), "inorder_clk": int(r[5]),
                                           "elements": int(r[6]), "window_load_clk": int(r[7])}}
                                  for i, r in enumerate(prof)]}
    got = dd.cpu().numpy()
    assert all(np.array_equal(got[int(doff[i]):int(doff[i + 1])], raws[i]) for i in range(len(raws)))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
