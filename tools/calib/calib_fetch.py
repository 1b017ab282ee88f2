"""Run the FETCH_SIZE calibration reads (calib_fetch.hip) under rocprofv3:
512 MiB per dispatch (> the 256 MiB Infinity Cache), widths 4/8/16 B, each
twice.  tools/calib/run.sh collects the counters."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libcalib.so"))
lib.calib_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_void_p]
NB = 512 << 20
bufs = [torch.ones(NB // 4, dtype=torch.int32, device="cuda") for _ in range(2)]
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for w in (4, 8, 16):
    for b in bufs:
        assert lib.calib_read(b.data_ptr(), NB, w, sink.data_ptr(), s) == 0
torch.cuda.synchronize()
print("calib bytes per dispatch", NB)
