"""GPU box: HBM copy rate of the tools/copybw kernel forms and torch copy_
(1 GiB -> 1 GiB, read + write bytes / time)."""
import ctypes
import torch
L = ctypes.CDLL("tools/copybw/libcopybw.so")
fn = L.copybw_copy_mode
fn.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
nb = 1 << 30
a = torch.empty(nb // 4, device="cuda")
b = torch.empty_like(a)
s = torch.cuda.current_stream()
names = ["grid-stride", "flat", "flat+nt", "grid-stride+nt", "torch copy_"]
for mode in range(5):
    run = (lambda: b.copy_(a)) if mode == 4 else (lambda: fn(b.data_ptr(), a.data_ptr(), nb, mode, s.cuda_stream))
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record(s)
    for _ in range(10):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    print(f"{names[mode]:16s} {2 * nb * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9:8.0f} GB/s")
