"""Flags of a full-CU-mask stream (how the library makes its shared FAST side
stream, runtime.cpp shared_side_stream): hipExtStreamCreateWithCUMask takes no
flags argument; hipStreamGetFlags says whether HIP made it blocking (0) or
non-blocking (1).  Also times a null-stream kernel issued while the masked
stream runs a long kernel (INTEGRATION.md "Streams")."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
torch.zeros(1, device="cuda")
s = ctypes.c_void_p()
n = torch.cuda.get_device_properties(0).multi_processor_count
words = (n + 31) // 32
mask = (ctypes.c_uint32 * words)(*[0xFFFFFFFF] * words)
assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, mask) == 0
f = ctypes.c_uint(7)
assert hip.hipStreamGetFlags(s, ctypes.byref(f)) == 0
print(f"cu-mask stream flags = {f.value} ({'non-blocking' if f.value & 1 else 'blocking'})")
ext = torch.cuda.ExternalStream(s.value)
a = torch.randn(8192, 8192, device="cuda")
torch.cuda.synchronize()
for trial in range(3):
    with torch.cuda.stream(ext):
        for _ in range(20):
            a = a @ a.T / 8192.0  # ~tens of ms on the masked stream
    t0 = time.perf_counter()
    torch.zeros(1, device="cuda").add_(1)  # default (null) stream
    torch.cuda.default_stream().synchronize()
    t_null = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"trial {trial}: null-stream op done after {t_null*1e3:.2f} ms; masked stream done after {t_all*1e3:.2f} ms")
