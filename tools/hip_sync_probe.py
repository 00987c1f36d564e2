"""Which HIP runtime calls of the search path block the host on this stack:
each call is timed on the host while ~100 ms of matrix products are queued
on the same stream (a blocking call takes about that long)."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p
st = vp(torch.cuda.current_stream().cuda_stream)
a = torch.randn(8192, 8192, device="cuda")
torch.mm(a, a)
torch.cuda.synchronize()


def busy():
    for _ in range(8):
        torch.mm(a, a)


def timed(name, fn):
    busy()
    t = time.perf_counter()
    fn()
    dt = time.perf_counter() - t
    pending = not torch.cuda.current_stream().query()
    torch.cuda.synchronize()
    print(f"{name:40s} {dt * 1e3:9.3f} ms  queue still busy after: {pending}", flush=True)


buf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
buf2 = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
pinned = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(pinned), ctypes.c_size_t(64), 0) == 0
p = vp()
timed("hipMallocAsync 64 MB (cold)", lambda: hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(64 << 20), st))
timed("hipFreeAsync", lambda: hip.hipFreeAsync(p, st))
timed("hipMallocAsync 64 MB (pooled)", lambda: hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(64 << 20), st))
timed("hipFreeAsync", lambda: hip.hipFreeAsync(p, st))
timed("hipMemsetAsync 1 MB", lambda: hip.hipMemsetAsync(vp(buf.data_ptr()), 0, ctypes.c_size_t(1 << 20), st))
timed("hipMemcpyAsync D2D 6 MB", lambda: hip.hipMemcpyAsync(vp(buf2.data_ptr()), vp(buf.data_ptr()), ctypes.c_size_t(6 << 20), 3, st))
timed("hipMemcpy2DAsync D2D 1024 x 6 KB", lambda: hip.hipMemcpy2DAsync(
    vp(buf2.data_ptr()), ctypes.c_size_t(6144), vp(buf.data_ptr()), ctypes.c_size_t(6144),
    ctypes.c_size_t(6144), ctypes.c_size_t(1024), 3, st))
timed("hipMemcpyAsync D2H 16 B pinned", lambda: hip.hipMemcpyAsync(pinned, vp(buf.data_ptr()), ctypes.c_size_t(16), 2, st))
ev = vp()
timed("hipEventCreate", lambda: hip.hipEventCreate(ctypes.byref(ev)))
timed("hipEventRecord", lambda: hip.hipEventRecord(ev, st))
timed("hipEventQuery", lambda: hip.hipEventQuery(ev))
timed("torch small kernel", lambda: buf.zero_())
timed("torch small kernel (again)", lambda: buf.zero_())
timed("torch small kernel (third)", lambda: buf.zero_())


def many():
    for _ in range(50):
        buf.zero_()


timed("50 torch small kernels", many)
