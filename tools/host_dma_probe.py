"""Host<->device DMA rates by host-buffer kind (round 5, the host-buffer path):
hipHostMalloc'd pinned memory, a pageable numpy array registered with
qpp_host_register (hipHostRegister), the same on a 2 MiB-aligned mmap with
MADV_HUGEPAGE, and pageable memory unregistered.  1.2 GB each way, H2D and
D2H alone, then both at once on two streams.  Prints one JSON line."""
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aioquic_amd import _crypto  # noqa: E402

N = 1200 * (1 << 20)
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
vp = ctypes.c_void_p
hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
hip.hipStreamSynchronize.argtypes = [vp]
H2D, D2H = 1, 2
dev = torch.device("cuda")
d_a = torch.empty(N, dtype=torch.uint8, device=dev)
d_b = torch.empty(N, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def rate(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(N / min(ts) / (1 << 30), 2)


def legs(ha, hb, chunk=32 << 20):
    def h2d():
        for o in range(0, N, chunk):
            assert hip.hipMemcpyAsync(d_a.data_ptr() + o, ha + o, min(chunk, N - o), H2D, s1.cuda_stream) == 0

    def d2h():
        for o in range(0, N, chunk):
            assert hip.hipMemcpyAsync(hb + o, d_b.data_ptr() + o, min(chunk, N - o), D2H, s2.cuda_stream) == 0

    def both():
        h2d()
        d2h()

    return {"h2d": rate(h2d), "d2h": rate(d2h), "duplex_each_way": rate(both)}


out = {}
# hipHostMalloc
pa, pb = vp(), vp()
assert hip.hipHostMalloc(ctypes.byref(pa), N, 0) == 0 and hip.hipHostMalloc(ctypes.byref(pb), N, 0) == 0
ctypes.memset(pa, 1, N)
out["hipHostMalloc"] = legs(pa.value, pb.value)
# numpy, registered
a = np.ones(N, np.uint8)
b = np.zeros(N, np.uint8)
_crypto.host_register(a.ctypes.data, N)
_crypto.host_register(b.ctypes.data, N)
out["numpy_registered"] = legs(a.ctypes.data, b.ctypes.data)
_crypto.host_unregister(a.ctypes.data)
_crypto.host_unregister(b.ctypes.data)
out["numpy_pageable"] = legs(a.ctypes.data, b.ctypes.data)
del a, b
# 2 MiB-aligned anonymous mmap with MADV_HUGEPAGE, registered
maps = []
for _ in range(2):
    m = mmap.mmap(-1, N + (2 << 20))
    try:
        m.madvise(mmap.MADV_HUGEPAGE)
    except (AttributeError, OSError):
        pass
    arr = np.frombuffer(m, np.uint8)
    base = arr.ctypes.data
    off = (-base) % (2 << 20)
    arr = arr[off : off + N]
    arr[:] = 1
    maps.append((m, arr))
_crypto.host_register(maps[0][1].ctypes.data, N)
_crypto.host_register(maps[1][1].ctypes.data, N)
out["mmap_hugepage_registered"] = legs(maps[0][1].ctypes.data, maps[1][1].ctypes.data)
_crypto.host_unregister(maps[0][1].ctypes.data)
_crypto.host_unregister(maps[1][1].ctypes.data)
try:
    out["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
except OSError:
    out["thp"] = None
print(json.dumps(out), flush=True)
