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
hip.hipHostRegister.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [vp]


def anon(huge):
    """An N-byte 2 MiB-aligned anonymous mapping (MADV_HUGEPAGE when huge)."""
    m = mmap.mmap(-1, N + (2 << 20))
    if huge:
        try:
            m.madvise(mmap.MADV_HUGEPAGE)
        except (AttributeError, OSError):
            pass
    arr = np.frombuffer(m, np.uint8)
    off = (-arr.ctypes.data) % (2 << 20)
    arr = arr[off : off + N]
    arr[:] = 1
    return m, arr


# one hipHostRegister per buffer (the copies stay inside it), by flags
for name, huge, flags in (("registered_default", False, 0), ("registered_coarse", False, 0x8),
                          ("registered_portable", False, 0x1), ("hugepage_registered_coarse", True, 0x8),
                          ("hugepage_registered_default", True, 0)):
    bufs = [anon(huge), anon(huge)]
    ok = all(hip.hipHostRegister(b[1].ctypes.data, N, flags) == 0 for b in bufs)
    out[name] = legs(bufs[0][1].ctypes.data, bufs[1][1].ctypes.data) if ok else "register failed"
    for b in bufs:
        hip.hipHostUnregister(b[1].ctypes.data)
    del bufs
# pageable (unregistered) numpy memory
a = np.ones(N, np.uint8)
b = np.zeros(N, np.uint8)
out["numpy_pageable"] = legs(a.ctypes.data, b.ctypes.data)
del a, b
try:
    out["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
except OSError:
    out["thp"] = None
print(json.dumps(out), flush=True)
