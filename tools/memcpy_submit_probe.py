"""Host time to SUBMIT one 39 MB hipMemcpyAsync (no synchronisation), H2D
and D2H, from hipHostMalloc'd memory and from hipHostRegister'ed memory
(flags 1 / 0 / 8), and the time until completion: is the registered-memory
copy asynchronous for the submitting thread?  Prints one JSON line."""
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np

import torch

N = 39 << 20
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
vp = ctypes.c_void_p
hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostRegister.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [vp]
dev = torch.device("cuda")
d = torch.empty(N, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream()


def measure(host):
    res = {}
    for name, kind in (("h2d", 1), ("d2h", 2)):
        sub, tot = [], []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if kind == 1:
                rc = hip.hipMemcpyAsync(d.data_ptr(), host, N, 1, s.cuda_stream)
            else:
                rc = hip.hipMemcpyAsync(host, d.data_ptr(), N, 2, s.cuda_stream)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            assert rc == 0, rc
            sub.append((t1 - t0) * 1e3)
            tot.append((t2 - t0) * 1e3)
        res[name] = {"submit_ms": round(min(sub), 3), "total_ms": round(min(tot), 3)}
    return res


out = {}
h = vp()
assert hip.hipHostMalloc(ctypes.byref(h), N, 0) == 0
ctypes.memset(h, 1, N)
out["hipHostMalloc"] = measure(h.value)
for f in (1, 0, 8):
    m = mmap.mmap(-1, N + 4096)
    a = np.frombuffer(m, np.uint8)
    a[:] = 1
    base = a.ctypes.data + ((-a.ctypes.data) % 4096)
    assert hip.hipHostRegister(base, N, f) == 0
    out[f"registered_{f}"] = measure(base)
    hip.hipHostUnregister(base)
a = np.ones(N, np.uint8)
out["pageable"] = measure(a.ctypes.data)
print(json.dumps(out), flush=True)
