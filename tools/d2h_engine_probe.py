"""Which engine moves D2H copies, and do they overlap a persistent kernel?
A 1.2 GB D2H into pinned host memory (hipHostMalloc) by hipMemcpyAsync with
kind DeviceToHost and with kind DeviceToDeviceNoCU (copy engines only), alone
and beside 20 back-to-back k_gcm protect launches (1 Mi packets, every CU
occupied) on another stream.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aioquic_amd.batch import PacketEngine  # noqa: E402
from aioquic_amd.bench_data import make_workload  # noqa: E402

N = 1200 * (1 << 20)
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
vp = ctypes.c_void_p
hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
dev = torch.device("cuda")
n = 1 << 20
w = make_workload(n, suite=0, n_keys=1, seed=0x9001, version=1)
eng = PacketEngine(1)
eng.set_key_records(w.keys)
d_plain = torch.from_numpy(w.plain).to(dev)
d_desc = torch.from_numpy(w.desc.view(np.uint8)).to(dev)
d_wire = torch.empty(w.wire_size, dtype=torch.uint8, device=dev)
d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
src = torch.empty(N, dtype=torch.uint8, device=dev)
h = vp()
assert hip.hipHostMalloc(ctypes.byref(h), N, 0) == 0
hd = vp()
assert hip.hipHostGetDevicePointer(ctypes.byref(hd), h, 0) == 0
s_k, s_c = torch.cuda.Stream(), torch.cuda.Stream()


def copies(kind, dst, chunk=32 << 20):
    for o in range(0, N, chunk):
        rc = hip.hipMemcpyAsync(dst + o, src.data_ptr() + o, min(chunk, N - o), kind, s_c.cuda_stream)
        if rc != 0:
            return rc
    return 0


def kernels(k=20):
    for _ in range(k):
        eng.protect(d_desc, n, d_plain, d_wire, d_res, s_k)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) * 1e3, 2), r


out = {"device_ptr_equals_host_ptr": hd.value == h.value}
kernels(3)
out["kernels_alone_ms"] = timed(kernels)[0]
for name, kind, dst in (("d2h", 2, h.value), ("nocu", 1024, hd.value)):
    t, rc = timed(lambda: copies(kind, dst))
    out[name + "_alone_ms"] = t
    out[name + "_rc"] = rc
    if rc == 0:
        out[name + "_beside_kernels_ms"] = timed(lambda: (kernels(), copies(kind, dst))[1])[0]
print(json.dumps(out), flush=True)
