"""The library's host-buffer path (MultiDeviceEngine on one device) with the
caller's arrays staged (pageable) or registered (the round-5 qpp_host_register
study, since removed: mode "registered" needs that build): 1 Mi
north-star packets, protect_into + unprotect_into, a few reps each, timed per
call.  For rocprofv3 runs (which copy engine / blit kernel moves the bytes)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aioquic_amd import layout as L  # noqa: E402
from aioquic_amd.batch import MultiDeviceEngine  # noqa: E402
from aioquic_amd.bench_data import make_workload  # noqa: E402

if os.environ.get("QPP_PROBE_INTERLEAVE") == "1":
    # study: every page this process touches from here on interleaved over
    # the host's NUMA nodes (set_mempolicy(MPOL_INTERLEAVE), syscall 238)
    import ctypes

    libc = ctypes.CDLL(None, use_errno=True)
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node"))
    mask = ctypes.c_ulong(sum(1 << k for k in nodes))
    rc = libc.syscall(238, 3, ctypes.byref(mask), ctypes.c_ulong(64))
    print("interleave over nodes", nodes, "rc", rc, file=sys.stderr)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["staged", "registered"]  # run in this order
w = make_workload(n, suite=0, n_keys=1, seed=0x9001, version=1)
eng = MultiDeviceEngine(w.n_keys, devices=[0])
eng.set_key_records(w.keys)
plain = np.ascontiguousarray(w.plain)
wire = np.empty(w.wire_size, np.uint8)
back = np.empty(w.plain_size, np.uint8)
r1 = np.empty(n, L.RESULT)
r2 = np.empty(n, L.RESULT)
out = {}
for mode in modes:
    if mode == "registered":
        from aioquic_amd.batch import register_host  # the removed study API
        regs = register_host(plain, wire, back, r1, r2)
    else:
        regs = []
    ts = []
    for rep in range(int(os.environ.get("QPP_PROBE_REPS", "4"))):
        t0 = time.perf_counter()
        eng.protect_into(w.desc, plain, wire, r1)
        t1 = time.perf_counter()
        eng.unprotect_into(w.udesc, wire, back, r2)
        t2 = time.perf_counter()
        ts.append((t1 - t0, t2 - t1))
    ok = bool((r1["status"] == 0).all() and (r2["status"] == 0).all() and np.array_equal(back, plain))
    for r in regs:
        r.close()
    best = min(ts, key=sum)
    med = sorted(sum(t) for t in ts)[len(ts) // 2]
    out[mode] = {"protect_ms": round(best[0] * 1e3, 2), "unprotect_ms": round(best[1] * 1e3, 2),
                 "gib_s": round(n * 1200 / sum(best) / (1 << 30), 3),
                 "median_gib_s": round(n * 1200 / med / (1 << 30), 3), "ok": ok}
print(json.dumps(out), flush=True)
