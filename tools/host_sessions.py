"""The library's host-buffer path split over K sessions (qpp_multi), all on
device 0 when the box has one GPU: the multi-device code path (one session,
key-table replica and host thread per range) at the session counts an
8-GPU node would use, round trip checked.

    python tools/host_sessions.py [packets] [counts...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aioquic_amd import layout as L  # noqa: E402
from aioquic_amd.batch import MultiDeviceEngine  # noqa: E402
from aioquic_amd.bench_data import make_workload  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
counts = [int(x) for x in sys.argv[2:]] or [2, 4, 8]
w = make_workload(n, suite=0, n_keys=1, seed=0x9001, version=1)
plain = np.ascontiguousarray(w.plain)
wire = np.empty(w.wire_size, np.uint8)
back = np.empty(w.plain_size, np.uint8)
r1 = np.empty(n, L.RESULT)
r2 = np.empty(n, L.RESULT)
for k in counts:
    eng = MultiDeviceEngine(w.n_keys, devices=[0] * k)
    eng.set_key_records(w.keys)
    rts = []
    for rep in range(4):
        back[:1] ^= 1
        t0 = time.perf_counter()
        eng.protect_into(w.desc, plain, wire, r1)
        eng.unprotect_into(w.udesc, wire, back, r2)
        rts.append(n * 1200 / (time.perf_counter() - t0) / (1 << 30))
    ok = bool((r1["status"] == 0).all() and (r2["status"] == 0).all() and np.array_equal(back, plain))
    print(json.dumps({"sessions": k, "round_trip_gib_s": [round(x, 2) for x in rts], "ok": ok}), flush=True)
    del eng
    if not ok:
        sys.exit(1)
