"""The library's host-buffer path with its per-call phase trace
(qpp_multi_trace): 1 Mi north-star packets, protect_into + unprotect_into
from / into caller-owned pageable arrays, REPS round trips, one line per call:
wall, host copies in / out, the GPU engines' busy sums and the GPU span.

    python tools/host_trace.py [packets] [reps]"""
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
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
w = make_workload(n, suite=0, n_keys=1, seed=0x9001, version=1)
eng = MultiDeviceEngine(w.n_keys, devices=[0])
eng.set_key_records(w.keys)
plain = np.ascontiguousarray(w.plain)
wire = np.empty(w.wire_size, np.uint8)
back = np.empty(w.plain_size, np.uint8)
r1 = np.empty(n, L.RESULT)
r2 = np.empty(n, L.RESULT)
eng.protect_into(w.desc, plain, wire, r1)
eng.unprotect_into(w.udesc, wire, back, r2)
eng.trace(True)
rts = []
for rep in range(reps):
    t0 = time.perf_counter()
    eng.protect_into(w.desc, plain, wire, r1)
    (tp,) = eng.trace()
    eng.unprotect_into(w.udesc, wire, back, r2)
    (tu,) = eng.trace()
    dt = time.perf_counter() - t0
    rts.append(n * 1200 / dt / (1 << 30))
    for name, t in (("protect", tp), ("unprotect", tu)):
        gbs = lambda b, ms: b / ms / 1e6 if ms else 0.0  # noqa: E731
        print(f"{rep} {name:9s} total {t['total_ms']:6.1f} submit {t['submit_ms']:6.1f} wait {t['wait_ms']:5.1f} "
              f"copy_in {t['copy_in_ms']:5.1f} copy_out(sum) {t['copy_out_ms']:5.1f} | h2d {t['h2d_ms']:5.1f} "
              f"({gbs(t['in_bytes'], t['h2d_ms']):4.1f} GB/s) kern {t['kernel_ms']:4.1f} d2h {t['d2h_ms']:5.1f} "
              f"({gbs(t['out_bytes'], t['d2h_ms']):4.1f} GB/s) span {t['gpu_span_ms']:5.1f}", flush=True)
ok = bool((r1["status"] == 0).all() and (r2["status"] == 0).all() and np.array_equal(back, plain))
print(json.dumps({"threads": os.environ.get("QPP_COPY_THREADS", "6"), "round_trip_gib_s": [round(x, 2) for x in rts],
                  "median": round(sorted(rts)[len(rts) // 2], 2), "ok": ok}), flush=True)
