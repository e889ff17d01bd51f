"""Host-buffer rate of the product's session path (qpp_session_protect /
_unprotect through PacketEngine.protect_host / unprotect_host): caller bytes ->
pinned staging -> H2D -> kernel -> D2H -> new bytes, pipelined (default) vs
serial (QPP_SESSION_SERIAL=1).  Prints one JSON line per mode.

    python tools/session_bench.py [--packets 1048576] [--reps 3]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from aioquic_amd.batch import PacketEngine
    from aioquic_amd.bench_data import make_workload

    w = make_workload(a.packets, suite=0, n_keys=1, seed=0x9003)
    eng = PacketEngine(w.n_keys)
    eng.set_key_records(w.keys)
    plain = w.plain.tobytes()
    for mode in ("pipelined", "serial"):
        if mode == "serial":
            os.environ["QPP_SESSION_SERIAL"] = "1"
        tp, tu = [], []
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            wire, r1 = eng.protect_host(w.desc, plain, w.wire_size)
            t1 = time.perf_counter()
            wb = wire.tobytes()
            t2 = time.perf_counter()
            back, r2 = eng.unprotect_host(w.udesc, wb, w.plain_size)
            t3 = time.perf_counter()
            tp.append(t1 - t0)
            tu.append(t3 - t2)
        ok = bool((r1["status"] == 0).all() and (r2["status"] == 0).all()
                  and np.array_equal(back, w.plain))
        tp, tu = float(np.median(tp[1:])), float(np.median(tu[1:]))
        b = a.packets * 1200
        print(json.dumps({"mode": mode, "packets": a.packets, "protect_gib_s": round(b / tp / GIB, 3),
                          "unprotect_gib_s": round(b / tu / GIB, 3),
                          "round_trip_gib_s": round(b / (tp + tu) / GIB, 3), "round_trip_ok": ok}),
              flush=True)
    os.environ.pop("QPP_SESSION_SERIAL", None)
    # caller-owned buffers reused across calls (protect_into / unprotect_into)
    from aioquic_amd import layout as L

    wire = np.empty(w.wire_size, np.uint8)
    back = np.empty(w.plain_size, np.uint8)
    r1 = np.zeros(a.packets, dtype=L.RESULT)
    r2 = np.zeros(a.packets, dtype=L.RESULT)
    tp, tu = [], []
    for _ in range(a.reps + 1):
        t0 = time.perf_counter()
        eng.protect_into(w.desc, w.plain, wire, r1)
        t1 = time.perf_counter()
        eng.unprotect_into(w.udesc, wire, back, r2)
        t2 = time.perf_counter()
        tp.append(t1 - t0)
        tu.append(t2 - t1)
    ok = bool((r1["status"] == 0).all() and (r2["status"] == 0).all()
              and np.array_equal(back, w.plain))
    tp, tu = float(np.median(tp[1:])), float(np.median(tu[1:]))
    b = a.packets * 1200
    print(json.dumps({"mode": "pipelined, reused buffers (protect_into)", "packets": a.packets,
                      "protect_gib_s": round(b / tp / GIB, 3), "unprotect_gib_s": round(b / tu / GIB, 3),
                      "round_trip_gib_s": round(b / (tp + tu) / GIB, 3), "round_trip_ok": ok}),
          flush=True)


if __name__ == "__main__":
    main()
