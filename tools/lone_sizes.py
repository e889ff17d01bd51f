#!/usr/bin/env python3
"""Crossover sweep between the lone-packet kernels (one wave per packet) and
the quad kernels: device-resident protect + unprotect of n x 1200-byte
packets, one key, timed with HIP events (median of 20 after 5 warm-ups).
Run once with QPP_LONE_MAX=<large> and once with QPP_LONE=0; prints one JSON
line per (suite, n)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from aioquic_amd import bench_data
    from aioquic_amd.batch import PacketEngine

    mode = ("quad" if os.environ.get("QPP_LONE") == "0" else
            "lone(max %s)" % os.environ["QPP_LONE_MAX"] if "QPP_LONE_MAX" in os.environ else "default thresholds")
    dev = torch.device("cuda")
    sizes = [int(x) for x in os.environ.get("LONE_SIZES", "1,4,16,64,256,1024,4096").split(",")]
    for suite in [int(x) for x in os.environ.get("LONE_SUITES", "0,2").split(",")]:
        for n in sizes:
            w = bench_data.make_workload(n, suite=suite, n_keys=1, seed=0x51 + n)
            eng = PacketEngine(1)
            eng.set_key_records(w.keys)
            d_in = torch.from_numpy(w.plain).to(dev)
            d_desc = torch.from_numpy(w.desc.view(np.uint8)).to(dev)
            d_udesc = torch.from_numpy(w.udesc.view(np.uint8)).to(dev)
            d_wire = torch.empty(w.wire_size, dtype=torch.uint8, device=dev)
            d_back = torch.zeros(w.plain_size, dtype=torch.uint8, device=dev)
            d_res = torch.empty(n * 16, dtype=torch.uint8, device=dev)
            s = torch.cuda.current_stream()
            ts = []
            for it in range(25):
                a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                a.record(s)
                eng.protect(d_desc, n, d_in, d_wire, d_res)
                b.record(s)
                eng.unprotect(d_udesc, n, d_wire, d_back, d_res)
                c.record(s)
                torch.cuda.synchronize()
                if it >= 5:
                    ts.append((a.elapsed_time(b) * 1e3, b.elapsed_time(c) * 1e3))
            ok = bool(torch.equal(d_back.cpu(), torch.from_numpy(w.plain)))
            p = float(np.median([t[0] for t in ts]))
            u = float(np.median([t[1] for t in ts]))
            print(json.dumps({"mode": mode, "suite": suite, "n": n, "protect_us": round(p, 2),
                              "unprotect_us": round(u, 2), "round_trip_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
