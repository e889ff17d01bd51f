"""HBM traffic per launch of the packet kernels from rocprofv3 --pmc passes.

    python tools/traffic.py WORKLOAD_NAME FETCH_DIR WRITE_DIR [--out profiles/traffic.json]

FETCH_SIZE / WRITE_SIZE are in KiB.  Corrections come from tools/calib_hbm.hip
run on the same pool (profiles/r1_calibration.md): for the engine's pattern
(4 lanes x 16 B contiguous per packet, LDS-DMA loads, 16 B stores, packet slots
1200 B apart) FETCH_SIZE reads 0.597 of the bytes moved (x1.675), WRITE_SIZE
1.035 (x0.966).  The guide's generic x2 read correction is for full 1 KiB-per-
wave streams and overshoots this pattern.
"""

import csv
import glob
import json
import os
import sys

FETCH_CORR = 1241513984 / (723791 * 1024)   # ld_pat<false>: pattern bytes / FETCH_SIZE bytes
WRITE_CORR = 1241513984 / (1254335 * 1024)  # st_pat<false>


def per_launch(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "k_packets" not in r["Kernel_Name"]:
                continue
            enc = "true" in r["Kernel_Name"].split("(")[0]
            out.setdefault("protect" if enc else "unprotect", []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) * 1024 for k, v in out.items()}


def main():
    name, fdir, wdir = sys.argv[1:4]
    dst = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "profiles/traffic.json"
    fetch, write = per_launch(fdir, "FETCH_SIZE"), per_launch(wdir, "WRITE_SIZE")
    data = json.load(open(dst)) if os.path.exists(dst) else {}
    entry = {}
    for k in ("protect", "unprotect"):
        if k in fetch and k in write:
            rb, wb = fetch[k] * FETCH_CORR, write[k] * WRITE_CORR
            entry[k] = {"read_bytes": round(rb), "write_bytes": round(wb), "bytes": round(rb + wb),
                        "fetch_size_kib_raw": round(fetch[k] / 1024), "write_size_kib_raw": round(write[k] / 1024)}
    entry["packets"] = int(sys.argv[sys.argv.index("--packets") + 1]) if "--packets" in sys.argv else 65536
    entry["source"] = (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes ({fdir}, {wdir}); "
                       f"corrections x{FETCH_CORR:.3f} / x{WRITE_CORR:.3f} from tools/calib_hbm.hip")
    data[name] = entry
    json.dump(data, open(dst, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
