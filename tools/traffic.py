"""HBM traffic per launch of the packet kernels from rocprofv3 --pmc passes.

    python tools/traffic.py WORKLOAD_NAME FETCH_DIR WRITE_DIR [--packets N] [--out profiles/traffic.json]

FETCH_SIZE / WRITE_SIZE are in KiB.  One calibration throughout, the one
MI355X_MICROARCH.md (HBM section) prescribes for gfx950: FETCH_SIZE reports
half the bytes of 16 B/lane streaming reads (x2), WRITE_SIZE reads the bytes
of 16 B/lane stores exactly (x1).  (Round 1's own pattern calibration,
tools/calib_hbm.hip, put the read factor at x1.675 for this access shape; the
guide's factor is used so that every number in profiles/ shares one basis.)
"""

import csv
import glob
import json
import os
import sys

FETCH_CORR = 2.0
WRITE_CORR = 1.0
KERNELS = ("k_gcm", "k_chacha", "k_packets")


def per_launch(d, counter):
    """Bytes per protect / unprotect call: each packet kernel's mean over its
    dispatches, summed over the kernels one call launches (a mixed-suite call
    runs k_gcm and k_chacha)."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or not any(k in r["Kernel_Name"] for k in KERNELS):
                continue
            kname = r["Kernel_Name"].split("(")[0]
            enc = "true" in kname
            out.setdefault("protect" if enc else "unprotect", {}).setdefault(kname, []).append(
                float(r["Counter_Value"]))
    return {k: sum(sum(v) / len(v) for v in ks.values()) * 1024 for k, ks in out.items()}


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
                       f"corrections x{FETCH_CORR:g} / x{WRITE_CORR:g} (MI355X_MICROARCH.md, HBM)")
    data[name] = entry
    json.dump(data, open(dst, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
