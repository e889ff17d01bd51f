"""Summarise a tools/profile.sh output directory into a markdown table.

    python tools/prof_summary.py gpurun_out/prof_TAG > profiles/TAG_summary.md

Per kernel: launches, average duration (rocprofv3 --kernel-trace --stats),
and the per-launch mean of every PMC counter collected in the separate
--pmc passes.  FETCH_SIZE / WRITE_SIZE are in KiB as rocprofv3 reports them;
the corrected HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE
of a 16 B/lane streaming read reads half the bytes on gfx950, WRITE_SIZE is
exact for 16 B/lane stores.  Both corrections are stated next to the numbers.
"""

import collections
import csv
import glob
import json
import os
import sys

BYTES_PER_PKT_KERNEL = 2440  # bench.py: algorithmic HBM bytes per packet per launch
HBM_PEAK_GBS = 8000.0


def short(name):
    return name.split("(")[0].replace("void ", "")


def bench_line(d):
    """The bench's JSON line from the kernel-trace pass's log."""
    try:
        for line in open(os.path.join(d, "kt.log")):
            if line.startswith("{") and '"metric"' in line:
                return json.loads(line)
    except OSError:
        pass
    return None


def timed_launches(d, out_csv=None):
    """Per kernel, the dispatches of the bench's K timed steps only (the
    first W steps are warm-up at a lower clock, and an N = 1 line's
    `sustained` steps follow the timed ones): each step launches every
    kernel the same number of times, so the timed ones are dispatches
    W x per .. (W + K) x per of each kernel in dispatch order."""
    b = bench_line(d)
    traces = glob.glob(os.path.join(d, "kt", "*kernel_trace.csv"))
    if not b or not traces:
        return None, b
    rows = list(csv.DictReader(open(traces[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in rows:
        by[short(r["Kernel_Name"])].append(r)
    steps, warm = int(b["steps"]), int(b["warmup"])
    extra = int((b.get("sustained") or {}).get("steps", 0))
    total = steps + warm + extra
    keep = {}
    for k, rs in by.items():
        if len(rs) % total:
            continue  # not a per-step kernel (setup, copies, the HBM copy probe)
        per = len(rs) // total
        keep[k] = rs[warm * per:(warm + steps) * per]
    if out_csv:
        kept = sorted((r for rs in keep.values() for r in rs), key=lambda r: int(r["Start_Timestamp"]))
        with open(out_csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(kept)
    return keep, b


def main(d, timed_csv=None):
    keep, b = timed_launches(d, timed_csv)
    if keep:
        n = int(b["config"]["packets_per_gpu"])
        print(f"# rocprofv3 summary: `{os.path.basename(d.rstrip('/'))}`\n")
        print(f"## Timed launches only ({b['steps']} timed steps after {b['warmup']} warm-up steps; "
              f"`{b['config']['workload']}`)\n")
        print("| kernel | timed calls | avg us | min us | max us | algorithmic GB/s | frac of 8 TB/s |")
        print("|---|---:|---:|---:|---:|---:|---:|")
        for k, rs in sorted(keep.items(), key=lambda kv: -sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                                                               for r in kv[1])):
            ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs]
            avg = sum(ds) / len(ds)
            gbs = BYTES_PER_PKT_KERNEL * n / (avg * 1e-6) / 1e9 if ("k_gcm" in k or "k_chacha" in k) else None
            extra = f"{gbs:.1f} | {gbs / HBM_PEAK_GBS:.4f}" if gbs else "- | -"
            print(f"| `{k}` | {len(ds)} | {avg:.2f} | {min(ds):.2f} | {max(ds):.2f} | {extra} |")
        print(f"\nThe bench line of this run: value {b['value']} {b['unit']}, kernels_ms {b['kernels_ms']}, "
              f"roofline.frac {b['roofline']['frac']}.\n")
    stats = os.path.join(d, "kt", "kt_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    if not keep:
        print(f"# rocprofv3 summary: `{os.path.basename(d.rstrip('/'))}`\n")
    print("## Kernel trace, every launch (`rocprofv3 --kernel-trace --stats`)\n")
    print("| kernel | calls | avg us | min us | max us | % time |")
    print("|---|---:|---:|---:|---:|---:|")
    for r in rows:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
              f"{float(r['MinNs'])/1e3:.2f} | {float(r['MaxNs'])/1e3:.2f} | {float(r['Percentage']):.1f} |")
    pmc = collections.defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            pmc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
            meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"],
                       r["Accum_VGPR_Count"], r["SGPR_Count"], r["Scratch_Size"])
    kern = sorted({k for k, _ in pmc if any(s in k for s in ("k_packets", "k_gcm", "k_chacha", "k_hp_mask"))})
    if not kern:
        return
    print("\n## Launch resources\n")
    print("| kernel | grid | WG | LDS B | VGPR | AGPR | SGPR | scratch |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for k in kern:
        print(f"| `{k}` | " + " | ".join(meta[k]) + " |")
    names = sorted({c for _, c in pmc})
    print("\n## PMC counters, mean per launch (separate `--pmc` passes)\n")
    print("| kernel | " + " | ".join(names) + " |")
    print("|---|" + "---:|" * len(names))
    for k in kern:
        vals = []
        for c in names:
            v = pmc.get((k, c))
            vals.append(f"{sum(v)/len(v):.4g}" if v else "-")
        print(f"| `{k}` | " + " | ".join(vals) + " |")
    print("\n## HBM traffic per launch\n")
    print("| kernel | FETCH_SIZE KiB (raw) | x2 gfx950 read correction, MB | WRITE_SIZE MB |")
    print("|---|---:|---:|---:|")
    for k in kern:
        f = pmc.get((k, "FETCH_SIZE"))
        w = pmc.get((k, "WRITE_SIZE"))
        fm = sum(f) / len(f) if f else float("nan")
        wm = sum(w) / len(w) if w else float("nan")
        print(f"| `{k}` | {fm:.0f} | {2 * fm * 1024 / 1e6:.1f} | {wm * 1024 / 1e6:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
