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
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def main(d):
    stats = os.path.join(d, "kt", "kt_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    print(f"# rocprofv3 summary: `{os.path.basename(d.rstrip('/'))}`\n")
    print("## Kernel trace (`rocprofv3 --kernel-trace --stats`)\n")
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
    main(sys.argv[1])
