#!/usr/bin/env python3
"""Per-kernel resource usage of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage)."""
import re, subprocess, sys
src = sys.argv[1] if len(sys.argv) > 1 else "aioquic_amd/csrc/qpp_engine.hip"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_"
extra = sys.argv[3:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude",
       "-Iaioquic_amd/csrc", "--cuda-device-only", "-c", src, "-o", "/tmp/regs.o",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None; rows = {}
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m: continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip(); rows[cur] = {}
    elif cur: rows[cur][k.split(" [")[0]] = v
for name, r in rows.items():
    if pat in name:
        short = re.sub(r"\(.*", "", name).replace("qpp::", "")
        print(f"{short:40s} V{r.get('VGPRs','-'):>4} A{r.get('AGPRs','0'):>3} S{r.get('SGPRs','-'):>4} "
              f"Vsp{r.get('VGPRs Spill','-'):>4} Ssp{r.get('SGPRs Spill','-'):>4} scr{r.get('ScratchSize','-'):>4} "
              f"LDS{r.get('LDS Size','-'):>7} occ{r.get('Occupancy','-')}")
if not rows: print(out[-3000:])
