"""Per-kernel VGPR / spill / LDS report of qpp_engine.hip for gfx950 (compile only)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "aioquic_amd/csrc/qpp_engine.hip"
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", "include",
                      "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: +(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|SGPRs): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    name = re.sub(r"PK.*", "", k.replace("_ZN3qpp", ""))
    print(f"{name:40s} vgpr {v.get('VGPRs')} agpr {v.get('AGPRs')} scratch {v.get('ScratchSize')} occ {v.get('Occupancy')} lds {v.get('LDS')}")
