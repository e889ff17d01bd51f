#!/usr/bin/env python3
"""Build an A/B variant of libquicpp.so with extra compile flags into
variants/<name>/libquicpp.so (the in-tree library is left alone):

    python tools/build_variant.py NAME -DQPP_SWITCH=0 ...

tools/gpu_ab2.sh runs the bench against such builds via LD_LIBRARY_PATH."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(ROOT, "variants", name)
os.makedirs(out, exist_ok=True)
obj = os.path.join(out, "qpp_engine.o")
hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include"),
                "-c", "-o", obj] + flags + [os.path.join(ROOT, "aioquic_amd", "csrc", "qpp_engine.hip")], check=True)
subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libquicpp.so"), obj,
                os.path.join(ROOT, "build", "obj", "qpp_plan.o")], check=True)
os.remove(obj)
print(os.path.join(out, "libquicpp.so"))
