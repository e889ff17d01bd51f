#!/usr/bin/env python3
"""Build an A/B variant of libquicpp.so with extra compile flags, or from
another version of qpp_engine.hip, into variants/<name>/libquicpp.so (the
in-tree library is left alone):

    python tools/build_variant.py NAME [--src FILE | --rev GITREV] -DQPP_SWITCH=0 ...

The variant links the in-tree source-hash object, so the in-tree _crypto
extension accepts it (a deliberate A/B, not a stale build).
tools/ab_lib.sh runs the bench against such builds via LD_LIBRARY_PATH."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = sys.argv[1:]
name = args.pop(0)
src = os.path.join(ROOT, "aioquic_amd", "csrc", "qpp_engine.hip")
if args and args[0] in ("--src", "--rev"):
    kind, val = args.pop(0), args.pop(0)
    if kind == "--src":
        src = os.path.abspath(val)
    else:
        # the engine of another revision, compiled beside today's headers
        src = os.path.join(ROOT, "aioquic_amd", "csrc", f".variant_{name}.hip")
        with open(src, "w") as f:
            f.write(subprocess.run(["git", "show", f"{val}:aioquic_amd/csrc/qpp_engine.hip"], cwd=ROOT,
                                   check=True, capture_output=True, text=True).stdout)
flags = args
out = os.path.join(ROOT, "variants", name)
os.makedirs(out, exist_ok=True)
obj = os.path.join(out, "qpp_engine.o")
hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
try:
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "aioquic_amd", "csrc"), "-c", "-o", obj] + flags + [src], check=True)
finally:
    if os.path.basename(src).startswith(".variant_"):
        os.remove(src)
objs = [obj, os.path.join(ROOT, "build", "obj", "qpp_plan.o"), os.path.join(ROOT, "build", "obj", "qpp_source_hash.o")]
subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libquicpp.so")] + objs,
               check=True)
os.remove(obj)
print(os.path.join(out, "libquicpp.so"))
