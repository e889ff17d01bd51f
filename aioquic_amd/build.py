"""In-tree build of the native parts (no setuptools, no JIT cache):

  aioquic_amd/libquicpp.so        HIP kernels + C ABI (include/quic_pp.h), gfx950 only
  aioquic_amd/_crypto.abi3.so     CPython binding of the C ABI, limited API 3.10 like the
                                  reference's extension (setup.py:30-39); links
                                  libquicpp.so via $ORIGIN

Each HIP translation unit compiles to its own object under build/ (the
rocPRIM radix sort of qpp_plan.hip is slow to compile and rarely changes).
The built files are git-ignored but travel to the GPU box with the repo snapshot.
"""

import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(PKG, "libquicpp.so")
EXT = os.path.join(PKG, "_crypto.abi3.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

COMMON_DEPS = ["qpp_device.h", "qpp_internal.h"]
# translation unit -> headers it depends on (besides COMMON_DEPS and quic_pp.h)
HIP_UNITS = {
    "qpp_engine.hip": ["qpp_chacha.h", "qpp_hkdf.h", "qpp_sha_consts.h"],
    "qpp_plan.hip": [],
}


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _obj(unit):
    return os.path.join(OBJ, unit.replace(".hip", ".o"))


def build_lib(force=False, extra=()):
    os.makedirs(OBJ, exist_ok=True)
    hdr = os.path.join(INCLUDE, "quic_pp.h")
    objs = []
    for unit, deps in HIP_UNITS.items():
        src = os.path.join(CSRC, unit)
        obj = _obj(unit)
        objs.append(obj)
        dl = [src, hdr] + [os.path.join(CSRC, d) for d in COMMON_DEPS + deps]
        if force or extra or _stale(obj, dl):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                   "-I", INCLUDE, "-c", "-o", obj + ".tmp"] + list(extra) + [src]
            _run(cmd)
            os.replace(obj + ".tmp", obj)
    if force or extra or _stale(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp"] + objs)
        os.replace(LIB + ".tmp", LIB)
    return LIB


def build_ext(force=False):
    src = os.path.join(CSRC, "_crypto_ext.c")
    if not force and not _stale(EXT, [src, LIB, os.path.join(INCLUDE, "quic_pp.h")]):
        return EXT
    # a full-API build of an earlier layout would shadow the abi3 module
    old = os.path.join(PKG, "_crypto" + sysconfig.get_config_var("EXT_SUFFIX"))
    if os.path.exists(old):
        os.remove(old)
    pyinc = sysconfig.get_paths()["include"]
    cmd = ["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-Wall", "-pthread", "-I", pyinc, "-I", INCLUDE,
           src, "-L", PKG, "-lquicpp", "-Wl,-rpath,$ORIGIN", "-o", EXT + ".tmp"]
    _run(cmd)
    os.replace(EXT + ".tmp", EXT)
    return EXT


def build_all(force=False):
    build_lib(force)
    build_ext(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
