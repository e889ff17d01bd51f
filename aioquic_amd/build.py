"""In-tree build of the native parts (no setuptools, no JIT cache):

  aioquic_amd/libquicpp.so   HIP kernels + C ABI (include/quic_pp.h), gfx950 only
  aioquic_amd/_crypto*.so    CPython binding of the C ABI (links libquicpp.so via $ORIGIN)

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
LIB = os.path.join(PKG, "libquicpp.so")
EXT = os.path.join(PKG, "_crypto" + sysconfig.get_config_var("EXT_SUFFIX"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

HIP_SOURCES = ["qpp_engine.hip"]
HIP_DEPS = HIP_SOURCES + ["qpp_device.h", "qpp_chacha.h", "qpp_hkdf.h", "qpp_sha_consts.h"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_lib(force=False, extra=()):
    deps = [os.path.join(CSRC, f) for f in HIP_DEPS] + [os.path.join(INCLUDE, "quic_pp.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-I", INCLUDE, "-o", LIB + ".tmp"]
    cmd += list(extra) + [os.path.join(CSRC, f) for f in HIP_SOURCES]
    _run(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_ext(force=False):
    src = os.path.join(CSRC, "_crypto_ext.c")
    if not force and not _stale(EXT, [src, LIB, os.path.join(INCLUDE, "quic_pp.h")]):
        return EXT
    pyinc = sysconfig.get_paths()["include"]
    cmd = ["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-Wall", "-I", pyinc, "-I", INCLUDE,
           src, "-L", PKG, "-lquicpp", "-Wl,-rpath,$ORIGIN", "-o", EXT + ".tmp"]
    _run(cmd)
    os.replace(EXT + ".tmp", EXT)
    return EXT


def build_all(force=False):
    build_lib(force)
    build_ext(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
