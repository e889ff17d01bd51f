"""Stale-binary guard: the built libquicpp.so and
_crypto.abi3.so carry the hash of the native sources they were built from
(aioquic_amd/_srchash.py), and the extension refuses to import when the tree's
sources differ, so a snapshot with skewed file times cannot run old kernels.
CPU only: loading the extension needs no device."""

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "aioquic_amd")


def _copy_tree(dst):
    shutil.copytree(PKG, os.path.join(dst, "aioquic_amd"), ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(dst, "include"))


def _import(root):
    code = "import sys; sys.path.insert(0, %r); import aioquic_amd._crypto as c; print(c.source_hash())" % root
    return subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)


def test_built_objects_carry_the_tree_hash():
    from aioquic_amd import _srchash, build

    tree = _srchash.tree_hash()
    assert tree and len(tree) == 16
    assert build.embedded_hash(build.LIB) == tree
    assert build.embedded_hash(build.EXT) == tree


def test_import_refuses_edited_sources(tmp_path):
    root = str(tmp_path)
    _copy_tree(root)
    ok = _import(root)
    assert ok.returncode == 0, ok.stderr
    from aioquic_amd import _srchash

    assert ok.stdout.strip() == _srchash.tree_hash()
    # an edit to any native source, however small, and whatever its mtime
    src = os.path.join(root, "aioquic_amd", "csrc", "qpp_device.h")
    st = os.stat(src)
    with open(src, "a") as f:
        f.write("\n// edited\n")
    os.utime(src, (st.st_atime, st.st_mtime - 3600))  # older than the binaries
    bad = _import(root)
    assert bad.returncode != 0
    assert "ImportError" in bad.stderr and "changed since _crypto was built" in bad.stderr


def test_import_refuses_mismatched_library(tmp_path):
    """_crypto and libquicpp.so from different builds: the hash inside each."""
    root = str(tmp_path)
    _copy_tree(root)
    lib = os.path.join(root, "aioquic_amd", "libquicpp.so")
    data = bytearray(open(lib, "rb").read())
    from aioquic_amd import build

    i = data.find(build.MARKER)
    assert i >= 0
    j = i + len(build.MARKER)
    data[j:j + 16] = b"0123456789abcdef"
    with open(lib, "wb") as f:
        f.write(data)
    bad = _import(root)
    assert bad.returncode != 0
    assert "come from different builds" in bad.stderr


@pytest.mark.parametrize("unit", ["qpp_engine.hip"])
def test_objects_rebuild_on_content_not_time(tmp_path, unit):
    """build.py's staleness is the hash of an object's inputs recorded beside
    it: a file whose mtime moves without a content change is not stale."""
    from aioquic_amd import build

    obj = build._obj(unit)
    if not os.path.exists(obj + ".inputs"):
        pytest.skip("objects not built by this tree's build.py")
    deps = [os.path.join(build.CSRC, unit), os.path.join(build.INCLUDE, "quic_pp.h")] + \
        [os.path.join(build.CSRC, d) for d in build.COMMON_DEPS + build.HIP_UNITS[unit]]
    stale, _ = build._stale(obj, deps)
    assert not stale
    stale2, _ = build._stale(obj, deps, ["-DQPP_SOMETHING"])
    assert stale2  # other flags: rebuild
