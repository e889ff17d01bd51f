"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
entry point include/quic_pp.h declares, and the record layouts the Python side
builds match the header's structs.  No compute calls (no GPU here)."""

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "quic_pp.h")
LIB = os.path.join(ROOT, "aioquic_amd", "libquicpp.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(qpp_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("qpp_protect", "qpp_unprotect", "qpp_hp_mask", "qpp_keytab_create",
                 "qpp_keytab_set", "qpp_session_protect", "qpp_session_unprotect"):
        assert must in names
    assert len(names) >= 18


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build() first: aioquic_amd/libquicpp.so missing"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, f"declared in quic_pp.h but not exported: {missing}"


def test_library_loads_and_reports_abi():
    import aioquic_amd  # noqa: F401  (binds torch's HIP runtime first)

    lib = ctypes.CDLL(LIB)
    for n in declared_functions():
        getattr(lib, n)
    lib.qpp_abi_version.restype = ctypes.c_int
    assert lib.qpp_abi_version() == 3
    lib.qpp_strerror.restype = ctypes.c_char_p
    lib.qpp_strerror.argtypes = [ctypes.c_int]
    assert lib.qpp_strerror(0)


def _struct_sizes_from_header():
    # the header comments state each struct's size; the numpy views must agree
    src = open(HEADER).read()
    return {m.group(1): int(m.group(2))
            for m in re.finditer(r"\}\s*(qpp_[a-z_]+);\s*/\*\s*(\d+) bytes", src)}


def test_record_layouts_match_header():
    from aioquic_amd import layout as L

    sizes = _struct_sizes_from_header()
    assert sizes["qpp_desc"] == L.DESC.itemsize == 40
    assert sizes["qpp_result"] == L.RESULT.itemsize == 16
    assert sizes["qpp_key_material"] == L.KEY_MATERIAL.itemsize == 84
    assert sizes["qpp_secret"] == L.SECRET.itemsize == 80
    assert L.DESC.fields["pn"][1] == 24 and L.DESC.fields["slot"][1] == 32
    assert L.RESULT.fields["status"][1] == 8


def test_extension_module_surface():
    """The CPython binding exposes aioquic._crypto's names (_crypto.pyi:1-15)."""
    from aioquic_amd import _crypto

    for name in ("AEAD", "HeaderProtection", "CryptoError"):
        assert hasattr(_crypto, name)
    assert issubclass(_crypto.CryptoError, ValueError)
    for meth in ("encrypt", "decrypt"):
        assert hasattr(_crypto.AEAD, meth)
    for meth in ("apply", "remove"):
        assert hasattr(_crypto.HeaderProtection, meth)


def test_constructor_errors_without_device():
    """Argument validation happens before any device work, with the
    reference's exact messages (_crypto.c:79-90)."""
    from aioquic_amd import _crypto

    with pytest.raises(_crypto.CryptoError, match="Invalid cipher name: aes-512-gcm"):
        _crypto.AEAD(b"aes-512-gcm", bytes(16), bytes(12))
    with pytest.raises(_crypto.CryptoError, match="Invalid key length"):
        _crypto.AEAD(b"aes-128-gcm", bytes(33), bytes(12))
    with pytest.raises(_crypto.CryptoError, match="Invalid iv length"):
        _crypto.AEAD(b"aes-128-gcm", bytes(16), bytes(13))


def test_key_material_record():
    from aioquic_amd import layout as L

    rec = L.key_material(7, L.AES_256_GCM, bytes(range(32)), bytes(range(12)), bytes(32), 1)
    assert rec["slot"][0] == 7 and rec["suite"][0] == 1 and rec["key_phase"][0] == 1
    assert bytes(rec["key"][0]) == bytes(range(32))
    assert rec.tobytes()[8:20] == bytes(range(12))
    assert np.frombuffer(rec.tobytes(), dtype=L.KEY_MATERIAL)[0]["slot"] == 7
