"""CPU check of the device key schedule's HKDF (aioquic_amd/csrc/qpp_hkdf.h,
built for the host here) against the stdlib restatement of the reference's
hkdf_expand_label (tls.py:164-185) and the RFC 9001 / 9369 derivations."""

import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("hkdf") / "libhkdf_host.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tests", "hkdf_host.cc")], check=True)
    lib = ctypes.CDLL(so)
    lib.qpp_test_expand_label.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                          ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_char_p]
    return lib


def _expand(lib, big, secret, label, length):
    out = ctypes.create_string_buffer(48)
    lib.qpp_test_expand_label(int(big), secret, len(secret), label, len(label), length, out)
    return out.raw[:length]


@pytest.mark.parametrize("big", [False, True], ids=["sha256", "sha384"])
def test_expand_label_matches_stdlib(lib, big):
    from aioquic_amd.tls import SHA256, SHA384, hkdf_expand_label

    alg = SHA384 if big else SHA256
    rng = np.random.default_rng(3 + big)
    for label in (b"quic key", b"quic iv", b"quic hp", b"quicv2 key", b"quicv2 iv",
                  b"quicv2 hp", b"quic ku", b"client in", b"server in"):
        for slen in (32, 48, 1, 64):
            secret = rng.bytes(slen)
            for length in (12, 16, 32, alg.digest_size):
                assert _expand(lib, big, secret, label, length) == \
                    hkdf_expand_label(alg, secret, label, b"", length)


def test_rfc9001_client_initial_key(lib):
    """RFC 9001 App. A.1: client_initial_secret -> key / iv / hp."""
    from tests.rfc import V1, V2

    for v in (V1, V2):
        secret, key, iv, hp = v.derive_client
        pre = b"quicv2 " if v.version == 0x6B3343CF else b"quic "
        assert _expand(lib, False, secret, pre + b"key", 16) == key
        assert _expand(lib, False, secret, pre + b"iv", 12) == iv
        assert _expand(lib, False, secret, pre + b"hp", 16) == hp
