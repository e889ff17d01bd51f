"""CPU check of the table-free GF(2^128) multiply of the lone-packet kernel
(aioquic_amd/csrc/qpp_gf128.h, built for the host here) against SP 800-38D
Algorithm 1, on random blocks and on the GCM test case's H and GHASH input
(H = E_K(0) of the all-zero key: 66e94bd4ef8a2c3b884cfa59ca342b2e)."""

import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("gf") / "libgf_host.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tests", "gf_host.cc")], check=True)
    lib = ctypes.CDLL(so)
    lib.qpp_test_gf_mul.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return lib


def _gf_mul(x: bytes, y: bytes) -> bytes:
    """SP 800-38D sec. 6.3, Algorithm 1."""
    X, V, Z = int.from_bytes(x, "big"), int.from_bytes(y, "big"), 0
    R = 0xE1 << 120
    for i in range(128):
        if (X >> (127 - i)) & 1:
            Z ^= V
        V = (V >> 1) ^ R if V & 1 else V >> 1
    return Z.to_bytes(16, "big")


def _mul(lib, xs, ys):
    n = len(xs)
    x = np.frombuffer(b"".join(xs), np.uint8).copy()
    y = np.frombuffer(b"".join(ys), np.uint8).copy()
    out = np.zeros(16 * n, np.uint8)
    lib.qpp_test_gf_mul(x.ctypes.data, y.ctypes.data, out.ctypes.data, n)
    return [out[16 * i : 16 * i + 16].tobytes() for i in range(n)]


def test_random_products(lib):
    rng = np.random.default_rng(128)
    xs = [rng.bytes(16) for _ in range(300)]
    ys = [rng.bytes(16) for _ in range(300)]
    # edge elements: zero, one (x^0 = 0x80 in byte 0), x^127, all ones
    edge = [bytes(16), b"\x80" + bytes(15), bytes(15) + b"\x01", b"\xff" * 16]
    xs += edge * 4
    ys += [e for e in edge for _ in range(4)]
    for x, y, z in zip(xs, ys, _mul(lib, xs, ys)):
        assert z == _gf_mul(x, y), (x.hex(), y.hex())


def test_gcm_test_case_2(lib):
    """GCM spec test case 2 (K = 0, P = 0^128, IV = 0^96): GHASH(H, {}, C) =
    f38cbb1ad69223dcc3457ae5b6b0f885, computed as (C H + L) H."""
    h = bytes.fromhex("66e94bd4ef8a2c3b884cfa59ca342b2e")
    c = bytes.fromhex("0388dace60b6a392f328c2b971b2fe78")
    lens = bytes(8) + (128).to_bytes(8, "big")
    (ch,) = _mul(lib, [c], [h])
    (g,) = _mul(lib, [bytes(a ^ b for a, b in zip(ch, lens))], [h])
    assert g.hex() == "f38cbb1ad69223dcc3457ae5b6b0f885"
