"""CPU check of the bitsliced AES (tools/bitslice/qpp_bitslice.h, built for
the host here): the Boyar-Peralta S-box circuit against the FIPS-197 S-box
for all 256 inputs, the FIPS-197 App. C known answers, and random blocks
against the oracle's AES-ECB (the header-protection mask of the AES suites,
HeaderProtection_mask, _crypto.c:278-287)."""

import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("bs") / "libbs_host.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tests", "bs_host.cc")], check=True)
    return ctypes.CDLL(so)


def _gmul(a, b):
    r = 0
    for _ in range(8):
        if b & 1:
            r ^= a
        a = ((a << 1) ^ (0x1B if a & 0x80 else 0)) & 0xFF
        b >>= 1
    return r


def test_sbox_circuit_matches_fips197(lib):
    out = ctypes.create_string_buffer(256)
    lib.qpp_test_bs_sbox(out)
    for x in range(256):
        inv = 0 if x == 0 else next(y for y in range(1, 256) if _gmul(x, y) == 1)
        s = inv
        for i in range(1, 5):
            s ^= ((inv << i) | (inv >> (8 - i))) & 0xFF
        assert out.raw[x] == s ^ 0x63, x


def _enc(lib, key, blocks, gen=False):
    out = ctypes.create_string_buffer(512)
    fn = lib.qpp_test_bs_encrypt_gen if gen else lib.qpp_test_bs_encrypt
    nr = fn(key, len(key), bytes(blocks), out)
    return nr, out.raw


@pytest.mark.parametrize("gen", [False, True], ids=["plain", "bitop3"])
@pytest.mark.parametrize("klen,want", [
    (16, "69c4e0d86a7b0430d8cdb78070b4c55a"),
    (32, "8ea2b7ca516745bfeafc49904b496089")], ids=["aes128", "aes256"])
def test_fips197_known_answer(lib, klen, want, gen):
    key = bytes(range(klen))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    nr, out = _enc(lib, key, pt * 32, gen)
    assert nr == (10 if klen == 16 else 14)
    for s in range(32):
        assert out[16 * s : 16 * s + 16].hex() == want


@pytest.mark.parametrize("gen", [False, True], ids=["plain", "bitop3"])
@pytest.mark.parametrize("klen", [16, 32])
def test_random_blocks_vs_oracle(lib, oracle, klen, gen):
    rng = np.random.default_rng(klen)
    suite = 0 if klen == 16 else 1
    for _ in range(8):
        key = rng.bytes(klen)
        blocks = rng.bytes(512)
        _, out = _enc(lib, key, blocks, gen)
        for s in range(32):
            assert out[16 * s : 16 * s + 16] == oracle.hp_mask(suite, key, blocks[16 * s : 16 * s + 16])


def test_transpose_round_trip(lib):
    data = np.random.default_rng(1).bytes(512)
    out = ctypes.create_string_buffer(512)
    lib.qpp_test_bs_transpose_roundtrip(data, out)
    assert out.raw == data
