#!/usr/bin/env python3
"""Per-call latency breakdown of the object API (one packet per call): run
under rocprofv3 --kernel-trace --hip-trace --stats to split the ~50 us of an
AEAD.encrypt into kernel time and HIP runtime calls.  Prints the mean wall
time per call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aioquic_amd._crypto import AEAD  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
aead = AEAD(b"aes-128-gcm", bytes(range(16)), bytes(12))
hdr = bytes([0x41]) + bytes(10)
payload = bytes(1173)
for _ in range(50):
    aead.encrypt(payload, hdr, 1)
t = time.perf_counter()
for i in range(n):
    aead.encrypt(payload, hdr, i)
print(f"AEAD.encrypt: {(time.perf_counter() - t) / n * 1e6:.2f} us per call over {n} calls")
