#!/usr/bin/env python3
"""Single-packet latency probe (for rocprofv3 --kernel-trace --stats)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aioquic_amd._crypto import AEAD
import numpy as np
rng = np.random.default_rng(1)
for name, kl in ((b"aes-128-gcm", 16), (b"chacha20-poly1305", 32)):
    a = AEAD(name, rng.bytes(kl), rng.bytes(12))
    p = rng.bytes(1173); h = rng.bytes(11)
    for _ in range(50): a.encrypt(p, h, 1)
    t = time.perf_counter()
    for _ in range(300): a.encrypt(p, h, 1)
    print(name.decode(), round((time.perf_counter() - t) / 300 * 1e6, 1), "us")
