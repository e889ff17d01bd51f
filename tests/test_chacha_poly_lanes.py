"""The lane schedule of k_chacha's Poly1305 (aioquic_amd/csrc/qpp_engine.hip,
chacha_packet), restated over integers mod 2^130 - 5 and checked against the
direct polynomial sum_i X_i r^(m - i) of RFC 8439 sec. 2.5 over
[AAD blocks | ciphertext blocks | lengths] (the tag before + s).

A quad's lane j takes 64-byte chunks j - 1, j + 3, ... (lane 0 first folds
the associated data); per chunk c it moves its chain by
    acc <- (acc + x0) r^e0 + x1 r^e1 + x2 r^e2 + x3 r^e3
with e = 16 .. 13 while the lane has a later chunk, else the chunk's own
valid block count nbv - b (a missing block adds zero, no chunk at all:
r^0); the close combines the four chains as
    (A[L+1] r^8 + A[L+2] r^4 + A[L+3]) r^(nb+1) + (A[L] + lens) r,
L = chunks mod 4.  No GPU: this pins the exponent rule the kernel uses
(round 6), the GPU parity tests pin the kernel itself."""
import random

import pytest

P = (1 << 130) - 5


def lane_schedule(aad, ct, lens, r):
    n_a, n_c = len(aad), len(ct)
    chunks = (n_c + 3) // 4
    steps = (chunks + 4) >> 2
    acc = [0, 0, 0, 0]
    r13 = pow(r, 13, P)
    for g in range(n_a):  # lane 0: the associated data (its next chunk is chunk 3)
        acc[0] = (acc[0] + aad[g]) * (r13 if (g == n_a - 1 and 3 < chunks) else r) % P

    def chunk(sub, c):
        inc = 0 <= c < chunks
        nbv = min(4, n_c - 4 * c)
        tot = 0
        for b in range(4):
            valid = inc and b < nbv
            e = 0 if not inc else (16 - b if c + 4 < chunks else (nbv - b if valid else 0))
            m = ct[4 * c + b] if valid else 0
            if b == 0:
                m += acc[sub]
            tot += m * pow(r, e, P)
        acc[sub] = tot % P

    for k in range(steps):
        for sub in range(4):
            chunk(sub, 4 * k + sub - 1)
    L = chunks & 3
    nb = n_c - 4 * (chunks - 1) if chunks > 0 else 1
    u = v = 0
    for sub in range(4):
        role = (sub - L - 1) & 3  # 0: lane L+1, 1: L+2, 2: L+3, 3: L
        a = acc[sub] + (lens if role == 3 else 0)
        m = a * pow(r, (8, 4, 0, 1)[role], P)
        if role == 3:
            v += m
        else:
            u += m
    return (u * pow(r, nb + 1, P) + v) % P


def direct(aad, ct, lens, r):
    seq = aad + ct + [lens]
    m = len(seq)
    return sum(x * pow(r, m - i, P) for i, x in enumerate(seq)) % P


@pytest.mark.parametrize("seed", range(4))
def test_lane_schedule_equals_poly1305_polynomial(seed):
    rng = random.Random(seed)
    for _ in range(150):
        hlen = rng.choice([0, 1, 11, 16, 20, 33, 48, 60])
        clen = rng.choice([0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 129, 191, 192, 255, 256, 257,
                           1173, 1184, 1500, rng.randrange(0, 1600)])
        aad = [rng.randrange(1 << 129) for _ in range((hlen + 15) // 16)]
        ct = [rng.randrange(1 << 129) for _ in range((clen + 15) // 16)]
        lens = rng.randrange(1 << 129)
        r = rng.randrange(1, P)
        assert lane_schedule(aad, ct, lens, r) == direct(aad, ct, lens, r), (hlen, clen)
