// qpp_chacha.h -- ChaCha20 block function and Poly1305 (radix 2^26) for the
// MI355X engine.  RFC 8439 sec. 2.3 / 2.5.  VALU only.
#pragma once

#include "qpp_device.h"

namespace qpp {

#define QPP_QR(a, b, c, d)                                      \
    a += b; d = rotl(d ^ a, 16);                                \
    c += d; b = rotl(b ^ c, 12);                                \
    a += b; d = rotl(d ^ a, 8);                                 \
    c += d; b = rotl(b ^ c, 7)

// 64-byte ChaCha20 block as 16 little-endian words.
__device__ __forceinline__ void chacha_block(const uint32_t *key, uint32_t ctr, uint32_t n0,
                                             uint32_t n1, uint32_t n2, uint32_t out[16])
{
    uint32_t x0 = 0x61707865, x1 = 0x3320646e, x2 = 0x79622d32, x3 = 0x6b206574;
    uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
    uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
    uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        QPP_QR(x0, x4, x8, x12);
        QPP_QR(x1, x5, x9, x13);
        QPP_QR(x2, x6, x10, x14);
        QPP_QR(x3, x7, x11, x15);
        QPP_QR(x0, x5, x10, x15);
        QPP_QR(x1, x6, x11, x12);
        QPP_QR(x2, x7, x8, x13);
        QPP_QR(x3, x4, x9, x14);
    }
    out[0] = x0 + 0x61707865; out[1] = x1 + 0x3320646e;
    out[2] = x2 + 0x79622d32; out[3] = x3 + 0x6b206574;
    out[4] = x4 + key[0]; out[5] = x5 + key[1]; out[6] = x6 + key[2]; out[7] = x7 + key[3];
    out[8] = x8 + key[4]; out[9] = x9 + key[5]; out[10] = x10 + key[6]; out[11] = x11 + key[7];
    out[12] = x12 + ctr; out[13] = x13 + n0; out[14] = x14 + n1; out[15] = x15 + n2;
}

// chacha_block with side(i) called after double round i (i = 0..9), in the
// same straight-line code: independent work placed there (Poly1305 of the
// previous chunk) shares a basic block with the rounds, so the scheduler can
// interleave the two dependency chains.
template <class SIDE>
__device__ __forceinline__ void chacha_block_beside(const uint32_t *key, uint32_t ctr, uint32_t n0,
                                                    uint32_t n1, uint32_t n2, uint32_t out[16], SIDE side)
{
    uint32_t x0 = 0x61707865, x1 = 0x3320646e, x2 = 0x79622d32, x3 = 0x6b206574;
    uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
    uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
    uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        QPP_QR(x0, x4, x8, x12);
        QPP_QR(x1, x5, x9, x13);
        QPP_QR(x2, x6, x10, x14);
        QPP_QR(x3, x7, x11, x15);
        QPP_QR(x0, x5, x10, x15);
        QPP_QR(x1, x6, x11, x12);
        QPP_QR(x2, x7, x8, x13);
        QPP_QR(x3, x4, x9, x14);
        side(i);
    }
    out[0] = x0 + 0x61707865; out[1] = x1 + 0x3320646e;
    out[2] = x2 + 0x79622d32; out[3] = x3 + 0x6b206574;
    out[4] = x4 + key[0]; out[5] = x5 + key[1]; out[6] = x6 + key[2]; out[7] = x7 + key[3];
    out[8] = x8 + key[4]; out[9] = x9 + key[5]; out[10] = x10 + key[6]; out[11] = x11 + key[7];
    out[12] = x12 + ctr; out[13] = x13 + n0; out[14] = x14 + n1; out[15] = x15 + n2;
}

// One ChaCha20 block computed by the 4 lanes of a quad together (all four
// hold the same inputs): lane j keeps column j (words j, 4+j, 8+j, 12+j), the
// column rounds are lane-local and the diagonal rounds rotate rows 1-3 by
// 1/2/3 lanes with DPP.  ~30 VALU per double round and 4 state registers, for
// the header-protection block every lane of the quad needs (sec. 5.4.4 of
// RFC 9001), instead of 96 VALU and 16 registers per lane for a private copy.
// Returns output words 0..3 (the first 16 keystream bytes) in every lane.
template <int CTRL>
__device__ __forceinline__ uint32_t qdpp(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

__device__ __forceinline__ u32x4 chacha_block_quad_row0(const uint32_t *key, uint32_t ctr,
                                                        uint32_t n0, uint32_t n1, uint32_t n2,
                                                        int sub)
{
    constexpr int kRot1 = 0x39, kRot2 = 0x4E, kRot3 = 0x93;  // lane j <- lane j+1 / j+2 / j+3
    const uint32_t sig = sub == 0 ? 0x61707865u : sub == 1 ? 0x3320646eu : sub == 2 ? 0x79622d32u : 0x6b206574u;
    const uint32_t kb = sub == 0 ? key[0] : sub == 1 ? key[1] : sub == 2 ? key[2] : key[3];
    const uint32_t kc = sub == 0 ? key[4] : sub == 1 ? key[5] : sub == 2 ? key[6] : key[7];
    const uint32_t kd = sub == 0 ? ctr : sub == 1 ? n0 : sub == 2 ? n1 : n2;
    uint32_t a = sig, b = kb, c = kc, d = kd;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        QPP_QR(a, b, c, d);
        b = qdpp<kRot1>(b); c = qdpp<kRot2>(c); d = qdpp<kRot3>(d);
        QPP_QR(a, b, c, d);
        b = qdpp<kRot3>(b); c = qdpp<kRot2>(c); d = qdpp<kRot1>(d);
    }
    a += sig;  // output word `sub` of row 0
    return u32x4{qdpp<0x00>(a), qdpp<0x55>(a), qdpp<0xAA>(a), qdpp<0xFF>(a)};
}
#undef QPP_QR

// ------------------------------------------------------------ Poly1305 ----

struct P130 {
    uint32_t v[5];  // 26-bit limbs (slightly larger between reductions)
};

constexpr uint32_t kM26 = 0x3ffffff;

__device__ __forceinline__ P130 p130_zero() { return P130{{0, 0, 0, 0, 0}}; }

// 16-byte little-endian block plus 2^128 (every AEAD block is full, RFC 8439 sec. 2.8)
__device__ __forceinline__ P130 p130_block(u32x4 m)
{
    return P130{{m.x & kM26, ((m.x >> 26) | (m.y << 6)) & kM26, ((m.y >> 20) | (m.z << 12)) & kM26,
                 ((m.z >> 14) | (m.w << 18)) & kM26, (m.w >> 8) | (1u << 24)}};
}

__device__ __forceinline__ P130 p130_add(P130 a, P130 b)
{
    return P130{{a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3],
                 a.v[4] + b.v[4]}};
}

// h * r mod 2^130-5 with partial carry; r limbs < 2^26, h limbs < 2^29.
__device__ __forceinline__ P130 p130_mul(P130 h, P130 r)
{
    const uint32_t r0 = r.v[0], r1 = r.v[1], r2 = r.v[2], r3 = r.v[3], r4 = r.v[4];
    const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
    const uint64_t h0 = h.v[0], h1 = h.v[1], h2 = h.v[2], h3 = h.v[3], h4 = h.v[4];
    uint64_t d0 = h0 * r0 + h1 * s4 + h2 * s3 + h3 * s2 + h4 * s1;
    uint64_t d1 = h0 * r1 + h1 * r0 + h2 * s4 + h3 * s3 + h4 * s2;
    uint64_t d2 = h0 * r2 + h1 * r1 + h2 * r0 + h3 * s4 + h4 * s3;
    uint64_t d3 = h0 * r3 + h1 * r2 + h2 * r1 + h3 * r0 + h4 * s4;
    uint64_t d4 = h0 * r4 + h1 * r3 + h2 * r2 + h3 * r1 + h4 * r0;
    d1 += d0 >> 26;
    d2 += d1 >> 26;
    d3 += d2 >> 26;
    d4 += d3 >> 26;
    uint32_t o0 = (uint32_t)d0 & kM26, o1 = (uint32_t)d1 & kM26, o2 = (uint32_t)d2 & kM26;
    uint32_t o3 = (uint32_t)d3 & kM26, o4 = (uint32_t)d4 & kM26;
    uint64_t c = (d4 >> 26) * 5 + o0;
    o0 = (uint32_t)c & kM26;
    o1 += (uint32_t)(c >> 26);
    return P130{{o0, o1, o2, o3, o4}};
}

// d += h * r: the five 64-bit column sums of p130_mul without its carry.  A
// sum of four such products stays below 2^64 for h limbs < 2^27 and r limbs
// < 2^26 + 2^11 (each column < 2^57.7 per product), so four blocks of a chunk
// can be multiplied by their own powers of r and carried once (p130_carry).
__device__ __forceinline__ void p130_mac(uint64_t (&d)[5], P130 h, P130 r)
{
    const uint32_t r0 = r.v[0], r1 = r.v[1], r2 = r.v[2], r3 = r.v[3], r4 = r.v[4];
    const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
    const uint64_t h0 = h.v[0], h1 = h.v[1], h2 = h.v[2], h3 = h.v[3], h4 = h.v[4];
    d[0] += h0 * r0 + h1 * s4 + h2 * s3 + h3 * s2 + h4 * s1;
    d[1] += h0 * r1 + h1 * r0 + h2 * s4 + h3 * s3 + h4 * s2;
    d[2] += h0 * r2 + h1 * r1 + h2 * r0 + h3 * s4 + h4 * s3;
    d[3] += h0 * r3 + h1 * r2 + h2 * r1 + h3 * r0 + h4 * s4;
    d[4] += h0 * r4 + h1 * r3 + h2 * r2 + h3 * r1 + h4 * r0;
}

// the partial carry of p130_mul on column sums (limbs < 2^26 but limb 1)
__device__ __forceinline__ P130 p130_carry(uint64_t d0, uint64_t d1, uint64_t d2, uint64_t d3, uint64_t d4)
{
    d1 += d0 >> 26;
    d2 += d1 >> 26;
    d3 += d2 >> 26;
    d4 += d3 >> 26;
    uint32_t o0 = (uint32_t)d0 & kM26, o1 = (uint32_t)d1 & kM26, o2 = (uint32_t)d2 & kM26;
    uint32_t o3 = (uint32_t)d3 & kM26, o4 = (uint32_t)d4 & kM26;
    uint64_t c = (d4 >> 26) * 5 + o0;
    o0 = (uint32_t)c & kM26;
    o1 += (uint32_t)(c >> 26);
    return P130{{o0, o1, o2, o3, o4}};
}

// clamp(r) from the first 16 bytes of the one-time key (RFC 8439 sec. 2.5)
__device__ __forceinline__ P130 p130_r(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3)
{
    k0 &= 0x0fffffff; k1 &= 0x0ffffffc; k2 &= 0x0ffffffc; k3 &= 0x0ffffffc;
    return P130{{k0 & kM26, ((k0 >> 26) | (k1 << 6)) & kM26, ((k1 >> 20) | (k2 << 12)) & kM26,
                 ((k2 >> 14) | (k3 << 18)) & kM26, k3 >> 8}};
}

// full reduction mod 2^130-5, then + s mod 2^128 -> tag words
__device__ __forceinline__ u32x4 p130_finish(P130 h, uint32_t s0, uint32_t s1, uint32_t s2,
                                             uint32_t s3)
{
    uint32_t h0 = h.v[0], h1 = h.v[1], h2 = h.v[2], h3 = h.v[3], h4 = h.v[4], c;
    c = h1 >> 26; h1 &= kM26; h2 += c;
    c = h2 >> 26; h2 &= kM26; h3 += c;
    c = h3 >> 26; h3 &= kM26; h4 += c;
    c = h4 >> 26; h4 &= kM26; h0 += c * 5;
    c = h0 >> 26; h0 &= kM26; h1 += c;
    c = h1 >> 26; h1 &= kM26; h2 += c;
    // g = h + 5 - 2^130; take g when it does not borrow
    uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= kM26;
    uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= kM26;
    uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= kM26;
    uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= kM26;
    uint32_t g4 = h4 + c - (1u << 26);
    uint32_t keep_h = (uint32_t)((int32_t)g4 >> 31);  // all ones if g4 borrowed
    h0 = (h0 & keep_h) | (g0 & ~keep_h);
    h1 = (h1 & keep_h) | (g1 & ~keep_h);
    h2 = (h2 & keep_h) | (g2 & ~keep_h);
    h3 = (h3 & keep_h) | (g3 & ~keep_h);
    h4 = (h4 & keep_h) | (g4 & ~keep_h);
    uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14),
             w3 = (h3 >> 18) | (h4 << 8);
    uint64_t f = (uint64_t)w0 + s0;
    w0 = (uint32_t)f;
    f = (uint64_t)w1 + s1 + (f >> 32);
    w1 = (uint32_t)f;
    f = (uint64_t)w2 + s2 + (f >> 32);
    w2 = (uint32_t)f;
    w3 = w3 + s3 + (uint32_t)(f >> 32);
    return u32x4{w0, w1, w2, w3};
}

}  // namespace qpp
