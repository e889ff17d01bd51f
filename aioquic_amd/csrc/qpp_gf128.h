// qpp_gf128.h -- GF(2^128) multiplication of two arbitrary elements in the
// GCM convention (SP 800-38D sec. 6.3), table-free, for the lone-packet
// kernel's per-lane powers of H (k_lone_gcm): no carry-less multiply
// instruction exists on gfx950, so 32 x 32 carry-less products come from
// integer multiplies with "holes" -- each operand split into 4 interleaved
// bit classes (every 4th bit), so that the at most 8 terms meeting in one
// product bit never carry into the next bit of the same class -- and
// Karatsuba on top (9 such products for 128 x 128 bits), then the reduction
// by x^128 + x^7 + x^2 + x + 1.  ~650 VALU with 9-way independent work,
// against ~1,900 in a dependent chain for the bit-serial algorithm.
//
// Elements are 16-byte blocks as four little-endian 32-bit words (the
// kernels' loads).  GCM numbers the bits of a block from the most significant
// bit of byte 0 (coefficient of x^0), so a word becomes a plain polynomial
// limb by reversing the bits within each byte.
//
// Plain C++ so that the CPU unit test (tests/gf_host.cc) builds it for the host.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define QPP_GF_HD __host__ __device__ __forceinline__
#else
#define QPP_GF_HD inline
#endif

namespace qpp {
namespace gf {

// bits reversed within each byte of a word (an involution)
QPP_GF_HD uint32_t rev_bytes(uint32_t w)
{
#if defined(__HIPCC__)
    return __builtin_bswap32(__builtin_bitreverse32(w));
#else
    w = ((w >> 1) & 0x55555555u) | ((w & 0x55555555u) << 1);
    w = ((w >> 2) & 0x33333333u) | ((w & 0x33333333u) << 2);
    return ((w >> 4) & 0x0f0f0f0fu) | ((w & 0x0f0f0f0fu) << 4);
#endif
}

// carry-less 32 x 32 -> 64 bits through 16 integer multiplies
QPP_GF_HD uint64_t clmul32(uint32_t a, uint32_t b)
{
    const uint32_t a0 = a & 0x11111111u, a1 = a & 0x22222222u, a2 = a & 0x44444444u, a3 = a & 0x88888888u;
    const uint32_t b0 = b & 0x11111111u, b1 = b & 0x22222222u, b2 = b & 0x44444444u, b3 = b & 0x88888888u;
    const uint64_t z0 = ((uint64_t)a0 * b0) ^ ((uint64_t)a1 * b3) ^ ((uint64_t)a2 * b2) ^ ((uint64_t)a3 * b1);
    const uint64_t z1 = ((uint64_t)a0 * b1) ^ ((uint64_t)a1 * b0) ^ ((uint64_t)a2 * b3) ^ ((uint64_t)a3 * b2);
    const uint64_t z2 = ((uint64_t)a0 * b2) ^ ((uint64_t)a1 * b1) ^ ((uint64_t)a2 * b0) ^ ((uint64_t)a3 * b3);
    const uint64_t z3 = ((uint64_t)a0 * b3) ^ ((uint64_t)a1 * b2) ^ ((uint64_t)a2 * b1) ^ ((uint64_t)a3 * b0);
    return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) | (z2 & 0x4444444444444444ull) |
           (z3 & 0x8888888888888888ull);
}

// carry-less 64 x 64 -> 128 bits (Karatsuba over 32-bit halves): lo, hi
QPP_GF_HD void clmul64(uint64_t a, uint64_t b, uint64_t &lo, uint64_t &hi)
{
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t l = clmul32(a0, b0), h = clmul32(a1, b1);
    const uint64_t m = clmul32(a0 ^ a1, b0 ^ b1) ^ l ^ h;
    lo = l ^ (m << 32);
    hi = h ^ (m >> 32);
}

// x * y in GF(2^128), GCM convention, 16-byte blocks as little-endian words
struct Blk {
    uint32_t w[4];
};

QPP_GF_HD Blk mul(Blk x, Blk y)
{
    // plain polynomial limbs: bit i of (a1:a0) = coefficient of x^i
    const uint64_t a0 = (uint64_t)rev_bytes(x.w[1]) << 32 | rev_bytes(x.w[0]);
    const uint64_t a1 = (uint64_t)rev_bytes(x.w[3]) << 32 | rev_bytes(x.w[2]);
    const uint64_t b0 = (uint64_t)rev_bytes(y.w[1]) << 32 | rev_bytes(y.w[0]);
    const uint64_t b1 = (uint64_t)rev_bytes(y.w[3]) << 32 | rev_bytes(y.w[2]);
    // 256-bit product c3:c2:c1:c0 (Karatsuba over 64-bit halves)
    uint64_t l0, l1, h0, h1, m0, m1;
    clmul64(a0, b0, l0, l1);
    clmul64(a1, b1, h0, h1);
    clmul64(a0 ^ a1, b0 ^ b1, m0, m1);
    m0 ^= l0 ^ h0;
    m1 ^= l1 ^ h1;
    const uint64_t c0 = l0, c1 = l1 ^ m0, c2 = h0 ^ m1, c3 = h1;
    // x^128 = x^7 + x^2 + x + 1: fold c3:c2 down, then the <= 7 bits that
    // the shifts carried past x^127
    const uint64_t t = (c3 >> 63) ^ (c3 >> 62) ^ (c3 >> 57);
    const uint64_t r0 = c0 ^ c2 ^ (c2 << 1) ^ (c2 << 2) ^ (c2 << 7) ^ t ^ (t << 1) ^ (t << 2) ^ (t << 7);
    const uint64_t r1 = c1 ^ c3 ^ (c3 << 1 | c2 >> 63) ^ (c3 << 2 | c2 >> 62) ^ (c3 << 7 | c2 >> 57);
    return Blk{{rev_bytes((uint32_t)r0), rev_bytes((uint32_t)(r0 >> 32)), rev_bytes((uint32_t)r1),
                rev_bytes((uint32_t)(r1 >> 32))}};
}

}  // namespace gf
}  // namespace qpp
