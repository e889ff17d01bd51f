// qpp_bitslice.h -- bitsliced AES on 32-bit lanes: one lane encrypts 32
// blocks at once, holding 128 bit planes (plane 8 i + b = bit b of byte i of
// each of its 32 blocks, one block per bit position).  Every AES step is
// then plain VALU logic -- no table lookups, no LDS -- which is what gfx950
// has plenty of (v_bitop3_b32 evaluates any 3-input boolean function in one
// instruction): SubBytes is a 113-gate boolean circuit per byte, ShiftRows
// is register renaming, MixColumns and AddRoundKey are XORs.
//
// The S-box circuit is the public depth-16 circuit of Boyar and Peralta ("A
// depth-16 circuit for the AES S-box", 2012): a top linear layer, a
// GF(2^4)-inversion core and a bottom linear layer.  AES itself follows
// FIPS-197.  Round keys enter as masks, one 32-bit word per key bit (all
// zeros or all ones), so AddRoundKey is one XOR per plane.
//
// Written as plain C++ so the same code compiles for the host (the CPU unit
// test tests/bs_host.cc checks it against FIPS-197) and for gfx950, where
// the compiler maps the logic onto v_bitop3_b32.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define QPP_BS_HD __host__ __device__ __forceinline__
#else
#define QPP_BS_HD inline
#endif

// Scheduling fence on the device: keeps the compiler from interleaving the
// 16 independent S-boxes of a round, whose temporaries together would not
// fit the register file.  Nothing on the host.
// QPP_BS_FENCE_SBOX separates the four S-boxes of one output column,
// QPP_BS_FENCE the columns (A/B switches: QPP_BS_SBOX_FENCES, QPP_BS_COLUMN_FENCES).
#ifndef QPP_BS_SBOX_FENCES
#define QPP_BS_SBOX_FENCES 1
#endif
#ifndef QPP_BS_COLUMN_FENCES
#define QPP_BS_COLUMN_FENCES 1
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define QPP_BS_FENCE() do { if (QPP_BS_COLUMN_FENCES) __builtin_amdgcn_sched_barrier(0); } while (0)
#define QPP_BS_FENCE_SBOX() do { if (QPP_BS_SBOX_FENCES) __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define QPP_BS_FENCE() ((void)0)
#define QPP_BS_FENCE_SBOX() ((void)0)
#endif

// One v_bitop3_b32: bit ((s0 << 2) | (s1 << 1) | s2) of imm, for each bit.
#if defined(__HIP_DEVICE_COMPILE__)
#define QPP_LUT3(s0, s1, s2, imm) __builtin_amdgcn_bitop3_b32((s0), (s1), (s2), (imm))
#else
#define QPP_LUT3(s0, s1, s2, imm) qpp::bs::lut3_host((s0), (s1), (s2), (imm))
#endif

namespace qpp {
namespace bs {

inline uint32_t lut3_host(uint32_t a, uint32_t b, uint32_t c, uint32_t imm)
{
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i)
        if ((imm >> i) & 1)
            r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
}

}  // namespace bs
}  // namespace qpp

#include "qpp_bs_gen.h"

namespace qpp {
namespace bs {

// SubBytes of one byte position: q[b] = plane of bit b (b = 0 least significant).
QPP_BS_HD void sbox(uint32_t *q)
{
    const uint32_t x0 = q[7], x1 = q[6], x2 = q[5], x3 = q[4], x4 = q[3], x5 = q[2], x6 = q[1],
                   x7 = q[0];
    // top linear layer
    const uint32_t y14 = x3 ^ x5, y13 = x0 ^ x6, y9 = x0 ^ x3, y8 = x0 ^ x5, t0 = x1 ^ x2;
    const uint32_t y1 = t0 ^ x7, y4 = y1 ^ x3, y12 = y13 ^ y14, y2 = y1 ^ x0, y5 = y1 ^ x6;
    const uint32_t y3 = y5 ^ y8, t1 = x4 ^ y12, y15 = t1 ^ x5, y20 = t1 ^ x1, y6 = y15 ^ x7;
    const uint32_t y10 = y15 ^ t0, y11 = y20 ^ y9, y7 = x7 ^ y11, y17 = y10 ^ y11, y19 = y10 ^ y8;
    const uint32_t y16 = t0 ^ y11, y21 = y13 ^ y16, y18 = x0 ^ y16;
    // shared non-linear core (inversion in GF(2^4)^2)
    const uint32_t t2 = y12 & y15, t3 = y3 & y6, t4 = t3 ^ t2, t5 = y4 & x7, t6 = t5 ^ t2;
    const uint32_t t7 = y13 & y16, t8 = y5 & y1, t9 = t8 ^ t7, t10 = y2 & y7, t11 = t10 ^ t7;
    const uint32_t t12 = y9 & y11, t13 = y14 & y17, t14 = t13 ^ t12, t15 = y8 & y10, t16 = t15 ^ t12;
    const uint32_t t17 = t4 ^ t14, t18 = t6 ^ t16, t19 = t9 ^ t14, t20 = t11 ^ t16;
    const uint32_t t21 = t17 ^ y20, t22 = t18 ^ y19, t23 = t19 ^ y21, t24 = t20 ^ y18;
    const uint32_t t25 = t21 ^ t22, t26 = t21 & t23, t27 = t24 ^ t26, t28 = t25 & t27;
    const uint32_t t29 = t28 ^ t22, t30 = t23 ^ t24, t31 = t22 ^ t26, t32 = t31 & t30;
    const uint32_t t33 = t32 ^ t24, t34 = t23 ^ t33, t35 = t27 ^ t33, t36 = t24 & t35;
    const uint32_t t37 = t36 ^ t34, t38 = t27 ^ t36, t39 = t29 & t38, t40 = t25 ^ t39;
    const uint32_t t41 = t40 ^ t37, t42 = t29 ^ t33, t43 = t29 ^ t40, t44 = t33 ^ t37, t45 = t42 ^ t41;
    const uint32_t z0 = t44 & y15, z1 = t37 & y6, z2 = t33 & x7, z3 = t43 & y16, z4 = t40 & y1;
    const uint32_t z5 = t29 & y7, z6 = t42 & y11, z7 = t45 & y17, z8 = t41 & y10, z9 = t44 & y12;
    const uint32_t z10 = t37 & y3, z11 = t33 & y4, z12 = t43 & y13, z13 = t40 & y5, z14 = t29 & y2;
    const uint32_t z15 = t42 & y9, z16 = t45 & y14, z17 = t41 & y8;
    // bottom linear layer
    const uint32_t t46 = z15 ^ z16, t47 = z10 ^ z11, t48 = z5 ^ z13, t49 = z9 ^ z10, t50 = z2 ^ z12;
    const uint32_t t51 = z2 ^ z5, t52 = z7 ^ z8, t53 = z0 ^ z3, t54 = z6 ^ z7, t55 = z16 ^ z17;
    const uint32_t t56 = z12 ^ t48, t57 = t50 ^ t53, t58 = z4 ^ t46, t59 = z3 ^ t54, t60 = t46 ^ t57;
    const uint32_t t61 = z14 ^ t57, t62 = t52 ^ t58, t63 = t49 ^ t58, t64 = z4 ^ t59, t65 = t61 ^ t62;
    const uint32_t t66 = z1 ^ t63;
    const uint32_t s0 = t59 ^ t63, s6 = t56 ^ ~t62, s7 = t48 ^ ~t60, t67 = t64 ^ t65;
    const uint32_t s3 = t53 ^ t66, s4 = t51 ^ t66, s5 = t47 ^ t65, s1 = t64 ^ ~s3, s2 = t55 ^ ~t67;
    q[7] = s0; q[6] = s1; q[5] = s2; q[4] = s3; q[3] = s4; q[2] = s5; q[1] = s6; q[0] = s7;
}

// One full round on st[128] (SubBytes, ShiftRows, MixColumns, AddRoundKey
// with the masks k[128]); LAST: no MixColumns.  ShiftRows is folded into the
// indexing: output column c row r takes input byte (column (c + r) mod 4, row r).
template <bool LAST>
QPP_BS_HD void round(uint32_t *st, const uint32_t *k)
{
    // output column by output column: its four input bytes (one per row,
    // ShiftRows) go through the S-box and MixColumns and are dead after, so
    // at most one column of outputs and the remaining inputs are live
    uint32_t o[128];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t *a[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            a[r] = st + 8 * (4 * ((c + r) & 3) + r);
            sbox(a[r]);
            QPP_BS_FENCE();
        }
        if (LAST) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int b = 0; b < 8; ++b) o[8 * (4 * c + r) + b] = a[r][b] ^ k[8 * (4 * c + r) + b];
            continue;
        }
        // out_r = 2 a_r ^ 3 a_{r+1} ^ a_{r+2} ^ a_{r+3}
        //       = a_r ^ t ^ xtime(a_r ^ a_{r+1}),  t = a_0 ^ a_1 ^ a_2 ^ a_3
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t *x = a[r], *y = a[(r + 1) & 3], *z = a[(r + 2) & 3], *w = a[(r + 3) & 3];
            uint32_t u[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) u[b] = x[b] ^ y[b];
            // xtime(u): bit b <- u[b-1], plus u[7] into bits 0, 1, 3, 4 (x^8 = x^4+x^3+x+1)
            uint32_t xt[8];
            xt[0] = u[7];
            xt[1] = u[0] ^ u[7];
            xt[2] = u[1];
            xt[3] = u[2] ^ u[7];
            xt[4] = u[3] ^ u[7];
            xt[5] = u[4];
            xt[6] = u[5];
            xt[7] = u[6];
#pragma unroll
            for (int b = 0; b < 8; ++b)
                o[8 * (4 * c + r) + b] = xt[b] ^ y[b] ^ z[b] ^ w[b] ^ k[8 * (4 * c + r) + b];
        }
        QPP_BS_FENCE();
    }
#pragma unroll
    for (int j = 0; j < 128; ++j) st[j] = o[j];
}

// AES-NR encryption of the 32 blocks in st (planes), round-key masks
// km[(NR + 1) * 128] (round r at km + 128 r).
template <int NR>
QPP_BS_HD void encrypt(uint32_t *st, const uint32_t *km)
{
#pragma unroll
    for (int j = 0; j < 128; ++j) st[j] ^= km[j];
#pragma unroll 1
    for (int r = 1; r < NR; ++r) round<false>(st, km + 128 * r);
    round<true>(st, km + 128 * NR);
}

// In-place transpose of the 32 x 32 bit matrix r[i] bit j <-> r[j] bit i
// (slot-major words <-> bit planes).  Five SWAPMOVE stages.
QPP_BS_HD void transpose32(uint32_t *r)
{
    const uint32_t m[5] = {0x0000ffffu, 0x00ff00ffu, 0x0f0f0f0fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int w = 16 >> s;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (i & w) continue;
            const uint32_t t = ((r[i] >> w) ^ r[i + w]) & m[s];
            r[i + w] ^= t;
            r[i] ^= t << w;
        }
    }
}

// 32 blocks (blk[s] = 4 little-endian words of slot s's 16 bytes) <-> planes
// st[8 i + b] (bit b of byte i).  Word k of the block holds bytes 4k..4k+3, so
// transposing the k-th words of the 32 slots yields planes 32k..32k+31.
QPP_BS_HD void to_planes(const uint32_t (*blk)[4], uint32_t *st)
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int s = 0; s < 32; ++s) st[32 * k + s] = blk[s][k];
        transpose32(st + 32 * k);
    }
}

QPP_BS_HD void from_planes(uint32_t *st, uint32_t (*blk)[4])
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        transpose32(st + 32 * k);
#pragma unroll
        for (int s = 0; s < 32; ++s) blk[s][k] = st[32 * k + s];
    }
}

// Round-key masks of an expanded AES key (little-endian words rk[4 (NR + 1)],
// word w of round r = bytes 4w..4w+3 of that round key): km[128 r + 8 i + b] =
// bit b of byte i, spread to 0 or ~0.
QPP_BS_HD void key_masks(const uint32_t *rk, int nr, uint32_t *km)
{
    for (int r = 0; r <= nr; ++r)
        for (int i = 0; i < 16; ++i)
            for (int b = 0; b < 8; ++b)
                km[128 * r + 8 * i + b] = ((rk[4 * r + (i >> 2)] >> (8 * (i & 3) + b)) & 1u) ? ~0u : 0u;
}

// ---- the production form: generated bitop3 columns, keys folded in ------

// Words of the bitsliced key table of one expanded key (rk as in key_masks):
// rounds 1..NR, each 4 output columns x 4 rows x kKeyWordsPerSbox scalar words
// (the S-box input key of that output position = round key r - 1 at the
// ShiftRows source byte), then the last round's own key bits, 4 x 4 x 8.
constexpr int kBsRoundWords = 16 * kKeyWordsPerSbox;
QPP_BS_HD constexpr int bs_key_words(int nr) { return nr * kBsRoundWords + 128; }

QPP_BS_HD void key_table(const uint32_t *rk, int nr, uint32_t *kt)
{
    auto bit = [&](int r, int byte, int b) -> uint32_t {
        return ((rk[4 * r + (byte >> 2)] >> (8 * (byte & 3) + b)) & 1u) ? ~0u : 0u;
    };
    for (int r = 1; r <= nr; ++r)
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row) {
                const int src = 4 * ((c + row) & 3) + row;  // ShiftRows source byte
                uint32_t *w = kt + (r - 1) * kBsRoundWords + (4 * c + row) * kKeyWordsPerSbox;
                // x_i = bit 7 - i; order of tools/lutmap.py KEY_WORDS
                auto x = [&](int i) { return bit(r - 1, src, 7 - i); };
                const uint32_t v[12] = {x(3) ^ x(5), x(0) ^ x(6), x(0) ^ x(3), x(0) ^ x(5), x(1) ^ x(2),
                                        x(0), x(1), x(3), x(4), x(5), x(6), x(7)};
                for (int j = 0; j < 12; ++j) w[j] = v[j];
            }
    uint32_t *last = kt + nr * kBsRoundWords;
    for (int c = 0; c < 4; ++c)
        for (int row = 0; row < 4; ++row)
            for (int b = 0; b < 8; ++b) last[8 * (4 * c + row) + b] = bit(nr, 4 * c + row, b);
}

// AES-NR of the 32 blocks in st (planes, in place) with the key table kt.
template <bool LAST>
QPP_BS_HD void round_gen(uint32_t *st, const uint32_t *rkw, const uint32_t *last_key)
{
    uint32_t o[4][4][8];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t a[4][8];
#pragma unroll
        for (int row = 0; row < 4; ++row)
#pragma unroll
            for (int b = 0; b < 8; ++b) a[row][b] = st[8 * (4 * ((c + row) & 3) + row) + b];
        if (LAST) column_last(a, rkw + 48 * c, last_key + 32 * c, o[c]);
        else column(a, rkw + 48 * c, o[c]);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int row = 0; row < 4; ++row)
#pragma unroll
            for (int b = 0; b < 8; ++b) st[8 * (4 * c + row) + b] = o[c][row][b];
}

template <int NR>
QPP_BS_HD void encrypt_gen(uint32_t *st, const uint32_t *kt)
{
#pragma unroll 1
    for (int r = 1; r < NR; ++r) round_gen<false>(st, kt + (r - 1) * kBsRoundWords, nullptr);
    round_gen<true>(st, kt + (NR - 1) * kBsRoundWords, kt + NR * kBsRoundWords);
}

}  // namespace bs
}  // namespace qpp
