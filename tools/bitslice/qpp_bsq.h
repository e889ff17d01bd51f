// qpp_bsq.h -- quad-bitsliced AES-CTR keystream for the GCM step loop.
//
// The T-table form (qpp_device.h aes_ctr2) spends ~4.2 LDS-array cycles per
// block and leaves VALU issue half idle; this form computes the same eight
// counter blocks of a quad step (two per lane) in VALU logic, so a share of
// the steps can move off the LDS array.
//
// Layout ("row in lane"): the quad's eight blocks j = lane + 4 * slot are held
// as eight 32-bit bit planes per lane.  Lane L holds state row L: plane b,
// byte c, bit j = bit b of state byte (row L, column c) of block j.  Then
//   SubBytes   = the Boyar-Peralta circuit on the 8 planes (qpp_bsq_sbox.h),
//   ShiftRows  = rotate lane L's planes right by 8 L bits (one v_alignbit),
//   MixColumns = rows from the quad neighbours by DPP (two xors per plane),
//   AddRoundKey = xor with the lane's row of the round key, spread to planes
// and every step of a round serves all eight blocks.  Rounds 1-2 come from the
// packet's counter cache by T-table (10 lookups per lane, as aes_ctr2), so the
// planes start at round 3; transposing in and out costs a 4x4 byte transpose
// per block, a 4x4 word transpose across the quad and an 8x8 bit transpose of
// each byte column.
//
// Round-key planes (bsq_key_planes): rounds 3..NR, 128 bytes per round,
// word [r - 3][L][b] = for each column c, byte c = 0xff if bit b of round-key
// byte (row L, column c) is set.  AES itself follows FIPS-197.
#pragma once

#include "../../aioquic_amd/csrc/qpp_device.h"

#define QPP_BSQ_HD __device__ __forceinline__
#define QPP_BSQ_LUT3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))
#include "qpp_bsq_sbox.h"

namespace qpp {
namespace bsq {

constexpr int kRoundPlaneBytes = 128;  // 4 rows x 8 planes x 4 bytes
// key-plane bytes of a slot (rounds 3..NR)
constexpr int key_plane_bytes(int nr) { return (nr - 2) * kRoundPlaneBytes; }

// A quad DPP move the compiler folds into the VALU instruction that consumes
// it (v_xor_b32_dpp, v_cndmask_b32_dpp): update_dpp with bound_ctrl, where a
// plain mov_dpp stays a separate v_mov_b32_dpp.  Every lane of the quad is
// active, so bound_ctrl never applies.
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}

// (x & ~m) | (y & m)
__device__ __forceinline__ uint32_t sel(uint32_t x, uint32_t y, uint32_t m)
{
    return __builtin_amdgcn_bitop3_b32(x, y, m, 0xd8);
}

// 4x4 byte transpose within a lane: w[c] byte r -> w[r] byte c (columns of a
// block <-> its rows).  An involution.
__device__ __forceinline__ void byte_t4(uint32_t &w0, uint32_t &w1, uint32_t &w2, uint32_t &w3)
{
    // perm(S0, S1, sel): selector bytes 0-3 pick S1's bytes, 4-7 S0's
    const uint32_t lo01 = __builtin_amdgcn_perm(w1, w0, 0x06020400u);  // w0.0 w1.0 w0.2 w1.2
    const uint32_t hi01 = __builtin_amdgcn_perm(w1, w0, 0x07030501u);  // w0.1 w1.1 w0.3 w1.3
    const uint32_t lo23 = __builtin_amdgcn_perm(w3, w2, 0x06020400u);
    const uint32_t hi23 = __builtin_amdgcn_perm(w3, w2, 0x07030501u);
    w0 = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);  // w0.0 w1.0 w2.0 w3.0
    w2 = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);  // w0.2 w1.2 w2.2 w3.2
    w1 = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
    w3 = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
}

// 4x4 word transpose across the quad: lane L's x[j] <- lane j's x[L].  Two
// exchange stages (lane ^ 1, lane ^ 2), each lane sending the word its
// partner keeps.  An involution.
__device__ __forceinline__ void quad_t4(uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3, bool odd, bool hi)
{
    {
        const uint32_t r = qperm<kQuadSwap1>(odd ? x0 : x1);
        x0 = odd ? r : x0;
        x1 = odd ? x1 : r;
    }
    {
        const uint32_t r = qperm<kQuadSwap1>(odd ? x2 : x3);
        x2 = odd ? r : x2;
        x3 = odd ? x3 : r;
    }
    {
        const uint32_t r = qperm<kQuadSwap2>(hi ? x0 : x2);
        x0 = hi ? r : x0;
        x2 = hi ? x2 : r;
    }
    {
        const uint32_t r = qperm<kQuadSwap2>(hi ? x1 : x3);
        x1 = hi ? r : x1;
        x3 = hi ? x3 : r;
    }
}

// 8x8 bit transpose in every byte column of w[0..7]: bit b of byte c of w[j]
// <-> bit j of byte c of w[b].  Three SWAPMOVE stages, each swap two shifts
// and two v_bitop3 selects.  An involution.
template <int S>
__device__ __forceinline__ void swapmove(uint32_t &a, uint32_t &b)
{
    constexpr uint32_t m = S == 4 ? 0x0f0f0f0fu : S == 2 ? 0x33333333u : 0x55555555u;
    const uint32_t na = sel(a, b << S, m << S);
    const uint32_t nb = sel(b, a >> S, m);
    a = na;
    b = nb;
}
__device__ __forceinline__ void bit_t8(uint32_t (&w)[8])
{
#pragma unroll
    for (int j = 0; j < 4; ++j) swapmove<4>(w[j], w[j + 4]);
    swapmove<2>(w[0], w[2]);
    swapmove<2>(w[1], w[3]);
    swapmove<2>(w[4], w[6]);
    swapmove<2>(w[5], w[7]);
#pragma unroll
    for (int j = 0; j < 8; j += 2) swapmove<1>(w[j], w[j + 1]);
}

// Eight counter-cached blocks of the quad's packet to planes and back.  In:
// lane s holds the round-2 states of blocks s (a) and s + 4 (b) as column
// words.  Out: the same lanes hold the blocks' keystream.
__device__ __forceinline__ void to_planes(const uint32_t (&a)[4], const uint32_t (&b)[4], uint32_t (&p)[8],
                                          bool odd, bool hi)
{
    uint32_t x0 = a[0], x1 = a[1], x2 = a[2], x3 = a[3];
    uint32_t y0 = b[0], y1 = b[1], y2 = b[2], y3 = b[3];
    byte_t4(x0, x1, x2, x3);  // rows of block s
    byte_t4(y0, y1, y2, y3);
    quad_t4(x0, x1, x2, x3, odd, hi);  // row L of blocks 0..3
    quad_t4(y0, y1, y2, y3, odd, hi);  // row L of blocks 4..7
    p[0] = x0; p[1] = x1; p[2] = x2; p[3] = x3;
    p[4] = y0; p[5] = y1; p[6] = y2; p[7] = y3;
    bit_t8(p);  // p[b] = plane b
}

__device__ __forceinline__ void from_planes(uint32_t (&p)[8], u32x4 &o0, u32x4 &o1, bool odd, bool hi)
{
    bit_t8(p);  // p[j] = row L of block j
    uint32_t x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
    uint32_t y0 = p[4], y1 = p[5], y2 = p[6], y3 = p[7];
    quad_t4(x0, x1, x2, x3, odd, hi);  // rows of block s
    quad_t4(y0, y1, y2, y3, odd, hi);  // rows of block s + 4
    byte_t4(x0, x1, x2, x3);           // columns
    byte_t4(y0, y1, y2, y3);
    o0 = u32x4{x0, x1, x2, x3};
    o1 = u32x4{y0, y1, y2, y3};
}

// One full round on the planes: SubBytes, ShiftRows (sr = 8 L), MixColumns
// (out_r = a_r ^ t ^ xtime(a_r ^ a_{r+1}), t = a_0 ^ a_1 ^ a_2 ^ a_3, rows
// r + 1 and r + 2 from the quad neighbours), AddRoundKey (k: the lane's row).
__device__ __forceinline__ void round_mid(uint32_t (&p)[8], const uint32_t (&k)[8], uint32_t sr)
{
    constexpr int kNext1 = 0x39;  // lane j <- lane j + 1 (row r + 1)
    constexpr int kNext2 = 0x4E;  // lane j <- lane j + 2
    sbox(p);
    uint32_t u[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        p[b] = __builtin_amdgcn_alignbit(p[b], p[b], sr);
        u[b] = p[b] ^ qperm<kNext1>(p[b]);
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint32_t t = u[b] ^ qperm<kNext2>(u[b]);
        const uint32_t pk = xor3(p[b], t, k[b]);
        // xtime: bit b <- bit b - 1, bit 7 into bits 0, 1, 3, 4
        if (b == 0) p[b] = pk ^ u[7];
        else if (b == 1 || b == 3 || b == 4) p[b] = xor3(pk, u[b - 1], u[7]);
        else p[b] = pk ^ u[b - 1];
    }
}

__device__ __forceinline__ void round_last(uint32_t (&p)[8], const uint32_t (&k)[8], uint32_t sr)
{
    sbox(p);
#pragma unroll
    for (int b = 0; b < 8; ++b) p[b] = __builtin_amdgcn_alignbit(p[b], p[b], sr) ^ k[b];
}

// The lane's key planes of round r (3 <= r <= NR) from LDS.
__device__ __forceinline__ void load_key(const uint8_t *kp, int r, uint32_t row, uint32_t (&k)[8])
{
    const u32x4 *q = (const u32x4 *)(kp + (r - 3) * kRoundPlaneBytes + row * 32);
    const u32x4 k0 = q[0], k1 = q[1];
    k[0] = k0.x; k[1] = k0.y; k[2] = k0.z; k[3] = k0.w;
    k[4] = k1.x; k[5] = k1.y; k[6] = k1.z; k[7] = k1.w;
}

// Rounds 3..NR of the eight blocks in planes.
template <int NR>
__device__ __forceinline__ void rounds(uint32_t (&p)[8], const uint8_t *kp, uint32_t row)
{
    const uint32_t sr = 8u * row;
#pragma unroll 1
    for (int r = 3; r < NR; ++r) {
        uint32_t k[8];
        load_key(kp, r, row, k);
        round_mid(p, k, sr);
    }
    uint32_t k[8];
    load_key(kp, NR, row, k);
    round_last(p, k, sr);
}

// Rounds 3..NR of two independent plane sets (16 blocks per quad): twice the
// instruction-level parallelism per wave for the same key loads.
template <int NR>
__device__ __forceinline__ void rounds2(uint32_t (&p)[8], uint32_t (&q)[8], const uint8_t *kp, uint32_t row)
{
    const uint32_t sr = 8u * row;
#pragma unroll 1
    for (int r = 3; r < NR; ++r) {
        uint32_t k[8];
        load_key(kp, r, row, k);
        round_mid(p, k, sr);
        round_mid(q, k, sr);
    }
    uint32_t k[8];
    load_key(kp, NR, row, k);
    round_last(p, k, sr);
    round_last(q, k, sr);
}

// rounds 1-2 of two counter blocks by T-table (aes_ctr2's first two phases)
template <class TE>
__device__ __forceinline__ void ctr_r2(const CtrCache &c, uint32_t cb0, uint32_t cb1, const uint32_t *rk,
                                       const TE &T, uint32_t (&a)[4], uint32_t (&b)[4])
{
    const uint32_t x0 = T.t3(rk[3] ^ (cb0 << 24)), x1 = T.t3(rk[3] ^ (cb1 << 24));
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t u0 = c.c0 ^ x0, u1 = c.c0 ^ x1;
    const uint32_t v0 = T.t0(u0), v1 = T.t3(u0), v2 = T.t2(u0), v3 = T.t1(u0);
    const uint32_t w0 = T.t0(u1), w1 = T.t3(u1), w2 = T.t2(u1), w3 = T.t1(u1);
    __builtin_amdgcn_sched_barrier(0);
    a[0] = c.d0 ^ v0; a[1] = c.d1 ^ v1; a[2] = c.d2 ^ v2; a[3] = c.d3 ^ v3;
    b[0] = c.d0 ^ w0; b[1] = c.d1 ^ w1; b[2] = c.d2 ^ w2; b[3] = c.d3 ^ w3;
}

}  // namespace bsq

// Sixteen blocks of the quad's packet, four per lane (two aes_ctr2 calls'
// worth: (cb0, cb1) and (cb2, cb3)), as two plane sets walked together.
template <int NR, class TE>
__device__ __forceinline__ void bsq_ctr4(const CtrCache &c, uint32_t cb0, uint32_t cb1, uint32_t cb2, uint32_t cb3,
                                         const uint32_t *rk, const TE &T, const uint8_t *kp, uint32_t sub,
                                         u32x4 &o0, u32x4 &o1, u32x4 &o2, u32x4 &o3)
{
    uint32_t a[4], b[4], e[4], f[4];
    bsq::ctr_r2(c, cb0, cb1, rk, T, a, b);
    bsq::ctr_r2(c, cb2, cb3, rk, T, e, f);
    const bool odd = (sub & 1) != 0, hi = (sub & 2) != 0;
    uint32_t p[8], q[8];
    bsq::to_planes(a, b, p, odd, hi);
    bsq::to_planes(e, f, q, odd, hi);
    bsq::rounds2<NR>(p, q, kp, sub);
    bsq::from_planes(p, o0, o1, odd, hi);
    bsq::from_planes(q, o2, o3, odd, hi);
}

// E_K of the quad's eight counter blocks, two per lane (cb0: block sub,
// cb1: block sub + 4), from the packet's counter cache: the same result as
// aes_ctr2 on every lane.  Every lane of the quad must be active and hold the
// same packet (cache and keys).  kp: the slot's key planes in LDS.
template <int NR, class TE>
__device__ __forceinline__ void bsq_ctr2(const CtrCache &c, uint32_t cb0, uint32_t cb1, const uint32_t *rk,
                                         const TE &T, const uint8_t *kp, uint32_t sub, u32x4 &o0, u32x4 &o1)
{
    // rounds 1-2 by T-table (aes_ctr2's first two phases)
    const uint32_t x0 = T.t3(rk[3] ^ (cb0 << 24)), x1 = T.t3(rk[3] ^ (cb1 << 24));
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t u0 = c.c0 ^ x0, u1 = c.c0 ^ x1;
    const uint32_t v0 = T.t0(u0), v1 = T.t3(u0), v2 = T.t2(u0), v3 = T.t1(u0);
    const uint32_t w0 = T.t0(u1), w1 = T.t3(u1), w2 = T.t2(u1), w3 = T.t1(u1);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t a[4] = {c.d0 ^ v0, c.d1 ^ v1, c.d2 ^ v2, c.d3 ^ v3};
    const uint32_t b[4] = {c.d0 ^ w0, c.d1 ^ w1, c.d2 ^ w2, c.d3 ^ w3};
    const bool odd = (sub & 1) != 0, hi = (sub & 2) != 0;
    uint32_t p[8];
    bsq::to_planes(a, b, p, odd, hi);
    bsq::rounds<NR>(p, kp, sub);
    bsq::from_planes(p, o0, o1, odd, hi);
}

}  // namespace qpp
