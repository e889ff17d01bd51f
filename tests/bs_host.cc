// Host build of tools/bitslice/qpp_bitslice.h for the CPU unit test
// (tests/test_bitslice.py): 32 blocks per call through the bitsliced path.
#include <stdint.h>
#include <string.h>

#include "../tools/bitslice/qpp_bitslice.h"

namespace {

uint8_t gmul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

// S-box through the bitsliced circuit itself (slot s of plane b = bit b of s)
void sbox_table(uint8_t *t)
{
    for (int base = 0; base < 256; base += 32) {
        uint32_t q[8] = {0};
        for (int s = 0; s < 32; ++s)
            for (int b = 0; b < 8; ++b)
                if (((base + s) >> b) & 1) q[b] |= 1u << s;
        qpp::bs::sbox(q);
        for (int s = 0; s < 32; ++s) {
            int y = 0;
            for (int b = 0; b < 8; ++b) y |= (int)((q[b] >> s) & 1) << b;
            t[base + s] = (uint8_t)y;
        }
    }
}

// FIPS-197 sec. 5.2, little-endian words
int expand(const uint8_t *key, int klen, uint32_t *rk)
{
    uint8_t sb[256];
    sbox_table(sb);
    const int nk = klen / 4, nr = nk + 6;
    for (int i = 0; i < nk; ++i) memcpy(&rk[i], key + 4 * i, 4);
    uint8_t rcon = 1;
    for (int i = nk; i < 4 * (nr + 1); ++i) {
        uint32_t t = rk[i - 1];
        auto sub = [&](uint32_t v) {
            return (uint32_t)sb[v & 255] | (uint32_t)sb[(v >> 8) & 255] << 8 |
                   (uint32_t)sb[(v >> 16) & 255] << 16 | (uint32_t)sb[v >> 24] << 24;
        };
        if (i % nk == 0) {
            t = sub((t >> 8) | (t << 24)) ^ rcon;
            rcon = gmul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = sub(t);
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return nr;
}

}  // namespace

extern "C" {

void qpp_test_bs_sbox(uint8_t *out256) { sbox_table(out256); }

// AES-128/256 of 32 blocks (in/out: 32 x 16 bytes) through the bitsliced path
int qpp_test_bs_encrypt(const uint8_t *key, int klen, const uint8_t *in, uint8_t *out)
{
    uint32_t rk[60], km[15 * 128], st[128], blk[32][4];
    const int nr = expand(key, klen, rk);
    qpp::bs::key_masks(rk, nr, km);
    memcpy(blk, in, sizeof blk);
    qpp::bs::to_planes(blk, st);
    if (nr == 10) qpp::bs::encrypt<10>(st, km);
    else qpp::bs::encrypt<14>(st, km);
    qpp::bs::from_planes(st, blk);
    memcpy(out, blk, sizeof blk);
    return nr;
}

// the generated bitop3 round columns (qpp_bs_gen.h) with the folded key table
int qpp_test_bs_encrypt_gen(const uint8_t *key, int klen, const uint8_t *in, uint8_t *out)
{
    uint32_t rk[60], kt[qpp::bs::bs_key_words(14)], st[128], blk[32][4];
    const int nr = expand(key, klen, rk);
    qpp::bs::key_table(rk, nr, kt);
    memcpy(blk, in, sizeof blk);
    qpp::bs::to_planes(blk, st);
    if (nr == 10) qpp::bs::encrypt_gen<10>(st, kt);
    else qpp::bs::encrypt_gen<14>(st, kt);
    qpp::bs::from_planes(st, blk);
    memcpy(out, blk, sizeof blk);
    return nr;
}

// to_planes then from_planes: identity
void qpp_test_bs_transpose_roundtrip(const uint8_t *in, uint8_t *out)
{
    uint32_t st[128], blk[32][4];
    memcpy(blk, in, sizeof blk);
    qpp::bs::to_planes(blk, st);
    qpp::bs::from_planes(st, blk);
    memcpy(out, blk, sizeof blk);
}

}
