/*
 * qpp_oracle.c -- CPU ORACLE for the QUIC packet-protection hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (aioquic_amd/, the HIP
 * library, the CPython extension) links, loads or calls this file.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker.
 *
 * It is a plain-C restatement of what the reference computes per packet:
 *   - aioquic src/aioquic/_crypto.c      AEAD_encrypt        :157-194
 *                                        AEAD_decrypt        :115-155
 *                                        HeaderProtection_mask  :278-287
 *                                        HeaderProtection_apply :289-319
 *                                        HeaderProtection_remove:321-350
 *   - aioquic src/aioquic/quic/crypto.py CryptoContext.encrypt_packet :105-116
 *                                        CryptoContext.decrypt_packet :75-103
 *   - aioquic src/aioquic/quic/packet.py decode_packet_number :118-132
 * The cipher arithmetic itself lives in OpenSSL libcrypto (third-party, not in
 * /root/reference; wheels pin OpenSSL 3.5.4, scripts/fetch-vendor.json:2).  It
 * is restated here from the published standards:
 *   AES            FIPS-197
 *   GCM / GHASH    NIST SP 800-38D (96-bit IV: J0 = IV || 0^31 || 1)
 *   ChaCha20, Poly1305, ChaCha20-Poly1305 AEAD   RFC 8439
 *   Header protection  RFC 9001 sec. 5.4.3 (AES-ECB) and 5.4.4 (ChaCha20)
 *
 * Parity is PINNED: tests/test_oracle.py checks this file against the RFC 9001
 * and RFC 9369 Appendix-A vectors (as carried by the reference's
 * tests/test_crypto_v1.py / test_crypto_v2.py) and against golden vectors that
 * tests/golden/make_golden.py generated with the reference's own _crypto.c
 * compiled from /root/reference (oracle/Makefile, target `ref`).
 *
 * Written for clarity, not speed: byte-wise AES, bit-serial GHASH.
 */
#include <stdint.h>
#include <string.h>

#include "qpp_oracle.h"

/* ------------------------------------------------------------------ AES -- */

static uint8_t g_sbox[256];
static int g_sbox_ready = 0;

static uint8_t gf8_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

/* FIPS-197 sec. 5.1.1: multiplicative inverse in GF(2^8) followed by the affine map. */
static void sbox_init(void)
{
    if (g_sbox_ready) return;
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; ++y)
                if (gf8_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        }
        uint8_t s = inv;
        for (int i = 1; i <= 4; ++i) s ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
        g_sbox[x] = (uint8_t)(s ^ 0x63);
    }
    g_sbox_ready = 1;
}

/* FIPS-197 sec. 5.2 key expansion; rk holds 4*(nr+1) big-endian words. */
int qo_aes_expand(const uint8_t *key, int key_len, uint32_t *rk)
{
    sbox_init();
    int nk = key_len / 4;
    if (key_len != 16 && key_len != 32) return -1;
    int nr = nk + 6;
    for (int i = 0; i < nk; ++i)
        rk[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 |
                (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
    uint8_t rcon = 1;
    for (int i = nk; i < 4 * (nr + 1); ++i) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = (t << 8) | (t >> 24);
            t = (uint32_t)g_sbox[t >> 24] << 24 | (uint32_t)g_sbox[(t >> 16) & 255] << 16 |
                (uint32_t)g_sbox[(t >> 8) & 255] << 8 | g_sbox[t & 255];
            t ^= (uint32_t)rcon << 24;
            rcon = gf8_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t)g_sbox[t >> 24] << 24 | (uint32_t)g_sbox[(t >> 16) & 255] << 16 |
                (uint32_t)g_sbox[(t >> 8) & 255] << 8 | g_sbox[t & 255];
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return nr;
}

/* FIPS-197 sec. 5.1 cipher, state as a column-major byte array. */
void qo_aes_block(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16])
{
    uint8_t s[16], t[16];
    memcpy(s, in, 16);
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) s[4 * c + r] ^= (uint8_t)(rk[c] >> (24 - 8 * r));
    for (int round = 1; round <= nr; ++round) {
        for (int i = 0; i < 16; ++i) s[i] = g_sbox[s[i]];                 /* SubBytes  */
        for (int c = 0; c < 4; ++c)                                         /* ShiftRows */
            for (int r = 0; r < 4; ++r) t[4 * c + r] = s[4 * ((c + r) & 3) + r];
        if (round != nr) {                                                  /* MixColumns */
            for (int c = 0; c < 4; ++c) {
                uint8_t *a = &t[4 * c];
                uint8_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
                a[0] = (uint8_t)(gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3);
                a[1] = (uint8_t)(a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3);
                a[2] = (uint8_t)(a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3));
                a[3] = (uint8_t)(gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2));
            }
        }
        for (int c = 0; c < 4; ++c)                                         /* AddRoundKey */
            for (int r = 0; r < 4; ++r)
                s[4 * c + r] = t[4 * c + r] ^ (uint8_t)(rk[4 * round + c] >> (24 - 8 * r));
    }
    memcpy(out, s, 16);
}

/* ----------------------------------------------------------- GCM / GHASH -- */

/* SP 800-38D Algorithm 1: X * Y in GF(2^128), bit 0 = MSB of byte 0. */
static void gf128_mul(uint8_t x[16], const uint8_t y[16])
{
    uint8_t z[16] = {0}, v[16];
    memcpy(v, y, 16);
    for (int i = 0; i < 128; ++i) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int k = 0; k < 16; ++k) z[k] ^= v[k];
        int lsb = v[15] & 1;
        for (int k = 15; k > 0; --k) v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xe1;
    }
    memcpy(x, z, 16);
}

static void ghash_update(uint8_t y[16], const uint8_t h[16], const uint8_t *p, size_t n)
{
    while (n) {
        size_t k = n < 16 ? n : 16;
        for (size_t i = 0; i < k; ++i) y[i] ^= p[i];
        gf128_mul(y, h);
        p += k;
        n -= k;
    }
}

static void inc32(uint8_t ctr[16])
{
    for (int i = 15; i >= 12; --i)
        if (++ctr[i]) break;
}

static void gcm_core(const uint8_t *key, int key_len, const uint8_t nonce[12],
                     const uint8_t *aad, size_t alen, const uint8_t *in, size_t len,
                     uint8_t *out, uint8_t tag[16], int decrypt)
{
    uint32_t rk[60];
    int nr = qo_aes_expand(key, key_len, rk);
    uint8_t h[16] = {0}, j0[16], ctr[16], ks[16], y[16] = {0}, lens[16];
    qo_aes_block(rk, nr, h, h);
    memcpy(j0, nonce, 12);
    j0[12] = j0[13] = j0[14] = 0;
    j0[15] = 1;
    memcpy(ctr, j0, 16);
    ghash_update(y, h, aad, alen);
    /* GHASH runs over the ciphertext: input when decrypting, output when encrypting. */
    if (decrypt) ghash_update(y, h, in, len);
    for (size_t off = 0; off < len; off += 16) {
        inc32(ctr);
        qo_aes_block(rk, nr, ctr, ks);
        size_t k = len - off < 16 ? len - off : 16;
        for (size_t i = 0; i < k; ++i) out[off + i] = in[off + i] ^ ks[i];
    }
    if (!decrypt) ghash_update(y, h, out, len);
    uint64_t abits = (uint64_t)alen * 8, cbits = (uint64_t)len * 8;
    for (int i = 0; i < 8; ++i) {
        lens[i] = (uint8_t)(abits >> (56 - 8 * i));
        lens[8 + i] = (uint8_t)(cbits >> (56 - 8 * i));
    }
    ghash_update(y, h, lens, 16);
    qo_aes_block(rk, nr, j0, ks);
    for (int i = 0; i < 16; ++i) tag[i] = y[i] ^ ks[i];
}

/* ------------------------------------------------------ ChaCha20/Poly1305 -- */

static uint32_t rd32le(const uint8_t *p)
{
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

static uint64_t rd64le(const uint8_t *p) { return rd32le(p) | (uint64_t)rd32le(p + 4) << 32; }

static void wr32le(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

#define ROTL32(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QR(a, b, c, d)                                   \
    a += b; d ^= a; d = ROTL32(d, 16);                   \
    c += d; b ^= c; b = ROTL32(b, 12);                   \
    a += b; d ^= a; d = ROTL32(d, 8);                    \
    c += d; b ^= c; b = ROTL32(b, 7)

/* RFC 8439 sec. 2.3 */
void qo_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                       uint8_t out[64])
{
    uint32_t s[16], x[16];
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; ++i) s[4 + i] = rd32le(key + 4 * i);
    s[12] = counter;
    for (int i = 0; i < 3; ++i) s[13 + i] = rd32le(nonce + 4 * i);
    memcpy(x, s, sizeof x);
    for (int i = 0; i < 10; ++i) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) wr32le(out + 4 * i, x[i] + s[i]);
}

/* RFC 8439 sec. 2.5, radix 2^64 with a 2-bit top limb. */
typedef struct { uint64_t r0, r1, s0, s1, h0, h1, h2; } poly_t;

static void poly_init(poly_t *p, const uint8_t k[32])
{
    p->r0 = rd64le(k) & 0x0ffffffc0fffffffULL;
    p->r1 = rd64le(k + 8) & 0x0ffffffc0ffffffcULL;
    p->s0 = rd64le(k + 16);
    p->s1 = rd64le(k + 24);
    p->h0 = p->h1 = p->h2 = 0;
}

/* h = (h + m + 2^128) * r mod 2^130-5 for one full 16-byte block */
static void poly_block(poly_t *p, const uint8_t m[16])
{
    typedef unsigned __int128 u128;
    u128 t0 = (u128)p->h0 + rd64le(m);
    u128 t1 = (u128)p->h1 + rd64le(m + 8) + (uint64_t)(t0 >> 64);
    uint64_t h0 = (uint64_t)t0, h1 = (uint64_t)t1, h2 = p->h2 + (uint64_t)(t1 >> 64) + 1;
    uint64_t r0 = p->r0, r1 = p->r1, sr1 = r1 + (r1 >> 2); /* 5*r1/4, exact since r1%4==0 */
    /* h*r mod p with 2^130 == 5 folded into r1's contribution */
    u128 d0 = (u128)h0 * r0 + (u128)h1 * sr1;
    u128 d1 = (u128)h0 * r1 + (u128)h1 * r0 + (u128)h2 * sr1;
    uint64_t d2 = h2 * r0;
    d1 += (uint64_t)(d0 >> 64);
    d2 += (uint64_t)(d1 >> 64);
    h0 = (uint64_t)d0;
    h1 = (uint64_t)d1;
    /* partial reduction: d2 holds bits >= 128; keep 2 bits, fold the rest times 5 */
    uint64_t c = (d2 >> 2) + (d2 & ~3ULL); /* (d2>>2)*5 = (d2>>2) + (d2>>2)*4 */
    h2 = d2 & 3;
    u128 t = (u128)h0 + c;
    h0 = (uint64_t)t;
    t = (u128)h1 + (uint64_t)(t >> 64);
    h1 = (uint64_t)t;
    h2 += (uint64_t)(t >> 64);
    p->h0 = h0; p->h1 = h1; p->h2 = h2;
}

static void poly_finish(poly_t *p, uint8_t tag[16])
{
    typedef unsigned __int128 u128;
    /* full reduction: compute h + 5 - 2^130 and select */
    u128 t = (u128)p->h0 + 5;
    uint64_t g0 = (uint64_t)t;
    t = (u128)p->h1 + (uint64_t)(t >> 64);
    uint64_t g1 = (uint64_t)t;
    uint64_t g2 = p->h2 + (uint64_t)(t >> 64);
    uint64_t h0 = p->h0, h1 = p->h1;
    if (g2 >> 2) { h0 = g0; h1 = g1; }
    t = (u128)h0 + p->s0;
    h0 = (uint64_t)t;
    h1 = h1 + p->s1 + (uint64_t)(t >> 64);
    for (int i = 0; i < 8; ++i) {
        tag[i] = (uint8_t)(h0 >> (8 * i));
        tag[8 + i] = (uint8_t)(h1 >> (8 * i));
    }
}

static void poly_padded(poly_t *p, const uint8_t *d, size_t n)
{
    uint8_t blk[16];
    while (n) {
        size_t k = n < 16 ? n : 16;
        memset(blk, 0, 16);
        memcpy(blk, d, k);
        poly_block(p, blk);
        d += k;
        n -= k;
    }
}

/* RFC 8439 sec. 2.8 */
static void chachapoly_core(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                            size_t alen, const uint8_t *in, size_t len, uint8_t *out,
                            uint8_t tag[16], int decrypt)
{
    uint8_t blk[64], lens[16];
    poly_t p;
    qo_chacha20_block(key, 0, nonce, blk);
    poly_init(&p, blk);
    poly_padded(&p, aad, alen);
    if (decrypt) poly_padded(&p, in, len);
    for (size_t off = 0; off < len; off += 64) {
        qo_chacha20_block(key, (uint32_t)(1 + off / 64), nonce, blk);
        size_t k = len - off < 64 ? len - off : 64;
        for (size_t i = 0; i < k; ++i) out[off + i] = in[off + i] ^ blk[i];
    }
    if (!decrypt) poly_padded(&p, out, len);
    for (int i = 0; i < 8; ++i) {
        lens[i] = (uint8_t)((uint64_t)alen >> (8 * i));
        lens[8 + i] = (uint8_t)((uint64_t)len >> (8 * i));
    }
    poly_block(&p, lens);
    poly_finish(&p, tag);
}

/* ---------------------------------------------------------------- AEAD -- */

/* nonce = iv XOR big-endian pn in the low 8 bytes (_crypto.c:173-176) */
static void make_nonce(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12])
{
    memcpy(nonce, iv, 12);
    for (int i = 0; i < 8; ++i) nonce[11 - i] ^= (uint8_t)(pn >> (8 * i));
}

static int key_len_for(int suite)
{
    return suite == QO_AES_128_GCM ? 16 : 32;
}

/* AEAD.encrypt (_crypto.c:157-194): returns ct||tag length, or -1 */
long qo_aead_encrypt(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *data,
                     size_t len, const uint8_t *aad, size_t alen, uint64_t pn, uint8_t *out)
{
    uint8_t nonce[12];
    if (len > QO_PACKET_MAX) return -1;
    make_nonce(iv, pn, nonce);
    if (suite == QO_CHACHA20_POLY1305)
        chachapoly_core(key, nonce, aad, alen, data, len, out, out + len, 0);
    else
        gcm_core(key, key_len_for(suite), nonce, aad, alen, data, len, out, out + len, 0);
    return (long)len + 16;
}

/* AEAD.decrypt (_crypto.c:115-155): returns plaintext length, -1 bad length, -2 tag mismatch */
long qo_aead_decrypt(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *data,
                     size_t len, const uint8_t *aad, size_t alen, uint64_t pn, uint8_t *out)
{
    uint8_t nonce[12], tag[16];
    if (len < 16 || len > QO_PACKET_MAX) return -1;
    make_nonce(iv, pn, nonce);
    size_t clen = len - 16;
    if (suite == QO_CHACHA20_POLY1305)
        chachapoly_core(key, nonce, aad, alen, data, clen, out, tag, 1);
    else
        gcm_core(key, key_len_for(suite), nonce, aad, alen, data, clen, out, tag, 1);
    uint8_t diff = 0;
    for (int i = 0; i < 16; ++i) diff |= (uint8_t)(tag[i] ^ data[clen + i]);
    return diff ? -2 : (long)clen;
}

/* ---------------------------------------------------- header protection -- */

/* HeaderProtection_mask (_crypto.c:278-287) */
void qo_hp_mask(int suite, const uint8_t *hp_key, const uint8_t sample[16], uint8_t mask[16])
{
    if (suite == QO_CHACHA20_POLY1305) {
        uint8_t blk[64];
        qo_chacha20_block(hp_key, rd32le(sample), sample + 4, blk);
        memcpy(mask, blk, 16);
    } else {
        uint32_t rk[60];
        int nr = qo_aes_expand(hp_key, key_len_for(suite), rk);
        qo_aes_block(rk, nr, sample, mask);
    }
}

static uint8_t first_byte_mask(uint8_t b0) { return (b0 & 0x80) ? 0x0f : 0x1f; }

/* HeaderProtection.apply (_crypto.c:289-319); out = hdr || payload, masked. */
int qo_hp_apply(int suite, const uint8_t *hp_key, const uint8_t *hdr, size_t hlen,
                const uint8_t *payload, size_t plen, uint8_t *out)
{
    if (hlen < 1) return -1;
    int pn_len = (hdr[0] & 3) + 1;
    if ((size_t)pn_len > hlen || plen < (size_t)(20 - pn_len)) return -1;
    size_t pn_off = hlen - pn_len;
    uint8_t mask[16];
    qo_hp_mask(suite, hp_key, payload + 4 - pn_len, mask);
    memmove(out + hlen, payload, plen);
    memmove(out, hdr, hlen);
    out[0] ^= mask[0] & first_byte_mask(out[0]);
    for (int i = 0; i < pn_len; ++i) out[pn_off + i] ^= mask[1 + i];
    return 0;
}

/* HeaderProtection.remove (_crypto.c:321-350).  Writes the unmasked header
 * (pn_off + pn_len bytes) to hdr_out; returns the header length, -1 if the
 * sample does not fit.  *pn_trunc gets the truncated packet number. */
int qo_hp_remove(int suite, const uint8_t *hp_key, const uint8_t *pkt, size_t len,
                 size_t pn_off, uint8_t *hdr_out, uint32_t *pn_trunc)
{
    if (pn_off + 20 > len || pn_off < 1) return -1;
    uint8_t mask[16];
    qo_hp_mask(suite, hp_key, pkt + pn_off + 4, mask);
    memcpy(hdr_out, pkt, pn_off + 4);
    hdr_out[0] ^= mask[0] & first_byte_mask(hdr_out[0]);
    int pn_len = (hdr_out[0] & 3) + 1;
    uint32_t t = 0;
    for (int i = 0; i < pn_len; ++i) {
        hdr_out[pn_off + i] ^= mask[1 + i];
        t = (t << 8) | hdr_out[pn_off + i];
    }
    *pn_trunc = t;
    return (int)(pn_off + pn_len);
}

/* decode_packet_number (quic/packet.py:118-132, RFC 9000 App. A.3), with
 * Python's unbounded-int semantics.  `truncated` is what the reference feeds it:
 * HeaderProtection.remove returns the truncated number through the "i" format
 * (_crypto.c:349), so a 4-byte value >= 2^31 arrives NEGATIVE.  The result is
 * reduced mod 2^64 the way AEAD.decrypt's "K" format does (_crypto.c:123). */
uint64_t qo_decode_pn(int64_t truncated, int num_bits, uint64_t expected)
{
    typedef __int128 i128;
    i128 window = (i128)1 << num_bits;
    i128 half = window / 2;
    i128 exp = (i128)expected;
    i128 candidate = (exp & ~(window - 1)) | (i128)truncated;
    if (candidate <= exp - half && candidate < ((i128)1 << 62) - window)
        return (uint64_t)(candidate + window);
    if (candidate > exp + half && candidate >= window) return (uint64_t)(candidate - window);
    return (uint64_t)candidate;
}

/* the value HeaderProtection.remove hands to Python ("i" of a uint32, _crypto.c:349) */
int64_t qo_pn_trunc_as_int(uint32_t t) { return (int64_t)(int32_t)t; }

/* --------------------------------------------------- packet protection -- */

/* CryptoContext.encrypt_packet (quic/crypto.py:105-116): out = protected packet */
long qo_protect(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp_key,
                const uint8_t *hdr, size_t hlen, const uint8_t *payload, size_t plen,
                uint64_t pn, uint8_t *out)
{
    /* the reference's defined domain: AEAD.encrypt's output fits buffer[1500]
     * (_crypto.c:168-171,193) and HeaderProtection.apply copies header ||
     * payload into buffer[1500] (_crypto.c:305-306); beyond that it overruns */
    if (plen > QO_PACKET_MAX - 16 || hlen + plen + 16 > QO_PACKET_MAX) return -1;
    long n = qo_aead_encrypt(suite, key, iv, payload, plen, hdr, hlen, pn, out + hlen);
    if (n < 0) return -1;
    if (qo_hp_apply(suite, hp_key, hdr, hlen, out + hlen, (size_t)n, out) != 0) return -1;
    return (long)hlen + n;
}

/* CryptoContext.decrypt_packet (quic/crypto.py:75-103), without the key-phase
 * switch: the caller passes the key it wants used.  Returns the payload length
 * or a negative QO_E_* code; fills header (out), payload (out + *hdr_len). */
/* rfc_pn != 0: the truncated number decodes unsigned (RFC 9000 App. A.3, the
 * algorithm of packet.py:118-132 without the int32 hand-over of _crypto.c:349),
 * as the product's QPP_F_RFC_PN flag asks (include/quic_pp.h) */
long qo_unprotect_ex(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp_key,
                     const uint8_t *pkt, size_t len, size_t pn_off, uint64_t expected_pn,
                     uint8_t *out, size_t *hdr_len, uint64_t *pn, int rfc_pn)
{
    uint32_t trunc;
    int h = qo_hp_remove(suite, hp_key, pkt, len, pn_off, out, &trunc);
    if (h < 0) return QO_E_LENGTH;
    int pn_len = (out[0] & 3) + 1;
    *pn = qo_decode_pn(rfc_pn ? (int64_t)trunc : qo_pn_trunc_as_int(trunc), pn_len * 8, expected_pn);
    *hdr_len = (size_t)h;
    long r = qo_aead_decrypt(suite, key, iv, pkt + h, len - h, out, (size_t)h, *pn, out + h);
    if (r == -1) return QO_E_LENGTH;
    if (r == -2) return QO_E_DECRYPT;
    return r;
}

long qo_unprotect(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp_key,
                  const uint8_t *pkt, size_t len, size_t pn_off, uint64_t expected_pn,
                  uint8_t *out, size_t *hdr_len, uint64_t *pn)
{
    return qo_unprotect_ex(suite, key, iv, hp_key, pkt, len, pn_off, expected_pn, out, hdr_len, pn, 0);
}

/* ------------------------------------------------------------ batch forms -- */
#include "../include/quic_pp.h"

static int slot_ok(const qpp_key_material *keys, uint32_t n_keys, uint32_t slot)
{
    return slot < n_keys && keys[slot].suite <= QPP_CHACHA20_POLY1305;
}

void qo_protect_batch(const qpp_key_material *keys, uint32_t n_keys, const qpp_desc *desc,
                      uint32_t n, const uint8_t *in, uint8_t *out, qpp_result *res)
{
    for (uint32_t i = 0; i < n; ++i) {
        const qpp_desc *d = &desc[i];
        qpp_result *r = &res[i];
        r->pn = d->pn;
        r->hdr_len = d->hdr_len;
        r->out_len = 0;
        if (!slot_ok(keys, n_keys, d->slot)) { r->status = QPP_S_NO_KEY; continue; }
        const qpp_key_material *k = &keys[d->slot];
        const uint8_t *hdr = in + d->in_off, *pl = hdr + d->hdr_len;
        uint8_t *o = out + d->out_off;
        long m;
        if (d->flags & QPP_F_NO_HP) {
            memmove(o, hdr, d->hdr_len);
            m = qo_aead_encrypt(k->suite, k->key, k->iv, pl, d->len, hdr, d->hdr_len, d->pn,
                                o + d->hdr_len);
            if (m >= 0) m += d->hdr_len;
        } else {
            m = qo_protect(k->suite, k->key, k->iv, k->hp, hdr, d->hdr_len, pl, d->len, d->pn, o);
        }
        r->status = m < 0 ? QPP_S_LENGTH : QPP_S_OK;
        r->out_len = m < 0 ? 0 : (uint32_t)m;
    }
}

void qo_unprotect_batch(const qpp_key_material *keys, uint32_t n_keys, const qpp_desc *desc,
                        uint32_t n, const uint8_t *in, uint8_t *out, qpp_result *res)
{
    for (uint32_t i = 0; i < n; ++i) {
        const qpp_desc *d = &desc[i];
        qpp_result *r = &res[i];
        r->pn = d->pn;
        r->hdr_len = 0;
        r->out_len = 0;
        if (!slot_ok(keys, n_keys, d->slot)) { r->status = QPP_S_NO_KEY; continue; }
        const qpp_key_material *k = &keys[d->slot];
        const uint8_t *p = in + d->in_off;
        uint8_t *o = out + d->out_off;
        long m;
        if (d->flags & QPP_F_NO_HP) {
            if (d->len < d->hdr_len) { r->status = QPP_S_LENGTH; continue; }
            memmove(o, p, d->hdr_len);
            m = qo_aead_decrypt(k->suite, k->key, k->iv, p + d->hdr_len, d->len - d->hdr_len, p,
                                d->hdr_len, d->pn, o + d->hdr_len);
            r->hdr_len = d->hdr_len;
            if (m == -1) m = QO_E_LENGTH;
            else if (m == -2) m = QO_E_DECRYPT;
            else m += d->hdr_len; /* out_len counts the copied AAD, as for protect */
        } else {
            /* key-phase check needs the unmasked first byte: remove HP first */
            uint8_t hdr[QPP_MAX_HDR + 4];
            uint32_t trunc;
            if (d->hdr_len > QPP_MAX_HDR - 4 ||
                qo_hp_remove(k->suite, k->hp, p, d->len, d->hdr_len, hdr, &trunc) < 0) {
                r->status = QPP_S_LENGTH;
                continue;
            }
            if (!(hdr[0] & 0x80) && ((hdr[0] >> 2) & 1) != k->key_phase) {
                int pn_len = (hdr[0] & 3) + 1;
                r->pn = qo_decode_pn((d->flags & QPP_F_RFC_PN) ? (int64_t)trunc : qo_pn_trunc_as_int(trunc),
                                     8 * pn_len, d->pn);
                r->hdr_len = (uint16_t)(d->hdr_len + pn_len);
                r->status = QPP_S_KEY_PHASE;
                continue;
            }
            size_t hl;
            uint64_t pn;
            m = qo_unprotect_ex(k->suite, k->key, k->iv, k->hp, p, d->len, d->hdr_len, d->pn, o, &hl,
                                &pn, (d->flags & QPP_F_RFC_PN) != 0);
            r->pn = pn;
            r->hdr_len = (uint16_t)hl;
            if (m >= 0) m += (long)hl;
        }
        if (m == QO_E_LENGTH) r->status = QPP_S_LENGTH;
        else if (m == QO_E_DECRYPT) r->status = QPP_S_DECRYPT;
        else { r->status = QPP_S_OK; r->out_len = (uint32_t)m; }
    }
}
