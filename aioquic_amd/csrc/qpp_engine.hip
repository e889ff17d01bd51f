// qpp_engine.hip -- MI355X (gfx950) QUIC packet-protection kernels.
//
// Replaces aioquic's per-packet path (src/aioquic/_crypto.c AEAD_encrypt :157,
// AEAD_decrypt :115, HeaderProtection_apply :289 / remove :321 / mask :278, and
// quic/crypto.py CryptoContext.encrypt_packet :105 / decrypt_packet :75) with
// batched kernels.  Design:
//   * 4 lanes per packet ("quad"), 64 packets per 256-thread workgroup.
//     Lane j of a quad owns GHASH/CTR blocks v = 4k + j at step k, where the
//     block sequence [AAD | CT | lengths] is front-padded to a multiple of 4.
//     AES-CTR of block v and its GHASH term live in the same lane, so no data
//     moves between lanes until the final 2-step DPP xor of the tag.
//   * GHASH: Horner with H^4 per lane, H^(4-j) on the last step; products via
//     4-bit windowed tables (32 windows x 16 entries x 16 B per power, 32 KiB
//     for H^1..H^4) in LDS.  Every lane reads window w of the same table at
//     once and a window is exactly one 256-byte LDS bank row: conflict-free.
//   * AES: Te0 replicated 32x in LDS (lane l reads bank l&31: conflict-free),
//     round keys in SGPRs (a workgroup works key slot by key slot).
//   * ChaCha20-Poly1305: lane j owns 64-byte chunks c = 4k + j; Poly1305 by
//     per-lane Horner (r per block, r^12 more between chunks) and one DPP sum.
//   * No MFMA: the work is byte/bit arithmetic, bound by LDS and VALU issue.
#include <hip/hip_runtime.h>

#include "qpp_chacha.h"
#include "qpp_gf128.h"
#include "qpp_device.h"
#include "qpp_hkdf.h"
#include "qpp_internal.h"

namespace qpp {

__constant__ AesTables c_aes = kAesTables;

// GCM: a workgroup shares one 64 KiB AES image and its GHASH table entries;
// one 1024-thread workgroup per CU, or two of 512 (launch_packets), at 4
// waves per SIMD (128 VGPRs) either way.
// ChaCha20-Poly1305 needs no tables.  4 lanes per packet in every case.
constexpr int kSetupWG = 256;
// Per-packet LDS scratch of the ChaCha20-Poly1305 kernel (the GCM kernel
// keeps nothing of a packet in LDS): [0, 32) ct[0..32) (+ tag) for the
// protect HP sample; [48, 64) the Poly1305 one-time key's s half; [64, 96)
// the parked packet view; [96, 112) input bytes [0, 16) (the first header
// block) for the header write.
constexpr int kScratch = 112;
constexpr int kScrEj0 = 48, kScrPark = 64, kScrHdr = 96;
constexpr uint32_t kNoSlot = 0xffffffffu;
// Descriptor flag set by the host session for a descriptor whose extents do
// not fit the caller's buffers: the packet reports QPP_S_LENGTH and no byte
// of it is read or written.
constexpr uint32_t kFlagReject = 0x8000u;
// ChaCha20-Poly1305: minimum waves per SIMD (4: 128 VGPRs, 8 spilled; r2i
// same box against 1 (146 VGPRs, 3 waves): 64 Ki +4 %, 1 Mi +1 %, config 5 +1 %)
constexpr int kChachaWpe = 4;

// ChaCha20-Poly1305 per-wave LDS staging: at step k a quad works on 4
// consecutive 64-byte chunks of its packet (lane j: chunk 4k - 1 + j).  Its
// loads and stores run coalesced, chunk by chunk (instruction t: lane j moves
// 16-byte block j of chunk 4k - 1 + t), through 4 regions of 64 x 16 bytes
// (region t: instruction t's LDS-DMA destination / store source), each padded
// by 16 bytes so that a quad's 4 lanes reading one chunk hit distinct banks.
constexpr int kChRegion = 64 * 16 + 16;
constexpr int kChStage = 4 * kChRegion;

// pw entries: 1, r, r^2 .. r^5, r^8, r^13 .. r^16
#ifndef QPP_CH_POLY4
#define QPP_CH_POLY4 1  // study switch: 0 = one Horner multiply (and carry) per Poly1305 block
#endif
#ifndef QPP_CH_DPP_T
#define QPP_CH_DPP_T 0  // study switch: one-round launches transpose a step's output blocks by DPP
#endif
#ifndef QPP_CH_DIRECT_ST
#define QPP_CH_DIRECT_ST 0  // study switch: 1 = each lane stores its own blocks (no LDS round trip back)
#endif
#ifndef QPP_CH_CARRY_AT
#define QPP_CH_CARRY_AT 7  // study switch: the double round after which the chunk sum is carried
#endif
constexpr int kPwOne = 0, kPw1 = 1, kPw8 = 6, kPw13 = 7, kPwEntries = QPP_CH_POLY4 ? 11 : 7;

template <int WG>
struct __attribute__((aligned(16))) ChachaSmem {
    uint8_t stage[WG / 64][kChStage];
    uint8_t scratch[WG / 4][kScratch];
    uint32_t pw[WG / 4][5 * kPwEntries];  // per packet: the tag close's powers of r (5 limbs each)
};

// Fill the LDS AES image: row x = [Te0[x] x 32 | Te1[x] x 32], 16-byte stores.
// Every thread's table reads are issued before the first LDS store, so the
// fill costs one memory round trip, not one per 16-byte store per thread.
template <int NT>
__device__ __forceinline__ void load_te(uint8_t *te)
{
    constexpr int kIters = (256 * 16 + NT - 1) / NT;
    uint32_t v0[kIters];
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
        const int i = (int)threadIdx.x + k * NT;
        v0[k] = i < 256 * 16 ? c_aes.te0[i >> 4] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
        const int i = (int)threadIdx.x + k * NT;
        if (i < 256 * 16) {
            const int x = i >> 4, part = i & 15;
            const uint32_t v = part < 8 ? v0[k] : rotl(v0[k], 8);
            *(u32x4 *)(te + x * 256 + part * 16) = u32x4{v, v, v, v};
        }
    }
}

// ------------------------------------------------------- packet numbers --

// decode_packet_number (quic/packet.py:118-132).  Bit-exact with the
// reference, which receives the truncated number from HeaderProtection.remove
// as a SIGNED int (_crypto.c:349): a 4-byte value >= 2^31 is negative there.
__device__ __forceinline__ uint64_t decode_pn(uint32_t trunc, int pn_len, uint64_t expected,
                                              bool rfc)
{
    if (pn_len == 4 && trunc >= 0x80000000u && !rfc)
        return expected >= (uint64_t)trunc - 0x80000000ull ? (uint64_t)trunc
                                                            : (0xffffffff00000000ull | trunc);
    const uint64_t window = 1ull << (8 * pn_len), half = window >> 1;
    const uint64_t cand = (expected & ~(window - 1)) | trunc;
    if (expected >= half && cand <= expected - half && cand < (1ull << 62) - window)
        return cand + window;
    if (cand > expected + half && cand >= window) return cand - window;
    return cand;
}

// XOR pattern that (un)masks header bytes [base, base+16): first byte with
// mask[0] & (0x0f long / 0x1f short), packet number bytes with mask[1..pn_len]
// (_crypto.c:308-316, :337-347).
__device__ __forceinline__ u32x4 hp_pattern(int base, u32x4 mask, uint32_t fb_mask, int pn_off,
                                            int pn_len)
{
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int pos = base + j, q = pos - pn_off;
        uint32_t m = 0;
        if (pos == 0) m = byte_of(mask, 0) & fb_mask;
        if (q >= 0 && q < pn_len) m = byte_of(mask, 1 + q);
        w[j >> 2] |= m << (8 * (j & 3));
    }
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ uint32_t first_byte_mask(uint32_t b0) { return (b0 & 0x80) ? 0x0f : 0x1f; }

// 16 bytes at byte offset s (0..3) of an LDS scratch line
__device__ __forceinline__ u32x4 lds_sample(const uint8_t *scr, int s)
{
    const uint32_t *w = (const uint32_t *)scr;
    uint32_t a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
    return u32x4{__builtin_amdgcn_alignbyte(b, a, s), __builtin_amdgcn_alignbyte(c, b, s),
                 __builtin_amdgcn_alignbyte(d, c, s), __builtin_amdgcn_alignbyte(e, d, s)};
}

// HeaderProtection_mask (_crypto.c:278-287): AES-ECB(hp, sample), or the
// first ChaCha20 block with counter = sample[0:4] and nonce = sample[4:16].
// The same, computed jointly by a packet's quad (every lane holds the same
// sample): ChaCha20 and AES by columns across the quad.
template <int SUITE, class TE>
__device__ __forceinline__ u32x4 hp_mask_quad(const KeySlot *ks, u32x4 sample, const TE &T, int sub)
{
    if constexpr (SUITE == QPP_CHACHA20_POLY1305)
        return chacha_block_quad_row0(ks->hrk, sample.x, sample.y, sample.z, sample.w, sub);
    else
        return aes_encrypt_quad<SUITE == QPP_AES_256_GCM ? 14 : 10>(sample, ks->hrk, T, sub);
}

template <int SUITE, class TE>
__device__ __forceinline__ u32x4 hp_mask_of(const KeySlot *ks, u32x4 sample, const TE &T)
{
    if constexpr (SUITE == QPP_CHACHA20_POLY1305) {
        uint32_t blk[16];
        chacha_block(ks->hrk, sample.x, sample.y, sample.z, sample.w, blk);
        return u32x4{blk[0], blk[1], blk[2], blk[3]};
    } else {
        return aes_encrypt<SUITE == QPP_AES_256_GCM ? 14 : 10>(sample, ks->hrk, T);
    }
}

template <class TE>
__device__ __forceinline__ u32x4 hp_mask_any(const KeySlot *ks, uint32_t suite, u32x4 sample,
                                             const TE &T)
{
    if (suite == QPP_CHACHA20_POLY1305) return hp_mask_of<QPP_CHACHA20_POLY1305>(ks, sample, T);
    if (suite == QPP_AES_256_GCM) return hp_mask_of<QPP_AES_256_GCM>(ks, sample, T);
    return hp_mask_of<QPP_AES_128_GCM>(ks, sample, T);
}

// -------------------------------------------------------- per-packet view --

struct Pkt {
    const uint8_t *src;
    uint8_t *dst;
    int hlen, clen;         // header/AAD length, ciphertext length
    int pn_off, pn_len;
    uint32_t fbm;           // first-byte mask bits
    uint32_t status;
    uint64_t pn;
    bool hp;
    u32x4 mask;             // header-protection mask (unprotect: known up front)
    u32x4 nonce;            // iv ^ pn, with word 3 = 0
};

// Header analysis shared by both suites.  Unprotect removes header
// protection here (it decides the header length and the packet number).
// Header bytes that header protection needs, requested with the descriptor
// (before the key slot is known): byte 0 and, for unprotect, the packet-number
// bytes and the sample.  Reads only what pkt_begin's length checks allow.
struct HdrPre {
    u32x4 h0;        // input bytes [0, 16) when the readable region holds them
    u32x4 pnw, smp;  // unprotect: packet-number bytes, sample
    uint32_t b0;
};

template <bool ENC>
__device__ __forceinline__ HdrPre prefetch_hdr(const qpp_desc &d, const uint8_t *gin, bool valid)
{
    HdrPre r = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, 0};
    if (!valid || (d.flags & kFlagReject)) return r;
    const uint8_t *src = gin + d.in_off;
    const bool hp = !(d.flags & QPP_F_NO_HP) && d.hdr_len >= 1;
    const uint64_t region = ENC ? (uint64_t)d.hdr_len + d.len : (uint64_t)d.len;
    if (region >= 16) {
        r.h0 = ld16(src);
        r.b0 = r.h0.x & 0xff;
    } else if (hp) {
        r.b0 = src[0];
    }
    if (!ENC && hp && (int)d.hdr_len + 20 <= (int)d.len && d.hdr_len <= QPP_MAX_HDR - 4) {
        r.pnw = ld16(src + d.hdr_len);
        r.smp = ld16(src + d.hdr_len + 4);
    }
    return r;
}

template <bool ENC, int SUITE, class TE>
__device__ __forceinline__ Pkt pkt_begin(const qpp_desc &d, const HdrPre &pre, const uint8_t *gin,
                                         uint8_t *gout, const KeySlot *ks, const TE &T)
{
    Pkt P;
    P.src = gin + d.in_off;
    P.dst = gout + d.out_off;
    P.hp = !(d.flags & QPP_F_NO_HP);
    P.status = QPP_S_OK;
    P.pn = d.pn;
    P.mask = u32x4{0, 0, 0, 0};
    P.pn_off = 0;
    P.pn_len = 0;
    P.fbm = 0;
    P.hlen = 0;
    P.clen = 0;
    if (d.flags & kFlagReject) {
        P.status = QPP_S_LENGTH;
    } else if (ENC) {
        P.hlen = d.hdr_len;
        P.clen = (int)d.len;
        if (P.clen > QPP_PACKET_MAX || P.hlen > QPP_MAX_HDR) P.status = QPP_S_LENGTH;
        if (P.hp) {
            // CryptoContext.encrypt_packet -> HeaderProtection.apply (_crypto.c:298-302)
            if (P.hlen < 1) {
                P.status = QPP_S_LENGTH;
            } else {
                const uint32_t b0 = pre.b0;
                P.pn_len = (int)(b0 & 3) + 1;
                P.pn_off = P.hlen - P.pn_len;
                P.fbm = first_byte_mask(b0);
                // defined domain of the reference: AEAD.encrypt output fits
                // buffer[1500] (_crypto.c:168-171,193) and apply's header ||
                // payload copy fits buffer[1500] (_crypto.c:305-306)
                if (P.pn_off < 0 || P.clen + QPP_TAG_LEN < 20 - P.pn_len ||
                    P.hlen + P.clen + QPP_TAG_LEN > QPP_PACKET_MAX)
                    P.status = QPP_S_LENGTH;
            }
        }
    } else if (P.hp) {
        // HeaderProtection.remove (_crypto.c:321-350) + decode (crypto.py:84-89)
        P.pn_off = d.hdr_len;
        const int len = (int)d.len;
        if (P.pn_off < 1 || P.pn_off + 20 > len || P.pn_off > QPP_MAX_HDR - 4) {
            P.status = QPP_S_LENGTH;
        } else {
            P.mask = hp_mask_quad<SUITE>(ks, pre.smp, T, (int)(lane_fresh() & 3));
            uint32_t b0 = pre.b0;
            P.fbm = first_byte_mask(b0);
            b0 ^= byte_of(P.mask, 0) & P.fbm;
            P.pn_len = (int)(b0 & 3) + 1;
            uint32_t trunc = 0;
            for (int i = 0; i < P.pn_len; ++i)
                trunc = (trunc << 8) | (byte_of(pre.pnw, i) ^ byte_of(P.mask, 1 + i));
            P.pn = decode_pn(trunc, P.pn_len, d.pn, d.flags & QPP_F_RFC_PN);
            P.hlen = P.pn_off + P.pn_len;
            const int body = len - P.hlen;
            if (body < QPP_TAG_LEN || body > QPP_PACKET_MAX) P.status = QPP_S_LENGTH;
            else if (!(b0 & 0x80) && ((b0 >> 2) & 1) != ks->key_phase) P.status = QPP_S_KEY_PHASE;
            P.clen = body - QPP_TAG_LEN;
        }
    } else {
        // AEAD.decrypt (_crypto.c:115-155): data = in[hdr_len:len]
        P.hlen = d.hdr_len;
        const int body = (int)d.len - P.hlen;
        if (P.hlen > QPP_MAX_HDR || body < QPP_TAG_LEN || body > QPP_PACKET_MAX)
            P.status = QPP_S_LENGTH;
        P.clen = body - QPP_TAG_LEN;
    }
    // nonce = iv ^ (pn as big-endian in the last 8 bytes) (_crypto.c:173-176)
    P.nonce = u32x4{ks->iv[0], ks->iv[1] ^ bswap((uint32_t)(P.pn >> 32)),
                    ks->iv[2] ^ bswap((uint32_t)P.pn), 0};
    return P;
}

// 128-bit little-endian shift right by s bytes (0..15)
__device__ __forceinline__ u32x4 shr_bytes(u32x4 v, int s)
{
    uint64_t lo = (uint64_t)v.y << 32 | v.x, hi = (uint64_t)v.w << 32 | v.z;
    if (s >= 8) {
        lo = hi >> (8 * (s - 8));
        hi = 0;
    } else if (s > 0) {
        lo = (lo >> (8 * s)) | (hi << (64 - 8 * s));
        hi >>= 8 * s;
    }
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

// 128-bit little-endian shift left by s bytes (0..15)
__device__ __forceinline__ u32x4 shl_bytes(u32x4 v, int s)
{
    uint64_t lo = (uint64_t)v.y << 32 | v.x, hi = (uint64_t)v.w << 32 | v.z;
    if (s >= 8) {
        hi = lo << (8 * (s - 8));
        lo = 0;
    } else if (s > 0) {
        hi = (hi << (8 * s)) | (lo >> (64 - 8 * s));
        lo <<= 8 * s;
    }
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

// n (0..16) bytes at p, zero padded, by one 16-byte load: [lo, hi) is
// readable (a packet's region).  A block near the region's end is loaded
// end-aligned and shifted down, so no byte loop (one memory round trip per
// byte) runs; regions under 16 bytes take ld_part.
__device__ __forceinline__ u32x4 ld_win(const uint8_t *p, int n, const uint8_t *lo, const uint8_t *hi)
{
    if (n >= 16) return ld16(p);
    if (hi - lo < 16) return ld_part(p, n);
    const uint8_t *a = (p + 16 <= hi) ? p : hi - 16;
    return keep_bytes(shr_bytes(ld16(a), (int)(p - a)), n);
}

// Protect: header protection over the finished (ct||tag) and the header write.
template <int SUITE, class TE>
__device__ __forceinline__ void protect_finish_hp(Pkt &P, const KeySlot *ks, int sub,
                                                  uint8_t *scr, u32x4 tag, const TE &T,
                                                  const uint8_t *h0 = nullptr)
{
    // sample = (ct||tag)[4-pn_len : 20-pn_len]; the tag only matters when clen < 20
    if (P.clen < 32 && sub == 0) {
        for (int j = 0; j < 16 && P.clen + j < 32; ++j)
            scr[P.clen + j] = (uint8_t)byte_of(tag, j);
    }
    __builtin_amdgcn_wave_barrier();
    const u32x4 sample = lds_sample(scr, 4 - P.pn_len);
    P.mask = hp_mask_quad<SUITE>(ks, sample, T, sub);
    const int n_a = (P.hlen + 15) >> 4;
    for (int q = sub; q < n_a; q += 4) {
        const int nb = min(16, P.hlen - 16 * q);
        u32x4 h = (q == 0 && h0) ? *(const u32x4 *)h0 : ld_win(P.src + 16 * q, nb, P.src, P.src + P.hlen + P.clen);
        h ^= hp_pattern(16 * q, P.mask, P.fbm, P.pn_off, P.pn_len);
        st_part(P.dst + 16 * q, h, nb);
    }
}

// Header out: the plain header (unprotect), or the input header with the HP
// mask applied (protect).  Outside the step loop; byte tails allowed here.
// h0: the input's first 16 bytes already in LDS (or null: read them).
// rlen: the readable input region (header + payload, + tag for unprotect).
__device__ __forceinline__ void write_header(const Pkt &P, int sub, bool masked, int rlen,
                                             const uint8_t *h0 = nullptr)
{
    const int n_a = (P.hlen + 15) >> 4;
    for (int q = sub; q < n_a; q += 4) {
        const int nb = min(16, P.hlen - 16 * q);
        u32x4 h = (q == 0 && h0) ? *(const u32x4 *)h0 : ld_win(P.src + 16 * q, nb, P.src, P.src + rlen);
        if (masked) h ^= hp_pattern(16 * q, P.mask, P.fbm, P.pn_off, P.pn_len);
        st_part(P.dst + 16 * q, h, nb);
    }
}

// A packet whose tag does not verify leaves no plaintext behind: its quad
// overwrites the payload it streamed out with zeros (quic_pp.h, Authentication
// failures).  Runs only on the failure path.  Each 16-byte block is cleared
// by the lane that wrote it (own(i) = that lane), so the zeros land after the
// plaintext in that lane's program order.
template <class OWN>
__device__ __forceinline__ void wipe_payload(const Pkt &P, int sub, OWN own)
{
    uint8_t *o = P.dst + P.hlen;
    for (int i = 0; 16 * i < P.clen; ++i)
        if (own(i) == sub) {
            // made here: a zero the compiler hoists to the kernel's entry is
            // held (or spilled) across everything before this rare path
            u32x4 z = {0, 0, 0, 0};
            asm volatile("" : "+v"(z));
            st_part(o + 16 * i, z, min(16, P.clen - 16 * i));
        }
}

// Buffer descriptors over the whole input / output buffers.  Offsets at or
// above kOob are out of range: loads return zeros, stores are dropped.  This
// lets every step issue exactly one load and one store per lane with no
// branch around them, so the compiler can count vmcnt instead of draining.
constexpr uint32_t kBufBytes = 0xffffff00u;
constexpr uint32_t kOob = 0xfffffff0u;

struct Bufs {
    __amdgpu_buffer_rsrc_t in, out;
};

// --------------------------------------------------------------- AES-GCM --

// Phase times per wave (tools/probe.hip builds with -DQPP_PROBE): each mark
// adds the 100 MHz s_memrealtime ticks since the wave's previous mark to
// g_probe[wave][i] (slot kProbeItems counts items; kProbeStart / kProbeEnd
// hold the wave's first and last timestamps).
#ifdef QPP_PROBE
constexpr int kProbeSlots = 16, kProbeItems = 12, kProbeStart = 13, kProbeEnd = 14;
constexpr uint32_t kProbeWaves = 8192;  // waves recorded
__device__ unsigned long long g_probe[kProbeWaves * kProbeSlots];
__device__ __forceinline__ unsigned long long *probe_marks()
{
    __shared__ unsigned long long m[16];
    return m;
}
__device__ __forceinline__ void probe_mark(int i)
{
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const uint32_t wl = threadIdx.x >> 6, w = blockIdx.x * (blockDim.x / 64) + wl;
    if (w < kProbeWaves && __lane_id() == __ffsll((long long)__ballot(1)) - 1) {
        unsigned long long *m = probe_marks();
        unsigned long long *g = g_probe + (size_t)w * kProbeSlots;
        if (i == kProbeStart) g[kProbeStart] = t;
        else atomicAdd(&g[i], t - m[wl]);
        g[kProbeEnd] = t;
        m[wl] = t;
    }
}
#define QPP_PROBE_AT(i) probe_mark(i)
#define QPP_PROBE_COUNT()                                                                     \
    do {                                                                                      \
        const uint32_t w_ = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);              \
        if (w_ < kProbeWaves && __lane_id() == __ffsll((long long)__ballot(1)) - 1)           \
            atomicAdd(&g_probe[(size_t)w_ * kProbeSlots + kProbeItems], 1ull);                \
    } while (0)
#else
#define QPP_PROBE_COUNT() ((void)0)
#define QPP_PROBE_AT(i) ((void)0)
#endif

// Per-packet state that the ChaCha20-Poly1305 slot loop does not touch waits
// in LDS (scratch [64, 96)) while the loop runs, so the loop keeps its VGPRs.
// mask = false: the HP mask is not parked (a protect computes it after the
// payload; unpark then returns zeros), so no zero vector is held for it
__device__ __forceinline__ void park(const Pkt &P, uint8_t *scr, bool mask = true)
{
    if (mask) *(u32x4 *)(scr + kScrPark) = P.mask;
    *(u32x4 *)(scr + kScrPark + 16) =
        u32x4{(uint32_t)P.pn, (uint32_t)(P.pn >> 32),
              P.fbm | (uint32_t)P.pn_off << 8 | (uint32_t)P.pn_len << 24 | (uint32_t)P.hp << 28,
              (uint32_t)P.hlen | (uint32_t)P.clen << 16};
}
__device__ __forceinline__ Pkt unpark(const uint8_t *scr, const uint8_t *src, uint8_t *dst, bool mask = true)
{
    Pkt P;
    const u32x4 w = *(const u32x4 *)(scr + kScrPark + 16);
    P.src = src;
    P.dst = dst;
    P.hlen = (int)(w.w & 0xffff);
    P.clen = (int)(w.w >> 16);
    P.mask = mask ? *(const u32x4 *)(scr + kScrPark) : zero4();
    P.pn = (uint64_t)w.y << 32 | w.x;
    P.fbm = w.z & 0xff;
    P.pn_off = (int)((w.z >> 8) & 0xffff);
    P.pn_len = (int)((w.z >> 24) & 0xf);
    P.hp = (w.z >> 28) & 1;
    P.status = QPP_S_OK;
    P.nonce = u32x4{0, 0, 0, 0};
    return P;
}

// GHASH tables of a GCM packet's key slot: the step loop's H^4 from one of
// the workgroup's LDS table entries, the few other powers from the slot's
// tables in global memory (gcm_packet).  The wave's slot and entry live in
// LDS, re-read where needed rather than kept in SGPRs.
// Workgroup-shared bookkeeping words in LDS, read and written as relaxed
// workgroup-scope atomics: volatile accesses through generic pointers compile
// to flat instructions, and a flat load waits for the vector memory counter
// too (behind the item's outstanding stores), where an LDS load waits only
// for LDS.
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct GhashTabs {
    const uint8_t *lds;     // LDS table entries
    const uint8_t *gtab;    // every slot's tables, global memory
    const uint32_t *wslot;  // LDS: the wave's key slot
    const uint32_t *went;   // LDS: the wave's table entry
    __device__ __forceinline__ uint32_t t4() const
    {
        return __builtin_amdgcn_readfirstlane(lds_ld(went)) * (uint32_t)kGhLdsEntry;
    }
    // the slot's table of H^(pw + 1) in global memory
    __device__ __forceinline__ const uint8_t *global(uint32_t pw) const
    {
        const uint32_t s = __builtin_amdgcn_readfirstlane(lds_ld(wslot));
        return gtab + (size_t)s * kGhashTabBytes + pw * (uint32_t)kGhashPowBytes;
    }
};

// Sequence positions per quad step: BPL blocks per lane.  Lane j owns the
// positions v = j (mod 4) in either form; with BPL = 2 a step covers two of
// them (8 contiguous blocks per quad: two AES chains per lane in one set of
// LDS round trips, and 128 contiguous output bytes per quad step).
template <int BPL>
__device__ __forceinline__ int gcm_pad(int n_g)
{
    constexpr int QS = 4 * BPL;
    return QS * ((n_g + QS - 1) / QS) - n_g;
}

// Protect with header protection: the HP sample lies in CT blocks 0 and 1
// (sample = ct[4-pn_len, 20-pn_len), _crypto.c:302).  When both blocks are
// written by the quad's first step (BPL = 2: positions q = pad + za and
// q + 1 within the first 8) and the sample lies inside the ciphertext, the
// quad takes them by DPP in that step, computes the mask and writes the
// header there ("fast"); otherwise the sample is read back from the output
// after the step loop.
template <int BPL>
__device__ __forceinline__ bool gcm_fast_hp(int hlen, int clen)
{
    if constexpr (BPL != 2) {
        return false;
    } else {
        const int n_a = (hlen + 15) >> 4, n_c = (clen + 15) >> 4, za = n_a > 0 ? 1 : 0;
        return gcm_pad<BPL>(za + n_c + 1) + za <= 6 && clen >= 19;
    }
}

// n (0..15) bytes of v to buffer offset off (a partial tail block, stored by
// the lane that computed it inside the step loop).
__device__ __forceinline__ void buf_st_part(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v, int n)
{
    const int nd = n >> 2, rb = n & 3;
    if (nd > 0) __builtin_amdgcn_raw_buffer_store_b32(v.x, r, (int)off, 0, 0);
    if (nd > 1) __builtin_amdgcn_raw_buffer_store_b32(v.y, r, (int)off + 4, 0, 0);
    if (nd > 2) __builtin_amdgcn_raw_buffer_store_b32(v.z, r, (int)off + 8, 0, 0);
    if (rb) {
        uint32_t t = nd == 0 ? v.x : nd == 1 ? v.y : nd == 2 ? v.z : v.w;
        const int o = (int)off + 4 * nd;
        if (rb & 2) {
            __builtin_amdgcn_raw_buffer_store_b16((unsigned short)t, r, o, 0, 0);
            t >>= 16;
        }
        if (rb & 1) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)t, r, o + (rb & 2), 0, 0);
    }
}

// The header out, block q of it by lane q (mod 4): the input header with the
// HP mask applied (protect) or removed (unprotect), or as is (no HP).  h0 =
// the input's first 16 bytes (have_h0), other blocks are read from P.src.
__device__ __forceinline__ void write_header_v(const Pkt &P, int sub, bool masked, int rlen, u32x4 h0,
                                               bool have_h0)
{
    const int n_a = (P.hlen + 15) >> 4;
    for (int q = sub; q < n_a; q += 4) {
        const int nb = min(16, P.hlen - 16 * q);
        u32x4 h = (q == 0 && have_h0) ? h0 : ld_win(P.src + 16 * q, nb, P.src, P.src + rlen);
        if (masked) h ^= hp_pattern(16 * q, P.mask, P.fbm, P.pn_off, P.pn_len);
        st_part(P.dst + 16 * q, h, nb);
    }
}

// AES-GCM of one packet by its quad (SP 800-38D; _crypto.c:157-204 / :115-155).
//   * The associated data (header) is first folded to one block
//     Z = sum_g A_g H^(n_a-1-g) by every lane of the quad; GHASH is linear, so
//     Z then stands for the whole header as the first block of the sequence
//     [Z | CT | lengths] that the step loop walks (front-padded to 8S).
//   * Step k: lane `sub` owns blocks 8k+sub and 8k+4+sub: their AES-CTR
//     keystream (rounds 1-2 from the packet's counter cache), the register
//     prefetch of the next step's input, two buffer stores (dropped out of
//     range; a partial tail block is stored by its lane with byte stores), two
//     H^4 multiplies.
//   * Nothing of a packet waits in LDS: unprotect writes its header before the
//     loop (the mask is known), protect in its first step (gcm_fast_hp) or
//     after the loop; E_K(J0) stays in the lengths lane's registers.
// The input region holds >= 16 bytes except for tiny packets (< 16 bytes),
// whose input is loaded once by a partial load.  Returns the tag; got_tag =
// the received tag (unprotect).  Inside the step loop every lane-derived value
// is recomputed from lane_fresh(): at 128 VGPRs nothing else stays live.
// GHASH tables of the packet's key slot: the step loop multiplies by H^4 from
// one of the workgroup's LDS table entries; the few multiplies outside the
// loop (associated data beyond 16 bytes by H^1, each lane's closing H^(4-j))
// read the slot's tables in global memory.
// PRIO (k_gcm with 512-thread workgroups: launches of at most one item per
// wave): the step loop sets the wave's issue priority by its progress.
template <int NR, bool ENC, int BPL, int SUITE, bool PRIO>
__device__ __forceinline__ u32x4 gcm_packet(const Pkt &P, const KeySlot *ks, const u32x4 h0,
                                            const uint32_t *rk, int sub, const GhashTabs &G,
                                            const uint8_t *te, const Bufs &B, uint32_t ioff, uint32_t ooff,
                                            u32x4 &got_tag, uint32_t pbase = 0u)
{
    const LdsTe T{te, (lane_fresh() & 31) * 4};
    const int hlen = P.hlen, clen = P.clen;
    const int n_a = (hlen + 15) >> 4, n_c = (clen + 15) >> 4, za = n_a > 0 ? 1 : 0;
    const int n_g = za + n_c + 1, pad = gcm_pad<BPL>(n_g), S = (n_g + pad) / (4 * BPL);
    const int rlen = hlen + clen + (ENC ? 0 : QPP_TAG_LEN);
    const bool tiny = rlen < 16;
    // the H^4 entry, read once: an LDS read inside the step loop would make
    // every step wait for all of its outstanding table lookups
    const uint32_t t4 = G.t4();
    const u32x4 tiny_in = tiny ? ld_part(P.src, rlen) : zero4();
    const int q = pad + za;  // sequence position of CT block 0
    const uint32_t cin = ioff + (uint32_t)hlen, cout = ooff + (uint32_t)hlen;
    // buffer offset of CT block i's input (or out of range)
    auto ct_load = [&](int i) -> uint32_t {
        if (i < 0 || 16 * i >= clen) return kOob;
        return cin + (uint32_t)(ENC ? min(16 * i, clen - 16) : 16 * i);
    };
    // BPL = 2: the first step's two input blocks, requested before the
    // associated data and the counter cache so that their latency overlaps them
    u32x4 nxt0 = {0, 0, 0, 0}, nxt1 = {0, 0, 0, 0};
    if constexpr (BPL == 2) {
        nxt0 = __builtin_amdgcn_raw_buffer_load_b128(B.in, (int)ct_load(sub - q), 0, 0);
        nxt1 = __builtin_amdgcn_raw_buffer_load_b128(B.in, (int)ct_load(sub - q + 4), 0, 0);
    }

    // fold the associated data (unmasked for unprotect) into Z
    u32x4 z = {0, 0, 0, 0};
    for (int g = 0; g < n_a; ++g) {
        u32x4 a;
        if (tiny) {
            a = tiny_in;
        } else if (g == 0) {
            a = h0;  // requested with the descriptor
        } else {
            // 16 bytes at region offset 16 g: end-aligned load + shift
            const int ld = min(16 * g, rlen - 16);
            a = shr_bytes(__builtin_amdgcn_raw_buffer_load_b128(B.in, (int)(ioff + ld), 0, 0),
                          16 * g - ld);
        }
        a = keep_bytes(a, min(16, hlen - 16 * g));
        if (!ENC && P.hp) a ^= hp_pattern(16 * g, P.mask, P.fbm, P.pn_off, P.pn_len);
        if (g > 0) z = ghash_mul_global(z, G.global(0));  // H^1
        z ^= a;
    }
    // the header out: unprotect (mask known) and protect without HP now;
    // protect with HP in its first step or after the loop
    if (!ENC || !P.hp) write_header_v(P, sub, !ENC && P.hp, rlen, tiny ? tiny_in : h0, true);
    const bool fast_hp = ENC && P.hp && gcm_fast_hp<BPL>(hlen, clen);
    // BPL = 1: Z enters as lane `pad`'s initial accumulator (position pad is
    // in its first step's only block); BPL = 2: Z may sit at the second block
    // of a lane's first step, so it enters through that step's input (step2)
    u32x4 acc = (BPL == 1 && za && sub == pad) ? z : u32x4{0, 0, 0, 0};
    const CtrCache cc = ctr_cache(P.nonce, rk, T);
    const uint32_t lens_h = bswap((uint32_t)hlen * 8u);

    // The last step: lane j closes its Horner chain with H^(4-j) (the slot's
    // global table of power 3 - j), and the lengths block's lane (lane 3, the
    // last position of the sequence) adds E_K(J0), which its AES slot just
    // produced (keystream ksl): the tag is then the quad's xor of acc
    auto close = [&](u32x4 ksl) {
        const uint32_t lf = lane_fresh();
        acc = ghash_mul_global(acc, G.global(3u - (lf & 3)));
        if ((lf & 3) == 3) acc ^= ksl;
    };
    // the output side of one block given its keystream: CT block i (input
    // `raw` loaded from CT offset min(16 i, clen - 16) for protect, i.e.
    // end-aligned for a partial tail), the lengths block (i == n_c), or
    // padding; returns the GHASH input of the block
    auto blk_out = [&](int i, u32x4 ksb, u32x4 raw) -> u32x4 {
        const bool is_ct = i >= 0 && 16 * i < clen;
        u32x4 x = {0, 0, 0, 0}, out = {0, 0, 0, 0};
        uint32_t soff = kOob;
        if (is_ct) {
            const int nb = clen - 16 * i;
            if (__builtin_expect(nb >= 16, 1)) {
                // a full block: no byte shifts or masks (a branch, skipped by
                // the waves whose lanes hold no partial block this step)
                out = raw ^ ksb;
                x = ENC ? out : raw;
                soff = cout + 16u * (uint32_t)i;
            } else {
                const u32x4 cur = ENC ? shr_bytes(raw, 16 - nb) : raw;
                out = cur ^ ksb;
                x = keep_bytes(ENC ? out : cur, nb);
                buf_st_part(B.out, cout + 16u * (uint32_t)i, out, nb);
            }
        } else if (i >= 0 && 16 * i < clen + 16) {
            // lengths block; this lane's AES slot produced E_K(J0) (close)
            x = u32x4{0u, lens_h, 0u, bswap((uint32_t)clen * 8u)};
        }
        __builtin_amdgcn_raw_buffer_store_b128(out, B.out, (int)soff, 0, 0);
        return x;
    };
    // one block (BPL = 1)
    auto step = [&](int i, bool last, auto first_c, u32x4 raw) {
        (void)first_c;
        const LdsTe Tl{te, (lane_fresh() & 31) * 4};
        const bool is_ct = i >= 0 && 16 * i < clen;
        const u32x4 ksb = aes_ctr<NR>(cc, is_ct ? (uint32_t)(i + 2) : 1u, rk, Tl);
        acc ^= blk_out(i, ksb, raw);
        __builtin_amdgcn_sched_barrier(0);
        // H^4 inside the loop (resident LDS table); the last step closes
        if (!last) acc = ghash_mul_h4(acc, G.lds, t4);
        else close(ksb);
    };
    // BPL = 2: lane blocks i and i + 4 (CT indices) in one step
    auto step2 = [&](int i, bool last, u32x4 raw0, u32x4 raw1, auto first_c) {
        constexpr bool first = decltype(first_c)::value;
        const LdsTe Tl{te, (lane_fresh() & 31) * 4};
        const uint32_t cb0 = (i >= 0 && 16 * i < clen) ? (uint32_t)(i + 2) : 1u;
        const uint32_t cb1 = (i + 4 >= 0 && 16 * (i + 4) < clen) ? (uint32_t)(i + 6) : 1u;
        u32x4 ks0, ks1;
        if (first && pad >= 4) {
            // the quad's first four positions are all front padding: only
            // the second block of the first step is real
            ks0 = zero4();
            ks1 = aes_ctr<NR>(cc, cb1, rk, Tl);
        } else {
            aes_ctr2<NR>(cc, cb0, cb1, rk, Tl, ks0, ks1);
        }
        u32x4 x0 = blk_out(i, ks0, raw0);
        u32x4 x1 = blk_out(i + 4, ks1, raw1);
        if constexpr (first) {
            if constexpr (ENC) {
                if (fast_hp) {
                    // CT blocks 0 and 1 from the lanes that hold them
                    u32x4 c0 = (i == 0) ? x0 : (i + 4 == 0) ? x1 : zero4();
                    u32x4 c1 = (i == 1) ? x0 : (i + 4 == 1) ? x1 : zero4();
                    c0 = quad_xor_all(c0);
                    c1 = quad_xor_all(c1);
                    const int s = 4 - P.pn_len;
                    const u32x4 smp = {__builtin_amdgcn_alignbyte(c0.y, c0.x, s),
                                       __builtin_amdgcn_alignbyte(c0.z, c0.y, s),
                                       __builtin_amdgcn_alignbyte(c0.w, c0.z, s),
                                       __builtin_amdgcn_alignbyte(c1.x, c0.w, s)};
                    Pkt H = P;
                    H.mask = hp_mask_quad<SUITE>(ks, smp, Tl, sub);
                    write_header_v(H, sub, true, rlen, h0, true);
                }
            }
            // position q - 1 = pad holds Z (zero without associated data)
            if (i == -1) x0 ^= z;
            if (i + 4 == -1) x1 ^= z;
        }
        __builtin_amdgcn_sched_barrier(0);
        // (0 ^ 0) H^4 = 0 over front padding
        if (first && pad >= 4) acc = x1;
        else acc = ghash_mul_h4(acc ^ x0, G.lds, t4) ^ x1;
        if (!last) acc = ghash_mul_h4(acc, G.lds, t4);
        else close(ks1);
    };
    got_tag = u32x4{0, 0, 0, 0};
    if constexpr (BPL == 2) {
        if (tiny) {
            QPP_PROBE_AT(4);
            const u32x4 st = shl_bytes(tiny_in, 16 - rlen);
            step2(sub - q, true, st, st, std::true_type{});
        } else {
            int i = sub - q;
            // register prefetch of both blocks, one step ahead (the first
            // step's since the top); on the last step the first of them is the
            // received tag (unprotect)
            auto one2 = [&](int k, auto first_c) {
                const u32x4 raw0 = nxt0, raw1 = nxt1;
                const uint32_t l0 = (!ENC && k == 1) ? cin + (uint32_t)clen : ct_load(i + 8);
                nxt0 = __builtin_amdgcn_raw_buffer_load_b128(B.in, (int)l0, 0, 0);
                nxt1 = __builtin_amdgcn_raw_buffer_load_b128(B.in, (int)ct_load(i + 12), 0, 0);
                step2(i, k == 1, raw0, raw1, first_c);
                i += 8;
            };
            QPP_PROBE_AT(4);
            // the first step is peeled: it alone may carry Z and the HP sample
            one2(S, std::true_type{});
#pragma unroll 1
            for (int k = S - 1; k > 0; --k) {
                if constexpr (PRIO) {
                    // waves further from the item's end issue first (the
                    // sequencer arbitrates by priority, then age), so a
                    // launch's waves progress together instead of oldest
                    // first, and its tail of half-empty CUs shortens:
                    // +3-5 % at 64 Ki (profiles/r5y_gcm_priority.txt; with
                    // persistent 1024-thread workgroups, for every item or
                    // only each share's last ones, no gain at 1 Mi)
                    const int kr = __builtin_amdgcn_readfirstlane(k);
#if QPP_COMBO_PRIO
                    // study: the workgroup's share level (pbase 0 or 2) plus
                    // one for the item's first half
                    const uint32_t lv = __builtin_amdgcn_readfirstlane(pbase) + (kr >= 5 ? 1u : 0u);
                    if (lv >= 3) __builtin_amdgcn_s_setprio(3);
                    else if (lv == 2) __builtin_amdgcn_s_setprio(2);
                    else if (lv == 1) __builtin_amdgcn_s_setprio(1);
                    else __builtin_amdgcn_s_setprio(0);
#else
                    if (kr >= 7) __builtin_amdgcn_s_setprio(3);
                    else if (kr >= 4) __builtin_amdgcn_s_setprio(2);
                    else if (kr >= 2) __builtin_amdgcn_s_setprio(1);
                    else __builtin_amdgcn_s_setprio(0);
#endif
                }
                one2(k, std::false_type{});
            }
            if (!ENC) got_tag = nxt0;
        }
    } else if (tiny) {
        // < 16 input bytes: one step (n_a, n_c <= 1)
        QPP_PROBE_AT(4);
        step(sub - q, true, std::true_type{}, shl_bytes(tiny_in, 16 - rlen));
    } else {
        int i = sub - q;
        // one step: this step's input block, the next step's load (on the
        // last step the received tag), the block.  Register prefetch, one
        // step ahead.  The input of the step after step k (counting down to
        // 1; step 0 is the received tag of an unprotect), block j = i + 4 (S - k)
        auto in_of = [&](int k, int j) -> uint32_t {
            return (!ENC && k == 0) ? cin + (uint32_t)clen : ct_load(j);
        };
        u32x4 nxt = __builtin_amdgcn_raw_buffer_load_b128(B.in, (int)ct_load(i), 0, 0);
        QPP_PROBE_AT(4);
        auto one = [&](int k, auto first_c) {
            const u32x4 raw = nxt;
            nxt = __builtin_amdgcn_raw_buffer_load_b128(B.in, (int)in_of(k - 1, i + 4), 0, 0);
            step(i, k == 1, first_c, raw);
            i += 4;
        };
        one(S, std::true_type{});
#pragma unroll 1
        for (int k = S - 1; k > 0; --k) one(k, std::false_type{});
        if (!ENC) got_tag = nxt;
    }
    QPP_PROBE_AT(5);
    return quad_xor_all(acc);
}

// Output side of a GCM packet after the step loop: the tag (protect), the
// header when the first step could not write it (gcm_fast_hp), the tag check
// for unprotect.  P: re-derived from the descriptor (src, dst, hlen, clen, hp).
template <bool ENC, int SUITE, int BPL>
__device__ __forceinline__ void gcm_finish(Pkt &P, const KeySlot *ks, int sub, const LdsTe &T, u32x4 tag,
                                           u32x4 got_tag)
{
    if (ENC) {
        if (sub == 0) st16(P.dst + P.hlen + P.clen, tag);
        if (P.hp && !gcm_fast_hp<BPL>(P.hlen, P.clen)) {
            // the header's first byte decides pn_len (HeaderProtection.apply,
            // _crypto.c:298-302); the sample is read back from the output once
            // this wave's ciphertext and tag stores have completed (a
            // coherent load: another lane of the quad may have stored it)
            const int rlen = P.hlen + P.clen;
            const bool have = rlen >= 16;
            const u32x4 hb = have ? ld16(P.src) : ld_part(P.src, rlen);
            const uint32_t b0 = hb.x & 0xff;
            P.pn_len = (int)(b0 & 3) + 1;
            P.pn_off = P.hlen - P.pn_len;
            P.fbm = first_byte_mask(b0);
            // (the tag went out by a flat store: both counters)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const __amdgpu_buffer_rsrc_t r =
                __builtin_amdgcn_make_buffer_rsrc((void *)(P.dst + P.hlen), 0, 64, 0x00020000);
            const u32x4 smp = __builtin_amdgcn_raw_buffer_load_b128(r, 4 - P.pn_len, 0, 1);
            P.mask = hp_mask_quad<SUITE>(ks, smp, T, sub);
            write_header_v(P, sub, true, rlen, hb, true);
        }
    } else {
        const int n_a = (P.hlen + 15) >> 4, n_c = (P.clen + 15) >> 4, za = n_a > 0 ? 1 : 0;
        const int pad = gcm_pad<BPL>(za + n_c + 1);
        const u32x4 diff = got_tag ^ tag;
        if ((diff.x | diff.y | diff.z | diff.w) != 0) {
            P.status = QPP_S_DECRYPT;
            // CT block i sits at sequence position pad + za + i (gcm_packet)
            wipe_payload(P, sub, [&](int i) { return (pad + za + i) & 3; });
        }
    }
}

// ---------------------------------------------------- ChaCha20-Poly1305 --

// Work of a packet's quad (RFC 8439 sec. 2.8; _crypto.c:157-204 / :115-155).
// Units u = 4k + sub: u < 3 -> ChaCha20 chunk u, u = 3 -> the Poly1305 key
// block (counter 0, RFC 8439 sec. 2.6), u > 3 -> chunk u - 1.  So lane 3
// produces the one-time key while lanes 0-2 encrypt chunks 0-2, and a
// 1173-byte payload (19 chunks + key = 20 units) takes 5 ChaCha blocks per
// lane instead of 6.  Poly1305 is per-lane Horner over the lane's blocks
// (r per block; r^8 / r^12 across the 2 / 3 other lanes' chunks) and one
// quad sum at the end.
template <int CTRL>
__device__ __forceinline__ uint32_t quad_dpp(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

// values the compiler must not keep live across the chunk loop: pass them
// through an empty asm so powers of r are recomputed after it
__device__ __forceinline__ P130 launder(P130 x)
{
#pragma unroll
    for (int l = 0; l < 5; ++l) asm volatile("" : "+v"(x.v[l]));
    return x;
}

// lane J's value in every lane of the quad (DPP quad_perm [J,J,J,J])
template <int J>
__device__ __forceinline__ P130 p130_from_lane(P130 x)
{
#pragma unroll
    for (int l = 0; l < 5; ++l) x.v[l] = quad_dpp<J * 0x55>(x.v[l]);
    return x;
}

// limb-wise sum over the quad, in every lane (no carries: 4 limbs of < 2^27)
__device__ __forceinline__ P130 p130_quad_sum(P130 x)
{
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        x.v[l] += quad_dpp<0xB1>(x.v[l]);
        x.v[l] += quad_dpp<0x4E>(x.v[l]);
    }
    return x;
}

// 16 bytes per lane from buffer offset `off` (out of range: zeros) into LDS at
// lds + 16 * lane (LDS-DMA)
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t rsrc, uint8_t *lds, uint32_t off)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)lds, 16, off, 0, 0,
                                             0);
}

// Work of a packet's quad, staged form (RFC 8439 sec. 2.8; _crypto.c:157-204
// / :115-155).  Unit u = ChaCha20 block counter u: u = 0 is the Poly1305 key
// block (RFC 8439 sec. 2.6), u >= 1 encrypts 64-byte chunk u - 1.  Lane j
// runs unit 4k + j at step k, so a quad's step covers chunks 4k - 1 .. 4k + 2,
// 256 contiguous payload bytes, moved by 4 coalesced LDS-DMA loads and 4
// coalesced stores (kChRegion).  Poly1305 is per-lane Horner over the lane's
// chunks (r per block, r^12 across the other 3 lanes' chunks), lane 0 starting
// with the associated data, and one quad sum at the end.  B / ioff / ooff:
// the wave's buffer views and the packet's offsets in them.
template <bool ENC, bool PRIO>
__device__ void chacha_packet(Pkt &P, const KeySlot *ks, int sub, uint8_t *scr, uint8_t *stage, uint32_t *pw,
                              const Bufs &B, uint32_t ioff, uint32_t ooff)
{
    const uint32_t *key = ks->rk;
    const uint32_t n0 = P.nonce.x, n1 = P.nonce.y, n2 = P.nonce.z;
    const int n_a = (P.hlen + 15) >> 4, n_c = (P.clen + 15) >> 4;
    const int chunks = (P.clen + 63) >> 6;
    const bool unmask = !ENC && P.hp;
    const uint8_t *pin = P.src + P.hlen;
    uint8_t *pout = P.dst + P.hlen;
    const int rlen = P.hlen + P.clen + (ENC ? 0 : QPP_TAG_LEN);
    // < 16 readable bytes (AEAD-only protect of a short input): byte loads
    const bool tiny = rlen < 16;
    const uint8_t *h0 = tiny ? nullptr : scr + kScrHdr;
    const int steps = (chunks + 4) >> 2;  // units 0..chunks, 4 per step
    // payload block i: its 16 input bytes, end-aligned within the region for
    // a protect's partial last block (the consumer shifts it down)
    auto blk_off = [&](int i) -> uint32_t {
        if (i < 0 || i >= n_c || tiny) return kOob;
        const int o = P.hlen + 16 * i;
        return ioff + (uint32_t)(ENC ? min(o, rlen - 16) : o);
    };
    // LDS-DMA of step k's 4 chunks: instruction t, lane j -> block j of chunk 4k - 1 + t
    auto dma = [&](int k) {
#pragma unroll
        for (int t = 0; t < 4; ++t) lds_dma16(B.in, stage + t * kChRegion, blk_off(4 * (4 * k - 1 + t) + sub));
    };
    QPP_PROBE_AT(1);  // (probe build) descriptor, header, pkt_begin
    const uint32_t qoff = (lane_fresh() >> 2) * 64;  // the quad's 64 bytes in each region
    // the packet fields the chunk loop does not use (HP mask, packet number,
    // header layout) wait in LDS until the tag: 128 VGPRs at 4 waves per SIMD
    // leave no room for them across the loop
    park(P, scr, !ENC);

    dma(0);
    // r13 = r^13: the multiply of a lane's last block before its next chunk
    // also jumps over the other 3 lanes' chunks (12 blocks), so a chunk costs
    // 4 multiplies instead of 4 + 1
    P130 acc = p130_zero(), r = p130_zero(), r13 = p130_zero();
    // Poly1305 over the 4 blocks of chunk c (their inputs x), branch-free so
    // that it shares a basic block with the next ChaCha20 block and the
    // scheduler can fill the latency of its 64-bit multiply-add chains with
    // the block's independent quarter rounds.  Blocks that do not exist
    // (c < 0: the key unit; past the payload's end) multiply by one and add
    // zero, which leaves the chain as it is.
#if !QPP_CH_POLY4
    auto poly_blk = [&](const u32x4 (&x)[4], int c, int b) {
        {
            const int i = 4 * c + b;
            const bool valid = c >= 0 && i < n_c;
            const P130 m = p130_block(x[b]);
            const P130 &rm = (b == 3 && c + 4 < chunks) ? r13 : r;
            // (x[b] is zero for a block that does not exist: only the 2^128
            // bit of p130_block needs masking)
            P130 a = acc, f;
#pragma unroll
            for (int l = 0; l < 5; ++l) {
                a.v[l] += l < 4 ? m.v[l] : valid ? m.v[l] : 0u;
                f.v[l] = valid ? rm.v[l] : (l == 0 ? 1u : 0u);
            }
            acc = p130_mul(a, f);
        }
    };
#endif
#if QPP_CH_POLY4
    // The chunk as one sum: the lane's chain moves by
    //   acc <- (acc + x0) r^e0 + x1 r^e1 + x2 r^e2 + x3 r^e3,
    // e = 16 .. 13 when the lane has a later chunk (its Horner steps r, r, r
    // and the r^13 jump over the other lanes' chunks, multiplied out), else
    // the chunk's own valid blocks nbv - b .. 1 (a block past the payload
    // adds zero; no chunk at all: acc r^0).  Four independent products from
    // the pw powers into 64-bit column sums (part b after double round 2b + 1)
    // and one carry after the rounds, instead of four dependent multiplies
    // each with its carry and selects.
    uint64_t dsum[5];
    auto poly_part = [&](const u32x4 (&x)[4], int c, int b) {
        const bool inc = c >= 0 && c < chunks;
        const int nbv = min(4, n_c - 4 * c);  // the chunk's blocks (fewer in the final chunk only)
        const bool valid = inc && b < nbv;
        const int e = !inc ? 0 : (c + 4 < chunks) ? 16 - b : valid ? nbv - b : 0;
        const int idx = e < 13 ? e : e - (13 - kPw13);
        P130 m = p130_block(x[b]);
        // (x[b] is zero for a block that does not exist: only the 2^128
        // bit of p130_block needs masking)
        m.v[4] = valid ? m.v[4] : 0u;
        if (b == 0) m = p130_add(m, acc);
        P130 rp;
#pragma unroll
        for (int l = 0; l < 5; ++l) rp.v[l] = pw[5 * idx + l];
        if (b == 0) {
#pragma unroll
            for (int l = 0; l < 5; ++l) dsum[l] = 0;
        }
        p130_mac(dsum, m, rp);
    };
    auto poly_carry = [&]() { acc = p130_carry(dsum[0], dsum[1], dsum[2], dsum[3], dsum[4]); };
    auto poly = [&](const u32x4 (&x)[4], int c) {
#pragma unroll
        for (int b = 0; b < 4; ++b) poly_part(x, c, b);
        poly_carry();
    };
#else
    auto poly = [&](const u32x4 (&x)[4], int c) {
#pragma unroll
        for (int b = 0; b < 4; ++b) poly_blk(x, c, b);
    };
#endif
    // the memory side of step k: the lane's chunk c from region `sub` xor
    // its keystream, back through LDS to 4 coalesced stores, the next step's
    // LDS-DMA; x = the chunk's Poly1305 inputs
    auto chunk_io = [&](int k, int c, const uint32_t (&blk)[16], u32x4 (&x)[4]) {
        // (the DMA retires in issue order, after the previous step's stores:
        // vmcnt(0) waits for both)
#ifdef QPP_CH_MEMPRIO
        __builtin_amdgcn_s_setprio(QPP_CH_MEMPRIO);  // study: the memory side first
#endif
        QPP_PROBE_AT(4);  // (probe build) the ChaCha20 block and Poly1305 before this wait
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        QPP_PROBE_AT(5);  // the wait for this step's input (and the last step's stores)
        uint8_t *mine = stage + sub * kChRegion + qoff;
#if QPP_CH_DPP_T
        u32x4 o4[4];
#endif
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int i = 4 * c + b;
            const bool valid = c >= 0 && i < n_c;
            const int nb = P.clen - 16 * i;
            u32x4 in = *(const u32x4 *)(mine + 16 * b);
            const u32x4 ks = u32x4{blk[4 * b], blk[4 * b + 1], blk[4 * b + 2], blk[4 * b + 3]};
            u32x4 o;
            x[b] = u32x4{0, 0, 0, 0};
            if (__builtin_expect(valid && nb >= 16 && !tiny, 1)) {
                // a full block: no byte shifts or masks (a branch, skipped by
                // the waves whose lanes hold no partial block this step)
                o = in ^ ks;
                x[b] = ENC ? o : in;
            } else {
                if (tiny) in = valid ? ld_part(pin + 16 * i, min(16, nb)) : in;
                else if (ENC && nb < 16) in = shr_bytes(in, 16 - nb);
                o = in ^ ks;
                if (valid) {
                    x[b] = keep_bytes(ENC ? o : in, min(16, nb));
                    if (nb < 16) st_part(pout + 16 * i, o, nb);  // partial block: byte-exact, direct
                }
            }
            if (valid && ENC && P.hp && i < 2) *(u32x4 *)(scr + 16 * i) = x[b];
#if QPP_CH_DPP_T
            if constexpr (PRIO) {
                o4[b] = o;  // transposed across the quad below, no LDS round trip
            } else {
                *(u32x4 *)(mine + 16 * b) = o;
            }
#elif QPP_CH_DIRECT_ST
            {
                // the lane's own full block straight out (a quad's 4 stores
                // of one instruction are 64 B apart; the 4 instructions
                // complete the quad's 256 B)
                const uint32_t so = (valid && nb >= 16 && !tiny) ? ooff + (uint32_t)(P.hlen + 16 * i) : kOob;
                __builtin_amdgcn_raw_buffer_store_b128(o, B.out, (int)so, 0, 0);
            }
#else
            *(u32x4 *)(mine + 16 * b) = o;
#endif
        }
#if QPP_CH_DPP_T
        if constexpr (PRIO) {
            // one-round launches (latency-bound, VALU to spare): the quad's
            // 4x4 transpose of blocks in registers, two DPP butterflies
            // (lanes j^1, then j^2; each lane sends the block it replaces),
            // so o4[t] = lane t's block `sub` = this lane's block of chunk
            // 4k - 1 + t, for the same coalesced stores without writing the
            // blocks back through LDS and reading them again
            const bool p0 = (sub & 1) != 0, p1 = (sub & 2) != 0;
#pragma unroll
            for (int a = 0; a < 4; a += 2) {
                const u32x4 snd = p0 ? o4[a] : o4[a + 1];
                const u32x4 rcv = u32x4{quad_dpp<0xB1>(snd.x), quad_dpp<0xB1>(snd.y), quad_dpp<0xB1>(snd.z),
                                        quad_dpp<0xB1>(snd.w)};
                if (p0) o4[a] = rcv;
                else o4[a + 1] = rcv;
            }
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const u32x4 snd = p1 ? o4[a] : o4[a + 2];
                const u32x4 rcv = u32x4{quad_dpp<0x4E>(snd.x), quad_dpp<0x4E>(snd.y), quad_dpp<0x4E>(snd.z),
                                        quad_dpp<0x4E>(snd.w)};
                if (p1) o4[a] = rcv;
                else o4[a + 2] = rcv;
            }
            // the xor consumed every lane's input: the regions are free
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            QPP_PROBE_AT(6);  // (probe build) xor and transpose
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int i = 4 * (4 * k - 1 + t) + sub;
                const uint32_t so = (i >= 0 && 16 * i + 16 <= P.clen && !tiny) ? ooff + (uint32_t)(P.hlen + 16 * i) : kOob;
                __builtin_amdgcn_raw_buffer_store_b128(o4[t], B.out, (int)so, 0, 0);
            }
            QPP_PROBE_AT(8);  // (probe build) the stores' issue
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            QPP_PROBE_AT(6);  // (probe build) xor through LDS
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int i = 4 * (4 * k - 1 + t) + sub;
                const uint32_t so = (i >= 0 && 16 * i + 16 <= P.clen && !tiny) ? ooff + (uint32_t)(P.hlen + 16 * i) : kOob;
                const u32x4 v = *(const u32x4 *)(stage + t * kChRegion + qoff + 16 * sub);
                __builtin_amdgcn_raw_buffer_store_b128(v, B.out, (int)so, 0, 0);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            QPP_PROBE_AT(8);  // (probe build) the stores' reads and issue
        }
#elif QPP_CH_DIRECT_ST
        // the xor consumed every lane's input: the regions are free for the
        // next step's DMA
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        QPP_PROBE_AT(6);  // (probe build) xor and stores
#else
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        QPP_PROBE_AT(6);  // (probe build) xor through LDS
        // coalesced stores of the quad's full blocks: instruction t, lane j ->
        // block j of chunk 4k - 1 + t
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int i = 4 * (4 * k - 1 + t) + sub;
            const uint32_t so = (i >= 0 && 16 * i + 16 <= P.clen && !tiny) ? ooff + (uint32_t)(P.hlen + 16 * i) : kOob;
            const u32x4 v = *(const u32x4 *)(stage + t * kChRegion + qoff + 16 * sub);
            __builtin_amdgcn_raw_buffer_store_b128(v, B.out, (int)so, 0, 0);
        }
        // the regions are read: next step's input (hidden behind this step's
        // Poly1305 and the next ChaCha20 block)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        QPP_PROBE_AT(8);  // (probe build) the stores' reads and issue
#endif
        if (k + 1 < steps) dma(k + 1);
#ifdef QPP_CH_MEMPRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        QPP_PROBE_AT(3);  // (probe build) next step's DMA issue
    };

    // step 0: unit `sub` (lane 0: the one-time key, lanes 1-3: chunks 0-2)
    u32x4 x[4];
    {
        uint32_t blk[16];
        chacha_block(key, (uint32_t)sub, n0, n1, n2, blk);
        // one-time key from lane 0: r, and s parked in LDS until the tag
        uint32_t kw[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) kw[w] = quad_dpp<0x00>(blk[w]);
        *(u32x4 *)(scr + kScrEj0) = u32x4{kw[4], kw[5], kw[6], kw[7]};
        r = p130_r(kw[0], kw[1], kw[2], kw[3]);
        // powers, lane-parallel: r^2; lane 0 r^3 beside lane 1 r^4; lane 0
        // r^5 beside lane 1 r^8; r^13 = r^8 r^5 -- 4 multiplies per lane
        // instead of 5 plus lane 0's r^3
        const P130 r2 = p130_mul(r, r);
        const P130 b34 = p130_mul(r2, sub == 0 ? r : r2);
        const P130 r3 = p130_from_lane<0>(b34), r4 = p130_from_lane<1>(b34);
        const P130 b58 = p130_mul(r4, sub == 0 ? r : r4);
        const P130 r5 = p130_from_lane<0>(b58), r8 = p130_from_lane<1>(b58);
        r13 = p130_mul(r8, r5);
#if QPP_CH_POLY4
        {
            // the chunk sums' powers r^13 .. r^16, one multiply per lane:
            // lane 0 r^13 r, lane 1 r^8 r^8, lane 2 r^13 r^2, lane 3 r^13
            const P130 one = P130{{1u, 0u, 0u, 0u, 0u}};
            const P130 pa = sub == 1 ? r8 : r13;
            const P130 pb = sub == 0 ? r : sub == 1 ? r8 : sub == 2 ? r2 : one;
            const P130 pr = p130_mul(pa, pb);
            const int slot = kPw13 + (sub == 0 ? 1 : sub == 1 ? 3 : sub == 2 ? 2 : 0);
#pragma unroll
            for (int l = 0; l < 5; ++l) pw[5 * slot + l] = pr.v[l];
        }
#endif
        if (sub == 0) {  // the close's powers (kPwOne .. kPw8)
#pragma unroll
            for (int l = 0; l < 5; ++l) {
                pw[5 * kPwOne + l] = l == 0 ? 1u : 0u;
                pw[5 * kPw1 + l] = r.v[l];
                pw[5 * (kPw1 + 1) + l] = r2.v[l];
                pw[5 * (kPw1 + 2) + l] = r3.v[l];
                pw[5 * (kPw1 + 3) + l] = r4.v[l];
                pw[5 * (kPw1 + 4) + l] = r5.v[l];
                pw[5 * kPw8 + l] = r8.v[l];
            }
        }
        // lane 0 starts its chain with the associated data (its next chunk,
        // if any, is chunk 3)
        if (sub == 0) {
            const Pkt Q = unpark(scr, P.src, P.dst, !ENC);
            for (int g = 0; g < n_a; ++g) {
                const int nb = min(16, P.hlen - 16 * g);
                u32x4 a = (g == 0 && h0) ? keep_bytes(*(const u32x4 *)h0, nb)
                                         : ld_win(P.src + 16 * g, nb, P.src, P.src + rlen);
                if (unmask) a ^= hp_pattern(16 * g, Q.mask, Q.fbm, Q.pn_off, Q.pn_len);
                if (!ENC || !P.hp) st_part(P.dst + 16 * g, a, nb);
                acc = p130_mul(p130_add(acc, p130_block(a)), (g == n_a - 1 && 3 < chunks) ? r13 : r);
            }
        }
        QPP_PROBE_AT(2);  // key block, powers, associated data
        chunk_io(0, sub - 1, blk, x);
    }
    // step k: the ChaCha20 block of unit 4k + sub beside Poly1305 of the
    // lane's previous chunk (software-pipelined by one step)
#pragma unroll 1
    for (int k = 1; k < steps; ++k) {
        if constexpr (PRIO) {
            // waves further from the packet's end issue first (the sequencer
            // arbitrates by priority, then age), so a launch of one wave per
            // slot progresses together instead of oldest first, as k_gcm's
            // 512-thread shape does
            const int kr = __builtin_amdgcn_readfirstlane(steps - k);
            if (kr >= 4) __builtin_amdgcn_s_setprio(3);
            else if (kr == 3) __builtin_amdgcn_s_setprio(2);
            else if (kr == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        const int c = 4 * k + sub - 1;
        uint32_t blk[16];
        // the previous chunk's 4 Poly1305 blocks after double rounds 1, 3, 5, 7
#if QPP_CH_POLY4
        // the previous chunk's 4 Poly1305 products after double rounds 1, 3,
        // 5, 7, its carry after the last
        chacha_block_beside(key, (uint32_t)(c + 1), n0, n1, n2, blk, [&](int i) {
            if (i & 1 && i < 8) poly_part(x, c - 4, i >> 1);
            if (i == QPP_CH_CARRY_AT) poly_carry();
        });
#else
        chacha_block_beside(key, (uint32_t)(c + 1), n0, n1, n2, blk, [&](int i) {
            if (i & 1 && i < 8) poly_blk(x, c - 4, i >> 1);
        });
#endif
        // pin the chain here: otherwise the compiler sinks this Poly1305 step
        // to the next iteration's top (beside the loop's exit test), out of
        // the rounds' basic block
        acc = launder(acc);
        chunk_io(k, c, blk, x);
    }
    poly(x, 4 * (steps - 1) + sub - 1);
    QPP_PROBE_AT(4);
    {
        const uint8_t *src = P.src;
        uint8_t *dst = P.dst;
        P = unpark(scr, src, dst, !ENC);
    }
    // Close the four chains.  Lane j's chain ends at the last block of its
    // last chunk (lane 0 without a chunk: the last header block, position
    // -1); the lanes' ends follow one another in the order L + 1, L + 2,
    // L + 3, L (mod 4), L = chunks mod 4 holding the final chunk, 4 blocks
    // apart except the final chunk's nb blocks (a lane with no block at all
    // holds 0), and the lengths block follows, so the tag's polynomial is
    //   A[L+1] r^(9+nb) + A[L+2] r^(5+nb) + A[L+3] r^(1+nb) + (A[L] + lens) r
    //   = (A[L+1] r^8 + A[L+2] r^4 + A[L+3]) r^(nb+1) + (A[L] + lens) r.
    // Two multiplies per lane: each lane's own chain by its role's power
    // (r^8, r^4, 1, r: pw entries parked at the key block), two quad sums,
    // then the first sum by r^(nb+1) -- instead of a 4-multiply Horner pass
    // over chains exchanged through LDS.
    const int L = chunks & 3;
    const int nb = chunks > 0 ? n_c - 4 * (chunks - 1) : 1;
    const int role = (sub - L - 1) & 3;  // 0: lane L+1, 1: L+2, 2: L+3, 3: L
    auto power = [&](int e) -> P130 {    // pw entry e
        P130 x;
#pragma unroll
        for (int l = 0; l < 5; ++l) x.v[l] = pw[5 * e + l];
        return x;
    };
    const u32x4 lens = u32x4{(uint32_t)P.hlen, 0u, (uint32_t)P.clen, 0u};
    const P130 lb = p130_block(lens);
    P130 a = acc;
#pragma unroll
    for (int l = 0; l < 5; ++l) a.v[l] += role == 3 ? lb.v[l] : 0u;
    const P130 m = p130_mul(a, power(role == 0 ? kPw8 : role == 1 ? kPw1 + 3 : role == 2 ? kPwOne : kPw1));
    P130 u = m, v = p130_zero();
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        u.v[l] = role == 3 ? 0u : m.v[l];
        v.v[l] = role == 3 ? m.v[l] : 0u;
    }
    const P130 sum = p130_add(p130_mul(p130_quad_sum(u), power(kPw1 + nb)), p130_quad_sum(v));
    const u32x4 sw = *(const u32x4 *)(scr + kScrEj0);
    const u32x4 tag = p130_finish(sum, sw.x, sw.y, sw.z, sw.w);
    if (ENC) {
        if (sub == 0) st16(pout + P.clen, tag);
        if (P.hp) protect_finish_hp<QPP_CHACHA20_POLY1305>(P, ks, sub, scr, tag, ConstTe{}, h0);
    } else {
        const u32x4 got = ld16(pin + P.clen);
        const u32x4 diff = got ^ tag;
        if ((diff.x | diff.y | diff.z | diff.w) != 0) {
            P.status = QPP_S_DECRYPT;
            // chunk c (blocks 4c..4c+3) is unit c + 1, run by lane (c + 1) & 3
            wipe_payload(P, sub, [&](int i) { return ((i >> 2) + 1) & 3; });
        }
    }
    QPP_PROBE_AT(7);  // close, tag, header protection
}

template <bool ENC>
__device__ __forceinline__ void write_result(qpp_result *res, uint32_t p, int sub, const Pkt &P)
{
    if (sub != 0) return;  // p: the packet's index in the caller's order
    const uint32_t out_len =
        P.status == QPP_S_OK ? (uint32_t)(P.hlen + P.clen + (ENC ? QPP_TAG_LEN : 0)) : 0u;
    res[p] = qpp_result{P.pn, (uint16_t)P.status, (uint16_t)P.hlen, out_len};
}

// ---------------------------------------------------------------- kernels --

// ---------------------------------------------------------------- kernels --
//
// One kernel per cipher suite and direction: a launch handles the packets
// whose key slot holds SUITE and leaves the others to the launch of their
// suite.  Register allocation is then sized for one cipher.
//
// Unplanned launch: positions [0, n) of desc, 16 per wave, result of
// position p at res[p].  Planned launch (items != null): desc is the plan's
// bucket-ordered copy, each wave takes one item of this suite's items
// [irange[2 SUITE], irange[2 SUITE + 1]) (wave_span), and a packet's result
// goes to res[desc.rsv] (its index in the caller's order).

// GCM: a persistent kernel, one 1024-thread workgroup per CU (its LDS use
// allows no second one).  The workgroup fills the AES image once and then
// works through a contiguous share of the launch's wave items: each wave
// takes the next item of the share (an LDS counter) as soon as it finishes
// the last, so no wave waits for the others and no CU idles between
// workgroups.  An item is <= 16 packets (one per quad): planned, one key
// slot's run (qpp_plan.hip); unplanned, 16 consecutive positions.
//
// GHASH tables: kTabEntries LDS entries, each the H^4 table of one key slot,
// shared by the waves running that slot (a reference count per entry).  A
// wave that needs a slot no entry holds loads it into the least recently
// used free entry (LDS-DMA, 8 KiB); with every entry in use by other slots
// it waits for one to come free.  A share of a bucketed batch walks its
// slots in order, so the 16 waves hold one or two slots at a time.
constexpr int kTabEntries = 4;
// Two 512-thread workgroups per CU (launch_packets: small single-key
// launches) hold one table entry each.
template <int WG>
constexpr int gcm_tab_entries() { return WG == 512 ? 1 : kTabEntries; }
static_assert(kGhLdsEntry % 1024 == 0, "LDS-DMA pieces of 1 KiB");

// Watchdog events since the library loaded (tab_acquire gave up on a GHASH
// table entry, or a pair launch's hand-over timed out: the packets concerned
// report QPP_S_INTERNAL); never expected.
__device__ uint32_t g_qpp_watchdog;

// The bounded waits' limits, in sleep rounds: a GHASH table entry (tab_acquire;
// ~1 s at 2^22) and a pair launch's hand-over (k_lone_gcm).  Read where they
// are used, not kept in registers (an SGPR live across k_gcm's step loop
// spills); the host lowers both only under QPP_SPIN_LIMIT, a test switch.
__device__ uint32_t g_qpp_spin_tab = 1u << 22;
__device__ uint32_t g_qpp_spin_lone = 1u << 18;
// Test switch (QPP_PAIR_DELAY): sleep rounds the second wave of a pair launch
// spends before handing its share over, so that with QPP_SPIN_LIMIT=0 the
// first wave gives up deterministically (tests/test_gpu_watchdog.py).  0 in
// every product run.
__device__ uint32_t g_qpp_pair_delay = 0u;

template <int WG, int NE = gcm_tab_entries<WG>()>
struct __attribute__((aligned(16))) GcmSmem {
    // GHASH table entries first (LDS offset 0: the entry's offset rides in
    // the 5-bit window address), then the AES image, whose base stays within
    // the 16-bit ds_read immediate range
    uint8_t h4[NE][kGhLdsEntry];              // 14 KiB each
    uint8_t te[kTeBytes];                     // Te0|Te1 x 32 bank copies   64 KiB
    uint32_t eslot[NE];                       // slot held by entry e (kNoSlot: none)
    uint32_t eref[NE];                        // waves running entry e's slot
    uint32_t eready[NE];                      // entry e's table has landed
    uint32_t eused[NE];                       // last acquisition (LRU tick)

    uint32_t lock, tick, next;                // entry lock; LRU clock; next item of the share
    uint32_t exited;                          // pooled: waves past their last item
    uint32_t wslot[WG / 64];                  // per wave: the slot it is running
    uint32_t went[WG / 64];                   // per wave: that slot's table entry
};

// Entry of slot `cur` for the calling wave (wave-uniform control flow):
// found, or loaded into a free entry.  Lane 0 does the bookkeeping under the
// workgroup's LDS lock.  Returns once the entry's table is in LDS, or kNoSlot
// when `spin` rounds of waiting for a free entry, or for another wave's load
// of the entry, ran out (a watchdog: the caller fails the slot's packets with
// QPP_S_INTERNAL; QPP_SPIN_LIMIT=0 forces it in tests, g_qpp_spin_tab).  (Returning
// before the table has landed, to overlap its LDS-DMA with the packets'
// descriptors and headers, measured 2-4 % slower at 64 Ki: those loads queue
// behind the DMA in the vector memory counter, profiles/r4d_ab_tab_defer.txt.)
template <int WG>
__device__ uint32_t tab_acquire(GcmSmem<WG> &sm, const uint8_t *gtab, uint32_t cur)
{
    const uint32_t spin = __builtin_nontemporal_load(&g_qpp_spin_tab);
    typedef const __attribute__((address_space(1))) void *gptr_t;
    typedef __attribute__((address_space(3))) void *lptr_t;
    uint32_t e = kNoSlot, load = 0;
    // bounded: every entry in use means other waves are running their slots,
    // and each of them releases its entry when done (watchdog, not a limit
    // that a correct run reaches: ~1 s of sleeps at the default 2^22)
#pragma unroll 1
    for (uint32_t it = 0; it < spin; ++it) {
        uint32_t got = kNoSlot, ld = 0;
        if (lane_fresh() == 0) {
            while (atomicCAS(&sm.lock, 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(1);
            int hit = -1, vic = -1;
            uint32_t best = 0xffffffffu;
#pragma unroll
            for (int i = 0; i < gcm_tab_entries<WG>(); ++i) {
                const uint32_t s = lds_ld(&sm.eslot[i]);
                const uint32_t r = lds_ld(&sm.eref[i]);
                const uint32_t u = lds_ld(&sm.eused[i]);
                if (s == cur) hit = i;
                else if (r == 0u && u < best) {
                    best = u;
                    vic = i;
                }
            }
            if (hit < 0 && vic >= 0) {
                hit = vic;
                ld = 1;
                lds_st(&sm.eslot[vic], cur);
                lds_st(&sm.eready[vic], 0u);
            }
            if (hit >= 0) {
                got = (uint32_t)hit;
                atomicAdd(&sm.eref[hit], 1u);  // atomic: releases decrement without the lock
                const uint32_t t = lds_ld(&sm.tick) + 1u;
                lds_st(&sm.tick, t);
                lds_st(&sm.eused[hit], t);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // bookkeeping before the unlock
            atomicExch(&sm.lock, 0u);
        }
        got = __builtin_amdgcn_readfirstlane(got);
        if (got != kNoSlot) {
            e = got;
            load = __builtin_amdgcn_readfirstlane(ld);
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
    if (e == kNoSlot) return e;  // watchdog: no entry came free
    if (load) {
        // H^4 of the slot in the step loop's layout: 14 pieces of 1 KiB
        const uint8_t *src = gtab + (size_t)cur * kGhashTabBytes + kGh5Off;
        const uint32_t l = lane_fresh();
#pragma unroll
        for (int c = 0; c < kGhLdsEntry / 1024; ++c)
            __builtin_amdgcn_global_load_lds((gptr_t)(src + c * 1024 + l * 16), (lptr_t)(sm.h4[e] + c * 1024),
                                             16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane_fresh() == 0) lds_st(&sm.eready[e], 1u);
    } else {
        bool ready = false;
#pragma unroll 1
        for (uint32_t it = 0; it < spin; ++it) {
            if (__builtin_amdgcn_readfirstlane(lds_ld(&sm.eready[e]))) {
                ready = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ready) {
            // watchdog: the loading wave never published the table; drop the
            // reference taken above rather than read a table not yet landed
            if (lane_fresh() == 0) atomicSub(&sm.eref[e], 1u);
            return kNoSlot;
        }
    }
    return e;
}

template <int WG>
__device__ __forceinline__ void tab_release(GcmSmem<WG> &sm, uint32_t e)
{
    if (lane_fresh() == 0) atomicSub(&sm.eref[e], 1u);
}

// Study build only (-DQPP_STUDY_SYNTH, tools/build_variant.py): the north
// star's descriptors and header byte 0 synthesized from the packet index
// instead of loaded, to bound what prefetching them could gain (round 5,
// VERDICT r4 item 3).  Wrong output by design: timing only.
#ifdef QPP_STUDY_SYNTH
__device__ __forceinline__ qpp_desc study_desc(const qpp_desc *, uint32_t p)
{
    return qpp_desc{1200ull * p, 1200ull * p, 1173u, 11, 0, (uint64_t)p, 0u, p};
}
#define QPP_DESC(i) study_desc(desc, (i))
#else
#define QPP_DESC(i) desc[i]
#endif

// Launch-wide item pool of a 1024-thread GCM launch (pool != null, a slot of
// the key table's PoolRing): the workgroups' contiguous shares cover all but
// the last 1/kPoolDiv of the launch's items, which any wave takes, once its
// workgroup's share is done, from the pool's counter (pool[0]; one global
// atomic per pooled item).  The CUs of the 8 XCDs do not run at one rate
// (static shares ended 1313-1366 us by XCD on one box, profiles/r5ad_gcm_pool.txt),
// so the pool lets the faster ones take the slower ones' last items.  The
// last wave of the last workgroup (pool[1] counts workgroups out) zeroes the
// slot for its next launch.  Single-key launches only: in a bucketed launch
// over many keys the pooled items scatter each key over many workgroups'
// GHASH table entries (config 4 -6 %, config 5 -0.4 %; the north star +0.4
// to +1.6 %, profiles/r5ad_gcm_pool.txt).
#ifndef QPP_POOL_DIV
#define QPP_POOL_DIV 12  // build-time study switch
#endif
constexpr uint32_t kPoolDiv = QPP_POOL_DIV;
#ifndef QPP_POOL512
#define QPP_POOL512 0  // study switch: the item pool for the 512-thread shape too
#endif
#ifndef QPP_COMBO_PRIO
#define QPP_COMBO_PRIO 0  // study switch: 512-thread shape, share level + item progress in one priority
#endif
#ifndef QPP_SHARE_PRIO
#define QPP_SHARE_PRIO 0  // study switch: 512-thread shape, issue priority by the workgroup's share left
#endif
#ifndef QPP_PRIO512
#define QPP_PRIO512 1  // study switch: issue priority by progress in the 512-thread shape
#endif

template <int SUITE, bool ENC, int WG, int BPL>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4))) void k_gcm(const KeySlot *__restrict__ slots,
                                              const uint8_t *__restrict__ gtab, uint32_t cap,
                                              const qpp_desc *__restrict__ desc, uint32_t n,
                                              const uint8_t *gin, uint8_t *gout,
                                              qpp_result *__restrict__ res,
                                              const uint32_t *__restrict__ items,
                                              const uint32_t *__restrict__ irange,
                                              uint32_t *__restrict__ pool)
{
    constexpr int kNR = SUITE == QPP_AES_256_GCM ? 14 : 10;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    QPP_PROBE_AT(kProbeStart);
    const bool planned = irange != nullptr;
    // this workgroup's share [sb, se) of the launch's items
    uint32_t ib = 0, ie = (n + 15u) / 16u;
    if (planned) {
        ib = irange[2 * SUITE];
        ie = irange[2 * SUITE + 1];
    }
    const uint32_t total = ie > ib ? ie - ib : 0u;
    // the pooled items [ib + stat, ie) (pool: every workgroup stays to the
    // end, which counts it out)
    const uint32_t pool_n = pool ? total / kPoolDiv : 0u, stat = total - pool_n;
    const uint32_t per = (stat + gridDim.x - 1) / gridDim.x;
    const uint32_t sb = ib + min(stat, per * blockIdx.x), se = ib + min(stat, per * (blockIdx.x + 1));
    if (!pool && sb >= se) return;  // uniform over the workgroup
    __shared__ GcmSmem<WG> sm;
    // Thread-derived values are recomputed where they are used, from the
    // wave index (an SGPR) and a fresh lane id, instead of being kept live
    // across the packet loops: at 128 VGPRs anything live across the GCM step
    // loop is spilled to scratch (HBM traffic and latency).
    auto tid_now = [&]() -> uint32_t { return (wv << 6) | lane_fresh(); };
    load_te<WG>(sm.te);
    if (threadIdx.x < gcm_tab_entries<WG>()) {
        sm.eslot[threadIdx.x] = kNoSlot;
        sm.eref[threadIdx.x] = 0u;
        sm.eready[threadIdx.x] = 0u;
        sm.eused[threadIdx.x] = 0u;
    }
    if (threadIdx.x == 0) {
        sm.lock = 0u;
        sm.tick = 0u;
        sm.next = sb;
        sm.exited = 0u;
    }
    if (threadIdx.x < WG / 64) sm.wslot[threadIdx.x] = kNoSlot;
    __syncthreads();
    QPP_PROBE_AT(0);  // prologue

    // The wave's table entry stays held across its items while they run one
    // slot (a single-key batch acquires it once; wslot / went in LDS, not
    // SGPRs, which are spent): an item of the held slot skips the slot's
    // suite lookup and the entry's acquisition.
#pragma unroll 1
    for (;;) {
        uint32_t j = 0;
        if (lane_fresh() == 0) j = atomicAdd(&sm.next, 1u);
        j = __builtin_amdgcn_readfirstlane(j);
        if (j >= se) {
            // the share is done: the launch's pool (bounded: each grab
            // takes a new ticket)
            if (!pool) break;
            uint32_t q = 0;
            if (lane_fresh() == 0) q = atomicAdd(&pool[0], 1u);
            q = __builtin_amdgcn_readfirstlane(q);
            if (q >= pool_n) break;
            j = ib + stat + q;
        }
#if QPP_COMBO_PRIO
        uint32_t pbase = 0u;
        if constexpr (WG == 512) pbase = (j < se && 2u * (se - j) > se - sb) ? 2u : 0u;
#endif
#if QPP_SHARE_PRIO
        if constexpr (WG == 512) {
            // the two workgroups of a CU progress through their shares
            // together: the one with more of its share left issues first
            // (pooled items, at the launch's end, at the bottom)
            const uint32_t tot = se - sb, rem = j < se ? se - j : 0u;
            const uint32_t pr = tot ? min(3u, (4u * rem) / (tot + 1u)) : 0u;
            if (pr >= 3) __builtin_amdgcn_s_setprio(3);
            else if (pr == 2) __builtin_amdgcn_s_setprio(2);
            else if (pr == 1) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
#endif
        QPP_PROBE_AT(1);  // the previous item's tail, the grab
        QPP_PROBE_COUNT();
        // the item's positions [wb, we) of desc
        uint32_t wb, we;
        if (planned) {
            wb = __builtin_amdgcn_readfirstlane(items[j]);
            we = __builtin_amdgcn_readfirstlane(items[j + 1]);
        } else {
            wb = 16u * j;
            we = min(n, wb + 16u);
        }
        auto pkt_of = [&](uint32_t t) -> uint32_t { return wb + ((t & 63) >> 2); };
        // a lane's key slot, or kNoSlot (no packet, or a slot beyond the table)
        auto slot_of = [&](const qpp_desc &d, uint32_t p) -> uint32_t {
            return (p < we && d.slot < cap) ? d.slot : kNoSlot;
        };
        // 32-bit buffer views based at the item's lowest input / output
        // offsets (an item's packets must lie within 4 GiB of each other);
        // slots beyond the table: KeyUnavailableError
        uint64_t bi, bo;
        {
            const uint32_t t = tid_now(), p = pkt_of(t);
            uint64_t in0 = ~0ull, out0 = ~0ull;
            if (p < we) {
                const qpp_desc d = QPP_DESC(p);
                in0 = d.in_off;
                out0 = d.out_off;
                if (d.slot >= cap && (t & 3) == 0) res[planned ? d.rsv : p] = qpp_result{d.pn, QPP_S_NO_KEY, 0, 0};
            }
            bi = wave_min_u64(in0);
            bo = wave_min_u64(out0);
        }

        // The packets of one key slot `cur` among the item's
        auto run_slot = [&](uint32_t cur) {
            const KeySlot *ks = slots + cur;
            const uint32_t t1 = tid_now(), p1 = pkt_of(t1);
            const qpp_desc d = p1 < we ? QPP_DESC(p1) : qpp_desc{0, 0, 0, 0, 0, 0, kNoSlot, 0};
            if (slot_of(d, p1) != cur) return;  // the lambda's only early exit, at its top
#ifdef QPP_STUDY_SYNTH
            const HdrPre pre = {{0x41u, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, 0x41u};
#else
            const HdrPre pre = prefetch_hdr<ENC>(d, gin, true);
#endif
            const LdsTe T{sm.te, (t1 & 31) * 4};
            Pkt P = pkt_begin<ENC, SUITE>(d, pre, gin, gout, ks, T);
            if (P.status == QPP_S_OK) {
                // plain keys for rounds 0-2 (counter cache) and NR, rotated between
                uint32_t rk[4 * (kNR + 1)];
#pragma unroll
                for (int i = 0; i < 4 * (kNR + 1); ++i)
                    rk[i] = __builtin_amdgcn_readfirstlane((i >= 12 && i < 4 * kNR) ? ks->rkr[i] : ks->rk[i]);
                const uint64_t ioff = d.in_off - bi, ooff = d.out_off - bo;
                const uint64_t rlen = (uint64_t)(P.hlen + P.clen + (ENC ? 0 : QPP_TAG_LEN));
                const uint64_t wlen = (uint64_t)(P.hlen + P.clen + QPP_TAG_LEN);
                if (ioff + rlen <= kBufBytes && ooff + wlen <= kBufBytes) {
                    const Bufs B{
                        __builtin_amdgcn_make_buffer_rsrc((void *)(gin + bi), 0, (int)kBufBytes, 0x00020000),
                        __builtin_amdgcn_make_buffer_rsrc((void *)(gout + bo), 0, (int)kBufBytes, 0x00020000)};
                    const GhashTabs G{&sm.h4[0][0], gtab, &sm.wslot[wv], &sm.went[wv]};
                    QPP_PROBE_AT(3);
                    // unprotect: what the results need after the loop
                    const uint64_t pn = P.pn;
                    const int hlen = P.hlen;
                    u32x4 got_tag;
                    const u32x4 tag = gcm_packet<kNR, ENC, BPL, SUITE, WG == 512 && QPP_PRIO512>(P, ks, pre.h0, rk, t1 & 3, G, sm.te, B,
                                                                       (uint32_t)ioff, (uint32_t)ooff, got_tag
#if QPP_COMBO_PRIO
                                                                       , pbase
#endif
                                                                       );
                    QPP_PROBE_AT(6);
                    // everything below is re-derived after the step loop
                    const uint32_t t2 = tid_now(), p2 = pkt_of(t2);
                    const qpp_desc d2 = QPP_DESC(p2);
                    Pkt Q;
                    Q.src = gin + d2.in_off;
                    Q.dst = gout + d2.out_off;
                    Q.hp = !(d2.flags & QPP_F_NO_HP);
                    Q.status = QPP_S_OK;
                    Q.hlen = ENC ? (int)d2.hdr_len : hlen;
                    Q.clen = ENC ? (int)d2.len : (int)d2.len - hlen - QPP_TAG_LEN;
                    Q.pn = ENC ? d2.pn : pn;
                    Q.pn_off = Q.pn_len = 0;
                    Q.fbm = 0;
                    Q.mask = zero4();
                    Q.nonce = zero4();
                    const LdsTe T2{sm.te, (t2 & 31) * 4};
                    const KeySlot *ks2 =
                        slots + __builtin_amdgcn_readfirstlane(lds_ld(&sm.wslot[wv]));
                    gcm_finish<ENC, SUITE, BPL>(Q, ks2, t2 & 3, T2, tag, got_tag);
                    P = Q;
                } else {
                    P.status = QPP_S_LENGTH;  // the item spans more than 4 GiB
                }
            }
            const uint32_t t3 = tid_now(), p3 = pkt_of(t3);
            write_result<ENC>(res, planned ? QPP_DESC(p3).rsv : p3, t3 & 3, P);
            QPP_PROBE_AT(7);
        };

        // slot by slot among the item's packets, lowest first (planned: one);
        // bounded: an item holds at most 16 distinct slots (watchdog against
        // a logic error turning into a hung GPU)
        uint32_t last = kNoSlot;
#pragma unroll 1
        for (int guard = 0; guard < 17; ++guard) {
            const uint32_t t = tid_now(), p = pkt_of(t);
            const uint32_t s = p < we ? slot_of(QPP_DESC(p), p) : kNoSlot;
            const uint32_t cur = wave_min_u32((last == kNoSlot || s > last) ? s : kNoSlot);
            if (cur == kNoSlot) break;
            last = cur;
            // no packet of the item on a later slot: this slot is its last, so
            // the loop ends after it without reading the descriptors again
            // (a load there would wait behind the item's stores)
            const bool final_slot = __builtin_amdgcn_ballot_w64(s != kNoSlot && s > cur) == 0;
            const uint32_t held = __builtin_amdgcn_readfirstlane(lds_ld(&sm.wslot[wv]));
            const uint32_t suite =
                cur == held ? (uint32_t)SUITE : __builtin_amdgcn_readfirstlane(slots[cur].suite);
            // a status for every packet of the slot instead of running them
            uint32_t fail = 0u;
            if (suite > QPP_CHACHA20_POLY1305) {
                fail = QPP_S_NO_KEY;  // an empty slot: KeyUnavailableError (every suite's launch writes it)
            } else if (suite != SUITE) {
                continue;  // another suite's launch
            } else if (cur != held) {
                QPP_PROBE_AT(1);
                // release before acquiring: a wave never waits holding an entry
                if (held != kNoSlot) {
                    tab_release<WG>(sm, __builtin_amdgcn_readfirstlane(lds_ld(&sm.went[wv])));
                    if (lane_fresh() == 0) lds_st(&sm.wslot[wv], kNoSlot);
                }
                const uint32_t e = tab_acquire<WG>(sm, gtab, cur);
                if (e == kNoSlot) {
                    // the watchdog gave up: the slot's packets are not
                    // processed and report QPP_S_INTERNAL (no stale result
                    // from an earlier launch survives); the launch also
                    // counts the event (qpp_watchdog_count)
                    if (lane_fresh() == 0) atomicAdd(&g_qpp_watchdog, 1u);
                    fail = QPP_S_INTERNAL;
                } else if (lane_fresh() == 0) {
                    lds_st(&sm.wslot[wv], cur);
                    lds_st(&sm.went[wv], e);
                }
            }
            if (fail) {
                if (s == cur && (t & 3) == 0) {
                    const qpp_desc d = QPP_DESC(p);
                    res[planned ? d.rsv : p] = qpp_result{d.pn, (uint16_t)fail, 0, 0};
                }
                continue;
            }
            QPP_PROBE_AT(2);  // table entry
            run_slot(cur);
            QPP_PROBE_AT(8);
            if (final_slot) break;
        }
    }
    if (__builtin_amdgcn_readfirstlane(lds_ld(&sm.wslot[wv])) != kNoSlot)
        tab_release<WG>(sm, __builtin_amdgcn_readfirstlane(lds_ld(&sm.went[wv])));
    // the last wave of the last workgroup zeroes the pool for its next launch
    // (every wave has taken its last ticket by then)
    if (pool && lane_fresh() == 0 && atomicAdd(&sm.exited, 1u) == (uint32_t)(WG / 64 - 1) &&
        atomicAdd(&pool[1], 1u) == gridDim.x - 1) {
        atomicExch(&pool[0], 0u);
        atomicExch(&pool[1], 0u);
    }
    QPP_PROBE_AT(9);
}

// The packets of one wave: positions [b, e) of desc.  Unplanned: 16
// consecutive positions per wave.  Planned: the wave's item of the plan (<= 16
// positions on one key slot, qpp_plan.hip).  empty_wg: the whole workgroup is
// past the batch / the suite's items (uniform, so it may return before any
// barrier).
struct WaveSpan {
    uint32_t b, e;
    bool empty_wg;
};
template <int WG, int SUITE>
__device__ __forceinline__ WaveSpan wave_span(uint32_t n, const uint32_t *items, const uint32_t *irange,
                                              uint32_t wv, uint32_t blk)
{
    constexpr uint32_t kWaves = WG / 64;
    WaveSpan w{0u, 0u, false};
    if (irange) {
        const uint32_t ib = irange[2 * SUITE], ie = irange[2 * SUITE + 1];
        const uint32_t j0 = ib + blk * kWaves;
        w.empty_wg = j0 >= ie;
        const uint32_t j = j0 + wv;
        if (j < ie) {
            w.b = __builtin_amdgcn_readfirstlane(items[j]);
            w.e = __builtin_amdgcn_readfirstlane(items[j + 1]);
        }
    } else {
        const uint32_t b0 = blk * (kWaves * 16u);
        w.empty_wg = b0 >= n;
        w.b = b0 + wv * 16u;
        w.e = w.b < n ? min(n, w.b + 16u) : w.b;
    }
    return w;
}

// ChaCha20-Poly1305: no tables, so every wave runs its packets slot by slot
// on its own, with the keys read from the slot (scalar loads).  One wave
// item W (<= 16 packets) of k_chacha.
template <bool ENC, int WG, bool PRIO>
__device__ __forceinline__ void chacha_wave(const WaveSpan &W, ChachaSmem<WG> &sm, const KeySlot *__restrict__ slots,
                                            uint32_t cap, const qpp_desc *__restrict__ desc, const uint8_t *gin,
                                            uint8_t *gout, qpp_result *__restrict__ res,
                                            const uint32_t *__restrict__ irange)
{
    constexpr int SUITE = QPP_CHACHA20_POLY1305;
#ifdef QPP_CH_STAGGER
    {
        // study: waves start QPP_CH_STAGGER x 64 cycles apart by their slot in the SIMD
        const uint32_t slot = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (3 << 11));
        for (uint32_t i = 0; i < slot * QPP_CH_STAGGER; ++i) __builtin_amdgcn_s_sleep(1);
    }
#endif
    QPP_PROBE_AT(kProbeStart);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);  // set-up and key block: every wave at the top
    const uint32_t lim = W.e, planned = irange != nullptr;
    // the lane's packet and quad lane, re-derived from a fresh lane id where
    // used (held across the slot loop, the thread id is spilled at 128 VGPRs)
    auto p_now = [&]() -> uint32_t { return W.b + (lane_fresh() >> 2); };
    auto sub_now = [&]() -> uint32_t { return lane_fresh() & 3; };
    const uint32_t p1 = p_now();
    // 32-bit buffer views based at the wave's lowest input / output offsets
    // (a wave's packets must lie within 4 GiB of each other, as for GCM)
    uint64_t bi, bo;
    {
        uint64_t in0 = ~0ull, out0 = ~0ull;
        if (p1 < lim) {
            const qpp_desc d = desc[p1];
            in0 = d.in_off;
            out0 = d.out_off;
            if (d.slot >= cap && sub_now() == 0) res[planned ? d.rsv : p1] = qpp_result{d.pn, QPP_S_NO_KEY, 0, 0};
        }
        bi = wave_min_u64(in0);
        bo = wave_min_u64(out0);
    }
    // slot by slot among the wave's packets, lowest first (usually one); the
    // descriptor is re-read each time rather than kept live (VGPRs)
    // (bounded: a wave holds at most 16 distinct slots; structured, with no
    // continue, so every lane reaches the loop's end each trip)
    uint32_t last = kNoSlot;
    #pragma unroll 1
    for (int guard = 0; guard < 17; ++guard) {
        const uint32_t pl = p_now();
        const uint32_t s = pl < lim ? desc[pl].slot : kNoSlot;
        const uint32_t cur = wave_min_u32(s < cap && (last == kNoSlot || s > last) ? s : kNoSlot);
        if (cur == kNoSlot) break;
        const KeySlot *ks = slots + cur;
        const uint32_t suite = ks->suite;
        if (s == cur && suite > QPP_CHACHA20_POLY1305 && sub_now() == 0) {
            const qpp_desc d = desc[pl];
            res[planned ? d.rsv : pl] = qpp_result{d.pn, QPP_S_NO_KEY, 0, 0};
        }
        if (s == cur && suite == SUITE) {
            const qpp_desc d = desc[pl];
            const HdrPre pre = prefetch_hdr<ENC>(d, gin, true);
            const ConstTe T;
            Pkt P = pkt_begin<ENC, SUITE>(d, pre, gin, gout, ks, T);
            // lane-derived values from a fresh lane id: derived from t1 they
            // would be hoisted out of the loop and held live across it
            const uint32_t tf = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) << 6 | lane_fresh();
            const uint64_t ioff = d.in_off - bi, ooff = d.out_off - bo;
            if (P.status == QPP_S_OK &&
                (ioff + (uint64_t)(P.hlen + P.clen + QPP_TAG_LEN) > kBufBytes ||
                 ooff + (uint64_t)(P.hlen + P.clen + QPP_TAG_LEN) > kBufBytes))
                P.status = QPP_S_LENGTH;  // the wave's packets span more than 4 GiB
            if (P.status == QPP_S_OK) {
                *(u32x4 *)(sm.scratch[tf >> 2] + kScrHdr) = pre.h0;
                const Bufs B{
                    __builtin_amdgcn_make_buffer_rsrc((void *)(gin + bi), 0, (int)kBufBytes, 0x00020000),
                    __builtin_amdgcn_make_buffer_rsrc((void *)(gout + bo), 0, (int)kBufBytes, 0x00020000)};
                chacha_packet<ENC, PRIO>(P, ks, tf & 3, sm.scratch[tf >> 2], sm.stage[tf >> 6], sm.pw[tf >> 2], B, (uint32_t)ioff,
                                   (uint32_t)ooff);
            }
            const uint32_t pr = p_now();
            write_result<ENC>(res, planned ? desc[pr].rsv : pr, lane_fresh() & 3, P);
        }
        last = cur;
    }
    QPP_PROBE_AT(9);
}

#ifndef QPP_CH_PERSIST
#define QPP_CH_PERSIST 0  // study switch: > 0 = grid capped at that many rounds of resident workgroups, each looping
#endif
template <bool ENC, int WG, bool PRIO>
__global__ __launch_bounds__(WG, kChachaWpe) void k_chacha(const KeySlot *__restrict__ slots,
                                                             uint32_t cap,
                                                             const qpp_desc *__restrict__ desc,
                                                             uint32_t n, const uint8_t *gin,
                                                             uint8_t *gout,
                                                             qpp_result *__restrict__ res,
                                                             const uint32_t *__restrict__ items,
                                                             const uint32_t *__restrict__ irange)
{
    constexpr int SUITE = QPP_CHACHA20_POLY1305;
    __shared__ ChachaSmem<WG> sm;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if QPP_CH_PERSIST
    // study: each wave walks the blocks blockIdx.x, + gridDim.x, ... on its
    // own (no barrier: a wave that ends its item takes the next at once)
#pragma unroll 1
    for (uint32_t vb = blockIdx.x;; vb += gridDim.x) {
        const WaveSpan W = wave_span<WG, SUITE>(n, items, irange, wv, vb);
        if (W.empty_wg) break;
        chacha_wave<ENC, WG, PRIO>(W, sm, slots, cap, desc, gin, gout, res, irange);
    }
#else
    const WaveSpan W = wave_span<WG, SUITE>(n, items, irange, wv, blockIdx.x);
    if (W.empty_wg) return;
    chacha_wave<ENC, WG, PRIO>(W, sm, slots, cap, desc, gin, gout, res, irange);
#endif
}

// ----------------------------------------------------------- lone packets --
//
// A launch of a few packets -- the object API, one packet per call
// (AEAD.encrypt / decrypt, _crypto.c:157-194 / :115-155, through
// CryptoContext, quic/crypto.py:75-116) -- is bound by latency, not by
// throughput: the quad kernels walk a 1200-byte packet in ~10 dependent steps
// (k_gcm: ~38 us for one packet, profiles/r3o_latency).  Here one wave takes
// one packet and all of its blocks at once: AES-GCM gives every lane 1-3 of
// the packet's 16-byte blocks, ChaCha20-Poly1305 one 64-byte chunk (or 4
// blocks of associated data).  The authenticator is then
//   sum_i X_i K^(m - i)   over the m blocks [AAD | CT | lengths],
// each lane multiplying its blocks by their own power of K (H^e from the
// slot's power table, r^e by square-and-multiply), and one wave reduction.
// Launches stay latency-bound up to a few thousand packets (one workgroup
// of 16 packets per CU), so unplanned launches up to lone_max take these
// kernels; past that the quad kernels' ~7x fewer instructions per packet win.
constexpr int kLoneWG = 1024;      // 16 packets per workgroup, one AES image

// A small host call handed to a lone kernel whole (qpp_session): the kernel
// copies the call's descriptors and input from the pinned staging (src, its
// device view) into the device staging (dst) itself, every thread 16 bytes
// in one bus round trip, instead of a copy-engine blit scheduled between
// stream operations.  bytes == 0: nothing staged (device-buffer launches).
// One workgroup (at most 16 packets); the workgroup barrier makes the copy
// visible to its waves (vector L1 writes through to L2).
struct LoneStage {
    const uint8_t *src;
    uint8_t *dst;
    uint32_t bytes;  // multiple of 16, <= kLoneStageMax
};
constexpr uint32_t kLoneStageMax = 2 * kLoneWG * 16;

__device__ __forceinline__ void lone_stage_load(const LoneStage &st, u32x4 &a, u32x4 &b)
{
    const uint32_t o = threadIdx.x * 16u;
    a = o < st.bytes ? ld16(st.src + o) : zero4();
    b = o + kLoneWG * 16u < st.bytes ? ld16(st.src + o + kLoneWG * 16u) : zero4();
}

__device__ __forceinline__ void lone_stage_store(const LoneStage &st, u32x4 a, u32x4 b)
{
    const uint32_t o = threadIdx.x * 16u;
    if (o < st.bytes) st16(st.dst + o, a);
    if (o + kLoneWG * 16u < st.bytes) st16(st.dst + o + kLoneWG * 16u, b);
}

__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t v)
{
    v ^= dpp_mov<kDppQuadSwap1>(v);
    v ^= dpp_mov<kDppQuadSwap2>(v);
    v ^= dpp_mov<kDppHalfMirror>(v);
    v ^= dpp_mov<kDppMirror>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 16) ^
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
    v += dpp_mov<kDppQuadSwap1>(v);
    v += dpp_mov<kDppQuadSwap2>(v);
    v += dpp_mov<kDppHalfMirror>(v);
    v += dpp_mov<kDppMirror>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

__device__ __forceinline__ u32x4 readlane4(u32x4 v, int l)
{
    return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v.x, l), (uint32_t)__builtin_amdgcn_readlane((int)v.y, l),
                 (uint32_t)__builtin_amdgcn_readlane((int)v.z, l), (uint32_t)__builtin_amdgcn_readlane((int)v.w, l)};
}

// The packet's slot for a lone-packet launch of SUITE, as the quad kernels
// decide it: beyond the table or empty -> KeyUnavailableError (written by
// every suite's launch alike), another suite -> that suite's launch.
template <int SUITE>
__device__ __forceinline__ bool lone_slot(const qpp_desc &d, const KeySlot *slots, uint32_t cap,
                                          qpp_result *res, uint32_t p)
{
    bool none = d.slot >= cap;
    if (!none) {
        const uint32_t suite = __builtin_amdgcn_readfirstlane(slots[d.slot].suite);
        if (suite != (uint32_t)SUITE) {
            if (suite <= QPP_CHACHA20_POLY1305) return false;
            none = true;
        }
    }
    if (none) {
        if (lane_fresh() == 0) res[p] = qpp_result{d.pn, QPP_S_NO_KEY, 0, 0};
        return false;
    }
    return true;
}

// Protect with header protection: the sample from ct[0, 32) staged by the
// lanes of CT blocks 0 and 1 (and the tag, for ciphertexts under 32 bytes),
// the mask by every quad, the header out by the lanes of its blocks.
template <int SUITE, class TE>
// own / own_ok: header block `lane` as the lane loaded it already (no reload
// on the call's path); have_mask / mask: the mask computed by the caller.
__device__ __forceinline__ void lone_protect_hp(Pkt &P, const KeySlot *ks, uint8_t *scr, u32x4 tag,
                                                const TE &T, u32x4 own, bool own_ok, bool have_mask = false,
                                                u32x4 mask = {0, 0, 0, 0})
{
    const uint32_t lane = lane_fresh();
    if (have_mask) {
        P.mask = mask;  // computed by the caller from the ciphertext
    } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (P.clen < 32 && lane == 0)
            for (int j = 0; j < 16 && P.clen + j < 32; ++j) scr[P.clen + j] = (uint8_t)byte_of(tag, j);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        P.mask = hp_mask_quad<SUITE>(ks, lds_sample(scr, 4 - P.pn_len), T, (int)(lane & 3));
    }
    const int n_a = (P.hlen + 15) >> 4;
    for (int q = (int)lane; q < n_a; q += 64) {
        const int nb = min(16, P.hlen - 16 * q);
        u32x4 h = (own_ok && q == (int)lane) ? keep_bytes(own, nb)
                                              : ld_win(P.src + 16 * q, nb, P.src, P.src + P.hlen + P.clen);
        h ^= hp_pattern(16 * q, P.mask, P.fbm, P.pn_off, P.pn_len);
        st_part(P.dst + 16 * q, h, nb);
    }
}

__device__ __forceinline__ u32x4 gf_mul(u32x4 x, u32x4 y)
{
    const gf::Blk z = gf::mul(gf::Blk{{x.x, x.y, x.z, x.w}}, gf::Blk{{y.x, y.y, y.z, y.w}});
    return u32x4{z.w[0], z.w[1], z.w[2], z.w[3]};
}

// One AES-GCM packet per wave (SP 800-38D; _crypto.c:157-204 / :115-155).
// Lane l takes sequence positions l and l + 64 (and l + 128 beyond 128
// blocks: long associated data): every load is issued before the first
// use, both counter blocks run as one aes_ctr2 chain, and the two GHASH
// terms are independent table-free multiplies (qpp_gf128.h).
// A launch of at most 8 packets (the object API's calls) gives each packet
// two waves instead ("pair"): wave 2k + h takes positions 64 h + l
// (+ 128 j), so a lane multiplies once where one wave would multiply twice;
// wave 2k + 1 hands its share of the tag over through LDS.  Protect: wave 2k
// computes the header-protection mask while wave 2k + 1 finishes its
// multiplies.  Unprotect: wave 2k hands the verdict back, and on a failed tag
// each wave zeroes the plaintext blocks it wrote (stores of one wave to one
// address stay in order; another wave's could overtake them).
template <int SUITE, bool ENC>
// (desc is not __restrict__: with a staged call it is the copy this kernel
// writes, so its loads must not move above the staging)
__global__ __launch_bounds__(kLoneWG) void k_lone_gcm(const KeySlot *__restrict__ slots,
                                                      const uint8_t *__restrict__ gtab, uint32_t cap,
                                                      const qpp_desc *desc, uint32_t n,
                                                      const uint8_t *gin, uint8_t *gout,
                                                      qpp_result *__restrict__ res, LoneStage st)
{
    constexpr int kNR = SUITE == QPP_AES_256_GCM ? 14 : 10;
    __shared__ __attribute__((aligned(16))) uint8_t te[kTeBytes];
    __shared__ __attribute__((aligned(16))) uint8_t scr[kLoneWG / 64][48];
    // pair launches: the second wave's share of a packet's tag, and its flag
    __shared__ u32x4 xch[kLoneWG / 128];
    __shared__ uint32_t xflag[kLoneWG / 128];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool pair = n <= (uint32_t)(kLoneWG / 128);  // uniform over the launch
    const int part = pair ? (int)(wv & 1u) : 0;
    const uint32_t ps = pair ? wv >> 1 : wv;  // the packet's index in the workgroup
    const uint32_t p = pair ? ps : blockIdx.x * (kLoneWG / 64) + wv;  // (pair: one workgroup)
    const bool live = p < n;
    qpp_desc d = {0, 0, 0, 0, 0, 0, kNoSlot, 0};
    QPP_PROBE_AT(kProbeStart);
    if (threadIdx.x < kLoneWG / 128) xflag[threadIdx.x] = 0u;
    if (st.bytes) {
        // the call's bytes in flight beside the AES image build
        u32x4 a, b;
        lone_stage_load(st, a, b);
        load_te<kLoneWG>(te);
        lone_stage_store(st, a, b);
        QPP_PROBE_AT(0);  // staging read, AES image
        __syncthreads();
        if (live) d = desc[p];
    } else {
        // the descriptor is requested before the AES image is built
        if (live) d = desc[p];
        load_te<kLoneWG>(te);
        __syncthreads();
    }
    QPP_PROBE_AT(1);  // barrier, descriptor
    if (!live || !lone_slot<SUITE>(d, slots, cap, res, p)) return;
    QPP_PROBE_AT(2);  // the slot's suite
    const KeySlot *ks = slots + d.slot;
    const uint32_t lane = lane_fresh();
    const LdsTe T{te, (lane & 31) * 4};
    const HdrPre pre = prefetch_hdr<ENC>(d, gin, true);
    Pkt P = pkt_begin<ENC, SUITE>(d, pre, gin, gout, ks, T);
    QPP_PROBE_AT(3);  // header, pkt_begin (unprotect: header protection)
    if (P.status == QPP_S_OK) {
        const int hlen = P.hlen, clen = P.clen;
        const int n_a = (hlen + 15) >> 4, n_c = (clen + 15) >> 4, m = n_a + n_c + 1;
        const int rlen = hlen + clen + (ENC ? 0 : QPP_TAG_LEN);
        const uint8_t *src = P.src;
        uint8_t *dst = P.dst;
        const uint8_t *hpw = gtab + gh_powers_off(cap, d.slot);
        const bool masked = !ENC && P.hp;
        // a position's input block (AAD or CT; zero otherwise), its power of H
        auto input = [&](int pos) -> u32x4 {
            if (pos < n_a) return ld_win(src + 16 * pos, min(16, hlen - 16 * pos), src, src + rlen);
            const int i = pos - n_a;
            if (i < n_c) return ld_win(src + hlen + 16 * i, min(16, clen - 16 * i), src, src + rlen);
            return zero4();
        };
        auto power = [&](int pos) -> u32x4 { return pos < m ? ld16(hpw + 16 * (m - 1 - pos)) : zero4(); };
        const int stride = pair ? 128 : 64;
        const int pos0 = (int)lane + 64 * part, pos1 = pos0 + stride;
        const u32x4 in0 = input(pos0), in1 = input(pos1), h0 = power(pos0), h1 = power(pos1);
        uint32_t rk[4 * (kNR + 1)];
#pragma unroll
        for (int i = 0; i < 4 * (kNR + 1); ++i)
            rk[i] = __builtin_amdgcn_readfirstlane((i >= 12 && i < 4 * kNR) ? ks->rkr[i] : ks->rk[i]);
        const CtrCache cc = ctr_cache(P.nonce, rk, T);
        QPP_PROBE_AT(4);  // inputs and powers requested, round keys, counter cache
        // CT block i: counter i + 2; the lengths position: J0 (counter 1)
        auto ctr = [&](int pos) -> uint32_t {
            return (pos >= n_a && pos < n_a + n_c) ? (uint32_t)(pos - n_a + 2) : 1u;
        };
        // a position's output and GHASH input given its keystream
        u32x4 ej0 = zero4();
        auto out = [&](int pos, u32x4 in, u32x4 ksb) -> u32x4 {
            u32x4 x = zero4();
            if (pos < n_a) {
                x = in;
                if (masked) x ^= hp_pattern(16 * pos, P.mask, P.fbm, P.pn_off, P.pn_len);
                if (!ENC || !P.hp) st_part(dst + 16 * pos, x, min(16, hlen - 16 * pos));
            } else if (pos < n_a + n_c) {
                const int i = pos - n_a, nb = min(16, clen - 16 * i);
                const u32x4 o = in ^ ksb;
                st_part(dst + hlen + 16 * i, o, nb);
                x = keep_bytes(ENC ? o : in, nb);
                if (ENC && P.hp && i < 2) *(u32x4 *)(scr[ps] + 16 * i) = x;
            } else if (pos == m - 1) {
                x = u32x4{0u, bswap((uint32_t)hlen * 8u), 0u, bswap((uint32_t)clen * 8u)};
                ej0 = ksb;
            }
            return x;
        };
        u32x4 ks0, ks1;
        aes_ctr2<kNR>(cc, ctr(pos0), ctr(pos1), rk, T, ks0, ks1);
        QPP_PROBE_AT(5);  // AES-CTR
        const u32x4 x0 = out(pos0, in0, ks0), x1 = out(pos1, in1, ks1);
        QPP_PROBE_AT(6);  // output stores, the inputs' wait
        // pair, first wave: the header-protection mask from CT blocks 0-1
        // (its lanes n_a, n_a + 1) before the multiplies, beside the second
        // wave's; otherwise after the tag (lone_protect_hp)
        const bool hp_early = pair && part == 0 && P.hp && clen >= 20 && n_a + 1 < 64;
        u32x4 hp_mask = zero4();
        if (hp_early) {
            const int na = __builtin_amdgcn_readfirstlane(n_a), sh = 4 - P.pn_len;
            const u32x4 c0 = readlane4(x0, na), c1 = readlane4(x0, na + 1);
            const u32x4 smp = {__builtin_amdgcn_alignbyte(c0.y, c0.x, sh), __builtin_amdgcn_alignbyte(c0.z, c0.y, sh),
                               __builtin_amdgcn_alignbyte(c0.w, c0.z, sh), __builtin_amdgcn_alignbyte(c1.x, c0.w, sh)};
            hp_mask = hp_mask_quad<SUITE>(ks, smp, T, (int)(lane & 3));
        }
        u32x4 y = gf_mul(x0, h0);
        // the second term only where some lane holds a second position
        if (__builtin_amdgcn_ballot_w64(pos1 < m) != 0) y ^= gf_mul(x1, h1);
        for (int pos = pos1 + stride; pos < m; pos += stride)  // long associated data
            y ^= gf_mul(out(pos, input(pos), aes_ctr<kNR>(cc, ctr(pos), rk, T)), power(pos));
        // (the lane of position m - 1 holds E_K(J0) in its wave; zero elsewhere)
        u32x4 tag = u32x4{wave_xor_u32(y.x), wave_xor_u32(y.y), wave_xor_u32(y.z), wave_xor_u32(y.w)} ^
                    readlane4(ej0, (m - 1) & 63);
        // a wave's plaintext blocks, zeroed after a failed tag (unprotect)
        auto wipe_own = [&]() {
            for (int pos = pos0; pos < m; pos += stride) {
                const int i = pos - n_a;
                if (i >= 0 && i < n_c) st_part(dst + hlen + 16 * i, zero4(), min(16, clen - 16 * i));
            }
        };
        // The hand-over's flag (pair launches), moved only by compare-and-swap
        // so that a wave that gives up cannot be overwritten by the other:
        // 0 start, 1 the second wave's share is in xch, 2 / 3 the first
        // wave's verdict (unprotect: tag ok / failed), 4 the first wave gave
        // up waiting for the share, 5 the second wave gave up waiting for the
        // verdict.  Both waves are resident in one workgroup, so the bounded
        // waits (g_qpp_spin_lone sleeps: milliseconds) are a watchdog that a
        // correct run never reaches; when one fires, the packet reports
        // QPP_S_INTERNAL and unprotect zeroes its plaintext on both sides.
        auto flag_cas = [&](uint32_t from, uint32_t to) -> uint32_t {
            uint32_t prev = from;
            if (lane == 0)
                __hip_atomic_compare_exchange_strong(&xflag[ps], &prev, to, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
            return __builtin_amdgcn_readfirstlane(prev);
        };
        auto wait_flag = [&](uint32_t below) -> uint32_t {
            uint32_t f = 0u;
            const uint32_t spin = __builtin_nontemporal_load(&g_qpp_spin_lone);
            for (uint32_t it = 0; it < spin; ++it) {
                f = __hip_atomic_load(&xflag[ps], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (f >= below) break;
                __builtin_amdgcn_s_sleep(2);
            }
            return __builtin_amdgcn_readfirstlane(f);
        };
        bool handed = false;  // first wave: the second wave's share arrived
        if (pair) {
            if (part == 1) {
                {
                    const uint32_t dl = __builtin_nontemporal_load(&g_qpp_pair_delay);
                    for (uint32_t it = 0; it < dl; ++it) __builtin_amdgcn_s_sleep(127);
                }
                // hand the share over (and CT blocks 0-1 in scr, if this wave
                // wrote them); the release orders those stores before the flag
                if (lane == 0) xch[ps] = tag;
                const uint32_t prev = flag_cas(0u, 1u);
                if (!ENC) {
                    // unprotect: keep this wave's plaintext only on verdict 2
                    uint32_t f = prev;
                    if (prev == 0u) {
                        f = wait_flag(2u);
                        if (f < 2u) {
                            const uint32_t q = flag_cas(1u, 5u);
                            f = q == 1u ? 5u : q;
                        }
                    }
                    if (f != 2u) wipe_own();
                }
                return;  // the first wave writes the result
            }
            uint32_t f = wait_flag(1u);
            if (f < 1u) {
                const uint32_t q = flag_cas(0u, 4u);
                f = q == 0u ? 4u : q;
            }
            if (f == 1u) {
                handed = true;
                tag ^= xch[ps];
            } else {
                P.status = QPP_S_INTERNAL;
                if (lane == 0) atomicAdd(&g_qpp_watchdog, 1u);
            }
        }
        QPP_PROBE_AT(7);  // GHASH (powers' wait, multiplies, wave xor)
        if (ENC) {
            if (P.status == QPP_S_OK) {
                if (lane == 0) st16(dst + hlen + clen, tag);
                // (lane q of the first wave loaded header block q as its position q)
                if (P.hp)
                    lone_protect_hp<SUITE>(P, ks, scr[ps], tag, T, x0, part == 0 && (int)lane < n_a, hp_early,
                                           hp_mask);
            }
        } else {
            const u32x4 got = ld16(src + hlen + clen), diff = got ^ tag;
            bool bad = (diff.x | diff.y | diff.z | diff.w) != 0 || P.status != QPP_S_OK;
            if (handed && flag_cas(1u, bad ? 3u : 2u) != 1u) {
                // the second wave gave up waiting for the verdict (and wiped
                // its blocks): the packet fails here too
                P.status = QPP_S_INTERNAL;
                bad = true;
                if (lane == 0) atomicAdd(&g_qpp_watchdog, 1u);
            }
            if (bad) {
                if (P.status == QPP_S_OK) P.status = QPP_S_DECRYPT;
                wipe_own();
            }
        }
    }
    QPP_PROBE_AT(8);  // header protection, tag, header
    write_result<ENC>(res, p, (int)lane_fresh(), P);
    QPP_PROBE_AT(9);  // result
}

// One ChaCha20-Poly1305 packet per wave (RFC 8439 sec. 2.8).  Lane 0: the
// one-time key block; lane u = 1..24: chunk u - 1 (4 CT blocks); lane 32 + g:
// AAD blocks 4g..4g+3; lane 63: the lengths block.  Each lane folds its
// blocks by Horner in r and scales the result by r^e, e = m - (position of
// its last block); r^e by square-and-multiply beside the Horner chain; the
// 26-bit limbs of <= 49 terms sum without carries.  The lane's input blocks
// are requested before its ChaCha20 block.
template <bool ENC>
__global__ __launch_bounds__(kLoneWG) void k_lone_chacha(const KeySlot *__restrict__ slots, uint32_t cap,
                                                         const qpp_desc *desc, uint32_t n,
                                                         const uint8_t *gin, uint8_t *gout,
                                                         qpp_result *__restrict__ res, LoneStage st)
{
    constexpr int SUITE = QPP_CHACHA20_POLY1305;
    __shared__ __attribute__((aligned(16))) uint8_t scr[kLoneWG / 64][48];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t p = blockIdx.x * (kLoneWG / 64) + wv;
    QPP_PROBE_AT(kProbeStart);
    if (st.bytes) {
        u32x4 a, b;
        lone_stage_load(st, a, b);
        lone_stage_store(st, a, b);
        QPP_PROBE_AT(0);  // staging read
        __syncthreads();
    }
    if (p >= n) return;
    const qpp_desc d = desc[p];
    QPP_PROBE_AT(1);  // barrier, descriptor
    if (!lone_slot<SUITE>(d, slots, cap, res, p)) return;
    QPP_PROBE_AT(2);  // the slot's suite
    const KeySlot *ks = slots + d.slot;
    const uint32_t lane = lane_fresh();
    const ConstTe T;
    const HdrPre pre = prefetch_hdr<ENC>(d, gin, true);
    Pkt P = pkt_begin<ENC, SUITE>(d, pre, gin, gout, ks, T);
    QPP_PROBE_AT(3);  // header, pkt_begin (unprotect: header protection)
    if (P.status == QPP_S_OK) {
        const int hlen = P.hlen, clen = P.clen;
        const int n_a = (hlen + 15) >> 4, n_c = (clen + 15) >> 4, m = n_a + n_c + 1;
        const int chunks = (clen + 63) >> 6;
        const int rlen = hlen + clen + (ENC ? 0 : QPP_TAG_LEN);
        const uint8_t *src = P.src;
        uint8_t *dst = P.dst;
        // this lane's blocks: first sequence position q, count cnt
        const bool is_ct = lane >= 1 && (int)lane <= chunks;
        const int g = (int)lane - 32, c0 = 4 * ((int)lane - 1);
        int q = 0, cnt = 0;
        if (is_ct) {
            q = n_a + c0;
            cnt = min(4, n_c - c0);
        } else if (g >= 0 && 4 * g < n_a) {
            q = 4 * g;
            cnt = min(4, n_a - 4 * g);
        } else if (lane == 63) {
            q = m - 1;
            cnt = 1;
        }
        // the blocks' inputs first
        u32x4 in[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            in[b] = zero4();
            if (b < cnt && lane != 63) {
                const int j = is_ct ? hlen + 16 * (c0 + b) : 16 * (4 * g + b);
                const int nb = is_ct ? min(16, clen - 16 * (c0 + b)) : min(16, hlen - 16 * (4 * g + b));
                in[b] = ld_win(src + j, nb, src, src + rlen);
            }
        }
        uint32_t key[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) key[w] = __builtin_amdgcn_readfirstlane(ks->rk[w]);
        uint32_t blk[16];
        QPP_PROBE_AT(4);  // inputs requested, key
        chacha_block(key, lane, P.nonce.x, P.nonce.y, P.nonce.z, blk);
        QPP_PROBE_AT(5);  // the ChaCha20 block
        uint32_t kw[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) kw[w] = (uint32_t)__builtin_amdgcn_readlane((int)blk[w], 0);
        const P130 r = p130_r(kw[0], kw[1], kw[2], kw[3]);
        // r^e, e = m - (q + cnt - 1): lane j holds r^(j + 1) after an
        // inclusive prefix product over the wave (6 multiplies per lane), a
        // lane reads r^(1 + (e - 1) mod 64) from its lane by ds_bpermute and
        // multiplies by r^64 (lane 63's) once per 64 -- 7-8 multiplies where
        // square-and-multiply over 8 bits of e took 15
        const P130 one = {{1u, 0u, 0u, 0u, 0u}};
        P130 tp = r;
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            P130 u;
#pragma unroll
            for (int l = 0; l < 5; ++l) u.v[l] = (uint32_t)__shfl_up((int)tp.v[l], (unsigned)k);
            tp = p130_mul(tp, (int)lane >= k ? u : one);
        }
        const int e = cnt > 0 ? m - (q + cnt - 1) : 1;
        const int e1 = e - 1, hi = e1 >> 6;
        P130 re, r64;
#pragma unroll
        for (int l = 0; l < 5; ++l) {
            re.v[l] = (uint32_t)__shfl((int)tp.v[l], e1 & 63);
            r64.v[l] = (uint32_t)__builtin_amdgcn_readlane((int)tp.v[l], 63);
        }
        for (int h = 1; h <= 3; ++h)  // e <= 1 + 3 * 64 + 63 (m <= 190)
            if (__builtin_amdgcn_ballot_w64(hi >= h) != 0) re = p130_mul(re, hi >= h ? r64 : one);
        const bool masked = !ENC && P.hp;
        P130 w = p130_zero();
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            u32x4 x = zero4();
            if (b < cnt) {
                if (is_ct) {
                    const int i = c0 + b, nb = min(16, clen - 16 * i);
                    const u32x4 o = in[b] ^ u32x4{blk[4 * b], blk[4 * b + 1], blk[4 * b + 2], blk[4 * b + 3]};
                    st_part(dst + hlen + 16 * i, o, nb);
                    x = keep_bytes(ENC ? o : in[b], nb);
                    if (ENC && P.hp && i < 2) *(u32x4 *)(scr[wv] + 16 * i) = x;
                } else if (lane == 63) {
                    x = u32x4{(uint32_t)hlen, 0u, (uint32_t)clen, 0u};
                } else {
                    const int j = 4 * g + b;
                    x = in[b];
                    if (masked) x ^= hp_pattern(16 * j, P.mask, P.fbm, P.pn_off, P.pn_len);
                    if (!ENC || !P.hp) st_part(dst + 16 * j, x, min(16, hlen - 16 * j));
                }
            }
            // Horner: w = w r + M_b over the lane's blocks (one more block
            // than it has only multiplies zero)
            const P130 mb = p130_block(x);
            if (b < cnt) w = p130_add(b == 0 ? w : p130_mul(w, r), mb);
        }
        QPP_PROBE_AT(6);  // Horner and r^e, outputs
        w = p130_mul(w, re);
        P130 sum;
#pragma unroll
        for (int l = 0; l < 5; ++l) sum.v[l] = wave_sum_u32(w.v[l]);
        const u32x4 tag = p130_finish(sum, kw[4], kw[5], kw[6], kw[7]);
        QPP_PROBE_AT(7);  // scaling multiply, wave sum, tag
        if (ENC) {
            if (lane == 0) st16(dst + hlen + clen, tag);
            // (header block 0: requested with the descriptor, pre.h0)
            if (P.hp) lone_protect_hp<SUITE>(P, ks, scr[wv], tag, T, pre.h0, lane == 0 && hlen + clen >= 16);
        } else {
            const u32x4 got = ld16(src + hlen + clen), diff = got ^ tag;
            if ((diff.x | diff.y | diff.z | diff.w) != 0) {
                P.status = QPP_S_DECRYPT;
                if (is_ct)
                    for (int b = 0; b < cnt; ++b) {
                        const int i = c0 + b;
                        st_part(dst + hlen + 16 * i, zero4(), min(16, clen - 16 * i));
                    }
            }
        }
    }
    QPP_PROBE_AT(8);  // header protection, tag, header
    write_result<ENC>(res, p, (int)lane_fresh(), P);
    QPP_PROBE_AT(9);  // result
}

// Header-protection masks only (HeaderProtection_mask, _crypto.c:278-287).
constexpr int kMaskWG = 256;

__global__ __launch_bounds__(kMaskWG) void k_hp_mask(const KeySlot *__restrict__ slots,
                                                     uint32_t cap,
                                                     const uint32_t *__restrict__ sidx,
                                                     const uint8_t *__restrict__ samples,
                                                     uint32_t n, uint8_t *__restrict__ masks)
{
    __shared__ __attribute__((aligned(16))) uint8_t te[kTeBytes];
    const uint32_t i = blockIdx.x * kMaskWG + threadIdx.x;
    // the slot and sample are requested before the AES image is built (a
    // one-mask call is latency: HeaderProtection.apply / remove)
    uint32_t s = kNoSlot;
    u32x4 smp = {0, 0, 0, 0};
    if (i < n) {
        s = sidx[i];
        smp = ld16(samples + 16 * (size_t)i);
    }
    load_te<kMaskWG>(te);
    __syncthreads();
    const LdsTe T{te, (uint32_t)(threadIdx.x & 31) * 4};
    if (i >= n) return;
    u32x4 m = {0, 0, 0, 0};
    if (s < cap && slots[s].suite <= QPP_CHACHA20_POLY1305) m = hp_mask_any(slots + s, slots[s].suite, smp, T);
    st16(masks + 16 * (size_t)i, m);
}

// --------------------------------------------------------------- key setup --

// FIPS-197 sec. 5.2 in little-endian words (RotWord = rotr 8, Rcon in byte 0).
__device__ int expand_key(const uint8_t *key, int klen, uint32_t *rk)
{
    const int nk = klen / 4, nr = nk + 6;
    for (int i = 0; i < nk; ++i)
        rk[i] = key[4 * i] | (uint32_t)key[4 * i + 1] << 8 | (uint32_t)key[4 * i + 2] << 16 |
                (uint32_t)key[4 * i + 3] << 24;
    uint32_t rcon = 1;
    auto sub_word = [](uint32_t t) {
        return (uint32_t)c_aes.sbox[t & 255] | (uint32_t)c_aes.sbox[(t >> 8) & 255] << 8 |
               (uint32_t)c_aes.sbox[(t >> 16) & 255] << 16 | (uint32_t)c_aes.sbox[t >> 24] << 24;
    };
    for (int i = nk; i < 4 * (nr + 1); ++i) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = sub_word((t >> 8) | (t << 24)) ^ rcon;
            rcon = gf8_mul((uint8_t)rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = sub_word(t);
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return nr;
}

__device__ __forceinline__ uint32_t le32(const uint8_t *p)
{
    return p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// One workgroup per key: round keys / ChaCha keys, H = E_K(0^128), H^2..H^4
// and the 2048 GHASH table entries (AEAD_init + HeaderProtection_init).
__global__ __launch_bounds__(kSetupWG) void k_key_setup(KeySlot *__restrict__ slots,
                                                   uint8_t *__restrict__ gtab, uint32_t cap,
                                                   const qpp_key_material *__restrict__ km,
                                                   uint32_t n)
{
    __shared__ KeySlot ks;
    __shared__ u32x4 hpow[kGhashPowers];
    const qpp_key_material &m = km[blockIdx.x];
    if (m.slot >= cap) return;
    if (threadIdx.x == 0) {
        ks.suite = m.suite;
        ks.key_phase = m.key_phase & 1;
        ks.rsv = 0;
        for (int i = 0; i < 3; ++i) ks.iv[i] = le32(m.iv + 4 * i);
        ks.iv[3] = 0;
        for (int i = 0; i < 60; ++i) ks.rk[i] = ks.hrk[i] = ks.rkr[i] = 0;
        for (int i = 0; i < 4; ++i) ks.pad[i] = 0;
        if (m.suite == QPP_CHACHA20_POLY1305) {
            ks.nr = 0;
            for (int i = 0; i < 8; ++i) {
                ks.rk[i] = le32(m.key + 4 * i);
                ks.hrk[i] = le32(m.hp + 4 * i);
            }
        } else {
            const int klen = m.suite == QPP_AES_256_GCM ? 32 : 16;
            ks.nr = (uint32_t)expand_key(m.key, klen, ks.rk);
            expand_key(m.hp, klen, ks.hrk);
            for (int i = 0; i < 60; ++i) ks.rkr[i] = rotl(ks.rk[i], 16);
            const ConstTe CT;
            const u32x4 zero = {0, 0, 0, 0};
            const u32x4 h = ks.nr == 14 ? aes_encrypt<14>(zero, ks.rk, CT)
                                        : aes_encrypt<10>(zero, ks.rk, CT);
            hpow[0] = h;
            for (int p = 1; p < kGhashPowers; ++p) hpow[p] = gf128_mul_slow(hpow[p - 1], h);
        }
    }
    __syncthreads();
    KeySlot *dst = slots + m.slot;
    for (int i = threadIdx.x; i < (int)(sizeof(KeySlot) / 4); i += kSetupWG)
        ((uint32_t *)dst)[i] = ((const uint32_t *)&ks)[i];
    if (m.suite == QPP_AES_128_GCM || m.suite == QPP_AES_256_GCM) {
        // H^1 .. H^192 (k_lone) by doubling: H^(h + t + 1) = H^(t + 1) H^h
        __shared__ u32x4 hall[kGhPowCount];
        if (threadIdx.x < kGhashPowers) hall[threadIdx.x] = hpow[threadIdx.x];
        __syncthreads();
        for (int have = kGhashPowers; have < kGhPowCount; have *= 2) {
            const int t = threadIdx.x;
            if (t < have && have + t < kGhPowCount) hall[have + t] = gf128_mul_slow(hall[t], hall[have - 1]);
            __syncthreads();
        }
        u32x4 *hp = (u32x4 *)(gtab + gh_powers_off(cap, m.slot));
        for (int i = threadIdx.x; i < kGhPowCount; i += kSetupWG) hp[i] = hall[i];
        u32x4 *tab = (u32x4 *)(gtab + (size_t)m.slot * kGhashTabBytes);
        for (int e = threadIdx.x; e < kGhashPowers * 32 * 16; e += kSetupWG) {
            const int p = e >> 9, w = (e >> 4) & 31, v = e & 15;
            // element with nibble v at window w: byte w/2, low (w even) or high nibble
            uint32_t words[4] = {0, 0, 0, 0};
            const int byte = w >> 1;
            words[byte >> 2] = (uint32_t)(v << (4 * (w & 1))) << (8 * (byte & 3));
            tab[e] = gf128_mul_slow(u32x4{words[0], words[1], words[2], words[3]}, hpow[p]);
        }
        // H^4 in 5-bit windows (ghash_mul_lds5): entry e of window w = the
        // element with bits [5w, 5w + 5) = e, times H^4; low / high 8 bytes in
        // 256-byte rows w and kGh5Hi / 256 + w
        uint32_t *t5 = (uint32_t *)(gtab + (size_t)m.slot * kGhashTabBytes + kGh5Off);
        for (int i = threadIdx.x; i < kGh5Windows * 32; i += kSetupWG) {
            const int w = i >> 5, e = i & 31;
            uint32_t words[4] = {0, 0, 0, 0};
            for (int b = 0; b < 5; ++b) {
                const int bit = 5 * w + b;
                if (bit < 128 && ((e >> b) & 1)) words[bit >> 5] |= 1u << (bit & 31);
            }
            const u32x4 v = gf128_mul_slow(u32x4{words[0], words[1], words[2], words[3]}, hpow[3]);
            uint32_t *row = t5 + w * 64, *rhi = t5 + (kGh5Hi / 4) + w * 64;
            row[2 * e] = v.x;
            row[2 * e + 1] = v.y;
            rhi[2 * e] = v.z;
            rhi[2 * e + 1] = v.w;
        }
    }
}

// Batched derive_key_iv_hp (quic/crypto.py:34-56), one lane per connection:
// `updates` x "quic ku" (next_key_phase, :157-168), then key / iv / hp by
// HKDF-Expand-Label with the v1 or v2 labels.  Cold path (once per key).
constexpr int kDeriveWG = 64;

__global__ __launch_bounds__(kDeriveWG) void k_derive(const qpp_secret *__restrict__ sec,
                                                      uint32_t n,
                                                      qpp_key_material *__restrict__ km)
{
    const uint32_t i = blockIdx.x * kDeriveWG + threadIdx.x;
    if (i >= n) return;
    const qpp_secret &s = sec[i];
    const bool big = s.suite == QPP_AES_256_GCM;
    const int hl = big ? 48 : 32, klen = s.suite == QPP_AES_128_GCM ? 16 : 32;
    uint8_t secret[64];
    int len = s.secret_len;
    for (int j = 0; j < 64; ++j) secret[j] = j < len ? s.secret[j] : 0;
    qpp_hkdf::Hmac m;
    for (uint32_t u = 0; u < s.updates; ++u) {
        qpp_hkdf::hmac_init(m, big, secret, len);
        qpp_hkdf::expand_label(m, "quic ku", 7, hl, secret);
        len = hl;
    }
    qpp_hkdf::hmac_init(m, big, secret, len);
    qpp_key_material r;
    memset(&r, 0, sizeof(r));
    r.slot = s.slot;
    r.suite = s.suite;
    r.key_phase = s.key_phase & 1;
    if (s.flags & QPP_DERIVE_V2) {
        qpp_hkdf::expand_label(m, "quicv2 key", 10, klen, r.key);
        qpp_hkdf::expand_label(m, "quicv2 iv", 9, 12, r.iv);
        qpp_hkdf::expand_label(m, "quicv2 hp", 9, klen, r.hp);
    } else {
        qpp_hkdf::expand_label(m, "quic key", 8, klen, r.key);
        qpp_hkdf::expand_label(m, "quic iv", 7, 12, r.iv);
        qpp_hkdf::expand_label(m, "quic hp", 7, klen, r.hp);
    }
    km[i] = r;
}

__global__ void k_clear_slots(KeySlot *slots, const uint32_t *idx, uint32_t n, uint32_t cap)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && idx[i] < cap) slots[idx[i]].suite = 0xffu;
}

// PCIe copies by the GPU's own loads and stores (qpp_session's D2H legs, and
// H2D under QPP_H2D_KERNEL): range y of the launch copies n_y bytes from src_y
// to dst_y, one of them a pinned host buffer's device view, in 16-byte
// non-temporal accesses (D2H: posted PCIe writes; bytes at a range's unaligned
// ends one by one).  The runtime's D2H
// on the copy engines ran at 27-30 GB/s in some processes on these boxes and
// 56-57 GB/s in others, while this kernel ran at 53-54 GB/s in every one
// (tools/d2h_probe.hip, profiles/r6_host_path/d2h_probe.txt).
typedef unsigned int xfer_v4 __attribute__((ext_vector_type(4)));
constexpr int kXferWG = 256;
__global__ __launch_bounds__(kXferWG) void k_xfer(const uint8_t *__restrict__ s0, uint8_t *d0, size_t n0,
                                                const uint8_t *__restrict__ s1, uint8_t *d1, size_t n1)
{
    const uint8_t *src = blockIdx.y ? s1 : s0;
    uint8_t *dst = blockIdx.y ? d1 : d0;
    const size_t n = blockIdx.y ? n1 : n0;
    const size_t tid = (size_t)blockIdx.x * kXferWG + threadIdx.x, step = (size_t)gridDim.x * kXferWG;
    if ((((uintptr_t)src ^ (uintptr_t)dst) & 15) != 0) {  // never in the session (same offsets)
        for (size_t i = tid; i < n; i += step) dst[i] = src[i];
        return;
    }
    size_t head = (16 - ((uintptr_t)src & 15)) & 15;
    if (head > n) head = n;
    const size_t body = (n - head) >> 4, tail = n - head - 16 * body;
    if (tid < head) dst[tid] = src[tid];
    const xfer_v4 *s16 = (const xfer_v4 *)(src + head);
    xfer_v4 *d16 = (xfer_v4 *)(dst + head);
    for (size_t i = tid; i < body; i += step) __builtin_nontemporal_store(__builtin_nontemporal_load(&s16[i]), &d16[i]);
    if (tid < tail) dst[head + 16 * body + tid] = src[head + 16 * body + tid];
}

}  // namespace qpp

// ======================================================== host: C ABI ======

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <immintrin.h>
#include <pthread.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

using namespace qpp;

// Item-pool slots of the persistent GCM launches (k_gcm's pool argument):
// kPoolSlots counter pairs in device memory, one 128-byte line each, zero
// between launches.  A launch takes a slot whose previous launch has
// completed (its event, recorded on that launch's stream after it, has
// fired) and which no other launch holds, so launches on different streams
// or threads never share a slot; with none free the launch runs on static
// shares alone (pool = null).
constexpr int kPoolSlots = 32;
constexpr uint32_t kPoolStride = 32;  // uint32 per slot
struct PoolRing {
    std::mutex mu;
    uint32_t *d = nullptr;
    hipEvent_t ev[kPoolSlots] = {};
    uint8_t state[kPoolSlots] = {};  // 0 free, 1 held by a launch being enqueued, 2 event recorded
    int next = 0;
};

struct qpp_keytab {
    uint32_t cap;
    int device;
    KeySlot *d_slots;
    uint8_t *d_gtab;
    qpp_key_material *d_km;
    uint32_t km_cap;
    uint8_t *h_suite;      // host mirror: suite of every slot (0xff = empty)
    uint32_t n_suite[3];   // installed slots per suite
    PoolRing *pool;        // item pools of the GCM launches
};

// QPP_GCM_POOL=0 (a study switch, read once per process): static shares only.
static bool pool_choice()
{
    static const bool b = [] {
        const char *v = getenv("QPP_GCM_POOL");
        return !(v && v[0] == '0');
    }();
    return b;
}

// Launches that found every pool slot held and ran on static shares alone
// (qpp_pool_fallbacks; tests/test_gpu_pool.py).
static std::atomic<uint64_t> g_pool_fallbacks{0};

// A free pool slot (its counters zero) or -1.
static int pool_acquire(const qpp_keytab *kt)
{
    PoolRing *r = kt->pool;
    if (!r || !pool_choice()) return -1;
    std::lock_guard<std::mutex> l(r->mu);
    for (int i = 0; i < kPoolSlots; ++i) {
        const int sl = (r->next + i) % kPoolSlots;
        if (r->state[sl] == 1) continue;
        if (r->state[sl] == 2) {
            const hipError_t q = hipEventQuery(r->ev[sl]);
            if (q != hipSuccess) {
                (void)hipGetLastError();  // still in flight (hipErrorNotReady) or failed: not reusable now
                continue;
            }
        } else if (!r->ev[sl] && hipEventCreateWithFlags(&r->ev[sl], hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            r->ev[sl] = nullptr;
            continue;
        }
        r->state[sl] = 1;
        r->next = (sl + 1) % kPoolSlots;
        return sl;
    }
    g_pool_fallbacks.fetch_add(1, std::memory_order_relaxed);
    return -1;
}

// After the launch that held slot sl was enqueued on s: the slot is reusable
// once the event recorded here fires.  (Recorded whether or not the launch
// reported an error -- an error may predate it -- a launch that did not
// happen leaves the counters at zero, and the event fires all the same.)
static void pool_release(const qpp_keytab *kt, int sl, hipStream_t s)
{
    if (sl < 0) return;
    PoolRing *r = kt->pool;
    std::lock_guard<std::mutex> l(r->mu);
    if (hipEventRecord(r->ev[sl], s) != hipSuccess) {
        (void)hipGetLastError();
        r->state[sl] = 1;  // never reused: its launch may still be running
        return;
    }
    r->state[sl] = 2;
}

// Host mirror of the slots' suites, so a launch goes only to the suites the
// table holds right now (set, derive and clear keep it current).
static void keytab_note(qpp_keytab *kt, uint32_t slot, uint32_t suite)
{
    const uint8_t old = kt->h_suite[slot];
    if (old <= QPP_CHACHA20_POLY1305) --kt->n_suite[old];
    kt->h_suite[slot] = (uint8_t)suite;
    if (suite <= QPP_CHACHA20_POLY1305) ++kt->n_suite[suite];
}

static uint32_t keytab_suite_mask(const qpp_keytab *kt)
{
    uint32_t m = 0;
    for (int s = 0; s < 3; ++s)
        if (kt->n_suite[s]) m |= 1u << s;
    return m;
}

// Host batches of at least 2 x kPipeChunkBytes of output go through the
// session as a three-stage pipeline of up to kPipeMaxChunks chunks (see
// session_run_pipelined): up to kPipeRegular chunks of about equal size, the
// first and last of them cut into quarter, quarter and half (kPipeTaper) so
// the pipeline fills and drains on small pieces.
constexpr size_t kPipeChunkBytes = (size_t)32 << 20;
constexpr int kPipeRegular = 32, kPipeTaper = 2;
constexpr int kPipeMaxChunks = kPipeRegular + 2 * kPipeTaper;
constexpr int kMultiMaxDevices = 16;  // qpp_multi: devices per host-batch engine

struct qpp_session {
    hipStream_t stream;             // kernels (and everything of the serial path)
    hipStream_t s_in, s_out;        // pipelined path: H2D and D2H copy streams
    hipEvent_t ev_in[kPipeMaxChunks], ev_k[kPipeMaxChunks], ev_out[kPipeMaxChunks];
    int device;
    size_t max_bytes;
    uint32_t max_packets;
    uint8_t *h_in, *h_out, *h_misc;  // pinned
    uint8_t *hd_in, *hd_out, *hd_misc;  // their device views (zero-copy small calls)
    uint8_t *d_in, *d_out, *d_misc;
    size_t misc_bytes;
    qpp_plan *plan;                  // bucketing of batches of >= kSessionPlanMin packets
    // qpp_session_trace: timing events around every chunk's H2D, kernels and
    // D2H (start / end), created on first enable; the last traced call
    bool trace;
    hipEvent_t tev[6][kPipeMaxChunks];
    qpp_trace last;
};

// Host batches of at least this many packets are bucketed by (suite, slot)
// on the device before launch (qpp_plan); smaller ones launch as given.
constexpr uint32_t kSessionPlanMin = 128;

#define HIPCHK(x)                          \
    do {                                   \
        if ((x) != hipSuccess) {           \
            (void)hipGetLastError();       \
            return QPP_E_HIP;              \
        }                                  \
    } while (0)

extern "C" {

int qpp_abi_version(void) { return QPP_ABI_VERSION; }

uint64_t qpp_pool_fallbacks(void) { return g_pool_fallbacks.load(std::memory_order_relaxed); }

uint32_t qpp_watchdog_count(void)
{
    uint32_t v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_qpp_watchdog), sizeof v, 0, hipMemcpyDeviceToHost) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return v;
}

const char *qpp_strerror(int rc)
{
    switch (rc) {
    case QPP_OK: return "ok";
    case QPP_E_ARG: return "invalid argument";
    case QPP_E_HIP: return "HIP runtime error";
    case QPP_E_NODEV: return "no gfx950 device";
    case QPP_E_NOMEM: return "out of memory";
    default: return "unknown error";
    }
}

int qpp_device_check(void)
{
    int dev = 0, count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1) {
        (void)hipGetLastError();
        return QPP_E_NODEV;
    }
    HIPCHK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? QPP_OK : QPP_E_NODEV;
}

int qpp_keytab_create(uint32_t capacity, qpp_keytab **out)
{
    if (!out || capacity == 0 || capacity > (1u << 24)) return QPP_E_ARG;
    *out = NULL;
    int rc = qpp_device_check();
    if (rc != QPP_OK) return rc;
    qpp_keytab *kt = (qpp_keytab *)calloc(1, sizeof(qpp_keytab));
    if (!kt) return QPP_E_NOMEM;
    kt->cap = capacity;
    (void)hipGetDevice(&kt->device);
    kt->h_suite = (uint8_t *)malloc(capacity);
    if (!kt->h_suite) {
        free(kt);
        return QPP_E_NOMEM;
    }
    memset(kt->h_suite, 0xff, capacity);
    kt->pool = new (std::nothrow) PoolRing();
    if (!kt->pool || hipMalloc(&kt->pool->d, (size_t)kPoolSlots * kPoolStride * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(kt->pool->d, 0, (size_t)kPoolSlots * kPoolStride * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&kt->d_slots, (size_t)capacity * sizeof(KeySlot)) != hipSuccess ||
        hipMalloc(&kt->d_gtab, (size_t)capacity * (kGhashTabBytes + kGhPowBytes)) != hipSuccess ||
        hipMemset(kt->d_slots, 0xff, (size_t)capacity * sizeof(KeySlot)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        (void)hipGetLastError();
        qpp_keytab_destroy(kt);
        return QPP_E_NOMEM;
    }
    *out = kt;
    return QPP_OK;
}

void qpp_keytab_destroy(qpp_keytab *kt)
{
    if (!kt) return;
    if (kt->d_slots) (void)hipFree(kt->d_slots);
    if (kt->d_gtab) (void)hipFree(kt->d_gtab);
    if (kt->d_km) (void)hipFree(kt->d_km);
    if (kt->pool) {
        // (the caller has completed every launch on the table before
        // destroying it, quic_pp.h; the events go with the counters)
        for (hipEvent_t &e : kt->pool->ev)
            if (e) (void)hipEventDestroy(e);
        if (kt->pool->d) (void)hipFree(kt->pool->d);
        delete kt->pool;
    }
    free(kt->h_suite);
    free(kt);
}

uint32_t qpp_keytab_capacity(const qpp_keytab *kt) { return kt ? kt->cap : 0; }

int qpp_keytab_set(qpp_keytab *kt, const qpp_key_material *km, uint32_t n, void *stream)
{
    if (!kt || (!km && n)) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (km[i].slot >= kt->cap || km[i].suite > QPP_CHACHA20_POLY1305) return QPP_E_ARG;
    for (uint32_t i = 0; i < n; ++i) keytab_note(kt, km[i].slot, km[i].suite);
    hipStream_t s = (hipStream_t)stream;
    if (n > kt->km_cap) {
        if (kt->d_km) HIPCHK(hipFree(kt->d_km));
        kt->d_km = NULL;
        kt->km_cap = 0;
        HIPCHK(hipMalloc(&kt->d_km, (size_t)n * sizeof(qpp_key_material)));
        kt->km_cap = n;
    }
    HIPCHK(hipMemcpyAsync(kt->d_km, km, (size_t)n * sizeof(qpp_key_material),
                          hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_key_setup, dim3(n), dim3(kSetupWG), 0, s, kt->d_slots, kt->d_gtab, kt->cap,
                       kt->d_km, n);
    HIPCHK(hipGetLastError());
    // key material is host memory owned by the caller: finish before returning
    HIPCHK(hipStreamSynchronize(s));
    return QPP_OK;
}

int qpp_keytab_derive(qpp_keytab *kt, const qpp_secret *sec, uint32_t n,
                      qpp_key_material *km_out, void *stream)
{
    if (!kt || (!sec && n)) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (sec[i].slot >= kt->cap || sec[i].suite > QPP_CHACHA20_POLY1305 ||
            sec[i].secret_len < 1 || sec[i].secret_len > 64)
            return QPP_E_ARG;
    for (uint32_t i = 0; i < n; ++i) keytab_note(kt, sec[i].slot, sec[i].suite);
    hipStream_t s = (hipStream_t)stream;
    if (n > kt->km_cap) {
        if (kt->d_km) HIPCHK(hipFree(kt->d_km));
        kt->d_km = NULL;
        kt->km_cap = 0;
        HIPCHK(hipMalloc(&kt->d_km, (size_t)n * sizeof(qpp_key_material)));
        kt->km_cap = n;
    }
    qpp_secret *d_sec = NULL;
    HIPCHK(hipMalloc(&d_sec, (size_t)n * sizeof(qpp_secret)));
    int rc = QPP_OK;
    if (hipMemcpyAsync(d_sec, sec, (size_t)n * sizeof(qpp_secret), hipMemcpyHostToDevice, s) !=
        hipSuccess) {
        rc = QPP_E_HIP;
    } else {
        hipLaunchKernelGGL(k_derive, dim3((n + kDeriveWG - 1) / kDeriveWG), dim3(kDeriveWG), 0, s,
                           d_sec, n, kt->d_km);
        hipLaunchKernelGGL(k_key_setup, dim3(n), dim3(kSetupWG), 0, s, kt->d_slots, kt->d_gtab,
                           kt->cap, kt->d_km, n);
        if (hipGetLastError() != hipSuccess) rc = QPP_E_HIP;
        else if (km_out && hipMemcpyAsync(km_out, kt->d_km, (size_t)n * sizeof(qpp_key_material),
                                          hipMemcpyDeviceToHost, s) != hipSuccess)
            rc = QPP_E_HIP;
    }
    // the secrets are caller host memory: finish before returning
    if (hipStreamSynchronize(s) != hipSuccess && rc == QPP_OK) rc = QPP_E_HIP;
    (void)hipFree(d_sec);
    (void)hipGetLastError();
    return rc;
}

int qpp_keytab_clear(qpp_keytab *kt, const uint32_t *slots, uint32_t n, void *stream)
{
    if (!kt || (!slots && n)) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (slots[i] < kt->cap) keytab_note(kt, slots[i], 0xffu);
    hipStream_t s = (hipStream_t)stream;
    uint32_t *d = NULL;
    HIPCHK(hipMalloc(&d, (size_t)n * 4));
    if (hipMemcpyAsync(d, slots, (size_t)n * 4, hipMemcpyHostToDevice, s) != hipSuccess) {
        (void)hipFree(d);
        return QPP_E_HIP;
    }
    hipLaunchKernelGGL(k_clear_slots, dim3((n + 255) / 256), dim3(256), 0, s, kt->d_slots, d, n,
                       kt->cap);
    hipError_t e = hipStreamSynchronize(s);
    (void)hipFree(d);
    return e == hipSuccess ? QPP_OK : QPP_E_HIP;
}

// Workgroup sizes (tuned on MI355X, tools/sweep_wg.sh): GCM 1024 (one
// persistent workgroup per CU, 4 waves per SIMD), ChaCha20-Poly1305 256.
static const int kGcmWG = 1024;

#ifndef QPP_CHACHA_WG
#define QPP_CHACHA_WG 256  // study switch: the ChaCha20-Poly1305 kernel's workgroup size
#endif
static const int kChachaWG = QPP_CHACHA_WG;

// GCM blocks per lane per step (gcm_pad): 2 (r2i, same box: north star
// 1.419 -> 1.389 ms protect, config 4 310 -> 316 GiB/s; WRITE_SIZE 2.08 ->
// 1.78 GB per 1 Mi launch).  QPP_GCM_BPL=1 selects the one-block form (kept
// under test); read once per process.
static int gcm_bpl_choice()
{
    static const int b = [] {
        const char *v = getenv("QPP_GCM_BPL");
        return (v && atoi(v) == 1) ? 1 : 2;
    }();
    return b;
}

// Lone-packet kernels for unplanned launches up to lone_max (k_lone_gcm /
// k_lone_chacha); QPP_LONE=0 sends them through the quad kernels instead
// (a study and test switch, read once per process).
static bool lone_choice()
{
    static const bool b = [] {
        const char *v = getenv("QPP_LONE");
        return !(v && v[0] == '0');
    }();
    return b;
}

// The largest unplanned launch of a suite that takes the lone kernels: where
// one wave per packet stops beating the quad kernels on the same box
// (profiles/r4o_lone_crossover.txt, protect: AES-GCM 28.9 against 57.9 us at
// 4096 packets, 49 against 59 at 8192, 88 against 63 at 16384; ChaCha20
// 12.9 against 28.9 at 2 packets, then within +-1-3 us of the quad kernel up
// to 4096 and 47.5 against 30.6 at 8192, so past the host path's small
// calls the quad kernel's fewer instructions keep it).  QPP_LONE_MAX
// overrides both (a study switch for tools/lone_sizes.py).
static uint32_t lone_max(int suite)
{
    static const long env = [] {
        const char *v = getenv("QPP_LONE_MAX");
        return v ? atol(v) : -1L;
    }();
    if (env >= 0) return (uint32_t)(env > (1 << 20) ? (1 << 20) : env);
    return suite == QPP_CHACHA20_POLY1305 ? 64u : 8192u;
}

// Small host calls on the lone-packet kernels (and small header-protection
// mask calls) read and write the session's pinned staging from the kernel
// instead of through two copy-engine blits (~3.8 us each plus their
// scheduling, profiles/r4j_lone_latency); QPP_ZERO_COPY=0 keeps the copies
// (a study and test switch, read once per process).
static bool zero_copy_choice()
{
    static const bool b = [] {
        const char *v = getenv("QPP_ZERO_COPY");
        return !(v && v[0] == '0');
    }();
    return b;
}

// A small host call of one workgroup's packets staged by the lone kernel
// itself instead of a copy (QPP_LONE_STAGE=0: the copy; a study and test
// switch, read once per process).
static bool lone_stage_choice()
{
    static const bool b = [] {
        const char *v = getenv("QPP_LONE_STAGE");
        return !(v && v[0] == '0');
    }();
    return b;
}

// QPP_SPIN_LIMIT (a test switch, read once per process) replaces the bounded
// waits' limits (g_qpp_spin_tab, g_qpp_spin_lone) on each device before its
// first launch: 0 makes every bounded wait give up at once, so the watchdog
// paths' QPP_S_INTERNAL reporting can be checked.
static int apply_spin_env(hipStream_t s)
{
    static const long env = [] {
        const char *v = getenv("QPP_SPIN_LIMIT");
        return v ? atol(v) : -1L;
    }();
    static const long delay = [] {
        const char *v = getenv("QPP_PAIR_DELAY");  // test switch, g_qpp_pair_delay
        return v ? atol(v) : -1L;
    }();
    if (env < 0 && delay < 0) return QPP_OK;
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load() & bit) return QPP_OK;
    if (env >= 0) {
        const uint32_t v = (uint32_t)env;
        HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_qpp_spin_tab), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_qpp_spin_lone), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
    }
    if (delay >= 0) {
        const uint32_t v = (uint32_t)delay;
        HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_qpp_pair_delay), &v, sizeof v, 0, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    done.fetch_or(bit);
    return QPP_OK;
}

static uint32_t cu_count()
{
    static int cus[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (!cus[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) {
            (void)hipGetLastError();
            c = 256;
        }
        cus[dev] = c;
    }
    return (uint32_t)cus[dev];
}

// Persistent GCM grid: one 1024-thread workgroup per CU (or two of 512),
// fewer when the batch has fewer than a workgroup's worth of items per CU.
static uint32_t gcm_grid(uint32_t items, uint32_t waves_per_wg)
{
    const uint32_t need = (items + waves_per_wg - 1) / waves_per_wg;
    const uint32_t cap = cu_count() * (waves_per_wg == 8 ? 2u : 1u);
    return need < cap ? (need ? need : 1u) : cap;
}

// GCM launch shape.  Two 512-thread workgroups per CU run the step loop's
// lookups ~9 % faster than one of 1024 (profiles/r3u_probe_wg*.txt), but the
// two workgroups sharing a CU do not progress at the same rate, so over many
// items per wave one ends well before the other; and each holds one GHASH
// table entry.  So: two per CU when the table holds one key of the suite and
// the launch has at most one item per wave.  (Round 4: two per CU for every
// single-key launch, its waves drawing pooled chunks of 8 items from a
// launch-wide counter fetched ahead of need, measured no faster than one of
// 1024 at the north star, profiles/r4f_ab_pooled.txt.)
#ifndef QPP_TWO_WG_ITEMS
#define QPP_TWO_WG_ITEMS 16u  // study switch: items per CU up to which the 512 shape runs
#endif
static bool gcm_two_wg(const qpp_keytab *kt, uint32_t suite, uint32_t items)
{
    return kt->n_suite[suite] == 1 && items <= cu_count() * (uint32_t)QPP_TWO_WG_ITEMS;  // 2 workgroups x 8 waves per CU
}

// ChaCha20-Poly1305 issue priority by progress (k_chacha PRIO): for launches
// whose waves all fit the chip at once (kChachaWpe per SIMD, one round), so
// each SIMD's waves end together instead of oldest first.  QPP_CHACHA_PRIO=0
// turns it off, =2 forces it on for every launch (A/B switches, read once).
static bool chacha_prio(uint32_t waves)
{
    static const int m = [] {
        const char *v = getenv("QPP_CHACHA_PRIO");
        return v ? atoi(v) : 1;
    }();
    return m == 2 || (m == 1 && waves <= cu_count() * 4u * kChachaWpe);
}

static int launch_packets(bool enc, const qpp_keytab *kt, const qpp_desc *d_desc, uint32_t n,
                          const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res, void *stream,
                          const qpp_plan *plan = nullptr, const LoneStage *stage = nullptr)
{
    if (!kt || (n && (!d_desc || !d_in || !d_out || !d_res))) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    hipStream_t s = (hipStream_t)stream;
    if (int rc = apply_spin_env(s)) return rc;
    // one launch per suite the table holds now; unplanned, an empty table
    // still gets one launch so every packet reports QPP_S_NO_KEY (planned,
    // the no-key bucket has its own kernel)
    uint32_t mask = keytab_suite_mask(kt);
    if (!mask && !plan) mask = 1u;
    // planned: each suite's launch covers at most every wave item of the batch
    const uint32_t *d_items = plan ? plan->d_items : nullptr, *d_irange = plan ? plan->d_irange : nullptr;
    const uint32_t waves = plan ? qpp_internal_plan_max_items(n, kt->cap) : (n + 15) / 16;
    const int bpl_gcm = gcm_bpl_choice();
    // up to a few thousand packets (the object API's one, small flushes):
    // one wave per packet (k_lone_*), see lone_max
    const bool lone = !plan && lone_choice();
    const dim3 lgrid((n + kLoneWG / 64 - 1) / (kLoneWG / 64)), lblock(kLoneWG);
    const LoneStage lst = stage ? *stage : LoneStage{nullptr, nullptr, 0u};
#define QPP_LAUNCH_GCM_W(SUITE, BPLV, WGV)                                                     \
    do {                                                                                       \
        const dim3 grid(gcm_grid(waves, WGV / 64)), block(WGV);                                 \
        const int psl = (WGV == 1024 || QPP_POOL512) && kt->n_suite[SUITE] == 1 ? pool_acquire(kt) : -1; \
        uint32_t *pl = psl >= 0 ? kt->pool->d + (size_t)psl * kPoolStride : nullptr;          \
        if (enc)                                                                               \
            hipLaunchKernelGGL((k_gcm<SUITE, true, WGV, BPLV>), grid, block, 0, s,             \
                               kt->d_slots, kt->d_gtab, kt->cap, d_desc, n, d_in, d_out, d_res, \
                               d_items, d_irange, pl);                                         \
        else                                                                                   \
            hipLaunchKernelGGL((k_gcm<SUITE, false, WGV, BPLV>), grid, block, 0, s,            \
                               kt->d_slots, kt->d_gtab, kt->cap, d_desc, n, d_in, d_out, d_res, \
                               d_items, d_irange, pl);                                         \
        pool_release(kt, psl, s);                                                              \
    } while (0)
#define QPP_LAUNCH_GCM_B(SUITE, BPLV)                                                          \
    do {                                                                                       \
        if (BPLV == 2 && gcm_two_wg(kt, SUITE, waves)) QPP_LAUNCH_GCM_W(SUITE, BPLV, 512);       \
        else QPP_LAUNCH_GCM_W(SUITE, BPLV, kGcmWG);                                             \
    } while (0)
#define QPP_LAUNCH_GCM(SUITE)                                                                  \
    if (mask & (1u << SUITE)) {                                                                \
        if (lone && n <= lone_max(SUITE)) {                                                    \
            if (enc)                                                                           \
                hipLaunchKernelGGL((k_lone_gcm<SUITE, true>), lgrid, lblock, 0, s, kt->d_slots, \
                                   kt->d_gtab, kt->cap, d_desc, n, d_in, d_out, d_res, lst);   \
            else                                                                               \
                hipLaunchKernelGGL((k_lone_gcm<SUITE, false>), lgrid, lblock, 0, s, kt->d_slots, \
                                   kt->d_gtab, kt->cap, d_desc, n, d_in, d_out, d_res, lst);   \
        } else if (bpl_gcm == 1) {                                                             \
            QPP_LAUNCH_GCM_B(SUITE, 1);                                                         \
        } else {                                                                               \
            QPP_LAUNCH_GCM_B(SUITE, 2);                                                         \
        }                                                                                      \
        HIPCHK(hipGetLastError());                                                             \
    }
    QPP_LAUNCH_GCM(QPP_AES_128_GCM)
    QPP_LAUNCH_GCM(QPP_AES_256_GCM)
    if ((mask & (1u << QPP_CHACHA20_POLY1305)) && lone && n <= lone_max(QPP_CHACHA20_POLY1305)) {
        if (enc)
            hipLaunchKernelGGL((k_lone_chacha<true>), lgrid, lblock, 0, s, kt->d_slots, kt->cap, d_desc, n, d_in,
                               d_out, d_res, lst);
        else
            hipLaunchKernelGGL((k_lone_chacha<false>), lgrid, lblock, 0, s, kt->d_slots, kt->cap, d_desc, n, d_in,
                               d_out, d_res, lst);
        HIPCHK(hipGetLastError());
    } else if (mask & (1u << QPP_CHACHA20_POLY1305)) {
        uint32_t cgrid = (waves + kChachaWG / 64 - 1) / (kChachaWG / 64);
        if (QPP_CH_PERSIST > 0) {  // study: at most QPP_CH_PERSIST rounds of resident workgroups
            const uint32_t resident = cu_count() * (uint32_t)(4 * kChachaWpe / (kChachaWG / 64)) * (uint32_t)QPP_CH_PERSIST;
            cgrid = cgrid < resident ? cgrid : resident;
        }
        const dim3 grid(cgrid ? cgrid : 1u), block(kChachaWG);
        if (chacha_prio(waves)) {
            if (enc)
                hipLaunchKernelGGL((k_chacha<true, kChachaWG, true>), grid, block, 0, s, kt->d_slots, kt->cap,
                                   d_desc, n, d_in, d_out, d_res, d_items, d_irange);
            else
                hipLaunchKernelGGL((k_chacha<false, kChachaWG, true>), grid, block, 0, s, kt->d_slots, kt->cap,
                                   d_desc, n, d_in, d_out, d_res, d_items, d_irange);
        } else if (enc) {
            hipLaunchKernelGGL((k_chacha<true, kChachaWG, false>), grid, block, 0, s, kt->d_slots, kt->cap,
                               d_desc, n, d_in, d_out, d_res, d_items, d_irange);
        } else {
            hipLaunchKernelGGL((k_chacha<false, kChachaWG, false>), grid, block, 0, s, kt->d_slots, kt->cap,
                               d_desc, n, d_in, d_out, d_res, d_items, d_irange);
        }
        HIPCHK(hipGetLastError());
    }
#undef QPP_LAUNCH_GCM
#undef QPP_LAUNCH_GCM_B
#undef QPP_LAUNCH_GCM_W
    return QPP_OK;
}

int qpp_protect(const qpp_keytab *kt, const qpp_desc *d_desc, uint32_t n, const uint8_t *d_in,
                uint8_t *d_out, qpp_result *d_res, void *stream)
{
    return launch_packets(true, kt, d_desc, n, d_in, d_out, d_res, stream);
}

int qpp_unprotect(const qpp_keytab *kt, const qpp_desc *d_desc, uint32_t n,
                  const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res, void *stream)
{
    return launch_packets(false, kt, d_desc, n, d_in, d_out, d_res, stream);
}

int qpp_plan_build(qpp_plan *p, const qpp_keytab *kt, const qpp_desc *d_desc, uint32_t n,
                   void *stream)
{
    if (!p || !kt || (n && !d_desc)) return QPP_E_ARG;
    return qpp_internal_plan_build(p, kt->d_slots, kt->cap, d_desc, n, (hipStream_t)stream);
}

static int launch_planned(bool enc, const qpp_keytab *kt, const qpp_plan *p, const qpp_desc *d_desc,
                          uint32_t n, const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res,
                          void *stream)
{
    if (!kt || !p || (n && (!d_desc || !d_in || !d_out || !d_res))) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    hipStream_t s = (hipStream_t)stream;
    int rc = qpp_internal_plan_gather(p, d_desc, n, s);
    if (rc == QPP_OK)
        rc = launch_packets(enc, kt, p->d_sorted, n, d_in, d_out, d_res, stream, p);
    if (rc == QPP_OK) rc = qpp_internal_plan_nokey(p, d_res, s);
    return rc;
}

int qpp_protect_planned(const qpp_keytab *kt, const qpp_plan *p, const qpp_desc *d_desc, uint32_t n,
                        const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res, void *stream)
{
    return launch_planned(true, kt, p, d_desc, n, d_in, d_out, d_res, stream);
}

int qpp_unprotect_planned(const qpp_keytab *kt, const qpp_plan *p, const qpp_desc *d_desc,
                          uint32_t n, const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res,
                          void *stream)
{
    return launch_planned(false, kt, p, d_desc, n, d_in, d_out, d_res, stream);
}

int qpp_hp_mask(const qpp_keytab *kt, const uint32_t *d_slots, const uint8_t *d_samples,
                uint32_t n, uint8_t *d_masks, void *stream)
{
    if (!kt || (n && (!d_slots || !d_samples || !d_masks))) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    hipLaunchKernelGGL(k_hp_mask, dim3((n + kMaskWG - 1) / kMaskWG), dim3(kMaskWG), 0,
                       (hipStream_t)stream,
                       kt->d_slots, kt->cap, d_slots, d_samples, n, d_masks);
    HIPCHK(hipGetLastError());
    return QPP_OK;
}

// ------------------------------------------------------------- sessions --

static void session_free_buffers(qpp_session *s)
{
    if (s->h_in) (void)hipHostFree(s->h_in);
    if (s->h_out) (void)hipHostFree(s->h_out);
    if (s->h_misc) (void)hipHostFree(s->h_misc);
    if (s->d_in) (void)hipFree(s->d_in);
    if (s->d_out) (void)hipFree(s->d_out);
    if (s->d_misc) (void)hipFree(s->d_misc);
    s->h_in = s->h_out = s->h_misc = s->d_in = s->d_out = s->d_misc = NULL;
    s->hd_in = s->hd_out = s->hd_misc = NULL;
}

static size_t misc_bytes_for(uint32_t max_packets)
{
    // descriptors + results + slot ids + samples + masks
    return (size_t)max_packets * (sizeof(qpp_desc) + sizeof(qpp_result) + 4 + 16 + 16) + 256;
}

static int session_reserve(qpp_session *s, size_t bytes, uint32_t packets)
{
    if (bytes <= s->max_bytes && packets <= s->max_packets && s->h_in) return QPP_OK;
    size_t nb = bytes > s->max_bytes ? bytes : s->max_bytes;
    uint32_t np = packets > s->max_packets ? packets : s->max_packets;
    if (nb < 4096) nb = 4096;
    if (np < 64) np = 64;
    session_free_buffers(s);
    s->max_bytes = nb;
    s->max_packets = np;
    s->misc_bytes = misc_bytes_for(np);
    if (hipHostMalloc(&s->h_in, nb, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s->h_out, nb, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s->h_misc, s->misc_bytes, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&s->d_in, nb) != hipSuccess || hipMalloc(&s->d_out, nb) != hipSuccess ||
        hipMalloc(&s->d_misc, s->misc_bytes) != hipSuccess ||
        hipHostGetDevicePointer((void **)&s->hd_in, s->h_in, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&s->hd_out, s->h_out, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&s->hd_misc, s->h_misc, 0) != hipSuccess) {
        (void)hipGetLastError();
        session_free_buffers(s);
        s->max_bytes = 0;
        s->max_packets = 0;
        return QPP_E_NOMEM;
    }
    return QPP_OK;
}

int qpp_session_create(size_t max_bytes, uint32_t max_packets, qpp_session **out)
{
    if (!out) return QPP_E_ARG;
    *out = NULL;
    int rc = qpp_device_check();
    if (rc != QPP_OK) return rc;
    qpp_session *s = (qpp_session *)calloc(1, sizeof(qpp_session));
    if (!s) return QPP_E_NOMEM;
    (void)hipGetDevice(&s->device);
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        free(s);
        return QPP_E_HIP;
    }
    bool ok = hipStreamCreateWithFlags(&s->s_in, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&s->s_out, hipStreamNonBlocking) == hipSuccess;
    for (int c = 0; ok && c < kPipeMaxChunks; ++c)
        ok = hipEventCreateWithFlags(&s->ev_in[c], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s->ev_k[c], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s->ev_out[c], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        qpp_session_destroy(s);
        return QPP_E_HIP;
    }
    rc = session_reserve(s, max_bytes, max_packets);
    if (rc != QPP_OK) {
        qpp_session_destroy(s);
        return rc;
    }
    *out = s;
    return QPP_OK;
}

void qpp_session_destroy(qpp_session *s)
{
    if (!s) return;
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->s_in) (void)hipStreamSynchronize(s->s_in);
    if (s->s_out) (void)hipStreamSynchronize(s->s_out);
    session_free_buffers(s);
    qpp_plan_destroy(s->plan);
    for (int c = 0; c < kPipeMaxChunks; ++c) {
        if (s->ev_in[c]) (void)hipEventDestroy(s->ev_in[c]);
        if (s->ev_k[c]) (void)hipEventDestroy(s->ev_k[c]);
        if (s->ev_out[c]) (void)hipEventDestroy(s->ev_out[c]);
        for (int k = 0; k < 6; ++k)
            if (s->tev[k][c]) (void)hipEventDestroy(s->tev[k][c]);
    }
    if (s->s_in) (void)hipStreamDestroy(s->s_in);
    if (s->s_out) (void)hipStreamDestroy(s->s_out);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    free(s);
}

void *qpp_session_stream(qpp_session *s) { return s ? (void *)s->stream : NULL; }

// Large host batches: chunk c of the packets (in descriptor order) is copied
// into pinned staging by the host and sent H2D on s_in, processed on the
// kernel stream once its input event fires, and returned D2H on s_out once its
// kernel event fires; the host copies chunk c out while later chunks are still
// in flight.  The host memcpys, both PCIe directions and the kernels of
// different chunks overlap.  Requires out_off non-decreasing in descriptor
// order: chunk c's D2H then covers [out_off of its first packet, out_off of
// the next chunk's first packet) -- chunk 0 from 0, the last chunk to out_len
// -- so the chunks tile the output, and bytes a packet writes past its tile
// are copied by a later chunk's D2H, which runs after this chunk's kernel.
// Each chunk's H2D covers the input extent of its own packets (over-copying
// bytes of a neighbour is harmless: same host bytes).
// Host copies between caller memory and pinned staging: one thread streams
// ~10 GB/s, well under the PCIe rate, so large copies are split over a
// process-wide pool of copy threads (started on first use, never torn down:
// its threads sleep on a condition variable between copies).  Round 5: the
// pool replaces a std::thread per part and copy (up to 8 x 64 thread starts
// per 1 Mi-packet call), and a chunk's copy-out runs on it while the calling
// thread stages the next chunks.
// Host copies between caller memory and pinned staging with non-temporal
// stores: a plain memcpy below glibc's non-temporal threshold reads each
// destination line before writing it (write-allocate), so a copy moves three
// times its size through host memory instead of two.  QPP_COPY_NT=0 (a study
// switch, read once per process) keeps memcpy.
static bool copy_nt_choice()
{
    static const bool b = [] {
        const char *v = getenv("QPP_COPY_NT");
        return !(v && v[0] == '0') && __builtin_cpu_supports("avx2");
    }();
    return b;
}

__attribute__((target("avx2"))) static void copy_nt_avx2(uint8_t *dst, const uint8_t *src, size_t n)
{
    size_t head = (size_t)((32u - ((uintptr_t)dst & 31u)) & 31u);
    if (head > n) head = n;
    memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i *)(src + i));
        const __m256i b = _mm256_loadu_si256((const __m256i *)(src + i + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i *)(src + i + 64));
        const __m256i d = _mm256_loadu_si256((const __m256i *)(src + i + 96));
        _mm256_stream_si256((__m256i *)(dst + i), a);
        _mm256_stream_si256((__m256i *)(dst + i + 32), b);
        _mm256_stream_si256((__m256i *)(dst + i + 64), c);
        _mm256_stream_si256((__m256i *)(dst + i + 96), d);
    }
    memcpy(dst + i, src + i, n - i);
    _mm_sfence();  // the streamed lines are visible before the copy is reported done
}

static void copy_bytes(uint8_t *dst, const uint8_t *src, size_t n)
{
    if (n >= ((size_t)1 << 16) && copy_nt_choice()) copy_nt_avx2(dst, src, n);
    else memcpy(dst, src, n);
}

struct CopyGroup {
    std::mutex mu;
    std::condition_variable cv;
    int pending = 0;
    std::atomic<uint64_t> busy_ns{0};  // summed duration of the pool's tasks (qpp_trace)
    void wait()
    {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return pending == 0; });
    }
};

class CopyPool {
  public:
    static CopyPool &get()
    {
        // never destroyed (no join at exit); a forked child, which inherits
        // the pointer but not the threads, starts a pool of its own
        static std::once_flag once;
        std::call_once(once, [] { pthread_atfork(nullptr, nullptr, [] { g_pool.store(nullptr); }); });
        CopyPool *p = g_pool.load();
        if (!p) {
            std::lock_guard<std::mutex> l(g_pool_mu);
            p = g_pool.load();
            if (!p) {
                p = new CopyPool();
                g_pool.store(p);
            }
        }
        return *p;
    }
    int threads() const { return n_; }
    void submit(uint8_t *dst, const uint8_t *src, size_t len, CopyGroup *g)
    {
        {
            std::lock_guard<std::mutex> l(g->mu);
            ++g->pending;
        }
        {
            std::lock_guard<std::mutex> l(mu_);
            q_.push_back(Task{dst, src, len, g});
        }
        cv_.notify_one();
    }

  private:
    struct Task {
        uint8_t *dst;
        const uint8_t *src;
        size_t len;
        CopyGroup *g;
    };
    CopyPool()
    {
        const char *v = getenv("QPP_COPY_THREADS");  // A/B switch, default 6
        const int t = v ? atoi(v) : 6;
        n_ = t < 1 ? 1 : t > 32 ? 32 : t;
        // (round 5 also pinned the threads to the CPUs of the device's NUMA
        // node: 13.0-16.6 against 11.5-17.7 GiB/s unpinned on one two-socket
        // box, interleaved -- no difference through the run-to-run spread,
        // profiles/r5e_host_path/host_path_studies.txt; removed)
        for (int i = 0; i < n_; ++i) std::thread([this] { run(); }).detach();
    }
    void run()
    {
        for (;;) {
            Task t;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return !q_.empty(); });
                t = q_.front();
                q_.pop_front();
            }
            const auto t0 = std::chrono::steady_clock::now();
            copy_bytes(t.dst, t.src, t.len);
            t.g->busy_ns.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                       std::chrono::steady_clock::now() - t0).count(),
                                   std::memory_order_relaxed);
            {
                // notify while holding the group's lock: the waiter cannot see
                // pending == 0 (and destroy the group, which lives on its
                // stack) until this worker has released the lock, after which
                // it never touches the group again
                std::lock_guard<std::mutex> l(t.g->mu);
                if (--t.g->pending == 0) t.g->cv.notify_all();
            }
        }
    }
    int n_ = 8;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Task> q_;
    static std::atomic<CopyPool *> g_pool;
    static std::mutex g_pool_mu;
};
std::atomic<CopyPool *> CopyPool::g_pool{nullptr};
std::mutex CopyPool::g_pool_mu;

// dst <- src over the pool's threads in parts of >= 4 MiB; with g, return at
// once (g->wait() before the bytes are used), else when the copy is done.
static void par_memcpy(uint8_t *dst, const uint8_t *src, size_t bytes, CopyGroup *g = nullptr)
{
    constexpr size_t kPart = (size_t)4 << 20;
    if (bytes < 2 * kPart) {
        const auto t0 = std::chrono::steady_clock::now();
        copy_bytes(dst, src, bytes);
        if (g)
            g->busy_ns.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                     std::chrono::steady_clock::now() - t0).count(),
                                 std::memory_order_relaxed);
        return;
    }
    CopyPool &pool = CopyPool::get();
    size_t parts = bytes / kPart;
    if (parts > (size_t)pool.threads()) parts = (size_t)pool.threads();
    const size_t step = (bytes / parts + 63) & ~(size_t)63;
    CopyGroup local;
    CopyGroup *grp = g ? g : &local;
    for (size_t lo = g ? 0 : step; lo < bytes; lo += step)
        pool.submit(dst + lo, src + lo, lo + step < bytes ? step : bytes - lo, grp);
    if (!g) {
        copy_bytes(dst, src, step < bytes ? step : bytes);  // the caller's own part
        local.wait();
    }
}

// Descriptor extents against the caller's buffer sizes (quic_pp.h, Buffers):
// a descriptor that does not fit is flagged so the kernel reports
// QPP_S_LENGTH for it without touching memory.  Protect reads header +
// payload and writes header + ciphertext + tag; unprotect reads and writes
// at most the packet's length.
static void reject_out_of_bounds(bool enc, qpp_desc *d, uint32_t n, size_t in_len, size_t out_len)
{
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t rd = enc ? (uint64_t)d[i].hdr_len + d[i].len : (uint64_t)d[i].len;
        const uint64_t wr = enc ? rd + QPP_TAG_LEN : rd;
        const bool ok = d[i].in_off <= in_len && rd <= in_len - d[i].in_off && d[i].out_off <= out_len &&
                        wr <= out_len - d[i].out_off;
        d[i].flags = ok ? (uint16_t)(d[i].flags & ~kFlagReject) : (uint16_t)(d[i].flags | kFlagReject);
    }
}

// One launch over n device descriptors of the session: bucketed by (suite,
// slot) through the session's plan when the batch is large enough.
static int session_launch(bool enc, qpp_session *s, const qpp_keytab *kt, const qpp_desc *dd,
                          uint32_t n, qpp_result *dr)
{
    if (n < kSessionPlanMin) return launch_packets(enc, kt, dd, n, s->d_in, s->d_out, dr, s->stream);
    if (s->plan && s->plan->cap < n) {
        HIPCHK(hipStreamSynchronize(s->stream));  // the old plan may still be in use
        qpp_plan_destroy(s->plan);
        s->plan = NULL;
    }
    if (!s->plan) {
        const int rc = qpp_plan_create(n > s->max_packets ? n : s->max_packets, &s->plan);
        if (rc != QPP_OK) return rc;
    }
    int rc = qpp_plan_build(s->plan, kt, dd, n, s->stream);
    if (rc == QPP_OK) rc = launch_planned(enc, kt, s->plan, dd, n, s->d_in, s->d_out, dr, s->stream);
    return rc;
}

// D2H of a session: up to two device ranges into pinned host memory (device
// views), by k_xfer.  QPP_D2H_KERNEL=0 (a study switch, read once per
// process) uses hipMemcpyAsync on the stream instead.
static bool d2h_kernel_choice()
{
    static const bool b = [] {
        const char *v = getenv("QPP_D2H_KERNEL");
        return !(v && v[0] == '0');
    }();
    return b;
}

static int launch_xfer(uint8_t *d0, const uint8_t *s0, size_t n0, uint8_t *d1, const uint8_t *s1, size_t n1,
                       hipStream_t st)
{
    if (!n0 && !n1) return QPP_OK;
    const size_t units = (std::max(n0, n1) + 15) / 16;
    // ~8 16-byte units per thread, at most xfer_wgs() workgroups per range
    static const size_t cap = [] {
        const char *v = getenv("QPP_XFER_WGS");  // study switch, read once per process
        const long c = v ? atol(v) : 1024;
        return (size_t)(c < 1 ? 1 : c > 4096 ? 4096 : c);
    }();
    size_t g = (units + (size_t)kXferWG * 8 - 1) / ((size_t)kXferWG * 8);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    hipLaunchKernelGGL(k_xfer, dim3((uint32_t)g, n1 ? 2u : 1u), dim3(kXferWG), 0, st, s0, d0, n0, s1, d1, n1);
    HIPCHK(hipGetLastError());
    return QPP_OK;
}

static int session_d2h(uint8_t *h0, uint8_t *hd0, const uint8_t *s0, size_t n0, uint8_t *h1, uint8_t *hd1,
                       const uint8_t *s1, size_t n1, hipStream_t st)
{
    if (!d2h_kernel_choice()) {
        if (n0) HIPCHK(hipMemcpyAsync(h0, s0, n0, hipMemcpyDeviceToHost, st));
        if (n1) HIPCHK(hipMemcpyAsync(h1, s1, n1, hipMemcpyDeviceToHost, st));
        return QPP_OK;
    }
    return launch_xfer(hd0, s0, n0, hd1, s1, n1, st);
}

// QPP_H2D_KERNEL=1 (a study switch, read once per process): the pipelined
// session's H2D legs by k_xfer too (default: hipMemcpyAsync, the copy engines)
static bool h2d_kernel_choice()
{
    static const bool b = [] {
        const char *v = getenv("QPP_H2D_KERNEL");
        return v && v[0] == '1';
    }();
    return b;
}

// QPP_SESSION_TRACE=1: one stderr line per pipelined call with its host
// phases (a study switch, read once per process)
static bool trace_on()
{
    static const bool b = getenv("QPP_SESSION_TRACE") != nullptr;
    return b;
}

// Chunk c of the batch: its descriptors are copied into pinned staging and
// bounds-checked by the host, its input extent is copied into pinned staging
// by the copy pool, and both go H2D on s_in (the copy engines); the chunk's
// kernels run on the kernel stream once that lands; its output tile and
// results go D2H on s_out (a blit kernel, the runtime's choice, which runs
// beside the packet kernels: profiles/r5g_d2h_engines.txt), and the pool
// copies them out while later chunks are in flight.  So host copies, both
// PCIe directions and the kernels of different chunks overlap, and no work
// on the whole batch precedes the first chunk's copies.  (Round 5 also built
// DMA straight from / to caller memory pinned by hipHostRegister: correct,
// but 9.6-10.7 GiB/s against 17-19 GiB/s for this staged pipeline on the
// same boxes whatever the flags and D2H form, so it was removed;
// profiles/r5e_host_path/.)
static int session_run_pipelined(bool enc, qpp_session *s, const qpp_keytab *kt,
                                 const qpp_desc *desc, uint32_t n, const uint8_t *in,
                                 size_t in_len, uint8_t *out, size_t out_len, qpp_result *res,
                                 int chunks)
{
    qpp_desc *hd = (qpp_desc *)s->h_misc;
    qpp_result *hr = (qpp_result *)(s->h_misc + (size_t)s->max_packets * sizeof(qpp_desc));
    qpp_desc *dd = (qpp_desc *)s->d_misc;
    qpp_result *dr = (qpp_result *)(s->d_misc + (size_t)s->max_packets * sizeof(qpp_desc));
    qpp_result *hrd = (qpp_result *)(s->hd_misc + (size_t)s->max_packets * sizeof(qpp_desc));  // hr's device view
    const bool tr = s->trace;
    const auto clk = [] { return std::chrono::duration<double, std::milli>(
                              std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_start = clk();
    double t_copy_in = 0.0;
    double in_bytes = 0.0, out_bytes = 0.0;
    // the caller may have assembled its input / wants its output in the
    // session's own staging (qpp_session_stage): no host copy then
    const bool in_direct = in == s->h_in, out_direct = out == s->h_out;
    HIPCHK(hipMemsetAsync(s->d_out, 0, out_len, s->stream));
    size_t olo[kPipeMaxChunks + 1];
    uint32_t first[kPipeMaxChunks + 1];
    // chunk weights in quarters of a regular chunk: 1, 1, 2 at the start and
    // 2, 1, 1 at the end when there are enough regular chunks to taper
    const int regular = chunks;
    const bool taper = regular >= 8;
    if (taper) chunks = regular + 2 * kPipeTaper;
    auto weight = [&](int c) -> uint64_t {
        if (!taper) return 4;
        if (c < 3) return c < 2 ? 1 : 2;
        if (c >= chunks - 3) return c >= chunks - 2 ? 1 : 2;
        return 4;
    };
    const uint64_t wsum = 4ull * (uint64_t)regular;
    uint64_t wacc = 0;
    for (int c = 0; c <= chunks; ++c) {
        first[c] = (uint32_t)((uint64_t)n * wacc / wsum);
        if (c < chunks) wacc += weight(c);
        olo[c] = c == 0 ? 0 : c == chunks ? out_len : (size_t)desc[first[c]].out_off;
        if (olo[c] > out_len) olo[c] = out_len;
    }
    // a chunk handed back to the caller: its output tile and results, copied
    // out by the pool while this thread goes on staging later chunks
    CopyGroup outg;
    struct WaitAll {
        CopyGroup &g;
        ~WaitAll() { g.wait(); }  // every return path: no pool copy outlives the call
    } wait_all{outg};
    auto hand_back = [&](int d) {
        if (olo[d + 1] > olo[d] && !out_direct)
            par_memcpy(out + olo[d], s->h_out + olo[d], olo[d + 1] - olo[d], &outg);
        memcpy(res + first[d], hr + first[d], (size_t)(first[d + 1] - first[d]) * sizeof(qpp_result));
    };
    int rc = QPP_OK;
    int next_out = 0;
    for (int c = 0; c < chunks; ++c) {
        const uint32_t a = first[c], b = first[c + 1];
        hipStream_t sin = s->s_in;
        memcpy(hd + a, desc + a, (size_t)(b - a) * sizeof(qpp_desc));
        reject_out_of_bounds(enc, hd + a, b - a, in_len, out_len);
        if (tr) HIPCHK(hipEventRecord(s->tev[0][c], sin));
        const bool h2dk = h2d_kernel_choice();
        if (b > a && !h2dk)
            HIPCHK(hipMemcpyAsync(dd + a, hd + a, (size_t)(b - a) * sizeof(qpp_desc), hipMemcpyHostToDevice,
                                  sin));
        size_t lo = SIZE_MAX, hi = 0;
        for (uint32_t i = a; i < b; ++i) {
            if (hd[i].flags & kFlagReject) continue;
            const size_t o = (size_t)desc[i].in_off;
            const size_t e = o + (size_t)desc[i].hdr_len + desc[i].len + 16;
            if (o < lo) lo = o;
            if (e > hi) hi = e;
        }
        if (hi > in_len) hi = in_len;
        if (lo < hi) {
            if (!in_direct) {
                const double t0 = tr ? clk() : 0.0;
                par_memcpy(s->h_in + lo, in + lo, hi - lo);
                if (tr) t_copy_in += clk() - t0;
            }
            if (!h2dk) HIPCHK(hipMemcpyAsync(s->d_in + lo, s->h_in + lo, hi - lo, hipMemcpyHostToDevice, sin));
            in_bytes += (double)(hi - lo);
        }
        if (h2dk) {
            rc = launch_xfer((uint8_t *)(dd + a), s->hd_misc + (size_t)a * sizeof(qpp_desc),
                             (size_t)(b - a) * sizeof(qpp_desc), lo < hi ? s->d_in + lo : nullptr,
                             lo < hi ? s->hd_in + lo : nullptr, lo < hi ? hi - lo : 0, sin);
            if (rc != QPP_OK) break;
        }
        in_bytes += (double)(b - a) * sizeof(qpp_desc);
        HIPCHK(hipEventRecord(s->ev_in[c], sin));
        if (tr) HIPCHK(hipEventRecord(s->tev[1][c], sin));
        HIPCHK(hipStreamWaitEvent(s->stream, s->ev_in[c], 0));
        if (tr) HIPCHK(hipEventRecord(s->tev[2][c], s->stream));
        if (b > a) {
            rc = session_launch(enc, s, kt, dd + a, b - a, dr + a);
            if (rc != QPP_OK) break;
        }
        HIPCHK(hipEventRecord(s->ev_k[c], s->stream));
        if (tr) HIPCHK(hipEventRecord(s->tev[3][c], s->stream));
        HIPCHK(hipStreamWaitEvent(s->s_out, s->ev_k[c], 0));
        if (tr) HIPCHK(hipEventRecord(s->tev[4][c], s->s_out));
        out_bytes += (double)(olo[c + 1] - olo[c]) + (double)(b - a) * sizeof(qpp_result);
        {
            const size_t tl = olo[c + 1] > olo[c] ? olo[c + 1] - olo[c] : 0;
            const size_t rl = (size_t)(b - a) * sizeof(qpp_result);
            rc = session_d2h(s->h_out + olo[c], s->hd_out + olo[c], s->d_out + olo[c], tl, (uint8_t *)(hr + a),
                             (uint8_t *)(hrd + a), (const uint8_t *)(dr + a), rl, s->s_out);
            if (rc != QPP_OK) break;
        }
        HIPCHK(hipEventRecord(s->ev_out[c], s->s_out));
        if (tr) HIPCHK(hipEventRecord(s->tev[5][c], s->s_out));
        // hand back chunks whose D2H has already landed while later ones fly
        while (next_out < c) {
            if (hipEventQuery(s->ev_out[next_out]) != hipSuccess) {
                (void)hipGetLastError();  // hipErrorNotReady must not reach a later HIPCHK
                break;
            }
            hand_back(next_out++);
        }
    }
    if (rc != QPP_OK) return rc;
    const double t_sub = clk();
    const int early = next_out;
    for (int c = next_out; c < chunks; ++c) {
        HIPCHK(hipEventSynchronize(s->ev_out[c]));
        hand_back(c);
    }
    HIPCHK(hipStreamSynchronize(s->s_out));
    outg.wait();
    const double t_end = clk();
    if (tr) {
        qpp_trace &T = s->last;
        T = qpp_trace{};
        T.pipelined = 1;
        T.chunks = (uint32_t)chunks;
        T.total_ms = t_end - t_start;
        T.submit_ms = t_sub - t_start;
        T.copy_in_ms = t_copy_in;
        T.copy_out_ms = (double)outg.busy_ns.load() * 1e-6;
        T.wait_ms = t_end - t_sub;
        T.in_bytes = in_bytes;
        T.out_bytes = out_bytes;
        float ms = 0.f;
        for (int c = 0; c < chunks; ++c) {
            HIPCHK(hipEventElapsedTime(&ms, s->tev[0][c], s->tev[1][c]));
            T.h2d_ms += ms;
            HIPCHK(hipEventElapsedTime(&ms, s->tev[2][c], s->tev[3][c]));
            T.kernel_ms += ms;
            HIPCHK(hipEventElapsedTime(&ms, s->tev[4][c], s->tev[5][c]));
            T.d2h_ms += ms;
        }
        HIPCHK(hipEventElapsedTime(&ms, s->tev[0][0], s->tev[5][chunks - 1]));
        T.gpu_span_ms = ms;
    }
    if (trace_on())
        fprintf(stderr, "qpp session: %s %u packets %d chunks in %d out %d: submit %.2f ms, wait %.2f ms (%d handed back early)\n",
                enc ? "protect" : "unprotect", n, chunks, (int)in_direct, (int)out_direct,
                t_sub - t_start, t_end - t_sub, early);
    return QPP_OK;
}

// On a failure, drain the session's streams before returning, so no copy into
// its staging is still in flight when the staging is reused or freed.
static int session_drain_on_error(qpp_session *s, int rc)
{
    if (rc != QPP_OK && s) {
        if (s->s_in) (void)hipStreamSynchronize(s->s_in);
        (void)hipStreamSynchronize(s->stream);
        if (s->s_out) (void)hipStreamSynchronize(s->s_out);
        (void)hipGetLastError();
    }
    return rc;
}

constexpr uint32_t kSmallPackets = 64;
constexpr size_t kSmallBytes = (size_t)256 << 10;
static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static int session_run(bool enc, qpp_session *s, const qpp_keytab *kt, const qpp_desc *desc,
                       uint32_t n, const uint8_t *in, size_t in_len, uint8_t *out, size_t out_len,
                       qpp_result *res)
{
    if (!s || !kt || (n && (!desc || !res))) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    size_t need = in_len > out_len ? in_len : out_len;
    int rc = session_reserve(s, need, n);
    if (rc != QPP_OK) return rc;
    size_t want = out_len / kPipeChunkBytes;
    int chunks = want > (size_t)kPipeRegular ? kPipeRegular : (int)want;
    if (chunks > (int)n) chunks = (int)n;
    const char *serial = getenv("QPP_SESSION_SERIAL");  // A/B switch: "1" = serial path
    if (chunks >= 2 && !(serial && serial[0] == '1')) {
        bool mono = true;
        for (uint32_t i = 1; i < n && mono; ++i) mono = desc[i].out_off >= desc[i - 1].out_off;
        if (mono)
            return session_run_pipelined(enc, s, kt, desc, n, in, in_len, out, out_len, res,
                                         chunks);
    }
    // Small batches (the per-call object API: one packet per call): one H2D
    // copy of [descriptors | input | zeroed output] and one D2H copy of
    // [output | results] through the session's input staging, instead of
    // four copies and a device memset.
    const size_t sd = al256((size_t)n * sizeof(qpp_desc)), si = al256(in_len), so = al256(out_len);
    const size_t small = sd + si + so + (size_t)n * sizeof(qpp_result);
    if (n <= kSmallPackets && small <= kSmallBytes && in != s->h_in && out != s->h_out) {
        rc = session_reserve(s, small > need ? small : need, n);
        if (rc != QPP_OK) return rc;
        uint8_t *h = s->h_in, *d = s->d_in;
        memcpy(h, desc, (size_t)n * sizeof(qpp_desc));
        reject_out_of_bounds(enc, (qpp_desc *)h, n, in_len, out_len);
        if (in_len) memcpy(h + sd, in, in_len);
        memset(h + sd + si, 0, out_len);  // bytes the kernel does not write come back as zeros
        if (n <= std::min(lone_max(QPP_AES_128_GCM), lone_max(QPP_CHACHA20_POLY1305)) && lone_choice() &&
            zero_copy_choice()) {
            // one wave per packet; the output and results are written by
            // the kernel straight into the pinned staging (PCIe writes post;
            // reads there would put a bus round trip on each of the kernel's
            // dependent loads).  Descriptors and input: copied by the kernel
            // itself in one round trip when the call fits one workgroup,
            // else by one copy
            uint8_t *dh = s->hd_in;
            LoneStage st{dh, d, 0u};
            if (n <= (uint32_t)(kLoneWG / 64) && sd + si <= kLoneStageMax && lone_stage_choice())
                st.bytes = (uint32_t)(sd + si);  // 256-byte multiples
            else
                HIPCHK(hipMemcpyAsync(d, h, sd + si, hipMemcpyHostToDevice, s->stream));
            rc = launch_packets(enc, kt, (const qpp_desc *)d, n, d + sd, dh + sd + si,
                                (qpp_result *)(dh + sd + si + so), s->stream, nullptr, &st);
            if (rc != QPP_OK) return rc;
            HIPCHK(hipStreamSynchronize(s->stream));
            if (out_len) memcpy(out, h + sd + si, out_len);
            memcpy(res, h + sd + si + so, (size_t)n * sizeof(qpp_result));
            return QPP_OK;
        }
        HIPCHK(hipMemcpyAsync(d, h, sd + si + out_len, hipMemcpyHostToDevice, s->stream));
        rc = launch_packets(enc, kt, (const qpp_desc *)d, n, d + sd, d + sd + si,
                            (qpp_result *)(d + sd + si + so), s->stream);
        if (rc != QPP_OK) return rc;
        HIPCHK(hipMemcpyAsync(h + sd + si, d + sd + si, so + (size_t)n * sizeof(qpp_result),
                              hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        if (out_len) memcpy(out, h + sd + si, out_len);
        memcpy(res, h + sd + si + so, (size_t)n * sizeof(qpp_result));
        return QPP_OK;
    }
    qpp_desc *hd = (qpp_desc *)s->h_misc;
    qpp_result *hr = (qpp_result *)(s->h_misc + (size_t)s->max_packets * sizeof(qpp_desc));
    qpp_desc *dd = (qpp_desc *)s->d_misc;
    qpp_result *dr = (qpp_result *)(s->d_misc + (size_t)s->max_packets * sizeof(qpp_desc));
    memcpy(hd, desc, (size_t)n * sizeof(qpp_desc));
    reject_out_of_bounds(enc, hd, n, in_len, out_len);
    if (in_len && in != s->h_in) memcpy(s->h_in, in, in_len);  // staged by the caller already?
    HIPCHK(hipMemcpyAsync(dd, hd, (size_t)n * sizeof(qpp_desc), hipMemcpyHostToDevice, s->stream));
    if (in_len) HIPCHK(hipMemcpyAsync(s->d_in, s->h_in, in_len, hipMemcpyHostToDevice, s->stream));
    // bytes the kernel does not write (gaps, failed packets) come back as zeros
    if (out_len) HIPCHK(hipMemsetAsync(s->d_out, 0, out_len, s->stream));
    rc = session_launch(enc, s, kt, dd, n, dr);
    if (rc != QPP_OK) return rc;
    rc = session_d2h(s->h_out, s->hd_out, s->d_out, out_len, (uint8_t *)hr,
                     s->hd_misc + (size_t)s->max_packets * sizeof(qpp_desc), (const uint8_t *)dr,
                     (size_t)n * sizeof(qpp_result), s->stream);
    if (rc != QPP_OK) return rc;
    HIPCHK(hipStreamSynchronize(s->stream));
    if (out_len && out != s->h_out) memcpy(out, s->h_out, out_len);
    memcpy(res, hr, (size_t)n * sizeof(qpp_result));
    return QPP_OK;
}

int qpp_session_protect(qpp_session *s, const qpp_keytab *kt, const qpp_desc *desc, uint32_t n,
                        const uint8_t *in, size_t in_len, uint8_t *out, size_t out_len,
                        qpp_result *res)
{
    return session_drain_on_error(s, session_run(true, s, kt, desc, n, in, in_len, out, out_len, res));
}

int qpp_session_unprotect(qpp_session *s, const qpp_keytab *kt, const qpp_desc *desc,
                          uint32_t n, const uint8_t *in, size_t in_len, uint8_t *out,
                          size_t out_len, qpp_result *res)
{
    return session_drain_on_error(s, session_run(false, s, kt, desc, n, in, in_len, out, out_len, res));
}

int qpp_session_trace(qpp_session *s, int enable, qpp_trace *last)
{
    if (!s) return QPP_E_ARG;
    if (last) *last = s->last;
    if (enable > 0 && !s->tev[0][0]) {
        for (int k = 0; k < 6; ++k)
            for (int c = 0; c < kPipeMaxChunks; ++c)
                if (hipEventCreate(&s->tev[k][c]) != hipSuccess) {
                    (void)hipGetLastError();
                    for (int k2 = 0; k2 < 6; ++k2)
                        for (int c2 = 0; c2 < kPipeMaxChunks; ++c2) {
                            if (s->tev[k2][c2]) (void)hipEventDestroy(s->tev[k2][c2]);
                            s->tev[k2][c2] = nullptr;
                        }
                    return QPP_E_HIP;
                }
    }
    if (enable >= 0) s->trace = enable > 0;
    if (s->trace) s->last = qpp_trace{};  // a call that does not pipeline reports pipelined = 0
    return QPP_OK;
}

int qpp_session_stage(qpp_session *s, size_t bytes, uint32_t n, uint8_t **h_in, uint8_t **h_out)
{
    if (!s || !h_in || !h_out) return QPP_E_ARG;
    const int rc = session_reserve(s, bytes, n);
    if (rc != QPP_OK) return rc;
    *h_in = s->h_in;
    *h_out = s->h_out;
    return QPP_OK;
}

int qpp_session_hp_mask(qpp_session *s, const qpp_keytab *kt, const uint32_t *slots,
                        const uint8_t *samples, uint32_t n, uint8_t *masks)
{
    if (!s || !kt || (n && (!slots || !samples || !masks))) return QPP_E_ARG;
    if (n == 0) return QPP_OK;
    int rc = session_reserve(s, (size_t)n * 32, n);
    if (rc != QPP_OK) return rc;
    uint8_t *hs = s->h_in, *hm = s->h_out;
    uint32_t *hidx = (uint32_t *)s->h_misc;
    memcpy(hidx, slots, (size_t)n * 4);
    memcpy(hs, samples, (size_t)n * 16);
    if (n <= kSmallPackets && zero_copy_choice()) {
        rc = qpp_hp_mask(kt, (const uint32_t *)s->hd_misc, s->hd_in, n, s->hd_out, s->stream);
        if (rc != QPP_OK) return rc;
        HIPCHK(hipStreamSynchronize(s->stream));
        memcpy(masks, hm, (size_t)n * 16);
        return QPP_OK;
    }
    HIPCHK(hipMemcpyAsync(s->d_misc, hidx, (size_t)n * 4, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(s->d_in, hs, (size_t)n * 16, hipMemcpyHostToDevice, s->stream));
    rc = qpp_hp_mask(kt, (const uint32_t *)s->d_misc, s->d_in, n, s->d_out, s->stream);
    if (rc != QPP_OK) return rc;
    HIPCHK(hipMemcpyAsync(hm, s->d_out, (size_t)n * 16, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    memcpy(masks, hm, (size_t)n * 16);
    return QPP_OK;
}

int qpp_session_set_keys(qpp_session *s, qpp_keytab *kt, const qpp_key_material *km, uint32_t n)
{
    if (!s) return QPP_E_ARG;
    return qpp_keytab_set(kt, km, n, s->stream);
}

// ------------------------------------------------------ several devices --
//
// One host batch over several GPUs of the node (packets
// are independent, so no collective): a session and a replica of the key
// table per device; the batch is cut into contiguous descriptor ranges, one
// per device, each range's input and output extents are staged and run by its
// own host thread on its own device, and every result lands at its packet's
// position in the caller's arrays.  Each range needs its own output extent,
// so the ranges' output extents must not overlap (descriptors in output
// order, the layout of a socket batch); otherwise the batch runs on the first
// device alone.  Output bytes outside every packet are zeros, as for one
// session.

struct qpp_multi {
    int n;
    int device[kMultiMaxDevices];
    qpp_session *s[kMultiMaxDevices];
    qpp_keytab *kt[kMultiMaxDevices];
};

int qpp_multi_create(const int *devices, int n_devices, uint32_t key_capacity, qpp_multi **out)
{
    if (!out || !devices || n_devices < 1 || n_devices > kMultiMaxDevices) return QPP_E_ARG;
    *out = NULL;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return QPP_E_NODEV;
    for (int k = 0; k < n_devices; ++k)
        if (devices[k] < 0 || devices[k] >= count) return QPP_E_ARG;
    qpp_multi *m = (qpp_multi *)calloc(1, sizeof(qpp_multi));
    if (!m) return QPP_E_NOMEM;
    int prev = 0;
    (void)hipGetDevice(&prev);
    int rc = QPP_OK;
    for (int k = 0; k < n_devices && rc == QPP_OK; ++k) {
        m->device[k] = devices[k];
        if (hipSetDevice(devices[k]) != hipSuccess) rc = QPP_E_HIP;
        if (rc == QPP_OK) rc = qpp_session_create(1 << 16, 64, &m->s[k]);
        if (rc == QPP_OK) rc = qpp_keytab_create(key_capacity, &m->kt[k]);
        m->n = k + 1;
    }
    (void)hipSetDevice(prev);
    if (rc != QPP_OK) {
        qpp_multi_destroy(m);
        return rc;
    }
    *out = m;
    return QPP_OK;
}

void qpp_multi_destroy(qpp_multi *m)
{
    if (!m) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (int k = 0; k < m->n; ++k) {
        (void)hipSetDevice(m->device[k]);
        qpp_session_destroy(m->s[k]);
        qpp_keytab_destroy(m->kt[k]);
    }
    (void)hipSetDevice(prev);
    free(m);
}

int qpp_multi_devices(const qpp_multi *m) { return m ? m->n : 0; }

int qpp_multi_set_keys(qpp_multi *m, const qpp_key_material *km, uint32_t n)
{
    if (!m) return QPP_E_ARG;
    int prev = 0, rc = QPP_OK;
    (void)hipGetDevice(&prev);
    for (int k = 0; k < m->n && rc == QPP_OK; ++k) {
        if (hipSetDevice(m->device[k]) != hipSuccess) rc = QPP_E_HIP;
        if (rc == QPP_OK) rc = qpp_session_set_keys(m->s[k], m->kt[k], km, n);
        if (rc == QPP_OK) rc = hipStreamSynchronize((hipStream_t)qpp_session_stream(m->s[k])) == hipSuccess
                                   ? QPP_OK : QPP_E_HIP;
    }
    (void)hipSetDevice(prev);
    return rc;
}

static int multi_run(bool enc, qpp_multi *m, const qpp_desc *desc, uint32_t n, const uint8_t *in,
                     size_t in_len, uint8_t *out, size_t out_len, qpp_result *res)
{
    if (!m || (n && (!desc || !res))) return QPP_E_ARG;
    if (n == 0) {
        if (out_len) memset(out, 0, out_len);
        return QPP_OK;
    }
    if (m->n == 1) {
        // one device: the session itself (its bounds checks and staging),
        // without the range split's copy and passes over the descriptors
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(m->device[0]);
        const int rc = enc ? qpp_session_protect(m->s[0], m->kt[0], desc, n, in, in_len, out, out_len, res)
                           : qpp_session_unprotect(m->s[0], m->kt[0], desc, n, in, in_len, out, out_len, res);
        (void)hipSetDevice(prev);
        return rc;
    }
    int parts = m->n < (int)n ? m->n : (int)n;
    // bounds first (as a session does), so that extents use only packets
    // that fit; rejected ones stay rejected in their range and touch nothing
    std::vector<qpp_desc> d(desc, desc + n);
    reject_out_of_bounds(enc, d.data(), n, in_len, out_len);
    struct Range {
        uint32_t b, e;
        size_t ilo, ihi, olo, ohi;
    };
    std::vector<Range> r(parts);
    for (int k = 0; k < parts; ++k) {
        Range &x = r[k];
        x.b = (uint32_t)((uint64_t)n * k / parts);
        x.e = (uint32_t)((uint64_t)n * (k + 1) / parts);
        x.ilo = x.olo = SIZE_MAX;
        x.ihi = x.ohi = 0;
        for (uint32_t i = x.b; i < x.e; ++i) {
            if (d[i].flags & kFlagReject) continue;
            const size_t rd = enc ? (size_t)d[i].hdr_len + d[i].len : d[i].len;
            const size_t wr = enc ? rd + QPP_TAG_LEN : rd;
            x.ilo = std::min<size_t>(x.ilo, d[i].in_off);
            x.ihi = std::max<size_t>(x.ihi, d[i].in_off + rd);
            x.olo = std::min<size_t>(x.olo, d[i].out_off);
            x.ohi = std::max<size_t>(x.ohi, d[i].out_off + wr);
        }
        if (x.ilo == SIZE_MAX) x.ilo = x.ihi = x.olo = x.ohi = 0;
    }
    // ranges in output order with disjoint extents, or one device: every
    // non-empty range starts at or after the end of all earlier non-empty
    // ones (an empty range -- every packet rejected -- compares with nothing)
    size_t seen_hi = 0;
    bool seen = false;
    for (int k = 0; k < parts; ++k) {
        if (r[k].ohi <= r[k].olo) continue;
        if (seen && seen_hi > r[k].olo) {
            parts = 1;
            r.assign(1, Range{0, n, 0, in_len, 0, out_len});
            break;
        }
        seen_hi = std::max(seen_hi, r[k].ohi);
        seen = true;
    }
    if (parts == 1) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(m->device[0]);
        const int rc = enc ? qpp_session_protect(m->s[0], m->kt[0], desc, n, in, in_len, out, out_len, res)
                           : qpp_session_unprotect(m->s[0], m->kt[0], desc, n, in, in_len, out, out_len, res);
        (void)hipSetDevice(prev);
        return rc;
    }
    // rebase each range onto its extents
    for (int k = 0; k < parts; ++k)
        for (uint32_t i = r[k].b; i < r[k].e; ++i) {
            if (d[i].flags & kFlagReject) {
                // past every range buffer: the range's session rejects it again
                d[i].in_off = d[i].out_off = ~0ull;
                continue;
            }
            d[i].in_off -= r[k].ilo;
            d[i].out_off -= r[k].olo;
        }
    // output bytes outside every range's extent: zeros, as one session leaves them
    size_t pos = 0;
    for (int k = 0; k < parts; ++k) {
        if (r[k].ohi <= r[k].olo) continue;
        if (r[k].olo > pos) memset(out + pos, 0, r[k].olo - pos);
        pos = r[k].ohi;
    }
    if (out_len > pos) memset(out + pos, 0, out_len - pos);
    std::vector<int> rcs(parts, QPP_OK);
    std::vector<std::thread> th;
    for (int k = 0; k < parts; ++k)
        th.emplace_back([&, k] {
            const Range &x = r[k];
            if (hipSetDevice(m->device[k]) != hipSuccess) {
                rcs[k] = QPP_E_HIP;
                return;
            }
            const uint32_t cnt = x.e - x.b;
            rcs[k] = enc ? qpp_session_protect(m->s[k], m->kt[k], d.data() + x.b, cnt, in + x.ilo, x.ihi - x.ilo,
                                               out + x.olo, x.ohi - x.olo, res + x.b)
                         : qpp_session_unprotect(m->s[k], m->kt[k], d.data() + x.b, cnt, in + x.ilo, x.ihi - x.ilo,
                                                 out + x.olo, x.ohi - x.olo, res + x.b);
        });
    for (auto &t : th) t.join();
    for (int k = 0; k < parts; ++k)
        if (rcs[k] != QPP_OK) return rcs[k];
    return QPP_OK;
}

int qpp_multi_protect(qpp_multi *m, const qpp_desc *desc, uint32_t n, const uint8_t *in, size_t in_len,
                      uint8_t *out, size_t out_len, qpp_result *res)
{
    return multi_run(true, m, desc, n, in, in_len, out, out_len, res);
}

int qpp_multi_unprotect(qpp_multi *m, const qpp_desc *desc, uint32_t n, const uint8_t *in, size_t in_len,
                        uint8_t *out, size_t out_len, qpp_result *res)
{
    return multi_run(false, m, desc, n, in, in_len, out, out_len, res);
}

int qpp_multi_trace(qpp_multi *m, int enable, qpp_trace *last, int max)
{
    if (!m || max < 0 || (max > 0 && !last)) return QPP_E_ARG;
    int prev = 0, rc = QPP_OK, k = 0;
    (void)hipGetDevice(&prev);
    for (; k < m->n && rc == QPP_OK; ++k) {
        if (hipSetDevice(m->device[k]) != hipSuccess) rc = QPP_E_HIP;
        if (rc == QPP_OK) rc = qpp_session_trace(m->s[k], enable, k < max ? last + k : nullptr);
    }
    (void)hipSetDevice(prev);
    return rc == QPP_OK ? (m->n < max ? m->n : max) : rc;
}

}  // extern "C"
