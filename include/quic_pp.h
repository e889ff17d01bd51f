/*
 * quic_pp.h -- C ABI of the MI355X QUIC packet-protection engine (libquicpp.so).
 *
 * This is the drop-in boundary for aioquic's per-packet protection path.  The
 * reference binds that path as a CPython extension, aioquic._crypto
 * (src/aioquic/_crypto.c, API stub src/aioquic/_crypto.pyi:1-15), called from
 * src/aioquic/quic/crypto.py:4.  Each entry point below names the reference
 * function(s) it replaces.  Plain pointers and sizes only: no HIP, torch or
 * Python types cross this boundary (streams are passed as void*, i.e. a
 * hipStream_t; NULL = the null stream).
 *
 * Threading: a qpp_keytab may be shared between threads for launches; setting
 * keys and launching on the same slots concurrently is the caller's race (as
 * with the reference's per-object scratch, _crypto.c:39-42).  A qpp_session and
 * a qpp_plan are single-threaded: use one per thread (the CPython binding
 * keeps one session per OS thread).
 *
 * Buffers: the device-pointer launches (qpp_protect, qpp_unprotect and the
 * planned forms) cannot see buffer sizes, so every descriptor's input and
 * output extents must lie inside the caller's allocations, and the 16
 * packets of one wavefront (consecutive descriptors, or consecutive in a
 * plan's bucket order) must lie within 4 GiB of each other (else
 * QPP_S_LENGTH).  The session forms check every descriptor against in_len /
 * out_len and report QPP_S_LENGTH for one that does not fit, without touching
 * memory for it.
 *
 * Authentication failures: unprotect decrypts as it authenticates, so the
 * plaintext of a packet whose tag does not verify is produced before the
 * verdict.  The kernels then overwrite that packet's payload region at
 * out_off + hdr_len with zeros (out_len = 0), so no unauthenticated plaintext
 * is left in the output.  An in-place unprotect (in == out) of a forged
 * packet therefore also destroys its ciphertext, as the reference's copy-out
 * semantics never do (_crypto.c:145-154 returns an error, not bytes).
 */
#ifndef QUIC_PP_H
#define QUIC_PP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QPP_ABI_VERSION 3

/* cipher suites (quic/crypto.py:12-16 CIPHER_SUITES) */
#define QPP_AES_128_GCM 0        /* aes-128-gcm + aes-128-ecb header protection */
#define QPP_AES_256_GCM 1        /* aes-256-gcm + aes-256-ecb header protection */
#define QPP_CHACHA20_POLY1305 2  /* chacha20-poly1305 + chacha20 header protection */

#define QPP_PACKET_MAX 1500      /* _crypto.c:13 PACKET_LENGTH_MAX */
#define QPP_TAG_LEN 16           /* _crypto.c:11 AEAD_TAG_LENGTH */
#define QPP_MAX_HDR 1500         /* longest header / associated data the kernels accept */

/* return codes of the API calls */
#define QPP_OK 0
#define QPP_E_ARG (-1)           /* bad argument (NULL, n too large, bad slot) */
#define QPP_E_HIP (-2)           /* a HIP runtime call failed */
#define QPP_E_NODEV (-3)         /* no usable gfx950 device */
#define QPP_E_NOMEM (-4)

/* per-packet status codes (qpp_result.status) */
#define QPP_S_OK 0
#define QPP_S_LENGTH 1      /* "Invalid payload length" (_crypto.c:126-129,168-171) or sample out of range */
#define QPP_S_DECRYPT 2     /* "Payload decryption failed" (_crypto.c:148-152) */
#define QPP_S_KEY_PHASE 3   /* short header whose key-phase bit differs from the slot's
                               (quic/crypto.py:91-96): caller retries with the next-phase key */
#define QPP_S_NO_KEY 4      /* slot never installed: KeyUnavailableError (quic/crypto.py:78-79) */
#define QPP_S_INTERNAL 5    /* the engine gave up on the packet: a bounded wait inside a kernel
                               (a GHASH table entry, a two-wave hand-over) ran out.  Nothing at
                               out_off is valid (unprotect: no plaintext is left there), and the
                               call raises CryptoError, as a failed reference call does
                               (_crypto.c:17-29).  Never expected; counted by qpp_watchdog_count */

/* descriptor flags */
#define QPP_F_NO_HP 1u      /* AEAD only (AEAD.encrypt/.decrypt): no header protection, no
                               packet-number decode, no key-phase check; hdr_len = AAD length */
#define QPP_F_RFC_PN 2u     /* decode a 4-byte truncated packet number as unsigned (RFC 9000
                               App. A.3).  Default: bit-exact with the reference, which hands
                               the truncated number to Python as a signed int (_crypto.c:349),
                               so values >= 2^31 decode differently once pn >= 2^32. */

/* One packet of a batch.  Offsets are byte offsets into the caller's device
 * buffers; no alignment is required. */
typedef struct qpp_desc {
    uint64_t in_off;   /* protect: header then payload; unprotect: the protected packet */
    uint64_t out_off;  /* protect: header||ciphertext||tag; unprotect: header||plaintext */
    uint32_t len;      /* protect: payload length; unprotect: packet length (>= pn_off + 20) */
    uint16_t hdr_len;  /* protect: header (= AAD) length; unprotect: packet-number offset
                          ("encrypted_offset"), or the AAD length with QPP_F_NO_HP */
    uint16_t flags;    /* QPP_F_* */
    uint64_t pn;       /* protect: packet number; unprotect: expected packet number,
                          or the exact packet number with QPP_F_NO_HP */
    uint32_t slot;     /* key-table slot */
    uint32_t rsv;
} qpp_desc;            /* 40 bytes */

typedef struct qpp_result {
    uint64_t pn;       /* unprotect: decoded packet number; protect: pn used */
    uint16_t status;   /* QPP_S_* */
    uint16_t hdr_len;  /* plain header length (pn_off + pn_len for unprotect) */
    uint32_t out_len;  /* bytes written at out_off */
} qpp_result;          /* 16 bytes */

/* Raw key material for one slot, as produced by derive_key_iv_hp
 * (quic/crypto.py:34-56).  key/hp use 16 bytes for AES-128, 32 otherwise. */
typedef struct qpp_key_material {
    uint32_t slot;
    uint8_t suite;      /* QPP_AES_128_GCM / QPP_AES_256_GCM / QPP_CHACHA20_POLY1305 */
    uint8_t key_phase;  /* 0/1, compared with bit 2 of a short header */
    uint8_t rsv[2];
    uint8_t iv[12];
    uint8_t key[32];
    uint8_t hp[32];
} qpp_key_material;     /* 84 bytes */

/* One connection's traffic secret for the batched key schedule (qpp_keytab_derive). */
#define QPP_DERIVE_V2 1u    /* QUIC v2 labels "quicv2 key/iv/hp" (quic/crypto.py:52-56) */

typedef struct qpp_secret {
    uint32_t slot;
    uint8_t suite;       /* QPP_AES_128_GCM (SHA-256) / QPP_AES_256_GCM (SHA-384) /
                            QPP_CHACHA20_POLY1305 (SHA-256), tls.py:1108-1112 */
    uint8_t key_phase;
    uint8_t flags;       /* QPP_DERIVE_* */
    uint8_t secret_len;  /* bytes of secret[] used: 1..64 */
    uint32_t updates;    /* key updates applied first: secret = HKDF-Expand-Label(secret,
                            "quic ku", "", hash_len) per step (next_key_phase,
                            quic/crypto.py:157-168; the label is "quic ku" for v2 too) */
    uint32_t rsv;
    uint8_t secret[64];
} qpp_secret;            /* 80 bytes */

typedef struct qpp_keytab qpp_keytab;   /* device-resident expanded keys */
typedef struct qpp_session qpp_session; /* pinned staging + device buffers + stream */

/* library / device */
int qpp_abi_version(void);
/* 16 hex digits: the hash of the native sources the library was built from
 * (aioquic_amd/_srchash.py); a binding checks it against its own at load. */
const char *qpp_source_hash(void);
/* Watchdog events on the current device since the library loaded: a launch
 * whose kernel waited ~1 s for a GHASH table entry (that key slot's packets),
 * or a two-wave packet whose hand-over timed out, reported QPP_S_INTERNAL
 * for the packets concerned.  Never expected
 * (it would be a bug); tests check it stays 0.  A synchronous read. */
uint32_t qpp_watchdog_count(void);
/* Single-key AES-GCM launches (process-wide, since the library loaded) that
 * found all of their key table's launch-pool slots held by launches still in
 * flight and so ran without the launch-wide item pool (static shares only;
 * the same bytes, a possibly longer tail).  Diagnostic. */
uint64_t qpp_pool_fallbacks(void);
const char *qpp_strerror(int rc);
int qpp_device_check(void);             /* QPP_OK if the current device is gfx950 */

/* Key tables.  qpp_keytab_set replaces AEAD_init (_crypto.c:68-102) and
 * HeaderProtection_init (_crypto.c:232-266): one device launch expands AES
 * round keys, H = E_K(0^128) and the GHASH tables for every slot in km. */
int qpp_keytab_create(uint32_t capacity, qpp_keytab **out);
/* Every launch that uses the table must have completed (its stream
 * synchronized) before the table is destroyed. */
void qpp_keytab_destroy(qpp_keytab *kt);
uint32_t qpp_keytab_capacity(const qpp_keytab *kt);
int qpp_keytab_set(qpp_keytab *kt, const qpp_key_material *km, uint32_t n, void *stream);
int qpp_keytab_clear(qpp_keytab *kt, const uint32_t *slots, uint32_t n, void *stream);
/* Batched CryptoContext.setup (quic/crypto.py:121-136) for n connections at once:
 * derive_key_iv_hp (quic/crypto.py:34-56 = HKDF-Expand-Label, tls.py:164-185)
 * on the device, one lane per secret, after `updates` key updates, then the same
 * slot expansion as qpp_keytab_set.  km_out (host memory, may be NULL) receives
 * the derived key material, e.g. for the host-side AEAD objects. */
int qpp_keytab_derive(qpp_keytab *kt, const qpp_secret *sec, uint32_t n,
                      qpp_key_material *km_out, void *stream);

/* Batched packet protection on device buffers (asynchronous on `stream`).
 * qpp_protect replaces AEAD_encrypt (_crypto.c:157-194) + HeaderProtection_apply
 * (_crypto.c:289-319), i.e. CryptoContext.encrypt_packet (quic/crypto.py:105-116).
 * qpp_unprotect replaces HeaderProtection_remove (_crypto.c:321-350) +
 * decode_packet_number (quic/packet.py:118-132) + AEAD_decrypt (_crypto.c:115-155),
 * i.e. CryptoContext.decrypt_packet (quic/crypto.py:75-103).
 * Packets with the same slot should be contiguous for speed (any order is correct). */
int qpp_protect(const qpp_keytab *kt, const qpp_desc *d_desc, uint32_t n, const uint8_t *d_in,
                uint8_t *d_out, qpp_result *d_res, void *stream);
int qpp_unprotect(const qpp_keytab *kt, const qpp_desc *d_desc, uint32_t n,
                  const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res, void *stream);

/* Bucketing by (suite, key slot).  A server's batch interleaves many
 * connections (src/aioquic/asyncio/server.py:60-152 demultiplexes them per
 * datagram), but a kernel wants each workgroup on one key and one suite.
 * qpp_plan_build sorts the batch's packet indices on the device by
 * (suite, slot) and counts the packets of each suite; the order of the
 * packets within one (suite, slot) run is unspecified (results are mapped
 * back to the caller's order, so it is not observable).  A *_planned launch gathers its descriptors into that order, runs
 * each suite's kernel over its own bucket only, and writes every result at
 * the packet's position in the CALLER's descriptor order.  A plan is built
 * once per batch and serves every launch over descriptors with the same
 * slots in the same positions (e.g. protect, then unprotect of the same
 * packets).  Asynchronous on `stream`; a plan serves one stream at a time.
 * Empty or unknown slots are reported QPP_S_NO_KEY, as by qpp_protect. */
typedef struct qpp_plan qpp_plan;
int qpp_plan_create(uint32_t max_packets, qpp_plan **out);
void qpp_plan_destroy(qpp_plan *p);
int qpp_plan_build(qpp_plan *p, const qpp_keytab *kt, const qpp_desc *d_desc, uint32_t n,
                   void *stream);
int qpp_protect_planned(const qpp_keytab *kt, const qpp_plan *p, const qpp_desc *d_desc,
                        uint32_t n, const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res,
                        void *stream);
int qpp_unprotect_planned(const qpp_keytab *kt, const qpp_plan *p, const qpp_desc *d_desc,
                          uint32_t n, const uint8_t *d_in, uint8_t *d_out, qpp_result *d_res,
                          void *stream);

/* Header-protection masks: replaces HeaderProtection_mask (_crypto.c:278-287).
 * d_samples: n x 16 bytes, d_masks: n x 16 bytes (first 5 used). */
int qpp_hp_mask(const qpp_keytab *kt, const uint32_t *d_slots, const uint8_t *d_samples,
                uint32_t n, uint8_t *d_masks, void *stream);

/* Synchronous host-buffer forms (pinned staging, H2D, kernel, D2H), used by the
 * per-packet object API and the batched send/receive callers.  A batch with at
 * least 64 MiB of output and out_off non-decreasing in descriptor order runs as
 * a chunked H2D / kernel / D2H pipeline on three streams (QPP_SESSION_SERIAL=1
 * in the environment forces the serial form); the bytes written are the same. */
int qpp_session_create(size_t max_bytes, uint32_t max_packets, qpp_session **out);
void qpp_session_destroy(qpp_session *s);
void *qpp_session_stream(qpp_session *s);
int qpp_session_protect(qpp_session *s, const qpp_keytab *kt, const qpp_desc *desc, uint32_t n,
                        const uint8_t *in, size_t in_len, uint8_t *out, size_t out_len,
                        qpp_result *res);
int qpp_session_unprotect(qpp_session *s, const qpp_keytab *kt, const qpp_desc *desc,
                          uint32_t n, const uint8_t *in, size_t in_len, uint8_t *out,
                          size_t out_len, qpp_result *res);
int qpp_session_hp_mask(qpp_session *s, const qpp_keytab *kt, const uint32_t *slots,
                        const uint8_t *samples, uint32_t n, uint8_t *masks);
/* The session's own pinned staging buffers, sized for at least `bytes` of
 * input and of output and n packets; valid until the next call on the
 * session.  A caller that assembles its input straight into *h_in and passes
 * h_in / h_out as `in` / `out` to qpp_session_protect / _unprotect saves both
 * staging copies (the batched Python callers do). */
int qpp_session_stage(qpp_session *s, size_t bytes, uint32_t n, uint8_t **h_in, uint8_t **h_out);
int qpp_session_set_keys(qpp_session *s, qpp_keytab *kt, const qpp_key_material *km,
                         uint32_t n);

/* Phases of one pipelined host-buffer call (the chunked form of
 * qpp_session_protect / _unprotect), for a caller that wants to see where a
 * host batch's time goes: host copies into and out of pinned staging, both
 * PCIe directions and the kernels.  GPU phases come from timing events around
 * every chunk's H2D, kernels and D2H (sums of the chunks' durations; the
 * engines overlap, so they add up to more than the call). */
typedef struct qpp_trace {
    uint32_t pipelined;  /* 1 if the last call ran as the chunked pipeline (else the rest is 0) */
    uint32_t chunks;
    double total_ms;     /* the call, entry to return */
    double submit_ms;    /* the submission loop: staging copies in, enqueues, early hand-backs */
    double copy_in_ms;   /* caller -> pinned staging copies, wall time on the calling thread */
    double copy_out_ms;  /* pinned staging -> caller copies, summed over the copy threads' tasks */
    double wait_ms;      /* after the submission loop: the last chunks' D2H and copy-out */
    double h2d_ms;       /* sum of the chunks' H2D durations (descriptors and input) */
    double kernel_ms;    /* sum of the chunks' kernel durations */
    double d2h_ms;       /* sum of the chunks' D2H durations (output and results) */
    double gpu_span_ms;  /* first H2D start to last D2H end */
    double in_bytes, out_bytes;  /* bytes sent H2D / returned D2H */
} qpp_trace;
/* enable != 0 turns tracing on for the session's following calls (0 off, -1
 * unchanged); last (may be NULL) receives the previous traced call's phases. */
int qpp_session_trace(qpp_session *s, int enable, qpp_trace *last);


/* One host batch over several GPUs of the node (the
 * server socket of src/aioquic/asyncio/server.py:60-152 feeds all
 * connections, and that is the batch to split).  A qpp_multi holds a session
 * and a replica of the key table per device; *_protect / *_unprotect cut the
 * batch into contiguous descriptor ranges, one per device, run them at once
 * (one host thread each) and write every result at its packet's position in
 * the caller's arrays -- the same bytes and results as one session.  Ranges
 * need disjoint output extents (descriptors in output order); otherwise the
 * batch runs on the first device.  Up to 16 devices; a device may be listed
 * twice (two sessions on one GPU).  Like a session, single-threaded. */
typedef struct qpp_multi qpp_multi;
int qpp_multi_create(const int *devices, int n_devices, uint32_t key_capacity, qpp_multi **out);
void qpp_multi_destroy(qpp_multi *m);
int qpp_multi_devices(const qpp_multi *m);
int qpp_multi_set_keys(qpp_multi *m, const qpp_key_material *km, uint32_t n);
int qpp_multi_protect(qpp_multi *m, const qpp_desc *desc, uint32_t n, const uint8_t *in, size_t in_len,
                      uint8_t *out, size_t out_len, qpp_result *res);
int qpp_multi_unprotect(qpp_multi *m, const qpp_desc *desc, uint32_t n, const uint8_t *in, size_t in_len,
                        uint8_t *out, size_t out_len, qpp_result *res);
/* qpp_session_trace on every device's session; last[k] for device k (up to
 * max entries).  Returns the number of devices written, or a QPP_E_* code. */
int qpp_multi_trace(qpp_multi *m, int enable, qpp_trace *last, int max);

#ifdef __cplusplus
}
#endif
#endif
