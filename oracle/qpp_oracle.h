/* qpp_oracle.h -- CPU oracle (TEST INFRASTRUCTURE ONLY; see qpp_oracle.c header). */
#ifndef QPP_ORACLE_H
#define QPP_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#define QO_AES_128_GCM 0
#define QO_AES_256_GCM 1
#define QO_CHACHA20_POLY1305 2

#define QO_PACKET_MAX 1500 /* _crypto.c:13 PACKET_LENGTH_MAX */

#define QO_E_LENGTH (-1)
#define QO_E_DECRYPT (-2)

#ifdef __cplusplus
extern "C" {
#endif

int qo_aes_expand(const uint8_t *key, int key_len, uint32_t *rk);
void qo_aes_block(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16]);
void qo_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                       uint8_t out[64]);

long qo_aead_encrypt(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *data,
                     size_t len, const uint8_t *aad, size_t alen, uint64_t pn, uint8_t *out);
long qo_aead_decrypt(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *data,
                     size_t len, const uint8_t *aad, size_t alen, uint64_t pn, uint8_t *out);

void qo_hp_mask(int suite, const uint8_t *hp_key, const uint8_t sample[16], uint8_t mask[16]);
int qo_hp_apply(int suite, const uint8_t *hp_key, const uint8_t *hdr, size_t hlen,
                const uint8_t *payload, size_t plen, uint8_t *out);
int qo_hp_remove(int suite, const uint8_t *hp_key, const uint8_t *pkt, size_t len,
                 size_t pn_off, uint8_t *hdr_out, uint32_t *pn_trunc);
uint64_t qo_decode_pn(int64_t truncated, int num_bits, uint64_t expected);
int64_t qo_pn_trunc_as_int(uint32_t t);

long qo_protect(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp_key,
                const uint8_t *hdr, size_t hlen, const uint8_t *payload, size_t plen,
                uint64_t pn, uint8_t *out);
long qo_unprotect(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp_key,
                  const uint8_t *pkt, size_t len, size_t pn_off, uint64_t expected_pn,
                  uint8_t *out, size_t *hdr_len, uint64_t *pn);
long qo_unprotect_ex(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp_key,
                     const uint8_t *pkt, size_t len, size_t pn_off, uint64_t expected_pn,
                     uint8_t *out, size_t *hdr_len, uint64_t *pn, int rfc_pn);

/* Batch forms over the product's descriptor layout (include/quic_pp.h), so a
 * test can run the oracle and the GPU on byte-identical inputs.  keys is
 * indexed by qpp_desc.slot; a slot whose suite is 0xff is "not installed". */
struct qpp_key_material;
struct qpp_desc;
struct qpp_result;
void qo_protect_batch(const struct qpp_key_material *keys, uint32_t n_keys,
                      const struct qpp_desc *desc, uint32_t n, const uint8_t *in, uint8_t *out,
                      struct qpp_result *res);
void qo_unprotect_batch(const struct qpp_key_material *keys, uint32_t n_keys,
                        const struct qpp_desc *desc, uint32_t n, const uint8_t *in, uint8_t *out,
                        struct qpp_result *res);

#ifdef __cplusplus
}
#endif
#endif
