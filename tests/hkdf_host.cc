// Host build of aioquic_amd/csrc/qpp_hkdf.h for the CPU test (tests/test_hkdf.py).
#include "../aioquic_amd/csrc/qpp_hkdf.h"

extern "C" int qpp_test_expand_label(int big, const uint8_t *secret, int secret_len,
                                     const char *label, int label_len, int length, uint8_t *out)
{
    qpp_hkdf::Hmac m;
    qpp_hkdf::hmac_init(m, big != 0, secret, secret_len);
    qpp_hkdf::expand_label(m, label, label_len, length, out);
    return 0;
}
