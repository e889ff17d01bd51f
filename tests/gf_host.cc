// Host build of aioquic_amd/csrc/qpp_gf128.h for the CPU unit test
// (tests/test_gf128.py): n products of 16-byte blocks.
#include <stdint.h>
#include <string.h>

#include "../aioquic_amd/csrc/qpp_gf128.h"

extern "C" void qpp_test_gf_mul(const uint8_t *x, const uint8_t *y, uint8_t *out, int n)
{
    for (int i = 0; i < n; ++i) {
        qpp::gf::Blk a, b;
        memcpy(a.w, x + 16 * i, 16);
        memcpy(b.w, y + 16 * i, 16);
        const qpp::gf::Blk c = qpp::gf::mul(a, b);
        memcpy(out + 16 * i, c.w, 16);
    }
}
