// Phase times of the one-packet kernels (k_lone_gcm, k_lone_chacha) on the
// object API's path: the engine built with -DQPP_PROBE, qpp_session_protect /
// _unprotect of one 1200-byte packet per call (the call staged by the
// kernel), wave 0's marks averaged over the calls.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DQPP_PROBE -c -o /tmp/lone_probe.o tools/lone_probe.hip && \
//        hipcc --offload-arch=gfx950 -o tools/lone_probe /tmp/lone_probe.o build/obj/qpp_plan.o
// Run:   tools/lone_probe [calls] [suite: 0 AES-128-GCM, 2 ChaCha20-Poly1305]
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../aioquic_amd/csrc/qpp_engine.hip"

#ifndef QPP_PROBE  // without the marks: the calls and their statuses only
constexpr int kProbeSlots = 16, kProbeStart = 13, kProbeEnd = 14;
#endif

static const char *kNamesChacha[] = {"staging read", "barrier, descriptor", "the slot's suite",
                                     "header, pkt_begin (unprotect: HP removal)", "inputs requested, key",
                                     "the ChaCha20 block", "Horner and r^e (prefix product), outputs",
                                     "scaling multiply, wave sum, tag",
                                     "protect: HP, tag, header / unprotect: tag check", "result"};
static const char *const *g_names;
static const char *kNames[] = {"staging read, AES image", "barrier, descriptor", "the slot's suite",
                               "header, pkt_begin (unprotect: HP removal)",
                               "inputs/powers requested, round keys, counter cache", "AES-CTR",
                               "output stores, the inputs' wait", "GHASH: powers' wait, multiplies, wave xor",
                               "protect: HP, tag, header / unprotect: tag check", "result"};

static int run(qpp_session *s, qpp_keytab *kt, bool enc, int calls, std::vector<uint8_t> &pkt)
{
    std::vector<uint8_t> plain(11 + 1173), out(1200);
    for (size_t i = 0; i < plain.size(); ++i) plain[i] = (uint8_t)(i * 7 + 3);
    plain[0] = 0x41;  // short header, 2-byte packet number 5 at offset 9
    plain[9] = 0;
    plain[10] = 5;
    std::vector<unsigned long long> zero(kProbeSlots * 16, 0), g(kProbeSlots * 16);
    double sum[10] = {}, span = 0;
    int n_ok = 0;
    for (int c = 0; c < calls; ++c) {
#ifdef QPP_PROBE
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_probe), zero.data(), zero.size() * 8) != hipSuccess) return 1;
#endif
        qpp_result r;
        int rc;
        if (enc) {
            const qpp_desc d = {0, 0, 1173, 11, 0, 5, 0, 0};
            rc = qpp_session_protect(s, kt, &d, 1, plain.data(), plain.size(), out.data(), out.size(), &r);
            pkt = out;
        } else {
            const qpp_desc d = {0, 0, 1200, 9, 0, 5, 0, 0};
            rc = qpp_session_unprotect(s, kt, &d, 1, pkt.data(), pkt.size(), out.data(), out.size(), &r);
        }
        if (rc != QPP_OK || r.status != QPP_S_OK) {
            printf("call %d: rc %d status %d\n", c, rc, r.status);
            return 1;
        }
#ifdef QPP_PROBE
        if (hipMemcpyFromSymbol(g.data(), HIP_SYMBOL(g_probe), g.size() * 8) != hipSuccess) return 1;
#endif
        if (c < 20) continue;  // warm-up
        ++n_ok;
        for (int ph = 0; ph < 10; ++ph) sum[ph] += g[ph] / 100.0;
        span += (g[kProbeEnd] - g[kProbeStart]) / 100.0;
    }
    printf("%s, wave 0, mean of %d calls: start to last mark %.2f us\n", enc ? "protect" : "unprotect", n_ok,
           span / n_ok);
    for (int ph = 0; ph < 10; ++ph) printf("  %-52s %6.2f us\n", g_names[ph], sum[ph] / n_ok);
    return 0;
}

int main(int argc, char **argv)
{
    const int calls = argc > 1 ? atoi(argv[1]) : 300;
    const int suite = argc > 2 ? atoi(argv[2]) : QPP_AES_128_GCM;
    g_names = suite == QPP_CHACHA20_POLY1305 ? kNamesChacha : kNames;
    qpp_keytab *kt = nullptr;
    qpp_session *s = nullptr;
    if (qpp_keytab_create(4, &kt) != QPP_OK || qpp_session_create(1 << 16, 64, &s) != QPP_OK) return 1;
    qpp_key_material km = {};
    km.slot = 0;
    km.suite = (uint8_t)suite;
    for (int i = 0; i < 12; ++i) km.iv[i] = (uint8_t)(i + 1);
    for (int i = 0; i < 32; ++i) km.key[i] = (uint8_t)(3 * i), km.hp[i] = (uint8_t)(5 * i + 1);
    if (qpp_session_set_keys(s, kt, &km, 1) != QPP_OK) return 1;
    std::vector<uint8_t> pkt;
    if (run(s, kt, true, calls, pkt) || run(s, kt, false, calls, pkt)) return 1;
    qpp_session_destroy(s);
    qpp_keytab_destroy(kt);
    return 0;
}
