// Phase-timing probe of the packet kernels: the engine built with -DQPP_PROBE,
// 64Ki x 1200 B AES-128-GCM (the bench workload), per-wave timestamps.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DQPP_PROBE \
//            -o tools/probe tools/probe.hip
// Run:   tools/probe [packets] [suite]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../aioquic_amd/csrc/qpp_engine.hip"

static void fill(uint8_t *p, size_t n, uint32_t seed)
{
    for (size_t i = 0; i < n; ++i) {
        seed = seed * 1664525u + 1013904223u;
        p[i] = (uint8_t)(seed >> 24);
    }
}

static void report(const char *what, const std::vector<unsigned long long> &pr, int waves)
{
    const char *names[] = {"  desc load", "  load_te", "  hdr prefetch", "  sync 1", "  atomics + sync 2", "prologue (te, desc, hdr, 2 syncs)", "slot + GHASH table", "pkt_begin",
                           "AAD fold + ctr cache", "step loop", "finish + result", "final sync"};
    const int from[] = {0, 10, 11, 12, 13, 0, 7, 1, 2, 3, 4, 5}, to[] = {10, 11, 12, 13, 7, 7, 1, 2, 3, 4, 5, 6};
    constexpr int NP = 12;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int w = 0; w < waves; ++w) {
        t0 = std::min(t0, pr[w * 16 + 0]);
        t1 = std::max(t1, pr[w * 16 + 6]);
    }
    printf("%s: waves %d, span %.2f us\n", what, waves, (t1 - t0) / 100.0);
    for (int ph = 0; ph < NP; ++ph) {
        double sum = 0, mx = 0;
        for (int w = 0; w < waves; ++w) {
            const double d = (double)(pr[w * 16 + to[ph]] - pr[w * 16 + from[ph]]) / 100.0;
            sum += d;
            mx = std::max(mx, d);
        }
        printf("  %-34s mean %8.2f us  max %8.2f us\n", names[ph], sum / waves, mx);
    }
    // start / end spread
    double s_max = 0, e_min = 1e30;
    for (int w = 0; w < waves; ++w) {
        s_max = std::max(s_max, (pr[w * 16 + 0] - t0) / 100.0);
        e_min = std::min(e_min, (pr[w * 16 + 6] - t0) / 100.0);
    }
    printf("  last wave start %.2f us, first wave end %.2f us\n", s_max, e_min);
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536;
    const int suite = argc > 2 ? atoi(argv[2]) : 0;
#ifdef QPP_PROBE
    if (n == 0 || n > kProbeWaves * 16) {  // 16 packets per wave are recorded
        printf("probe: n must be 1..%u\n", kProbeWaves * 16);
        return 2;
    }
#else
    if (n == 0) return 2;
#endif
    // header length (argv[4], default 11): 16 puts every ciphertext block on a 16-byte boundary
    const int hdr = argc > 4 ? atoi(argv[4]) : 11, slot = 1200, payload = slot - 16 - hdr;
    qpp_keytab *kt = nullptr;
    if (qpp_keytab_create(4, &kt) != QPP_OK) { printf("keytab failed\n"); return 1; }
    qpp_key_material km = {};
    km.slot = 0;
    km.suite = (uint8_t)suite;
    fill(km.iv, 12, 1);
    fill(km.key, 32, 2);
    fill(km.hp, 32, 3);
    if (qpp_keytab_set(kt, &km, 1, nullptr) != QPP_OK) { printf("set failed\n"); return 1; }

    std::vector<uint8_t> h_in((size_t)n * slot);
    fill(h_in.data(), h_in.size(), 4);
    std::vector<qpp_desc> pd(n), ud(n);
    for (uint32_t i = 0; i < n; ++i) {
        h_in[(size_t)i * slot] = 0x41;  // short header, 2-byte packet number = i
        h_in[(size_t)i * slot + hdr - 2] = (uint8_t)(i >> 8);
        h_in[(size_t)i * slot + hdr - 1] = (uint8_t)i;
        pd[i] = qpp_desc{(uint64_t)i * slot, (uint64_t)i * slot, (uint32_t)payload, (uint16_t)hdr, 0,
                         i, 0, 0};
        ud[i] = qpp_desc{(uint64_t)i * slot, (uint64_t)i * slot, (uint32_t)slot, (uint16_t)(hdr - 2),
                         0, i, 0, 0};
    }
    uint8_t *d_in, *d_ct, *d_pt;
    qpp_desc *d_pd, *d_ud;
    qpp_result *d_res;
    (void)hipMalloc(&d_in, h_in.size());
    (void)hipMalloc(&d_ct, h_in.size());
    (void)hipMalloc(&d_pt, h_in.size());
    (void)hipMalloc(&d_pd, n * sizeof(qpp_desc));
    (void)hipMalloc(&d_ud, n * sizeof(qpp_desc));
    (void)hipMalloc(&d_res, n * sizeof(qpp_result));
    (void)hipMemcpy(d_in, h_in.data(), h_in.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_pd, pd.data(), n * sizeof(qpp_desc), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ud, ud.data(), n * sizeof(qpp_desc), hipMemcpyHostToDevice);

    if (argc > 3 && strcmp(argv[3], "bench") == 0) {
        // bench.py's step: protect then unprotect, alternating, event-timed
        const int steps = 30;
        hipEvent_t ev[3];
        for (auto &e : ev) (void)hipEventCreate(&e);
        double tp = 0, tu = 0;
        for (int k = -5; k < steps; ++k) {
            (void)hipEventRecord(ev[0], nullptr);
            (void)qpp_protect(kt, d_pd, n, d_in, d_ct, d_res, nullptr);
            (void)hipEventRecord(ev[1], nullptr);
            (void)qpp_unprotect(kt, d_ud, n, d_ct, d_pt, d_res, nullptr);
            (void)hipEventRecord(ev[2], nullptr);
            (void)hipEventSynchronize(ev[2]);
            float a = 0, b = 0;
            (void)hipEventElapsedTime(&a, ev[0], ev[1]);
            (void)hipEventElapsedTime(&b, ev[1], ev[2]);
            if (k >= 0) { tp += a; tu += b; }
        }
        tp /= steps;
        tu /= steps;
        printf("bench: protect %.1f us unprotect %.1f us -> %.1f GiB/s\n", tp * 1e3, tu * 1e3,
               (double)n * 1200 / ((tp + tu) * 1e-3) / (1u << 30));
        return 0;
    }
    const int wg = suite == QPP_CHACHA20_POLY1305 ? wg_choice("QPP_WG_CHACHA_ENC", kChachaWGEnc, true)
                                                  : wg_choice("QPP_WG_GCM", kGcmWG, false);
    const int waves = (int)(((n + wg / 4 - 1) / (wg / 4)) * (wg / 64));
    std::vector<unsigned long long> pr((size_t)waves * 16);
    // warm up in bench.py's order (protect, unprotect alternating)
    for (int rep = 0; rep < 3; ++rep) {
        int rc = qpp_protect(kt, d_pd, n, d_in, d_ct, d_res, nullptr);
        rc |= qpp_unprotect(kt, d_ud, n, d_ct, d_pt, d_res, nullptr);
        if (rc != QPP_OK) { printf("launch rc %d\n", rc); return 1; }
    }
    for (int enc = 1; enc >= 0; --enc) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipEventRecord(a, nullptr);
        if (enc) (void)qpp_protect(kt, d_pd, n, d_in, d_ct, d_res, nullptr);
        else (void)qpp_unprotect(kt, d_ud, n, d_ct, d_pt, d_res, nullptr);
        (void)hipEventRecord(b, nullptr);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
#ifdef QPP_PROBE
        (void)hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(g_probe), pr.size() * 8, 0,
                                  hipMemcpyDeviceToHost);
#endif
        std::vector<qpp_result> res(n);
        (void)hipMemcpy(res.data(), d_res, n * sizeof(qpp_result), hipMemcpyDeviceToHost);
        uint32_t bad = 0;
        uint32_t hist[8] = {};
        for (auto &r : res) {
            bad += r.status != QPP_S_OK;
            hist[r.status & 7]++;
        }
        printf("status histogram: ok %u length %u decrypt %u key_phase %u no_key %u\n", hist[0],
               hist[1], hist[2], hist[3], hist[4]);
        if (!enc) {
            // round trip: plaintext bytes that differ from the input, per region
            std::vector<uint8_t> pt(h_in.size());
            (void)hipMemcpy(pt.data(), d_pt, pt.size(), hipMemcpyDeviceToHost);
            for (int i = 0; i < 2; ++i) {
                int bh = 0, bp = 0, first = -1;
                for (int j = 0; j < hdr + payload; ++j) {
                    const bool diff = pt[(size_t)i * slot + j] != h_in[(size_t)i * slot + j];
                    if (diff && first < 0) first = j;
                    (j < hdr ? bh : bp) += diff;
                }
                printf("  pkt %d: header diffs %d payload diffs %d first %d\n", i, bh, bp, first);
            }
        }
        for (int i = 0; i < 3; ++i)
            printf("  res[%d] pn %llu status %u hdr_len %u out_len %u\n", i,
                   (unsigned long long)res[i].pn, res[i].status, res[i].hdr_len, res[i].out_len);
        printf("%s: %.1f us (event), WG %d, bad %u\n", enc ? "protect" : "unprotect", ms * 1e3, wg, bad);
#ifdef QPP_PROBE
        report(enc ? "protect" : "unprotect", pr, waves);
#endif
    }
    return 0;
}
