// Phase-timing probe of the packet kernels: the engine built with -DQPP_PROBE,
// n x 1200 B AES-128-GCM (default 1 Mi, the bench workload), per-wave phase sums.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DQPP_PROBE -c -o /tmp/probe.o tools/probe.hip && \
//        hipcc --offload-arch=gfx950 -o tools/probe /tmp/probe.o build/obj/qpp_plan.o
// Run:   tools/probe [packets] [suite]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../aioquic_amd/csrc/qpp_engine.hip"

static void fill(uint8_t *p, size_t n, uint32_t seed)
{
    for (size_t i = 0; i < n; ++i) {
        seed = seed * 1664525u + 1013904223u;
        p[i] = (uint8_t)(seed >> 24);
    }
}

#ifdef QPP_PROBE
static int g_wpg = 16;  // waves per workgroup of the probed kernel
static bool g_chacha = false;
static void report(const char *what, const std::vector<unsigned long long> &pr)
{
    // phases of the persistent GCM kernel (qpp_engine.hip QPP_PROBE_AT marks)
    static const char *gcm_names[] = {"prologue (AES image, entry init, sync)", "item tail + grab", "table entry (acquire)",
                           "descriptor, pkt_begin, park", "AAD fold + counter cache", "step loop",
                           "closing GHASH multiply (global tables)", "finish: tail, tag, header, result",
                           "release", "exit"};
    static const char *chacha_names[] = {"-", "descriptor, header, pkt_begin", "key block, r powers, AAD",
                           "next step's DMA issue", "ChaCha20 block + Poly1305 (compute)",
                           "wait: step input DMA (+ last stores)", "xor via LDS (ds_read, xor, ds_write)",
                           "close, tag, HP, result", "stores (LDS reads, buffer stores)", "exit"};
    const char **names = g_chacha ? chacha_names : gcm_names;
    constexpr int NP = 10;
    int waves = 0;
    unsigned long long t0 = ~0ull, t1 = 0, items = 0;
    double sum[NP] = {}, mx[NP] = {};
    for (int w = 0; w < kProbeWaves; ++w) {
        const unsigned long long *g = &pr[(size_t)w * kProbeSlots];
        if (!g[kProbeStart]) continue;
        ++waves;
        t0 = std::min(t0, g[kProbeStart]);
        t1 = std::max(t1, g[kProbeEnd]);
        items += g[kProbeItems];
        for (int ph = 0; ph < NP; ++ph) {
            sum[ph] += g[ph] / 100.0;
            mx[ph] = std::max(mx[ph], g[ph] / 100.0);
        }
    }
    if (!waves) { printf("%s: no probe data\n", what); return; }
    printf("%s: waves %d, items %llu (%.1f per wave), span %.2f us\n", what, waves, items,
           (double)items / waves, (t1 - t0) / 100.0);
    double tot = 0;
    for (int ph = 0; ph < NP; ++ph) tot += sum[ph];
    for (int ph = 0; ph < NP; ++ph)
        printf("  %-40s per wave mean %9.2f us (%5.1f %%)  max %9.2f us  per item %7.3f us\n", names[ph],
               sum[ph] / waves, 100.0 * sum[ph] / tot, mx[ph], sum[ph] / (double)items);
    double e_min = 1e30, e_max = 0;
    for (int w = 0; w < kProbeWaves; ++w) {
        const unsigned long long *g = &pr[(size_t)w * kProbeSlots];
        if (!g[kProbeStart]) continue;
        e_min = std::min(e_min, (g[kProbeEnd] - t0) / 100.0);
        e_max = std::max(e_max, (g[kProbeEnd] - t0) / 100.0);
    }
    printf("  wave ends: first %.2f us, last %.2f us\n", e_min, e_max);
    // start and end times as quantiles over the waves (dispatch ramp, tail)
    std::vector<double> st, en;
    for (int w = 0; w < kProbeWaves; ++w) {
        const unsigned long long *g = &pr[(size_t)w * kProbeSlots];
        if (!g[kProbeStart]) continue;
        st.push_back((g[kProbeStart] - t0) / 100.0);
        en.push_back((g[kProbeEnd] - t0) / 100.0);
    }
    std::sort(st.begin(), st.end());
    std::sort(en.begin(), en.end());
    auto q = [](const std::vector<double> &v, double f) { return v[(size_t)(f * (v.size() - 1))]; };
    printf("  wave starts: q10 %.2f q50 %.2f q90 %.2f max %.2f us; ends: q10 %.2f q50 %.2f q90 %.2f us\n",
           q(st, 0.1), q(st, 0.5), q(st, 0.9), q(st, 1.0), q(en, 0.1), q(en, 0.5), q(en, 0.9));
    // per workgroup (16 waves): its last wave's end, and the spread inside it
    double g_first = 1e30, g_last = 0, spread = 0, spread_max = 0;
    int groups = 0;
    for (int b = 0; b < kProbeWaves / 16; ++b) {
        double lo = 1e30, hi = 0;
        for (int w = b * 16; w < b * 16 + 16; ++w) {
            const unsigned long long *g = &pr[(size_t)w * kProbeSlots];
            if (!g[kProbeStart]) continue;
            lo = std::min(lo, (g[kProbeEnd] - t0) / 100.0);
            hi = std::max(hi, (g[kProbeEnd] - t0) / 100.0);
        }
        if (hi == 0) continue;
        ++groups;
        g_first = std::min(g_first, hi);
        g_last = std::max(g_last, hi);
        spread += hi - lo;
        spread_max = std::max(spread_max, hi - lo);
    }
    printf("  workgroup ends: first %.2f us, last %.2f us; wave-end spread inside a workgroup mean %.2f max %.2f us\n",
           g_first, g_last, spread / groups, spread_max);
    // workgroup ends by XCD (workgroups are dealt round-robin to the 8 XCDs)
    {
        double xs[8] = {}, xmin[8], xmax[8] = {};
        int xn[8] = {};
        for (int x = 0; x < 8; ++x) xmin[x] = 1e30;
        for (int b = 0; b < kProbeWaves / g_wpg; ++b) {
            double hi = 0;
            for (int w = b * g_wpg; w < b * g_wpg + g_wpg; ++w) {
                const unsigned long long *g = &pr[(size_t)w * kProbeSlots];
                if (g[kProbeStart]) hi = std::max(hi, (g[kProbeEnd] - t0) / 100.0);
            }
            if (hi == 0) continue;
            const int x = b % 8;
            xs[x] += hi;
            xn[x]++;
            xmin[x] = std::min(xmin[x], hi);
            xmax[x] = std::max(xmax[x], hi);
        }
        printf("  workgroup ends by XCD (mean min max):");
        for (int x = 0; x < 8; ++x)
            if (xn[x]) printf(" [%d] %.0f %.0f %.0f", x, xs[x] / xn[x], xmin[x], xmax[x]);
        printf("\n");
    }
}
#endif

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const int suite = argc > 2 ? atoi(argv[2]) : 0;
    if (n == 0) return 2;
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
    const int wg = suite == QPP_CHACHA20_POLY1305 ? kChachaWG : kGcmWG;
#ifdef QPP_PROBE
    g_wpg = wg / 64;
    g_chacha = suite == QPP_CHACHA20_POLY1305;
#endif
#ifdef QPP_PROBE
    std::vector<unsigned long long> pr((size_t)kProbeWaves * kProbeSlots);
#endif
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
#ifdef QPP_PROBE
        std::fill(pr.begin(), pr.end(), 0ull);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_probe), pr.data(), pr.size() * 8, 0, hipMemcpyHostToDevice);
#endif
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
        report(enc ? "protect" : "unprotect", pr);
#endif
    }
    return 0;
}
