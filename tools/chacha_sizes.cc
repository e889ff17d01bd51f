// Packet-size sweep of one suite's kernels through the C ABI: n packets of
// header 11 B + payload P, protect and unprotect timed with events (median of
// 20 after 3 warm-ups).  Run under rocprofv3 --pmc SQ_INSTS_VALU to split a
// kernel's instructions into a per-packet part and a per-64-byte-unit part.
//   g++ -O2 -std=c++17 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/chacha_sizes.cc \
//       -L aioquic_amd -lquicpp -L /opt/rocm/lib -lamdhip64 -o tools/chacha_sizes
//   LD_LIBRARY_PATH=aioquic_amd tools/chacha_sizes [suite=2] [packets=65536] [payloads=53,245,501,757,1173]
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "quic_pp.h"

static void fill(uint8_t *p, size_t n, uint32_t seed)
{
    for (size_t i = 0; i < n; ++i) {
        seed = seed * 1664525u + 1013904223u;
        p[i] = (uint8_t)(seed >> 24);
    }
}

int main(int argc, char **argv)
{
    const int suite = argc > 1 ? atoi(argv[1]) : QPP_CHACHA20_POLY1305;
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536u;
    std::vector<int> sizes = {53, 245, 501, 757, 1173};
    if (argc > 3) {
        sizes.clear();
        std::string s = argv[3];
        size_t p = 0;
        while (p < s.size()) {
            size_t q = s.find(',', p);
            if (q == std::string::npos) q = s.size();
            sizes.push_back(atoi(s.substr(p, q - p).c_str()));
            p = q + 1;
        }
    }
    qpp_keytab *kt = nullptr;
    if (qpp_keytab_create(4, &kt) != QPP_OK) { printf("keytab failed\n"); return 1; }
    qpp_key_material km = {};
    km.slot = 0;
    km.suite = (uint8_t)suite;
    fill(km.iv, 12, 1);
    fill(km.key, 32, 2);
    fill(km.hp, 32, 3);
    if (qpp_keytab_set(kt, &km, 1, nullptr) != QPP_OK) { printf("set failed\n"); return 1; }
    const int hdr = 11, slot = 1200;
    std::vector<uint8_t> h_in((size_t)n * slot);
    fill(h_in.data(), h_in.size(), 4);
    uint8_t *d_in, *d_ct, *d_pt;
    qpp_desc *d_pd, *d_ud;
    qpp_result *d_res;
    if (hipMalloc(&d_in, h_in.size()) || hipMalloc(&d_ct, h_in.size()) || hipMalloc(&d_pt, h_in.size()) ||
        hipMalloc(&d_pd, n * sizeof(qpp_desc)) || hipMalloc(&d_ud, n * sizeof(qpp_desc)) ||
        hipMalloc(&d_res, n * sizeof(qpp_result))) {
        printf("hipMalloc failed\n");
        return 1;
    }
    for (uint32_t i = 0; i < n; ++i) {
        h_in[(size_t)i * slot] = 0x41;  // short header, 2-byte packet number
        h_in[(size_t)i * slot + hdr - 2] = (uint8_t)(i >> 8);
        h_in[(size_t)i * slot + hdr - 1] = (uint8_t)i;
    }
    (void)hipMemcpy(d_in, h_in.data(), h_in.size(), hipMemcpyHostToDevice);
    std::vector<qpp_desc> pd(n), ud(n);
    std::vector<qpp_result> res(n);
    hipEvent_t ev[3];
    for (auto &e : ev) (void)hipEventCreate(&e);
    for (int payload : sizes) {
        if (payload < 20 || payload + hdr + 16 > slot) continue;
        for (uint32_t i = 0; i < n; ++i) {
            pd[i] = qpp_desc{(uint64_t)i * slot, (uint64_t)i * slot, (uint32_t)payload, (uint16_t)hdr, 0, i, 0, 0};
            ud[i] = qpp_desc{(uint64_t)i * slot, (uint64_t)i * slot, (uint32_t)(hdr + payload + 16),
                             (uint16_t)(hdr - 2), 0, i, 0, 0};
        }
        (void)hipMemcpy(d_pd, pd.data(), n * sizeof(qpp_desc), hipMemcpyHostToDevice);
        (void)hipMemcpy(d_ud, ud.data(), n * sizeof(qpp_desc), hipMemcpyHostToDevice);
        std::vector<float> tp, tu;
        for (int k = -3; k < 20; ++k) {
            (void)hipEventRecord(ev[0], nullptr);
            int rc = qpp_protect(kt, d_pd, n, d_in, d_ct, d_res, nullptr);
            (void)hipEventRecord(ev[1], nullptr);
            rc |= qpp_unprotect(kt, d_ud, n, d_ct, d_pt, d_res, nullptr);
            (void)hipEventRecord(ev[2], nullptr);
            (void)hipEventSynchronize(ev[2]);
            if (rc != QPP_OK) { printf("launch rc %d\n", rc); return 1; }
            float a = 0, b = 0;
            (void)hipEventElapsedTime(&a, ev[0], ev[1]);
            (void)hipEventElapsedTime(&b, ev[1], ev[2]);
            if (k >= 0) { tp.push_back(a); tu.push_back(b); }
        }
        std::sort(tp.begin(), tp.end());
        std::sort(tu.begin(), tu.end());
        (void)hipMemcpy(res.data(), d_res, n * sizeof(qpp_result), hipMemcpyDeviceToHost);
        uint32_t bad = 0;
        for (auto &r : res) bad += r.status != QPP_S_OK;
        const int units = (payload + 63) / 64 + 1;
        printf("payload %4d B (%2d units): protect %8.1f us  unprotect %8.1f us  (%.3f us per packet-unit)  bad %u\n",
               payload, units, tp[10] * 1e3, tu[10] * 1e3, tp[10] * 1e3 / ((double)n * units) * 1e3, bad);
        if (bad) return 1;
    }
    return 0;
}
