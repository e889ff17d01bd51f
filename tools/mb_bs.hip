// Bitsliced AES throughput on one MI355X (tools/bitslice/qpp_bitslice.h): each lane runs
// 32 blocks per AES call.  MODE 0: AES only; MODE 1: plus the transposes in
// and out (slot words <-> planes).  Prints CU-cycles per 16-byte block at the
// measured clock (s_memtime / s_memrealtime).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mb_bs tools/mb_bs.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <vector>

#include "bitslice/qpp_bitslice.h"

__device__ unsigned long long g_clk[8192 * 4];
#ifndef QPP_MB_WAVES
#define QPP_MB_WAVES
#endif

template <int NR, int MODE, int WG>
__global__ __launch_bounds__(WG) QPP_MB_WAVES void k_bs(const uint32_t *__restrict__ km, int steps, uint32_t *__restrict__ out)
{
    uint32_t st[128];
#pragma unroll
    for (int j = 0; j < 128; ++j) st[j] = (threadIdx.x * 0x9e3779b9u) ^ (j * 0x85ebca6bu) ^ blockIdx.x;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < steps; ++k) {
        if (MODE == 2) qpp::bs::encrypt_gen<NR>(st, km);
        else qpp::bs::encrypt<NR>(st, km);
        if (MODE == 1) {
            uint32_t blk[32][4];
            qpp::bs::from_planes(st, blk);
#pragma unroll
            for (int s = 0; s < 32; ++s) blk[s][3] ^= (uint32_t)k;
            qpp::bs::to_planes(blk, st);
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
        g_clk[blockIdx.x * 4 + 0] = c0;
        g_clk[blockIdx.x * 4 + 1] = c1;
        g_clk[blockIdx.x * 4 + 2] = t0;
        g_clk[blockIdx.x * 4 + 3] = t1;
    }
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 128; ++j) r ^= st[j];
    out[blockIdx.x * WG + threadIdx.x] = r;
}

template <int NR, int MODE, int WG>
static void run(const char *name, const uint32_t *km, uint32_t *out, int blocks)
{
    const int steps = 8;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((k_bs<NR, MODE, WG>), dim3(blocks), dim3(WG), 0, 0, km, steps, out);
    const int reps = 5;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_bs<NR, MODE, WG>), dim3(blocks), dim3(WG), 0, 0, km, steps, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    std::vector<unsigned long long> clk(8192 * 4);
    (void)hipMemcpyFromSymbol(clk.data(), HIP_SYMBOL(g_clk), clk.size() * 8, 0, hipMemcpyDeviceToHost);
    double cyc = 0, tick = 0;
    const int nb = blocks < 8192 ? blocks : 8192;
    for (int i = 0; i < nb; ++i) {
        cyc += (double)(clk[i * 4 + 1] - clk[i * 4 + 0]);
        tick += (double)(clk[i * 4 + 3] - clk[i * 4 + 2]);
    }
    const double mhz = cyc / (tick / 100.0);
    const double aes_blocks = (double)blocks * WG * steps * 32;
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / aes_blocks;
    printf("%-12s NR %2d WG %4d blocks %6d  %8.3f ms  clock %5.0f MHz  %6.3f CU-cycles/block  %7.1f VALU-op-eq/block\n",
           name, NR, WG, blocks, ms, mhz, cu_cyc, cu_cyc * 128);
    fflush(stdout);
}

// FIPS-197 App. C.1 through the generated bitop3 path on the device: every
// lane's 32 slots hold the same plaintext; returns slot 0 of lane 0.
__global__ void k_kat(const uint32_t *__restrict__ kt, const uint32_t *__restrict__ pt, uint32_t *__restrict__ out)
{
    uint32_t blk[32][4], st[128];
    for (int s = 0; s < 32; ++s)
        for (int k = 0; k < 4; ++k) blk[s][k] = pt[k];
    qpp::bs::to_planes(blk, st);
    qpp::bs::encrypt_gen<10>(st, kt);
    qpp::bs::from_planes(st, blk);
    if (threadIdx.x == 0)
        for (int s = 0; s < 32; ++s)
            for (int k = 0; k < 4; ++k) out[4 * s + k] = blk[s][k];
}

static void kat()
{
    // FIPS-197 key expansion of 000102..0f (host, via the same header's key_table)
    uint8_t sb[256];
    for (int x = 0; x < 256; ++x) {
        auto gm = [](uint8_t a, uint8_t b) { uint8_t r = 0; for (int i = 0; i < 8; ++i) { if (b & 1) r ^= a; a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); b >>= 1; } return r; };
        uint8_t inv = 1, b = (uint8_t)x;
        for (int e = 254; e; e >>= 1) { if (e & 1) inv = gm(inv, b); b = gm(b, b); }
        uint8_t y = inv;
        for (int i = 1; i <= 4; ++i) y ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
        sb[x] = y ^ 0x63;
    }
    uint32_t rk[44];
    for (int i = 0; i < 4; ++i) rk[i] = (uint32_t)(4 * i) | (uint32_t)(4 * i + 1) << 8 | (uint32_t)(4 * i + 2) << 16 | (uint32_t)(4 * i + 3) << 24;
    uint8_t rcon = 1;
    for (int i = 4; i < 44; ++i) {
        uint32_t t = rk[i - 1];
        if (i % 4 == 0) {
            t = (t >> 8) | (t << 24);
            t = (uint32_t)sb[t & 255] | (uint32_t)sb[(t >> 8) & 255] << 8 | (uint32_t)sb[(t >> 16) & 255] << 16 | (uint32_t)sb[t >> 24] << 24;
            t ^= rcon;
            rcon = (uint8_t)((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0));
        }
        rk[i] = rk[i - 4] ^ t;
    }
    std::vector<uint32_t> kt(qpp::bs::bs_key_words(10));
    qpp::bs::key_table(rk, 10, kt.data());
    const uint32_t pt[4] = {0x33221100u, 0x77665544u, 0xbbaa9988u, 0xffeeddccu};
    uint32_t *d_kt, *d_pt, *d_out;
    (void)hipMalloc(&d_kt, kt.size() * 4);
    (void)hipMalloc(&d_pt, 16);
    (void)hipMalloc(&d_out, 512);
    (void)hipMemcpy(d_kt, kt.data(), kt.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_pt, pt, 16, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_kat, dim3(1), dim3(64), 0, 0, d_kt, d_pt, d_out);
    uint32_t out[128];
    (void)hipMemcpy(out, d_out, 512, hipMemcpyDeviceToHost);
    const uint32_t want[4] = {0xd8e0c469u, 0x30047b6au, 0x80b7cdd8u, 0x5ac5b470u};
    bool ok = true;
    for (int s = 0; s < 32; ++s)
        for (int k = 0; k < 4; ++k) ok = ok && out[4 * s + k] == want[k];
    printf("FIPS-197 C.1 on the device (generated bitop3 columns): %s (%08x %08x %08x %08x)\n", ok ? "OK" : "MISMATCH",
           out[0], out[1], out[2], out[3]);
}

int main()
{
    kat();
    uint32_t *km, *out;
    (void)hipMalloc(&km, 15 * 128 * 4);
    (void)hipMalloc(&out, (size_t)8192 * 1024 * 4);
    std::vector<uint32_t> h(15 * 128);
    for (int i = 0; i < 15 * 128; ++i) h[i] = ((i * 2654435761u) >> 7) & 1 ? ~0u : 0u;
    (void)hipMemcpy(km, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    uint32_t *kt;
    (void)hipMalloc(&kt, qpp::bs::bs_key_words(14) * 4);
    (void)hipMemset(kt, 0x5a, qpp::bs::bs_key_words(14) * 4);
    run<10, 2, 256>("aes-gen", kt, out, 2048);
    run<10, 2, 256>("aes-gen", kt, out, 1024);
    run<10, 2, 512>("aes-gen", kt, out, 1024);
    run<14, 2, 256>("aes-gen", kt, out, 2048);
    return 0;
}
