// Building-block throughput on one MI355X, with the clock the chip actually
// holds (s_memtime shader cycles over s_memrealtime 100 MHz ticks):
//   valu     8 independent chains of v_bitop3 (the VALU issue ceiling)
//   aes      T-table AES-128 (10 rounds), the engine's LDS image
//   ctr      counter-cached AES-128 CTR block (rounds 3..10 + 5 lookups)
//   ghash    one 4-bit-window GHASH multiply (32 ds_read_b128)
//   ctr+gh   the engine's step: one CTR block + one GHASH multiply
// CH = independent chains per lane.  Prints CU-cycles per 16-byte block at the
// measured clock and the fraction of the LDS-array model floor reached.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mb_aes tools/mb_aes.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <type_traits>
#include <vector>

#include "../aioquic_amd/csrc/qpp_device.h"

using namespace qpp;

namespace qpp { __constant__ AesTables c_aes = kAesTables; }

__device__ unsigned long long g_clk[4096 * 4];

template <int NT>
__device__ void fill_te(uint8_t *te)
{
    for (int i = threadIdx.x; i < 256 * 16; i += NT) {
        const int x = i >> 4, part = i & 15;
        const uint32_t v0 = c_aes.te0[x];
        const uint32_t v = part < 8 ? v0 : rotl(v0, 8);
        *(u32x4 *)(te + x * 256 + part * 16) = u32x4{v, v, v, v};
    }
}

struct __attribute__((aligned(16))) Smem {
    uint8_t gt[kGhashTabBytes];
    uint8_t te[kTeBytes];
};
// AES-only variants: just the 64 KiB image, so two 1024-thread workgroups
// (8 waves per SIMD) fit on a CU
struct __attribute__((aligned(16))) SmemTe {
    uint8_t te[kTeBytes];
    uint8_t gt[16];
};

enum { M_VALU = 0, M_AES = 1, M_CTR = 2, M_GH = 3, M_CTRGH = 4 };

template <int WG, int MODE, int CH, bool SMALL = false>
__global__ __launch_bounds__(WG) void k_mb(const uint32_t *rk_g, const uint8_t *gt_g, int steps,
                                           uint32_t *out)
{
    __shared__ typename std::conditional<SMALL, SmemTe, Smem>::type sm;
    if (MODE != M_VALU) {
        fill_te<WG>(sm.te);
        if (!SMALL) for (int i = threadIdx.x; i < kGhashTabBytes / 16; i += WG)
            ((u32x4 *)sm.gt)[i] = ((const u32x4 *)gt_g)[i];
    }
    __syncthreads();
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_g[i]);
    const LdsTe T{sm.te, (uint32_t)(threadIdx.x & 31) * 4};
    u32x4 acc[CH];
    CtrCache cc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        acc[c] = u32x4{threadIdx.x, blockIdx.x, (uint32_t)c, 0};
        if (MODE == M_CTR || MODE == M_CTRGH)
            cc[c] = ctr_cache(u32x4{blockIdx.x, threadIdx.x, 7u + c, 0}, rk, T);
    }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < steps; ++k) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (MODE == M_VALU) {
                uint32_t a = acc[c].x, b = acc[c].y, d = acc[c].z, e = acc[c].w;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    a = __builtin_amdgcn_bitop3_b32(a, b, d, 0x96);
                    b = __builtin_amdgcn_bitop3_b32(b, d, e, 0xe8);
                    d = __builtin_amdgcn_bitop3_b32(d, e, a, 0x6a);
                    e = __builtin_amdgcn_bitop3_b32(e, a, b, 0x1e);
                }
                acc[c] = u32x4{a, b, d, e};
            } else if (MODE == M_AES) {
                acc[c] ^= aes_encrypt<10>(u32x4{acc[c].x, acc[c].y, (uint32_t)k, (uint32_t)c}, rk, T);
            } else if (MODE == M_CTR) {
                acc[c] ^= aes_ctr<10>(cc[c], (uint32_t)(k & 255) ^ (acc[c].x & 1), rk, T);
            } else if (MODE == M_GH) {
                acc[c] = ghash_mul(acc[c] ^ u32x4{(uint32_t)k, 0, 0, 0}, sm.gt, 3 * 8192);
            } else {
                const u32x4 ks = aes_ctr<10>(cc[c], (uint32_t)(k & 255) ^ (acc[c].x & 1), rk, T);
                acc[c] = ghash_mul(acc[c] ^ ks, sm.gt, 3 * 8192);
            }
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 4096) {
        g_clk[blockIdx.x * 4 + 0] = c0;
        g_clk[blockIdx.x * 4 + 1] = c1;
        g_clk[blockIdx.x * 4 + 2] = t0;
        g_clk[blockIdx.x * 4 + 3] = t1;
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) r ^= acc[c].x ^ acc[c].y ^ acc[c].z ^ acc[c].w;
    out[blockIdx.x * WG + threadIdx.x] = r;
}

// LDS-array cycles per block per wave-instruction model (MI355X_MICROARCH.md sec. LDS):
// ds_read_b32 = 2 cycles, ds_read_b128 = 4 cycles per 64 lanes
static double lds_model(int mode)
{
    switch (mode) {
    case M_AES: return (160.0 * 2) / 64;
    case M_CTR: return (133.0 * 2) / 64;
    case M_GH: return (32.0 * 4) / 64;
    case M_CTRGH: return (133.0 * 2 + 32.0 * 4) / 64;
    default: return 0;
    }
}

template <int WG, int MODE, int CH, bool SMALL = false>
static void run(const char *name, const uint32_t *rk, const uint8_t *gt, uint32_t *out)
{
    const int blocks = 2048 * (1024 / WG) / CH * (MODE == M_VALU ? 1 : 1);
    const int steps = MODE == M_VALU ? 256 : 64;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL((k_mb<WG, MODE, CH, SMALL>), dim3(blocks), dim3(WG), 0, 0, rk, gt, steps, out);
    const int reps = 5;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_mb<WG, MODE, CH, SMALL>), dim3(blocks), dim3(WG), 0, 0, rk, gt, steps, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    std::vector<unsigned long long> clk(4096 * 4);
    (void)hipMemcpyFromSymbol(clk.data(), HIP_SYMBOL(g_clk), clk.size() * 8, 0, hipMemcpyDeviceToHost);
    double cyc = 0, tick = 0;
    const int nb = blocks < 4096 ? blocks : 4096;
    for (int i = 0; i < nb; ++i) {
        cyc += (double)(clk[i * 4 + 1] - clk[i * 4 + 0]);
        tick += (double)(clk[i * 4 + 3] - clk[i * 4 + 2]);
    }
    const double mhz = cyc / (tick / 100.0);
    const double units = (double)blocks * WG * steps * CH;  // lane-blocks (or lane-iterations)
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / units;
    if (MODE == M_VALU) {
        // 64 bitop3 per lane-iteration: lane-ops per CU-cycle
        printf("%-8s WG %4d CH %d  %8.3f ms  clock %5.0f MHz  %6.1f lane-ops/CU-cycle (peak 128)\n", name,
               WG, CH, ms, mhz, 64.0 / cu_cyc);
    } else {
        const double f = lds_model(MODE);
        printf("%-8s WG %4d CH %d%s  %8.3f ms  clock %5.0f MHz  %6.2f CU-cycles/block  LDS floor %5.2f  frac %.2f\n",
               name, WG, CH, SMALL ? " 2WG" : "", ms, mhz, cu_cyc, f, f / cu_cyc);
    }
    fflush(stdout);
}

int main()
{
    uint32_t *rk, *out;
    uint8_t *gt;
    (void)hipMalloc(&rk, 44 * 4);
    (void)hipMalloc(&gt, kGhashTabBytes);
    (void)hipMalloc(&out, (size_t)2048 * 1024 * 4 * 4);
    std::vector<uint32_t> hrk(44);
    for (int i = 0; i < 44; ++i) hrk[i] = 0x9e3779b9u * (i + 1);
    (void)hipMemcpy(rk, hrk.data(), 44 * 4, hipMemcpyHostToDevice);
    std::vector<uint8_t> hgt(kGhashTabBytes);
    for (int i = 0; i < kGhashTabBytes; ++i) hgt[i] = (uint8_t)(i * 131 + 7);
    (void)hipMemcpy(gt, hgt.data(), kGhashTabBytes, hipMemcpyHostToDevice);
    run<256, M_VALU, 1>("valu", rk, gt, out);
    run<256, M_VALU, 2>("valu", rk, gt, out);
    run<1024, M_VALU, 1>("valu", rk, gt, out);
    run<1024, M_AES, 1>("aes", rk, gt, out);
    run<1024, M_AES, 2>("aes", rk, gt, out);
    run<512, M_AES, 2>("aes", rk, gt, out);
    run<1024, M_AES, 1, true>("aes", rk, gt, out);
    run<1024, M_AES, 2, true>("aes", rk, gt, out);
    run<1024, M_CTR, 1>("ctr", rk, gt, out);
    run<1024, M_CTR, 1, true>("ctr", rk, gt, out);
    run<1024, M_CTR, 2, true>("ctr", rk, gt, out);
    run<1024, M_CTR, 2>("ctr", rk, gt, out);
    run<512, M_CTR, 2>("ctr", rk, gt, out);
    run<512, M_CTR, 4>("ctr", rk, gt, out);
    run<1024, M_GH, 1>("ghash", rk, gt, out);
    run<1024, M_GH, 2>("ghash", rk, gt, out);
    run<1024, M_CTRGH, 1>("ctr+gh", rk, gt, out);
    run<1024, M_CTRGH, 2>("ctr+gh", rk, gt, out);
    run<512, M_CTRGH, 2>("ctr+gh", rk, gt, out);
    run<768, M_CTRGH, 1>("ctr+gh", rk, gt, out);
    return 0;
}
