// Quad-bitsliced AES-CTR (aioquic_amd/csrc/qpp_bsq.h) against the T-table form,
// alone and mixed into the GCM step loop's LDS work (two counter blocks and
// two 5-bit GHASH multiplies per lane-step, as gcm_packet<BPL=2>):
//   check    bsq_ctr2 == aes_ctr2 on every lane (random nonces, counters)
//   ctr      counter blocks only: T-table / bitsliced
//   step P   the step: every P-th step of a wave bitsliced (0 = never),
//            phase offset by the wave index so a CU always runs a mix
// Prints CU-cycles per 16-byte block at the clock the chip holds.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mb_bsq tools/mb_bsq.hip
// Run with counters: gpurun -- bash tools/pmc_bsq.sh <tag>  (profiles/r4a_bsq_mix.txt)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "bitslice/qpp_bsq.h"

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

constexpr int kNR = 10;
// dynamic LDS so that one 1024-thread workgroup fills a CU (16 waves, as k_gcm)
constexpr int kDyn = 48 * 1024;
constexpr int kKp = bsq::key_plane_bytes(14);

struct __attribute__((aligned(16))) Smem {
    uint8_t gh[kGh5Bytes];
    uint8_t kp[kKp];
    uint8_t te[kTeBytes];
};

template <int NT>
__device__ void fill_common(Smem &sm, const uint8_t *gt_g, const uint8_t *kp_g)
{
    fill_te<NT>(sm.te);
    for (int i = threadIdx.x; i < kGh5Bytes / 16; i += NT) ((u32x4 *)sm.gh)[i] = ((const u32x4 *)gt_g)[i];
    for (int i = threadIdx.x; i < kKp / 16; i += NT) ((u32x4 *)sm.kp)[i] = ((const u32x4 *)kp_g)[i];
}

__global__ __launch_bounds__(1024) void k_check(const uint32_t *rk_g, const uint8_t *gt_g, const uint8_t *kp_g,
                                                uint32_t *bad)
{
    __shared__ Smem sm;
    fill_common<1024>(sm, gt_g, kp_g);
    __syncthreads();
    uint32_t rk[44];
    for (int i = 0; i < 44; ++i) rk[i] = rk_g[i];
    const LdsTe T{sm.te, (uint32_t)(threadIdx.x & 31) * 4};
    const uint32_t q = (blockIdx.x * 1024 + threadIdx.x) >> 2, sub = threadIdx.x & 3;
    const CtrCache cc = ctr_cache(u32x4{q * 0x9e3779b9u, q * 977u + 5, 0x1234567u ^ (q * 31u), 0}, rk, T);
    for (int it = 0; it < 4; ++it) {
        const uint32_t cb0 = 1 + ((q * 7 + sub * 13 + it * 29) % 250), cb1 = 1 + ((q * 11 + sub * 3 + it * 71) % 250);
        u32x4 a0, a1, b0, b1;
        aes_ctr2<kNR>(cc, cb0, cb1, rk, T, a0, a1);
        bsq_ctr2<kNR>(cc, cb0, cb1, rk, T, sm.kp, sub, b0, b1);
        u32x4 c0, c1, c2, c3;
        bsq_ctr4<kNR>(cc, cb1, cb0, cb0, cb1, rk, T, sm.kp, sub, c0, c1, c2, c3);
        const u32x4 e0 = c0 ^ a1, e1 = c1 ^ a0, e2 = c2 ^ a0, e3 = c3 ^ a1;
        if ((e0.x | e0.y | e0.z | e0.w | e1.x | e1.y | e1.z | e1.w | e2.x | e2.y | e2.z | e2.w | e3.x | e3.y | e3.z |
             e3.w) != 0)
            atomicAdd(bad, 1u);
        const u32x4 d0 = a0 ^ b0, d1 = a1 ^ b1;
        if ((d0.x | d0.y | d0.z | d0.w | d1.x | d1.y | d1.z | d1.w) != 0) atomicAdd(bad, 1u);
        if (blockIdx.x == 0 && threadIdx.x < 4 && it == 0)
            printf("lane %u cb %u %u  ttab %08x %08x %08x %08x  bsq %08x %08x %08x %08x\n", threadIdx.x, cb0, cb1,
                   a0.x, a0.y, a0.z, a0.w, b0.x, b0.y, b0.z, b0.w);
    }
}

enum { M_CTR = 0, M_STEP = 1, M_CTR4 = 2 };

template <int MODE, int P>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) void k_run(
    const uint32_t *rk_g, const uint8_t *gt_g, const uint8_t *kp_g, int steps, uint32_t *out)
{
    __shared__ Smem sm;
    fill_common<1024>(sm, gt_g, kp_g);
    __syncthreads();
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_g[i]);
    const LdsTe T{sm.te, (uint32_t)(threadIdx.x & 31) * 4};
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32x4 acc = u32x4{threadIdx.x, blockIdx.x, 0u, 0u};
    const CtrCache cc = ctr_cache(u32x4{blockIdx.x, threadIdx.x >> 2, 7u, 0}, rk, T);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t ph = P > 0 ? wv % P : 0;
    for (int k = 0; k < steps; ++k) {
        u32x4 o0, o1;
        const uint32_t cb = (uint32_t)(k & 63) ^ (acc.x & 1);
        if (MODE == M_CTR4) {
            // four blocks per lane-iteration: two T-table pairs or one 16-block bitsliced set
            u32x4 o2, o3;
            if (P > 0 && ph == 0) {
                bsq_ctr4<kNR>(cc, 4 * cb + 1, 4 * cb + 2, 4 * cb + 3, 4 * cb + 4, rk, T, sm.kp, threadIdx.x & 3, o0,
                              o1, o2, o3);
            } else {
                aes_ctr2<kNR>(cc, 4 * cb + 1, 4 * cb + 2, rk, T, o0, o1);
                aes_ctr2<kNR>(cc, 4 * cb + 3, 4 * cb + 4, rk, T, o2, o3);
            }
            if (P > 0) ph = ph + 1 == (uint32_t)P ? 0 : ph + 1;
            acc ^= o0 ^ o1 ^ o2 ^ o3;
            continue;
        }
        if (P > 0 && ph == 0) {
            bsq_ctr2<kNR>(cc, 2 * cb + 1, 2 * cb + 2, rk, T, sm.kp, threadIdx.x & 3, o0, o1);
        } else {
            aes_ctr2<kNR>(cc, 2 * cb + 1, 2 * cb + 2, rk, T, o0, o1);
        }
        if (P > 0) ph = ph + 1 == (uint32_t)P ? 0 : ph + 1;
        if (MODE == M_STEP) {
            __builtin_amdgcn_sched_barrier(0);
            acc = ghash_mul_h4(acc ^ o0, sm.gh, 0) ^ o1;
            acc = ghash_mul_h4(acc, sm.gh, 0);
        } else {
            acc ^= o0 ^ o1;
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
    out[blockIdx.x * 1024 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int MODE, int P>
static void run(const char *name, const uint32_t *rk, const uint8_t *gt, const uint8_t *kp, uint32_t *out)
{
    const int blocks = 2048, steps = 32;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_run<MODE, P>), dim3(blocks), dim3(1024), kDyn, 0, rk, gt, kp, steps, out);
    const int reps = 5;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_run<MODE, P>), dim3(blocks), dim3(1024), kDyn, 0, rk, gt, kp, steps, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    std::vector<unsigned long long> clk(4096 * 4);
    (void)hipMemcpyFromSymbol(clk.data(), HIP_SYMBOL(g_clk), clk.size() * 8, 0, hipMemcpyDeviceToHost);
    double cyc = 0, tick = 0;
    for (int i = 0; i < blocks; ++i) {
        cyc += (double)(clk[i * 4 + 1] - clk[i * 4 + 0]);
        tick += (double)(clk[i * 4 + 3] - clk[i * 4 + 2]);
    }
    const double mhz = cyc / (tick / 100.0);
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / ((double)blocks * 1024 * steps * (MODE == M_CTR4 ? 4 : 2));
    printf("%-24s P %d  %8.3f ms  clock %5.0f MHz  %6.2f CU-cycles/block\n", name, P, ms, mhz, cu_cyc);
    fflush(stdout);
}

// FIPS-197 key expansion (AES-128), little-endian words
static void expand128(const uint8_t *key, uint32_t *w)
{
    static const uint8_t rcon[10] = {1, 2, 4, 8, 16, 32, 64, 128, 27, 54};
    for (int i = 0; i < 4; ++i) w[i] = key[4 * i] | key[4 * i + 1] << 8 | key[4 * i + 2] << 16 | (uint32_t)key[4 * i + 3] << 24;
    for (int i = 4; i < 44; ++i) {
        uint32_t t = w[i - 1];
        if (i % 4 == 0) {
            t = (t >> 8) | (t << 24);
            t = kAesTables.sbox[t & 255] | kAesTables.sbox[(t >> 8) & 255] << 8 |
                kAesTables.sbox[(t >> 16) & 255] << 16 | (uint32_t)kAesTables.sbox[t >> 24] << 24;
            t ^= rcon[i / 4 - 1];
        }
        w[i] = w[i - 4] ^ t;
    }
}

int main()
{
    uint32_t *rk, *out, *bad;
    uint8_t *gt, *kp;
    (void)hipMalloc(&rk, 44 * 4);
    (void)hipMalloc(&gt, kGh5Bytes);
    (void)hipMalloc(&kp, kKp);
    (void)hipMalloc(&bad, 4);
    (void)hipMalloc(&out, (size_t)2048 * 1024 * 4);
    uint8_t key[16];
    for (int i = 0; i < 16; ++i) key[i] = (uint8_t)(i * 17 + 3);
    uint32_t plain[44], hrk[44];
    expand128(key, plain);
    for (int i = 0; i < 44; ++i) hrk[i] = (i >= 12 && i < 40) ? ((plain[i] >> 16) | (plain[i] << 16)) : plain[i];
    std::vector<uint32_t> planes(kKp / 4, 0);
    for (int r = 3; r <= kNR; ++r)
        for (int L = 0; L < 4; ++L)
            for (int b = 0; b < 8; ++b) {
                uint32_t w = 0;
                for (int c = 0; c < 4; ++c)
                    if ((plain[4 * r + c] >> (8 * L + b)) & 1) w |= 0xffu << (8 * c);
                planes[(r - 3) * 32 + L * 8 + b] = w;
            }
    (void)hipMemcpy(rk, hrk, 44 * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(kp, planes.data(), kKp, hipMemcpyHostToDevice);
    std::vector<uint8_t> hgt(kGh5Bytes);
    for (int i = 0; i < kGh5Bytes; ++i) hgt[i] = (uint8_t)(i * 131 + 7);
    (void)hipMemcpy(gt, hgt.data(), kGh5Bytes, hipMemcpyHostToDevice);
    (void)hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k_check, dim3(64), dim3(1024), 0, 0, rk, gt, kp, bad);
    uint32_t hb = 0;
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("check bsq_ctr2 == aes_ctr2: %u mismatching lane-iterations of %d\n", hb, 64 * 1024 * 4);
    fflush(stdout);
    if (hb) return 1;
    run<M_CTR, 0>("ctr ttable", rk, gt, kp, out);
    run<M_CTR, 1>("ctr bitsliced", rk, gt, kp, out);
    run<M_CTR, 2>("ctr mix", rk, gt, kp, out);
    run<M_CTR, 3>("ctr mix", rk, gt, kp, out);
    run<M_CTR, 4>("ctr mix", rk, gt, kp, out);
    run<M_CTR4, 0>("ctr4 ttable", rk, gt, kp, out);
    run<M_CTR4, 1>("ctr4 bitsliced x2", rk, gt, kp, out);
    run<M_CTR4, 2>("ctr4 mix", rk, gt, kp, out);
    run<M_CTR4, 3>("ctr4 mix", rk, gt, kp, out);
    run<M_CTR4, 4>("ctr4 mix", rk, gt, kp, out);
    run<M_STEP, 0>("step ttable", rk, gt, kp, out);
    run<M_STEP, 1>("step bitsliced", rk, gt, kp, out);
    run<M_STEP, 2>("step mix", rk, gt, kp, out);
    run<M_STEP, 3>("step mix", rk, gt, kp, out);
    run<M_STEP, 4>("step mix", rk, gt, kp, out);
    run<M_STEP, 5>("step mix", rk, gt, kp, out);
    return 0;
}
