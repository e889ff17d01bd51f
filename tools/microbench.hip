// Ablation microbenchmark for the GCM building blocks (no global traffic):
// AES-CTR alone, GHASH alone, both, on the same LDS layouts as the engine.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../aioquic_amd/csrc/qpp_device.h"

using namespace qpp;

namespace qpp { __constant__ AesTables c_aes = kAesTables; }

template <int NT>
__device__ void load_te(uint8_t *te)
{
    for (int i = threadIdx.x; i < 256 * 16; i += NT) {
        const int x = i >> 4, part = i & 15;
        const uint32_t v0 = c_aes.te0[x];
        const uint32_t v = part < 8 ? v0 : rotl(v0, 8);
        *(u32x4 *)(te + x * 256 + part * 16) = u32x4{v, v, v, v};
    }
}

struct __attribute__((aligned(16))) S {
    uint8_t te[kTeBytes];
    uint8_t gt[kGhashTabBytes];
};

// MODE bit 0: AES, bit 1: GHASH; CH independent chains per lane (ILP)
template <int WG, int MODE, int CH = 1>
__global__ __launch_bounds__(WG) void k_bench(const uint32_t *rk_g, const uint8_t *gt_g, int steps,
                                              uint32_t *out)
{
    __shared__ S sm;
    load_te<WG>(sm.te);
    for (int i = threadIdx.x; i < kGhashTabBytes / 16; i += WG)
        ((u32x4 *)sm.gt)[i] = ((const u32x4 *)gt_g)[i];
    __syncthreads();
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_g[i]);
    const LdsTe T{sm.te, (uint32_t)(threadIdx.x & 31) * 4};
    u32x4 acc[CH], ctr[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        acc[c] = u32x4{threadIdx.x, blockIdx.x, (uint32_t)c, 0};
        ctr[c] = u32x4{blockIdx.x, threadIdx.x, 7u + c, 0};
    }
    for (int k = 0; k < steps; ++k) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            ctr[c].w = k;
            u32x4 x = ctr[c];
            if (MODE & 1) x = aes_encrypt<10>(ctr[c], rk, T);
            acc[c] ^= x;
            if (MODE & 2) acc[c] = ghash_mul(acc[c], sm.gt, 3 * 8192);
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) r ^= acc[c].x ^ acc[c].y ^ acc[c].z ^ acc[c].w;
    out[blockIdx.x * WG + threadIdx.x] = r;
}

template <int WG, int MODE, int CH = 1>
static float run(const uint32_t *rk, const uint8_t *gt, uint32_t *out, int blocks, int steps)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_bench<WG, MODE, CH>), dim3(blocks), dim3(WG), 0, 0, rk, gt, steps, out);
    (void)hipEventRecord(a, 0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_bench<WG, MODE, CH>), dim3(blocks), dim3(WG), 0, 0, rk, gt, steps, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <int WG, int CH = 1>
static void sweep(const uint32_t *rk, const uint8_t *gt, uint32_t *out)
{
    const int blocks = 256 * (1024 / WG) / CH;  // same block count for every variant
    const int steps = 80;
    const double lane_blocks = (double)blocks * WG * steps * CH;
    const char *names[] = {"none", "aes", "ghash", "aes+ghash"};
    float t[4] = {run<WG, 0, CH>(rk, gt, out, blocks, steps), run<WG, 1, CH>(rk, gt, out, blocks, steps),
                  run<WG, 2, CH>(rk, gt, out, blocks, steps), run<WG, 3, CH>(rk, gt, out, blocks, steps)};
    for (int m = 0; m < 4; ++m)
        printf("WG %4d x%d %-10s %8.3f ms  %7.2f Gblock/s  %6.2f CU-cycles/block @2.4GHz\n", WG, CH,
               names[m], t[m], lane_blocks / (t[m] * 1e-3) / 1e9,
               t[m] * 1e-3 * 2.4e9 * 256 / lane_blocks);
}

int main()
{
    uint32_t *rk;
    uint8_t *gt;
    uint32_t *out;
    (void)hipMalloc(&rk, 44 * 4);
    (void)hipMalloc(&gt, kGhashTabBytes);
    (void)hipMalloc(&out, 256 * 1024 * 4 * 4);
    (void)hipMemset(rk, 0x5a, 44 * 4);
    (void)hipMemset(gt, 0x33, kGhashTabBytes);
    sweep<512>(rk, gt, out);
    sweep<1024>(rk, gt, out);
    sweep<512, 2>(rk, gt, out);
    sweep<256, 2>(rk, gt, out);
    sweep<256, 4>(rk, gt, out);
    return 0;
}
