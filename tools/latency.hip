// Launch-time latency probe: what does a dependent global load cost when
// every CU starts at once, and what does cold straight-line code cost?
// Shapes match k_packets (1024-thread workgroups, ~150 KB LDS -> 1 WG/CU).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/latency tools/latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int WG = 1024;

__device__ unsigned long long g_t[8192 * 8], g_c[8192 * 8];

// wall clock (100 MHz) and shader clock: their ratio is the running frequency
#define STAMP(i)                                                                           \
    do {                                                                                   \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                    \
        const unsigned long long c_ = __builtin_amdgcn_s_memtime();                        \
        if ((threadIdx.x & 63) == 0) {                                                     \
            g_t[(blockIdx.x * (WG / 64) + (threadIdx.x >> 6)) * 8 + (i)] = t_;             \
            g_c[(blockIdx.x * (WG / 64) + (threadIdx.x >> 6)) * 8 + (i)] = c_;             \
        }                                                                                  \
    } while (0)

#define NOPS16 "v_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\t" \
               "v_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\tv_nop\n\t"
#define NOPS256 NOPS16 NOPS16 NOPS16 NOPS16 NOPS16 NOPS16 NOPS16 NOPS16 \
                NOPS16 NOPS16 NOPS16 NOPS16 NOPS16 NOPS16 NOPS16 NOPS16

// chain: idx -> a[idx] -> b[a[idx]] ... three dependent loads, then cold code
__global__ __launch_bounds__(WG) void k_lat(const uint32_t *a, const uint32_t *b, const uint8_t *big,
                                           uint32_t *out, int stride)
{
    __shared__ uint8_t pad[150 * 1024];
    STAMP(0);
    const uint32_t p = blockIdx.x * (WG / 4) + (threadIdx.x >> 2);
    const uint32_t v0 = a[p];                    // like the descriptor
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(1);
    const uint32_t v1 = *(const uint32_t *)(big + (size_t)v0 * stride);  // like the header
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(2);
    const uint32_t v2 = *(const uint32_t *)(big + (size_t)v0 * stride + 512);  // same packet again
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(3);
    asm volatile(NOPS256 NOPS256 NOPS256 NOPS256);  // 1024 x 4 B of cold straight-line code
    STAMP(4);
    // the same 256 instructions 4 times: warm after the first pass
    for (int r = 0; r < 4; ++r) asm volatile(NOPS256);
    STAMP(5);
    pad[threadIdx.x] = (uint8_t)(v1 ^ v2);
    __syncthreads();
    STAMP(6);
    out[blockIdx.x * WG + threadIdx.x] = v1 + v2 + pad[(threadIdx.x + 1) % WG] + b[0];
}

int main()
{
    const int n = 65536, stride = 1200, blocks = n / (WG / 4);
    uint32_t *a, *b, *out;
    uint8_t *big;
    (void)hipMalloc(&a, n * 4);
    (void)hipMalloc(&b, 4096);
    (void)hipMalloc(&out, blocks * WG * 4);
    (void)hipMalloc(&big, (size_t)n * stride);
    std::vector<uint32_t> h(n);
    for (int i = 0; i < n; ++i) h[i] = i;
    (void)hipMemcpy(a, h.data(), n * 4, hipMemcpyHostToDevice);
    (void)hipMemset(big, 1, (size_t)n * stride);
    const int waves = blocks * (WG / 64);
    std::vector<unsigned long long> t((size_t)waves * 8), c((size_t)waves * 8);
    const char *names[] = {"desc load", "dependent load (cold line)", "same packet +512 B",
                           "1024 cold v_nop", "256 v_nop x4 (loop)", "LDS write + barrier"};
    for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(k_lat, dim3(blocks), dim3(WG), 0, 0, a, b, big, out, stride);
        (void)hipDeviceSynchronize();
        (void)hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_t), t.size() * 8, 0, hipMemcpyDeviceToHost);
        (void)hipMemcpyFromSymbol(c.data(), HIP_SYMBOL(g_c), c.size() * 8, 0, hipMemcpyDeviceToHost);
        printf("launch %d:\n", rep);
        for (int ph = 0; ph < 6; ++ph) {
            double sum = 0, mx = 0, cyc = 0;
            for (int w = 0; w < waves; ++w) {
                const double d = (double)(t[w * 8 + ph + 1] - t[w * 8 + ph]) / 100.0;
                sum += d;
                cyc += (double)(c[w * 8 + ph + 1] - c[w * 8 + ph]);
                mx = std::max(mx, d);
            }
            printf("  %-28s mean %7.2f us  max %7.2f us  clock %6.0f MHz (%8.0f cyc)\n", names[ph],
                   sum / waves, mx, cyc / sum, cyc / waves);
        }
    }
    return 0;
}
