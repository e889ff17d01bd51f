// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the engine's access
// pattern (MI355X_MICROARCH.md: "calibrate on a known byte count in your own
// access pattern").  Each kernel moves exactly N_PKT x 1184 bytes:
//   st_pkt  : 16 B/lane stores, 4 lanes x 16 B = 64 contiguous bytes per packet
//             per step, packet slots 1200 B apart, starting at slot offset 11
//             (the header length) -- the protect kernel's store pattern
//   st_al   : the same bytes with the run start rounded down to 16 B
//   ld_pkt  : the same pattern as LDS-DMA loads (global_load_lds_dwordx4)
//   ld_al   : aligned variant
// Prints per-kernel time; run under rocprofv3 --pmc to read the counters.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/calib_hbm tools/calib_hbm.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSlot = 1200, kSteps = 19;  // 19 x 64 B = 1216 >= 1184

template <bool ALIGNED>
__global__ __launch_bounds__(256) void st_pat(uint8_t *out, uint32_t n_pkt)
{
    const uint32_t lp = blockIdx.x * 64 + (threadIdx.x >> 2), sub = threadIdx.x & 3;
    if (lp >= n_pkt) return;
    uint8_t *base = out + (size_t)lp * kSlot + (ALIGNED ? 0 : 11);
    const u32x4 v = {lp, sub, 0x5a5a5a5au, 0xa5a5a5a5u};
    for (int k = 0; k < kSteps; ++k) {
        const int off = 64 * k + 16 * (int)sub;
        if (off + 16 <= 1184) __builtin_memcpy(base + off, &v, 16);
    }
}

template <bool ALIGNED>
__global__ __launch_bounds__(256) void ld_pat(const uint8_t *in, uint32_t n_pkt, uint32_t *sink)
{
    __shared__ u32x4 stage[4][64];
    const uint32_t lp = blockIdx.x * 64 + (threadIdx.x >> 2), sub = threadIdx.x & 3;
    const int w = threadIdx.x >> 6;
    typedef const __attribute__((address_space(1))) void *gptr_t;
    typedef __attribute__((address_space(3))) void *lptr_t;
    u32x4 acc = {0, 0, 0, 0};
    const uint8_t *base = in + (size_t)(lp < n_pkt ? lp : 0) * kSlot + (ALIGNED ? 0 : 11);
    for (int k = 0; k < kSteps; ++k) {
        const int off = 64 * k + 16 * (int)sub;
        __builtin_amdgcn_global_load_lds((gptr_t)(base + (off + 16 <= 1184 ? off : 0)),
                                         (lptr_t)&stage[w][0], 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= stage[w][threadIdx.x & 63];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc.x;
}

int main()
{
    const uint32_t n = 1u << 20;  // 1 Mi packets: 1.26 GB per buffer, past the 256 MiB L3
    uint8_t *a, *b;
    uint32_t *sink;
    (void)hipMalloc(&a, (size_t)n * kSlot);
    (void)hipMalloc(&b, (size_t)n * kSlot);
    (void)hipMalloc(&sink, 4096);
    (void)hipMemset(a, 1, (size_t)n * kSlot);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const dim3 g(n / 64), blk(256);
    auto timeit = [&](const char *name, auto launch) {
        launch();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < 5; ++r) launch();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        printf("%-8s %8.3f ms  %7.1f GB/s of the %zu pattern bytes\n", name, ms,
               (double)n * 1184 / (ms * 1e-3) / 1e9, (size_t)n * 1184);
    };
    timeit("st_pkt", [&] { hipLaunchKernelGGL(st_pat<false>, g, blk, 0, 0, b, n); });
    timeit("st_al", [&] { hipLaunchKernelGGL(st_pat<true>, g, blk, 0, 0, b, n); });
    timeit("ld_pkt", [&] { hipLaunchKernelGGL(ld_pat<false>, g, blk, 0, 0, a, n, sink); });
    timeit("ld_al", [&] { hipLaunchKernelGGL(ld_pat<true>, g, blk, 0, 0, a, n, sink); });
    (void)hipDeviceSynchronize();
    return 0;
}
