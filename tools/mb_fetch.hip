// FETCH_SIZE calibration for the GCM kernel's read pattern (VERDICT r2 item 4,
// config 4): 1 Mi packets of 1200 B, each read once by its quad with the
// engine's step pattern (lane j loads 16-byte blocks 8k + j and 8k + 4 + j at
// step k, from payload offset 11), 16 packets per wave.  The packets a wave
// reads are either consecutive (the north star's grouped arrival) or a random
// permutation of the buffer (config 4's random arrival), so that the counter's
// bytes can be compared with the 1.25 GB actually read in both layouts.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb_fetch tools/mb_fetch.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <random>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kPkt = 1200, kIn = 1189, kOff = 11;
constexpr uint32_t kOob = 0x80000000u;

template <int K>
__global__ __launch_bounds__(256) void k_fetch(const uint8_t *in, const uint32_t *order, uint32_t *out, int n)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    const int p = gid >> 2, j = gid & 3;
    if (p >= n) return;
    const uint32_t pk = K == 0 ? (uint32_t)p : order[p];
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(in + (size_t)pk * kPkt), 0, kPkt, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    for (int s = kOff; s < kOff + kIn; s += 128) {
        for (int h = 0; h < 2; ++h) {
            const int b = s + 16 * (j + 4 * h);
            const uint32_t o = b + 16 <= kOff + kIn ? (uint32_t)b : kOob;
            acc ^= __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, 0);
        }
    }
    out[gid] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int K>
static void run(const char *name, const uint8_t *in, const uint32_t *order, uint32_t *out, int n)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int grid = (4 * n + 255) / 256;
    hipLaunchKernelGGL(k_fetch<K>, dim3(grid), dim3(256), 0, 0, in, order, out, n);
    (void)hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_fetch<K>, dim3(grid), dim3(256), 0, 0, in, order, out, n);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-44s %8.3f ms/launch  %.1f GB/s of %.0f MB read\n", name, ms / reps,
           (double)n * kIn / (ms / reps * 1e-3) / 1e9, (double)n * kIn / 1e6);
}

int main()
{
    const int n = 1 << 20;
    uint8_t *in;
    uint32_t *order, *out;
    (void)hipMalloc(&in, (size_t)n * kPkt);
    (void)hipMalloc(&order, (size_t)n * 4);
    (void)hipMalloc(&out, (size_t)n * 16);
    (void)hipMemset(in, 0x5a, (size_t)n * kPkt);
    std::vector<uint32_t> h(n);
    for (int i = 0; i < n; ++i) h[i] = i;
    std::shuffle(h.begin(), h.end(), std::mt19937(7));
    (void)hipMemcpy(order, h.data(), (size_t)n * 4, hipMemcpyHostToDevice);
    run<0>("K0: packets in buffer order (grouped)", in, order, out, n);
    run<1>("K1: packets in random order (config 4)", in, order, out, n);
    return 0;
}
