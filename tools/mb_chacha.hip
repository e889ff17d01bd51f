// ChaCha20-Poly1305 building-block microbenchmark (no global traffic in the
// loop): ChaCha20 blocks alone, with the 4 Poly1305 multiplies of a 64-byte
// chunk, and CH independent chunks per lane (ILP), at several waves per SIMD.
// Reports CU-cycles per 64-byte chunk at 2.4 GHz; the engine's k_chacha runs
// a 1 Mi-packet protect at ~38 (1.30 ms, profiles/r2f_sweep.jsonl).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/mb_chacha tools/mb_chacha.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../aioquic_amd/csrc/qpp_chacha.h"

using namespace qpp;

// MODE bit 0: ChaCha20 block, bit 1: Poly1305 (4 multiplies per chunk)
template <int WG, int MODE, int CH, int WPE>
__global__ __launch_bounds__(WG, WPE) void k_mb(const uint32_t *key_g, int steps, uint32_t *out)
{
    uint32_t key[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) key[i] = __builtin_amdgcn_readfirstlane(key_g[i]);
    const uint32_t t = blockIdx.x * WG + threadIdx.x;
    P130 acc[CH], r;
    uint32_t sink[CH];
    r = p130_r(t, t * 3u, t * 5u, t * 7u);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        acc[c] = p130_zero();
        sink[c] = c;
    }
    for (int k = 0; k < steps; ++k) {
        uint32_t blk[CH][16];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (MODE & 1) {
                chacha_block(key, (uint32_t)(k * CH + c), t, sink[c], 7u, blk[c]);
            } else {
#pragma unroll
                for (int w = 0; w < 16; ++w) blk[c][w] = sink[c] + w + k;
            }
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (MODE & 2) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[c] = p130_mul(p130_add(acc[c], p130_block(u32x4{blk[c][4 * q], blk[c][4 * q + 1],
                                                                          blk[c][4 * q + 2], blk[c][4 * q + 3]})),
                                      r);
                sink[c] ^= acc[c].v[0] ^ blk[c][15];
            } else {
                uint32_t x = 0;
#pragma unroll
                for (int w = 0; w < 16; ++w) x ^= blk[c][w];
                sink[c] ^= x;
            }
        }
    }
    uint32_t o = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) o ^= sink[c] ^ acc[c].v[1];
    out[t] = o;
}

template <int WG, int MODE, int CH, int WPE>
static void run(const uint32_t *key, uint32_t *out)
{
    // 16 waves per CU of lanes, whatever WG / CH: same chunks per launch
    const int blocks = 256 * (1024 / WG) * WPE / 4;
    const int steps = 64 / CH;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_mb<WG, MODE, CH, WPE>), dim3(blocks), dim3(WG), 0, 0, key, steps, out);
    (void)hipEventRecord(a, 0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((k_mb<WG, MODE, CH, WPE>), dim3(blocks), dim3(WG), 0, 0, key, steps, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double chunks = (double)blocks * WG * steps * CH;
    const char *names[] = {"none", "chacha", "poly", "chacha+poly"};
    printf("WG %4d x%d wpe %d %-12s %8.3f ms  %6.2f CU-cycles/chunk @2.4GHz\n", WG, CH, WPE, names[MODE], ms,
           ms * 1e-3 * 2.4e9 * 256 / chunks);
}

// The engine's grid shape: one packet per quad, lane `sub` owns chunks
// 4k + sub of a 1173-byte payload at byte offset OFF of a 1200-byte packet;
// MEM: 0 compute only, 1 loads + stores of the lane's chunks, 2 the same
// amount with the quad's 4 lanes on one chunk per instruction (coalesced).
template <int OFF, int MEM>
__global__ __launch_bounds__(256) void k_grid(const uint32_t *key_g, const uint8_t *in, uint8_t *outb,
                                             uint32_t *out)
{
    uint32_t key[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) key[i] = __builtin_amdgcn_readfirstlane(key_g[i]);
    const uint32_t t = blockIdx.x * 256 + threadIdx.x, p = t >> 2, sub = t & 3;
    const P130 r = p130_r(t, t * 3u, t * 5u, t * 7u);
    P130 acc = p130_zero();
    const uint8_t *src = in + (size_t)p * 1200 + OFF;
    uint8_t *dst = outb + (size_t)p * 1200 + OFF;
    for (int c = sub; c < 16; c += 4) {  // 16 full chunks of 64 B (1024 B + OFF < 1200)
        uint32_t blk[16];
        chacha_block(key, (uint32_t)c + 1, p, 5u, 7u, blk);
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            v[q] = u32x4{blk[4 * q], blk[4 * q + 1], blk[4 * q + 2], blk[4 * q + 3]};
            if (MEM == 1) v[q] ^= ld16(src + 64 * c + 16 * q);
            // coalesced: the quad reads chunk (c - sub + q) contiguously (data placement only)
            if (MEM == 2) v[q] ^= ld16(src + 64 * (c - (int)sub + q) + 16 * sub);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (MEM == 1) st16(dst + 64 * c + 16 * q, v[q]);
            if (MEM == 2) st16(dst + 64 * (c - (int)sub + q) + 16 * sub, v[q]);
            acc = p130_mul(p130_add(acc, p130_block(v[q])), r);
        }
    }
    out[t] = acc.v[0] ^ acc.v[3];
}

template <int OFF, int MEM>
static void run_grid(const uint32_t *key, const uint8_t *in, uint8_t *outb, uint32_t *out)
{
    const int blocks = (1 << 20) * 4 / 256;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_grid<OFF, MEM>), dim3(blocks), dim3(256), 0, 0, key, in, outb, out);
    (void)hipEventRecord(a, 0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_grid<OFF, MEM>), dim3(blocks), dim3(256), 0, 0, key, in, outb, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double chunks = (double)(1 << 20) * 16;
    printf("grid 1Mi pkts off %2d mem %d  %8.3f ms  %6.2f CU-cycles/chunk @2.4GHz\n", OFF, MEM, ms,
           ms * 1e-3 * 2.4e9 * 256 / chunks);
}

int main()
{
    uint32_t *key, *out;
    (void)hipMalloc(&key, 32);
    (void)hipMalloc(&out, 256 * 1024 * 8 * 4);
    (void)hipMemset(key, 0x5a, 32);
    run<256, 1, 1, 4>(key, out);
    run<256, 2, 1, 4>(key, out);
    run<256, 3, 1, 4>(key, out);
    run<256, 3, 1, 8>(key, out);
    run<256, 1, 2, 4>(key, out);
    run<256, 3, 2, 4>(key, out);
    run<256, 3, 2, 8>(key, out);
    run<256, 3, 4, 4>(key, out);
    uint8_t *in, *outb;
    (void)hipMalloc(&in, (size_t)1200 << 20);
    (void)hipMalloc(&outb, (size_t)1200 << 20);
    (void)hipMemset(in, 0x11, (size_t)1200 << 20);
    (void)hipMalloc(&out, (size_t)4 << 22);
    run_grid<11, 0>(key, in, outb, out);
    run_grid<11, 1>(key, in, outb, out);
    run_grid<16, 1>(key, in, outb, out);
    run_grid<11, 2>(key, in, outb, out);
    run_grid<16, 2>(key, in, outb, out);
    return 0;
}
