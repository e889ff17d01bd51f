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
#include <stdlib.h>

#include <type_traits>
#include <vector>

#include "../aioquic_amd/csrc/qpp_device.h"

using namespace qpp;

namespace qpp { __constant__ AesTables c_aes = kAesTables; }

// Study (r3, not adopted: same LDS occupancy as aes_ctr2, +0.4 % in the
// kernel, profiles/r3p_mb_stagger.txt).
namespace qpp {
// Two counter blocks of one packet as two chains offset by half a phase: the
// LDS lookups of one block are issued while the other block mixes the
// lookups it issued half a phase earlier, so a wave alternates 16 lookups
// with one block's VALU instead of 32 lookups then both blocks' VALU.
// Stages per block: 0 = the round-1 lookup of byte 15, 1 = round 2's four,
// 2 .. NR-2 = full rounds 3 .. NR-1, NR-1 = the final round.  Same result as
// aes_ctr2.
template <int NR, class TE>
struct Ctr2Stagger {
    const CtrCache &c;
    const uint32_t *rk;
    const TE &T;
    uint32_t cb[2];
    uint32_t s[2][4];
    uint32_t e[2][16];
    template <int B, int K>
    __device__ __forceinline__ void issue()
    {
        if constexpr (K == 0) {
            e[B][0] = T.t3(rk[3] ^ (cb[B] << 24));
        } else if constexpr (K == 1) {
            const uint32_t u = s[B][0];
            e[B][0] = T.t0(u);
            e[B][1] = T.t3(u);
            e[B][2] = T.t2(u);
            e[B][3] = T.t1(u);
        } else if constexpr (K < NR - 1) {
#pragma unroll
            for (int col = 0; col < 4; ++col) {
                e[B][4 * col + 0] = T.t0(s[B][col]);
                e[B][4 * col + 1] = T.t1(s[B][(col + 1) & 3]);
                e[B][4 * col + 2] = T.t2r(s[B][(col + 2) & 3]);
                e[B][4 * col + 3] = T.t3r(s[B][(col + 3) & 3]);
            }
        } else {
#pragma unroll
            for (int col = 0; col < 4; ++col) {
                e[B][4 * col + 0] = T.fr0(s[B][col]);
                e[B][4 * col + 1] = T.fr1(s[B][(col + 1) & 3]);
                e[B][4 * col + 2] = T.fr2(s[B][(col + 2) & 3]);
                e[B][4 * col + 3] = T.fr3(s[B][(col + 3) & 3]);
            }
        }
    }
    template <int B, int K>
    __device__ __forceinline__ void mix()
    {
        if constexpr (K == 0) {
            s[B][0] = c.c0 ^ e[B][0];
        } else if constexpr (K == 1) {
            s[B][0] = c.d0 ^ e[B][0];
            s[B][1] = c.d1 ^ e[B][1];
            s[B][2] = c.d2 ^ e[B][2];
            s[B][3] = c.d3 ^ e[B][3];
        } else if constexpr (K < NR - 1) {
            const uint32_t *k = rk + 4 * (K + 1);
#pragma unroll
            for (int col = 0; col < 4; ++col)
                s[B][col] = xor3(e[B][4 * col], e[B][4 * col + 1],
                                 rotl(xor3(e[B][4 * col + 2], e[B][4 * col + 3], k[col]), 16));
        } else {
            const uint32_t *k = rk + 4 * NR;
#pragma unroll
            for (int col = 0; col < 4; ++col)
                s[B][col] = fin_col(e[B][4 * col], e[B][4 * col + 1], e[B][4 * col + 2], e[B][4 * col + 3], k[col]);
        }
    }
    template <int K>
    __device__ __forceinline__ void run()
    {
        if constexpr (K < NR) {
            issue<1, K>();
            __builtin_amdgcn_sched_barrier(0);
            mix<0, K>();
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (K + 1 < NR) {
                issue<0, K + 1>();
                __builtin_amdgcn_sched_barrier(0);
            }
            mix<1, K>();
            __builtin_amdgcn_sched_barrier(0);
            run<K + 1>();
        }
    }
};

template <int NR, class TE>
__device__ __forceinline__ void aes_ctr2s(const CtrCache &c, uint32_t cb0, uint32_t cb1, const uint32_t *rk,
                                          const TE &T, u32x4 &o0, u32x4 &o1)
{
    Ctr2Stagger<NR, TE> g{c, rk, T, {cb0, cb1}, {}, {}};
    g.template issue<0, 0>();
    __builtin_amdgcn_sched_barrier(0);
    g.template run<0>();
    o0 = u32x4{g.s[0][0], g.s[0][1], g.s[0][2], g.s[0][3]};
    o1 = u32x4{g.s[1][0], g.s[1][1], g.s[1][2], g.s[1][3]};
}

}  // namespace qpp


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

enum { M_VALU = 0, M_AES = 1, M_CTR = 2, M_GH = 3, M_CTRGH = 4, M_CTR2 = 5, M_CTR2S = 6 };

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
        if (MODE == M_CTR || MODE == M_CTRGH || MODE == M_CTR2 || MODE == M_CTR2S)
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
            } else if (MODE == M_CTR2 || MODE == M_CTR2S) {
                // two counter blocks of one packet per call (the engine's BPL=2 step)
                u32x4 o0, o1;
                const uint32_t cb = (uint32_t)(k & 127) ^ (acc[c].x & 1);
                if (MODE == M_CTR2) aes_ctr2<10>(cc[c], 2 * cb, 2 * cb + 1, rk, T, o0, o1);
                else aes_ctr2s<10>(cc[c], 2 * cb, 2 * cb + 1, rk, T, o0, o1);
                acc[c] ^= o0 ^ o1;
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


// aes_ctr2s against aes_ctr2 on every lane: mismatches counted into out[0]
__global__ __launch_bounds__(1024) void k_check(const uint32_t *rk_g, uint32_t *bad)
{
    __shared__ uint8_t te[kTeBytes];
    fill_te<1024>(te);
    __syncthreads();
    uint32_t rk[44];
    for (int i = 0; i < 44; ++i) rk[i] = rk_g[i];
    const LdsTe T{te, (uint32_t)(threadIdx.x & 31) * 4};
    const CtrCache cc = ctr_cache(u32x4{blockIdx.x * 977u, threadIdx.x * 31u, 0x1234567u ^ threadIdx.x, 0}, rk, T);
    const uint32_t cb = 1 + (threadIdx.x % 200);
    u32x4 a0, a1, b0, b1;
    aes_ctr2<10>(cc, cb, cb + 7, rk, T, a0, a1);
    aes_ctr2s<10>(cc, cb, cb + 7, rk, T, b0, b1);
    const u32x4 r = aes_ctr<10>(cc, cb, rk, T);
    const bool ok = a0.x == b0.x && a0.y == b0.y && a0.z == b0.z && a0.w == b0.w && a1.x == b1.x && a1.y == b1.y &&
                    a1.z == b1.z && a1.w == b1.w && r.x == a0.x && r.w == a0.w;
    if (!ok) atomicAdd(bad, 1u);
}


// The counter-cached AES block with the T-table image at LDS byte offset OFF;
// the launch's dynamic LDS decides how many workgroups share a CU.
template <int OFF>
struct __attribute__((aligned(16))) SmemOff {
    uint8_t pad[OFF + 16];
    uint8_t te[kTeBytes];
};
template <int WG, int OFF>
__global__ __launch_bounds__(WG) void k_occ(const uint32_t *rk_g, int steps, uint32_t *out)
{
    __shared__ SmemOff<OFF> sm;
    fill_te<WG>(sm.te);
    if (threadIdx.x < 4) ((uint32_t *)sm.pad)[threadIdx.x] = 0;
    __syncthreads();
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_g[i]);
    const LdsTe T{sm.te, (uint32_t)(threadIdx.x & 31) * 4};
    u32x4 acc = u32x4{threadIdx.x, blockIdx.x, 0u, ((const uint32_t *)sm.pad)[threadIdx.x & 3]};
    const CtrCache cc = ctr_cache(u32x4{blockIdx.x, threadIdx.x, 7u, 0}, rk, T);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < steps; ++k) acc ^= aes_ctr<10>(cc, (uint32_t)(k & 255) ^ (acc.x & 1), rk, T);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 4096) {
        g_clk[blockIdx.x * 4 + 0] = c0;
        g_clk[blockIdx.x * 4 + 1] = c1;
        g_clk[blockIdx.x * 4 + 2] = t0;
        g_clk[blockIdx.x * 4 + 3] = t1;
    }
    out[blockIdx.x * WG + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int WG, int OFF>
static void run_occ(const char *name, int dyn, const uint32_t *rk, uint32_t *out)
{
    const int blocks = 2048 * 1024 / WG, steps = 64;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_occ<WG, OFF>), dim3(blocks), dim3(WG), dyn, 0, rk, steps, out);
    const int reps = 5;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_occ<WG, OFF>), dim3(blocks), dim3(WG), dyn, 0, rk, steps, out);
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
    const double units = (double)blocks * WG * steps;
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / units;
    const double f = (133.0 * 2) / 64;
    printf("%-40s te@%6d dyn %6d  %8.3f ms  clock %5.0f MHz  %6.2f CU-cycles/block  frac %.2f\n", name, OFF, dyn, ms,
           mhz, cu_cyc, f / cu_cyc);
    fflush(stdout);
}


// One 1024-thread workgroup with NC copies of the T-table image: wave w
// looks up copy w % NC (is the 2-workgroup gain about copies or workgroups?)
struct LdsTe2 : LdsTe {
    template <int R>
    __device__ __forceinline__ uint32_t addr(uint32_t s) const
    {
        return __builtin_amdgcn_perm(s, lo, 0x0c020000u | ((4u + R) << 8));
    }
    __device__ __forceinline__ uint32_t t0(uint32_t s) const { return *(const uint32_t *)(te + addr<0>(s)); }
    __device__ __forceinline__ uint32_t t1(uint32_t s) const { return *(const uint32_t *)(te + 128 + addr<1>(s)); }
    __device__ __forceinline__ uint32_t t2(uint32_t s) const { return rotl(*(const uint32_t *)(te + addr<2>(s)), 16); }
    __device__ __forceinline__ uint32_t t3(uint32_t s) const { return rotl(*(const uint32_t *)(te + 128 + addr<3>(s)), 16); }
    __device__ __forceinline__ uint32_t t2r(uint32_t s) const { return *(const uint32_t *)(te + addr<2>(s)); }
    __device__ __forceinline__ uint32_t t3r(uint32_t s) const { return *(const uint32_t *)(te + 128 + addr<3>(s)); }
    __device__ __forceinline__ uint32_t fr0(uint32_t s) const { return *(const uint32_t *)(te + addr<0>(s)); }
    __device__ __forceinline__ uint32_t fr1(uint32_t s) const { return *(const uint32_t *)(te + addr<1>(s)); }
    __device__ __forceinline__ uint32_t fr2(uint32_t s) const { return *(const uint32_t *)(te + 128 + addr<2>(s)); }
    __device__ __forceinline__ uint32_t fr3(uint32_t s) const { return *(const uint32_t *)(te + 128 + addr<3>(s)); }
};
template <int NC>
__global__ __launch_bounds__(1024) void k_copies(const uint32_t *rk_g, int steps, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t te_all[NC * kTeBytes + 16];
    for (int c = 0; c < NC; ++c) fill_te<1024>(te_all + c * kTeBytes);
    __syncthreads();
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_g[i]);
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // copy c at LDS 64 KiB * c: the copy index rides in byte 2 of the v_perm
    // constant (LdsTe2), so every copy costs one v_perm per lookup
    const LdsTe2 T{te_all, (uint32_t)(threadIdx.x & 31) * 4 | ((wv % NC) << 16)};
    u32x4 acc = u32x4{threadIdx.x, blockIdx.x, 0u, 0u};
    const CtrCache cc = ctr_cache(u32x4{blockIdx.x, threadIdx.x, 7u, 0}, rk, T);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < steps; ++k) acc ^= aes_ctr<10>(cc, (uint32_t)(k & 255) ^ (acc.x & 1), rk, T);
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
template <int NC>
static void run_copies(const char *name, int dyn, const uint32_t *rk, uint32_t *out)
{
    const int blocks = 2048, steps = 64;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_copies<NC>), dim3(blocks), dim3(1024), dyn, 0, rk, steps, out);
    const int reps = 5;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_copies<NC>), dim3(blocks), dim3(1024), dyn, 0, rk, steps, out);
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
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / ((double)blocks * 1024 * steps);
    printf("%-40s %8.3f ms  clock %5.0f MHz  %6.2f CU-cycles/block  frac %.2f\n", name, ms, mhz, cu_cyc,
           (133.0 * 2) / 64 / cu_cyc);
    fflush(stdout);
}


// The GCM step loop's LDS work without its memory side: per lane-step two
// counter-cached AES blocks (aes_ctr2) and two 5-bit-window GHASH multiplies
// by H^4 from a 14 KiB LDS table (ghash_mul_h4), as in gcm_packet<BPL=2>.
struct __attribute__((aligned(16))) SmemStep {
    uint8_t gh[kGh5Bytes];
    uint8_t te[kTeBytes];
};
template <int WG>
__global__ __launch_bounds__(WG) void k_step(const uint32_t *rk_g, const uint8_t *gt_g, int steps, uint32_t *out)
{
    __shared__ SmemStep sm;
    fill_te<WG>(sm.te);
    for (int i = threadIdx.x; i < kGh5Bytes / 16; i += WG) ((u32x4 *)sm.gh)[i] = ((const u32x4 *)gt_g)[i];
    __syncthreads();
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_g[i]);
    const LdsTe T{sm.te, (uint32_t)(threadIdx.x & 31) * 4};
    u32x4 acc = u32x4{threadIdx.x, blockIdx.x, 0u, 0u};
    const CtrCache cc = ctr_cache(u32x4{blockIdx.x, threadIdx.x, 7u, 0}, rk, T);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < steps; ++k) {
        u32x4 o0, o1;
        const uint32_t cb = (uint32_t)(k & 127) ^ (acc.x & 1);
        aes_ctr2<10>(cc, 2 * cb, 2 * cb + 1, rk, T, o0, o1);
        __builtin_amdgcn_sched_barrier(0);
        acc = ghash_mul_h4(acc ^ o0, sm.gh, 0) ^ o1;
        acc = ghash_mul_h4(acc, sm.gh, 0);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 4096) {
        g_clk[blockIdx.x * 4 + 0] = c0;
        g_clk[blockIdx.x * 4 + 1] = c1;
        g_clk[blockIdx.x * 4 + 2] = t0;
        g_clk[blockIdx.x * 4 + 3] = t1;
    }
    out[blockIdx.x * WG + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}
template <int WG>
static void run_step(const char *name, int dyn, const uint32_t *rk, const uint8_t *gt, uint32_t *out)
{
    const int blocks = 2048 * 1024 / WG, steps = 32;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_step<WG>), dim3(blocks), dim3(WG), dyn, 0, rk, gt, steps, out);
    const int reps = 5;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_step<WG>), dim3(blocks), dim3(WG), dyn, 0, rk, gt, steps, out);
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
    // two blocks per lane-step
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / ((double)blocks * WG * steps * 2);
    const double f = (133.0 * 2 + 26.0 * 2) / 64;  // per block: 133 ds_read_b32 + one multiply's 26 b64 pairs
    printf("%-40s %8.3f ms  clock %5.0f MHz  %6.2f CU-cycles/block  LDS floor %.2f frac %.2f\n", name, ms, mhz, cu_cyc,
           f, f / cu_cyc);
    fflush(stdout);
}


// k_step with the kernel's memory side: per lane-step two 16-byte loads one
// step ahead and two 16-byte stores, a quad covering 128 contiguous bytes
// (16 packets of 1200 bytes per wave, each quad walking its packet).
template <int WG>
__global__ __launch_bounds__(WG) void k_stepm(const uint32_t *rk_g, const uint8_t *gt_g, int steps,
                                              const uint8_t *gin, uint8_t *gout, uint32_t *out)
{
    __shared__ SmemStep sm;
    fill_te<WG>(sm.te);
    for (int i = threadIdx.x; i < kGh5Bytes / 16; i += WG) ((u32x4 *)sm.gh)[i] = ((const u32x4 *)gt_g)[i];
    __syncthreads();
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; ++i) rk[i] = __builtin_amdgcn_readfirstlane(rk_g[i]);
    const LdsTe T{sm.te, (uint32_t)(threadIdx.x & 31) * 4};
    u32x4 acc = u32x4{threadIdx.x, blockIdx.x, 0u, 0u};
    const CtrCache cc = ctr_cache(u32x4{blockIdx.x, threadIdx.x, 7u, 0}, rk, T);
    // packet of this quad: 1200-byte slots, 11-byte header
    const uint32_t pk = (blockIdx.x * WG + threadIdx.x) >> 2, j = threadIdx.x & 3;
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)gin, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)gout, 0, 0x7fffffff, 0x00020000);
    const uint32_t base = pk * 1200u + 11u;
    auto off = [&](int k, int h) -> uint32_t { return base + (uint32_t)(((8 * k + 4 * h + (int)j) % 72) * 16); };
    u32x4 n0 = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)off(0, 0), 0, 0);
    u32x4 n1 = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)off(0, 1), 0, 0);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < steps; ++k) {
        const u32x4 r0 = n0, r1 = n1;
        n0 = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)off(k + 1, 0), 0, 0);
        n1 = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)off(k + 1, 1), 0, 0);
        u32x4 o0, o1;
        const uint32_t cb = (uint32_t)(k & 127) ^ (acc.x & 1);
        aes_ctr2<10>(cc, 2 * cb, 2 * cb + 1, rk, T, o0, o1);
        o0 ^= r0;
        o1 ^= r1;
        __builtin_amdgcn_raw_buffer_store_b128(o0, ro, (int)off(k, 0), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(o1, ro, (int)off(k, 1), 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        acc = ghash_mul_h4(acc ^ o0, sm.gh, 0) ^ o1;
        acc = ghash_mul_h4(acc, sm.gh, 0);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 4096) {
        g_clk[blockIdx.x * 4 + 0] = c0;
        g_clk[blockIdx.x * 4 + 1] = c1;
        g_clk[blockIdx.x * 4 + 2] = t0;
        g_clk[blockIdx.x * 4 + 3] = t1;
    }
    out[blockIdx.x * WG + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}
template <int WG>
static void run_stepm(const char *name, int dyn, const uint32_t *rk, const uint8_t *gt, uint32_t *out,
                      const uint8_t *gin, uint8_t *gout)
{
    const int blocks = 2048 * 1024 / WG, steps = 32;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL((k_stepm<WG>), dim3(blocks), dim3(WG), dyn, 0, rk, gt, steps, gin, gout, out);
    const int reps = 5;
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((k_stepm<WG>), dim3(blocks), dim3(WG), dyn, 0, rk, gt, steps, gin, gout, out);
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
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / ((double)blocks * WG * steps * 2);
    const double f = (133.0 * 2 + 26.0 * 2) / 64;
    printf("%-40s %8.3f ms  clock %5.0f MHz  %6.2f CU-cycles/block  LDS floor %.2f frac %.2f\n", name, ms, mhz, cu_cyc,
           f, f / cu_cyc);
    fflush(stdout);
}

// LDS-array cycles per block per wave-instruction model (MI355X_MICROARCH.md sec. LDS):
// ds_read_b32 = 2 cycles, ds_read_b128 = 4 cycles per 64 lanes
static double lds_model(int mode)
{
    switch (mode) {
    case M_AES: return (160.0 * 2) / 64;
    case M_CTR: case M_CTR2: case M_CTR2S: return (133.0 * 2) / 64;
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
    const double units = (double)blocks * WG * steps * CH * ((MODE == M_CTR2 || MODE == M_CTR2S) ? 2 : 1);  // lane-blocks (or lane-iterations)
    const double cu_cyc = ms * 1e-3 * mhz * 1e6 * 256 / units;
    if (MODE == M_VALU) {
        // 64 bitop3 per lane-iteration: lane-ops per CU-cycle
        printf("%-8s WG %4d CH %d  %8.3f ms  clock %5.0f MHz  %6.1f lane-ops/CU-cycle (peak 128)\n", name,
               WG, CH, ms, mhz, 64.0 / cu_cyc);
    } else {
        const double f = lds_model(MODE);
        printf("%-22s WG %4d CH %d%s  %8.3f ms  clock %5.0f MHz  %6.2f CU-cycles/block  LDS floor %5.2f  frac %.2f\n",
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
    {
        uint32_t *bad;
        (void)hipMalloc(&bad, 4);
        (void)hipMemset(bad, 0, 4);
        hipLaunchKernelGGL(k_check, dim3(64), dim3(1024), 0, 0, rk, bad);
        uint32_t hb = 0;
        (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
        printf("check aes_ctr2s == aes_ctr2 == aes_ctr: %u mismatching lanes of %d\n", hb, 64 * 1024);
    }
    if (getenv("MB_STEPM_ONLY")) {
        // 2048 x 1024 lanes / 4 = 512 Ki packets of 1200 bytes
        uint8_t *gin, *gout;
        (void)hipMalloc(&gin, (size_t)512 * 1024 * 1200 + 4096);
        (void)hipMalloc(&gout, (size_t)512 * 1024 * 1200 + 4096);
        (void)hipMemset(gin, 7, (size_t)512 * 1024 * 1200 + 4096);
        for (int rep = 0; rep < 2; ++rep) {
            run_step<1024>("step 1x1024 (dyn)", 8 * 1024, rk, gt, out);
            run_step<512>("step 2x512", 0, rk, gt, out);
            run_stepm<1024>("step+mem 1x1024 (dyn)", 8 * 1024, rk, gt, out, gin, gout);
            run_stepm<512>("step+mem 2x512", 0, rk, gt, out, gin, gout);
        }
        return 0;
    }
    if (getenv("MB_OFF2_ONLY")) {
        // two 512-thread workgroups per CU with the image at the offsets the
        // engine's layouts put it (after 1 or 4 GHASH entries), against 0
        for (int rep = 0; rep < 2; ++rep) {
            run_occ<512, 0>("2x512, te at 0", 0, rk, out);
            run_occ<512, 14336>("2x512, te at 14K (1 entry first)", 0, rk, out);
            run_occ<1024, 57344>("1x1024, te at 56K (engine)", 0, rk, out);
            run_occ<512, 0>("2x512, te at 0, dyn 14K", 14336, rk, out);
        }
        return 0;
    }
    if (getenv("MB_STEP_ONLY")) {
        for (int rep = 0; rep < 2; ++rep) {
            run_step<1024>("step 1x1024 (dyn)", 8 * 1024, rk, gt, out);
            run_step<1024>("step 2x1024 if VGPRs allow", 0, rk, gt, out);
            run_step<512>("step 2x512", 0, rk, gt, out);
            run_step<512>("step 1x512 (dyn)", 40 * 1024, rk, gt, out);
            run_step<768>("step 1x768", 0, rk, gt, out);
        }
        return 0;
    }
    if (getenv("MB_COPIES_ONLY")) {
        for (int rep = 0; rep < 2; ++rep) {
            run_copies<1>("1x1024, one image (dyn: 1 WG/CU)", 60 * 1024, rk, out);
            run_copies<1>("2x1024, one image each", 0, rk, out);
            run_copies<2>("1x1024, two images (wave % 2)", 0, rk, out);
            run_occ<512, 0>("2x512, te at 0", 0, rk, out);
        }
        return 0;
    }
    if (getenv("MB_OCC2_ONLY")) {
        const int one = 60 * 1024;  // dynamic LDS that leaves room for one workgroup per CU
        for (int rep = 0; rep < 2; ++rep) {
            run_occ<1024, 0>("1x1024, te at 0", one, rk, out);
            run_occ<1024, 47104>("1x1024, te at 46K (mb Smem)", 0, rk, out);
            run_occ<1024, 57344>("1x1024, te at 56K (engine)", 0, rk, out);
            run_occ<1024, 81920>("1x1024, te at 80K", 0, rk, out);
            run_occ<1024, 0>("2x1024, te at 0", 0, rk, out);
            run_occ<512, 0>("2x512, te at 0", 0, rk, out);
            run_occ<512, 0>("1x512, te at 0", one, rk, out);
            run_occ<256, 0>("2x256, te at 0", 0, rk, out);
        }
        return 0;
    }
    if (getenv("MB_OCC_ONLY")) {
        // occupancy curve of the counter-cached AES block: waves per SIMD set by
        // the workgroup size and two 64 KiB images per CU (SMALL), against one
        // 1024-thread workgroup per CU
        for (int rep = 0; rep < 2; ++rep) {
            run<1024, M_CTR, 1>("ctr 1x1024 (4/SIMD)", rk, gt, out);
            run<512, M_CTR, 1, true>("ctr 2x512 (4/SIMD)", rk, gt, out);
            run<640, M_CTR, 1, true>("ctr 2x640 (5/SIMD)", rk, gt, out);
            run<768, M_CTR, 1, true>("ctr 2x768 (6/SIMD)", rk, gt, out);
            run<896, M_CTR, 1, true>("ctr 2x896 (7/SIMD)", rk, gt, out);
            run<1024, M_CTR, 1, true>("ctr 2x1024 (8/SIMD)", rk, gt, out);
        }
        return 0;
    }
    if (getenv("MB_STAGGER_ONLY")) {
        for (int rep = 0; rep < 3; ++rep) {
            run<1024, M_CTR, 1>("ctr", rk, gt, out);
            run<1024, M_CTR2, 1>("ctr2", rk, gt, out);
            run<1024, M_CTR2S, 1>("ctr2-stagger", rk, gt, out);
            run<1024, M_CTR2, 1, true>("ctr2", rk, gt, out);
            run<1024, M_CTR2S, 1, true>("ctr2-stagger", rk, gt, out);
        }
        return 0;
    }
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
