// Table-lookup throughput on one MI355X: is the vector L1 (TA/TD path) a
// usable second lookup port beside the LDS for the GCM kernel's T-table and
// GHASH lookups?  Every lane runs 8 independent dependent chains
// x <- T[x & 255] ^ x (T-table shape) of one access kind, 16 waves per CU,
// one 1024-thread workgroup per CU; reported as CU-cycles per wave
// instruction at the measured clock (s_memtime over the loop).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb_gather tools/mb_gather.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 2048;

#define CH8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

// K = 0: LDS ds_read_b32, table replicated per bank (the engine's layout)
// K = 1: global_load_dword from a 1 KiB table
// K = 2: global_load_dword from a 16 KiB table (16 rows of 1 KiB, row by chain)
// K = 3: global_load_dwordx2 from a 256 B row per window (GHASH 5-bit shape)
// K = 4: 3 LDS chains-steps + 1 global per 4 (mixed issue)
// K = 5: buffer_load_dword (1 KiB table) with the nt bit clear
template <int K>
__global__ __launch_bounds__(1024) void k_gather(const uint32_t *__restrict__ gtab, uint32_t *out,
                                                 unsigned long long *cyc, uint32_t seed)
{
    __shared__ uint32_t lt[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += 1024) lt[i] = gtab[(i >> 5) & 255];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 31;
    uint32_t a0 = threadIdx.x * 0x9E3779B9u ^ seed, a1 = a0 * 3 + 1, a2 = a0 * 5 + 2, a3 = a0 * 7 + 3,
             a4 = a0 * 9 + 4, a5 = a0 * 11 + 5, a6 = a0 * 13 + 6, a7 = a0 * 15 + 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < kIters; ++i) {
        if constexpr (K == 0) {
#define OP(x) x ^= lt[((x & 255) << 5) | lane];
            CH8(OP)
#undef OP
        } else if constexpr (K == 1) {
#define OP(x) x ^= gtab[x & 255];
            CH8(OP)
#undef OP
        } else if constexpr (K == 2) {
            int r = 0;
#define OP(x) x ^= gtab[((r++) << 8) | (x & 255)];
            CH8(OP)
#undef OP
        } else if constexpr (K == 3) {
            const uint2 *g2 = (const uint2 *)gtab;
            int r = 0;
#define OP(q) { const uint2 v = g2[((r++ & 3) << 5) | (q & 31)]; q ^= v.x ^ v.y; }
            CH8(OP)
#undef OP
        } else if constexpr (K == 4) {
            a0 ^= lt[((a0 & 255) << 5) | lane];
            a1 ^= lt[((a1 & 255) << 5) | lane];
            a2 ^= lt[((a2 & 255) << 5) | lane];
            a3 ^= gtab[a3 & 255];
            a4 ^= lt[((a4 & 255) << 5) | lane];
            a5 ^= lt[((a5 & 255) << 5) | lane];
            a6 ^= lt[((a6 & 255) << 5) | lane];
            a7 ^= gtab[a7 & 255];
        } else if constexpr (K == 6) {
            // LDS, one v_and_or per address: row (x & 0xFF) << 7 | lane * 4
            const uint8_t *lb = (const uint8_t *)lt;
#define OP(x) x ^= *(const uint32_t *)(lb + ((x & 0x7F80u) | (lane << 2)));
            CH8(OP)
#undef OP
        } else if constexpr (K == 7) {
            // 6 LDS + 2 buffer loads (one v_and per address)
            const uint8_t *lb = (const uint8_t *)lt;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)gtab, 0, 1024, 0x00020000);
            a0 ^= *(const uint32_t *)(lb + ((a0 & 0x7F80u) | (lane << 2)));
            a1 ^= *(const uint32_t *)(lb + ((a1 & 0x7F80u) | (lane << 2)));
            a2 ^= *(const uint32_t *)(lb + ((a2 & 0x7F80u) | (lane << 2)));
            a3 ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a3 & 0x3FCu), 0, 0);
            a4 ^= *(const uint32_t *)(lb + ((a4 & 0x7F80u) | (lane << 2)));
            a5 ^= *(const uint32_t *)(lb + ((a5 & 0x7F80u) | (lane << 2)));
            a6 ^= *(const uint32_t *)(lb + ((a6 & 0x7F80u) | (lane << 2)));
            a7 ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a7 & 0x3FCu), 0, 0);
        } else if constexpr (K == 8) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)gtab, 0, 1024, 0x00020000);
#define OP(x) x ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(x & 0x3FCu), 0, 0);
            CH8(OP)
#undef OP
        } else if constexpr (K == 9) {
            // 4 LDS + 4 buffer loads
            const uint8_t *lb = (const uint8_t *)lt;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)gtab, 0, 1024, 0x00020000);
            a0 ^= *(const uint32_t *)(lb + ((a0 & 0x7F80u) | (lane << 2)));
            a1 ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a1 & 0x3FCu), 0, 0);
            a2 ^= *(const uint32_t *)(lb + ((a2 & 0x7F80u) | (lane << 2)));
            a3 ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a3 & 0x3FCu), 0, 0);
            a4 ^= *(const uint32_t *)(lb + ((a4 & 0x7F80u) | (lane << 2)));
            a5 ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a5 & 0x3FCu), 0, 0);
            a6 ^= *(const uint32_t *)(lb + ((a6 & 0x7F80u) | (lane << 2)));
            a7 ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(a7 & 0x3FCu), 0, 0);
        } else if constexpr (K == 5) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)gtab, 0, 1024, 0x00020000);
#define OP(x) x ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)((x & 255) << 2), 0, 0);
            CH8(OP)
#undef OP
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 1024 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
static void run(const char *name, const uint32_t *gtab, uint32_t *out, unsigned long long *cyc, int cus)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_gather<K>, dim3(cus), dim3(1024), 0, 0, gtab, out, cyc, 1u);
    hipEventRecord(e0);
    const int reps = 40;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k_gather<K>, dim3(cus), dim3(1024), 0, 0, gtab, out, cyc, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[1024];
    hipMemcpy(h, cyc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < cus; ++i) avg += (double)h[i];
    avg /= cus;
    // wave instructions per CU per launch: 16 waves x kIters x 8 lookups
    const double winst = 16.0 * kIters * 8;
    const double sec = ms / 1e3 / reps;
    const double ghz = avg / sec / 1e9;
    printf("%-44s %8.3f ms/launch  clock %.2f GHz  %6.2f CU-cycles per wave-instruction  (%.1f G lookups/s chip)\n",
           name, sec * 1e3, ghz, avg / winst, winst * 64 * cus / sec / 1e9);
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *gtab, *out;
    unsigned long long *cyc;
    hipMalloc(&gtab, 16 * 1024 * 4);
    hipMalloc(&out, (size_t)cus * 1024 * 4);
    hipMalloc(&cyc, sizeof(unsigned long long) * cus);
    uint32_t h[16 * 1024];
    for (int i = 0; i < 16 * 1024; ++i) h[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
    hipMemcpy(gtab, h, sizeof h, hipMemcpyHostToDevice);
    run<0>("LDS ds_read_b32 (bank-replicated)", gtab, out, cyc, cus);
    run<1>("global_load_dword, 1 KiB table", gtab, out, cyc, cus);
    run<2>("global_load_dword, 8 KiB (8 rows)", gtab, out, cyc, cus);
    run<3>("global_load_dwordx2, 256 B rows", gtab, out, cyc, cus);
    run<4>("mixed: 6 LDS + 2 global per 8", gtab, out, cyc, cus);
    run<5>("buffer_load_dword, 1 KiB table", gtab, out, cyc, cus);
    for (int rep = 0; rep < 2; ++rep) {
        run<6>("LDS, 2 VALU per lookup", gtab, out, cyc, cus);
        run<8>("buffer_load_dword, 2 VALU per lookup", gtab, out, cyc, cus);
        run<7>("mixed: 6 LDS + 2 buffer per 8", gtab, out, cyc, cus);
        run<9>("mixed: 4 LDS + 4 buffer per 8", gtab, out, cyc, cus);
    }
    return 0;
}
