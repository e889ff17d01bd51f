// VALU issue cost per instruction kind on gfx950 (ChaCha20 / Poly1305 building
// blocks): every lane runs 8 independent chains of one instruction, 16 waves
// per CU; reported as cycles per wave-instruction per SIMD at the measured
// clock (s_memtime over the loop).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb_valu tools/mb_valu.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kIters = 4096;

#define CHAINS8(OP)                                                                        \
    OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

template <int K>
__global__ __launch_bounds__(1024) void k_valu(uint32_t *out, uint64_t *cyc, uint32_t seed)
{
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
             a6 = a0 * 13, a7 = a0 * 15;
    uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3;
    const uint32_t b = seed | 1;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
        if constexpr (K == 0) {  // v_add_u32
#define OP(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
            CHAINS8(OP)
#undef OP
        } else if constexpr (K == 1) {  // v_xor_b32
#define OP(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
            CHAINS8(OP)
#undef OP
        } else if constexpr (K == 2) {  // v_alignbit_b32 (rotate)
#define OP(x) asm volatile("v_alignbit_b32 %0, %0, %0, 12" : "+v"(x));
            CHAINS8(OP)
#undef OP
        } else if constexpr (K == 3) {  // v_perm_b32 (byte rotate)
#define OP(x) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x) : "s"(0x01000302u));
            CHAINS8(OP)
#undef OP
        } else if constexpr (K == 4) {  // v_bitop3_b32
#define OP(x) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(x) : "v"(b));
            CHAINS8(OP)
#undef OP
        } else if constexpr (K == 5) {  // v_mad_u64_u32 (4 chains, 64-bit accumulators)
#define OP64(w, x) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w) : "v"(x), "v"(b) : "vcc");
            OP64(w0, a0) OP64(w1, a1) OP64(w2, a2) OP64(w3, a3) OP64(w0, a4) OP64(w1, a5) OP64(w2, a6) OP64(w3, a7)
#undef OP64
        } else if constexpr (K == 6) {  // v_mul_lo_u32
#define OP(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
            CHAINS8(OP)
#undef OP
        } else if constexpr (K == 7) {  // v_lshl_add_u64
#define OP64(w) asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(w));
            OP64(w0) OP64(w1) OP64(w2) OP64(w3) OP64(w0) OP64(w1) OP64(w2) OP64(w3)
#undef OP64
        } else if constexpr (K == 8) {  // v_add3_u32
#define OP(x) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x) : "v"(b));
            CHAINS8(OP)
#undef OP
        } else if constexpr (K == 9) {  // v_pk_add_u16 (no use for 32-bit lanes; reference point)
#define OP(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(b));
            CHAINS8(OP)
#undef OP
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(w0 ^ w1 ^ w2 ^ w3);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
static void run(const char *name, int cus, uint32_t *d_out, uint64_t *d_cyc)
{
    hipLaunchKernelGGL(k_valu<K>, dim3(cus), dim3(1024), 0, 0, d_out, d_cyc, 7u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_valu<K>, dim3(cus), dim3(1024), 0, 0, d_out, d_cyc, 9u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t cyc = 0;
    hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
    // 4 waves per SIMD, 8 instructions per iteration each
    const double insts = 4.0 * 8.0 * kIters;
    printf("%-16s %8.3f ms  %7.2f cycles per wave-instruction per SIMD (s_memtime %llu, %.0f MHz)\n", name,
           ms, cyc / insts, (unsigned long long)cyc, cyc / (ms * 1e3));
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *d_out;
    uint64_t *d_cyc;
    hipMalloc(&d_out, (size_t)cus * 1024 * 4);
    hipMalloc(&d_cyc, (size_t)cus * 8);
    run<0>("v_add_u32", cus, d_out, d_cyc);
    run<1>("v_xor_b32", cus, d_out, d_cyc);
    run<2>("v_alignbit_b32", cus, d_out, d_cyc);
    run<3>("v_perm_b32", cus, d_out, d_cyc);
    run<4>("v_bitop3_b32", cus, d_out, d_cyc);
    run<5>("v_mad_u64_u32", cus, d_out, d_cyc);
    run<6>("v_mul_lo_u32", cus, d_out, d_cyc);
    run<7>("v_lshl_add_u64", cus, d_out, d_cyc);
    run<8>("v_add3_u32", cus, d_out, d_cyc);
    run<9>("v_pk_add_u16", cus, d_out, d_cyc);
    return 0;
}
