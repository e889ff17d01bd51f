// Issue cost of the VALU forms ChaCha20 / Poly1305 can use on gfx950: every
// lane runs 8 independent chains of one instruction, 16 waves per CU (4 per
// SIMD); ns per wave-instruction per SIMD from events over 5 launches, and the
// ratio to v_add_u32 (VOP2), which issues in 2 cycles.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb_valu2 tools/mb_valu2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 8192;
#define CH8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

template <int K>
__global__ __launch_bounds__(1024) void k_v(uint32_t *out, uint32_t seed)
{
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11,
             a6 = a0 * 13, a7 = a0 * 15;
    uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3;
    const uint32_t b = seed | 1, c = seed * 7;
    for (int i = 0; i < kIters; ++i) {
        if constexpr (K == 0) {
#define OP(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 1) {
#define OP(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 2) {
#define OP(x) asm volatile("v_alignbit_b32 %0, %0, %0, 12" : "+v"(x));
            CH8(OP)
#undef OP
        } else if constexpr (K == 3) {
#define OP(x) asm volatile("v_alignbit_b32 %0, %0, %1, 12" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 4) {
#define OP(x) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 5) {
#define OP(x) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
            CH8(OP)
#undef OP
        } else if constexpr (K == 6) {
#define OP(x) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x));
            CH8(OP)
#undef OP
        } else if constexpr (K == 7) {
#define OP(x) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 8) {
#define OP64(w, x) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w) : "v"(x), "v"(b) : "vcc");
            OP64(w0, a0) OP64(w1, a1) OP64(w2, a2) OP64(w3, a3) OP64(w0, a4) OP64(w1, a5) OP64(w2, a6) OP64(w3, a7)
#undef OP64
        } else if constexpr (K == 9) {
#define OP(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
            CH8(OP)
#undef OP
        } else if constexpr (K == 10) {
#define OP(x) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 11) {
#define OP(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 12) {
#define OP(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
            CH8(OP)
#undef OP
        } else if constexpr (K == 13) {
#define OP64(w) asm volatile("v_lshrrev_b64 %0, 26, %0" : "+v"(w));
            OP64(w0) OP64(w1) OP64(w2) OP64(w3) OP64(w0) OP64(w1) OP64(w2) OP64(w3)
#undef OP64
        } else if constexpr (K == 14) {
            // dependent chain: one chain of 8 (latency, not throughput)
#define OP(x) asm volatile("v_alignbit_b32 %0, %0, %0, 12" : "+v"(a0));
            CH8(OP)
#undef OP
        } else if constexpr (K == 15) {
#define OP(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
            CH8(OP)
#undef OP
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(w0 ^ w1 ^ w2 ^ w3);
}

static double base_ns = 0;
template <int K>
static void run(const char *name, int cus, uint32_t *d)
{
    hipLaunchKernelGGL(k_v<K>, dim3(cus), dim3(1024), 0, 0, d, 7u);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_v<K>, dim3(cus), dim3(1024), 0, 0, d, 9u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double ns = ms * 1e6 / 5 / (4.0 * 8 * kIters);  // per wave-instruction per SIMD
    if (K == 0) base_ns = ns;
    printf("%-40s %7.3f ns per wave-instruction per SIMD  x%.2f of v_add_u32 (2 cycles)\n", name, ns, ns / base_ns);
}

int main()
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *d;
    (void)hipMalloc(&d, (size_t)cus * 1024 * 4);
    run<0>("v_add_u32 (VOP2)", cus, d);
    run<11>("v_xor_b32 (VOP2)", cus, d);
    run<6>("v_lshrrev_b32 (VOP2)", cus, d);
    run<12>("v_mul_u32_u24 (VOP2)", cus, d);
    run<1>("v_add_u32_e64 (VOP3 encoding)", cus, d);
    run<2>("v_alignbit_b32 x,x,x (rotate)", cus, d);
    run<3>("v_alignbit_b32 x,y (funnel)", cus, d);
    run<10>("v_perm_b32", cus, d);
    run<9>("v_bitop3_b32 (3 sources)", cus, d);
    run<5>("v_xad_u32", cus, d);
    run<7>("v_lshl_or_b32", cus, d);
    run<4>("v_xor_b32_sdwa (word select)", cus, d);
    run<8>("v_mad_u64_u32", cus, d);
    run<13>("v_lshrrev_b64", cus, d);
    run<14>("v_alignbit_b32, one dependent chain", cus, d);
    run<15>("v_add_u32, one dependent chain", cus, d);
    return 0;
}
