// HBM write bytes of the GCM kernel's output pattern:
// does a quad's 128-byte step that straddles two 128-byte lines cost extra
// WRITE_SIZE, and does 16-byte or 128-byte alignment of the stores fix it?
// Each "packet" is 1200 B at a stride of 1200 B; its 1189 output bytes start
// at byte OFF of the packet.  Lane j of the packet's quad writes the 16-byte
// blocks 8k + j and 8k + 4 + j at step k (two buffer stores, the engine's
// BPL = 2 form), 16 packets per wave, persistent-free grid.
//   K = 0: blocks at OFF + 16 b          (engine today: OFF = 11)
//   K = 1: blocks at the 16-aligned grid (OFF rounded up; the funnel-shifted form)
//   K = 2: as 1, and the step boundaries on 128-byte lines (front-padded)
//   K = 3, 4: K = 0, 2 with the engine's pacing: 16 waves per CU (LDS-capped)
//             and ~8 us between a quad's steps, so ~10 MB of packets per XCD
//             are in flight, as in the persistent GCM kernel at 1 Mi
// Run under rocprofv3 --pmc WRITE_SIZE; prints ms per launch.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb_store tools/mb_store.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kPkt = 1200, kOut = 1189, kOff = 11;
constexpr uint32_t kOob = 0x80000000u;

template <int K>
__global__ __launch_bounds__(256) void k_store(uint8_t *out, int n)
{
    extern __shared__ uint32_t pad_lds[];  // occupancy cap for K >= 3
    const int gid = blockIdx.x * 256 + threadIdx.x;
    const int p = gid >> 2, j = gid & 3;
    if (p >= n) return;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(out + (size_t)p * kPkt, 0, kPkt, 0x00020000);
    const uintptr_t base = (uintptr_t)(out + (size_t)p * kPkt);
    int lo = kOff, first = kOff;  // first byte written; block grid origin
    if (K == 1 || K == 2 || K == 4) first = (int)(((base + kOff + 15) & ~(uintptr_t)15) - base) - 16;
    if (K == 2 || K == 4) first = (int)(((base + kOff) & ~(uintptr_t)127) - base);
    const int hi = kOff + kOut;
    const u32x4 v = {0x01010101u * (uint32_t)p, 2u, 3u, (uint32_t)gid};
    for (int s = first; s < hi; s += 128) {
        if (K >= 3) {
            __builtin_amdgcn_s_sleep(127);
            __builtin_amdgcn_s_sleep(127);
            if (v.w == 0xffffffffu) pad_lds[threadIdx.x] = s;  // keep the LDS allocation
        }
        for (int h = 0; h < 2; ++h) {
            const int b = s + 16 * (j + 4 * h);
            // blocks wholly inside [lo, hi) go out with one store; partial
            // edge blocks are dropped (the engine writes them apart)
            const uint32_t o = (b >= lo && b + 16 <= hi) ? (uint32_t)b : kOob;
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)o, 0, 0);
        }
    }
}

template <int K>
static void run(const char *name, uint8_t *out, int n)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = (4 * n + 255) / 256;
    const size_t lds = K >= 3 ? 36 * 1024 : 0;  // 4 workgroups (16 waves) per CU
    hipLaunchKernelGGL(k_store<K>, dim3(grid), dim3(256), lds, 0, out, n);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_store<K>, dim3(grid), dim3(256), lds, 0, out, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-52s %8.3f ms/launch  %.1f GB/s of %.0f MB\n", name, ms / reps,
           (double)n * kOut / (ms / reps * 1e-3) / 1e9, (double)n * kOut / 1e6);
}

int main()
{
    const int n = 1 << 20;
    uint8_t *out;
    hipMalloc(&out, (size_t)n * kPkt + 256);
    run<0>("K0: 16-B stores at payload offset 11", out, n);
    run<1>("K1: 16-B stores on the 16-B grid", out, n);
    run<2>("K2: 16-B grid, steps on 128-B lines", out, n);
    run<3>("K3: as K0, engine pacing", out, n);
    run<4>("K4: as K2, engine pacing", out, n);
    hipFree(out);
    return 0;
}
