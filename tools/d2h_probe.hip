// D2H / H2D rates into hipHostMalloc'd pinned memory, as the session's
// pipeline uses them (one 1.26 GB buffer, whole and in 36 chunks, alone and
// with H2D on a second stream at the same time).  Round-6 host-path study.
//   hipcc --offload-arch=gfx950 -O3 -o tools/d2h_probe tools/d2h_probe.hip
//   tools/d2h_probe [flags_hex]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>
#include <chrono>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

// NUMA node of the page holding p (get_mempolicy, MPOL_F_NODE | MPOL_F_ADDR)
static int page_node(const void *p)
{
    int node = -1;
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, 3UL) != 0) return -1;
    return node;
}

static int gpu_numa_node()
{
    char bus[64] = {}, path[160];
    if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) != hipSuccess) return -2;
    for (char *c = bus; *c; ++c) *c = (char)tolower(*c);
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE *f = fopen(path, "r");
    int n = -3;
    if (f) {
        if (fscanf(f, "%d", &n) != 1) n = -4;
        fclose(f);
    }
    printf("gpu %s numa_node %d\n", bus, n);
    return n;
}

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// D2H by our own kernel: 16-byte loads from device memory, 16-byte stores
// through the host buffer's device view (posted PCIe writes)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy16(const v4u *__restrict__ src, v4u *dst, size_t n16)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(src[i], &dst[i]);
}

int main(int argc, char **argv)
{
    const unsigned flags = argc > 1 ? (unsigned)strtoul(argv[1], nullptr, 16) : 0u;
    const size_t n = (size_t)1 << 20, bytes = n * 1200;
    uint8_t *h_in, *h_out, *d_in, *d_out;
    if (hipHostMalloc(&h_in, bytes, flags) != hipSuccess || hipHostMalloc(&h_out, bytes, flags) != hipSuccess ||
        hipMalloc(&d_in, bytes) != hipSuccess || hipMalloc(&d_out, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    memset(h_in, 1, bytes);
    memset(h_out, 2, bytes);
    gpu_numa_node();
    printf("main thread cpu %d; h_out pages on nodes %d %d %d, h_in %d %d\n", sched_getcpu(), page_node(h_out),
           page_node(h_out + bytes / 2), page_node(h_out + bytes - 4096), page_node(h_in), page_node(h_in + bytes / 2));
    (void)hipMemset(d_out, 3, bytes);
    hipStream_t a, b;
    (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    const int chunks = 36;
    const size_t cb = bytes / chunks;
    for (int rep = 0; rep < 3; ++rep) {
        double t0 = now_ms();
        (void)hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, a);
        (void)hipStreamSynchronize(a);
        double t1 = now_ms();
        for (int c = 0; c < chunks; ++c)
            (void)hipMemcpyAsync(h_out + c * cb, d_out + c * cb, cb, hipMemcpyDeviceToHost, a);
        (void)hipStreamSynchronize(a);
        double t2 = now_ms();
        (void)hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, b);
        (void)hipStreamSynchronize(b);
        double t3 = now_ms();
        for (int c = 0; c < chunks; ++c) {
            (void)hipMemcpyAsync(d_in + c * cb, h_in + c * cb, cb, hipMemcpyHostToDevice, b);
            (void)hipMemcpyAsync(h_out + c * cb, d_out + c * cb, cb, hipMemcpyDeviceToHost, a);
        }
        (void)hipStreamSynchronize(a);
        double t4 = now_ms();
        (void)hipStreamSynchronize(b);
        double t5 = now_ms();
        const double g = bytes / 1e6;
        uint8_t *hd_out = nullptr;
        (void)hipHostGetDevicePointer((void **)&hd_out, h_out, 0);
        double t6 = now_ms();
        hipLaunchKernelGGL(k_copy16, dim3(2048), dim3(256), 0, a, (const v4u *)d_out, (v4u *)hd_out, bytes / 16);
        (void)hipStreamSynchronize(a);
        double t7 = now_ms();
        (void)hipMemcpyAsync(hd_out, d_out, bytes, hipMemcpyDeviceToDeviceNoCU, a);
        (void)hipStreamSynchronize(a);
        double t8 = now_ms();
        printf("  own kernel d2h %.1f GB/s, sdma (DeviceToDeviceNoCU) d2h %.1f GB/s\n", bytes / 1e6 / (t7 - t6),
               bytes / 1e6 / (t8 - t7));
        printf("flags %#x rep %d: d2h whole %.1f GB/s, d2h 36 chunks %.1f GB/s, h2d whole %.1f GB/s, duplex 36 chunks d2h %.1f h2d %.1f GB/s\n",
               flags, rep, g / (t1 - t0), g / (t2 - t1), g / (t3 - t2), g / (t4 - t3), g / (t5 - t3));
    }
    return 0;
}
