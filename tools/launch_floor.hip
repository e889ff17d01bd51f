// Floor of one kernel launch + stream synchronisation on the box (the part of
// a per-call object-API round trip that no kernel change removes):
// an empty kernel, and a one-wave kernel writing 16 bytes to pinned host
// memory, each launched and synchronised 2000 times.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_touch(uint32_t *h) { if (threadIdx.x < 4) h[threadIdx.x] = threadIdx.x; }

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main()
{
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *h = nullptr, *dh = nullptr;
    CHK(hipHostMalloc((void **)&h, 4096, hipHostMallocMapped));
    CHK(hipHostGetDevicePointer((void **)&dh, h, 0));
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            const int n = rep == 0 ? 200 : 2000;
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; ++i) {
                if (mode == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                else hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, dh);
                CHK(hipGetLastError());
                CHK(hipStreamSynchronize(s));
            }
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
            if (rep == 1) printf("%s launch + sync: %.2f us\n", mode == 0 ? "empty kernel" : "pinned-write kernel", us);
        }
    }
    CHK(hipHostFree(h));
    CHK(hipStreamDestroy(s));
    return 0;
}
