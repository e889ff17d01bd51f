// Host copy bandwidth, memcpy against non-temporal AVX2 stores, 1200 MB in 4 MiB parts over T threads
// (round 5 host-path study): gcc -O2 -pthread -o tools/ntbench tools/ntbench.c; tools/ntbench T
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
static size_t N = (size_t)1200 << 20;
static uint8_t *A, *B;
static int mode, T;
__attribute__((target("avx2"))) static void nt(uint8_t *d, const uint8_t *s, size_t n) {
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    __m256i a = _mm256_loadu_si256((const __m256i *)(s + i)), b = _mm256_loadu_si256((const __m256i *)(s + i + 32)),
            c = _mm256_loadu_si256((const __m256i *)(s + i + 64)), e = _mm256_loadu_si256((const __m256i *)(s + i + 96));
    _mm256_stream_si256((__m256i *)(d + i), a); _mm256_stream_si256((__m256i *)(d + i + 32), b);
    _mm256_stream_si256((__m256i *)(d + i + 64), c); _mm256_stream_si256((__m256i *)(d + i + 96), e);
  }
  memcpy(d + i, s + i, n - i); _mm_sfence();
}
static void *run(void *arg) {
  long t = (long)arg; size_t part = N / T, lo = t * part;
  for (size_t o = lo; o < lo + part; o += 4 << 20) {
    size_t n = (o + (4 << 20) <= lo + part) ? (4 << 20) : lo + part - o;
    if (mode) nt(B + o, A + o, n); else memcpy(B + o, A + o, n);
  }
  return 0;
}
int main(int argc, char **argv) {
  T = atoi(argv[1]);
  A = aligned_alloc(4096, N); B = aligned_alloc(4096, N);
  memset(A, 1, N); memset(B, 2, N);
  for (int rep = 0; rep < 6; ++rep) {
    mode = rep & 1;
    struct timespec t0, t1; clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_t th[64];
    for (long t = 0; t < T; ++t) pthread_create(&th[t], 0, run, (void *)t);
    for (int t = 0; t < T; ++t) pthread_join(th[t], 0);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double s = (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
    printf("threads %d %s %.1f GB/s\n", T, mode ? "nt" : "memcpy", N / s / 1e9);
  }
}
