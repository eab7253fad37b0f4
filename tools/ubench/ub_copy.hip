// Design microbenchmark (gfx950), not part of the product: the streaming
// copy bench.py divides by (csrc/hh_probe.hip), over the same byte count,
// by workgroup size, elements in flight per lane, workgroups per CU, grid
// shape (a grid-stride loop, or one element group per thread with no loop)
// and cache policy.  GB/s = (bytes read + bytes written) / time, best of 5.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/ub_copy tools/ubench/ub_copy.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int TB, int UNR, int CPOL>
__global__ __launch_bounds__(TB) void k_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t n) {
    const uint64_t step = (uint64_t)gridDim.x * TB * UNR;
    uint64_t i = (uint64_t)blockIdx.x * TB * UNR + threadIdx.x;
    for (; i + (UNR - 1) * TB < n; i += step) {
        u32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) v[u] = CPOL ? __builtin_nontemporal_load(src + i + u * TB) : src[i + u * TB];
#pragma unroll
        for (int u = 0; u < UNR; u++) {
            if (CPOL) __builtin_nontemporal_store(v[u], dst + i + u * TB);
            else dst[i + u * TB] = v[u];
        }
    }
    for (; i < n; i += TB) dst[i] = src[i];
}

template <int TB, int UNR, int CPOL>
static void run(const u32x4 *s, u32x4 *d, uint64_t n, int ncu, int wpc) {
    const uint64_t want = (n + (uint64_t)TB * UNR - 1) / ((uint64_t)TB * UNR);
    const uint64_t grid = wpc > 0 ? (uint64_t)ncu * wpc : want;   // wpc 0: no grid-stride loop
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 6; rep++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_copy<TB, UNR, CPOL>), dim3((unsigned)(grid < want ? grid : want)), dim3(TB), 0, 0, s, d, n);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep && ms < best) best = ms;
    }
    printf("tb %4d unr %d cpol %d wg/cu %2d: %.4f ms  %.1f GB/s\n", TB, UNR, CPOL, wpc, best, 2.0 * n * 16 / (best * 1e6));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
    const uint64_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : 1498497040ull;   // bench.py's (C + D) / 2
    const uint64_t n = bytes / 16;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    u32x4 *s, *d;
    CK(hipMalloc(&s, n * 16));
    CK(hipMalloc(&d, n * 16));
    CK(hipMemset(s, 1, n * 16));
    CK(hipMemset(d, 0, n * 16));
    const int W[] = {2, 4, 8, 16, 0};
    for (int w : W) run<256, 4, 0>(s, d, n, ncu, w);
    for (int w : W) run<256, 4, 2>(s, d, n, ncu, w);
    for (int w : W) run<256, 8, 2>(s, d, n, ncu, w);
    for (int w : W) run<256, 2, 2>(s, d, n, ncu, w);
    for (int w : W) run<512, 4, 2>(s, d, n, ncu, w);
    for (int w : W) run<1024, 4, 2>(s, d, n, ncu, w);
    for (int w : W) run<256, 1, 2>(s, d, n, ncu, w);
    return 0;
}
