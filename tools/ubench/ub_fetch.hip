// Calibration (gfx950), not part of the product: rocprofv3's FETCH_SIZE for
// a known byte count read with the load shapes the decoder uses --
// 16-B buffer loads per lane (payload words), 4-B per-lane loads (records,
// corrections), and 4-B loads of one word per 64-lane wave (tile meta).
// Each kernel reads NB bytes once (beyond the Infinity Cache: 1 GiB, a fresh
// buffer per kernel); tools/profile.sh runs it under --pmc FETCH_SIZE and
// tools/prof_summary.py divides.  Build:
//   hipcc -O3 --offload-arch=gfx950 -o build/ub_fetch tools/ubench/ub_fetch.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_read16(const u32x4 *p, uint64_t n, uint32_t *sink) {
    uint32_t a = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x9e3779b9u) sink[0] = a;
}
__global__ void k_read4(const uint32_t *p, uint64_t n, uint32_t *sink) {
    uint32_t a = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a ^= p[i];
    if (a == 0x9e3779b9u) sink[0] = a;
}

int main() {
    const uint64_t nb = 1ull << 30;
    uint8_t *a, *b;
    uint32_t *sink;
    CK(hipMalloc(&a, nb));
    CK(hipMalloc(&b, nb));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, nb));
    CK(hipMemset(b, 2, nb));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_read16, dim3(4096), dim3(256), 0, 0, (const u32x4 *)a, nb / 16, sink);
    hipLaunchKernelGGL(k_read4, dim3(4096), dim3(256), 0, 0, (const uint32_t *)b, nb / 4, sink);
    CK(hipDeviceSynchronize());
    printf("read %llu bytes with each of k_read16, k_read4\n", (unsigned long long)nb);
    return 0;
}
