// Design microbenchmark (gfx950), not part of the product: writing a wave's
// output when each lane holds its own run of bytes (40..75 B, contiguous
// runs, lane j's after lane j-1's), 3.6 KB per wave-tile, to HBM:
//   mode 0: each lane stores its run with unaligned 16-B stores, the tail
//           with 8/4/2/1-B stores (global addresses at any byte)
//   mode 1: the same bytes as 16-B aligned, wave-coalesced stores (the
//           staged copy-out: the floor)
// Build: hipcc -O3 --offload-arch=gfx950 -o build/ub_runstore tools/ubench/ub_runstore.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_store(uint8_t *out, uint32_t tiles, uint32_t tile_bytes) {
    const uint32_t j = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6), gw = blockIdx.x * (blockDim.x >> 6) + wv;
    for (uint32_t t = 0; t < tiles; t++) {
        const uint64_t tile = t * nw + gw;
        uint8_t *base = out + tile * tile_bytes + (hash((uint32_t)tile) & 15u);
        // run lengths: about tile_bytes / 64 each
        const uint32_t n = tile_bytes / 64 - 16 + (hash((uint32_t)tile * 64 + j) & 15u);
        uint32_t L = n;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(L, o, 64);
            if (j >= (uint32_t)o) L += y;
        }
        L -= n;
        const u32x4 v = {j, t, n, L};
        if (MODE == 0) {
            uint8_t *p = base + L;
            uint32_t i = 0;
            for (; i + 16 <= n; i += 16) *(u32x4 __attribute__((aligned(1))) *)(p + i) = v;
            if (n - i >= 8) { *(u32x2 __attribute__((aligned(1))) *)(p + i) = v.xy; i += 8; }
            if (n - i >= 4) { *(uint32_t __attribute__((aligned(1))) *)(p + i) = v.x; i += 4; }
            if (n - i >= 2) { *(uint16_t __attribute__((aligned(1))) *)(p + i) = (uint16_t)v.y; i += 2; }
            if (n - i >= 1) p[i] = (uint8_t)v.z;
        } else {
            const uint32_t tot = __shfl(L + n, 63, 64);
            u32x4 *q = (u32x4 *)(out + tile * tile_bytes);
            for (uint32_t i = j; i < tot / 16; i += 64) __builtin_nontemporal_store(v, q + i);
        }
    }
}

int main(int argc, char **argv) {
    const uint32_t tiles = argc > 1 ? atoi(argv[1]) : 64;
    const uint32_t tb = 3840;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t waves = 16;
    const uint64_t ntile = (uint64_t)ncu * waves * tiles;
    uint8_t *out;
    CK(hipMalloc(&out, ntile * tb + 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    void (*ks[2])(uint8_t *, uint32_t, uint32_t) = {k_store<0>, k_store<1>};
    for (int m = 0; m < 2; m++) {
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(ks[m], dim3(ncu), dim3(64 * waves), 0, 0, out, tiles, tb);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep == 2)
                printf("mode %d: %.3f ms for %.2f GB: %.0f GB/s; 1.92 GB of output -> %.3f ms\n", m, ms, ntile * tb * 1e-9,
                       ntile * tb / ms / 1e6, ms * 1.923e9 / (ntile * tb));
        }
    }
    return 0;
}
