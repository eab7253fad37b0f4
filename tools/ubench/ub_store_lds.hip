// Design microbenchmarks for the decode kernel (gfx950), not part of the
// product.  Answers two questions before the kernel layout is fixed:
//   (1) store shape: per-lane contiguous runs written as 16-B (or 4-B)
//       chunks, 64 distinct runs per wave-instruction, vs wave-coalesced
//       1-KiB stores of the same bytes;
//   (2) the dependent LDS lookup chain (two bitstream words + one u64 table
//       entry per step) that every decode loop is built on: steps/s chip-wide
//       at 1..8 waves per SIMD and with 1 or 2 independent chains per lane.
// Build: hipcc -O3 --offload-arch=gfx950 -o ub tools/ubench/ub_store_lds.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

// each lane writes run bytes at lane*run, in 16-B chunks
__global__ void k_scatter16(uint4 *out, uint32_t run16, uint64_t nlanes) {
    uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (l >= nlanes) return;
    uint4 *p = out + l * run16;
    for (uint32_t i = 0; i < run16; i++) p[i] = make_uint4(i, l, i ^ 7, 3);
}
__global__ void k_scatter4(uint32_t *out, uint32_t run4, uint64_t nlanes) {
    uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (l >= nlanes) return;
    uint32_t *p = out + l * run4;
    for (uint32_t i = 0; i < run4; i++) p[i] = i ^ (uint32_t)l;
}
// same bytes, each block writes its lanes' runs wave-contiguously
__global__ void k_coal16(uint4 *out, uint32_t run16, uint64_t nlanes) {
    uint64_t b0 = blockIdx.x * (uint64_t)blockDim.x * run16;
    uint64_t tot = (uint64_t)blockDim.x * run16;
    uint64_t lim = nlanes * run16;
    for (uint64_t i = threadIdx.x; i < tot; i += blockDim.x)
        if (b0 + i < lim) out[b0 + i] = make_uint4(i, b0, 1, 3);
}

__global__ __launch_bounds__(256) void k_chain(const uint32_t *g, const uint64_t *glut, uint32_t steps,
                                               uint32_t *sink, int two) {
    extern __shared__ uint32_t dyn[];
    __shared__ uint64_t lut[2048];
    __shared__ uint32_t w[2304];
    for (int i = threadIdx.x; i < 2048; i += 256) lut[i] = glut[i];
    for (int i = threadIdx.x; i < 2304; i += 256) w[i] = g[(blockIdx.x * 64 + i) & 65535];
    if (threadIdx.x == 0) dyn[0] = 0;
    __syncthreads();
    uint32_t p = threadIdx.x * 256, q2 = threadIdx.x * 256 + 128, n = 0, n2 = 0;
    for (uint32_t s = 0; s < steps; s++) {
        uint32_t i = p >> 5;
        uint32_t win = __builtin_amdgcn_alignbit(w[(i + 1) % 2300], w[i % 2300], p & 31);
        uint64_t e = lut[win & 2047];
        p += (uint32_t)(e >> 32) & 15;
        n += (uint32_t)(e >> 40) & 7;
        if (two) {
            uint32_t j = q2 >> 5;
            uint32_t win2 = __builtin_amdgcn_alignbit(w[(j + 1) % 2300], w[j % 2300], q2 & 31);
            uint64_t e2 = lut[win2 & 2047];
            q2 += (uint32_t)(e2 >> 32) & 15;
            n2 += (uint32_t)(e2 >> 40) & 7;
        }
    }
    if (n + n2 == 0xdeadbeef) sink[0] = p + q2;
}

int main() {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const uint64_t bytes = 2ull << 30;
    void *out;
    CK(hipMalloc(&out, bytes + 4096));
    float ms;
    for (uint32_t run : {64u, 256u, 1024u}) {
        uint64_t nl = bytes / run;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_scatter16, dim3((nl + 255) / 256), dim3(256), 0, 0, (uint4 *)out, run / 16, nl);
            CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        }
        printf("scatter16 run=%4u B: %.3f ms  %.0f GB/s\n", run, ms, bytes / ms / 1e6);
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_scatter4, dim3((nl + 255) / 256), dim3(256), 0, 0, (uint32_t *)out, run / 4, nl);
            CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        }
        printf("scatter4  run=%4u B: %.3f ms  %.0f GB/s\n", run, ms, bytes / ms / 1e6);
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_coal16, dim3((nl + 255) / 256), dim3(256), 0, 0, (uint4 *)out, run / 16, nl);
            CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        }
        printf("coal16    run=%4u B: %.3f ms  %.0f GB/s\n", run, ms, bytes / ms / 1e6);
    }
    // chain
    uint32_t *g; uint64_t *glut; uint32_t *sink;
    CK(hipMalloc(&g, 65536 * 4)); CK(hipMalloc(&glut, 2048 * 8)); CK(hipMalloc(&sink, 64));
    uint32_t *hg = (uint32_t *)malloc(65536 * 4); uint64_t *hl = (uint64_t *)malloc(2048 * 8);
    srand(1);
    for (int i = 0; i < 65536; i++) hg[i] = (uint32_t)rand() * 2654435761u;
    for (int i = 0; i < 2048; i++) hl[i] = ((uint64_t)(3 + rand() % 9) << 32) | ((uint64_t)(1 + rand() % 3) << 40);
    CK(hipMemcpy(g, hg, 65536 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(glut, hl, 2048 * 8, hipMemcpyHostToDevice));
    const uint32_t steps = 4096;
    for (int two = 0; two < 2; two++) {
        for (int wps : {1, 2, 4, 6, 8}) {   // 256-thread blocks: wps blocks per CU = wps waves/SIMD
            size_t dyn = (160 * 1024) / wps - 2048 * 8 - 2304 * 4 - 256;
            int per = 0;
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_chain, 256, dyn));
            uint32_t grid = 256 * per;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(k_chain, dim3(grid), dim3(256), dyn, 0, g, glut, steps, sink, two);
                CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
            }
            double lsteps = (double)grid * 256 * steps * (two ? 2 : 1);
            printf("chain chains/lane=%d blocks/CU=%d: %.3f ms  %.2f Glookups/s  (%.1f cyc/step/lane @2.4GHz)\n",
                   two + 1, per, ms, lsteps / ms / 1e6, ms * 1e-3 * 2.4e9 / steps);
        }
    }
    return 0;
}
