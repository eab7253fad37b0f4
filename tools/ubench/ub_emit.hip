// Design microbenchmark for the emission step of k_emf (gfx950), not part of
// the product: a lane runs the state machine over a 256-bit region held in
// registers in K = 7-bit steps of a u64 table in LDS (74 states x 128
// entries, as kjv), storing each step's symbols into the wave's LDS staging
// at its run's offset.  Store strategies:
//   mode 0: reads only (the chain of table lookups alone)
//   mode 1: the kernel's aligned-dword store with shift/spill every step
//   mode 2: one unaligned 4-byte store at the run's byte offset every step
//   mode 3: as 2, u64 accumulation, a store every second step
//   mode 4: mode 1 with the store exec-masked to full dwords
//   mode 6: pairs of steps, two dwords stored per pair (ds_write2_b32)
//   mode 7: mode 1's stores into lane-private columns (conflict-free)
// Tiles per wave and waves per workgroup are arguments; one workgroup per CU.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/ub_emit tools/ubench/ub_emit.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define NS 74
#define K 7

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_emit(const uint64_t *gt, uint32_t tiles, uint32_t *sink, uint32_t obw) {
    extern __shared__ __align__(16) uint8_t smem[];
    const uint32_t tid = threadIdx.x, j = tid & 63u, wv = tid >> 6;
    for (uint32_t i = tid; i < NS * 128; i += blockDim.x) ((uint64_t *)smem)[i] = gt[i];
    __syncthreads();
    const uint32_t tab = NS * 128 * 8;
    uint32_t acc = 0;
    for (uint32_t t = 0; t < tiles; t++) {
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = hash(((blockIdx.x * 64 + wv) * 4096 + t) * 512 + j * 8 + k);
        uint32_t row = (w[0] % NS) << (K + 3);
        const uint32_t base = tab + wv * obw + j * 57;
        uint32_t o = base, wd = base & ~3u, sh = (base & 3u) * 8u, a = 0;
        uint32_t cw = tab + wv * obw + j * 4;
        if (MODE == 7) sh = 0;
        uint64_t a64 = 0;
        uint32_t sh64 = 0;
#pragma unroll
        for (uint32_t k = 0; k < 256 / K; k++) {
            const uint32_t q = k * K, i = q >> 5, b = q & 31;
            const uint32_t win = (b + K <= 32 || i + 1 >= 8) ? (w[i] >> b) : __builtin_amdgcn_alignbit(w[i + 1], w[i], b);
            const uint64_t e = *(const uint64_t *)(smem + row + ((win & 127u) << 3));
            const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
            row = hi >> 15;
            if (MODE == 0) {
                acc += lo;
            } else if (MODE == 1) {
                const uint32_t u = sh + (hi & 255u);
                const uint32_t an = (lo << sh) | a;
                const uint32_t sp = __builtin_amdgcn_alignbit(0u, lo, (0u - sh) & 31u);
                *(uint32_t *)(smem + wd) = an;
                const bool full = u >= 32;
                a = full ? sp : an;
                wd += full ? 4u : 0u;
                sh = u & 31u;
            } else if (MODE == 2) {
                *(uint32_t __attribute__((aligned(1))) *)(smem + o) = lo;
                o += (hi & 255u) >> 3;
            } else if (MODE == 4) {
                // the dword stored only once it is full (exec-masked store)
                const uint32_t u = sh + (hi & 255u);
                const uint32_t an = (lo << sh) | a;
                const uint32_t sp = __builtin_amdgcn_alignbit(0u, lo, (0u - sh) & 31u);
                const bool full = u >= 32;
                if (full) *(uint32_t *)(smem + wd) = an;
                a = full ? sp : an;
                wd += full ? 4u : 0u;
                sh = u & 31u;
            } else if (MODE == 6) {
                // pairs of steps: the pair's bytes (<= 8) shifted into the
                // open dword; two dwords stored per pair (ds_write2_b32)
                if ((k & 1) == 0) {
                    a64 = lo;
                    sh64 = hi & 255u;
                } else {
                    const uint64_t pb = a64 | ((uint64_t)lo << sh64);   // the pair's bytes
                    const uint32_t nb = sh64 + (hi & 255u);             // their bits
                    const uint32_t p0 = (uint32_t)pb, p1 = (uint32_t)(pb >> 32);
                    const uint32_t v0 = (p0 << sh) | a;
                    const uint32_t v1 = sh ? __builtin_amdgcn_alignbit(p1, p0, 32u - sh) : p1;
                    const uint32_t v2 = sh ? p1 >> (32u - sh) : 0u;
                    uint32_t *q = (uint32_t *)(smem + wd);
                    q[0] = v0;
                    q[1] = v1;
                    const uint32_t u = sh + nb, full = u >> 5;
                    a = full == 0 ? v0 : full == 1 ? v1 : v2;
                    wd += 4u * full;
                    sh = u & 31u;
                }
            } else if (MODE == 7) {
                // mode 1's dword logic in a lane-private column (dword i of
                // lane j at (i * 64 + j) * 4): no bank shared within a group
                const uint32_t u = sh + (hi & 255u);
                const uint32_t an = (lo << sh) | a;
                const uint32_t sp = __builtin_amdgcn_alignbit(0u, lo, (0u - sh) & 31u);
                *(uint32_t *)(smem + cw) = an;
                const bool full = u >= 32;
                a = full ? sp : an;
                cw += full ? 256u : 0u;
                sh = u & 31u;
            } else if (MODE == 5) {
                // 64-bit accumulator, a dword stored when 4 bytes are ready
                a64 |= (uint64_t)lo << sh64;
                sh64 += hi & 255u;
                const bool full = sh64 >= 32;
                if (full) *(uint32_t *)(smem + wd) = (uint32_t)a64;
                a64 = full ? a64 >> 32 : a64;
                sh64 = full ? sh64 - 32 : sh64;
                wd += full ? 4u : 0u;
            } else {
                a64 |= (uint64_t)lo << sh64;
                sh64 += hi & 255u;
                if (k & 1) {
                    *(uint64_t __attribute__((aligned(1))) *)(smem + o) = a64;
                    o += sh64 >> 3;
                    a64 = 0;
                    sh64 = 0;
                }
            }
        }
        acc += a + o + wd + (uint32_t)a64 + cw;
    }
    __syncthreads();
    if (tid < 64) acc += *(const uint32_t *)(smem + tab + tid * 4);
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
    const uint32_t tiles = argc > 1 ? atoi(argv[1]) : 128;
    const uint32_t waves = argc > 2 ? atoi(argv[2]) : 16;
    const uint32_t obw = argc > 3 ? atoi(argv[3]) : 4096;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint64_t *ht = (uint64_t *)malloc(NS * 128 * 8);
    srand(1);
    for (int i = 0; i < NS * 128; i++) {
        uint32_t n = rand() % 3 + (rand() % 4 == 0);
        uint32_t sy = 0;
        for (uint32_t k = 0; k < n; k++) sy |= (uint32_t)(32 + rand() % 90) << (8 * k);
        uint32_t nx = rand() % NS;
        ht[i] = (uint64_t)sy | (uint64_t)(8 * n) << 32 | (uint64_t)(nx << (K + 3)) << 47;
    }
    uint64_t *gt;
    uint32_t *sink;
    CK(hipMalloc(&gt, NS * 128 * 8));
    CK(hipMalloc(&sink, 64));
    CK(hipMemcpy(gt, ht, NS * 128 * 8, hipMemcpyHostToDevice));
    const size_t lds = NS * 128 * 8 + (size_t)waves * obw;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    void (*ks[8])(const uint64_t *, uint32_t, uint32_t *, uint32_t) = {k_emit<0>, k_emit<1>, k_emit<2>, k_emit<3>,
                                                                       k_emit<4>, k_emit<5>, k_emit<6>, k_emit<7>};
    for (int m = 0; m < 8; m++) {
        if (m == 2 || m == 3 || m == 5) continue;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(ks[m], dim3(ncu), dim3(64 * waves), lds, 0, gt, tiles, sink, obw);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double tl = (double)ncu * waves * tiles;   // tiles (64 regions of 256 bits each)
            if (rep == 2)
                printf("mode %d waves %2u: %.3f ms, %.1f ns per tile per CU, 1 GiB kjv (524288 tiles) -> %.3f ms\n", m, waves,
                       ms, ms * 1e6 / (tl / ncu), ms * 524288.0 / tl);
        }
    }
    return 0;
}
