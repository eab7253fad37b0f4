// Design microbenchmark (gfx950), not part of the product: the state-machine
// (FSM) decode step the round-3 kernels are built on.  A lane holds its
// region's 8 words in registers; each step takes the next 8 (count) or 6
// (emit) stream bits at a compile-time offset and looks up (state, bits) in an
// LDS table; the chain runs through the state only.
//   count : u16 entries (next state | symbols completed << 8), 8-bit steps
//   emit  : u64 entries (3 symbol bytes | state << 24 | nsym << 32), 6-bit
//           steps, the symbols stored to a per-wave LDS staging buffer with
//           one 4-byte store at a byte offset (mode 0: unaligned ds_write_b32;
//           mode 1: aligned, 64-bit accumulator; mode 2: no store)
// Prints lane-steps/s chip-wide per configuration.
// Build: hipcc -O3 --offload-arch=gfx950 -o ub_fsm tools/ubench/ub_fsm.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define NST 84

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_count(const uint32_t *g, const uint16_t *gt, uint32_t rounds, uint32_t *sink) {
    __shared__ uint16_t t[NST * 256];
    for (int i = threadIdx.x; i < NST * 256; i += 64 * NW) t[i] = gt[i];
    __syncthreads();
    const uint32_t gid = blockIdx.x * 64 * NW + threadIdx.x;
    uint32_t s = gid % NST, n = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; i++) w[i] = g[((gid * 8 + i) ^ (r * 977)) & ((1 << 22) - 1)];
#pragma unroll
        for (int k = 0; k < 32; k++) {
            const uint32_t b = __builtin_amdgcn_ubfe(w[k >> 2], 8 * (k & 3), 8);
            const uint32_t e = t[(s << 8) | b];
            s = e & 0xffu;
            n += e >> 8;
        }
    }
    if (n == 0x12345) sink[0] = s;
    sink[1 + (gid & 1023)] = n;
}

template <int NW, int MODE>
__global__ __launch_bounds__(64 * NW) void k_emit(const uint32_t *g, const uint64_t *gt, uint32_t rounds, uint32_t *sink) {
    __shared__ uint64_t t[NST * 64];
    __shared__ uint32_t st[NW][1200];
    for (int i = threadIdx.x; i < NST * 64; i += 64 * NW) t[i] = gt[i];
    __syncthreads();
    const uint32_t gid = blockIdx.x * 64 * NW + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *sb = (uint8_t *)st[wv];
    uint32_t s = gid % NST, tot = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; i++) w[i] = g[((gid * 8 + i) ^ (r * 977)) & ((1 << 22) - 1)];
        uint32_t o = lane * 60;         // ~57 bytes per lane, runs back to back
        uint64_t acc = 0;
        uint32_t sh = (o & 3) * 8, wd = o >> 2;
#pragma unroll
        for (int k = 0; k < 42; k++) {
            const int bit = 6 * k, wi = bit >> 5, bo = bit & 31;
            uint32_t b;
            if (bo + 6 <= 32) b = __builtin_amdgcn_ubfe(w[wi], bo, 6);
            else b = __builtin_amdgcn_alignbit(w[wi + 1], w[wi], bo) & 63u;
            const uint64_t e = t[(s << 6) | b];
            s = (uint32_t)(e >> 24) & 0xffu;
            const uint32_t ns = (uint32_t)(e >> 32) & 3u;
            if (MODE == 0) {
                __builtin_memcpy(sb + o, &e, 4);   // unaligned 4-B store
                o += ns;
            } else if (MODE == 1) {
                acc |= (uint64_t)((uint32_t)e & 0xffffffu) << sh;
                ((uint32_t *)sb)[wd] = (uint32_t)acc;
                sh += 8 * ns;
                const bool f = sh >= 32;
                wd += f;
                acc = f ? acc >> 32 : acc;
                sh = f ? sh - 32 : sh;
            } else {
                o += ns;
            }
        }
        tot += o + wd;
    }
    __syncthreads();
    sink[1 + (gid & 1023)] = tot + st[wv][lane];
}

template <typename F>
static double timeit(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < 3; i++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 3;
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *g, *sink;
    uint16_t *t16;
    uint64_t *t64;
    CK(hipMalloc(&g, 4u << 22));
    CK(hipMalloc(&sink, 8192));
    CK(hipMalloc(&t16, NST * 256 * 2));
    CK(hipMalloc(&t64, NST * 64 * 8));
    uint32_t *h = (uint32_t *)malloc(4u << 22);
    uint64_t x = 88172645463325252ull;
    for (int i = 0; i < (1 << 22); i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (uint32_t)x; }
    CK(hipMemcpy(g, h, 4u << 22, hipMemcpyHostToDevice));
    uint16_t ht[NST * 256];
    uint64_t he[NST * 64];
    for (int i = 0; i < NST * 256; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; ht[i] = (uint16_t)(((x >> 8) % NST) | (((x >> 20) % 3) << 8)); }
    for (int i = 0; i < NST * 64; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const uint64_t ns = (x >> 40) % 3;
        he[i] = (x & 0xffffffull) | ((uint64_t)((x >> 24) % NST) << 24) | (ns << 32);
    }
    CK(hipMemcpy(t16, ht, sizeof(ht), hipMemcpyHostToDevice));
    CK(hipMemcpy(t64, he, sizeof(he), hipMemcpyHostToDevice));
    const uint32_t rounds = 64;
#define RUNC(NW, WPC)                                                                                   \
    {                                                                                                    \
        const int nb = ncu * (WPC) / (NW);                                                               \
        double ms = timeit([&] { hipLaunchKernelGGL(k_count<NW>, dim3(nb), dim3(64 * NW), 0, 0, g, t16, rounds, sink); }); \
        double steps = (double)nb * 64 * NW * rounds * 32;                                               \
        printf("count NW=%2d waves/CU=%2d: %.3f ms  %.3e lane-steps/s  (%.2f Gbit/s)\n", NW, WPC, ms, steps / ms * 1e3, steps * 8 / ms / 1e6); \
    }
#define RUNE(NW, WPC, M)                                                                                \
    {                                                                                                    \
        const int nb = ncu * (WPC) / (NW);                                                               \
        double ms = timeit([&] { hipLaunchKernelGGL((k_emit<NW, M>), dim3(nb), dim3(64 * NW), 0, 0, g, t64, rounds, sink); }); \
        double steps = (double)nb * 64 * NW * rounds * 42;                                               \
        printf("emit%d NW=%2d waves/CU=%2d: %.3f ms  %.3e lane-steps/s  (%.2f Gbit/s)\n", M, NW, WPC, ms, steps / ms * 1e3, steps * 6 / ms / 1e6); \
    }
    RUNC(8, 8) RUNC(8, 16) RUNC(8, 24) RUNC(8, 32)
    RUNE(8, 8, 0) RUNE(8, 16, 0) RUNE(16, 16, 0) RUNE(8, 24, 0)
    RUNE(8, 8, 1) RUNE(8, 16, 1) RUNE(16, 16, 1) RUNE(8, 24, 1)
    RUNE(8, 16, 2) RUNE(8, 24, 2)
    return 0;
}
