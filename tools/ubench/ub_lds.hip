// Design microbenchmark (gfx950), not part of the product: how fast can a CU
// run dependent chains of random LDS table lookups -- the state machine's
// count step (hh_fsm.hip k_cntm) -- as a function of waves per CU and of
// independent chains per lane.  Each lane steps CH chains over 32 random
// bytes per round; a step is one read of a table of NS states x 256 entries
// (ENT bytes each: 2 = the count table's u16, 8 = the emission table's u64
// rows read at a 7-bit window), the next address from the entry (AND-OR).
// Prints, per configuration, the time, the wave-level lookups per CU per
// cycle (at the measured clock-free ns: lookups per ns per CU) and the
// chip-wide lookups per second.
//
// Entry geometries of the count step (one configuration
// per run, `ub_lds rounds wpc ent`, for rocprofv3 --pmc SQ_INSTS_LDS
// SQ_LDS_BANK_CONFLICT): ent 2 = the count table (u16, row-major: the bank
// is bits 1..6 of the step's byte, whatever the state), ent 4 = u32 entries
// row-major (84 KB), ent 3 = u16 entries state-interleaved (entry (s, b) at
// (b x NS + s) x 2: the bank depends on the state as well as the byte).
// Build: hipcc -O3 --offload-arch=gfx950 -o build/ub_lds tools/ubench/ub_lds.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define NS 83

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// ENT 2: u16 entries, row = state << 9 (512 B), entry = next row | count
// ENT 8: u64 entries, row = state << 10 (128 x 8 B), 7-bit windows
template <int ENT, int CH>
__global__ void k_chain(const uint32_t *gt, uint32_t rounds, uint32_t *sink) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t RB = ENT == 2 || ENT == 3 ? 512u : 1024u;
    for (uint32_t i = threadIdx.x; i < NS * RB / 4; i += blockDim.x) ((uint32_t *)smem)[i] = gt[i];
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t row[CH], acc = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) row[c] = (mix(gid * 7 + c) % NS) * (ENT == 3 ? 2u : RB);
    for (uint32_t r = 0; r < rounds; r++) {
        uint32_t w[CH][8];
#pragma unroll
        for (int c = 0; c < CH; c++)
#pragma unroll
            for (int i = 0; i < 8; i++) w[c][i] = mix(gid * 64 + r * 8 + i + c * 1000003u);
#pragma unroll
        for (int k = 0; k < 32; k++) {
#pragma unroll
            for (int c = 0; c < CH; c++) {
                if (ENT == 2) {
                    const uint32_t b = __builtin_amdgcn_ubfe(w[c][k >> 2], 8 * (k & 3), 8) << 1;
                    const uint32_t e = *(const uint16_t __attribute__((address_space(3))) *)(uintptr_t)((row[c] & 0xfe00u) | b);
                    row[c] = e;
                    acc += e;
                    asm volatile("" : "+v"(acc));
                } else if (ENT == 4) {
                    const uint32_t b = __builtin_amdgcn_ubfe(w[c][k >> 2], 8 * (k & 3), 8) << 2;
                    const uint32_t e = *(const uint32_t __attribute__((address_space(3))) *)(uintptr_t)((row[c] & 0xfc00u) | b);
                    row[c] = e;
                    acc += e;
                    asm volatile("" : "+v"(acc));
                } else if (ENT == 3) {
                    // row[c]: the state x 2; entry = next state x 2 | count << 12
                    const uint32_t b = __builtin_amdgcn_ubfe(w[c][k >> 2], 8 * (k & 3), 8);
                    const uint32_t e = *(const uint16_t __attribute__((address_space(3))) *)(uintptr_t)(b * (2u * NS) + (row[c] & 0xffeu));
                    row[c] = e;
                    acc += e;
                    asm volatile("" : "+v"(acc));
                } else {
                    const uint32_t b = (__builtin_amdgcn_ubfe(w[c][k >> 2], 8 * (k & 3), 7)) << 3;
                    const uint64_t e = *(const uint64_t __attribute__((address_space(3))) *)(uintptr_t)(row[c] | b);
                    row[c] = (uint32_t)(e >> 47);
                    acc += (uint32_t)e;
                    asm volatile("" : "+v"(acc));
                }
            }
        }
    }
    uint32_t x = acc;
#pragma unroll
    for (int c = 0; c < CH; c++) x += row[c];
    if (x == 0x12345678u) sink[0] = x;
}

static void fill(uint32_t *h, int ent) {
    srand(3);
    if (ent == 2) {
        uint16_t *t = (uint16_t *)h;
        for (int i = 0; i < NS * 256; i++) t[i] = (uint16_t)(((rand() % NS) << 9) | (rand() % 4));
    } else if (ent == 3) {
        uint16_t *t = (uint16_t *)h;
        for (int i = 0; i < NS * 256; i++) t[i] = (uint16_t)(((rand() % NS) << 1) | (rand() % 4) << 12);
    } else if (ent == 4) {
        for (int i = 0; i < NS * 256; i++) h[i] = (uint32_t)(((rand() % NS) << 10) | (rand() % 4));
    } else {
        uint64_t *t = (uint64_t *)h;
        for (int i = 0; i < NS * 128; i++)
            t[i] = (uint64_t)(rand() & 0x7f7f7f) | (uint64_t)(8 * (rand() % 3)) << 32 | (uint64_t)((rand() % NS) << 10) << 47;
    }
}

template <int ENT, int CH>
static void run(int ncu, const uint32_t *gt, uint32_t *sink, int wpc, uint32_t rounds) {
    const int tb = 64 * (wpc < 16 ? wpc : 16), wgs = wpc / (tb / 64);
    const size_t lds = NS * (ENT == 2 || ENT == 3 ? 512 : 1024);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_chain<ENT, CH>), dim3(ncu * wgs), dim3(tb), lds, 0, gt, rounds, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double lk = (double)ncu * wpc * rounds * 32 * CH;   // wave-level lookups
    printf("ent %d chains/lane %d waves/CU %2d: %8.3f ms  %.3f wave-lookups/ns/CU  %.2f ns per chain step\n", ENT, CH, wpc,
           ms, lk / ncu / (ms * 1e6), ms * 1e6 / (rounds * 32.0));
}

int main(int argc, char **argv) {
    const uint32_t rounds = argc > 1 ? atoi(argv[1]) : 2000;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *h = (uint32_t *)calloc(NS * 1024, 1), *gt, *sink;
    CK(hipMalloc(&gt, NS * 1024));
    CK(hipMalloc(&sink, 64));
    if (argc > 2) {           // one configuration: rounds wpc ent (2 | 8), one chain per lane
        const int wpc = atoi(argv[2]), ent = argc > 3 ? atoi(argv[3]) : 2;
        fill(h, ent);
        CK(hipMemcpy(gt, h, NS * (ent == 2 || ent == 3 ? 512 : 1024), hipMemcpyHostToDevice));
        if (ent == 2) run<2, 1>(ncu, gt, sink, wpc, rounds);
        else if (ent == 3) run<3, 1>(ncu, gt, sink, wpc, rounds);
        else if (ent == 4) run<4, 1>(ncu, gt, sink, wpc, rounds);
        else run<8, 1>(ncu, gt, sink, wpc, rounds);
        return 0;
    }
    const int W[] = {4, 8, 12, 16, 32};
    fill(h, 2);
    CK(hipMemcpy(gt, h, NS * 512, hipMemcpyHostToDevice));
    for (int w : W) run<2, 1>(ncu, gt, sink, w, rounds);
    for (int w : W) run<2, 2>(ncu, gt, sink, w, rounds / 2);
    for (int w : W) run<2, 4>(ncu, gt, sink, w, rounds / 4);
    fill(h, 8);
    CK(hipMemcpy(gt, h, NS * 1024, hipMemcpyHostToDevice));
    for (int w : W) run<8, 1>(ncu, gt, sink, w, rounds);
    for (int w : W) run<8, 2>(ncu, gt, sink, w, rounds / 2);
    return 0;
}
