// hh_fsm_kern.h -- device helpers shared by the state-machine decode kernels:
// the two-pass pipeline (hh_fsm.hip: count, scan, emission) and the
// single-pass decode (hh_one.hip).  Tables and per-lane rules: hh_fsm.h,
// hh_fsm_algo.h.  HIP (gfx950) only, not part of the public ABI.
//
// LDS addressing: both pipelines' kernels declare NO static __shared__ and
// keep their tables at the start of the dynamic LDS, which then begins at
// LDS address 0 -- the table lookups and the stagings use the byte offset
// into the dynamic LDS as the LDS address itself (an address_space(3)
// pointer from the offset, no base add).  lds_base_is_zero() checks that
// assumption at run time in every such kernel (a kernel that adds a static
// __shared__ variable fails its decode instead of reading wrong bytes).
#ifndef HH_FSM_KERN_H_
#define HH_FSM_KERN_H_

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

#include "hh_fsm_algo.h"
#include "hh_fsm_dev.h"
#include "hiphuff.h"

#define FS_OK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "hiphuff: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return HH_ERR_DEVICE;                                             \
        }                                                                     \
    } while (0)

#define NR 64                 // regions per tile (a wave)
#define VMCNT0 0x0F70         // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): vector memory only

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t __attribute__((address_space(3))) *lds_u32p;
typedef const uint16_t __attribute__((address_space(3))) *lds_u16p;
typedef const uint32_t __attribute__((address_space(3))) *lds_cu32p;
typedef const uint64_t __attribute__((address_space(3))) *lds_u64p;

// The dynamic LDS of the calling kernel starts at LDS address 0 (see the top
// of this file).
__device__ __forceinline__ bool lds_base_is_zero(const void *smem) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)smem == 0u;
}

// A table into LDS at a workgroup's start: 16-B loads, 8 of them in flight
// per thread before their stores (a 42 or 85 KB table in one round trip to
// L2; a loop of 4-B load -> store pairs waited for each load in turn).
// Plain loads: the table stays in each XCD's L2 for its other workgroups,
// which all fill at once (round 6, same box: 64 MiB 0.0934-0.0953 ->
// 0.0904-0.0914 ms against nontemporal loads, 1 GiB equal within noise).
// bytes: a multiple of 16; dst and src 16-B aligned.
__device__ __forceinline__ void lds_fill16(uint8_t *dst, const void *src, uint32_t bytes) {
    constexpr uint32_t UNR = 8;
    const u32x4 *s = (const u32x4 *)src;
    u32x4 *d = (u32x4 *)dst;
    const uint32_t n = bytes / 16u, step = blockDim.x;
    for (uint32_t i = threadIdx.x; i < n; i += UNR * step) {
        u32x4 v[UNR];
#pragma unroll
        for (uint32_t u = 0; u < UNR; u++)
            if (i + u * step < n) v[u] = s[i + u * step];
#pragma unroll
        for (uint32_t u = 0; u < UNR; u++)
            if (i + u * step < n) d[i + u * step] = v[u];
    }
}

// Device copies of the state-machine tables (FsmDev's).
struct FsmTab {
    const uint16_t *ct;
    const uint32_t *b1;
    const uint8_t *tsym;
    const uint64_t *et;
    const uint64_t *er;
};

// ---------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t wave_incl_scan(int32_t x) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    return x;
}
__device__ __forceinline__ int32_t wave_sum(int32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t shfl_up1(uint32_t v) { return (uint32_t)__shfl_up((int)v, 1, 64); }
__device__ __forceinline__ uint32_t shfl_down1(uint32_t v) { return (uint32_t)__shfl_down((int)v, 1, 64); }
// a wave-uniform 64-bit value in scalar registers (the compiler cannot always
// tell; a buffer resource built from a vector value costs a waterfall loop)
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint32_t lane_id() {
    uint32_t ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    return ln;
}

#define WAVE_SYNC()                                                    \
    do {                                                               \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");         \
        __builtin_amdgcn_wave_barrier();                               \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");         \
    } while (0)

// ---------------------------------------------------------------------------
// payload words
// ---------------------------------------------------------------------------
// Words of a tile through a buffer resource over the readable words: loads
// past the payload return 0 (never read as stream bits).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fs_rsrc(const uint32_t *g, uint64_t w0, uint64_t nok) {
    const uint64_t left = nok > w0 ? nok - w0 : 0u;
    const uint32_t nbytes = left > 0x3fffffffull ? 0xfffffffcu : (uint32_t)left * 4u;
    return __builtin_amdgcn_make_buffer_rsrc((void *)(g + w0), 0, (int)nbytes, 0x00020000);
}
// SW words from word offset wo of the resource
template <uint32_t SW>
__device__ __forceinline__ void fs_load(uint32_t *v, __amdgpu_buffer_rsrc_t rs, uint32_t wo) {
    if (SW % 4 == 0) {
#pragma unroll
        for (uint32_t k = 0; k < SW; k += 4) {
            const u32x4 q = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(4u * (wo + k)), 0, 0));
            v[k] = q.x; v[k + 1] = q.y; v[k + 2] = q.z; v[k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) v[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * (wo + k)), 0, 0);
    }
}

// byte k / bits [q, q+n) of a region held in registers (compile-time k, q)
template <uint32_t SW>
__device__ __forceinline__ uint32_t rbyte(const uint32_t *w, uint32_t k) {
    return __builtin_amdgcn_ubfe(w[k >> 2], 8 * (k & 3), 8);
}
template <uint32_t SW>
__device__ __forceinline__ uint32_t rbits(const uint32_t *w, uint32_t q, uint32_t n) {
    const uint32_t i = q >> 5, o = q & 31;
    if (o + n <= 32 || i + 1 >= SW) return __builtin_amdgcn_ubfe(w[i], o, n);
    return __builtin_amdgcn_alignbit(w[i + 1], w[i], o) & ((1u << n) - 1u);
}
// bits [q, q+N) of a region times 2^SH: a byte offset into a table row
// (compile-time q)
template <uint32_t SW, uint32_t N, uint32_t SH>
__device__ __forceinline__ uint32_t winsh(const uint32_t *w, uint32_t q) {
    constexpr uint32_t M = ((1u << N) - 1u) << SH;
    if (q < SH) return (w[0] << (SH - q)) & M;
    const uint32_t p = q - SH, i = p >> 5, o = p & 31;
    if (o + N + SH <= 32 || i + 1 >= SW) return (w[i] >> o) & M;
    return __builtin_amdgcn_alignbit(w[i + 1], w[i], o) & M;
}
// bits [q, q+K) of a region times 8: a byte offset into a row of the
// emission table
template <uint32_t SW, uint32_t K>
__device__ __forceinline__ uint32_t win8(const uint32_t *w, uint32_t q) { return winsh<SW, K, 3>(w, q); }
// the same bits at bit 3 and up, the bits above them unmasked (the caller
// inserts them with a bit-field insert)
template <uint32_t SW, uint32_t K>
__device__ __forceinline__ uint32_t win8raw(const uint32_t *w, uint32_t q) {
    if (q < 3) return w[0] << (3 - q);
    const uint32_t p = q - 3, i = p >> 5, o = p & 31;
    if (o + K + 3 <= 32 || i + 1 >= SW) return w[i] >> o;
    return __builtin_amdgcn_alignbit(w[i + 1], w[i], o);
}
// the LDS byte address of the emission entry for the step's K bits at q from
// the high word of the previous entry (its row at bits >= 8, 8 x its symbols
// at bits 3..5, bits 0..2 zero; hh_fsm.h): one bit-field insert
template <uint32_t SW, uint32_t K>
__device__ __forceinline__ uint32_t et_addr(uint32_t hi, const uint32_t *w, uint32_t q) {
    constexpr uint32_t M = ((1u << K) - 1u) << 3;
    return (win8raw<SW, K>(w, q) & M) | (hi & ~M);
}
// bit q of a region held in registers, q not a compile-time constant (rare paths)
template <uint32_t SW>
__device__ __forceinline__ uint32_t rbit_dyn(const uint32_t *w, uint32_t q) {
    uint32_t x = 0;
#pragma unroll
    for (uint32_t k = 0; k < SW; k++) x = (q >> 5) == k ? w[k] : x;
    return (x >> (q & 31)) & 1u;
}

// Bytes of the emission tables in LDS: et, er, b1, tsym (16-B multiple).
__host__ __device__ constexpr uint32_t emf_tab_bytes(uint32_t ns, uint32_t K, uint32_t r) {
    return ((ns << HH_FSM_ET_LG(K)) * 8u + (r ? (ns << r) * 8u : 0u) + ns * 8u + ns + 15u) & ~15u;
}

#endif
