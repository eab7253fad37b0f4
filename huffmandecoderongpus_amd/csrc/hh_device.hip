// hh_device.hip -- HIP kernels (gfx950) and the device half of the C ABI.
//
// Fast path: ONE persistent launch, k_decode (O(N) memory, 64-bit offsets).
// Tiles of HH_NR regions of S bits are dispensed in order; each workgroup
// keeps two in flight: while it decodes tile B's regions from offset 0 with
// boundary masks (decodeallbits) it emits tile A's runs (calcresult), then
// walks B's region exits into their successors until the chains share a
// boundary (makebigtable) and publishes B's transfer table.  Output bases
// come from a decoupled look-back over those tables (calcbitsindex /
// findmax).  C is read once from HBM, D written once.
// Reference-shaped stage kernels (k_st_*) mirror the six .cl kernels one by
// one for intermediate-array parity.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hh_algo.h"
#include "hh_internal.h"
#include "hiphuff.h"

#define HH_S_DEFAULT 288          // 9 words: odd word stride spreads LDS banks
#define HH_S_MAX 320
#define HH_SPAN_MARGIN 320        // bits beyond the last walk region
#define HH_NW_MAX (((HH_NL + HH_KM + 1) * HH_S_MAX + HH_SPAN_MARGIN) / 32 + 4)
#define HH_MAXLEN_FAST 256        // longest code the fast path stages for

#define HIP_OK(x)                                                             \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "hiphuff: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return HH_ERR_DEVICE;                                             \
        }                                                                     \
    } while (0)

struct DevTab {
    const uint64_t *l1;
    const uint32_t *l2;
    const uint32_t *tree;
    const uint8_t *tsym;
    uint32_t l2_used;
};

// flags[0]: bit0 walk failed, bit1 output overflow, bit2 count mismatch
// flags[2..3]: total symbols (u64, written by k_scan)
enum { F_FAIL = 1, F_OVER = 2, F_MISMATCH = 4 };

// ---------------------------------------------------------------------------
// shared helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Exclusive block scan of u32 (blockDim == HH_NL, 4 waves).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_tmp, uint32_t *total) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_tmp[wv] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t i = 0; i < HH_NL / 64; i++) {
        uint32_t t = s_tmp[i];
        if (i < wv) base += t;
        tot += t;
    }
    *total = tot;
    __syncthreads();
    return base + x - v;
}

// The exceptions (walks with k > 1) of a tile, ascending, into s_exc.
__device__ __forceinline__ uint32_t collect_exceptions(bool is_exc, uint16_t *s_exc, uint32_t *s_cnt4) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t m = __ballot(is_exc);
    if (lane == 0) s_cnt4[wv] = __popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (uint32_t i = 0; i < HH_NL / 64; i++) {
        if (i < wv) off += s_cnt4[i];
        tot += s_cnt4[i];
    }
    if (is_exc) {
        uint64_t below = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
        s_exc[off + __popcll(below)] = (uint16_t)threadIdx.x;
    }
    __syncthreads();
    return tot;
}

// ---------------------------------------------------------------------------
// The fused decoder: one persistent kernel, tiles dispensed in order.
//
// Per tile: (1) stage the tile's bits (+ halo) in LDS; (2) every lane
// decodes its region from offset 0 and walks its exit into the next region
// until the chains share a boundary; (3) the tile resolves its live lanes for
// every entering state d and publishes its HH_KM-entry transfer table
// (AGGREGATE); (4) decoupled look-back over predecessors' tables / inclusive
// states yields this tile's entering state and output base, published as
// INCLUSIVE; (5) live lanes re-decode their runs into an LDS window, written
// out with 16-byte stores.  C is read once, D written once.
// ---------------------------------------------------------------------------
struct LookBack {
    uint64_t *gran;      // [ntiles] tagged granule: table published (+ count, state for d = 0)
    uint64_t *incl;      // [ntiles] tagged inclusive prefix of charged counts
    uint64_t *xst;       // [ntiles] tagged resolved outgoing state
    uint64_t *tabs;      // [ntiles][HH_KM] tile tables (sc1 stores)
    uint32_t *counter;   // tile dispenser
};

// 64-bit granules: the data is the flag (bits 62..63 = status, 0 = not yet).
#define HH_ST_SHIFT 62
#define HH_VAL_MASK ((1ull << HH_ST_SHIFT) - 1ull)

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

enum { F_TIMEOUT = 8 };

// Diagnostic build only (-DHH_STAMPS): wave 0 of every workgroup adds the
// shader-clock cycles of each phase into dbg[block][phase].
#define HH_NDBG 12
#ifdef HH_STAMPS
#define HH_NSTAMP HH_NDBG
#define STAMP_DECL uint64_t st_acc[HH_NSTAMP] = {0}; uint64_t st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { uint64_t t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } while (0)
#define STAMP_FLUSH(dbg) do { if (threadIdx.x == 0) for (int i_ = 0; i_ < HH_NSTAMP; i_++) (dbg)[blockIdx.x * HH_NSTAMP + i_] = st_acc[i_]; } while (0)
#define COUNT(i, v) do { st_acc[i] += (v); } while (0)
#define HH_TDBG_MAX (1u << 18)
#define TSTAMP(t, k) do { if (threadIdx.x == 0 && (t) < HH_TDBG_MAX) dbg[gridDim.x * HH_NDBG + (t) * 6 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define COUNT(i, v) do {} while (0)
#define TSTAMP(t, k) do {} while (0)
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH(dbg) do {} while (0)
#endif
#define HH_SPIN_LIMIT (1u << 22)

// Stage n u64 / u32 table words with all loads issued before any LDS store.
template <uint32_t N>
__device__ __forceinline__ void stage_l1(uint64_t *dst, const uint64_t *src) {
    constexpr uint32_t PER = N / HH_NL;
    uint64_t v[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) v[k] = src[threadIdx.x + k * HH_NL];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) dst[threadIdx.x + k * HH_NL] = v[k];
}

// Poll a tagged granule until its status bits are non-zero (bounded).
__device__ __forceinline__ uint64_t poll_granule(const uint64_t *p, uint32_t *flags) {
    uint64_t v;
    uint32_t spins = 0;
    while (((v = ld_sc1(p)) >> HH_ST_SHIFT) == 0) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > HH_SPIN_LIMIT) {
            atomicOr(flags, (uint32_t)F_TIMEOUT);
            return 3ull << HH_ST_SHIFT;
        }
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// Regions per tile: the last lane decodes the NEXT tile's first region too
// (its mask lets the tile's last walk merge without a two-pointer walk).
#define HH_NR (HH_NL - 1)

// Granule layout (gran[t], status 1 = tile t's table is published):
//   bits  0..19 count_t(0), signed: symbols charged to the tile for d = 0
//   bits 20..23 d_out, 24..35 e_out, 36..51 delta_out (the state for d = 0)
//   bit  61     CONST: every entering d leads to that same outgoing state
// Charging: count_t(d) = sum over the tile's live lanes of n + cov + delta,
// i.e. each walk's correction is charged to the walker's tile, so a tile's
// count depends on its predecessor only through d.  The first run of tile t
// then starts delta_in(t) symbols before the charged prefix of tiles < t.
#define HH_GR_PUB (1ull << 62)
#define HH_GR_CST (1ull << 61)
#define HH_INCL (2ull << 62)

__device__ __forceinline__ uint64_t gran_pack(uint64_t xf, bool cst) {
    return HH_GR_PUB | (cst ? HH_GR_CST : 0ull) | (uint64_t)(hh_xf_count(xf) & 0xfffffu) |
           ((uint64_t)hh_xf_d(xf) << 20) | ((uint64_t)hh_xf_e(xf) << 24) |
           ((uint64_t)((uint32_t)hh_xf_delta(xf) & 0xffffu) << 36);
}
__device__ __forceinline__ int32_t gran_cnt(uint64_t g) { return ((int32_t)((uint32_t)g << 12)) >> 12; }
// entering-state word of the successor: d | e << 4 | delta << 16
__device__ __forceinline__ uint64_t gran_state(uint64_t g) {
    return ((g >> 20) & 0xfu) | (((g >> 24) & 0xfffu) << 4) | (((g >> 36) & 0xffffu) << 16);
}
__device__ __forceinline__ uint64_t xf_state(uint64_t xf) {
    return (uint64_t)hh_xf_d(xf) | ((uint64_t)hh_xf_e(xf) << 4) |
           ((uint64_t)((uint32_t)hh_xf_delta(xf) & 0xffffu) << 16);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
    const uint32_t lo = __shfl((uint32_t)v, (int)src, 64), hi = __shfl((uint32_t)(v >> 32), (int)src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// Charged symbols of tiles < A (A >= 1), one wave.  64 predecessors per
// round: granule, inclusive word and the granule before it (which gives the
// predecessor's entering d).  The nearest inclusive prefix ends the round;
// the window's own inclusive prefixes are then published too, so later
// look-backs stop early.  Returns false if an entering d in the window is
// not CONST-resolvable (rare: caller takes the serial path).
#ifdef HH_STAMPS
#define COUNT_LB(i, v) do { lbd[i] += (v); } while (0)
#else
#define COUNT_LB(i, v) do {} while (0)
#endif
__device__ bool lookback_excl(const LookBack &lb, uint64_t A, uint32_t *flags, uint64_t *excl_out,
                              uint32_t *nrounds, uint32_t *nspins, uint64_t *lbd) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t excl = 0;
    int64_t top = (int64_t)A - 1;
    int32_t c0 = 0;
    uint32_t first0 = 64;
    bool r0 = true;
    for (;;) {
        const int64_t idx = top - (int64_t)lane;
        uint64_t iv = HH_INCL, gv = HH_GR_PUB | HH_GR_CST, gp = HH_GR_PUB | HH_GR_CST;
        uint32_t first, spins = 0;
        for (;;) {
            if (idx >= 0) {
                iv = ld_sc1(&lb.incl[idx]);
                gv = ld_sc1(&lb.gran[idx]);
            }
            if (idx >= 1) gp = ld_sc1(&lb.gran[idx - 1]);
            const uint64_t inc = __ballot((iv >> HH_ST_SHIFT) == 2);
            first = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
            const uint64_t miss = __ballot(lane < first && ((gv >> HH_ST_SHIFT) == 0 || (gp >> HH_ST_SHIFT) == 0));
            if (!miss) break;
            COUNT_LB(0, __builtin_ctzll(miss));
            COUNT_LB(1, 63 - __builtin_clzll(miss));
            COUNT_LB(2, (__ballot(lane < first && (gv >> HH_ST_SHIFT) == 0) != 0));
            COUNT_LB(3, first);
            __builtin_amdgcn_s_sleep(1);
            if (++spins > HH_SPIN_LIMIT) {
                if (lane == 0) atomicOr(flags, (uint32_t)F_TIMEOUT);
                *excl_out = 0;
                return true;
            }
        }
        *nrounds += 1;
        *nspins += spins;
        if (__ballot(lane < first && !(gp & HH_GR_CST))) return false;
        int32_t c = 0;
        if (lane < first) {
            const uint32_t din = (uint32_t)(gp >> 20) & 0xfu;
            c = din == 0 ? gran_cnt(gv) : (int32_t)hh_xf_count(ld_sc1(&lb.tabs[idx * HH_KM + din]));
        }
        excl += wave_sum64((uint64_t)(int64_t)c);
        if (first < 64) excl += shfl64(iv, first) & HH_VAL_MASK;
        if (r0) {
            c0 = c;
            first0 = first;
            r0 = false;
        }
        if (first < 64) break;
        top -= 64;
    }
    // inclusive prefixes of the first window: incl[A-1-i] = excl - sum_{j<i} c0_j
    int32_t x = c0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane < first0) st_sc1(&lb.incl[A - 1 - lane], ((excl - (uint64_t)(int64_t)(x - c0)) & HH_VAL_MASK) | HH_INCL);
    *excl_out = excl;
    return true;
}

// Tile staging: a tile's words (+ halo) are loaded to registers, then stored
// to LDS.  Plain loads: the emission pass re-stages the same words two
// iterations later, from L2.
#define HH_STAGE_PER ((HH_NW_MAX + HH_NL - 1) / HH_NL)
struct Staged {
    uint32_t v[HH_STAGE_PER];
};
__device__ __forceinline__ void stage_load(Staged &s, const uint32_t *g, uint64_t w0, uint32_t nw,
                                           uint64_t nwords_ok) {
#pragma unroll
    for (uint32_t k = 0; k < HH_STAGE_PER; k++) {
        const uint32_t i = threadIdx.x + k * HH_NL;
        const uint64_t gi = w0 + i;
        s.v[k] = (i < nw && gi < nwords_ok) ? g[gi] : 0u;
    }
}
__device__ __forceinline__ void stage_store(const Staged &s, uint32_t *dst, uint32_t nw) {
#pragma unroll
    for (uint32_t k = 0; k < HH_STAGE_PER; k++) {
        const uint32_t i = threadIdx.x + k * HH_NL;
        if (i < nw) dst[i] = s.v[k];
    }
}

// ---------------------------------------------------------------------------
// k_decode: persistent; a workgroup holds three tiles.  Iteration i:
//   (1) take tile B (dispenser) and load its bits (+ halo) into registers;
//       re-stage the bits of tile A (taken in iteration i-2) from L2;
//   (2) tile A: output base by look-back over its predecessors' granules.
//       Those were published when their tiles were decoded, at least one
//       full iteration ago, and a granule is published before its
//       workgroup's own look-back -- so a look-back never waits on a tile
//       whose publication itself waits (emitting one iteration after the
//       decode instead lets waits feed on waits without bound);
//       then A's live lanes and run offsets;
//   (3) one loop, two independent chains per lane: B's offset-0 region
//       decode with its boundary mask (decodeallbits) and A's run emission
//       (calcresult), dword stores straight to HBM;
//   (4) B's walks (makebigtable) and transfer table, published with its
//       granule.  Then A <- P (the tile decoded in iteration i-1), P <- B.
// C is read from HBM once (the re-stage hits L2) and D written once.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(HH_NL) void k_decode(const uint32_t *__restrict__ gdata, uint64_t bits,
                                                  uint64_t nwords_ok, uint32_t S, DevTab tab,
                                                  uint64_t ntiles, LookBack lb,
                                                  uint8_t *__restrict__ out, uint64_t cap,
                                                  uint32_t *flags, uint64_t *dbg) {
    __shared__ uint64_t s_l1[HH_L1_SIZE];
    __shared__ uint32_t s_w[2 * HH_NW_MAX];
    __shared__ uint32_t s_mask[HH_NL * HH_MW_MAX];
    __shared__ uint16_t s_x[HH_NL];
    __shared__ uint16_t s_n[HH_NL];
    __shared__ uint8_t s_mem[HH_NL];
    __shared__ uint8_t s_k[HH_NL];
    __shared__ uint16_t s_exc[HH_NL];
    __shared__ uint16_t s_ein[HH_NL];
    __shared__ int16_t s_din[HH_NL];
    __shared__ uint32_t s_cnt4[4];
    __shared__ int32_t s_part[4][HH_KM];
    __shared__ uint64_t s_out[HH_KM];
    __shared__ uint64_t s_tab[HH_KM];
    __shared__ uint64_t s_st[2];
    __shared__ uint32_t s_tile;
    extern __shared__ uint32_t s_l2[];

    const uint32_t lane = threadIdx.x;
    const uint32_t mw = (S + 31) / 32;
    const uint32_t span = (HH_NL + HH_KM + 1) * S + HH_SPAN_MARGIN;
    const uint32_t nw = (span + 31) / 32 + 3;
    stage_l1<HH_L1_SIZE>(s_l1, tab.l1);
    for (uint32_t i = lane; i < tab.l2_used; i += HH_NL) s_l2[i] = tab.l2[i];
    STAMP_DECL

    // tiles A (to emit) and P (decoded last iteration): index and this
    // lane's walk record
    uint64_t tA = ~0ull, tP = ~0ull;
    uint32_t aN = 0, aCov = 0, aE = 0, aK = 1;
    int32_t aDel = 0;
    uint32_t pN = 0, pCov = 0, pE = 0, pK = 1;
    int32_t pDel = 0;
    uint32_t *wB = s_w;                       // tile being decoded
    uint32_t *wA = s_w + HH_NW_MAX;           // tile being emitted

    for (;;) {
        if (lane == 0) s_tile = atomicAdd(lb.counter, 1u);
        __syncthreads();
        const uint64_t tB = s_tile;
        const bool hasB = tB < ntiles, hasA = tA < ntiles;
        if (!hasA && !hasB && tP >= ntiles) break;
        if (hasB) {
            TSTAMP(tB, 0);
#ifdef HH_STAMPS
            if (lane == 0 && tB < HH_TDBG_MAX) dbg[gridDim.x * HH_NDBG + tB * 6 + 4] = blockIdx.x;
#endif
        }
        uint64_t b0B = 0, b0A = 0;
        uint32_t btB = 0, btA = 0;
        Staged stg;
        if (hasB) {
            b0B = tB * (uint64_t)HH_NR * S;
            const uint64_t rem = bits - b0B;
            btB = rem < span ? (uint32_t)rem : span;
            stage_load(stg, gdata, b0B >> 5, nw, nwords_ok);
        }
        if (hasA) {
            b0A = tA * (uint64_t)HH_NR * S;
            const uint64_t rem = bits - b0A;
            btA = rem < span ? (uint32_t)rem : span;
            Staged sa;
            stage_load(sa, gdata, b0A >> 5, nw, nwords_ok);
            stage_store(sa, wA, nw);
        }
        STAMP(0);

        // (2) tile A: entering state and output base
        uint32_t pA = 0, peA = 0;
        uintptr_t dst = 0;
        if (hasA) {
            TSTAMP(tA, 2);
            if (lane < 64) {
                uint64_t excl = 0, stw = 0;
                bool ok = true;
                uint32_t nrounds = 0, nspins = 0;
                uint64_t lbd[4] = {0, 0, 0, 0};
                if (tA > 0) ok = lookback_excl(lb, tA, flags, &excl, &nrounds, &nspins, lbd);
                COUNT(8, lbd[0]);
                COUNT(9, lbd[1]);
                COUNT(10, lbd[2]);
                COUNT(11, lbd[3]);
                COUNT(6, nrounds + (ok ? 0ull : (1ull << 32)));
                COUNT(7, nspins);
                if (lane == 0) {
                    if (tA > 0) {
                        const uint64_t g = poll_granule(&lb.gran[tA - 1], flags);
                        stw = (g & HH_GR_CST) ? gran_state(g) : (poll_granule(&lb.xst[tA - 1], flags) & HH_VAL_MASK);
                        if (!ok) excl = poll_granule(&lb.incl[tA - 1], flags) & HH_VAL_MASK;
                    }
                    const uint64_t xf = ld_sc1(&lb.tabs[tA * HH_KM + (stw & 0xfu)]);
                    const uint64_t incl = excl + (uint64_t)(int64_t)(int32_t)hh_xf_count(xf);
                    st_sc1(&lb.xst[tA], xf_state(xf) | HH_GR_PUB);
                    st_sc1(&lb.incl[tA], (incl & HH_VAL_MASK) | HH_INCL);
                    if (tA == ntiles - 1) {
                        flags[2] = (uint32_t)incl;
                        flags[3] = (uint32_t)(incl >> 32);
                    }
                    s_st[0] = stw;
                    s_st[1] = excl;
                }
            }
            STAMP(1);
            TSTAMP(tA, 3);
            s_k[lane] = (uint8_t)aK;
            __syncthreads();
            const uint64_t sw = s_st[0];
            const uint32_t din = (uint32_t)(sw & 0xfu);
            s_mem[lane] = lane >= din && lane < HH_NR;
            const uint32_t nexc = collect_exceptions(aK > 1 && lane < HH_NR, s_exc, s_cnt4);
            if (lane == 0) {
                for (uint32_t i = 0; i < nexc; i++) {
                    const uint32_t j = s_exc[i], kj = s_k[j];
                    if (!s_mem[j]) continue;
                    for (uint32_t q = j + 1; q < j + kj && q < HH_NR; q++) s_mem[q] = 0;
                }
            }
            __syncthreads();
            const bool live = s_mem[lane] != 0;
            if (live && lane + aK < HH_NR) {
                s_ein[lane + aK] = (uint16_t)aE;
                s_din[lane + aK] = (int16_t)aDel;
            }
            __syncthreads();
            uint32_t e_in = 0;
            int32_t del_in = 0;
            if (live) {
                e_in = lane == din ? (uint32_t)((sw >> 4) & 0xfffu) : s_ein[lane];
                del_in = lane == din ? (int32_t)(int16_t)(uint16_t)(sw >> 16) : s_din[lane];
            }
            const uint32_t cnt = live ? (uint32_t)((int32_t)(aN + aCov) + del_in) : 0u;
            uint32_t total;
            const uint32_t off = block_excl_scan(cnt, s_cnt4, &total);
            const uint64_t base = s_st[1] - (uint64_t)(int64_t)(int32_t)(int16_t)(uint16_t)(sw >> 16);
            if (base + total > cap) {
                if (lane == 0) atomicOr(flags, (uint32_t)F_OVER);
            } else if (live) {
                pA = lane * S + e_in;
                const uint32_t end = (lane + aK) * S + aE;
                peA = end < btA ? end : btA;
                if (pA > peA) pA = peA;
                dst = (uintptr_t)(out + base + off);
            }
            STAMP(2);
        }
        if (hasB) stage_store(stg, wB, nw);
        __syncthreads();

        // (3) B's region decode + A's emission, interleaved
        hh_ctx cA, cB;
        cA.w = wA; cA.sh = (uint32_t)(b0A & 31); cA.l1 = s_l1; cA.l2 = s_l2; cA.tree = tab.tree; cA.tsym = tab.tsym; cA.bt = btA;
        cB.w = wB; cB.sh = (uint32_t)(b0B & 31); cB.l1 = s_l1; cB.l2 = s_l2; cB.tree = tab.tree; cB.tsym = tab.tsym;
        cB.bt = btB;
        const uint32_t p0 = lane * S;
        uint32_t pB = p0, limB = p0, nB = 0, mbase = p0, wdone = 0;
        uint64_t macc = 0;
        if (hasB && p0 < btB) limB = p0 + S < btB ? p0 + S : btB;
        uint64_t acc = 0;
        uint32_t nacc = 0;
        uint32_t *msk = &s_mask[lane * mw];
        for (;;) {
            const bool aB = pB < limB, aA = pA < peA;
            if (!aB && !aA) break;
            const uint32_t qB = pB + cB.sh, qA = pA + cA.sh;
            const uint32_t b0 = wB[qB >> 5], b1 = wB[(qB >> 5) + 1];
            const uint32_t a0 = wA[qA >> 5], a1 = wA[(qA >> 5) + 1];
            const uint32_t winB = __builtin_amdgcn_alignbit(b1, b0, qB & 31);
            const uint32_t winA = __builtin_amdgcn_alignbit(a1, a0, qA & 31);
            const uint64_t eB = s_l1[winB & (HH_L1_SIZE - 1u)];
            const uint64_t eA = s_l1[winA & (HH_L1_SIZE - 1u)];
            if (aB) {
                uint32_t ns = HH_L1_NSYM(eB), l, bm = 1u;
                if (ns && pB + HH_L1_NBITS(eB) <= limB) {
                    l = HH_L1_NBITS(eB);
                    bm = HH_L1_BMASK(eB);
                } else {
                    if (ns) {
                        l = HH_L1_LEN0(eB);
                    } else {
                        uint32_t s;
                        l = hh_escape(&cB, pB, winB, eB, &s);
                    }
                    ns = 1;
                }
                macc |= (uint64_t)bm << (pB - mbase);
                const uint32_t rem = btB - pB;
                pB += l < rem ? l : rem;
                nB += ns;
                while (pB - mbase >= 32 && wdone < mw) {
                    msk[wdone++] = (uint32_t)macc;
                    macc >>= 32;
                    mbase += 32;
                }
            }
            if (aA) {
                uint32_t ns = HH_L1_NSYM(eA), val, n, adv;
                if (ns && pA + HH_L1_NBITS(eA) <= peA) {
                    val = HH_L1_SYMS(eA);
                    n = ns;
                    adv = HH_L1_NBITS(eA);
                } else {
                    uint32_t s;
                    if (ns) {
                        adv = HH_L1_LEN0(eA);
                        s = HH_L1_SYMS(eA) & 0xffu;
                    } else {
                        adv = hh_escape(&cA, pA, winA, eA, &s);
                    }
                    if (adv > btA - pA) {
                        s = hh_tail_symbol(&cA, pA);
                        adv = btA - pA;
                    }
                    val = s;
                    n = 1;
                }
                acc |= (uint64_t)val << (8u * nacc);
                nacc += n;
                pA += adv;
                if (nacc >= 4) {
                    *(uint32_t *)dst = (uint32_t)acc;   // unaligned dword store (CDNA global memory)
                    dst += 4;
                    acc >>= 32;
                    nacc -= 4;
                }
            }
        }
        for (uint32_t i = 0; i < nacc; i++) *(uint8_t *)(dst + i) = (uint8_t)(acc >> (8 * i));
        while (wdone < mw) {
            msk[wdone++] = (uint32_t)macc;
            macc >>= 32;
        }
        s_x[lane] = (uint16_t)(pB - p0);
        s_n[lane] = (uint16_t)nB;
        __syncthreads();
        STAMP(3);

        // (4) B's walks and transfer table
        if (hasB) {
            hh_rec r;
            r.n = nB; r.k = 1; r.e = 0; r.delta = 0; r.cov = 0;
            if (lane < HH_NR) {
                hh_masks mk = {s_mask, s_x, s_n, HH_NL, mw};
                hh_walk_mask(&cB, &mk, lane, S, pB, &r);
                r.n = nB;
                if (r.k == 0) atomicOr(flags, (uint32_t)F_FAIL);
            }
            const uint32_t kk = r.k ? r.k : 1u;
            STAMP(4);
            s_mem[lane] = lane >= HH_NR ? 0u : (lane >= HH_KM - 1 ? 0xffu : (uint8_t)((1u << (lane + 1)) - 1u));
            s_k[lane] = (uint8_t)kk;
            const uint32_t nexc = collect_exceptions(kk > 1 && lane < HH_NR, s_exc, s_cnt4);
            if (lane == 0) {
                for (uint32_t i = 0; i < nexc; i++) {
                    const uint32_t j = s_exc[i], kj = s_k[j];
                    const uint8_t m = s_mem[j];
                    for (uint32_t q = j + 1; q < j + kj && q < HH_NR; q++) s_mem[q] &= (uint8_t)~m;
                }
            }
            __syncthreads();
            const uint32_t memd = s_mem[lane];
            const int32_t contrib = lane < HH_NR ? (int32_t)(r.n + r.cov) + r.delta : 0;
            if (lane < HH_NR && lane + kk >= HH_NR) {
                for (uint32_t d = 0; d < HH_KM; d++)
                    if ((memd >> d) & 1u) s_out[d] = hh_xf_pack(0, r.delta, r.e, lane + kk - HH_NR);
            }
#pragma unroll
            for (uint32_t d = 0; d < HH_KM; d++) {
                int32_t v = ((memd >> d) & 1u) ? contrib : 0;
                v = (int32_t)wave_sum((uint32_t)v);
                if ((lane & 63) == 0) s_part[lane >> 6][d] = v;
            }
            __syncthreads();
            if (lane < HH_KM) {
                const int32_t cnt = s_part[0][lane] + s_part[1][lane] + s_part[2][lane] + s_part[3][lane];
                const uint64_t o = s_out[lane];
                s_tab[lane] = hh_xf_pack((uint32_t)cnt, hh_xf_delta(o), hh_xf_e(o), hh_xf_d(o));
            }
            __syncthreads();
            if (lane == 0) {
                const uint64_t o0 = s_tab[0] >> 32;
                bool cst = true;
                for (uint32_t i = 0; i < HH_KM; i++) {
                    st_sc1(&lb.tabs[tB * HH_KM + i], s_tab[i]);
                    cst = cst && (s_tab[i] >> 32) == o0;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_sc1(&lb.gran[tB], gran_pack(s_tab[0], cst));
            }
            TSTAMP(tB, 1);
            STAMP(5);
            // A <- P, P <- B
            aN = pN; aCov = pCov; aE = pE; aK = pK; aDel = pDel;
            pN = r.n; pCov = r.cov; pE = r.e; pK = kk; pDel = r.delta;
        } else {
            aN = pN; aCov = pCov; aE = pE; aK = pK; aDel = pDel;
        }
        tA = tP;
        tP = hasB ? tB : ~0ull;
    }
    STAMP_FLUSH(dbg);
}

// ---------------------------------------------------------------------------
// Reference-shaped stage kernels (ReleaseCL/kernels/ *.cl, one each).
// ---------------------------------------------------------------------------
__global__ void k_st_init(int32_t *idx, int64_t bits) {
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < bits;
         b += (int64_t)gridDim.x * blockDim.x)
        idx[b] = -1;
}

// decodeallbits.cl:10-33: walk from every bit until a leaf or the end.
__global__ void k_st_decodeallbits(const uint8_t *__restrict__ data, int64_t bits, DevTab tab,
                                   uint8_t *__restrict__ bitdecode, int32_t *__restrict__ steps) {
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < bits;
         b += (int64_t)gridDim.x * blockDim.x) {
        int64_t p = b;
        uint32_t node = 0;
        for (;;) {
            uint32_t t = tab.tree[node];
            if ((t & HH_T_LEAF) || p >= bits) break;
            uint32_t bit = (data[p >> 3] >> (p & 7)) & 1u;
            node = bit ? (t >> 15) & 0x7fffu : t & 0x7fffu;
            p++;
        }
        bitdecode[b] = tab.tsym[node];
        steps[b] = (int32_t)(p - b);
    }
}

// makebigtable.cl:10-40 with the end-of-stream read made explicit: a span
// ending exactly at the end (b + s == bits) reads row step+1 in the serial
// form (pes.c:58) and always yields -1 there; here that case is -1 directly.
__global__ void k_st_makebigtable(int64_t bits, int32_t *steps, int32_t step) {
    const int32_t *cur = steps + (int64_t)step * bits;
    int32_t *nxt = steps + (int64_t)(step + 1) * bits;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < bits;
         b += (int64_t)gridDim.x * blockDim.x) {
        int32_t s = cur[b], v;
        if (s == -1 || b + s >= bits) {
            v = -1;
        } else {
            int32_t w = cur[b + s];
            v = (w == -1 || b + s + w > bits) ? -1 : s + w;
        }
        nxt[b] = v;
    }
}

// calcbitsindex.cl:5-22
__global__ void k_st_calcbitsindex(int64_t bits, int32_t *idx, const int32_t *steps, int32_t step,
                                   int32_t pw) {
    const int32_t *lv = steps + (int64_t)(step - 1) * bits;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < bits;
         b += (int64_t)gridDim.x * blockDim.x) {
        int32_t off = lv[b], cv = idx[b];
        if (off != -1 && cv != -1 && b + off < bits) idx[b + off] = cv + pw;
    }
}

// calcresult.cl:5-19
__global__ void k_st_calcresult(int64_t bits, const int32_t *idx, const uint8_t *bitdecode,
                                uint8_t *result, uint64_t cap) {
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < bits;
         b += (int64_t)gridDim.x * blockDim.x) {
        int32_t i = idx[b];
        if (i != -1 && (uint64_t)i < cap) result[i] = bitdecode[b];
    }
}

// findmax.cl:2-8 (max-reduction; the serial scan finds the same value)
__global__ void k_st_findmax(int64_t bits, const int32_t *idx, int32_t *maxv) {
    int32_t m = -1;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < bits;
         b += (int64_t)gridDim.x * blockDim.x)
        m = idx[b] > m ? idx[b] : m;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        int32_t y = __shfl_xor(m, o, 64);
        m = y > m ? y : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(maxv, m);
}

__global__ void k_st_flag(const int32_t *steps, int64_t bits, int32_t step, int32_t *out) {
    *out = steps[(int64_t)step * bits];
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct hh_decoder {
    int device;
    hh_config cfg;
    hipStream_t stream;
    hh_tables *ht;
    int have_tree;
    uint64_t *d_l1;
    uint32_t *d_l2;
    uint32_t *d_tree;
    uint8_t *d_tsym;
    DevTab tab;
    uint32_t S;
    // workspace
    void *ws;
    size_t ws_size;
    uint32_t *h_flags;   // pinned
    hipEvent_t ev[4];
    hh_stats stats;
    uint32_t grid;       // persistent grid size (occupancy x CUs)
    size_t grid_l2b;     // dynamic LDS the grid was sized for
    uint64_t *d_dbg;     // per-block phase cycles (HH_STAMPS builds)
};

static int ensure_ws(hh_decoder *d, size_t need) {
    if (d->ws_size >= need) return HH_OK;
    if (d->ws) HIP_OK(hipFree(d->ws));
    d->ws = nullptr;
    d->ws_size = 0;
    size_t sz = need + need / 4;
    if (hipMalloc(&d->ws, sz) != hipSuccess) return HH_ERR_NOMEM;
    d->ws_size = sz;
    return HH_OK;
}

extern "C" int hh_decoder_create(hh_decoder **out, const hh_config *cfg) {
    if (!out) return HH_ERR_ARG;
    *out = nullptr;
    hh_decoder *d = (hh_decoder *)calloc(1, sizeof(hh_decoder));
    if (!d) return HH_ERR_NOMEM;
    if (cfg) d->cfg = *cfg;
    d->device = d->cfg.device;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || d->device >= ndev) {
        free(d);
        return HH_ERR_DEVICE;
    }
    if (hipSetDevice(d->device) != hipSuccess) { free(d); return HH_ERR_DEVICE; }
    d->ht = (hh_tables *)calloc(1, sizeof(hh_tables));
    if (!d->ht) { free(d); return HH_ERR_NOMEM; }
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d->d_l1, sizeof(uint64_t) * HH_L1_SIZE) != hipSuccess ||
        hipMalloc(&d->d_l2, sizeof(uint32_t) * HH_L2_MAX) != hipSuccess ||
        hipMalloc(&d->d_tree, sizeof(uint32_t) * (HH_TREE_MAX + 1)) != hipSuccess ||
        hipMalloc(&d->d_tsym, HH_TREE_MAX + 1) != hipSuccess ||
        hipHostMalloc((void **)&d->h_flags, 64, hipHostMallocDefault) != hipSuccess) {
        hh_decoder_destroy(d);
        return HH_ERR_DEVICE;
    }
    for (int i = 0; i < 4; i++) hipEventCreate(&d->ev[i]);
    *out = d;
    return HH_OK;
}

extern "C" void hh_decoder_destroy(hh_decoder *d) {
    if (!d) return;
    hipSetDevice(d->device);
    if (d->ws) hipFree(d->ws);
    if (d->d_dbg) hipFree(d->d_dbg);
    if (d->d_l1) hipFree(d->d_l1);
    if (d->d_l2) hipFree(d->d_l2);
    if (d->d_tree) hipFree(d->d_tree);
    if (d->d_tsym) hipFree(d->d_tsym);
    if (d->h_flags) hipHostFree(d->h_flags);
    for (int i = 0; i < 4; i++)
        if (d->ev[i]) hipEventDestroy(d->ev[i]);
    if (d->stream) hipStreamDestroy(d->stream);
    free(d->ht);
    free(d);
}

static uint32_t pick_region_bits(const hh_tables *t, int req) {
    if (req > 0) return (uint32_t)req;
    // A region must hold a whole number of code-length periods, or chains
    // of codes whose lengths share a factor (E.coli: all 2 bits) could never
    // meet the true chain.  288 = 2^5 * 3^2 covers gcd 1,2,3,4,6,8,9,...
    uint32_t g = (uint32_t)(t->len_gcd > 0 ? t->len_gcd : 1);
    if (HH_S_DEFAULT % g == 0) return HH_S_DEFAULT;
    if (g <= HH_S_DEFAULT) return g * (HH_S_DEFAULT / g);
    return g <= HH_S_MAX ? g : 0;
}

extern "C" int hh_decoder_set_tree(hh_decoder *d, const hh_tree *tree) {
    if (!d || !tree) return HH_ERR_ARG;
    int rc = hh_tables_build(tree, d->ht);
    if (rc) return rc;
    HIP_OK(hipSetDevice(d->device));
    HIP_OK(hipMemcpy(d->d_l1, d->ht->l1, sizeof(uint64_t) * HH_L1_SIZE, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_l2, d->ht->l2, sizeof(uint32_t) * HH_L2_MAX, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_tree, d->ht->tree, sizeof(uint32_t) * (HH_TREE_MAX + 1), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_tsym, d->ht->tsym, HH_TREE_MAX + 1, hipMemcpyHostToDevice));
    d->tab.l1 = d->d_l1;
    d->tab.l2 = d->d_l2;
    d->tab.tree = d->d_tree;
    d->tab.tsym = d->d_tsym;
    d->tab.l2_used = d->ht->l2_used;
    d->S = pick_region_bits(d->ht, d->cfg.lane_bits);
    d->have_tree = 1;
    return HH_OK;
}

extern "C" int hh_decoder_stats(const hh_decoder *d, hh_stats *st) {
    if (!d || !st) return HH_ERR_ARG;
    *st = d->stats;
    return HH_OK;
}

static inline unsigned grid_for(int64_t n, unsigned bs) {
    int64_t g = (n + bs - 1) / bs;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (unsigned)g;
}

static int fast_path_ok(const hh_decoder *d) {
    return d->S >= 32 && d->S <= HH_S_MAX && d->ht->maxlen <= HH_MAXLEN_FAST &&
           !(d->cfg.flags & HH_FLAG_FORCE_EXACT);
}

static int stage_pipeline(hh_decoder *d, const void *d_data, int64_t bits, uint8_t *d_out,
                          uint64_t cap, uint64_t *out_len, hipStream_t st);

extern "C" int hh_decode_device(hh_decoder *d, const void *d_data, uint64_t bits, void *d_out,
                                uint64_t cap, uint64_t *out_len, void *hip_stream) {
    if (!d || !out_len || (!d_data && bits) || (!d_out && cap)) return HH_ERR_ARG;
    if (!d->have_tree) return HH_ERR_ARG;
    if (((uintptr_t)d_data & 3u) != 0) return HH_ERR_ARG;   // word loads
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : d->stream;
    HIP_OK(hipSetDevice(d->device));
    memset(&d->stats, 0, sizeof(d->stats));
    *out_len = 0;
    if (bits == 0) return HH_OK;
    if (!fast_path_ok(d)) {
        d->stats.exact_fallback = 1;
        return stage_pipeline(d, d_data, (int64_t)bits, (uint8_t *)d_out, cap, out_len, st);
    }
    const uint32_t S = d->S;
    const uint64_t tb = (uint64_t)HH_NR * S;
    const uint64_t ntiles = (bits + tb - 1) / tb;
    const uint64_t nwords_ok = ((bits + 7) / 8 + HH_PAYLOAD_PAD) / 4;
    // workspace: [flags 64 B | counter, gran, incl, xst (zeroed) | tables]
    const size_t zero_bytes = (16 + ntiles * 24 + 15) & ~(size_t)15;
    size_t need = 64 + zero_bytes + ntiles * HH_KM * 8 + 256;
    int rc = ensure_ws(d, need);
    if (rc) return rc;
    uint8_t *w = (uint8_t *)d->ws;
    uint32_t *d_flags = (uint32_t *)w;
    LookBack lb;
    lb.counter = (uint32_t *)(w + 64);
    lb.gran = (uint64_t *)(w + 64 + 16);
    lb.incl = lb.gran + ntiles;
    lb.xst = lb.incl + ntiles;
    lb.tabs = (uint64_t *)(w + 64 + zero_bytes);
    const size_t l2b = sizeof(uint32_t) * d->tab.l2_used;
    if (!d->grid || d->grid_l2b != l2b) {
        int per_cu = 0, ncu = 0;
        HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode, HH_NL, l2b));
        d->grid_l2b = l2b;
        if (d->d_dbg) HIP_OK(hipFree(d->d_dbg));
        HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d->device));
        d->grid = (uint32_t)((per_cu > 0 ? per_cu : 1) * ncu);
        size_t dbg_words = (size_t)d->grid * HH_NDBG;
#ifdef HH_STAMPS
        dbg_words += (size_t)HH_TDBG_MAX * 6;
#endif
        HIP_OK(hipMalloc(&d->d_dbg, dbg_words * sizeof(uint64_t)));
        HIP_OK(hipMemset(d->d_dbg, 0, dbg_words * sizeof(uint64_t)));
    }
    const uint32_t grid = (uint32_t)(ntiles < d->grid ? ntiles : d->grid);

    HIP_OK(hipMemsetAsync(d_flags, 0, 64 + zero_bytes, st));
    HIP_OK(hipEventRecord(d->ev[0], st));
    hipLaunchKernelGGL(k_decode, dim3(grid), dim3(HH_NL), l2b, st, (const uint32_t *)d_data, bits,
                       nwords_ok, S, d->tab, ntiles, lb, (uint8_t *)d_out, cap, d_flags, d->d_dbg);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(d->ev[1], st));
    HIP_OK(hipMemcpyAsync(d->h_flags, d_flags, 16, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    const uint32_t fl = d->h_flags[0];
    const uint64_t total = (uint64_t)d->h_flags[2] | ((uint64_t)d->h_flags[3] << 32);
    float ms = 0;
    hipEventElapsedTime(&ms, d->ev[0], d->ev[1]);
    d->stats.ms_total = ms;
    d->stats.ms_sync = 0;
    d->stats.ms_scan = 0;
    d->stats.ms_emit = ms;
    d->stats.lanes = ntiles * HH_NR;
    d->stats.out_len = total;
    if (fl & F_TIMEOUT) return HH_ERR_TIMEOUT;
    if (fl & F_FAIL) {
        // A walk found no shared boundary within HH_KM regions: the code does
        // not resynchronise (non-synchronising code) -- take the exact path.
        d->stats.exact_fallback = 1;
        return stage_pipeline(d, d_data, (int64_t)bits, (uint8_t *)d_out, cap, out_len, st);
    }
    *out_len = total;
    if (total > cap) return HH_ERR_CAPACITY;
    return HH_OK;
}

extern "C" int hh_decode_host(hh_decoder *d, const uint8_t *data, uint64_t bits, uint8_t *out,
                              uint64_t cap, uint64_t *out_len) {
    if (!d || !out_len || (!data && bits) || (!out && cap)) return HH_ERR_ARG;
    HIP_OK(hipSetDevice(d->device));
    const uint64_t nb = (bits + 7) / 8;
    void *dd = nullptr, *dout = nullptr;
    if (hipMalloc(&dd, nb + HH_PAYLOAD_PAD) != hipSuccess) return HH_ERR_NOMEM;
    uint64_t ocap = cap ? cap : 1;
    if (hipMalloc(&dout, ocap) != hipSuccess) { hipFree(dd); return HH_ERR_NOMEM; }
    int rc = HH_OK;
    if (hipMemsetAsync((uint8_t *)dd + nb, 0, HH_PAYLOAD_PAD, d->stream) != hipSuccess ||
        (nb && hipMemcpyAsync(dd, data, nb, hipMemcpyHostToDevice, d->stream) != hipSuccess))
        rc = HH_ERR_DEVICE;
    if (!rc) rc = hh_decode_device(d, dd, bits, dout, cap, out_len, d->stream);
    if (!rc && *out_len &&
        hipMemcpyAsync(out, dout, *out_len, hipMemcpyDeviceToHost, d->stream) != hipSuccess)
        rc = HH_ERR_DEVICE;
    if (!rc && hipStreamSynchronize(d->stream) != hipSuccess) rc = HH_ERR_DEVICE;
    hipFree(dd);
    hipFree(dout);
    return rc;
}

// ---------------------------------------------------------------------------
// stage API
// ---------------------------------------------------------------------------
extern "C" int hh_stage_initbitsindex(hh_decoder *d, int32_t *idx, int64_t bits, void *s) {
    if (!d || !idx || bits < 0) return HH_ERR_ARG;
    hipLaunchKernelGGL(k_st_init, dim3(grid_for(bits, 256)), dim3(256), 0, (hipStream_t)s, idx, bits);
    HIP_OK(hipGetLastError());
    return HH_OK;
}

extern "C" int hh_stage_decodeallbits(hh_decoder *d, const void *data, int64_t bits,
                                      uint8_t *bitdecode, int32_t *steps, void *s) {
    if (!d || !d->have_tree || !data || !bitdecode || !steps || bits < 0) return HH_ERR_ARG;
    hipLaunchKernelGGL(k_st_decodeallbits, dim3(grid_for(bits, 256)), dim3(256), 0, (hipStream_t)s,
                       (const uint8_t *)data, bits, d->tab, bitdecode, steps);
    HIP_OK(hipGetLastError());
    return HH_OK;
}

extern "C" int hh_stage_makebigtable(hh_decoder *d, int64_t bits, int32_t *steps, int32_t step,
                                     int32_t *flag, void *s) {
    if (!d || !steps || step < 0 || step >= 24) return HH_ERR_ARG;
    hipStream_t st = (hipStream_t)s;
    hipLaunchKernelGGL(k_st_makebigtable, dim3(grid_for(bits, 256)), dim3(256), 0, st, bits, steps, step);
    HIP_OK(hipGetLastError());
    if (flag) {   // the reference's blocking 4-byte read (openclapproach.c:718-727)
        HIP_OK(hipMemcpyAsync(flag, steps + (int64_t)step * bits, 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
    }
    return HH_OK;
}

extern "C" int hh_stage_calcbitsindex(hh_decoder *d, int64_t bits, int32_t *idx, const int32_t *steps,
                                      int32_t step, int32_t pw, void *s) {
    if (!d || !idx || !steps || step < 1) return HH_ERR_ARG;
    hipLaunchKernelGGL(k_st_calcbitsindex, dim3(grid_for(bits, 256)), dim3(256), 0, (hipStream_t)s,
                       bits, idx, steps, step, pw);
    HIP_OK(hipGetLastError());
    return HH_OK;
}

extern "C" int hh_stage_calcresult(hh_decoder *d, int64_t bits, const int32_t *idx,
                                   const uint8_t *bitdecode, uint8_t *result, void *s) {
    if (!d || !idx || !bitdecode || !result) return HH_ERR_ARG;
    hipLaunchKernelGGL(k_st_calcresult, dim3(grid_for(bits, 256)), dim3(256), 0, (hipStream_t)s,
                       bits, idx, bitdecode, result, (uint64_t)bits);
    HIP_OK(hipGetLastError());
    return HH_OK;
}

extern "C" int hh_stage_findmax(hh_decoder *d, int64_t bits, const int32_t *idx, int32_t *maxvalue,
                                void *s) {
    if (!d || !idx || !maxvalue) return HH_ERR_ARG;
    hipStream_t st = (hipStream_t)s;
    int32_t *dm = nullptr;
    HIP_OK(hipMalloc(&dm, 4));
    HIP_OK(hipMemsetAsync(dm, 0xff, 4, st));
    hipLaunchKernelGGL(k_st_findmax, dim3(grid_for(bits, 256)), dim3(256), 0, st, bits, idx, dm);
    HIP_OK(hipMemcpyAsync(maxvalue, dm, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipFree(dm));
    return HH_OK;
}

// The six stages driven like openclApproach (openclapproach.c:236-1047).
static int stage_pipeline(hh_decoder *d, const void *d_data, int64_t bits, uint8_t *d_out,
                          uint64_t cap, uint64_t *out_len, hipStream_t st) {
    *out_len = 0;
    if (bits <= 0) return HH_OK;
    if (bits > 0x7fffffffLL) return HH_ERR_UNSUPPORTED;   // int32 arrays, as the reference
    uint8_t *bitdecode = nullptr, *result = nullptr;
    int32_t *steps = nullptr, *idx = nullptr;
    int rc = HH_OK;
    if (hipMalloc(&bitdecode, bits) != hipSuccess || hipMalloc(&result, bits) != hipSuccess ||
        hipMalloc(&steps, (size_t)25 * bits * 4) != hipSuccess ||
        hipMalloc(&idx, (size_t)bits * 4) != hipSuccess) {
        rc = HH_ERR_NOMEM;
        goto done;
    }
    {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, st);
        if ((rc = hh_stage_initbitsindex(d, idx, bits, st))) goto done;
        if ((rc = hh_stage_decodeallbits(d, d_data, bits, bitdecode, steps, st))) goto done;
        int32_t step = 0, flag = 0;
        do {
            if (step + 1 >= 25) { rc = HH_ERR_UNSUPPORTED; goto done; }
            if ((rc = hh_stage_makebigtable(d, bits, steps, step, &flag, st))) goto done;
            step++;
        } while (flag != -1);
        int32_t pw = 1 << (step - 1);
        const int32_t zero = 0;
        if (hipMemcpyAsync(idx, &zero, 4, hipMemcpyHostToDevice, st) != hipSuccess) {
            rc = HH_ERR_DEVICE;
            goto done;
        }
        while (step > 0) {
            if ((rc = hh_stage_calcbitsindex(d, bits, idx, steps, step, pw, st))) goto done;
            step--;
            pw >>= 1;
        }
        if ((rc = hh_stage_calcresult(d, bits, idx, bitdecode, result, st))) goto done;
        int32_t mx = -1;
        if ((rc = hh_stage_findmax(d, bits, idx, &mx, st))) goto done;
        uint64_t n = (uint64_t)mx + 1;
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        d->stats.ms_total = ms;
        d->stats.out_len = n;
        *out_len = n;
        if (n > cap) { rc = HH_ERR_CAPACITY; goto done; }
        if (n && hipMemcpyAsync(d_out, result, n, hipMemcpyDeviceToDevice, st) != hipSuccess)
            rc = HH_ERR_DEVICE;
        if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = HH_ERR_DEVICE;
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
done:
    hipFree(bitdecode);
    hipFree(result);
    hipFree(steps);
    hipFree(idx);
    return rc;
}

extern "C" int hh_stage_pipeline(hh_decoder *d, const void *d_data, int64_t bits, uint8_t *d_out,
                                 uint64_t cap, uint64_t *out_len, void *s) {
    if (!d || !d->have_tree || !out_len) return HH_ERR_ARG;
    HIP_OK(hipSetDevice(d->device));
    hipStream_t st = s ? (hipStream_t)s : d->stream;
    return stage_pipeline(d, d_data, bits, d_out, cap, out_len, st);
}

// Diagnostic: per-block phase cycle sums of the last decode (HH_STAMPS
// builds; zeros otherwise).  Returns the number of blocks written.
// Diagnostic builds only: per-tile global timestamps (s_memrealtime, 100 MHz)
// [grab, granule published, look-back start, look-back end, block, -].
extern "C" int hh_debug_tile_times(hh_decoder *d, uint64_t *out, int max_tiles) {
#ifdef HH_STAMPS
    if (!d || !out || !d->d_dbg) return 0;
    int n = max_tiles < (int)HH_TDBG_MAX ? max_tiles : (int)HH_TDBG_MAX;
    if (hipMemcpy(out, d->d_dbg + (size_t)d->grid * HH_NDBG, (size_t)n * 6 * sizeof(uint64_t),
                  hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    return n;
#else
    (void)d; (void)out; (void)max_tiles;
    return 0;
#endif
}

extern "C" int hh_debug_phase_cycles(hh_decoder *d, uint64_t *out, int max_blocks) {
    if (!d || !out || !d->d_dbg) return 0;
    int n = (int)d->grid < max_blocks ? (int)d->grid : max_blocks;
    if (hipMemcpy(out, d->d_dbg, (size_t)n * HH_NDBG * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return HH_ERR_DEVICE;
    return n;
}
