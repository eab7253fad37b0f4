// hh_device.hip -- HIP kernels (gfx950) and the device half of the C ABI.
//
// Fast path: ONE persistent launch, k_decode (O(N) memory, 64-bit offsets).
// Workgroups claim tiles in order from a counter.  Per tile of HH_NR regions
// x S bits, pipelined over two tiles (front half of tile n, back half of the
// tile fronted one iteration earlier):
//   stage     the tile's words (+ the next tile's first HH_KM regions and a
//             halo), prefetched into registers one tile ahead, stored to LDS
//             transposed (conflict-free per-lane reads)
//   pass 1    every lane decodes its region from offset 0: count, exit and
//             boundary mask (decodeallbits)
//   walks     each exit is walked against the next regions' chains until
//             they share a boundary: delta (makebigtable)
//   publish   the tile's transfer table (charged count and leaving state for
//             every entering state) as look-back granules
//   look-back decoupled look-back -> entering state and output base
//             (calcbitsindex / findmax), inclusive granule published
//   pass 2    lanes re-decode their exact runs straight to HBM, dword stores
//             (calcresult)
// C is read from HBM once and D written once.
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

#define HH_MAXLEN_FAST 32           // longest code of the fast path (one cursor step <= 32 bits)

#define HIP_OK(x)                                                             \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "hiphuff: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return HH_ERR_DEVICE;                                             \
        }                                                                     \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct DevTab {
    const uint64_t *l1;
    const uint32_t *l2;
    const uint32_t *tree;
    const uint8_t *tsym;
    uint32_t l2_used;
};

// flags[0]: status bits; flags[2..3]: total symbols (u64, last tile)
enum { F_FAIL = 1, F_OVER = 2, F_TIMEOUT = 8 };
// A spin gives up after HH_SPIN_TICKS of the 100 MHz constant clock (4 s):
// wall time, not iterations, so that waves descheduled by another process
// sharing the GPU do not make a correct decode report a timeout.
#define HH_SPIN_TICKS 400000000ull
__device__ __forceinline__ bool spin_expired(uint32_t &spins, uint64_t &t0) {
    if ((++spins & 255u) != 0) return false;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (t0 == 0) { t0 = now; return false; }
    return now - t0 > HH_SPIN_TICKS;
}

struct LookBack {
    uint64_t *agg;       // [ntiles] aggregate granules (table row d = 0 + CONST)
    uint64_t *inc;       // [ntiles] inclusive granules (prefix + resolved state)
    uint64_t *tabs;      // [ntiles][HH_KM] table rows d >= 1 as granules
    uint32_t *agg32;     // [ntiles] compact aggregates (lookback_own)
    uint64_t *tdbg;      // diagnostic (HH_DEBUG_TILES): [ntiles][8] base, size|state, excl, table entry,
                         //   look-back: inclusive tile, its prefix, counts summed, rounds
};

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Diagnostic build only (-DHH_STAMPS): wave 0 of every workgroup adds the
// shader-clock cycles of each phase into dbg[block][phase].
#define HH_NDBG 12
#ifdef HH_STAMPS
#define STAMP_DECL uint64_t st_acc[HH_NDBG] = {0}; uint64_t st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { uint64_t t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } while (0)
#define STAMP_FLUSH(dbg) do { if (threadIdx.x == 0) for (int i_ = 0; i_ < HH_NDBG; i_++) (dbg)[blockIdx.x * HH_NDBG + i_] = st_acc[i_]; } while (0)
#define COUNT(i, v) do { st_acc[i] += (v); } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH(dbg) do {} while (0)
#define COUNT(i, v) do {} while (0)
#endif

// Inclusive wave scan (64 lanes) of u32.
__device__ __forceinline__ int32_t wave_incl_scan(int32_t x) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    return x;
}

// Exclusive block scan of int32 over HH_NL lanes; *total = block sum.
__device__ __forceinline__ int32_t block_excl_scan(int32_t v, int32_t *s_tmp, int32_t *total) {
    constexpr uint32_t NW = HH_NL / 64;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const int32_t x = wave_incl_scan(v);
    if (lane == 63) s_tmp[wv] = x;
    __syncthreads();
    int32_t base = 0, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < NW; i++) {
        const int32_t t = s_tmp[i];
        base += i < wv ? t : 0;
        tot += t;
    }
    *total = tot;
    __syncthreads();
    return base + x - v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// Poll a granule until its status bits are non-zero (bounded).
// A timeout sets F_TIMEOUT and *to; the caller then emits nothing.
__device__ __forceinline__ uint64_t poll_granule(const uint64_t *p, uint32_t *flags, bool *to) {
    uint64_t v, t0 = 0;
    uint32_t spins = 0;
    while (((v = ld_sc1(p)) >> HH_ST_SHIFT) == 0) {
        __builtin_amdgcn_s_sleep(1);
        if (spin_expired(spins, t0)) {
            atomicOr(flags, (uint32_t)F_TIMEOUT);
            *to = true;
            return HH_AGG;   // zero count: the decode is reported as failed
        }
    }
    return v;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// State entering tile t: the leaving state of tile t-1, read from its
// aggregate when that is CONST (the common case: available as soon as t-1's
// walks are done), else from its inclusive granule (t-1 resolved its own
// entering state first).
__device__ uint32_t entering_state(const LookBack &lb, uint64_t t, uint32_t in_state, uint32_t *flags,
                                   bool *to) {
    if (t == 0) return in_state;
    const uint64_t g = poll_granule(&lb.agg[t - 1], flags, to);
    if (g & HH_CST) return hh_tab_state(g);
    return hh_inc_state(poll_granule(&lb.inc[t - 1], flags, to));
}

// Exclusive charged prefix of tile t (t >= 1), one wave, 64 x HH_LBV
// predecessors per round; the nearest inclusive granule ends the look-back.
// Tile u counts with its table row for the state entering it: that state
// comes from the inclusive of u-1 if that is the nearest one, else from
// u-1's aggregate, which must be CONST (otherwise wait until an inclusive
// granule appears closer); row 0 is u's aggregate, rows d > 0 are granules
// of their own.
#ifndef HH_LBV
#define HH_LBV 2   // tiles per lane per look-back round (128-tile window). Same-box A/B on
                   // the 1 GiB stream: 1 -> 5.75 ms, 2 -> 5.67 ms, 4 -> 5.83 ms; 8 costs 28 VGPRs
#endif
__device__ uint64_t lookback_excl(const LookBack &lb, uint64_t t, uint32_t in_state, uint64_t emit_from,
                                  uint32_t *flags, bool *to) {
    constexpr uint32_t V = HH_LBV;
    const uint32_t lane = threadIdx.x & 63u;
    // tile -1: a CONST aggregate leaving in_state; its inclusive value is
    // the entry correction (so that tile 0's output base is 0), unless a
    // prologue carries it (see the table rows of prologue tiles)
    const uint64_t st0 = HH_AGG | HH_CST | hh_tab_pack(0, in_state);
    const uint64_t in0 = hh_inc_pack(emit_from ? 0ull : (uint64_t)(int64_t)hh_state_delta(in_state), in_state);
    uint64_t excl = 0;
    int64_t top = (int64_t)t - 1;
    uint32_t rounds = 0;
    for (;;) {
        // this lane: tiles ub, ub-1, ..., ub-V+1 (window offsets lane*V + i)
        const int64_t ub = top - (int64_t)(lane * V);
        uint64_t iv[V], av[V + 1];
        uint32_t ofirst, spins = 0, lf;
        uint64_t incv, t0 = 0;
        int64_t csum = 0;
        for (;;) {
#pragma unroll
            for (uint32_t i = 0; i <= V; i++) {
                const int64_t u = ub - (int64_t)i;
                if (i < V) iv[i] = u >= 0 ? ld_sc1(&lb.inc[u]) : in0;
                av[i] = u >= 0 ? ld_sc1(&lb.agg[u]) : st0;
            }
            lf = V;
#pragma unroll
            for (int i = (int)V - 1; i >= 0; i--)
                if ((iv[i] >> HH_ST_SHIFT) == 2) lf = (uint32_t)i;
            const uint64_t m = __ballot(lf < V);
            const uint32_t fl = m ? (uint32_t)__builtin_ctzll(m) : 64u;
            const uint32_t lff = (uint32_t)__shfl((int)lf, (int)(fl & 63u), 64);
            ofirst = fl < 64 ? fl * V + lff : 64u * V;
            // the nearest inclusive granule (value and resolved state)
            uint64_t myinc = 0;
#pragma unroll
            for (uint32_t i = 0; i < V; i++) if (i == lf) myinc = iv[i];
            incv = shfl64(myinc, (int)(fl & 63u));
            bool ok = true;
            csum = 0;
#pragma unroll
            for (uint32_t i = 0; i < V; i++) {
                const uint32_t o = lane * V + i;
                if (o < ofirst) {
                    // pinned to the inclusive granule found (none in this
                    // window: the last tile's state comes from its
                    // predecessor's aggregate, av[V], like every other)
                    const bool pin = o + 1 == ofirst && ofirst < 64u * V;
                    const uint64_t pv = av[i + 1];
                    const bool known = pin || ((pv >> HH_ST_SHIFT) != 0 && (pv & HH_CST));
                    const uint32_t d = hh_state_d(pin ? hh_inc_state(incv) : hh_tab_state(pv));
                    // entered with d > 0: that row of the tile's table (a granule)
                    uint64_t row = av[i];
                    if (known && d != 0) row = ld_sc1(&lb.tabs[(uint64_t)(ub - (int64_t)i) * HH_KM + d]);
                    ok = ok && (av[i] >> HH_ST_SHIFT) != 0 && known && (row >> HH_ST_SHIFT) != 0;
                    csum += hh_tab_count(row);
                }
            }
            if (!__ballot(!ok)) break;
            __builtin_amdgcn_s_sleep(1);
            if (spin_expired(spins, t0)) {
                if (lane == 0) atomicOr(flags, (uint32_t)F_TIMEOUT);
                *to = true;
                return 0;
            }
        }
        excl += wave_sum64((uint64_t)csum);
        rounds++;
        if (ofirst < 64u * V) {
            const uint64_t pre = hh_inc_prefix(incv);
            if (lb.tdbg && lane == 0) {
                lb.tdbg[t * 8 + 4] = (uint64_t)(top - (int64_t)ofirst);
                lb.tdbg[t * 8 + 5] = pre;
                lb.tdbg[t * 8 + 6] = excl;
                lb.tdbg[t * 8 + 7] = rounds;
            }
            return excl + pre;
        }
        top -= (int64_t)(64u * V);
    }
}

// Look-back that ends at this workgroup's previous tile pt (< t), whose
// inclusive value and leaving state it computed itself: the tiles between
// (the ones the other workgroups claimed meanwhile, about G - 1 of them)
// need only their aggregates, all loaded in one round -- no inclusive
// granules, no second window.  Returns false (the caller takes the general
// look-back) when the gap is wider than 64 * HH_LBO or a tile's entering
// state cannot be read from a CONST aggregate.
#define HH_LBO 12
#ifndef HH_USE_OWN
#define HH_USE_OWN 0   // measured at 512 lanes: 6.23 vs 5.83 ms (register pressure); kept for study
#endif
// compact aggregate (u32): bit 31 published, bit 30 CONST, bits 26..29 the
// leaving state's region d, bits 0..19 the charged count of row d = 0
__device__ __forceinline__ uint32_t agg32_pack(uint64_t row0, bool cst) {
    return 0x80000000u | (cst ? 0x40000000u : 0u) | (hh_state_d(hh_tab_state(row0)) << 26) |
           ((uint32_t)hh_tab_count(row0) & 0xfffffu);
}
__device__ __forceinline__ int32_t agg32_count(uint32_t a) { return (int32_t)(a << 12) >> 12; }

__device__ bool lookback_own(const LookBack &lb, uint64_t t, uint64_t pt, uint64_t p_incl,
                             uint32_t p_state, uint32_t *flags, uint64_t *excl, uint32_t *st_in,
                             bool *to) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t W = t - pt - 1;                  // tiles strictly between
    if (W > 64u * HH_LBO) return false;
    uint32_t av[HH_LBO];
    uint64_t a0 = 0, t0 = 0;                        // a0: full aggregate of tile t-1
    uint32_t spins = 0;
    for (;;) {
        if (W) a0 = ld_sc1(&lb.agg[t - 1]);
#pragma unroll
        for (uint32_t i = 0; i < HH_LBO; i++) {
            const uint64_t o = (uint64_t)lane * HH_LBO + i;     // tile t-1-o
            av[i] = o < W ? __hip_atomic_load(&lb.agg32[t - 1 - o], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                          : 0x80000000u;
        }
        bool ready = W == 0 || (a0 >> HH_ST_SHIFT) != 0;
#pragma unroll
        for (uint32_t i = 0; i < HH_LBO; i++) ready = ready && (av[i] >> 31) != 0;
        if (!__ballot(!ready)) break;
        __builtin_amdgcn_s_sleep(1);
        if (spin_expired(spins, t0)) {
            if (lane == 0) atomicOr(flags, (uint32_t)F_TIMEOUT);
            *to = true;
            *excl = 0;
            *st_in = 0;
            return true;
        }
    }
    const uint32_t nxt = (uint32_t)__shfl((int)av[0], (int)((lane + 1) & 63u));   // tile below lane's last
    bool ok = true;
    int32_t csum = 0;
    uint64_t rows = 0;                              // 4 bits per tile: the row d != 0 to fetch
#pragma unroll
    for (uint32_t i = 0; i < HH_LBO; i++) {
        const uint64_t o = (uint64_t)lane * HH_LBO + i;
        if (o < W) {
            const bool oldest = o + 1 == W;                     // entered from tile pt
            const uint32_t pv = i + 1 < HH_LBO ? av[i + 1 < HH_LBO ? i + 1 : 0] : nxt;
            const bool known = oldest || (pv & 0x40000000u);
            const uint32_t d = oldest ? hh_state_d(p_state) : (pv >> 26) & 0xfu;
            ok = ok && known;
            if (d == 0) csum += agg32_count(av[i]);
            else rows |= (uint64_t)d << (4 * i);
        }
    }
    if (__ballot(!ok)) return false;
    while (rows) {                                  // tiles entered with d > 0: rare
        const uint32_t i = (uint32_t)__builtin_ctzll(rows) / 4;
        const uint32_t d = (uint32_t)(rows >> (4 * i)) & 0xfu;
        rows &= ~(0xfull << (4 * i));
        const uint64_t o = (uint64_t)lane * HH_LBO + i;
        csum += hh_tab_count(poll_granule(&lb.tabs[(t - 1 - o) * HH_KM + d], flags, to));
    }
    if (W == 0) {
        *st_in = p_state;
    } else if (a0 & HH_CST) {
        *st_in = hh_tab_state(a0);
    } else {
        return false;
    }
    *excl = p_incl + wave_sum64((uint64_t)(int64_t)csum);
    return true;
}

// Stream word gi, zero past the readable payload.
__device__ __forceinline__ uint32_t ld_word(const uint32_t *g, uint64_t gi, uint64_t nok) {
    return gi < nok ? __builtin_nontemporal_load(&g[gi]) : 0u;
}

// Registers holding one tile's words for this lane: its region column and,
// for lanes < (HH_NCOL - HH_NR) * sw, one word of the columns past the tile
// (the next tile's first HH_KM regions and the halo).
#define HH_XW ((HH_NCOL - HH_NR) * HH_SW_MAX)
static_assert(HH_XW <= HH_NL, "extra columns must fit one word per lane");
struct Prefetch {
    uint32_t v[HH_SW_MAX];
    uint32_t halo;
};

template <uint32_t sw>
__device__ __forceinline__ void prefetch_tile(Prefetch &pf, const uint32_t *g, uint64_t tw0,
                                              uint64_t nok, bool vec4) {
    const uint32_t j = threadIdx.x;
    const uint64_t gi = tw0 + (uint64_t)j * sw;
    if (sw % 4 == 0 && vec4 && gi + HH_SW_MAX <= nok) {
#pragma unroll
        for (uint32_t k = 0; k < HH_SW_MAX; k += 4) {
            if (k < sw) {
                const u32x4 q = __builtin_nontemporal_load((const u32x4 *)(g + gi + k));
                pf.v[k] = q.x; pf.v[k + 1] = q.y; pf.v[k + 2] = q.z; pf.v[k + 3] = q.w;
            }
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < HH_SW_MAX; k++)
            if (k < sw) pf.v[k] = ld_word(g, gi + k, nok);
    }
    pf.halo = j < (HH_NCOL - HH_NR) * sw ? ld_word(g, tw0 + (uint64_t)HH_NR * sw + j, nok) : 0u;
}

template <uint32_t sw>
__device__ __forceinline__ void store_tile(const Prefetch &pf, uint32_t *s_w) {
    const uint32_t j = threadIdx.x;
#pragma unroll
    for (uint32_t k = 0; k < HH_SW_MAX; k++)
        if (k < sw) s_w[k * HH_NLS + j] = pf.v[k];
    if (j < (HH_NCOL - HH_NR) * sw) s_w[(j % sw) * HH_NLS + HH_NR + j / sw] = pf.halo;
}

// The walks with k > 1 (exceptions) of a tile, ascending, into s_exc.
__device__ __forceinline__ uint32_t collect_exceptions(bool is_exc, uint16_t *s_exc, uint32_t *s_cnt) {
    constexpr uint32_t NW = HH_NL / 64;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t m = __ballot(is_exc);
    if (lane == 0) s_cnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < NW; i++) {
        off += i < wv ? s_cnt[i] : 0u;
        tot += s_cnt[i];
    }
    if (is_exc) {
        const uint64_t below = lane ? (m & ((1ull << lane) - 1ull)) : 0ull;
        s_exc[off + (uint32_t)__popcll(below)] = (uint16_t)threadIdx.x;
    }
    __syncthreads();
    return tot;
}

__device__ __forceinline__ int32_t wave_sum(int32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------------------
// k_decode
// ---------------------------------------------------------------------------
struct Geometry {
    uint64_t bits;       // stream length
    uint64_t nwords;     // readable payload words
    uint64_t ntiles;
    uint32_t S, sw, magic;
    uint32_t vec4;       // 16-B aligned payload and sw % 4 == 0
    uint32_t maxadv;     // max(HH_P, longest code)
    uint32_t in_state;   // state entering tile 0 (a shard's entry; 0 at the stream start)
    uint64_t emit_from;  // tiles before this one are a prologue: decoded for their
                         // leaving state only (a shard's probe of its predecessor)
};

// Per-lane results of a tile's front half, kept in registers until its back
// half (one iteration later).
struct LaneRec {
    uint32_t n;          // own-chain symbols in the region (pass 1)
    uint32_t k, e, cov;  // walk: regions crossed, entry offset, covered symbols
    int32_t delta;       // walk correction
};

template <uint32_t SW>
// Tile buffers.  2: the front half of tile n runs before the back half of
// tile n-1 (the look-back of n-1 waits less), words, live masks and tables
// double-buffered.  1: back half first, one buffer each -- 9 KiB less LDS per
// workgroup, 4 workgroups per CU instead of 3.
#ifndef HH_NBUF
#define HH_NBUF 2
#endif
#ifndef HH_MINBLK
#define HH_MINBLK 4   // waves per SIMD the register budget is sized for (<= 128 VGPRs)
#endif
__global__ __launch_bounds__(HH_NL, HH_MINBLK) void k_decode(const uint32_t *__restrict__ gdata, Geometry geo,
                                                     DevTab tab, LookBack lb,
                                                     uint8_t *__restrict__ out, uint64_t cap,
                                                     uint32_t *flags, uint64_t *dbg) {
    extern __shared__ __align__(16) uint8_t smem[];
    __shared__ uint32_t s_ein[HH_NL];          // run entries pushed by walkers
    __shared__ int16_t s_din[HH_NL];           // their deltas
    __shared__ uint16_t s_exc[HH_NL];          // exception lanes (k > 1)
    __shared__ uint8_t s_mem[HH_NBUF][HH_NL];        // live masks over entering d (per pending tile)
    __shared__ uint8_t s_k[HH_NL];
    __shared__ int32_t s_part[HH_NL / 64][HH_KM];
    __shared__ int32_t s_cd[HH_KM];            // per-d counts of the partially live lanes
    __shared__ uint32_t s_ost[HH_KM];
    __shared__ uint64_t s_tab[HH_NBUF][HH_KM];       // transfer table (per pending tile)
    __shared__ int32_t s_tmp[HH_NL / 64];
    __shared__ uint32_t s_cnt[HH_NL / 64];
    __shared__ uint64_t s_bc[4];
    __shared__ uint64_t s_own[3];              // this workgroup's last completed tile: index,
                                               //   inclusive value, leaving state
    __shared__ uint32_t s_x[HH_NR];            // pass-1 exits and counts of the front tile
    __shared__ uint16_t s_n[HH_NR];

    constexpr uint32_t S = 32 * SW;
    uint32_t *s_l1m = (uint32_t *)smem;                          // L1 meta halves
    uint32_t *s_l1s = s_l1m + HH_L1_SIZE;                        // L1 symbol halves
    uint32_t *s_wb = (uint32_t *)(smem + HH_L1_SIZE * 8);       // HH_NBUF x SW * HH_NLS words
    uint32_t *s_mk = s_wb + HH_NBUF * SW * HH_NLS;               // SW * HH_NLS boundary-mask words
    uint32_t *s_l2 = s_mk + SW * HH_NLS;

    const uint32_t j = threadIdx.x;
    const uint64_t tile_bits = (uint64_t)HH_NR * S;
    const uint32_t span = HH_NCOL * S;          // bits staged per tile
    STAMP_DECL

    for (uint32_t i = j; i < HH_L1_SIZE; i += HH_NL) {
        const uint64_t e = tab.l1[i];
        s_l1m[i] = (uint32_t)(e >> 32);
        s_l1s[i] = (uint32_t)e;
    }
    for (uint32_t i = j; i < tab.l2_used; i += HH_NL) s_l2[i] = tab.l2[i];
    if (j == 0) s_own[0] = ~0ull;

    hh_ctx c;
    c.sw = SW;
    c.magic = 0;
    c.l1m = s_l1m;
    c.l1s = s_l1s;
    c.l2 = s_l2;
    c.tree = tab.tree;
    c.tsym = tab.tsym;
    c.maxadv = geo.maxadv;

    // Every tile is claimed in order from a counter, one iteration before its
    // front half (the first two per workgroup together), so the predecessors
    // of a tile entering its back half were claimed earlier by running
    // workgroups and normally have their aggregates published: no convoy
    // behind a slow workgroup as with a fixed stride, and no dependence on
    // which workgroups are resident (a GPU shared with another process).
    // HH_NBUF 1 claims one tile at a time, at the end of a front half: the
    // tile is fronted in the next iteration, right after one back half, so a
    // back half never waits on a chain of fronts queued behind other backs.
    if (j == 0) s_bc[2] = atomicAdd((unsigned long long *)(flags + 10), (unsigned long long)HH_NBUF);
    __syncthreads();
    Prefetch pf;
    uint64_t tn = s_bc[2];                      // tile for the next front half
    uint64_t tq = tn + 1;                       // (HH_NBUF 2) tile prefetched during that front half
    if (tn < geo.ntiles) prefetch_tile<SW>(pf, gdata, tn * tile_bits / 32, geo.nwords, geo.vec4);

    uint32_t cst_seen = 0;                      // lane 0: bit 0 prologue, bit 1 emitted tiles
    LaneRec rp = {0u, 1u, 0u, 0u, 0};           // the pending tile (front done)
    uint64_t tp = ~0ull;
    uint32_t par = 0;                           // buffer parity of the next front half

    for (;;) {
        const bool front = tn < geo.ntiles, back = tp < geo.ntiles;
        if (!front && !back) break;
        LaneRec rn = rp;
        __syncthreads();                        // buffer `par` no longer read by a back half
        const uint32_t fb = HH_NBUF == 2 ? par : 0u, pb = HH_NBUF == 2 ? par ^ 1u : 0u;
        auto front_half = [&]() {
            // ---------------- front half of tile tn ----------------
            uint32_t *s_w = s_wb + fb * SW * HH_NLS;
            c.w = s_w;
            const uint64_t rem = geo.bits - tn * tile_bits;
            c.bt = rem < span ? (uint32_t)rem : span;
            const uint32_t bt = c.bt;
            store_tile<SW>(pf, s_w);
            if (HH_NBUF == 2 && tq < geo.ntiles)
                prefetch_tile<SW>(pf, gdata, tq * tile_bits / 32, geo.nwords, geo.vec4);
            __syncthreads();
            STAMP(0);

            // pass 1: own region from offset 0
            const uint32_t p0 = j * S;
            uint32_t n = 0, x = bt;
            if (p0 < bt) {
                const uint32_t lim = p0 + S < bt ? p0 + S : bt;
                x = hh_region_count(&c, p0, lim, &n, s_mk);
            }
            s_x[j] = x;
            s_n[j] = (uint16_t)n;
            __syncthreads();
            STAMP(1);

            // walks: region j's exit against the next regions' own chains
            const hh_wk wk = hh_walk(&c, j, S, x, s_mk, s_x, s_n, HH_NR);
            if (wk.k == 0) {
                atomicOr(flags, (uint32_t)F_FAIL);
                if (atomicCAS(&flags[4], 0u, 1u) == 0u) {
                    flags[5] = (uint32_t)tn; flags[6] = j; flags[7] = x; flags[8] = n; flags[9] = bt;
                }
            }
            const uint32_t kk = wk.k ? wk.k : 1u;
            s_k[j] = (uint8_t)kk;
            s_mem[fb][j] = (uint8_t)hh_mem_init(j);
            STAMP(2);

            // transfer table: live masks (exceptions, ascending, by one lane),
            // charged count and leaving state for every entering d
            if (j < HH_KM) s_cd[j] = 0;
#ifdef HH_STAMPS
            __syncthreads();
            STAMP(7);
#endif
            // claim the tile after tq now; the claim's latency hides behind the table
            uint64_t claim = 0;
            if (j == 0 && (HH_NBUF == 1 || tq < geo.ntiles))
                claim = atomicAdd((unsigned long long *)(flags + 10), 1ull);
            const uint32_t nexc = collect_exceptions(kk > 1, s_exc, s_cnt);   // barriers inside
            if (j == 0) {
                for (uint32_t i = 0; i < nexc; i++) {
                    const uint32_t e = s_exc[i], ke = s_k[e];
                    const uint8_t m = s_mem[fb][e];
                    for (uint32_t q = e + 1; q < e + ke && q < HH_NR; q++) s_mem[fb][q] &= (uint8_t)~m;
                }
            }
            __syncthreads();
            const uint32_t mem = s_mem[fb][j];
            const int32_t charged = (int32_t)(n + wk.cov) + wk.delta;
            if (j + kk >= HH_NR) {
                const uint32_t os = hh_state_pack(j + kk - HH_NR, wk.e, wk.delta);
#pragma unroll
                for (uint32_t d = 0; d < HH_KM; d++)
                    if ((mem >> d) & 1u) s_ost[d] = os;
            }
            // lanes live for every entering d: one block sum; the few others
            // (lanes < HH_KM, covered lanes): per-d LDS atomics
            const uint32_t full = (1u << HH_KM) - 1u;
            const int32_t v = wave_sum(mem == full ? charged : 0);
            if ((j & 63u) == 0) s_part[j >> 6][0] = v;
            if (mem != full) {
#pragma unroll
                for (uint32_t d = 0; d < HH_KM; d++)
                    if ((mem >> d) & 1u) atomicAdd(&s_cd[d], charged);
            }
            __syncthreads();
            if (j < HH_KM) {
                int32_t cnt = s_cd[j];
#pragma unroll
                for (uint32_t w = 0; w < HH_NL / 64; w++) cnt += s_part[w][0];
                // a prologue tile emits nothing; the last one charges the
                // entry correction of the first emitted tile instead
                if (tn < geo.emit_from) cnt = tn + 1 == geo.emit_from ? hh_state_delta(s_ost[j]) : 0;
                const uint64_t row = hh_tab_pack(cnt, s_ost[j]);
                s_tab[fb][j] = row;
                if (j > 0) st_sc1(&lb.tabs[tn * HH_KM + j], HH_AGG | row);
            }
            __syncthreads();
            if (j == 0) {
                // aggregate = table row d = 0 (+ CONST: the leaving state is
                // the same for every entering d)
                bool cst = true;
                for (uint32_t d = 1; d < HH_KM; d++)
                    cst = cst && hh_tab_state(s_tab[fb][d]) == hh_tab_state(s_tab[fb][0]);
                st_sc1(&lb.agg[tn], HH_AGG | (cst ? HH_CST : 0ull) | s_tab[fb][0]);
                __hip_atomic_store(&lb.agg32[tn], agg32_pack(s_tab[fb][0], cst), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                cst_seen |= cst ? (tn < geo.emit_from ? 1u : 2u) : 0u;
                if (HH_NBUF == 1 || tq < geo.ntiles) s_bc[2] = claim;
            }
            rn.n = n; rn.k = kk; rn.e = wk.e; rn.cov = wk.cov; rn.delta = wk.delta;
            STAMP(3);
        };

        auto back_half = [&]() {
            // ---------------- back half of tile tp ----------------
            c.w = s_wb + pb * SW * HH_NLS;
            const uint64_t rem = geo.bits - tp * tile_bits;
            c.bt = rem < span ? (uint32_t)rem : span;
            const uint32_t bt = c.bt;
            // the state entering tp (from tp-1's aggregate, or its inclusive
            // granule) and tp's exclusive prefix (decoupled look-back), wave 0
            if (j < 64) {
#ifdef HH_STAMPS
                const uint64_t q0 = __builtin_amdgcn_s_memtime();
#endif
                uint32_t sti = 0;
                uint64_t excl = 0;
                bool to = false;                // a spin timed out: emit nothing
                const uint64_t own_t = s_own[0];
                if (!(HH_USE_OWN && own_t != ~0ull &&
                      lookback_own(lb, tp, own_t, s_own[1], (uint32_t)s_own[2], flags, &excl, &sti, &to))) {
                    sti = entering_state(lb, tp, geo.in_state, flags, &to);
                    excl = tp > 0 ? lookback_excl(lb, tp, geo.in_state, geo.emit_from, flags, &to)
                                  : (geo.emit_from ? 0ull : (uint64_t)(int64_t)hh_state_delta(geo.in_state));
                }
#ifdef HH_STAMPS
                COUNT(9, __builtin_amdgcn_s_memtime() - q0);
                COUNT(10, 1);
#endif
                const uint64_t tab_w = s_tab[pb][hh_state_d(sti)];
                const uint64_t incl = excl + (uint64_t)(int64_t)hh_tab_count(tab_w);
                const bool any_to = __ballot(to) != 0;
                if (j == 0) {
                    st_sc1(&lb.inc[tp], hh_inc_pack(incl, hh_tab_state(tab_w)));
                    s_own[0] = tp;
                    s_own[1] = incl;
                    s_own[2] = hh_tab_state(tab_w);
                    s_bc[0] = sti;
                    s_bc[1] = excl - (uint64_t)(int64_t)hh_state_delta(sti);   // output base
                    s_bc[3] = any_to ? 1u : 0u;
                    if (tp == geo.ntiles - 1) flags[14] = hh_tab_state(tab_w);
                    if (tp == geo.emit_from) flags[15] = sti;
                    if (lb.tdbg) {
                        lb.tdbg[tp * 8 + 2] = excl;
                        lb.tdbg[tp * 8 + 3] = tab_w;
                    }
                }
            }
            __syncthreads();
            const uint32_t mem = s_mem[pb][j];
            const uint32_t st_in = (uint32_t)s_bc[0];
            const uint32_t d_t = hh_state_d(st_in);
            const int32_t dprev = hh_state_delta(st_in);
            const bool live = (mem >> d_t) & 1u;
            if (live && j + rp.k < HH_NR) {
                s_ein[j + rp.k] = (j + rp.k) * S + rp.e;
                s_din[j + rp.k] = (int16_t)rp.delta;
            }
            __syncthreads();
            STAMP(4);
            const uint32_t e_in = j == d_t ? d_t * S + hh_state_e(st_in) : s_ein[j];
            const int32_t d_in = j == d_t ? dprev : (int32_t)s_din[j];
            const uint32_t rc = live && tp >= geo.emit_from ? (uint32_t)((int32_t)(rp.n + rp.cov) + d_in) : 0u;
            int32_t Tout_i;
            const uint32_t L = (uint32_t)block_excl_scan((int32_t)rc, s_tmp, &Tout_i);   // barriers inside
            const uint32_t Tout = (uint32_t)Tout_i;
            const uint64_t P0 = s_bc[1];
            // the tile's output fits [0, cap) (no wrap-around), and every
            // granule it was based on arrived
            const bool fits = P0 <= cap && Tout <= cap - P0 && s_bc[3] == 0;
            if (j == 0) {
                if (tp == geo.ntiles - 1) {
                    const uint64_t tot = P0 + Tout;
                    flags[2] = (uint32_t)tot;
                    flags[3] = (uint32_t)(tot >> 32);
                }
                if (tp >= geo.emit_from && !fits) atomicOr(flags, (uint32_t)F_OVER);
                if (lb.tdbg) {
                    lb.tdbg[tp * 8 + 0] = P0;
                    lb.tdbg[tp * 8 + 1] = Tout | ((uint64_t)st_in << 32);
                }
            }
            STAMP(5);

            // pass 2: this lane's symbols, straight to HBM (output bytes
            // [P0 + L, P0 + L + rc)); bytes up to a dword boundary, then
            // dwords, then the ragged end
            hh_cur cu = hh_cur_at(&c, live ? e_in : 0u);
            const uint32_t y = (j + rp.k) * S + rp.e;
            const uint32_t pe = (live && tp >= geo.emit_from && fits) ? (y < bt ? y : bt) : 0u;
            if (cu.p < pe) {
                uint8_t *ob = out + P0;
                uint32_t o = L, val, k;
                const uint32_t oend = L + rc;
                while (((P0 + o) & 3u) && cu.p < pe) {
                    const uint32_t ha = o + (4u - (uint32_t)((P0 + o) & 3u));
                    hh_emit_step(&c, cu, pe, o, ha, &val, &k);
                    for (uint32_t i = 0; i < k; i++) ob[o + i] = (uint8_t)(val >> (8 * i));
                    o += k;
                }
                uint64_t acc = 0;
                uint32_t nacc = 0;
                // whole lookups while the longest possible one still ends by pe
                const uint32_t pf = pe > geo.maxadv ? pe - geo.maxadv : 0u;
                while (cu.p < pf) {
                    const uint32_t win = hh_cur_win(cu);
                    const uint32_t ix = win & (HH_L1_SIZE - 1u);
                    const uint32_t m = c.l1m[ix];
                    uint32_t sy = c.l1s[ix], ns = HH_M_NSYM(m), nb = HH_M_NBITS(m);
                    if (ns == 0) {
                        nb = hh_escape(&c, cu.p, win, &sy);
                        ns = 1;
                    }
                    acc |= (uint64_t)sy << (8 * nacc);
                    nacc += ns;
                    if (nacc >= 4) {
                        *(uint32_t *)(ob + o) = (uint32_t)acc;
                        acc >>= 32;
                        nacc -= 4;
                        o += 4;
                    }
                    hh_cur_adv(&c, cu, nb);
                }
                while (cu.p < pe) {
                    hh_emit_step(&c, cu, pe, o + nacc, oend, &val, &k);
                    acc |= (uint64_t)val << (8 * nacc);
                    nacc += k;
                    if (nacc >= 4) {
                        *(uint32_t *)(ob + o) = (uint32_t)acc;
                        acc >>= 32;
                        nacc -= 4;
                        o += 4;
                    }
                }
                for (uint32_t i = 0; i < nacc; i++) ob[o + i] = (uint8_t)(acc >> (8 * i));
            }
            STAMP(6);
        };
#if HH_NBUF == 2
        if (front) front_half();
        if (back) back_half();
#else
        if (back) back_half();
        __syncthreads();                        // tile tp's words and tables no longer read
        if (front) front_half();
#endif
        // the front half's tile becomes the pending one
        rp = rn;
        tp = front ? tn : ~0ull;
        if (front) {
            __syncthreads();                    // s_bc[2] (claimed by lane 0) visible
            if (HH_NBUF == 2) {
                tn = tq;
                tq = tq < geo.ntiles ? s_bc[2] : tq;
            } else {
                tn = s_bc[2];
                if (tn < geo.ntiles) prefetch_tile<SW>(pf, gdata, tn * tile_bits / 32, geo.nwords, geo.vec4);
            }
        }
        par ^= 1u;
    }
    // CONST tables seen (prologue / emitted): one store per workgroup
    if (j == 0) {
        if (cst_seen & 1u) flags[12] = 1u;
        if (cst_seen & 2u) flags[13] = 1u;
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
typedef void (*kdec_t)(const uint32_t *, Geometry, DevTab, LookBack, uint8_t *, uint64_t, uint32_t *,
                       uint64_t *);

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
    size_t grid_lds;     // dynamic LDS the grid was sized for
    kdec_t grid_kf;      // and the kernel instance
    uint64_t *d_dbg;     // per-block phase cycles (HH_STAMPS builds)
    uint64_t last_ntiles;
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
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || d->device < 0 || d->device >= ndev) {
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
    uint32_t g = (uint32_t)(t->len_gcd > 0 ? t->len_gcd : 1);
    if (req > 0) {
        // a requested size must keep whole words; off the code lattice it is
        // still exact (walks that cannot merge report failure), only slower
        if (req % 32 || req > 32 * HH_SW_MAX) return 0;
        return (uint32_t)req;
    }
    return hh_pick_region_bits(g);
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
    return d->S >= 32 && d->S <= 32 * HH_SW_MAX && d->ht->maxlen <= HH_MAXLEN_FAST &&
           !(d->cfg.flags & HH_FLAG_FORCE_EXACT);
}

static int stage_pipeline(hh_decoder *d, const void *d_data, int64_t bits, uint8_t *d_out,
                          uint64_t cap, uint64_t *out_len, hipStream_t st);

static size_t lds_bytes(const hh_decoder *d) {
    // HH_LDS_PAD_KIB: experiment knob (fewer workgroups per CU)
    static const size_t pad = getenv("HH_LDS_PAD_KIB") ? (size_t)atoi(getenv("HH_LDS_PAD_KIB")) << 10 : 0;
    return (size_t)HH_L1_SIZE * 8 + (HH_NBUF + 1) * (size_t)(d->S / 32) * HH_NLS * 4 +
           (size_t)d->tab.l2_used * 4 + pad;
}

// k_decode instantiated per words-per-region (S = 32 * SW bits)
static kdec_t kdec_for(uint32_t sw) {
    switch (sw) {
    case 1: return k_decode<1>;
    case 2: return k_decode<2>;
    case 3: return k_decode<3>;
    case 4: return k_decode<4>;
    case 5: return k_decode<5>;
    case 6: return k_decode<6>;
    case 7: return k_decode<7>;
    case 8: return k_decode<8>;
    case 9: return k_decode<9>;
    case 10: return k_decode<10>;
    case 11: return k_decode<11>;
    case 12: return k_decode<12>;
    default: return nullptr;
    }
}

// Workgroups that can be resident at once (the persistent grid): the
// occupancy answer, capped by the SGPR rule of MI355X_MICROARCH.md
// ("Residency and cooperative launch") for one-block-per-CU-group sizing.
static int size_grid(hh_decoder *d, size_t lds, kdec_t kf) {
    if (d->grid && d->grid_lds == lds && d->grid_kf == kf) return HH_OK;
    int per_cu = 0, ncu = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, HH_NL, lds));
    HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d->device));
    if (per_cu < 1) return HH_ERR_UNSUPPORTED;
    d->grid = (uint32_t)(per_cu * ncu);
    d->grid_lds = lds;
    d->grid_kf = kf;
    if (d->d_dbg) HIP_OK(hipFree(d->d_dbg));
    d->d_dbg = nullptr;
    HIP_OK(hipMalloc(&d->d_dbg, (size_t)d->grid * HH_NDBG * sizeof(uint64_t)));
    HIP_OK(hipMemset(d->d_dbg, 0, (size_t)d->grid * HH_NDBG * sizeof(uint64_t)));
    return HH_OK;
}

// The fused decode of tiles [0, ntiles) of the segment at d_data
// (bits_avail readable stream bits), entered at in_state.
static int decode_fast(hh_decoder *d, const void *d_data, uint64_t bits_avail, uint64_t ntiles,
                       uint32_t in_state, uint64_t emit_from, void *d_out, uint64_t cap,
                       hipStream_t st, uint64_t *total, uint32_t *leave, uint32_t *cst_pro,
                       uint32_t *cst_seg, uint32_t *entry) {
    Geometry geo;
    geo.bits = bits_avail;
    geo.S = d->S;
    geo.sw = d->S / 32;
    geo.magic = hh_magic(geo.sw);
    geo.maxadv = d->ht->maxlen > HH_P ? (uint32_t)d->ht->maxlen : HH_P;
    geo.nwords = ((bits_avail + 7) / 8 + HH_PAYLOAD_PAD) / 4;
    geo.in_state = in_state;
    geo.emit_from = emit_from;
    const uint64_t tb = (uint64_t)HH_NR * d->S;
    const uint64_t all = (bits_avail + tb - 1) / tb;
    geo.ntiles = ntiles && ntiles < all ? ntiles : all;
    geo.vec4 = (((uintptr_t)d_data & 15u) == 0) && (geo.sw % 4 == 0);
    // workspace: [flags 64 B | agg[ntiles] | inc[ntiles] | tabs[ntiles][KM]] (zeroed)
    //            | (HH_DEBUG_TILES) tdbg[ntiles][8]
    const size_t zero_bytes = 64 + (size_t)geo.ntiles * (16 + 8 * HH_KM + 4);
    const int dbg_tiles = getenv("HH_DEBUG_TILES") != nullptr;
    int rc = ensure_ws(d, zero_bytes + (size_t)geo.ntiles * (dbg_tiles ? 8 : 0) * 8 + 256);
    if (rc) return rc;
    uint8_t *w = (uint8_t *)d->ws;
    uint32_t *d_flags = (uint32_t *)w;
    LookBack lb;
    lb.agg = (uint64_t *)(w + 64);
    lb.inc = lb.agg + geo.ntiles;
    lb.tabs = lb.inc + geo.ntiles;
    lb.agg32 = (uint32_t *)(lb.tabs + geo.ntiles * HH_KM);
    lb.tdbg = dbg_tiles ? (uint64_t *)(w + ((zero_bytes + 7) & ~(size_t)7)) : nullptr;
    d->last_ntiles = geo.ntiles;
    const size_t lds = lds_bytes(d);
    const kdec_t kf = kdec_for(geo.sw);
    if (!kf) return HH_ERR_UNSUPPORTED;
    rc = size_grid(d, lds, kf);
    if (rc) return rc;
    const uint32_t grid = (uint32_t)(geo.ntiles < d->grid ? geo.ntiles : d->grid);

    HIP_OK(hipMemsetAsync(d_flags, 0, zero_bytes, st));
    HIP_OK(hipEventRecord(d->ev[0], st));
    hipLaunchKernelGGL(kf, dim3(grid), dim3(HH_NL), lds, st, (const uint32_t *)d_data, geo,
                       d->tab, lb, (uint8_t *)d_out, cap, d_flags, d->d_dbg);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(d->ev[1], st));
    HIP_OK(hipMemcpyAsync(d->h_flags, d_flags, 64, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    const uint32_t fl = d->h_flags[0];
    *total = (uint64_t)d->h_flags[2] | ((uint64_t)d->h_flags[3] << 32);
    *leave = d->h_flags[14];
    *cst_pro = d->h_flags[12];
    *cst_seg = d->h_flags[13];
    *entry = emit_from < geo.ntiles ? d->h_flags[15] : in_state;
    if (emit_from >= geo.ntiles) *total = 0;
    float ms = 0;
    hipEventElapsedTime(&ms, d->ev[0], d->ev[1]);
    d->stats.ms_total = ms;
    d->stats.ms_emit = ms;
    d->stats.lanes = geo.ntiles * HH_NR;
    d->stats.out_len = *total;
    if (fl & F_TIMEOUT) return HH_ERR_TIMEOUT;
    if (fl & F_FAIL) return HH_ERR_UNSUPPORTED;
    if (*total > cap || (fl & F_OVER)) return HH_ERR_CAPACITY;
    return HH_OK;
}

extern "C" int hh_decode_device(hh_decoder *d, const void *d_data, uint64_t bits, void *d_out,
                                uint64_t cap, uint64_t *out_len, void *hip_stream) {
    if (!d || !out_len || (!d_data && bits) || (!d_out && cap)) return HH_ERR_ARG;
    if (!d->have_tree) return HH_ERR_ARG;
    if (((uintptr_t)d_data & 3u) != 0) return HH_ERR_ARG;   // word loads
    // NULL is the default stream (ordered with the caller's default-stream
    // work, e.g. torch's), never the decoder's private non-blocking stream
    hipStream_t st = (hipStream_t)hip_stream;
    HIP_OK(hipSetDevice(d->device));
    memset(&d->stats, 0, sizeof(d->stats));
    *out_len = 0;
    if (bits == 0) return HH_OK;
    if (!fast_path_ok(d)) {
        d->stats.exact_fallback = 1;
        return stage_pipeline(d, d_data, (int64_t)bits, (uint8_t *)d_out, cap, out_len, st);
    }
    uint64_t total = 0;
    uint32_t leave = 0, cp = 0, cs = 0, en = 0;
    int rc = decode_fast(d, d_data, bits, 0, hh_state_pack(0, 0, 0), 0, d_out, cap, st, &total,
                         &leave, &cp, &cs, &en);
    if (rc == HH_ERR_UNSUPPORTED) {
        // A walk found no shared boundary within HH_KM regions (a code that
        // does not resynchronise): take the exact path.
        d->stats.exact_fallback = 1;
        d->stats.repairs = 1;
        return stage_pipeline(d, d_data, (int64_t)bits, (uint8_t *)d_out, cap, out_len, st);
    }
    *out_len = total;
    return rc;
}

extern "C" int hh_decoder_tile_bits(const hh_decoder *d, uint64_t *tile_bits) {
    if (!d || !tile_bits || !d->have_tree) return HH_ERR_ARG;
    *tile_bits = (uint64_t)HH_NR * d->S;
    return HH_OK;
}

extern "C" int hh_decode_device_range(hh_decoder *d, const void *d_data, const hh_range *rg,
                                      void *d_out, uint64_t cap, hh_range_out *ro,
                                      void *hip_stream) {
    if (!d || !rg || !ro || (!d_data && rg->bits_avail) || (!d_out && cap)) return HH_ERR_ARG;
    if (!d->have_tree) return HH_ERR_ARG;
    if (((uintptr_t)d_data & 3u) != 0) return HH_ERR_ARG;
    hipStream_t st = (hipStream_t)hip_stream;
    HIP_OK(hipSetDevice(d->device));
    memset(&d->stats, 0, sizeof(d->stats));
    memset(ro, 0, sizeof(*ro));
    ro->leave_state = ro->entry_state = rg->in_state;
    if (rg->bits_avail == 0) return HH_OK;
    // segments need the fused path (tile tables, entry states); a tree it
    // does not support is decoded whole, unsharded
    if (!fast_path_ok(d) || hh_state_d(rg->in_state) >= HH_KM) return HH_ERR_UNSUPPORTED;
    uint32_t cp = 0;
    const int rc = decode_fast(d, d_data, rg->bits_avail, rg->ntiles, rg->in_state, rg->prologue,
                               d_out, cap, st, &ro->out_len, &ro->leave_state, &cp,
                               &ro->const_seen, &ro->entry_state);
    ro->entry_exact = rg->prologue == 0 || cp != 0;
    return rc;
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
    hipStream_t st = (hipStream_t)s;   // NULL = the default stream
    return stage_pipeline(d, d_data, bits, d_out, cap, out_len, st);
}

// Diagnostic: the first failed walk of the last decode (tile, lane, exit,
// count, tile end); 0 if none.
extern "C" int hh_debug_failure(hh_decoder *d, uint32_t *out5) {
    if (!d || !out5 || !d->ws) return 0;
    uint32_t f[10];
    if (hipMemcpy(f, d->ws, sizeof(f), hipMemcpyDeviceToHost) != hipSuccess) return HH_ERR_DEVICE;
    for (int i = 0; i < 5; i++) out5[i] = f[5 + i];
    return (int)f[4];
}

// Diagnostic (HH_DEBUG_TILES set at decode time): per-tile [base, size |
// entering state << 32, exclusive charged prefix, table entry, look-back's
// inclusive tile, its prefix, counts summed, rounds] of the last
// decode.  Returns the number of tiles written.
extern "C" int hh_debug_tiles(hh_decoder *d, uint64_t *out, int max_tiles) {
    if (!d || !out || !d->ws || !getenv("HH_DEBUG_TILES")) return 0;
    const uint64_t nt = d->last_ntiles;
    const int n = (int)(nt < (uint64_t)max_tiles ? nt : (uint64_t)max_tiles);
    // after [flags 64 B | agg | inc | tabs | agg32], 8-B aligned (decode_fast)
    const size_t zb = 64 + (size_t)nt * (16 + 8 * HH_KM + 4);
    const uint64_t *src = (const uint64_t *)((uint8_t *)d->ws + ((zb + 7) & ~(size_t)7));
    if (hipMemcpy(out, src, (size_t)n * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return HH_ERR_DEVICE;
    return n;
}

// Diagnostic: per-block phase cycle sums of the last decode (HH_STAMPS
// builds; zeros otherwise).  Returns the number of blocks written.
extern "C" int hh_debug_phase_cycles(hh_decoder *d, uint64_t *out, int max_blocks) {
    if (!d || !out || !d->d_dbg) return 0;
    int n = (int)d->grid < max_blocks ? (int)d->grid : max_blocks;
    if (hipMemcpy(out, d->d_dbg, (size_t)n * HH_NDBG * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return HH_ERR_DEVICE;
    return n;
}
