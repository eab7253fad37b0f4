// hh_device.hip -- HIP kernels (gfx950) and the device half of the C ABI.
//
// The decode is four launches on one stream, no in-kernel waits between
// workgroups (O(N) memory, 64-bit offsets):
//
//   k_front   one tile (HH_NR = 64 regions x S bits) per WAVE at a time,
//             persistent grid, independent of every other tile and wave:
//               stage     the tile's words (+ the next tile's first HH_KM
//                         regions and a halo), prefetched one tile ahead into
//                         registers, stored to the wave's LDS slice transposed
//               pass 1    every lane decodes its region from a G-bit overlap
//                         head: count, exit and boundary mask (decodeallbits)
//               walks     each exit that did not merge in the overlap window
//                         is walked against the next regions' chains until
//                         they share a boundary (makebigtable)
//               table     charged count and leaving state for every entering
//                         state d < HH_KM -> workspace; one 32-bit record per
//                         lane (regions crossed, entry offset, correction,
//                         count) -> workspace
//   k_scan1/2 the state entering every tile (the predecessor's leaving state,
//             composed through the tables back to the nearest CONST tile) and
//             the exclusive prefix of the tiles' charged counts
//             (calcbitsindex / findmax)
//   k_emit    one tile per WAVE at a time again: live lanes from the tile's
//             entering state, run offsets by a wave scan, each lane
//             re-decodes its exact run into the wave's LDS staging buffer,
//             copied out with 16-B stores (calcresult)
//
// Reference-shaped stage kernels (k_st_*) mirror the six .cl kernels one by
// one for intermediate-array parity.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>

#include "hh_algo.h"
#include "hh_fsm_algo.h"
#include "hh_fsm_dev.h"
#include "hh_internal.h"
#include "hiphuff.h"

#ifdef HH_WSPAN
#define HH_DBG_WORDS (16 + 10 * 8192)
#else
#define HH_DBG_WORDS 16
#endif
#define HH_MAXLEN_FAST 32           // longest code of the fast path (one cursor step <= 32 bits)
// k_emit's waves per workgroup share one copy of the tables: 16 (one
// workgroup per CU with the 12-bit L1, 32 KiB) when the tables fit beside
// them, else 8 (2 / 4 / 8 waves with the 11-bit L1: emit 3.02 / 2.07 / 1.80
// ms; 16 with the 12-bit L1: 1.43 ms).
#define HH_EMIT_NW_MAX 16
#ifndef HH_FW
#define HH_FW 8                     // waves per workgroup (k_front), sharing the 16 KiB F: 3
                                    // workgroups per CU (with the 13-bit F, 4 / 7 / 8 / 14 waves:
                                    // front + walks 1.29 / 1.21 / 1.13 / 1.26 ms)
#endif
#define HH_SCAN_TB 1024             // tiles per k_scan1 block
#define HH_SCAN_BACK 4096           // longest non-CONST chain k_scan1 composes (else host scan)
#ifndef HH_XPT
#define HH_XPT 4                    // k_emit: deferred runs per tile a wave's list holds
#endif
#define HH_OBW (4096 + 64)          // k_emit's LDS output staging per wave (bytes): a text tile's
                                    // output (~3.7 K symbols for kjv) plus the 16-B phase

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
    const uint16_t *f;   // the front's table (hh_internal.h F) and its escape directory
    const uint32_t *fdir;
    uint32_t fdir_used;
    const uint32_t *l2;
    const uint32_t *tree;
    const uint8_t *tsym;
    uint32_t l2_used;
    uint32_t tree_lds;   // compact tree nodes k_emit stages in LDS
};
#define HH_TREE_LDS_MAX 1024   // nodes: a byte alphabet's tree has <= 511 unless symbols repeat;
                               // larger trees take the stage pipeline

// flags[0]: status bits; [2..3] total symbols (u64); [4..9] first failed walk;
// [12] a prologue tile is CONST; [13] an emitted tile is CONST; [14] state
// leaving the last tile; [15] state entering the first emitted tile
enum { F_FAIL = 1, F_OVER = 2, F_SCAN = 4 };

// Per-lane record of the front pass (k_front -> k_emit), 32 bits:
//   bits 0..2 k-1 (regions the lane's walk crossed), 3..7 e (the walk's first
//   boundary in the merge region, < 32), 8..17 delta (signed), 18..29 n + cov
//   (own symbols + symbols of covered regions)
__device__ __forceinline__ uint32_t rec_pack(uint32_t k, uint32_t e, int32_t delta, uint32_t nc) {
    return (k - 1u) | (e << 3) | (((uint32_t)delta & 0x3ffu) << 8) | (nc << 18);
}
__device__ __forceinline__ uint32_t rec_k(uint32_t r) { return (r & 7u) + 1u; }
__device__ __forceinline__ uint32_t rec_e(uint32_t r) { return (r >> 3) & 31u; }
__device__ __forceinline__ int32_t rec_delta(uint32_t r) { return (int32_t)(r << 14) >> 22; }
__device__ __forceinline__ uint32_t rec_nc(uint32_t r) { return r >> 18; }

struct Geometry {
    uint64_t bits;       // stream length
    uint64_t nwords;     // readable payload words
    uint64_t ntiles;
    uint32_t S, sw;
    uint32_t maxadv;     // max(HH_P, longest code)
    uint32_t G;          // overlap bits (hh_region_head)
    uint32_t in_state;   // state entering tile 0 (a shard's entry; 0 at the stream start)
    uint64_t emit_from;  // tiles before this one are a prologue: decoded for their
                         // leaving state only (a shard's probe of its predecessor)
    uint32_t fwalk;      // lookups of a walk in k_front (longer: deferred to k_walk)
    uint32_t nfw;        // k_front's waves (each with its list of deferred walks)
    uint64_t qcap;       // entries per list (the wave's tiles x HH_NR)
    uint32_t xcap;       // k_emit: deferred runs per wave's list (HH_XPT per tile)
};

// Workspace carve (decode_fast).  Nothing but `flags` needs zeroing: every
// other word is written before it is read.
struct Work {
    uint32_t *flags;     // 64 B
    uint64_t *tabs;      // [ntiles][HH_KM] rows: count | state << 20; row 0 bit 61 = CONST
    uint32_t *recs;      // [ntiles][HH_NR] lane records (a group's are contiguous)
    uint32_t *st;        // [ntiles + 1] state entering each tile (st[ntiles]: leaving the last)
    int32_t *lex;        // [ntiles + 1] exclusive prefix of charged counts within its scan block
    int64_t *blk;        // [nblk] scan block totals, then exclusive block bases
    uint64_t *q;         // [nfw][qcap] deferred walks of each k_front wave: tile * HH_NR + lane |
                         // (exit | count << 16) << 32
    uint32_t *qn;        // [nfw] their counts
    uint32_t *xn;        // [ntiles * HH_NR] pass-1 exit | count << 16 of every region
    uint64_t *xq;        // [k_emit waves][xcap] deferred runs: output offset, tile << 32 | entry | end << 16
    uint32_t *xqn;       // [k_emit waves] their counts
};

// ---------------------------------------------------------------------------
// wave / block helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t wave_incl_scan(int32_t x) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    return x;
}

__device__ __forceinline__ int32_t wave_sum(int32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Exclusive block scan of int32 over NT threads; *total = block sum.
template <uint32_t NT>
__device__ __forceinline__ int32_t block_excl_scan(int32_t v, int32_t *s_tmp, int32_t *total) {
    constexpr uint32_t NW = NT / 64;
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

// Words of a staged span through a buffer resource over its readable words:
// the range check returns 0 past the payload, so no lane branches between
// load paths (with a per-lane branch the compiler waits for every load in
// flight before the second path's loads).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t words_rsrc(const uint32_t *g, uint64_t tw0, uint64_t nok) {
    const uint64_t left = nok > tw0 ? nok - tw0 : 0u;
    const uint32_t nbytes = left > 0x3fffffffull ? 0xfffffffcu : (uint32_t)left * 4u;
    return __builtin_amdgcn_make_buffer_rsrc((void *)(g + tw0), 0, (int)nbytes, 0x00020000);
}

template <uint32_t sw>
__device__ __forceinline__ void load_region(uint32_t *v, __amdgpu_buffer_rsrc_t r, uint32_t col) {
    const uint32_t v0 = 4u * col * sw;
    if (sw % 4 == 0) {
#pragma unroll
        for (uint32_t k = 0; k < HH_SW_MAX; k += 4) {
            if (k < sw) {
                const u32x4 q = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(v0 + 4u * k), 0, 0));
                v[k] = q.x; v[k + 1] = q.y; v[k + 2] = q.z; v[k + 3] = q.w;
            }
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < HH_SW_MAX; k++)
            if (k < sw) v[k] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(v0 + 4u * k), 0, 0);
    }
}

// Registers holding one tile's words for this lane: its region column and up
// to two words of the columns past the tile (the next tile's first HH_KM
// regions and the halo).
static_assert((HH_NCOL - HH_NR) * HH_SW_MAX <= 2 * 64, "a tile's extra columns: two words per lane");
static_assert(HH_NLS >= HH_NCOL && HH_NLS % 16 == 0, "LDS column stride");
struct Prefetch {
    uint32_t v[HH_SW_MAX];
    uint32_t halo, halo2;
};

// a wave's tile (lane = its region)
template <uint32_t sw>
__device__ __forceinline__ void prefetch_wtile(Prefetch &pf, const uint32_t *g, uint64_t tw0, uint64_t nok) {
    const uint32_t j = threadIdx.x & 63u;
    const __amdgpu_buffer_rsrc_t r = words_rsrc(g, tw0, nok);
    load_region<sw>(pf.v, r, j);
    constexpr uint32_t nx = (HH_NCOL - HH_NR) * sw;
    pf.halo = j < nx ? __builtin_amdgcn_raw_buffer_load_b32(r, (int)(4u * (HH_NR * sw + j)), 0, 0) : 0u;
    pf.halo2 = j + 64 < nx ? __builtin_amdgcn_raw_buffer_load_b32(r, (int)(4u * (HH_NR * sw + j + 64)), 0, 0) : 0u;
}
template <uint32_t sw>
__device__ __forceinline__ void store_wtile(const Prefetch &pf, uint32_t *s_w) {
    const uint32_t j = threadIdx.x & 63u;
    constexpr uint32_t nx = (HH_NCOL - HH_NR) * sw;
#pragma unroll
    for (uint32_t k = 0; k < HH_SW_MAX; k++)
        if (k < sw) s_w[k * HH_NLS + j] = pf.v[k];
    if (j < nx) s_w[(j % sw) * HH_NLS + HH_NR + j / sw] = pf.halo;
    if (j + 64 < nx) s_w[((j + 64) % sw) * HH_NLS + HH_NR + (j + 64) / sw] = pf.halo2;
}

// Lanes of one wave exchanging values through LDS: a wave's LDS operations
// execute in order, so a compiler fence is all the ordering needed.
#define WAVE_SYNC()                                                    \
    do {                                                               \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");         \
        __builtin_amdgcn_wave_barrier();                               \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");         \
    } while (0)

// Live masks over the entering state d of a wave's tile (bit d of mem: the
// lane is live when the tile is entered in region d): hh_mem_init, then the
// walks with k > 1 (exceptions), in ascending lane order, clear the lanes
// they cover (within the tile).  s_k, s_mem: the wave's 64 entries.  One
// lane; a tile rarely has more than one exception.
__device__ __forceinline__ uint32_t resolve_live_wave(uint32_t kk, uint8_t *s_k, uint8_t *s_mem) {
    const uint32_t j = threadIdx.x & 63u;
    const uint64_t ex = __ballot(kk > 1);
    if (ex == 0) return hh_mem_init(j);
    s_k[j] = (uint8_t)kk;
    s_mem[j] = (uint8_t)hh_mem_init(j);
    WAVE_SYNC();
    if (j == 0) {
        uint64_t m = ex;
        while (m) {
            const uint32_t e = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t ke = s_k[e];
            const uint8_t me = s_mem[e];
            for (uint32_t q = e + 1; q < e + ke && q < HH_NR; q++) s_mem[q] &= (uint8_t)~me;
        }
    }
    WAVE_SYNC();
    return s_mem[j];
}

// The front's tables into LDS: F, its escape directory, L2.
__device__ __forceinline__ void load_ftables(const DevTab &tab, uint16_t *s_f, uint32_t *s_fdir, uint32_t *s_l2) {
    const uint32_t *f32 = (const uint32_t *)tab.f;
    for (uint32_t i = threadIdx.x; i < HH_F_SIZE / 2; i += blockDim.x) ((uint32_t *)s_f)[i] = f32[i];
    for (uint32_t i = threadIdx.x; i < tab.fdir_used; i += blockDim.x) s_fdir[i] = tab.fdir[i];
    for (uint32_t i = threadIdx.x; i < tab.l2_used; i += blockDim.x) s_l2[i] = tab.l2[i];
}
__host__ __device__ constexpr uint32_t ftab_words(uint32_t fdir, uint32_t l2) {
    return HH_F_SIZE / 2 + ((fdir + 3u) & ~3u) + ((l2 + 3u) & ~3u);
}

#ifndef HH_FRONT_MINB
#define HH_FRONT_MINB 2   // workgroups per CU the front kernel's registers are sized for (it
                          // compiles to ~70 VGPRs: up to 7 waves per SIMD; its LDS allows 6)
#endif

// Diagnostic build only (-DHH_DIAG): every wave stamps the shader clock
// between the front kernel's phases and adds the cycles into dbg[phase]
// (0 staging, 4 own pass 1, 1 its barrier wait, 5 own walks, 2 their barrier
// wait, 3 table); walk statistics go to dbg[8..]: lanes, lookups, the sum over
// tiles of the longest walk, the longest walk.  hh_debug_counters reads them.
#ifdef HH_DIAG
#define DIAG_DECL uint64_t dg_acc[6] = {0, 0, 0, 0, 0, 0}, dg_w[4] = {0, 0, 0, 0}; uint64_t dg_t = __builtin_amdgcn_s_memtime();
#define DIAG_STAMP(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); dg_acc[i] += t_ - dg_t; dg_t = t_; } while (0)
#define DIAG_FLUSH(dbg) do { if ((threadIdx.x & 63u) == 0) for (int i_ = 0; i_ < 6; i_++) atomicAdd((unsigned long long *)&(dbg)[i_], (unsigned long long)dg_acc[i_]); \
    if ((threadIdx.x & 63u) == 0) { for (int i_ = 0; i_ < 3; i_++) atomicAdd((unsigned long long *)&(dbg)[8 + i_], (unsigned long long)dg_w[i_]); \
        atomicMax((unsigned long long *)&(dbg)[11], (unsigned long long)dg_w[3]); } } while (0)
#define EDIAG_DECL uint64_t eg_acc[5] = {0, 0, 0, 0, 0}; uint64_t eg_t = __builtin_amdgcn_s_memtime();
#define EDIAG_STAMP(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); eg_acc[i] += t_ - eg_t; eg_t = t_; } while (0)
#define EDIAG_FLUSH(dbg) do { if ((threadIdx.x & 63u) == 0) { const int ix_[5] = {6, 7, 12, 13, 14}; \
    for (int i_ = 0; i_ < 5; i_++) atomicAdd((unsigned long long *)&(dbg)[ix_[i_]], (unsigned long long)eg_acc[i_]); } } while (0)
#else
#define DIAG_DECL
#define DIAG_STAMP(i) do {} while (0)
#define DIAG_FLUSH(dbg) do {} while (0)
#define EDIAG_DECL
#define EDIAG_STAMP(i) do {} while (0)
#define EDIAG_FLUSH(dbg) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// k_front: pass 1 and the short walks of every tile, one tile per wave at a
// time (a persistent grid; wave gw takes tiles gw, gw + #waves, ...).  Within
// a tile the lanes exchange values through the wave's own LDS slice, never
// with other waves: no workgroup barrier after the tables.  A walk longer
// than geo.fwalk lookups is deferred to k_walk (a wave would otherwise wait
// for its longest walk: kjv's average walk is 0.5 lookups, a wave's longest
// 16); the tables follow from the records in k_table.
// ---------------------------------------------------------------------------
template <uint32_t SW>
__global__ __launch_bounds__(64 * HH_FW, HH_FRONT_MINB) void k_front(const uint32_t *__restrict__ gdata, Geometry geo,
                                                                 DevTab tab, Work wk, uint64_t *dbg) {
    extern __shared__ __align__(16) uint8_t smem[];
    __shared__ uint32_t s_ya[HH_FW][HH_NR];    // entry points of the regions' own chains

    constexpr uint32_t S = 32 * SW;
    const uint32_t j = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint16_t *s_f = (uint16_t *)smem;                   // F, its escape directory, L2 (shared),
    uint32_t *s_fdir = (uint32_t *)smem + HH_F_SIZE / 2;
    uint32_t *s_l2 = s_fdir + ((tab.fdir_used + 3u) & ~3u);
    uint32_t *s_w = (uint32_t *)smem + ftab_words(tab.fdir_used, tab.l2_used) + wv * (SW * HH_NLS);
    uint32_t *s_y = s_ya[wv];                           // then the waves' slices (SW * HH_NLS words)

    const uint64_t tile_bits = (uint64_t)HH_NR * S;
    const uint32_t span = HH_NCOL * S;                  // bits staged per tile
    load_ftables(tab, s_f, s_fdir, s_l2);
    __syncthreads();                                    // (the only workgroup barrier)

    hh_ctx c;
    c.w = s_w;
    c.sw = SW;
    c.nls = HH_NLS;
    c.magic = 0;
    c.l1m = nullptr;
    c.l1s = nullptr;
    c.l1 = nullptr;
    c.f = s_f;
    c.fdir = s_fdir;
    c.pf = HH_PF;
    c.l2 = s_l2;
    c.tree = tab.tree;
    c.tsym = tab.tsym;
    c.maxadv = geo.maxadv > HH_PF ? geo.maxadv : HH_PF;
    c.G = geo.G;

    // The next tile's words are loaded one tile ahead into registers and
    // stored to LDS once the walks are done (before the tile's record
    // stores: vmcnt retires in order and counts stores too).  The loads run
    // unconditionally (the last tile again past the end): a conditional load
    // merges two values, which the compiler waits for.
    const uint64_t nwv = (uint64_t)gridDim.x * HH_FW;
    const uint64_t tlast = geo.ntiles ? geo.ntiles - 1 : 0;
    auto clampt = [&](uint64_t tt) { return tt < tlast ? tt : tlast; };
    Prefetch pf;
    uint64_t t = (uint64_t)blockIdx.x * HH_FW + wv;
    // deferred walks: this wave's list q[qbase, qbase + qn), its length -> qn[gw]
    const uint32_t gw = (uint32_t)t;
    const uint64_t qbase = (uint64_t)gw * geo.qcap;
    uint32_t qn = 0;
    if (t < geo.ntiles) {
        prefetch_wtile<SW>(pf, gdata, t * tile_bits / 32, geo.nwords);
        store_wtile<SW>(pf, s_w);
        prefetch_wtile<SW>(pf, gdata, clampt(t + nwv) * tile_bits / 32, geo.nwords);
    }
    DIAG_DECL
    for (; t < geo.ntiles; t += nwv) {
        WAVE_SYNC();                                    // this tile's words stored
        const uint64_t rem = geo.bits - t * tile_bits;
        c.bt = rem < span ? (uint32_t)rem : span;
        const uint32_t bt = c.bt;
        DIAG_STAMP(0);

        // pass 1: the head (from G bits before the region, lanes > 0), then
        // the own chain from its entry point y, counted
        const uint32_t p0 = j * S;
        uint32_t n = 0, x = bt, y = bt;
        if (p0 < bt) {
            y = j > 0 && c.G ? hh_region_head(&c, p0 - c.G, p0, nullptr) : p0;
            const uint32_t lim = p0 + S < bt ? p0 + S : bt;
            x = y < lim ? hh_region_count(&c, y, lim, &n) : y;
        }
        s_y[j] = y;
        DIAG_STAMP(1);
        // chain j's exit is chain j+1's entry point: merged there, no walk
        // (the next tile's region 0 is entered at its start)
        const uint32_t R1 = (j + 1) * S;
        const uint32_t yn = (uint32_t)__shfl_down((int)y, 1, 64);
        const bool merged = R1 < bt && x == (j == 63u ? R1 : yn);
        WAVE_SYNC();                                    // s_y complete

        // walks: region j's exit against the next regions' own chains, two
        // pointers, at most geo.fwalk lookups here
        hh_wk w = {1u, x - R1, 0u, 0, 0u, 0u};
        if (!merged) {
            if (geo.fwalk) w = hh_walk(&c, j, S, x, nullptr, nullptr, nullptr, 0, geo.fwalk, s_y, HH_NR);
            else w.more = 1u;                           // (every walk to k_walk)
        }
        const uint32_t rec = rec_pack(w.k ? w.k : 1u, w.e, w.delta, n + w.cov);
        if (w.more) {
            const uint64_t dm = __ballot(1);            // (the deferring lanes)
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
            wk.q[qbase + qn + rank] = (uint64_t)(t * HH_NR + j) | ((uint64_t)(x | (n << 16)) << 32);
        }
        {
            // the wave's own list (an atomic on one counter per deferring
            // wave serialises: 4 ms per decode)
            const uint64_t dm = __ballot(w.more);
            qn += (uint32_t)__builtin_popcountll(dm);
        }
        if (!w.more && w.k == 0) {
            atomicOr(wk.flags, (uint32_t)F_FAIL);
            if (atomicCAS(&wk.flags[4], 0u, 1u) == 0u) {
                wk.flags[5] = (uint32_t)t; wk.flags[6] = j; wk.flags[7] = x; wk.flags[8] = n; wk.flags[9] = bt;
            }
        }
#ifdef HH_DIAG
        {
            const uint32_t st = w.steps;
            uint32_t mx = st;
            uint64_t sm = st;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
                sm += (uint32_t)__shfl_xor((int)(uint32_t)sm, o, 64);
            }
            dg_w[0] += 64;
            dg_w[1] += sm;
            dg_w[2] += mx;
            dg_w[3] = dg_w[3] > mx ? dg_w[3] : mx;
        }
#endif
        DIAG_STAMP(2);
        // the walks are done: the next tile's words go to LDS now, and the
        // tile after it is loaded
        WAVE_SYNC();
        store_wtile<SW>(pf, s_w);
        prefetch_wtile<SW>(pf, gdata, clampt(t + 2 * nwv) * tile_bits / 32, geo.nwords);
        wk.recs[t * HH_NR + j] = rec;                 // (a deferred lane's: k_walk's)
        wk.xn[t * HH_NR + j] = x | (n << 16);         // the region's exit and count, for k_walk
        DIAG_STAMP(3);
    }
    if (j == 0) wk.qn[gw] = qn;
    DIAG_FLUSH(dbg);
}

// ---------------------------------------------------------------------------
// k_walk: the deferred walks (k_front's lists), one lane each: exit
// comparisons (hh_walk_exits, restated here region by region) against the
// regions' pass-1 exits and counts (xn).  A lane stages only the words of
// the region it walks (from G bits before it, for the heads of regions that
// were not decoded, to a halo past it) at LDS index (q * HH_WALK_T + lane).
// The lane's record replaces k_front's placeholder.
// The merge/delta rule here must stay the one of hh_walk_exits (hh_algo.h),
// which the emulator checks against the mask walk: a change to either is a
// change to both (the GPU parity tests with HH_FLAG_LEGACY cover this copy:
// test_walk_bound_and_deferral_lists, test_fixture_legacy_pipeline).
// ---------------------------------------------------------------------------
#ifndef HH_WALK_T
#define HH_WALK_T 256   // lanes per k_walk workgroup (64: +0.05 ms; 512: same)
#endif
template <uint32_t SW>
struct WalkWin {
    static constexpr uint32_t n = SW + 6;   // words of one region's window
};

template <uint32_t SW>
__device__ __forceinline__ void walk_win_load(uint32_t (&v)[WalkWin<SW>::n], const uint32_t *gdata, uint64_t gw0,
                                              uint64_t glim) {
#pragma unroll
    for (uint32_t q = 0; q < WalkWin<SW>::n; q++) {
        const uint64_t gi = gw0 + q;
        v[q] = gdata[gi < glim ? gi : glim - 1];   // (past the payload: past the stream end, unused)
    }
}

template <uint32_t SW>
__global__ __launch_bounds__(HH_WALK_T) void k_walk(const uint32_t *__restrict__ gdata, Geometry geo, DevTab tab, Work wk) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t S = 32 * SW, NW = WalkWin<SW>::n;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    uint16_t *s_f = (uint16_t *)smem;                   // F, its escape directory, L2
    uint32_t *s_fdir = (uint32_t *)smem + HH_F_SIZE / 2;
    uint32_t *s_l2 = s_fdir + ((tab.fdir_used + 3u) & ~3u);
    uint32_t *s_win = (uint32_t *)smem + ftab_words(tab.fdir_used, tab.l2_used) + tid;   // NW words
    load_ftables(tab, s_f, s_fdir, s_l2);
    __syncthreads();
    const uint64_t tile_bits = (uint64_t)HH_NR * S;
    const uint32_t span = HH_NCOL * S;
    hh_ctx c;
    c.sw = 1024;                                        // hh_idx(g) = g * HH_WALK_T (below)
    c.nls = HH_WALK_T;
    c.magic = 0;
    c.l1m = nullptr;
    c.l1s = nullptr;
    c.l1 = nullptr;
    c.f = s_f;
    c.fdir = s_fdir;
    c.pf = HH_PF;
    c.l2 = s_l2;
    c.tree = tab.tree;
    c.tsym = tab.tsym;
    c.maxadv = geo.maxadv > HH_PF ? geo.maxadv : HH_PF;
    c.G = geo.G;
    // one k_front wave's list at a time, its entries over the wave's lanes;
    // the next entry is loaded one walk ahead
    const uint32_t nwv = gridDim.x * (HH_WALK_T / 64);
    uint32_t fw = blockIdx.x * (HH_WALK_T / 64) + (tid >> 6), i = lane, cnt = fw < geo.nfw ? wk.qn[fw] : 0u;
    auto next_entry = [&](uint64_t &e) -> bool {
        while (i >= cnt && fw < geo.nfw) {
            i -= cnt;
            fw += nwv;
            cnt = fw < geo.nfw ? wk.qn[fw] : 0u;
        }
        if (fw >= geo.nfw) return false;
        e = wk.q[(uint64_t)fw * geo.qcap + i];
        i += 64;
        return true;
    };
    uint32_t pre[NW];
    uint64_t en = 0;
    bool have_n = next_entry(en);
    while (have_n) {
        const uint64_t ent = en;
        have_n = next_entry(en);
        const uint32_t gl = (uint32_t)ent;
        const uint64_t t = gl / HH_NR;
        const uint32_t j = gl % HH_NR;
        const uint32_t r0 = (uint32_t)(ent >> 32);
        const uint64_t rem = geo.bits - t * tile_bits;
        c.bt = rem < span ? (uint32_t)rem : span;
        const uint32_t bt = c.bt;
        const uint64_t tw0 = t * tile_bits / 32;
        auto win0 = [&](uint32_t k) { const uint32_t g = (j + k) * SW; return g >= 2 ? g - 2 : 0u; };
        walk_win_load<SW>(pre, gdata, tw0 + win0(1), geo.nwords);
        // the regions' pass-1 exits and counts, all loaded at once (a tile
        // past the decoded ones, at a range's end: decoded below)
        const bool nxt_ok = t + 1 < geo.ntiles;
        uint32_t xv[HH_KM + 1];
#pragma unroll
        for (uint32_t k = 1; k <= HH_KM; k++) xv[k] = wk.xn[gl + k];   // (xn has a tile of slack)
        uint32_t A = r0 & 0xffffu, ca = 0;
        A = A < bt ? A : bt;
        hh_wk w = {0u, 0u, 0u, 0, 0u, 0u};
        for (uint32_t k = 1; k <= HH_KM; k++) {
            const uint32_t g0 = win0(k);
            // (most walks end in their first region: the next region's words
            // are loaded only when the walk goes on -- loading them ahead
            // doubled k_walk's HBM reads)
            if (k > 1) walk_win_load<SW>(pre, gdata, tw0 + g0, geo.nwords);
#pragma unroll
            for (uint32_t q = 0; q < NW; q++) s_win[q * HH_WALK_T] = pre[q];
            c.w = s_win - (int32_t)g0 * (int32_t)HH_WALK_T;                  // tile word g at (g - g0)
            const uint32_t rg = j + k, R = rg * S;
            const uint32_t Ec = R + S < bt ? R + S : bt;
            // the region's own chain: its pass-1 exit and count (a tile past
            // the decoded ones, at a range's end: decoded here)
            uint32_t xk, nk;
            if (rg < HH_NR || nxt_ok) {
                const uint32_t v = xv[k];
                xk = (v & 0xffffu) + (rg >= HH_NR ? HH_NR * S : 0u);
                nk = v >> 16;
            } else {
                uint32_t yy = R < bt ? R : bt;
                nk = 0;
                if (R < bt && c.G && rg % HH_NR) yy = hh_region_head(&c, R - c.G, R, nullptr);
                xk = yy < Ec ? hh_region_count(&c, yy, Ec, &nk) : yy;
            }
            const uint32_t e = A > R ? A - R : 0u;
            uint32_t n = 0;
            if (A < Ec) A = hh_region_count(&c, A, Ec, &n);
            if (A == (xk < bt ? xk : bt)) {
                w.k = k;
                w.e = e;
                w.cov = ca;
                w.delta = (int32_t)n - (int32_t)nk;
                break;
            }
            ca += n;
        }
        if (w.k == 0) {
            atomicOr(wk.flags, (uint32_t)F_FAIL);
            if (atomicCAS(&wk.flags[4], 0u, 1u) == 0u) {
                wk.flags[5] = (uint32_t)t; wk.flags[6] = j; wk.flags[7] = r0 & 0xffffu; wk.flags[8] = r0 >> 16; wk.flags[9] = bt;
            }
        } else {
            wk.recs[gl] = rec_pack(w.k, w.e, w.delta, (r0 >> 16) + w.cov);
        }
    }
}

// ---------------------------------------------------------------------------
// k_table: the transfer table of every tile from its lane records, one tile
// per wave: live masks over the entering state d < HH_KM, the charged count
// of the live lanes and the state leaving the tile (from the last live lane,
// the one whose walk crosses the tile end); CONST when the leaving state
// does not depend on d.
// ---------------------------------------------------------------------------
#define HH_TABLE_W 4
__global__ __launch_bounds__(64 * HH_TABLE_W) void k_table(Geometry geo, Work wk) {
    __shared__ uint8_t s_ka[HH_TABLE_W][HH_NR];
    __shared__ uint8_t s_mema[HH_TABLE_W][HH_NR];
    __shared__ int32_t s_cda[HH_TABLE_W][HH_KM];
    __shared__ uint32_t s_osta[HH_TABLE_W][HH_KM];
    const uint32_t j = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    int32_t *s_cd = s_cda[wv];
    uint32_t *s_ost = s_osta[wv];
    const uint64_t step = (uint64_t)gridDim.x * HH_TABLE_W;
    uint64_t t = (uint64_t)blockIdx.x * HH_TABLE_W + wv;
    const uint64_t tlast = geo.ntiles - 1;
    // records loaded two tiles ahead
    auto clampt = [&](uint64_t tt) { return tt < tlast ? tt : tlast; };
    uint32_t rec_n = t < geo.ntiles ? wk.recs[t * HH_NR + j] : 0u;
    uint32_t rec_n2 = t < geo.ntiles ? wk.recs[clampt(t + step) * HH_NR + j] : 0u;
    for (; t < geo.ntiles; t += step) {
        const uint32_t rec = rec_n;
        rec_n = rec_n2;
        rec_n2 = wk.recs[clampt(t + 2 * step) * HH_NR + j];
        const uint32_t kk = rec_k(rec), e = rec_e(rec);
        const int32_t delta = rec_delta(rec);
        const int32_t charged = (int32_t)rec_nc(rec) + delta;
        if (__ballot(kk > 1) == 0) {
            // no exceptions: lane j is live for entering d <= j (all d from
            // lane HH_KM - 1 on), so row d counts the lanes >= d; the last
            // lane leaves the tile for every d (CONST)
            const int32_t incl = wave_incl_scan(charged);
            const int32_t tot = __builtin_amdgcn_readlane(incl, 63);
            const uint32_t os = hh_state_pack(kk - 1u, e, delta);          // (lane 63: j + kk - HH_NR)
            const uint32_t os63 = (uint32_t)__builtin_amdgcn_readlane((int)os, 63);
            if (j < HH_KM)
                wk.tabs[t * HH_KM + j] = hh_tab_pack(tot - (incl - charged), os63) | (j == 0 ? HH_CST : 0ull);
            continue;
        }
        const uint32_t mem = resolve_live_wave(kk, s_ka[wv], s_mema[wv]);
        if (j < HH_KM) s_cd[j] = 0;
        WAVE_SYNC();
        if (j + kk >= HH_NR) {
            const uint32_t os = hh_state_pack(j + kk - HH_NR, e, delta);
#pragma unroll
            for (uint32_t d = 0; d < HH_KM; d++)
                if ((mem >> d) & 1u) s_ost[d] = os;
        }
        // lanes live for every entering d: one wave sum; the few others
        // (lanes < HH_KM, covered lanes): per-d LDS atomics
        const uint32_t full = (1u << HH_KM) - 1u;
        const int32_t v = wave_sum(mem == full ? charged : 0);
        if (mem != full) {
#pragma unroll
            for (uint32_t d = 0; d < HH_KM; d++)
                if ((mem >> d) & 1u) atomicAdd(&s_cd[d], charged);
        }
        WAVE_SYNC();
        const uint32_t dd = j < HH_KM ? j : 0u;
        const int32_t cnt = s_cd[dd] + v;
        const uint32_t os = s_ost[dd];
        // CONST: the leaving state is the same for every entering d
        const bool cst = __ballot(j < HH_KM && os != s_ost[0]) == 0;
        if (j < HH_KM) wk.tabs[t * HH_KM + j] = hh_tab_pack(cnt, os) | (j == 0 && cst ? HH_CST : 0ull);
        WAVE_SYNC();                                    // s_cd / s_ost read before the next tile
    }
}

// ---------------------------------------------------------------------------
// k_scan1 / k_scan2: entering states and output bases of every tile
// ---------------------------------------------------------------------------
// One thread per tile t in [0, ntiles] (t == ntiles: the state leaving the
// last tile).  The state entering t is the leaving state of the nearest
// CONST tile v < t, carried through the tables of v+1 .. t-1 (every tile of a
// natural code is CONST: v = t - 1).  Block-local exclusive prefix of the
// tiles' charged counts -> lex, block total -> blk.
__global__ __launch_bounds__(HH_SCAN_TB) void k_scan1(Geometry geo, Work wk) {
    __shared__ int32_t s_tmp[HH_SCAN_TB / 64];
    __shared__ uint32_t s_cf;
    const uint64_t t = (uint64_t)blockIdx.x * HH_SCAN_TB + threadIdx.x;
    const bool valid = t <= geo.ntiles;
    uint32_t s = geo.in_state;
    int32_t cnt = 0;
    bool cst = false;
    if (valid) {
        if (t > 0) {
            int64_t v = (int64_t)t - 1;
            uint32_t back = 0;
            while (v >= 0 && !(wk.tabs[(uint64_t)v * HH_KM] & HH_CST) && back < HH_SCAN_BACK) {
                v--;
                back++;
            }
            if (back >= HH_SCAN_BACK) {
                atomicOr(wk.flags, (uint32_t)F_SCAN);   // the host composes the chain instead
            } else {
                s = v >= 0 ? hh_tab_state(wk.tabs[(uint64_t)v * HH_KM]) : geo.in_state;
                for (uint64_t u = (uint64_t)(v + 1); u < t; u++)
                    s = hh_tab_state(wk.tabs[u * HH_KM + (hh_state_d(s) & (HH_KM - 1u))]);
            }
        }
        wk.st[t] = s;
        if (t < geo.ntiles) {
            const uint64_t row = wk.tabs[t * HH_KM + (hh_state_d(s) & (HH_KM - 1u))];
            cst = (wk.tabs[t * HH_KM] & HH_CST) != 0;
            cnt = hh_tab_count(row);
            // a prologue tile emits nothing; the last one carries the entry
            // correction of the first emitted tile, so that its base is 0
            if (t < geo.emit_from) cnt = t + 1 == geo.emit_from ? hh_state_delta(hh_tab_state(row)) : 0;
        }
    }
    // CONST seen in the prologue / in the emitted tiles: one atomic per
    // block (one per wave on a single address serialises at the L2)
    const uint64_t mp = __ballot(cst && t < geo.emit_from), me = __ballot(cst && t >= geo.emit_from);
    if (threadIdx.x == 0) s_cf = 0u;
    __syncthreads();
    if ((threadIdx.x & 63u) == 0 && (mp | me)) atomicOr(&s_cf, (mp ? 1u : 0u) | (me ? 2u : 0u));
    int32_t tot;
    const int32_t ex = block_excl_scan<HH_SCAN_TB>(cnt, s_tmp, &tot);   // (barriers inside)
    if (threadIdx.x == 0) {
        if (s_cf & 1u) atomicOr(&wk.flags[12], 1u);
        if (s_cf & 2u) atomicOr(&wk.flags[13], 1u);
    }
    if (valid) wk.lex[t] = ex;
    if (threadIdx.x == 0) wk.blk[blockIdx.x] = tot;
}

// One block: exclusive scan of the block totals (int64) into block bases,
// starting from the stream-entry correction; the decode's totals.
__global__ __launch_bounds__(1024) void k_scan2(Geometry geo, Work wk, uint32_t nblk) {
    __shared__ int64_t s_w[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    int64_t carry = geo.emit_from ? 0 : (int64_t)hh_state_delta(geo.in_state);
    for (uint32_t b0 = 0; b0 < nblk; b0 += 1024) {
        const int64_t v = b0 + tid < nblk ? wk.blk[b0 + tid] : 0;
        int64_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) s_w[wv] = x;
        __syncthreads();
        int64_t base = 0, tot = 0;
        for (uint32_t i = 0; i < 16; i++) {
            base += i < wv ? s_w[i] : 0;
            tot += s_w[i];
        }
        if (b0 + tid < nblk) wk.blk[b0 + tid] = carry + base + x - v;
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) {
        const uint32_t leave = wk.st[geo.ntiles];
        const uint64_t total = (uint64_t)(carry - (int64_t)hh_state_delta(leave));
        wk.flags[2] = (uint32_t)total;
        wk.flags[3] = (uint32_t)(total >> 32);
        wk.flags[14] = leave;
        wk.flags[15] = geo.emit_from < geo.ntiles ? wk.st[geo.emit_from] : geo.in_state;
    }
}

// ---------------------------------------------------------------------------
// The emission loops take whole L1 lookups while p < this bound, then one
// lookup or symbol at a time.  A run's symbols all end by its end pe (a
// boundary of the true chain): a lookup from p < pe - HH_P ends by pe, and so
// does an escape's single symbol.  Only the stream's last run, which may end
// in a code cut by the end of the stream (the tail rule), keeps the longest
// code's margin.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t whole_lookups_end(uint32_t pe, uint32_t bt, uint32_t maxadv) {
    const uint32_t m = pe < bt ? HH_P : maxadv;
    return pe > m ? pe - m : 0u;
}

// ---------------------------------------------------------------------------
// A run [cu.p, pe) of the true chain decoded straight to HBM at dst: bytes up
// to a dword boundary, then dwords, then the ragged end (the first and last
// dwords may be shared with the neighbouring runs).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void emit_run_direct(const hh_ctx *c, hh_cur cu, uint32_t pe, uint8_t *dst,
                                                uint32_t maxadv) {
    uint32_t o = 0, val, k;
    while ((((uintptr_t)dst + o) & 3u) && cu.p < pe) {
        const uint32_t ha = o + (4u - (uint32_t)(((uintptr_t)dst + o) & 3u));
        hh_emit_step(c, cu, pe, o, ha, &val, &k);
        for (uint32_t i = 0; i < k; i++) dst[o + i] = (uint8_t)(val >> (8 * i));
        o += k;
    }
    uint64_t acc = 0;
    uint32_t nacc = 0;
    const uint32_t pf_end = whole_lookups_end(pe, c->bt, maxadv);
    while (cu.p < pf_end) {
        const uint32_t win = hh_cur_win(cu);
        const uint64_t le = c->l1[win & (HH_L1_SIZE - 1u)];
        const uint32_t m = (uint32_t)(le >> 32);
        uint32_t sy = (uint32_t)le, ns = HH_M_NSYM(m), nb = HH_M_NBITS(m);
        if (ns == 0) {
            nb = hh_escape(c, cu.p, win, m, &sy);
            ns = 1;
        }
        acc |= (uint64_t)sy << (8 * nacc);
        nacc += ns;
        if (nacc >= 4) {
            *(uint32_t *)(dst + o) = (uint32_t)acc;
            acc >>= 32;
            nacc -= 4;
            o += 4;
        }
        hh_cur_adv(c, cu, nb);
    }
    while (cu.p < pe) {
        hh_emit_step(c, cu, pe, o + nacc, ~0ull, &val, &k);
        acc |= (uint64_t)val << (8 * nacc);
        nacc += k;
        if (nacc >= 4) {
            *(uint32_t *)(dst + o) = (uint32_t)acc;
            acc >>= 32;
            nacc -= 4;
            o += 4;
        }
    }
    for (uint32_t i = 0; i < nacc; i++) dst[o + i] = (uint8_t)(acc >> (8 * i));
}

// ---------------------------------------------------------------------------
// k_emit: pass 2 of every emitted tile, one tile per wave at a time (wave gw
// takes tiles f0 + gw, f0 + gw + #waves, ...; f0 = emit_from).  Like
// k_front, a wave never waits for another: its tile's words, live lanes,
// run offsets (a wave scan) and output staging are its own.
// ---------------------------------------------------------------------------
template <uint32_t SW, uint32_t NW>
__global__ __launch_bounds__(64 * NW) void k_emit(const uint32_t *__restrict__ gdata, Geometry geo,
                                                               DevTab tab, Work wk, uint8_t *__restrict__ out,
                                                               uint64_t cap, uint64_t *dbg) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t NL = 64 * NW;
    __shared__ uint16_t s_eina[NW][HH_NR];  // run entries pushed by walkers
    __shared__ int16_t s_dina[NW][HH_NR];   // their deltas
    __shared__ uint8_t s_ka[NW][HH_NR];
    __shared__ uint8_t s_mema[NW][HH_NR];

    constexpr uint32_t S = 32 * SW;
    const uint32_t j = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint64_t *s_l1 = (uint64_t *)smem;                  // L1 entries as in global memory: one
                                                        // 64-bit read gives meta and symbols
    uint32_t *s_out = (uint32_t *)(s_l1 + HH_L1_SIZE) + wv * (HH_OBW / 4);   // the wave's staging
    uint32_t *s_w = (uint32_t *)(s_l1 + HH_L1_SIZE) + NW * (HH_OBW / 4) + wv * (SW * HH_NLS);
    uint32_t *s_l2 = (uint32_t *)(s_l1 + HH_L1_SIZE) + NW * (HH_OBW / 4 + SW * HH_NLS);
    uint32_t *s_tree = s_l2 + tab.l2_used;              // the compact tree (tail rule, long codes)
    uint8_t *s_tsym = (uint8_t *)(s_tree + tab.tree_lds);
    uint16_t *s_ein = s_eina[wv];
    int16_t *s_din = s_dina[wv];

    const uint64_t tile_bits = (uint64_t)HH_NR * S;
    const uint32_t span = HH_NCOL * S;
    for (uint32_t i = threadIdx.x; i < HH_L1_SIZE; i += NL) s_l1[i] = tab.l1[i];
    for (uint32_t i = threadIdx.x; i < tab.l2_used; i += NL) s_l2[i] = tab.l2[i];
    // with the tree in LDS too, the decode loops issue no global load: a
    // global load there would make them wait for the next tile's prefetch
    for (uint32_t i = threadIdx.x; i < tab.tree_lds; i += NL) {
        s_tree[i] = tab.tree[i];
        s_tsym[i] = tab.tsym[i];
    }
    __syncthreads();                                    // (the only workgroup barrier)

    hh_ctx c;
    c.w = s_w;
    c.sw = SW;
    c.nls = HH_NLS;
    c.magic = 0;
    c.l1 = s_l1;
    c.l1m = nullptr;
    c.l1s = nullptr;
    c.l2 = s_l2;
    c.tree = s_tree;                                    // (fast_path_ok: the tree fits)
    c.tsym = s_tsym;
    c.maxadv = geo.maxadv;
    c.G = geo.G;

    // The next tile's words, lane record, entering state and output base are
    // loaded one tile ahead (they are the loads every phase below waits on),
    // the meta words BEFORE the words (vmcnt retires in order: consuming them
    // then does not wait for the words).  The entering state and base are
    // uniform, but a uniform load is moved to an SGPR -- and waited for -- at
    // once; so lanes 0..3 load one word each (state, base low, base high,
    // block-local prefix), read out of those lanes where consumed.  Loads run
    // unconditionally, past the last tile on the last tile again.
    const uint64_t f0 = geo.emit_from;
    const uint64_t nwv = (uint64_t)gridDim.x * NW;
    const uint64_t tlast = geo.ntiles - 1;              // (launched only when f0 < ntiles)
    auto clampt = [&](uint64_t tt) { return tt < tlast ? tt : tlast; };
    Prefetch pf;
    uint32_t rec_n = 0, meta_n = 0;
    auto prefetch_next = [&](uint64_t tt) {
        rec_n = wk.recs[tt * HH_NR + j];
        const uint32_t *blk32 = (const uint32_t *)wk.blk + 2 * (tt / HH_SCAN_TB);
        const uint32_t ln = j & 3u;
        const uint32_t *src = ln == 0 ? &wk.st[tt] : ln == 1 ? blk32 : ln == 2 ? blk32 + 1
                                                                   : (const uint32_t *)&wk.lex[tt];
        meta_n = *src;
        prefetch_wtile<SW>(pf, gdata, tt * tile_bits / 32, geo.nwords);
    };
    uint64_t t = f0 + (uint64_t)blockIdx.x * NW + wv;
    const uint32_t gwe = blockIdx.x * NW + wv;       // this wave's list of deferred runs
    uint32_t xqn = 0;
    if (t < geo.ntiles) prefetch_next(t);
    EDIAG_DECL
    for (; t < geo.ntiles; t += nwv) {
        WAVE_SYNC();                                    // the previous tile's LDS no longer read
        const uint64_t rem = geo.bits - t * tile_bits;
        c.bt = rem < span ? (uint32_t)rem : span;
        const uint32_t bt = c.bt;
        store_wtile<SW>(pf, s_w);
        const uint32_t rec = rec_n;
        // (readlane returns int: every word is cast to uint32_t before widening)
        const uint32_t st_in = (uint32_t)__builtin_amdgcn_readlane(meta_n, 0);
        const uint32_t blo = (uint32_t)__builtin_amdgcn_readlane(meta_n, 1);
        const uint32_t bhi = (uint32_t)__builtin_amdgcn_readlane(meta_n, 2);
        const int32_t lex_t = __builtin_amdgcn_readlane(meta_n, 3);
        const int64_t base_t = (int64_t)(((uint64_t)bhi << 32) | blo) + (int64_t)lex_t;
        prefetch_next(clampt(t + nwv));
        const uint32_t kk = rec_k(rec), ee = rec_e(rec);
        const int32_t dl = rec_delta(rec);
        const uint32_t mem = resolve_live_wave(kk, s_ka[wv], s_mema[wv]);

        // the entering state: first live lane d_t, entered e_t bits in
        const uint32_t d_t = hh_state_d(st_in);
        const int32_t dprev = hh_state_delta(st_in);
        const bool live = (mem >> d_t) & 1u;
        if (live && j + kk < HH_NR) {
            s_ein[j + kk] = (j + kk) * S + ee;
            s_din[j + kk] = (int16_t)dl;
        }
        WAVE_SYNC();
        const uint32_t e_in = j == d_t ? d_t * S + hh_state_e(st_in) : s_ein[j];
        const int32_t d_in = j == d_t ? dprev : (int32_t)s_din[j];
        const uint32_t rc = live ? (uint32_t)((int32_t)rec_nc(rec) + d_in) : 0u;
        const int32_t incl = wave_incl_scan((int32_t)rc);
        const uint32_t L = (uint32_t)incl - rc;
        const uint32_t Tout = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
        const int64_t P0s = base_t - (int64_t)dprev;
        const uint64_t P0 = (uint64_t)P0s;
        // the tile's output fits [0, cap) (no wrap-around)
        const bool fits = P0s >= 0 && P0 <= cap && Tout <= cap - P0;
        if (j == 0 && !fits) atomicOr(wk.flags, (uint32_t)F_OVER);

        hh_cur cu = hh_cur_at(&c, live ? e_in : 0u);
        const uint32_t y = (j + kk) * S + ee;
        uint32_t pe = (live && fits) ? (y < bt ? y : bt) : 0u;
        {
            // A run over several regions (a walk that crossed them) would hold
            // up the wave for as many regions: it goes to the wave's list for
            // k_emitx (lane-parallel), unless the list is full.  Its bytes
            // are copied out as zeros here and written by k_emitx after.
            const bool want = kk > 1 && cu.p < pe;
            const uint64_t dm = __ballot(want);
            const uint32_t nd = (uint32_t)__builtin_popcountll(dm);
            if (nd && xqn + nd <= geo.xcap) {
                if (want) {
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u));
                    uint64_t *xe = wk.xq + 2 * ((uint64_t)gwe * geo.xcap + xqn + rank);
                    xe[0] = P0 + L;
                    xe[1] = (t << 32) | cu.p | (pe << 16);
                    pe = 0;
                }
                xqn += nd;
            }
        }
        // The tile's output [P0, P0 + Tout) is staged in the wave's LDS at
        // byte a0 = P0 mod 16, so that 16-B blocks of LDS and of HBM line
        // up: lanes OR their symbols in as dwords (a dword two runs share
        // needs the OR; the buffer is zeroed first), then the wave copies it
        // out with whole 16-B stores -- every line written once.
        const uint32_t a0 = (uint32_t)(P0 & 15u);
        if (fits && a0 + Tout <= HH_OBW) {
            EDIAG_STAMP(0);                             // (records, live lanes, scan)
            const uint32_t nq = (a0 + Tout + 15u) / 16u;
            for (uint32_t i = j; i < nq; i += 64) *(u32x4 *)(s_out + 4 * i) = (u32x4){0u, 0u, 0u, 0u};
            WAVE_SYNC();
            EDIAG_STAMP(1);                             // (zeroing)
            if (cu.p < pe) {
                const uint32_t b = a0 + L;
                uint32_t wd = b >> 2, nacc = b & 3u, val, k;
                uint64_t acc = 0;
                const uint32_t pf_end = whole_lookups_end(pe, bt, geo.maxadv);
                while (cu.p < pf_end) {            // whole lookups
                    const uint32_t win = hh_cur_win(cu);
                    const uint32_t ix = win & (HH_L1_SIZE - 1u);
                    const uint64_t le = s_l1[ix];
                    const uint32_t m = (uint32_t)(le >> 32);
                    uint32_t sy = (uint32_t)le, ns = HH_M_NSYM(m), nb = HH_M_NBITS(m);
                    if (ns == 0) {
                        nb = hh_escape(&c, cu.p, win, m, &sy);
                        ns = 1;
                    }
                    acc |= (uint64_t)sy << (8 * nacc);
                    nacc += ns;
                    if (nacc >= 4) {
                        atomicOr(&s_out[wd], (uint32_t)acc);
                        wd++;
                        acc >>= 32;
                        nacc -= 4;
                    }
                    hh_cur_adv(&c, cu, nb);
                }
                uint32_t emitted = 4 * wd + nacc - b;
                while (cu.p < pe) {                // the end of the run (and of the stream)
                    hh_emit_step(&c, cu, pe, emitted, rc, &val, &k);
                    acc |= (uint64_t)val << (8 * nacc);
                    nacc += k;
                    emitted += k;
                    if (nacc >= 4) {
                        atomicOr(&s_out[wd], (uint32_t)acc);
                        wd++;
                        acc >>= 32;
                        nacc -= 4;
                    }
                }
                if (nacc) atomicOr(&s_out[wd], (uint32_t)acc);
            }
            EDIAG_STAMP(2);                             // (own decode)
            WAVE_SYNC();
            uint8_t *gb = out + (P0 - a0);
            const uint8_t *sb = (const uint8_t *)s_out;
            for (uint32_t i = j; i < nq; i += 64) {
                const uint32_t lo = 16 * i;
                if (lo >= a0 && lo + 16 <= a0 + Tout) {
                    __builtin_nontemporal_store(*(const u32x4 *)(sb + lo), (u32x4 *)(gb + lo));
                } else {                           // a block shared with a neighbouring tile
                    const uint32_t e = lo + 16 < a0 + Tout ? lo + 16 : a0 + Tout;
                    for (uint32_t q = lo > a0 ? lo : a0; q < e; q++) gb[q] = sb[q];
                }
            }
            EDIAG_STAMP(4);                             // (copy-out)
            continue;
        }
        // a tile too large for the staging buffer: this lane's symbols
        // straight to HBM (output bytes [P0 + L, P0 + L + rc))
        if (cu.p < pe) emit_run_direct(&c, cu, pe, out + P0 + L, geo.maxadv);
    }
    if (j == 0) wk.xqn[gwe] = xqn;
    EDIAG_FLUSH(dbg);
}

// ---------------------------------------------------------------------------
// k_emitx: the runs k_emit deferred (several regions long), one lane each,
// over the lane's own staging of the run's words at LDS index
// (g - g0) * 64 + lane; straight to HBM (emit_run_direct).
// ---------------------------------------------------------------------------
template <uint32_t SW>
struct EmitxWin {
    static constexpr uint32_t n = (HH_KM + 1) * SW + 6;
};

template <uint32_t SW>
__global__ __launch_bounds__(64) void k_emitx(const uint32_t *__restrict__ gdata, Geometry geo, DevTab tab, Work wk,
                                              uint8_t *__restrict__ out, uint32_t nwe) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t S = 32 * SW, NW = EmitxWin<SW>::n;
    const uint32_t lane = threadIdx.x;
    uint64_t *s_l1 = (uint64_t *)smem;
    uint32_t *s_l2 = (uint32_t *)(s_l1 + HH_L1_SIZE);
    uint32_t *s_win = s_l2 + ((tab.l2_used + 3u) & ~3u) + lane;   // NW x 64 words
    for (uint32_t i = lane; i < HH_L1_SIZE; i += 64) s_l1[i] = tab.l1[i];
    for (uint32_t i = lane; i < tab.l2_used; i += 64) s_l2[i] = tab.l2[i];
    __syncthreads();
    const uint64_t tile_bits = (uint64_t)HH_NR * S;
    const uint32_t span = HH_NCOL * S;
    hh_ctx c;
    c.sw = 1024;                                        // hh_idx(g) = g * 64 (below)
    c.nls = 64;
    c.magic = 0;
    c.l1m = nullptr;
    c.l1s = nullptr;
    c.l1 = s_l1;
    c.l2 = s_l2;
    c.tree = tab.tree;
    c.tsym = tab.tsym;
    c.maxadv = geo.maxadv;
    c.G = geo.G;
    uint32_t fw = blockIdx.x, i = lane, cnt = fw < nwe ? wk.xqn[fw] : 0u;
    for (;;) {
        while (i >= cnt && fw < nwe) {
            i -= cnt;
            fw += gridDim.x;
            cnt = fw < nwe ? wk.xqn[fw] : 0u;
        }
        if (fw >= nwe) break;
        const uint64_t *xe = wk.xq + 2 * ((uint64_t)fw * geo.xcap + i);
        i += 64;
        const uint64_t O = xe[0], w1 = xe[1];
        const uint64_t t = w1 >> 32;
        const uint32_t e_in = (uint32_t)w1 & 0xffffu, pe = ((uint32_t)w1 >> 16) & 0xffffu;
        const uint64_t rem = geo.bits - t * tile_bits;
        c.bt = rem < span ? (uint32_t)rem : span;
        const uint32_t g0 = e_in >> 5;
        const uint64_t gw0 = t * tile_bits / 32 + g0, glim = geo.nwords;
#pragma unroll 8
        for (uint32_t q = 0; q < NW; q++) {
            const uint64_t gi = gw0 + q;
            s_win[q * 64] = gdata[gi < glim ? gi : glim - 1];
        }
        c.w = s_win - (int32_t)(g0 * 64);
        emit_run_direct(&c, hh_cur_at(&c, e_in), pe, out + O, geo.maxadv);
    }
}

// ---------------------------------------------------------------------------
// k_fixed: a complete fixed-length code (2^L symbols, every code L <= 8
// bits) needs no chain: symbol i is the L bits at i * L.  One thread per 16
// symbols, a 16-B store each; the stream's last code, if the end cuts it,
// takes the reference's tail rule (the node its bits reach,
// decodeallbits.cl:20-31).  sym[w] is the symbol of the L-bit window w
// (stream bit p in bit 0).
// ---------------------------------------------------------------------------
#ifndef HH_FIXED_NT
#define HH_FIXED_NT 1         // k_fixed's 16-B output stores nontemporal (E.coli 1 GiB 1.063 -> 1.048 ms)
#endif
__device__ __forceinline__ void fixed_store16(uint8_t *p, u32x4 v) {
    if (HH_FIXED_NT) __builtin_nontemporal_store(v, (u32x4 *)p);
    else *(u32x4 *)p = v;
}
__global__ __launch_bounds__(256) void k_fixed(const uint32_t *__restrict__ gdata, uint64_t bits, uint32_t L,
                                               const uint8_t *__restrict__ fsym, DevTab tab,
                                               uint8_t *__restrict__ out, uint64_t nsym) {
    __shared__ uint8_t s_sym[256];
    __shared__ uint32_t s_b4[256];                      // L = 2: a byte's four symbols
    const bool a16 = ((uintptr_t)out & 15u) == 0;
    s_sym[threadIdx.x] = fsym[threadIdx.x];
    {
        const uint32_t b = threadIdx.x;
        s_b4[b] = fsym[b & 3u] | (uint32_t)fsym[(b >> 2) & 3u] << 8 | (uint32_t)fsym[(b >> 4) & 3u] << 16 |
                  (uint32_t)fsym[b >> 6] << 24;
    }
    __syncthreads();
    const uint64_t nfull = bits / L;                    // whole codes
    const uint32_t mask = (1u << L) - 1u;
    const uint64_t G = (uint64_t)gridDim.x * blockDim.x;
    uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (L == 2 && a16) {
        // (E.coli) four groups per pass, their words loaded together: one
        // word -> four byte lookups -> one 16-B store each
        for (; (g + 3 * G) * 16 + 16 <= nfull; g += 4 * G) {
            uint32_t w[4];
#pragma unroll
            for (uint32_t u = 0; u < 4; u++) w[u] = gdata[g + u * G];
#pragma unroll
            for (uint32_t u = 0; u < 4; u++)
                fixed_store16(out + (g + u * G) * 16, (u32x4){s_b4[w[u] & 255u], s_b4[(w[u] >> 8) & 255u],
                                                              s_b4[(w[u] >> 16) & 255u], s_b4[w[u] >> 24]});
        }
    }
    for (; g * 16 < nsym; g += G) {
        const uint64_t i0 = g * 16, p0 = i0 * L;
        if (L == 2 && i0 + 16 <= nfull && a16) {       // (E.coli) one word, four byte lookups
            const uint32_t w = gdata[g];
            fixed_store16(out + i0, (u32x4){s_b4[w & 255u], s_b4[(w >> 8) & 255u], s_b4[(w >> 16) & 255u],
                                            s_b4[w >> 24]});
            continue;
        }
        uint64_t wi = p0 >> 5;
        uint64_t buf = ((uint64_t)gdata[wi + 1] << 32 | gdata[wi]) >> (p0 & 31);
        uint32_t have = 64 - (uint32_t)(p0 & 31);
        wi += 2;
        uint32_t v[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
            if (have < L) {                             // (L <= 8: one word tops it up)
                buf |= (uint64_t)gdata[wi++] << have;
                have += 32;
            }
            v[k >> 2] |= (uint32_t)s_sym[(uint32_t)buf & mask] << (8 * (k & 3));
            buf >>= L;
            have -= L;
        }
        if (i0 + 16 <= nfull && a16) {
            *(u32x4 *)(out + i0) = (u32x4){v[0], v[1], v[2], v[3]};
        } else {                                        // the stream's end (or an unaligned output)
            for (uint32_t k = 0; k < 16 && i0 + k < nsym; k++) {
                uint8_t b = (uint8_t)(v[k >> 2] >> (8 * (k & 3)));
                if (i0 + k == nfull) {                  // a code cut by the end: the tail rule
                    uint32_t node = 0;
                    for (uint64_t p = nfull * L; p < bits; p++) {
                        const uint32_t tn = tab.tree[node];
                        if (tn & HH_T_LEAF) break;
                        const uint32_t bit = (gdata[p >> 5] >> (p & 31)) & 1u;
                        node = bit ? (tn >> 15) & 0x7fffu : tn & 0x7fffu;
                    }
                    b = tab.tsym[node];
                }
                out[i0 + k] = b;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Segment path: exact and O(N) for any code of at most 32 bits, whether or
// not it resynchronises (the fast path's walks need it to).  The stream is
// cut into segments of `seglen` bits.  The chain through a segment is fixed
// by the offset o in [0, maxadv) of its first boundary past the segment
// start, so k_seg_func decodes every segment from every o (one lane each):
// the exit offset into the next segment and the symbols starting in the
// segment.  The host composes the maps from segment 0 (offset 0): entry
// offsets and output bases.  k_seg_emit re-decodes every segment from its
// true entry (one lane each) straight to HBM.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void seg_ctx(hh_ctx &c, const uint32_t *gdata, uint64_t seg0, uint64_t bits,
                                        uint32_t seglen, const uint32_t *s_l1m, const DevTab &tab,
                                        uint32_t maxadv) {
    c.w = gdata + seg0 / 32;                            // linear words of the segment:
    c.sw = 1;                                           // hh_idx(g) == g
    c.nls = 1;
    c.magic = 0;
    c.l1m = s_l1m;
    c.l1s = nullptr;
    c.l1 = nullptr;
    c.l2 = tab.l2;
    c.tree = tab.tree;
    c.tsym = tab.tsym;
    c.maxadv = maxadv;
    c.G = 0;
    const uint64_t rem = bits - seg0;
    const uint64_t lim = (uint64_t)seglen + 2 * maxadv;
    c.bt = (uint32_t)(rem < lim ? rem : lim);
}

__global__ __launch_bounds__(256) void k_seg_func(const uint32_t *__restrict__ gdata, uint64_t bits,
                                                  uint32_t seglen, uint32_t nseg, uint32_t no,
                                                  DevTab tab, uint32_t maxadv, uint32_t *exits,
                                                  uint32_t *counts) {
    __shared__ uint32_t s_l1m[HH_L1_SIZE];
    for (uint32_t i = threadIdx.x; i < HH_L1_SIZE; i += blockDim.x) s_l1m[i] = (uint32_t)(tab.l1[i] >> 32);
    __syncthreads();
    const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (uint64_t)nseg * no) return;
    const uint32_t sg = (uint32_t)(id / no), o = (uint32_t)(id % no);
    const uint64_t seg0 = (uint64_t)sg * seglen;
    hh_ctx c;
    seg_ctx(c, gdata, seg0, bits, seglen, s_l1m, tab, maxadv);
    const uint32_t end = c.bt < seglen ? c.bt : seglen;  // symbols starting before it count
    uint32_t n = 0, x = o;
    if (o < end) x = hh_region_count(&c, o, end, &n);
    exits[id] = x >= end ? x - end : 0u;                // offset into the next segment
    counts[id] = n;
}

__global__ __launch_bounds__(256) void k_seg_emit(const uint32_t *__restrict__ gdata, uint64_t bits,
                                                  uint32_t seglen, uint32_t nseg, DevTab tab,
                                                  uint32_t maxadv, const uint32_t *entry,
                                                  const uint32_t *exitv, const uint64_t *base,
                                                  uint8_t *__restrict__ out) {
    __shared__ uint32_t s_l1m[HH_L1_SIZE];
    __shared__ uint32_t s_l1s[HH_L1_SIZE];
    for (uint32_t i = threadIdx.x; i < HH_L1_SIZE; i += blockDim.x) {
        const uint64_t e = tab.l1[i];
        s_l1m[i] = (uint32_t)(e >> 32);
        s_l1s[i] = (uint32_t)e;
    }
    __syncthreads();
    const uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= nseg) return;
    const uint64_t seg0 = (uint64_t)sg * seglen;
    hh_ctx c;
    seg_ctx(c, gdata, seg0, bits, seglen, s_l1m, tab, maxadv);
    c.l1s = s_l1s;
    const uint32_t end = c.bt < seglen ? c.bt : seglen;
    const uint32_t e0 = entry[sg];
    // the run ends at the first boundary at or past the segment end (or bt)
    const uint32_t pe0 = end + exitv[sg], pe = pe0 < c.bt ? pe0 : c.bt;
    if (e0 >= end) return;
    uint8_t *ob = out + base[sg];
    hh_cur cu = hh_cur_at(&c, e0);
    uint64_t o = 0;
    uint32_t val, k;
    while (cu.p < pe) {
        hh_emit_step(&c, cu, pe, o, ~0ull, &val, &k);
        for (uint32_t i = 0; i < k; i++) ob[o + i] = (uint8_t)(val >> (8 * i));
        o += k;
    }
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

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
typedef void (*kfront_t)(const uint32_t *, Geometry, DevTab, Work, uint64_t *);
typedef void (*kemit_t)(const uint32_t *, Geometry, DevTab, Work, uint8_t *, uint64_t, uint64_t *);

struct hh_decoder {
    int device;
    hh_config cfg;
    hipStream_t stream;
    hh_tables *ht;
    int have_tree;
    uint64_t *d_l1;
    uint16_t *d_f;
    uint32_t *d_fdir;
    uint32_t *d_l2;
    uint32_t *d_tree;
    uint8_t *d_tsym;
    DevTab tab;
    uint32_t S;
    uint32_t G;          // overlap bits (hh_pick_overlap; HH_OVERLAP overrides)
    // workspace
    void *ws;
    size_t ws_size;
    uint32_t *h_flags;   // pinned
    int32_t *d_max;      // findmax result (stage API)
    uint64_t *d_dbg;     // HH_DIAG counters (16 x u64)
    hipEvent_t ev[4];
    hipEvent_t ev2[4];         // result slot 1's events (an asynchronous decode behind another)
    hh_stats stats;
    uint32_t grid_f, grid_e, grid_w, grid_x;   // persistent grid sizes (occupancy x CUs)
    uint32_t fwalk;            // k_front's walk bound (HH_FRONT_WALK overrides)
    uint32_t ncu;              // compute units
    uint32_t fixed_len;        // L of a complete fixed-length code (k_fixed), else 0
    uint8_t *d_fsym;           // its 256-entry window -> symbol table
    uint32_t emit_nw;          // k_emit's waves per workgroup (size_grids)
    uint32_t emit_nw_max;      // the largest tried (HH_EMIT_NW = 8 forces the smaller one)
    uint32_t xpt;              // k_emit's deferred runs per tile (HH_EMIT_XPT overrides)
    uint32_t grid_sw;          // words per region they were sized for
    size_t grid_l2;            // and the L2 table size
    uint32_t grid_tree;        // and the LDS tree size
    uint32_t grid_fdir;        // and the F escape directory
    uint32_t grid_nw_max;      // and k_emit's largest workgroup
    // host staging of the evaluate() scope (hh_decode_host)
    uint8_t *h_stage;          // 2 x HH_HOST_CHUNK pinned (hh_decode_host)
    hipEvent_t h_ev[2];
    void *d_in, *d_out;
    size_t d_in_size, d_out_size;
    // the state-machine decode (hh_fsm.hip): tables, device copies, workspace
    hh_fsm_tables *ft;
    FsmDev fsm;
    FsmWs fsm_ws;
    // evaluate() scope pipeline (host_pipeline): copy streams, per-chunk events
    hipStream_t h2d, d2h;
    hipEvent_t *pipe_ev;
    uint32_t npipe_ev;
    // caller buffers kept page-locked across calls (HH_FLAG_KEEP_HOST_PINNED)
    const void *pin_p[2];
    size_t pin_n[2];
    int pin_own[2];      // 1: pin_p[k] registered for buffer k (pages pin_ra..pin_rb); 0: inside k^1's
    uintptr_t pin_ra[2], pin_rb[2];
    // the asynchronous decode not checked yet (hh_decode_device_async)
    struct {
        int active;
        int fixed;             // a k_fixed launch (the length was known at launch)
        FsmPend pd;
        const void *d_data;
        uint64_t bits;
        void *d_out;
        uint64_t *out_len;
        hipStream_t st;
        hh_range_out *ro;      // a segment's decode (hh_decode_device_range_async): its results
    } apend;
    int async_rc;              // the first failure since the last hh_decode_wait
    uint32_t async_seq;        // asynchronous decodes launched (the result slot alternates)
};

static int async_check(hh_decoder *d);

static int ensure_dev(void **p, size_t *have, size_t need) {
    if (*have >= need) return HH_OK;
    if (*p) HIP_OK(hipFree(*p));
    *p = nullptr;
    *have = 0;
    const size_t sz = need + need / 8;
    if (hipMalloc(p, sz) != hipSuccess) return HH_ERR_NOMEM;
    *have = sz;
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
    d->ft = (hh_fsm_tables *)calloc(1, sizeof(hh_fsm_tables));
    if (!d->ht || !d->ft) { free(d->ht); free(d->ft); free(d); return HH_ERR_NOMEM; }
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d->d_l1, sizeof(uint64_t) * HH_L1_SIZE) != hipSuccess ||
        hipMalloc(&d->d_l2, sizeof(uint32_t) * HH_L2_MAX) != hipSuccess ||
        hipMalloc(&d->d_f, sizeof(uint16_t) * HH_F_SIZE) != hipSuccess ||
        hipMalloc(&d->d_fdir, sizeof(uint32_t) * HH_L2_MAX) != hipSuccess ||
        hipMalloc(&d->d_fsym, 256) != hipSuccess ||
        hipMalloc(&d->d_tree, sizeof(uint32_t) * (HH_TREE_MAX + 1)) != hipSuccess ||
        hipMalloc(&d->d_tsym, HH_TREE_MAX + 1) != hipSuccess ||
        hipMalloc(&d->d_max, 16) != hipSuccess ||
        hipMalloc(&d->d_dbg, HH_DBG_WORDS * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc((void **)&d->h_flags, 64, hipHostMallocDefault) != hipSuccess) {
        hh_decoder_destroy(d);
        return HH_ERR_DEVICE;
    }
    for (int i = 0; i < 4; i++) {
        if (hipEventCreate(&d->ev[i]) != hipSuccess || hipEventCreate(&d->ev2[i]) != hipSuccess) {
            hh_decoder_destroy(d);
            return HH_ERR_DEVICE;
        }
    }
    *out = d;
    return HH_OK;
}

extern "C" void hh_decoder_destroy(hh_decoder *d) {
    if (!d) return;
    hipSetDevice(d->device);
    async_check(d);                     // (an asynchronous decode still running)
    hh_decoder_release_host(d);
    if (d->ws) hipFree(d->ws);
    if (d->d_l1) hipFree(d->d_l1);
    if (d->d_l2) hipFree(d->d_l2);
    if (d->d_f) hipFree(d->d_f);
    if (d->d_fdir) hipFree(d->d_fdir);
    if (d->d_fsym) hipFree(d->d_fsym);
    if (d->d_tree) hipFree(d->d_tree);
    if (d->d_tsym) hipFree(d->d_tsym);
    if (d->d_max) hipFree(d->d_max);
    if (d->d_dbg) hipFree(d->d_dbg);
    if (d->d_in) hipFree(d->d_in);
    if (d->d_out) hipFree(d->d_out);
    if (d->h_stage) {
        hipHostFree(d->h_stage);
        hipEventDestroy(d->h_ev[0]);
        hipEventDestroy(d->h_ev[1]);
    }
    if (d->h_flags) hipHostFree(d->h_flags);
    for (int i = 0; i < 4; i++) {
        if (d->ev[i]) hipEventDestroy(d->ev[i]);
        if (d->ev2[i]) hipEventDestroy(d->ev2[i]);
    }
    if (d->stream) hipStreamDestroy(d->stream);
    fsm_free(&d->fsm);
    fsm_ws_free(&d->fsm_ws);
    for (uint32_t i = 0; i < d->npipe_ev; i++) hipEventDestroy(d->pipe_ev[i]);
    free(d->pipe_ev);
    if (d->h2d) hipStreamDestroy(d->h2d);
    if (d->d2h) hipStreamDestroy(d->d2h);
    free(d->ht);
    free(d->ft);
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
    uint32_t S = hh_pick_region_bits(g);
    // A fixed-length code puts HH_NR * S / len symbols in every tile: keep
    // that within k_emit's staging buffer (E.coli: 2-bit codes, S = 128).
    if (t->fixed_len > 0 && S) {
        uint32_t x = 32, y = g;
        while (y) { const uint32_t r = x % y; x = y; y = r; }
        const uint32_t lcm = 32 / x * g;
        const uint64_t smax = (uint64_t)(HH_OBW - 64) * (uint32_t)t->fixed_len / HH_NR;
        while (S > smax && S > lcm) S -= lcm;
    }
    return S;
}

extern "C" int hh_decoder_set_tree(hh_decoder *d, const hh_tree *tree) {
    if (!d || !tree) return HH_ERR_ARG;
    HIP_OK(hipSetDevice(d->device));
    async_check(d);                     // (a pending asynchronous decode uses the current tables)
    int rc = hh_tables_build(tree, d->ht);
    if (rc) return rc;
    HIP_OK(hipSetDevice(d->device));
    HIP_OK(hipMemcpy(d->d_l1, d->ht->l1, sizeof(uint64_t) * HH_L1_SIZE, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_l2, d->ht->l2, sizeof(uint32_t) * HH_L2_MAX, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_tree, d->ht->tree, sizeof(uint32_t) * (HH_TREE_MAX + 1), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_tsym, d->ht->tsym, HH_TREE_MAX + 1, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_f, d->ht->f, sizeof(d->ht->f), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d->d_fdir, d->ht->fdir, sizeof(uint32_t) * (d->ht->fdir_used ? d->ht->fdir_used : 1), hipMemcpyHostToDevice));
    d->tab.f = d->d_f;
    d->tab.fdir = d->d_fdir;
    d->tab.fdir_used = d->ht->fdir_used;
    d->tab.l1 = d->d_l1;
    d->tab.l2 = d->d_l2;
    d->tab.tree = d->d_tree;
    d->tab.tsym = d->d_tsym;
    d->tab.l2_used = d->ht->l2_used;
    d->tab.tree_lds = d->ht->tree_used;
    d->S = pick_region_bits(d->ht, d->cfg.lane_bits);
    // trees of more than 127 states: the state machine counts in 7-bit steps
    // over 224-bit regions (hh_fsm.h), and the decoder's tiles are its tiles
    // (tile_bits, shards, the evaluate() chunks)
    if (!(d->cfg.flags & HH_FLAG_LEGACY) && d->cfg.lane_bits == 0) {
        const uint32_t Sf = hh_fsm_region_bits(hh_fsm_nstates(d->ht), (uint32_t)d->ht->len_gcd, d->S);
        if (Sf) d->S = Sf;
    }
    // a complete fixed-length code: every L-bit window is one symbol
    d->fixed_len = 0;
    const int L = d->ht->fixed_len;
    if (L >= 1 && L <= 8 && d->ht->tree_used == (2u << L) - 1u) {
        uint8_t fs[256];
        for (uint32_t w = 0; w < 256; w++) {
            uint32_t node = 0;
            for (int b = 0; b < L; b++) {
                const uint32_t tn = d->ht->tree[node];
                node = (w >> b) & 1u ? (tn >> 15) & 0x7fffu : tn & 0x7fffu;
            }
            fs[w] = (uint8_t)(d->ht->tree[node] & 0xffu);
        }
        HIP_OK(hipMemcpy(d->d_fsym, fs, 256, hipMemcpyHostToDevice));
        d->fixed_len = (uint32_t)L;
    }
    d->fwalk = HH_FRONT_WALK;
    const char *fw = getenv("HH_FRONT_WALK");            // experiments, tests
    if (fw && *fw) d->fwalk = (uint32_t)atoi(fw);
    d->xpt = HH_XPT;
    d->emit_nw_max = HH_EMIT_NW_MAX;
    const char *enw = getenv("HH_EMIT_NW");
    if (enw && atoi(enw) == 8) d->emit_nw_max = 8;
    const char *xp = getenv("HH_EMIT_XPT");
    if (xp && *xp) d->xpt = (uint32_t)atoi(xp);
    d->G = hh_pick_overlap(d->ht);
    if (getenv("HH_OVERLAP")) d->G = (uint32_t)atoi(getenv("HH_OVERLAP")) & ~31u;   // experiments
    if (d->G > HH_GMAX || d->G + 32 > d->S) d->G = 0;
    // the state machine (trees of at most HH_FSM_MAXS = 255 internal nodes)
    fsm_free(&d->fsm);
    // emission steps of 7 bits when their tables leave room for 16 stagings
    // of the expected tile output (fsm_k_fits), else 6 or 5 (smaller tables,
    // more waves), 6 when none does; HH_FSM_K: experiments.  Expected bits per symbol: the code lengths weighted by
    // 2^-length (exact for a code built from a dyadic distribution).
    double avg = 0.0;
    {
        uint32_t stk[64], dep[64], sp = 0;
        stk[sp] = 0; dep[sp++] = 0;
        while (sp) {
            const uint32_t id = stk[--sp], dd = dep[sp];
            const uint32_t e = d->ht->tree[id];
            if ((e & HH_T_LEAF) || dd >= 62) { avg += dd * ldexp(1.0, -(int)dd); continue; }
            stk[sp] = e & 0x7fffu; dep[sp++] = dd + 1;
            stk[sp] = (e >> 15) & 0x7fffu; dep[sp++] = dd + 1;
        }
    }
    const uint32_t est = avg > 0.0 ? (uint32_t)(64.0 * d->S / avg) : 64u * d->S;
    uint32_t Kf = getenv("HH_FSM_K") ? (uint32_t)atoi(getenv("HH_FSM_K")) : 0u;
    // the widest step whose tables leave room for 16 stagings: kjv-like
    // alphabets 7; a byte alphabet (255 states, at most 6) 5 -- its 6-bit
    // tables leave room for 6 waves' stagings (emit 1.07 -> 0.97 ms per GiB)
    for (uint32_t k = 7; !Kf && d->S && k >= 5; k--)
        if (hh_fsm_build(d->ht, d->S, k, d->ft) == HH_OK && d->ft->K == k && fsm_k_fits(d->ft, est)) Kf = k;
    if (d->S && hh_fsm_build(d->ht, d->S, Kf ? Kf : 6, d->ft) == HH_OK) {
        uint32_t Gf = hh_fsm_pick_head(d->ht, d->S, d->ft->cb);
        if (getenv("HH_FSM_HEAD")) Gf = (uint32_t)atoi(getenv("HH_FSM_HEAD")) / d->ft->cb * d->ft->cb;   // experiments
        if (Gf > d->S) Gf = 0;
        const int urc = fsm_upload(&d->fsm, d->ft, Gf, (uint32_t)d->ht->minlen, (uint32_t)d->ht->maxlen);
        d->fsm.dbg = d->d_dbg;
        d->fsm.phases = (d->cfg.flags & HH_FLAG_PHASE_TIMING) != 0;
        d->fsm.two_pass = (d->cfg.flags & HH_FLAG_TWO_PASS) != 0;
        if (urc != HH_OK && urc != HH_ERR_UNSUPPORTED) return urc;
        // the single pass (hh_one.hip): its head over the emission table's
        // K-bit steps, on the code lattice like the count pass's
        uint32_t G1 = hh_fsm_pick_head(d->ht, d->S, d->ft->K);
        if (getenv("HH_FSM_HEAD")) G1 = (uint32_t)atoi(getenv("HH_FSM_HEAD")) / d->ft->K * d->ft->K;   // experiments
        if (urc == HH_OK) one_setup(&d->fsm, G1 > d->S ? 0u : G1, avg, (uint32_t)d->ht->minlen);
    }
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
           d->ht->tree_used <= HH_TREE_LDS_MAX && !(d->cfg.flags & (HH_FLAG_FORCE_EXACT | HH_FLAG_FORCE_SEGMENT));
}

static int stage_pipeline(hh_decoder *d, const void *d_data, int64_t bits, uint8_t *d_out,
                          uint64_t cap, uint64_t *out_len, hipStream_t st);

static size_t lds_front(uint32_t sw, uint32_t l2, uint32_t fdir) {
    return ((size_t)ftab_words(fdir, l2) + (size_t)HH_FW * sw * HH_NLS) * 4;
}
static uint32_t walk_win(uint32_t sw) { return sw + 6; }   // WalkWin<sw>::n
static size_t lds_walk(uint32_t sw, uint32_t l2, uint32_t fdir) {
    return ((size_t)ftab_words(fdir, l2) + (size_t)walk_win(sw) * HH_WALK_T) * 4;
}
static size_t lds_emitx(uint32_t sw, uint32_t l2) {
    return (size_t)HH_L1_SIZE * 8 + (size_t)((l2 + 3) & ~3u) * 4 + (size_t)((HH_KM + 1) * sw + 6) * 64 * 4;
}
static size_t lds_emit(uint32_t sw, uint32_t l2, uint32_t tree, uint32_t nw) {
    return (2 * (size_t)HH_L1_SIZE + (size_t)nw * sw * HH_NLS + l2) * 4 + (size_t)nw * HH_OBW +
           (size_t)tree * 5;
}

// kernels instantiated per words-per-region (S = 32 * SW bits)
#define HH_SW_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
static kfront_t kfront_for(uint32_t sw) {
    switch (sw) {
#define X(n) case n: return k_front<n>;
        HH_SW_CASES(X)
#undef X
    default: return nullptr;
    }
}
typedef void (*kwalk_t)(const uint32_t *, Geometry, DevTab, Work);
static kwalk_t kwalk_for(uint32_t sw) {
    switch (sw) {
#define X(n) case n: return k_walk<n>;
        HH_SW_CASES(X)
#undef X
    default: return nullptr;
    }
}
typedef void (*kemitx_t)(const uint32_t *, Geometry, DevTab, Work, uint8_t *, uint32_t);
static kemitx_t kemitx_for(uint32_t sw) {
    switch (sw) {
#define X(n) case n: return k_emitx<n>;
        HH_SW_CASES(X)
#undef X
    default: return nullptr;
    }
}
static kemit_t kemit_for(uint32_t sw, uint32_t nw) {
    switch (sw) {
#define X(n) case n: return nw == 16 ? k_emit<n, 16> : k_emit<n, 8>;
        HH_SW_CASES(X)
#undef X
    default: return nullptr;
    }
}

// Persistent grids: the occupancy answer x CUs for each kernel.
static int size_grids(hh_decoder *d, uint32_t sw) {
    if (d->grid_f && d->grid_sw == sw && d->grid_l2 == d->tab.l2_used && d->grid_tree == d->tab.tree_lds &&
        d->grid_fdir == d->tab.fdir_used && d->grid_nw_max == d->emit_nw_max)
        return HH_OK;
    int pf = 0, pe = 0, pw = 0, px = 0, ncu = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pf, kfront_for(sw), 64 * HH_FW, lds_front(sw, d->tab.l2_used, d->tab.fdir_used)));
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pw, kwalk_for(sw), HH_WALK_T, lds_walk(sw, d->tab.l2_used, d->tab.fdir_used)));
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&px, kemitx_for(sw), 64, lds_emitx(sw, d->tab.l2_used)));
    uint32_t nw = d->emit_nw_max;
    for (;; nw /= 2) {
        pe = 0;
        const size_t lds = lds_emit(sw, d->tab.l2_used, d->tab.tree_lds, nw);
        if (lds + (size_t)nw * HH_NR * 6 <= 160 * 1024)   // (+ the static per-wave arrays)
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pe, kemit_for(sw, nw), 64 * nw, lds));
        if (pe >= 1 || nw == 8) break;
    }
    d->emit_nw = nw;
    HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d->device));
    if (pf < 1 || pe < 1 || pw < 1 || px < 1) return HH_ERR_UNSUPPORTED;
    d->grid_f = (uint32_t)(pf * ncu);
    d->grid_w = (uint32_t)(pw * ncu);
    d->grid_x = (uint32_t)(px * ncu);
    d->ncu = (uint32_t)ncu;
    d->grid_e = (uint32_t)(pe * ncu);
    d->grid_sw = sw;
    d->grid_l2 = d->tab.l2_used;
    d->grid_tree = d->tab.tree_lds;
    d->grid_fdir = d->tab.fdir_used;
    d->grid_nw_max = d->emit_nw_max;
    return HH_OK;
}

// The host's version of k_scan1/k_scan2 for streams whose non-CONST chains
// are longer than HH_SCAN_BACK tiles (codes that resynchronise but whose
// leaving state stays entry-dependent for thousands of tiles): one
// sequential pass over the tables.
static int scan_host(hh_decoder *d, const Geometry &geo, const Work &wk, uint32_t nblk, hipStream_t st) {
    const uint64_t nt = geo.ntiles;
    uint64_t *tabs = (uint64_t *)malloc(nt * HH_KM * 8);
    uint32_t *sts = (uint32_t *)malloc((nt + 1) * 4);
    int32_t *lex = (int32_t *)malloc((nt + 1) * 4);
    int64_t *blk = (int64_t *)malloc((size_t)nblk * 8);
    int rc = HH_OK;
    if (!tabs || !sts || !lex || !blk) { rc = HH_ERR_NOMEM; goto out; }
    if (hipMemcpyAsync(tabs, wk.tabs, nt * HH_KM * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { rc = HH_ERR_DEVICE; goto out; }
    {
        uint32_t s = geo.in_state;
        int64_t run = geo.emit_from ? 0 : hh_state_delta(geo.in_state), bsum = 0;
        for (uint64_t t = 0; t <= nt; t++) {
            if (t % HH_SCAN_TB == 0) {
                blk[t / HH_SCAN_TB] = run;
                bsum = 0;
            }
            sts[t] = s;
            lex[t] = (int32_t)bsum;
            if (t == nt) break;
            const uint64_t row = tabs[t * HH_KM + (hh_state_d(s) & (HH_KM - 1u))];
            int32_t cnt = hh_tab_count(row);
            if (t < geo.emit_from) cnt = t + 1 == geo.emit_from ? hh_state_delta(hh_tab_state(row)) : 0;
            bsum += cnt;
            run += cnt;
            s = hh_tab_state(row);
        }
        const uint64_t total = (uint64_t)(run - hh_state_delta(s));
        uint32_t fl[16];
        memcpy(fl, d->h_flags, sizeof(fl));
        fl[0] &= ~(uint32_t)F_SCAN;
        fl[2] = (uint32_t)total;
        fl[3] = (uint32_t)(total >> 32);
        fl[14] = s;
        fl[15] = geo.emit_from < nt ? sts[geo.emit_from] : geo.in_state;
        if (hipMemcpyAsync(wk.st, sts, (nt + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(wk.lex, lex, (nt + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(wk.blk, blk, (size_t)nblk * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(wk.flags, fl, sizeof(fl), hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = HH_ERR_DEVICE;
    }
out:
    free(tabs);
    free(sts);
    free(lex);
    free(blk);
    return rc;
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
    geo.maxadv = d->ht->maxlen > HH_P ? (uint32_t)d->ht->maxlen : HH_P;
    geo.G = d->G;
    geo.nwords = ((bits_avail + 7) / 8 + HH_PAYLOAD_PAD) / 4;
    geo.in_state = in_state;
    geo.emit_from = emit_from;
    geo.fwalk = d->fwalk;
    const uint64_t tb = (uint64_t)HH_NR * d->S;
    const uint64_t all = (bits_avail + tb - 1) / tb;
    geo.ntiles = ntiles && ntiles < all ? ntiles : all;
    const uint64_t nt = geo.ntiles;
    const uint32_t nblk = (uint32_t)((nt + 1 + HH_SCAN_TB - 1) / HH_SCAN_TB);
    // workspace: flags 64 B | tabs | recs | st | lex | blk | q
    const size_t o_tabs = 64, o_recs = o_tabs + nt * HH_KM * 8, o_st = o_recs + nt * HH_NR * 4;
    const size_t o_lex = (o_st + (nt + 1) * 4 + 7) & ~(size_t)7, o_blk = (o_lex + (nt + 1) * 4 + 7) & ~(size_t)7;
    int rc = size_grids(d, geo.sw);
    if (rc) return rc;
    // one tile per wave at a time in both kernels
    const uint64_t nfw = (nt + HH_FW - 1) / HH_FW;
    const uint32_t gf = (uint32_t)(nfw < d->grid_f ? nfw : d->grid_f);
    geo.nfw = gf * HH_FW;
    geo.qcap = (nt + geo.nfw - 1) / geo.nfw * HH_NR;
    const size_t o_qn = o_blk + (size_t)nblk * 8, o_q = (o_qn + (size_t)geo.nfw * 4 + 7) & ~(size_t)7;
    const size_t o_xn = o_q + (size_t)geo.nfw * geo.qcap * 8;
    const uint64_t ne = nt > emit_from ? nt - emit_from : 0;
    const uint32_t enw = d->emit_nw;
    const uint64_t ng = (ne + enw - 1) / enw;              // workgroups' worth of tiles
    const uint32_t ge = (uint32_t)(ng < d->grid_e ? (ng ? ng : 1) : d->grid_e);
    const uint32_t nwe = ge * enw;                          // k_emit's waves
    geo.xcap = (uint32_t)((ne + nwe - 1) / nwe * d->xpt);
    const size_t o_xqn = o_xn + (nt + 1) * HH_NR * 4, o_xq = (o_xqn + (size_t)nwe * 4 + 15) & ~(size_t)15;
    const size_t need = o_xq + (size_t)nwe * geo.xcap * 16;
    rc = ensure_dev(&d->ws, &d->ws_size, need);
    if (rc) return rc;
    uint8_t *w = (uint8_t *)d->ws;
    Work wk;
    wk.flags = (uint32_t *)w;
    wk.tabs = (uint64_t *)(w + o_tabs);
    wk.recs = (uint32_t *)(w + o_recs);
    wk.st = (uint32_t *)(w + o_st);
    wk.lex = (int32_t *)(w + o_lex);
    wk.blk = (int64_t *)(w + o_blk);
    wk.q = (uint64_t *)(w + o_q);
    wk.qn = (uint32_t *)(w + o_qn);
    wk.xn = (uint32_t *)(w + o_xn);
    wk.xqn = (uint32_t *)(w + o_xqn);
    wk.xq = (uint64_t *)(w + o_xq);
    const kfront_t kf = kfront_for(geo.sw);
    const kwalk_t kw = kwalk_for(geo.sw);
    const kemit_t ke = kemit_for(geo.sw, enw);
    const kemitx_t kx = kemitx_for(geo.sw);
    if (!kf || !kw || !ke || !kx) return HH_ERR_UNSUPPORTED;
    // k_emit, then the runs it deferred
    auto launch_emit = [&]() -> int {
        hipLaunchKernelGGL(ke, dim3(ge), dim3(64 * enw), lds_emit(geo.sw, d->tab.l2_used, d->tab.tree_lds, enw), st,
                           (const uint32_t *)d_data, geo, d->tab, wk, (uint8_t *)d_out, cap, d->d_dbg);
        HIP_OK(hipGetLastError());
        hipLaunchKernelGGL(kx, dim3(d->grid_x), dim3(64), lds_emitx(geo.sw, d->tab.l2_used), st,
                           (const uint32_t *)d_data, geo, d->tab, wk, (uint8_t *)d_out, nwe);
        HIP_OK(hipGetLastError());
        return HH_OK;
    };

    HIP_OK(hipMemsetAsync(wk.flags, 0, 64, st));
#ifdef HH_DIAG
    HIP_OK(hipMemsetAsync(d->d_dbg, 0, 16 * sizeof(uint64_t), st));
#endif
    HIP_OK(hipEventRecord(d->ev[0], st));
    hipLaunchKernelGGL(kf, dim3(gf), dim3(64 * HH_FW), lds_front(geo.sw, d->tab.l2_used, d->tab.fdir_used), st,
                       (const uint32_t *)d_data, geo, d->tab, wk, d->d_dbg);
    HIP_OK(hipGetLastError());
    // the deferred walks (their count is on the device: a persistent grid)
    hipLaunchKernelGGL(kw, dim3(d->grid_w), dim3(HH_WALK_T), lds_walk(geo.sw, d->tab.l2_used, d->tab.fdir_used), st,
                       (const uint32_t *)d_data, geo, d->tab, wk);
    HIP_OK(hipGetLastError());
    {
        // persistent: each wave's next record is loaded a tile ahead
        const uint64_t nb = (nt + HH_TABLE_W - 1) / HH_TABLE_W, cap = (uint64_t)d->ncu * 8;
        hipLaunchKernelGGL(k_table, dim3((unsigned)(nb < cap ? nb : cap)), dim3(64 * HH_TABLE_W), 0, st, geo, wk);
        HIP_OK(hipGetLastError());
    }
    HIP_OK(hipEventRecord(d->ev[1], st));
    hipLaunchKernelGGL(k_scan1, dim3(nblk), dim3(HH_SCAN_TB), 0, st, geo, wk);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_scan2, dim3(1), dim3(1024), 0, st, geo, wk, nblk);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(d->ev[2], st));
    if (ne && (rc = launch_emit())) return rc;
    HIP_OK(hipEventRecord(d->ev[3], st));
    HIP_OK(hipMemcpyAsync(d->h_flags, wk.flags, 64, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if ((d->h_flags[0] & F_SCAN) && !(d->h_flags[0] & F_FAIL)) {
        // a non-CONST chain too long for k_scan1: compose on the host, emit again
        rc = scan_host(d, geo, wk, nblk, st);
        if (rc) return rc;
        if (ne && (rc = launch_emit())) return rc;
        HIP_OK(hipEventRecord(d->ev[3], st));
        HIP_OK(hipMemcpyAsync(d->h_flags, wk.flags, 64, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        d->stats.repairs++;
    }
    const uint32_t fl = d->h_flags[0];
    *total = (uint64_t)d->h_flags[2] | ((uint64_t)d->h_flags[3] << 32);
    *leave = d->h_flags[14];
    *cst_pro = d->h_flags[12];
    *cst_seg = d->h_flags[13];
    *entry = d->h_flags[15];
    if (emit_from >= nt) *total = 0;
    float ms[3] = {0, 0, 0};
    hipEventElapsedTime(&ms[0], d->ev[0], d->ev[1]);
    hipEventElapsedTime(&ms[1], d->ev[1], d->ev[2]);
    hipEventElapsedTime(&ms[2], d->ev[2], d->ev[3]);
    d->stats.ms_sync = ms[0];
    d->stats.ms_scan = ms[1];
    d->stats.ms_emit = ms[2];
    d->stats.ms_total = ms[0] + ms[1] + ms[2];
    d->stats.lanes = nt * HH_NR;
    d->stats.out_len = *total;
    if (fl & F_FAIL) return HH_NOSYNC;
    if (*total > cap || (fl & F_OVER)) return HH_ERR_CAPACITY;
    return HH_OK;
}

// The segment path (above).  Memory: 8 bytes per (segment, offset) and 16
// per segment; the maps are composed on the host.
static int segment_path(hh_decoder *d, const void *d_data, uint64_t bits, uint8_t *d_out, uint64_t cap,
                        uint64_t *out_len, hipStream_t st) {
    const uint32_t maxadv = d->ht->maxlen > HH_P ? (uint32_t)d->ht->maxlen : HH_P;
    const uint32_t no = (uint32_t)d->ht->maxlen;        // boundary offsets past a segment start
    const uint32_t seglen = 1u << 16;
    const uint64_t nseg64 = (bits + seglen - 1) / seglen;
    if (nseg64 > 0xffffffffull / no) return HH_ERR_UNSUPPORTED;
    const uint32_t nseg = (uint32_t)nseg64;
    const size_t nmap = (size_t)nseg * no;
    uint32_t *dm = nullptr;
    uint64_t *dbase = nullptr;
    uint32_t *hx = (uint32_t *)malloc(nmap * 8), *hent = (uint32_t *)malloc((size_t)nseg * 8);
    uint64_t *hbase = (uint64_t *)malloc((size_t)nseg * 8);
    int rc = HH_OK;
    if (!hx || !hent || !hbase) { rc = HH_ERR_NOMEM; goto out; }
    if (hipMalloc(&dm, nmap * 8 + (size_t)nseg * 8) != hipSuccess || hipMalloc(&dbase, (size_t)nseg * 8) != hipSuccess) {
        rc = HH_ERR_NOMEM;
        goto out;
    }
    {
        uint32_t *dexit = dm, *dcnt = dm + nmap;
        const uint64_t nl = nmap;
        hipLaunchKernelGGL(k_seg_func, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, st,
                           (const uint32_t *)d_data, bits, seglen, nseg, no, d->tab, maxadv, dexit, dcnt);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(hx, dm, nmap * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) { rc = HH_ERR_DEVICE; goto out; }
        const uint32_t *hexit = hx, *hcnt = hx + nmap;
        uint32_t o = 0;
        uint64_t run = 0;
        for (uint32_t sg = 0; sg < nseg; sg++) {
            if (o >= no) { rc = HH_ERR_INTERNAL; goto out; }
            hent[sg] = o;
            hent[nseg + sg] = hexit[(size_t)sg * no + o];
            hbase[sg] = run;
            run += hcnt[(size_t)sg * no + o];
            o = hent[nseg + sg];
        }
        *out_len = run;
        if (run > cap) { rc = HH_ERR_CAPACITY; goto out; }
        uint32_t *dent = dm;                            // (the maps are no longer needed)
        if (hipMemcpyAsync(dent, hent, (size_t)nseg * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(dbase, hbase, (size_t)nseg * 8, hipMemcpyHostToDevice, st) != hipSuccess) {
            rc = HH_ERR_DEVICE;
            goto out;
        }
        hipLaunchKernelGGL(k_seg_emit, dim3((nseg + 255) / 256), dim3(256), 0, st, (const uint32_t *)d_data,
                           bits, seglen, nseg, d->tab, maxadv, dent, dent + nseg, dbase, d_out);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) rc = HH_ERR_DEVICE;
    }
out:
    if (dm) hipFree(dm);
    if (dbase) hipFree(dbase);
    free(hx);
    free(hent);
    free(hbase);
    return rc;
}

// A complete fixed-length code: k_fixed (above).
// (ev: the events of the launch; wait = false: returns once enqueued)
static int fixed_path(hh_decoder *d, const void *d_data, uint64_t bits, uint8_t *d_out, uint64_t cap,
                      uint64_t *out_len, hipStream_t st, hipEvent_t *ev = nullptr, bool wait = true) {
    if (!ev) ev = d->ev;
    const uint32_t L = d->fixed_len;
    const uint64_t nsym = bits / L + (bits % L ? 1 : 0);
    *out_len = nsym;
    d->stats.out_len = nsym;
    d->stats.fixed_length = 1;
    if (nsym > cap) return HH_ERR_CAPACITY;
    const uint64_t nthr = (nsym + 15) / 16, cap_blk = (uint64_t)(d->ncu ? d->ncu : 256) * 32;
    uint64_t nb = (nthr + 255) / 256;
    if (nb > cap_blk) nb = cap_blk;
    HIP_OK(hipEventRecord(ev[0], st));
    hipLaunchKernelGGL(k_fixed, dim3((unsigned)nb), dim3(256), 0, st, (const uint32_t *)d_data, bits, L,
                       (const uint8_t *)d->d_fsym, d->tab, d_out, nsym);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[3], st));
    if (!wait) return HH_OK;
    HIP_OK(hipEventSynchronize(ev[3]));
    float ms = 0;
    hipEventElapsedTime(&ms, ev[0], ev[3]);
    d->stats.ms_emit = ms;
    d->stats.ms_total = ms;
    return HH_OK;
}

// The state-machine path (hh_fsm.hip) decodes whenever its tables exist
// (trees of at most HH_FSM_MAXS internal nodes) and no other path is forced.
static bool fsm_path_ok(const hh_decoder *d) {
    return d->fsm.ok && !(d->cfg.flags & (HH_FLAG_LEGACY | HH_FLAG_FORCE_EXACT | HH_FLAG_FORCE_SEGMENT));
}
// ms: count, scan, emission (HH_FLAG_PHASE_TIMING; else 0), total
static void fsm_stats(hh_decoder *d, uint64_t bits, uint64_t total, const float *ms, uint32_t one) {
    d->stats.ms_sync = ms[0];
    d->stats.ms_scan = ms[1];
    d->stats.ms_emit = ms[2];
    d->stats.ms_total = ms[3];
    d->stats.lanes = (bits + d->S - 1) / d->S;
    d->stats.out_len = total;
    d->stats.state_machine = one ? 2 : 1;
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
    async_check(d);                     // (an asynchronous decode before it: its status is kept for hh_decode_wait)
    memset(&d->stats, 0, sizeof(d->stats));
    *out_len = 0;
    if (bits == 0) return HH_OK;
    if (d->fixed_len && !(d->cfg.flags & (HH_FLAG_NO_FIXED | HH_FLAG_FORCE_EXACT | HH_FLAG_FORCE_SEGMENT)))
        return fixed_path(d, d_data, bits, (uint8_t *)d_out, cap, out_len, st);
    const bool seg_ok = d->ht->maxlen <= HH_MAXLEN_FAST && !(d->cfg.flags & HH_FLAG_FORCE_EXACT);
    if (fsm_path_ok(d)) {
        uint64_t total = 0;
        uint32_t leave = 0, en = 0;
        float ms[4] = {0, 0, 0, 0};
        const int rc = fsm_decode(&d->fsm, &d->fsm_ws, d->h_flags, d->ev, d_data, bits, 0, 0, 0, d_out, cap, st,
                                  &total, &leave, &en, ms);
        fsm_stats(d, bits, total, ms, d->fsm_ws.last_one);
        if (rc == HH_NOSYNC) {
            // chains that did not meet within HH_FSM_KM regions: a code that
            // does not resynchronise
            d->stats.repairs = 1;
            if (seg_ok) {
                d->stats.exact_fallback = 2;
                return segment_path(d, d_data, bits, (uint8_t *)d_out, cap, out_len, st);
            }
            d->stats.exact_fallback = 1;
            return stage_pipeline(d, d_data, (int64_t)bits, (uint8_t *)d_out, cap, out_len, st);
        }
        *out_len = total;
        return rc;
    }
    if (!fast_path_ok(d) || (d->cfg.flags & HH_FLAG_FORCE_SEGMENT)) {
        if (seg_ok) {
            d->stats.exact_fallback = 2;
            return segment_path(d, d_data, bits, (uint8_t *)d_out, cap, out_len, st);
        }
        d->stats.exact_fallback = 1;
        return stage_pipeline(d, d_data, (int64_t)bits, (uint8_t *)d_out, cap, out_len, st);
    }
    uint64_t total = 0;
    uint32_t leave = 0, cp = 0, cs = 0, en = 0;
    int rc = decode_fast(d, d_data, bits, 0, hh_state_pack(0, 0, 0), 0, d_out, cap, st, &total,
                         &leave, &cp, &cs, &en);
    if (rc == HH_NOSYNC) {
        // A walk found no shared boundary within HH_KM regions (a code that
        // does not resynchronise): the segment path, exact and O(N).
        d->stats.exact_fallback = 2;
        d->stats.repairs = 1;
        return segment_path(d, d_data, bits, (uint8_t *)d_out, cap, out_len, st);
    }
    *out_len = total;
    return rc;
}

// ---------------------------------------------------------------------------
// Asynchronous decodes (hh_decode_device_async / hh_decode_wait): a decode is
// enqueued and the PREVIOUS one checked, so that the GPU has the next decode
// queued while the host reads the last one's results (from its own result
// slot and event set: the two alternate).
// ---------------------------------------------------------------------------
static hipEvent_t *slot_ev(hh_decoder *d, uint32_t slot) { return slot ? d->ev2 : d->ev; }

// Check the pending asynchronous decode: its length to *out_len, its status
// kept in async_rc (the first failure).  A stream that did not resynchronise
// is decoded again here, on the exact path, as hh_decode_device would.
static int async_check(hh_decoder *d) {
    if (!d->apend.active) return HH_OK;
    d->apend.active = 0;
    hipEvent_t *ev = slot_ev(d, d->apend.pd.slot);
    int rc;
    memset(&d->stats, 0, sizeof(d->stats));
    if (d->apend.fixed) {
        rc = hipEventSynchronize(ev[3]) == hipSuccess ? HH_OK : HH_ERR_DEVICE;
        float ms = 0;
        hipEventElapsedTime(&ms, ev[0], ev[3]);
        d->stats.ms_emit = d->stats.ms_total = ms;
        d->stats.fixed_length = 1;
        d->stats.out_len = *d->apend.out_len;
    } else {
        uint64_t total = 0;
        uint32_t leave = 0, en = 0;
        float ms[4] = {0, 0, 0, 0};
        rc = fsm_collect(&d->fsm_ws, ev, &d->apend.pd, &total, &leave, &en, ms);
        uint32_t one = d->apend.pd.one;
        if (rc == HH_ONE_RETRY) {
            // the single pass handed the decode back: the two passes decode
            // it again, synchronously, on the decode's stream
            FsmPend p2;
            memset(&p2, 0, sizeof(p2));
            rc = fsm_launch(&d->fsm, &d->fsm_ws, d->apend.pd.slot, ev, d->apend.d_data, d->apend.bits,
                            d->apend.pd.nt_arg, d->apend.pd.in_state, d->apend.pd.emit_from, d->apend.d_out,
                            d->apend.pd.cap, d->apend.st, &p2, true);
            if (rc == HH_OK) rc = fsm_collect(&d->fsm_ws, ev, &p2, &total, &leave, &en, ms);
            one = 0;
        }
        fsm_stats(d, d->apend.bits, total, ms, one);
        *d->apend.out_len = total;
        if (d->apend.ro) {
            // a segment: its states; one that does not resynchronise is
            // unsupported (decode such a code whole), as the synchronous call
            d->apend.ro->leave_state = leave;
            d->apend.ro->entry_state = en;
            if (rc == HH_NOSYNC) rc = HH_ERR_UNSUPPORTED;
        } else if (rc == HH_NOSYNC) {
            d->stats.repairs = 1;
            const bool seg_ok = d->ht->maxlen <= HH_MAXLEN_FAST && !(d->cfg.flags & HH_FLAG_FORCE_EXACT);
            d->stats.exact_fallback = seg_ok ? 2 : 1;
            rc = seg_ok ? segment_path(d, d->apend.d_data, d->apend.bits, (uint8_t *)d->apend.d_out, d->apend.pd.cap,
                                       d->apend.out_len, d->apend.st)
                        : stage_pipeline(d, d->apend.d_data, (int64_t)d->apend.bits, (uint8_t *)d->apend.d_out,
                                         d->apend.pd.cap, d->apend.out_len, d->apend.st);
        }
    }
    if (rc != HH_OK && d->async_rc == HH_OK) d->async_rc = rc;
    return rc;
}

extern "C" int hh_decode_device_async(hh_decoder *d, const void *d_data, uint64_t bits, void *d_out,
                                      uint64_t cap, uint64_t *out_len, void *hip_stream) {
    if (!d || !out_len || (!d_data && bits) || (!d_out && cap)) return HH_ERR_ARG;
    if (!d->have_tree) return HH_ERR_ARG;
    if (((uintptr_t)d_data & 3u) != 0) return HH_ERR_ARG;
    hipStream_t st = (hipStream_t)hip_stream;
    HIP_OK(hipSetDevice(d->device));
    *out_len = 0;
    const bool fixed = d->fixed_len && !(d->cfg.flags & (HH_FLAG_NO_FIXED | HH_FLAG_FORCE_EXACT | HH_FLAG_FORCE_SEGMENT));
    if (bits == 0 || !(fixed || fsm_path_ok(d))) {
        // the other paths decode synchronously (the pending decode first)
        async_check(d);
        const int rc = hh_decode_device(d, d_data, bits, d_out, cap, out_len, hip_stream);
        if (rc != HH_OK && d->async_rc == HH_OK) d->async_rc = rc;
        return HH_OK;
    }
    // the previous decode's slot and events stay untouched until it is checked
    const uint32_t slot = d->apend.active ? (d->apend.pd.slot ^ 1u) : 0u;
    FsmPend pd;
    memset(&pd, 0, sizeof(pd));
    pd.slot = slot;
    int rc;
    if (fixed) {
        uint64_t n = 0;
        rc = fixed_path(d, d_data, bits, (uint8_t *)d_out, cap, &n, st, slot_ev(d, slot), false);
        *out_len = n;
    } else {
        // The state-machine workspace (records, tile sums, corrections) is
        // one per decoder: a decode queued on another stream than the
        // pending one waits for that one's last kernel before its count pass
        // may overwrite what the pending emission still reads.  (On one
        // stream the order is the stream's.)
        if (d->apend.active && !d->apend.fixed && d->apend.st != st)
            HIP_OK(hipStreamWaitEvent(st, slot_ev(d, d->apend.pd.slot)[3], 0));
        rc = fsm_launch(&d->fsm, &d->fsm_ws, slot, slot_ev(d, slot), d_data, bits, 0, 0, 0, d_out, cap, st, &pd);
    }
    async_check(d);                     // the previous decode, while this one runs
    if (rc != HH_OK) {
        if (d->async_rc == HH_OK) d->async_rc = rc;
        return rc == HH_ERR_CAPACITY ? HH_OK : rc;   // (a capacity failure is reported by hh_decode_wait)
    }
    d->apend.active = 1;
    d->apend.fixed = fixed;
    d->apend.pd = pd;
    d->apend.d_data = d_data;
    d->apend.bits = bits;
    d->apend.d_out = d_out;
    d->apend.out_len = out_len;
    d->apend.st = st;
    d->apend.ro = nullptr;
    d->async_seq++;
    return HH_OK;
}

extern "C" int hh_decode_wait(hh_decoder *d) {
    if (!d) return HH_ERR_ARG;
    HIP_OK(hipSetDevice(d->device));
    async_check(d);
    const int rc = d->async_rc;
    d->async_rc = HH_OK;
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
    async_check(d);
    memset(&d->stats, 0, sizeof(d->stats));
    memset(ro, 0, sizeof(*ro));
    ro->leave_state = ro->entry_state = rg->in_state;
    // no tiles (a shard with none of its own when there are fewer tiles than
    // ranks): nothing written, the chain leaves in the state it entered
    ro->entry_exact = rg->prologue == 0;
    if (rg->bits_avail == 0 || rg->ntiles == 0) return HH_OK;
    if (fsm_path_ok(d)) {
        // states are state-machine states (0: the root, the stream start)
        if (rg->in_state >= d->fsm.ns) return HH_ERR_ARG;
        float ms[4] = {0, 0, 0, 0};
        const int rc = fsm_decode(&d->fsm, &d->fsm_ws, d->h_flags, d->ev, d_data, rg->bits_avail, rg->ntiles,
                                  rg->in_state, rg->prologue, d_out, cap, st, &ro->out_len, &ro->leave_state,
                                  &ro->entry_state, ms);
        fsm_stats(d, rg->bits_avail, ro->out_len, ms, d->fsm_ws.last_one);
        if (rc == HH_NOSYNC) return HH_ERR_UNSUPPORTED;   // (decode such a code whole)
        // the state leaving a segment does not depend on how it was entered
        // once the chain from its entry has met an entry-independent one
        // (a head's).  The count pass proves that meeting only through a
        // tile's lane-63 walk into its successor (a chain that does not meet
        // there fails the decode), so only a segment of two or more count
        // tiles has a leave state proven independent of its entry (the count
        // pass's tiles: fsm.cm emission tiles each); a one-tile segment's is
        // valid only when its entry is.  The entry after a prologue is
        // checked against the predecessor's leave state by the caller.
        ro->const_seen = rg->ntiles > (uint64_t)d->fsm.cm;
        ro->entry_exact = rg->prologue == 0;
        return rc;
    }
    // segments need the fast path (tile tables, entry states); a tree it
    // does not support is decoded whole, unsharded
    if (!fast_path_ok(d) || hh_state_d(rg->in_state) >= HH_KM) return HH_ERR_UNSUPPORTED;
    uint32_t cp = 0;
    const int rc = decode_fast(d, d_data, rg->bits_avail, rg->ntiles, rg->in_state, rg->prologue,
                               d_out, cap, st, &ro->out_len, &ro->leave_state, &cp,
                               &ro->const_seen, &ro->entry_state);
    ro->entry_exact = rg->prologue == 0 || cp != 0;
    return rc == HH_NOSYNC ? HH_ERR_UNSUPPORTED : rc;
}

// The asynchronous form (multi-GPU shards: a stream of segment decodes with
// no host wait between them).  ro is filled when the decode is checked: by
// the next asynchronous decode on this decoder or by hh_decode_wait.
extern "C" int hh_decode_device_range_async(hh_decoder *d, const void *d_data, const hh_range *rg,
                                            void *d_out, uint64_t cap, hh_range_out *ro,
                                            void *hip_stream) {
    if (!d || !rg || !ro || (!d_data && rg->bits_avail) || (!d_out && cap)) return HH_ERR_ARG;
    if (!d->have_tree) return HH_ERR_ARG;
    if (((uintptr_t)d_data & 3u) != 0) return HH_ERR_ARG;
    if (!fsm_path_ok(d) || rg->bits_avail == 0 || rg->ntiles == 0) {
        // (other paths, and empty segments: synchronously, as hh_decode_device_range)
        async_check(d);
        const int rc = hh_decode_device_range(d, d_data, rg, d_out, cap, ro, hip_stream);
        if (rc != HH_OK && d->async_rc == HH_OK) d->async_rc = rc;
        return rc == HH_ERR_CAPACITY ? HH_OK : rc;
    }
    if (rg->in_state >= d->fsm.ns) return HH_ERR_ARG;
    hipStream_t st = (hipStream_t)hip_stream;
    HIP_OK(hipSetDevice(d->device));
    memset(ro, 0, sizeof(*ro));
    ro->leave_state = ro->entry_state = rg->in_state;
    // (known at launch: see hh_decode_device_range)
    ro->const_seen = rg->ntiles > (uint64_t)d->fsm.cm;
    ro->entry_exact = rg->prologue == 0;
    const uint32_t slot = d->apend.active ? (d->apend.pd.slot ^ 1u) : 0u;
    FsmPend pd;
    memset(&pd, 0, sizeof(pd));
    if (d->apend.active && !d->apend.fixed && d->apend.st != st)
        HIP_OK(hipStreamWaitEvent(st, slot_ev(d, d->apend.pd.slot)[3], 0));
    const int rc = fsm_launch(&d->fsm, &d->fsm_ws, slot, slot_ev(d, slot), d_data, rg->bits_avail, rg->ntiles,
                              rg->in_state, rg->prologue, d_out, cap, st, &pd);
    async_check(d);                     // the previous decode, while this one runs
    if (rc != HH_OK) {
        if (d->async_rc == HH_OK) d->async_rc = rc;
        return rc;
    }
    d->apend.active = 1;
    d->apend.fixed = 0;
    d->apend.pd = pd;
    d->apend.d_data = d_data;
    d->apend.bits = rg->bits_avail;
    d->apend.d_out = d_out;
    d->apend.out_len = &ro->out_len;
    d->apend.st = st;
    d->apend.ro = ro;
    d->async_seq++;
    return HH_OK;
}

// evaluate() scope (decodeUtil.c:41-43 times the whole decoder call): host
// payload in, host symbols out.  Copies go through two pinned chunk buffers
// the decoder keeps (HH_HOST_CHUNK each): the CPU copy of one chunk into (or
// out of) pinned memory overlaps the DMA of the other, both ways.  Device
// buffers are kept too: no allocation after the first call of a size.
#define HH_HOST_CHUNK ((size_t)64 << 20)
#define HH_HOST_THREADS 8                  // CPU copies into / out of pinned memory

// The CPU side of a chunk: a single core copies ~10 GB/s, below PCIe's
// rate, so the chunk is split over a few threads.
static void par_memcpy(uint8_t *dst, const uint8_t *src, size_t len) {
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t nt = std::min<size_t>(hw ? std::min<unsigned>(hw, HH_HOST_THREADS) : 1, len >> 20);
    if (nt <= 1) {
        memcpy(dst, src, len);
        return;
    }
    std::thread th[HH_HOST_THREADS];
    const size_t part = (len / nt + 4095) & ~(size_t)4095;
    for (size_t i = 1; i < nt; i++) {
        const size_t o = i * part;
        if (o >= len) continue;
        try {
            th[i] = std::thread(memcpy, dst + o, src + o, std::min(part, len - o));
        } catch (...) {   // (no thread to be had: this part on the calling thread)
            memcpy(dst + o, src + o, std::min(part, len - o));
        }
    }
    memcpy(dst, src, std::min(part, len));
    for (size_t i = 1; i < nt; i++)
        if (th[i].joinable()) th[i].join();
}

static int host_pipe(hh_decoder *d, uint8_t *host, uint8_t *dev, size_t n, bool h2d) {
    if (!n) return HH_OK;
    const size_t nch = (n + HH_HOST_CHUNK - 1) / HH_HOST_CHUNK;
    for (size_t i = 0; i < nch + 1; i++) {
        // DMA chunk i (h2d: after the CPU has staged it; d2h: into its buffer)
        if (i < nch) {
            const size_t off = i * HH_HOST_CHUNK, len = n - off < HH_HOST_CHUNK ? n - off : HH_HOST_CHUNK;
            uint8_t *pin = d->h_stage + (i & 1) * HH_HOST_CHUNK;
            if (i >= 2) HIP_OK(hipEventSynchronize(d->h_ev[i & 1]));   // buffer free again
            if (h2d) {
                par_memcpy(pin, host + off, len);
                HIP_OK(hipMemcpyAsync(dev + off, pin, len, hipMemcpyHostToDevice, d->stream));
            } else {
                HIP_OK(hipMemcpyAsync(pin, dev + off, len, hipMemcpyDeviceToHost, d->stream));
            }
            HIP_OK(hipEventRecord(d->h_ev[i & 1], d->stream));
        }
        // d2h: the CPU drains chunk i-1 while chunk i is in flight
        if (!h2d && i >= 1) {
            const size_t k = i - 1, off = k * HH_HOST_CHUNK;
            const size_t len = n - off < HH_HOST_CHUNK ? n - off : HH_HOST_CHUNK;
            HIP_OK(hipEventSynchronize(d->h_ev[k & 1]));
            par_memcpy(host + off, d->h_stage + (k & 1) * HH_HOST_CHUNK, len);
        }
    }
    return HH_OK;
}

// The evaluate() scope, pipelined (state-machine path): the caller's buffers
// are page-locked for the call (hipHostRegister) so that the DMA engines read
// and write them directly; the payload goes up in chunks of whole tiles on
// one copy stream, chunk k is decoded as a segment as soon as it has landed
// (entered in the state chunk k-1 left), and its symbols go down on a second
// copy stream while later chunks are still uploading and decoding.
#define HH_PIPE_CHUNK ((uint64_t)128 << 20)          // payload bytes per chunk

static uint64_t pipe_chunk() {
    const char *e = getenv("HH_PIPE_CHUNK_KB");        // (tests: force many chunks)
    const uint64_t v = e ? strtoull(e, nullptr, 10) << 10 : 0;
    return v ? v : HH_PIPE_CHUNK;
}

// HH_FLAG_KEEP_HOST_PINNED: buffer k (0 payload, 1 output) page-locked
// from p for at least n bytes, the registration kept for later calls
// from p for at least n bytes, the registration kept for later calls.
// Registrations are whole pages and may not overlap: a buffer whose pages
// lie inside the other buffer's registration is recorded as covered by it
// (pin_own 0), one that overlaps it partly gets a registration of the union
// of both (the other then covered by it); when a registration goes, the
// buffer it covered is pinned again.
static bool pin_inside(const hh_decoder *d, int k, uintptr_t a, uintptr_t b) {
    return d->pin_p[k] && d->pin_own[k] && a >= d->pin_ra[k] && b <= d->pin_rb[k];
}
static void pin_drop(hh_decoder *d, int k) {
    if (d->pin_p[k] && d->pin_own[k]) (void)hipHostUnregister((void *)d->pin_ra[k]);
    d->pin_p[k] = nullptr;
    d->pin_n[k] = 0;
    d->pin_own[k] = 0;
    d->pin_ra[k] = d->pin_rb[k] = 0;
}
static int pin_host(hh_decoder *d, int k, const void *p, size_t n) {
    uintptr_t a = (uintptr_t)p & ~(uintptr_t)4095, b = ((uintptr_t)p + n + 4095) & ~(uintptr_t)4095;
    if (d->pin_p[k] == p && d->pin_n[k] >= n && (d->pin_own[k] || pin_inside(d, k ^ 1, a, b))) return HH_OK;
    const int o = k ^ 1;
    const void *op = d->pin_p[o];
    const size_t on = d->pin_n[o];
    bool repin = op && !d->pin_own[o];               // (o relied on k's registration)
    pin_drop(d, k);
    if (pin_inside(d, o, a, b)) {                     // (within the other buffer's pages)
        d->pin_p[k] = p;
        d->pin_n[k] = n;
        return HH_OK;
    }
    if (op && d->pin_own[o] && a < d->pin_rb[o] && d->pin_ra[o] < b) {
        // a partial overlap: one registration of both
        a = std::min(a, d->pin_ra[o]);
        b = std::max(b, d->pin_rb[o]);
        pin_drop(d, o);
        repin = true;
    }
    if (hipHostRegister((void *)a, b - a, hipHostRegisterDefault) != hipSuccess) return HH_ERR_UNSUPPORTED;
    d->pin_p[k] = p;
    d->pin_n[k] = n;
    d->pin_own[k] = 1;
    d->pin_ra[k] = a;
    d->pin_rb[k] = b;
    return repin ? pin_host(d, o, op, on) : HH_OK;
}

extern "C" int hh_decoder_release_host(hh_decoder *d) {
    if (!d) return HH_ERR_ARG;
    for (int k = 0; k < 2; k++) pin_drop(d, k);
    return HH_OK;
}

static int host_pipeline(hh_decoder *d, const uint8_t *data, uint64_t bits, uint8_t *out, uint64_t cap,
                         uint64_t *out_len) {
    const uint64_t nb = (bits + 7) / 8;
    const uint64_t tbb = (uint64_t)HH_NR * d->S / 8;                 // bytes per tile
    const uint64_t ch = pipe_chunk() > tbb ? pipe_chunk() / tbb * tbb : tbb;
    const uint64_t nch = (nb + ch - 1) / ch;
    if (!d->h2d) {
        HIP_OK(hipStreamCreateWithFlags(&d->h2d, hipStreamNonBlocking));
        HIP_OK(hipStreamCreateWithFlags(&d->d2h, hipStreamNonBlocking));
    }
    if (nch > d->npipe_ev) {
        for (uint32_t i = 0; i < d->npipe_ev; i++) (void)hipEventDestroy(d->pipe_ev[i]);
        free(d->pipe_ev);
        d->npipe_ev = 0;
        d->pipe_ev = (hipEvent_t *)calloc(nch, sizeof(hipEvent_t));
        if (!d->pipe_ev) return HH_ERR_NOMEM;
        for (uint64_t i = 0; i < nch; i++) {
            HIP_OK(hipEventCreateWithFlags(&d->pipe_ev[i], hipEventDisableTiming));
            d->npipe_ev = (uint32_t)(i + 1);
        }
    }
    const bool keep = (d->cfg.flags & HH_FLAG_KEEP_HOST_PINNED) != 0;
    if (keep) {
        // the buffers stay registered across calls: (re)register only a new
        // pointer or a longer length
        if (pin_host(d, 0, data, nb) != HH_OK) return HH_ERR_UNSUPPORTED;
        if (cap && pin_host(d, 1, out, cap) != HH_OK) return HH_ERR_UNSUPPORTED;
    } else {
        if (hipHostRegister((void *)data, nb, hipHostRegisterDefault) != hipSuccess) return HH_ERR_UNSUPPORTED;
        if (cap && hipHostRegister(out, cap, hipHostRegisterDefault) != hipSuccess) {
            (void)hipHostUnregister((void *)data);
            return HH_ERR_UNSUPPORTED;
        }
    }
    int rc = HH_OK;
    uint8_t *din = (uint8_t *)d->d_in, *dout = (uint8_t *)d->d_out;
    if (hipMemsetAsync(din + nb, 0, HH_PAYLOAD_PAD, d->h2d) != hipSuccess) rc = HH_ERR_DEVICE;
    for (uint64_t k = 0; k < nch && !rc; k++) {
        const uint64_t o = k * ch, len = nb - o < ch ? nb - o : ch;
        if (hipMemcpyAsync(din + o, data + o, len, hipMemcpyHostToDevice, d->h2d) != hipSuccess ||
            hipEventRecord(d->pipe_ev[k], d->h2d) != hipSuccess)
            rc = HH_ERR_DEVICE;
    }
    uint64_t total = 0;
    uint32_t state = 0;
    bool over = false;
    float ms_all[4] = {0, 0, 0, 0};
    for (uint64_t k = 0; k < nch && !rc; k++) {
        const uint64_t b0 = k * ch * 8;
        const uint64_t ntiles = (k + 1 < nch ? ch * 8 : bits - b0 + d->S * HH_NR - 1) / (d->S * HH_NR);
        // readable bits: the chunk and the first tile of the next (the stream
        // end lies beyond a chunk's tiles, except in the last one)
        const uint64_t avail = bits - b0 < (ch + tbb) * 8 ? bits - b0 : (ch + tbb) * 8;
        if (hipStreamWaitEvent(d->stream, d->pipe_ev[k], 0) != hipSuccess) { rc = HH_ERR_DEVICE; break; }
        // (the first tile of the next chunk may not have landed yet: the
        // kernels read it only for chains that this segment does not use)
        uint64_t n = 0;
        uint32_t leave = 0, en = 0;
        float ms[4] = {0, 0, 0, 0};
        // (past a capacity failure the later chunks are only counted -- no
        // room is left, nothing is written -- so that out_len is the stream's
        // total, as hh_decode_device reports it)
        const uint64_t room = over || total >= cap ? 0 : cap - total;
        rc = fsm_decode(&d->fsm, &d->fsm_ws, d->h_flags, d->ev, din + k * ch, avail, ntiles, state, 0,
                        room ? dout + total : dout, room, d->stream, &n, &leave, &en, ms);
        if (rc == HH_ERR_CAPACITY) {
            over = true;
            rc = HH_OK;
        }
        if (rc) break;
        for (int i = 0; i < 4; i++) ms_all[i] += ms[i];
        if (!over && n && hipMemcpyAsync(out + total, dout + total, n, hipMemcpyDeviceToHost, d->d2h) != hipSuccess) {
            rc = HH_ERR_DEVICE;
            break;
        }
        total += n;
        state = leave;
    }
    if (over && !rc) rc = HH_ERR_CAPACITY;
    if (hipStreamSynchronize(d->d2h) != hipSuccess || hipStreamSynchronize(d->h2d) != hipSuccess) rc = rc ? rc : HH_ERR_DEVICE;
    if (!keep) {
        (void)hipHostUnregister((void *)data);
        if (cap) (void)hipHostUnregister(out);
    }
    fsm_stats(d, bits, total, ms_all, d->fsm_ws.last_one);
    *out_len = total;
    return rc == HH_NOSYNC ? HH_ERR_UNSUPPORTED : rc;   // (no resync: the serial path decodes it whole)
}

extern "C" int hh_decode_host(hh_decoder *d, const uint8_t *data, uint64_t bits, uint8_t *out,
                              uint64_t cap, uint64_t *out_len) {
    if (!d || !out_len || (!data && bits) || (!out && cap)) return HH_ERR_ARG;
    HIP_OK(hipSetDevice(d->device));
    async_check(d);
    *out_len = 0;
    const uint64_t nb = (bits + 7) / 8;
    const uint64_t ocap = cap ? cap : 1;
    int rc = ensure_dev(&d->d_in, &d->d_in_size, nb + HH_PAYLOAD_PAD);
    if (!rc) rc = ensure_dev(&d->d_out, &d->d_out_size, ocap);
    if (rc) return rc;
    if (!d->h_stage) {
        if (hipHostMalloc((void **)&d->h_stage, 2 * HH_HOST_CHUNK, hipHostMallocDefault) != hipSuccess) {
            d->h_stage = nullptr;
            return HH_ERR_NOMEM;
        }
        if (hipEventCreateWithFlags(&d->h_ev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&d->h_ev[1], hipEventDisableTiming) != hipSuccess)
            return HH_ERR_DEVICE;
    }
    if (fsm_path_ok(d) && nb > pipe_chunk() && !getenv("HH_HOST_SERIAL")) {
        rc = host_pipeline(d, data, bits, out, cap, out_len);
        if (rc != HH_ERR_UNSUPPORTED) return rc;   // (unsupported: registration refused -> staged copies)
        rc = HH_OK;
    }
    HIP_OK(hipMemsetAsync((uint8_t *)d->d_in + nb, 0, HH_PAYLOAD_PAD, d->stream));
    rc = host_pipe(d, (uint8_t *)data, (uint8_t *)d->d_in, nb, true);
    if (!rc) rc = hh_decode_device(d, d->d_in, bits, d->d_out, cap, out_len, d->stream);
    if (!rc) rc = host_pipe(d, out, (uint8_t *)d->d_out, *out_len, false);
    if (!rc) HIP_OK(hipStreamSynchronize(d->stream));
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
    HIP_OK(hipMemsetAsync(d->d_max, 0xff, 4, st));
    hipLaunchKernelGGL(k_st_findmax, dim3(grid_for(bits, 256)), dim3(256), 0, st, bits, idx, d->d_max);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(maxvalue, d->d_max, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
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
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipMalloc(&bitdecode, bits) != hipSuccess || hipMalloc(&result, bits) != hipSuccess ||
        hipMalloc(&steps, (size_t)25 * bits * 4) != hipSuccess ||
        hipMalloc(&idx, (size_t)bits * 4) != hipSuccess) {
        rc = HH_ERR_NOMEM;
        goto done;
    }
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
        rc = HH_ERR_DEVICE;
        goto done;
    }
    {
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
    }
done:
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
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

// Diagnostic (HH_DIAG builds; zeros otherwise): the front kernel's phase
// cycles summed over workgroups [0..3] (staging, pass 1, walks, table) and
// walk statistics [8..11] (lanes, lookups, sum over waves of the wave's
// longest walk, longest walk) of the last decode.
// (HH_WSPAN builds: 16 + 6 x 8192 words -- the per-wave start / fill / end
// stamps of k_cntm and k_emf after the 16 counters)
extern "C" int hh_debug_counters(hh_decoder *d, uint64_t *out16) {
    if (!d || !out16) return HH_ERR_ARG;
    if (hipMemcpy(out16, d->d_dbg, HH_DBG_WORDS * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return HH_ERR_DEVICE;
    return HH_OK;
}

// Diagnostic: the state-machine count pass's arrays of the last decode of
// `ntiles` tiles (records, corrections, tile sums, leaving states).
extern "C" int hh_debug_fsm(hh_decoder *d, uint64_t ntiles, uint32_t *rec, uint32_t *fx, int32_t *tsum,
                            uint32_t *xs) {
    if (!d) return HH_ERR_ARG;
    HIP_OK(hipSetDevice(d->device));
    return fsm_debug_arrays(&d->fsm_ws, ntiles, rec, fx, tsum, xs);
}
