// hh_device.hip -- HIP kernels (gfx950) and the device half of the C ABI.
//
// Fast path (O(N) memory, 64-bit offsets), three launches:
//   k_sync  one workgroup per tile of HH_NL lane regions: tables and the
//           tile's bits (+ halo) staged in LDS; every lane decodes its region
//           from offset 0 (decodeallbits) and walks its exit against the next
//           region's chain until they share a boundary (makebigtable); the
//           tile resolves which lanes are live for each entering state and
//           writes an HH_KM-entry transfer table.
//   k_scan  composes the tile tables in order -> entering state and output
//           base of every tile (calcbitsindex / findmax).
//   k_emit  re-decodes every live run and writes its symbols through an LDS
//           staging window with 16-byte coalesced stores (calcresult).
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
#define HH_CAP (32 * 1024)        // emission staging window (bytes)
#define HH_SCAN_T 256             // threads of the tile-scan workgroup
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
__device__ __forceinline__ void stage_tables(uint64_t *s_l1, uint32_t *s_l2, const DevTab &tab) {
    for (uint32_t i = threadIdx.x; i < HH_L1_SIZE; i += blockDim.x) s_l1[i] = tab.l1[i];
    for (uint32_t i = threadIdx.x; i < tab.l2_used; i += blockDim.x) s_l2[i] = tab.l2[i];
}

// Tile words [w0, w0+nw) of the payload; words past nwords_ok read as 0.
__device__ __forceinline__ void stage_words(uint32_t *s_w, const uint32_t *g, uint64_t w0,
                                            uint32_t nw, uint64_t nwords_ok) {
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) {
        uint64_t gi = w0 + i;
        s_w[i] = gi < nwords_ok ? __builtin_nontemporal_load(&g[gi]) : 0u;
    }
}

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

struct TileGeom {
    uint64_t b0;       // first stream bit of the tile
    uint32_t nw;       // staged words
    uint32_t bt;       // stream end relative to the tile, clamped to the span
};

__device__ __forceinline__ TileGeom tile_geom(uint64_t tile, uint32_t S, uint64_t bits) {
    TileGeom g;
    g.b0 = tile * (uint64_t)HH_NL * S;
    uint32_t span = (HH_NL + HH_KM + 1) * S + HH_SPAN_MARGIN;
    g.nw = (span + 31) / 32 + 3;
    uint64_t rem = bits - g.b0;
    g.bt = rem < span ? (uint32_t)rem : span;
    return g;
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
    uint64_t *gran;      // [ntiles] tagged: table published + outgoing state if constant
    uint64_t *cnt;       // [ntiles] tagged: 1 = aggregate count, 2 = inclusive prefix
    uint64_t *tabs;      // [ntiles][HH_KM] tile tables (sc1 stores)
    uint32_t *counter;   // tile dispenser
};

// 64-bit granules: the data is the flag (bits 62..63 = status, 0 = not yet).
#define HH_ST_SHIFT 62
#define HH_VAL_MASK ((1ull << HH_ST_SHIFT) - 1ull)
#define HH_GR_CONST (1ull << 32)

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

enum { F_TIMEOUT = 8 };

// Diagnostic build only (-DHH_STAMPS): wave 0 of every workgroup adds the
// shader-clock cycles of each phase into dbg[block][phase].
#ifdef HH_STAMPS
#define HH_NSTAMP 8
#define STAMP_DECL uint64_t st_acc[HH_NSTAMP] = {0, 0, 0, 0, 0, 0, 0, 0}; uint64_t st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { uint64_t t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } while (0)
#define STAMP_FLUSH(dbg) do { if (threadIdx.x == 0) for (int i_ = 0; i_ < HH_NSTAMP; i_++) (dbg)[blockIdx.x * HH_NSTAMP + i_] = st_acc[i_]; } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH(dbg) do {} while (0)
#endif
#define HH_SPIN_LIMIT (1u << 22)

__device__ __forceinline__ uint64_t state_pack(const hh_state &s) {
    return (uint64_t)s.d | ((uint64_t)s.e << 8) | ((uint64_t)(uint32_t)s.delta << 32);
}
__device__ __forceinline__ hh_state state_unpack(uint64_t p, uint64_t base) {
    hh_state s;
    s.d = (uint32_t)(p & 0xff);
    s.e = (uint32_t)((p >> 8) & 0xffffff);
    s.delta = (int32_t)(uint32_t)(p >> 32);
    s.base = base;
    return s;
}

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

__device__ __forceinline__ void stage_tile_words(uint32_t *s_w, const uint32_t *g, uint64_t w0,
                                                 uint32_t nw, uint64_t nwords_ok) {
    constexpr uint32_t PER = (HH_NW_MAX + HH_NL - 1) / HH_NL;
    uint32_t v[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        uint32_t i = threadIdx.x + k * HH_NL;
        uint64_t gi = w0 + i;
        v[k] = (i < nw && gi < nwords_ok) ? __builtin_nontemporal_load(&g[gi]) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        uint32_t i = threadIdx.x + k * HH_NL;
        if (i < nw) s_w[i] = v[k];
    }
}

// Decode the run [p, pe) for output indices [o, we) into stage[idx - org]:
// whole dwords by ds_write_b32, the partial first / last dword by bytes (the
// neighbouring run owns its other bytes).
__device__ __forceinline__ void emit_run_lds(const hh_ctx *c, uint32_t &p, uint32_t pe, uint64_t &o,
                                             uint64_t we, uint8_t *stage, uint64_t org) {
    uint32_t q = (uint32_t)(o - org);
    while ((q & 3u) && p < pe && o < we) {
        uint32_t s;
        p += hh_dec1(c, p, &s);
        stage[q++] = (uint8_t)s;
        o++;
    }
    uint32_t *st32 = (uint32_t *)stage;
    uint64_t acc = 0;
    uint32_t nacc = 0;
    while (p < pe && o < we) {
        uint32_t win = hh_read32(c, p);
        uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
        uint32_t ns = HH_L1_NSYM(e), val, n, adv;
        if (ns && p + HH_L1_NBITS(e) <= pe && o + ns <= we) {
            val = HH_L1_SYMS(e);
            n = ns;
            adv = HH_L1_NBITS(e);
        } else {
            uint32_t s;
            adv = hh_dec1(c, p, &s);
            val = s;
            n = 1;
        }
        acc |= (uint64_t)val << (8u * nacc);
        nacc += n;
        o += n;
        p += adv;
        if (nacc >= 4) {
            st32[q >> 2] = (uint32_t)acc;
            acc >>= 32;
            nacc -= 4;
            q += 4;
        }
    }
    for (uint32_t i = 0; i < nacc; i++) stage[q + i] = (uint8_t)(acc >> (8 * i));
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

// Emit the run [p, pe) to global memory at dst: dword stores, bytes for the
// partial first / last dword (the neighbouring runs own their other bytes).
__device__ __forceinline__ void emit_run_global(const hh_ctx *c, uint32_t p, uint32_t pe, uint8_t *dst) {
    uintptr_t a = (uintptr_t)dst;
    while ((a & 3u) && p < pe) {
        uint32_t s;
        p += hh_dec1(c, p, &s);
        *(uint8_t *)a = (uint8_t)s;
        a++;
    }
    uint64_t acc = 0;
    uint32_t nacc = 0;
    while (p < pe) {
        uint32_t win = hh_read32(c, p);
        uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
        uint32_t ns = HH_L1_NSYM(e), val, n, adv;
        if (ns && p + HH_L1_NBITS(e) <= pe) {
            val = HH_L1_SYMS(e);
            n = ns;
            adv = HH_L1_NBITS(e);
        } else {
            uint32_t s;
            adv = hh_dec1(c, p, &s);
            val = s;
            n = 1;
        }
        acc |= (uint64_t)val << (8u * nacc);
        nacc += n;
        p += adv;
        if (nacc >= 4) {
            *(uint32_t *)a = (uint32_t)acc;
            a += 4;
            acc >>= 32;
            nacc -= 4;
        }
    }
    for (uint32_t i = 0; i < nacc; i++) *(uint8_t *)(a + i) = (uint8_t)(acc >> (8 * i));
}

// Regions per tile: the last lane decodes the NEXT tile's first region too
// (its mask lets the tile's last walk merge without a two-pointer walk).
#define HH_NR (HH_NL - 1)

__global__ __launch_bounds__(HH_NL) void k_decode(const uint32_t *__restrict__ gdata, uint64_t bits,
                                                  uint64_t nwords_ok, uint32_t S, DevTab tab,
                                                  uint64_t ntiles, LookBack lb,
                                                  uint8_t *__restrict__ out, uint64_t cap,
                                                  uint32_t *flags, uint32_t diag_stop,
                                                  uint64_t *dbg) {
    __shared__ uint64_t s_l1[HH_L1_SIZE];
    __shared__ uint32_t s_w[HH_NW_MAX];
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
    __shared__ uint64_t s_state[2];
    __shared__ uint32_t s_tile;
    extern __shared__ uint32_t s_l2[];

    const uint32_t lane = threadIdx.x;
    const uint32_t mw = (S + 31) / 32;
    stage_l1<HH_L1_SIZE>(s_l1, tab.l1);
    for (uint32_t i = lane; i < tab.l2_used; i += HH_NL) s_l2[i] = tab.l2[i];
    STAMP_DECL

    for (;;) {
        if (lane == 0) s_tile = atomicAdd(lb.counter, 1u);
        __syncthreads();                       // also fences LDS reuse
        const uint64_t tile = s_tile;
        if (tile >= ntiles) break;
        STAMP(0);
        TileGeom g;
        g.b0 = tile * (uint64_t)HH_NR * S;
        {
            const uint32_t span = (HH_NL + HH_KM + 1) * S + HH_SPAN_MARGIN;
            g.nw = (span + 31) / 32 + 3;
            const uint64_t rem = bits - g.b0;
            g.bt = rem < span ? (uint32_t)rem : span;
        }
        stage_tile_words(s_w, gdata, g.b0 >> 5, g.nw, nwords_ok);
        __syncthreads();
        STAMP(1);

        hh_ctx c;
        c.w = s_w; c.sh = (uint32_t)(g.b0 & 31); c.l1 = s_l1; c.l2 = s_l2;
        c.tree = tab.tree; c.tsym = tab.tsym; c.bt = g.bt;

        // (2) region decode from offset 0 (+ boundary mask), all NL lanes
        const uint32_t p0 = lane * S;
        uint32_t n = 0, x = p0;
        {
            struct MS {
                uint32_t *m;
                __device__ void operator()(uint32_t w, uint32_t v) { m[w] = v; }
            } ms{&s_mask[lane * mw]};
            if (p0 < c.bt) {
                x = hh_region_count_mask(&c, p0, p0 + S, mw, &n, ms);
            } else {
                for (uint32_t w2 = 0; w2 < mw; w2++) s_mask[lane * mw + w2] = 0;
            }
        }
        s_x[lane] = (uint16_t)(x - p0);
        s_n[lane] = (uint16_t)n;
        __syncthreads();
        STAMP(2);
        hh_rec r;
        r.n = n; r.k = 1; r.e = 0; r.delta = 0; r.cov = 0;
        if (lane < HH_NR) {
            hh_masks mk = {s_mask, s_x, s_n, HH_NL, mw};
            hh_walk_mask(&c, &mk, lane, S, x, &r);
            r.n = n;
            if (r.k == 0) atomicOr(flags, (uint32_t)F_FAIL);
        }
        const uint32_t kk = r.k ? r.k : 1u;
        STAMP(3);

        // (3) live regions for every entering d -> transfer table
        s_mem[lane] = lane >= HH_NR ? 0u : (lane >= HH_KM - 1 ? 0xffu : (uint8_t)((1u << (lane + 1)) - 1u));
        s_k[lane] = (uint8_t)kk;
        const uint32_t nexc = collect_exceptions(kk > 1 && lane < HH_NR, s_exc, s_cnt4);
        if (lane == 0) {
            for (uint32_t i = 0; i < nexc; i++) {
                uint32_t j = s_exc[i], kj = s_k[j];
                uint8_t m = s_mem[j];
                for (uint32_t q = j + 1; q < j + kj && q < HH_NR; q++) s_mem[q] &= (uint8_t)~m;
            }
        }
        __syncthreads();
        const uint32_t memd = s_mem[lane];
        const int32_t contrib = (int32_t)(r.n + r.cov) + (lane + kk < HH_NR ? r.delta : 0);
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
            int32_t cnt = s_part[0][lane] + s_part[1][lane] + s_part[2][lane] + s_part[3][lane];
            uint64_t o = s_out[lane];
            s_tab[lane] = hh_xf_pack((uint32_t)cnt, hh_xf_delta(o), hh_xf_e(o), hh_xf_d(o));
        }
        __syncthreads();
        STAMP(4);
        // (4a) publish the table (sc1) and its granule: outgoing state if
        // every entering d leads to the same one (the normal case).
        if (lane == 0) {
            uint64_t o0 = s_tab[0] >> 32;
            bool cst = true;
            for (uint32_t i = 0; i < HH_KM; i++) {
                st_sc1(&lb.tabs[tile * HH_KM + i], s_tab[i]);
                cst = cst && (s_tab[i] >> 32) == o0;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t o = s_tab[0];
            uint64_t gr = (uint64_t)hh_xf_d(o) | ((uint64_t)hh_xf_e(o) << 4) |
                          ((uint64_t)((uint32_t)hh_xf_delta(o) & 0xffffu) << 16) |
                          (cst ? HH_GR_CONST : 0ull) | (1ull << HH_ST_SHIFT);
            st_sc1(&lb.gran[tile], gr);
            // (4b) entering state from the predecessor's granule
            hh_state sin = {0, 0, 0, 0};
            if (tile > 0) {
                int64_t j = (int64_t)tile - 1;
                uint64_t gj = poll_granule(&lb.gran[j], flags);
                while (!(gj & HH_GR_CONST) && j > 0) {      // rare: walk back
                    j--;
                    gj = poll_granule(&lb.gran[j], flags);
                }
                int64_t m;
                if (gj & HH_GR_CONST) {
                    sin.d = (uint32_t)(gj & 0xf);
                    sin.e = (uint32_t)((gj >> 4) & 0xfff);
                    sin.delta = (int32_t)(int16_t)(uint16_t)(gj >> 16);
                    m = j + 1;
                } else {
                    m = 0;                                   // from tile 0's entry
                }
                for (; m < (int64_t)tile; m++) {             // apply tables forward
                    uint64_t v = ld_sc1(&lb.tabs[m * HH_KM + sin.d]);
                    sin.d = hh_xf_d(v);
                    sin.e = hh_xf_e(v);
                    sin.delta = hh_xf_delta(v);
                }
            }
            const uint64_t mycnt = (uint64_t)((int64_t)hh_xf_count(s_tab[sin.d]) + sin.delta);
            s_state[0] = state_pack(sin);
            s_state[1] = mycnt;
        }
        __syncthreads();
        STAMP(7);
        // (4c) output base: decoupled look-back over tagged counts, one wave
        if (lane < 64) {
            const uint64_t mycnt = s_state[1];
            uint64_t excl = 0;
            if (tile == 0) {
                if (lane == 0) st_sc1(&lb.cnt[0], mycnt | (2ull << HH_ST_SHIFT));
            } else {
                if (lane == 0) st_sc1(&lb.cnt[tile], mycnt | (1ull << HH_ST_SHIFT));
                int64_t top = (int64_t)tile - 1;
                for (;;) {
                    const int64_t idx = top - (int64_t)lane;
                    uint64_t w = idx >= 0 ? ld_sc1(&lb.cnt[idx]) : (2ull << HH_ST_SHIFT);
                    uint32_t spins = 0;
                    uint32_t first;
                    for (;;) {
                        const uint32_t stv = (uint32_t)(w >> HH_ST_SHIFT);
                        const uint64_t incl = __ballot(stv >= 2);
                        const uint64_t zero = __ballot(stv == 0);
                        first = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
                        const uint64_t rel = first < 63 ? ((2ull << first) - 1ull) : ~0ull;
                        if (!(zero & rel)) break;
                        if (stv == 0 && idx >= 0) w = ld_sc1(&lb.cnt[idx]);
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > HH_SPIN_LIMIT) {
                            if (lane == 0) atomicOr(flags, (uint32_t)F_TIMEOUT);
                            first = 0;
                            w = 2ull << HH_ST_SHIFT;
                            break;
                        }
                    }
                    const uint64_t v = lane <= first ? (w & HH_VAL_MASK) : 0ull;
                    excl += wave_sum64(v);
                    if (first < 64) break;
                    top -= 64;
                }
                if (lane == 0) st_sc1(&lb.cnt[tile], (excl + mycnt) | (2ull << HH_ST_SHIFT));
            }
            if (lane == 0) {
                if (tile == ntiles - 1) {
                    flags[2] = (uint32_t)(excl + mycnt);
                    flags[3] = (uint32_t)((excl + mycnt) >> 32);
                }
                s_state[1] = excl;
            }
        }
        __syncthreads();
        const hh_state sin = state_unpack(s_state[0], s_state[1]);
        STAMP(5);

        // (5) live regions of this tile and their runs, emitted to global
        s_mem[lane] = lane >= sin.d && lane < HH_NR;
        __syncthreads();
        if (lane == 0) {
            for (uint32_t i = 0; i < nexc; i++) {
                uint32_t j = s_exc[i], kj = s_k[j];
                if (!s_mem[j]) continue;
                for (uint32_t q = j + 1; q < j + kj && q < HH_NR; q++) s_mem[q] = 0;
            }
        }
        __syncthreads();
        const bool live = s_mem[lane] != 0;
        if (live && lane + kk < HH_NR) {
            s_ein[lane + kk] = (uint16_t)r.e;
            s_din[lane + kk] = (int16_t)r.delta;
        }
        __syncthreads();
        uint32_t e_in = 0;
        int32_t del_in = 0;
        if (live) {
            e_in = lane == sin.d ? sin.e : s_ein[lane];
            del_in = lane == sin.d ? sin.delta : s_din[lane];
        }
        const uint32_t cnt = live ? (uint32_t)((int32_t)(r.n + r.cov) + del_in) : 0u;
        uint32_t total;
        const uint32_t off = block_excl_scan(cnt, s_cnt4, &total);
        const uint64_t base = sin.base;
        if (base + total > cap) {
            if (lane == 0) atomicOr(flags, (uint32_t)F_OVER);
        } else if (live) {
            const uint32_t start = lane * S + e_in;
            const uint32_t end = (lane + kk) * S + r.e;
            const uint32_t pe = end < c.bt ? end : c.bt;
            if (start < pe) emit_run_global(&c, start, pe, out + base + off);
        }
        STAMP(6);
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
    uint32_t diag_stop;  // HIPHUFF_DIAG_STOP: time the phases (diagnostic only)
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
    const char *ds = getenv("HIPHUFF_DIAG_STOP");
    d->diag_stop = ds ? (uint32_t)atoi(ds) : 0u;
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
    // workspace: [flags 64 B | counter, granules, counts (zeroed) | tables]
    const size_t zero_bytes = (16 + ntiles * 16 + 15) & ~(size_t)15;
    size_t need = 64 + zero_bytes + ntiles * HH_KM * 8 + 256;
    int rc = ensure_ws(d, need);
    if (rc) return rc;
    uint8_t *w = (uint8_t *)d->ws;
    uint32_t *d_flags = (uint32_t *)w;
    LookBack lb;
    lb.counter = (uint32_t *)(w + 64);
    lb.gran = (uint64_t *)(w + 64 + 16);
    lb.cnt = lb.gran + ntiles;
    lb.tabs = (uint64_t *)(w + 64 + zero_bytes);
    const size_t l2b = sizeof(uint32_t) * d->tab.l2_used;
    if (!d->grid || d->grid_l2b != l2b) {
        int per_cu = 0, ncu = 0;
        HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_decode, HH_NL, l2b));
        d->grid_l2b = l2b;
        if (d->d_dbg) HIP_OK(hipFree(d->d_dbg));
        HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d->device));
        d->grid = (uint32_t)((per_cu > 0 ? per_cu : 1) * ncu);
        HIP_OK(hipMalloc(&d->d_dbg, (size_t)d->grid * 8 * sizeof(uint64_t)));
        HIP_OK(hipMemset(d->d_dbg, 0, (size_t)d->grid * 8 * sizeof(uint64_t)));
    }
    const uint32_t grid = (uint32_t)(ntiles < d->grid ? ntiles : d->grid);

    HIP_OK(hipMemsetAsync(d_flags, 0, 64 + zero_bytes, st));
    HIP_OK(hipEventRecord(d->ev[0], st));
    hipLaunchKernelGGL(k_decode, dim3(grid), dim3(HH_NL), l2b, st, (const uint32_t *)d_data, bits,
                       nwords_ok, S, d->tab, ntiles, lb, (uint8_t *)d_out, cap, d_flags, d->diag_stop,
                       d->d_dbg);
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
    if (d->diag_stop) { *out_len = 0; return HH_OK; }
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
extern "C" int hh_debug_phase_cycles(hh_decoder *d, uint64_t *out, int max_blocks) {
    if (!d || !out || !d->d_dbg) return 0;
    int n = (int)d->grid < max_blocks ? (int)d->grid : max_blocks;
    if (hipMemcpy(out, d->d_dbg, (size_t)n * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        return HH_ERR_DEVICE;
    return n;
}
