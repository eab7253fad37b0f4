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
// K1: speculative region decode + stitching walks + tile transfer table
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(HH_NL) void k_sync(const uint32_t *__restrict__ gdata, uint64_t bits,
                                                uint64_t nwords_ok, uint32_t S, DevTab tab,
                                                uint64_t *__restrict__ rec,
                                                uint64_t *__restrict__ ttab, uint32_t *flags) {
    __shared__ uint64_t s_l1[HH_L1_SIZE];
    __shared__ uint32_t s_w[HH_NW_MAX];
    __shared__ uint8_t s_mem[HH_NL];
    __shared__ uint8_t s_k[HH_NL];
    __shared__ uint16_t s_exc[HH_NL];
    __shared__ uint32_t s_cnt4[4];
    __shared__ int32_t s_part[4][HH_KM];
    __shared__ uint64_t s_out[HH_KM];
    extern __shared__ uint32_t s_l2[];

    const uint64_t tile = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    TileGeom g = tile_geom(tile, S, bits);
    stage_tables(s_l1, s_l2, tab);
    stage_words(s_w, gdata, g.b0 >> 5, g.nw, nwords_ok);
    __syncthreads();

    hh_ctx c;
    c.w = s_w; c.sh = (uint32_t)(g.b0 & 31); c.l1 = s_l1; c.l2 = s_l2;
    c.tree = tab.tree; c.tsym = tab.tsym; c.bt = g.bt;

    const uint32_t p0 = lane * S;
    uint32_t n = 0, x = p0;
    if (p0 < c.bt) x = hh_region_count(&c, p0, p0 + S, &n);
    hh_rec r;
    hh_walk(&c, lane, S, x, &r);
    r.n = n;
    rec[tile * HH_NL + lane] = hh_rec_pack(r);
    if (r.k == 0) atomicOr(flags, (uint32_t)F_FAIL);
    const uint32_t kk = r.k ? r.k : 1u;

    // live-lane sets for every entering d: bit d of s_mem[j] <=> lane j live
    s_mem[lane] = lane >= HH_KM - 1 ? 0xffu : (uint8_t)((1u << (lane + 1)) - 1u);
    s_k[lane] = (uint8_t)kk;
    uint32_t nexc = collect_exceptions(kk > 1, s_exc, s_cnt4);
    if (lane == 0) {
        for (uint32_t i = 0; i < nexc; i++) {
            uint32_t j = s_exc[i];
            uint32_t kj = s_k[j];
            uint8_t m = s_mem[j];
            for (uint32_t q = j + 1; q < j + kj && q < HH_NL; q++) s_mem[q] &= (uint8_t)~m;
        }
    }
    __syncthreads();
    const uint32_t mem = s_mem[lane];
    const int32_t contrib = (int32_t)(r.n + r.cov) + (lane + kk < HH_NL ? r.delta : 0);
    if (lane + kk >= HH_NL) {
        for (uint32_t d = 0; d < HH_KM; d++)
            if ((mem >> d) & 1u) s_out[d] = hh_xf_pack(0, r.delta, r.e, lane + kk - HH_NL);
    }
#pragma unroll
    for (uint32_t d = 0; d < HH_KM; d++) {
        int32_t v = ((mem >> d) & 1u) ? contrib : 0;
        v = (int32_t)wave_sum((uint32_t)v);
        if ((lane & 63) == 0) s_part[lane >> 6][d] = v;
    }
    __syncthreads();
    if (lane < HH_KM) {
        int32_t cnt = s_part[0][lane] + s_part[1][lane] + s_part[2][lane] + s_part[3][lane];
        uint64_t o = s_out[lane];
        ttab[tile * HH_KM + lane] = hh_xf_pack((uint32_t)cnt, hh_xf_delta(o), hh_xf_e(o), hh_xf_d(o));
    }
}

// ---------------------------------------------------------------------------
// K2: ordered composition of tile tables -> entering state of every tile.
// state[t] = {d | e<<8 | delta<<32, base}; state[ntiles] holds the total.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(HH_SCAN_T) void k_scan(const uint64_t *__restrict__ ttab, uint64_t ntiles,
                                                    uint64_t *__restrict__ state, uint32_t *flags) {
    __shared__ hh_fn s_agg[HH_SCAN_T];
    __shared__ uint64_t s_pre[HH_SCAN_T][2];
    const uint32_t t = threadIdx.x;
    const uint64_t per = (ntiles + HH_SCAN_T - 1) / HH_SCAN_T;
    const uint64_t t0 = t * per;
    const uint64_t t1 = t0 + per < ntiles ? t0 + per : ntiles;
    if (t0 < t1) {
        hh_fn f;
        hh_fn_from_tab(&ttab[t0 * HH_KM], &f);
        for (uint64_t i = t0 + 1; i < t1; i++) {
            hh_fn gfn;
            hh_fn_from_tab(&ttab[i * HH_KM], &gfn);
            hh_fn_compose(&f, &gfn, &f);
        }
        s_agg[t] = f;
    }
    __syncthreads();
    if (t == 0) {
        hh_state s = {0, 0, 0, 0};
        for (uint32_t i = 0; i < HH_SCAN_T; i++) {
            s_pre[i][0] = (uint64_t)s.d | ((uint64_t)s.e << 8) | ((uint64_t)(uint32_t)s.delta << 32);
            s_pre[i][1] = s.base;
            if (i * per < ntiles) s = hh_fn_apply(&s_agg[i], s);
        }
        state[ntiles * 2] = (uint64_t)s.d | ((uint64_t)s.e << 8) | ((uint64_t)(uint32_t)s.delta << 32);
        state[ntiles * 2 + 1] = s.base;
        flags[2] = (uint32_t)s.base;
        flags[3] = (uint32_t)(s.base >> 32);
    }
    __syncthreads();
    if (t0 < t1) {
        hh_state s;
        uint64_t p = s_pre[t][0];
        s.d = (uint32_t)(p & 0xff);
        s.e = (uint32_t)((p >> 8) & 0xffffff);
        s.delta = (int32_t)(uint32_t)(p >> 32);
        s.base = s_pre[t][1];
        for (uint64_t i = t0; i < t1; i++) {
            state[i * 2] = (uint64_t)s.d | ((uint64_t)s.e << 8) | ((uint64_t)(uint32_t)s.delta << 32);
            state[i * 2 + 1] = s.base;
            s = hh_xf_apply(&ttab[i * HH_KM], s);
        }
    }
}

// ---------------------------------------------------------------------------
// K3: emission of every live run through an LDS staging window.
// ---------------------------------------------------------------------------
struct StageSink {
    uint8_t *stage;
    uint64_t origin;   // output index of stage[0]
    __device__ __forceinline__ void operator()(uint64_t o, uint32_t b) {
        stage[o - origin] = (uint8_t)b;
    }
};

__global__ __launch_bounds__(HH_NL) void k_emit(const uint32_t *__restrict__ gdata, uint64_t bits,
                                                uint64_t nwords_ok, uint32_t S, DevTab tab,
                                                const uint64_t *__restrict__ rec,
                                                const uint64_t *__restrict__ state,
                                                uint8_t *__restrict__ out, uint64_t cap,
                                                uint32_t *flags) {
    __shared__ uint64_t s_l1[HH_L1_SIZE];
    __shared__ uint32_t s_w[HH_NW_MAX];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[HH_CAP];
    __shared__ uint8_t s_mem[HH_NL];
    __shared__ uint8_t s_k[HH_NL];
    __shared__ uint16_t s_exc[HH_NL];
    __shared__ uint16_t s_ein[HH_NL];
    __shared__ int16_t s_din[HH_NL];
    __shared__ uint32_t s_cnt4[4];
    extern __shared__ uint32_t s_l2[];

    const uint64_t tile = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    TileGeom g = tile_geom(tile, S, bits);
    stage_tables(s_l1, s_l2, tab);
    stage_words(s_w, gdata, g.b0 >> 5, g.nw, nwords_ok);
    const hh_rec r = hh_rec_unpack(rec[tile * HH_NL + lane]);
    const uint32_t kk = r.k ? r.k : 1u;
    const uint64_t sp = state[tile * 2];
    const uint32_t d_in = (uint32_t)(sp & 0xff);
    const uint32_t e_tile = (uint32_t)((sp >> 8) & 0xffffff);
    const int32_t del_tile = (int32_t)(uint32_t)(sp >> 32);
    const uint64_t base = state[tile * 2 + 1];
    const uint64_t base_next = state[tile * 2 + 3];

    s_mem[lane] = lane >= d_in;
    s_k[lane] = (uint8_t)kk;
    uint32_t nexc = collect_exceptions(kk > 1, s_exc, s_cnt4);   // syncs
    if (lane == 0) {
        for (uint32_t i = 0; i < nexc; i++) {
            uint32_t j = s_exc[i];
            if (!s_mem[j]) continue;
            uint32_t kj = s_k[j];
            for (uint32_t q = j + 1; q < j + kj && q < HH_NL; q++) s_mem[q] = 0;
        }
    }
    __syncthreads();
    const bool live = s_mem[lane] != 0;
    if (live && lane + kk < HH_NL) {
        s_ein[lane + kk] = (uint16_t)r.e;
        s_din[lane + kk] = (int16_t)r.delta;
    }
    __syncthreads();
    uint32_t e_in = 0;
    int32_t del_in = 0;
    if (live) {
        e_in = lane == d_in ? e_tile : s_ein[lane];
        del_in = lane == d_in ? del_tile : s_din[lane];
    }
    const uint32_t cnt = live ? (uint32_t)((int32_t)(r.n + r.cov) + del_in) : 0u;
    uint32_t total;
    const uint32_t off = block_excl_scan(cnt, s_cnt4, &total);
    if (lane == 0 && base + total != base_next) atomicOr(flags, (uint32_t)F_MISMATCH);

    hh_ctx c;
    c.w = s_w; c.sh = (uint32_t)(g.b0 & 31); c.l1 = s_l1; c.l2 = s_l2;
    c.tree = tab.tree; c.tsym = tab.tsym; c.bt = g.bt;
    uint32_t p = lane * S + e_in;
    const uint32_t end = (lane + kk) * S + r.e;
    const uint32_t pe = live ? (end < c.bt ? end : c.bt) : 0u;
    uint64_t o = base + off;

    // window in absolute addresses; never write at or beyond out + cap
    const uint64_t oaddr = (uint64_t)(uintptr_t)out;
    uint64_t hi_idx = base + total;
    if (hi_idx > cap) {
        if (lane == 0) atomicOr(flags, (uint32_t)F_OVER);
        hi_idx = cap;
    }
    if (base >= hi_idx) return;
    const uint64_t lo = oaddr + base, hi = oaddr + hi_idx;
    const uint64_t a0 = lo & ~(uint64_t)15;
    const uint32_t nrounds = (uint32_t)((hi - a0 + HH_CAP - 1) / HH_CAP);
    for (uint32_t rd = 0; rd < nrounds; rd++) {
        const uint64_t wa = a0 + (uint64_t)rd * HH_CAP;
        const uint64_t wend_idx = (wa + HH_CAP < hi ? wa + HH_CAP : hi) - oaddr;
        StageSink sink{s_stage, wa - oaddr};
        if (p < pe && o < wend_idx) hh_emit_run(&c, &p, pe, &o, wend_idx, sink);
        __syncthreads();
        for (uint32_t ch = lane; ch < HH_CAP / 16; ch += HH_NL) {
            uint64_t a = wa + 16ull * ch;
            if (a >= hi || a + 16 <= lo) continue;
            if (a >= lo && a + 16 <= hi) {
                *(uint4 *)(uintptr_t)a = *(const uint4 *)&s_stage[16 * ch];
            } else {
                for (uint32_t b = 0; b < 16; b++)
                    if (a + b >= lo && a + b < hi) *(uint8_t *)(uintptr_t)(a + b) = s_stage[16 * ch + b];
            }
        }
        __syncthreads();
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
    const uint64_t tb = (uint64_t)HH_NL * S;
    const uint64_t ntiles = (bits + tb - 1) / tb;
    const uint64_t nwords_ok = ((bits + 7) / 8 + HH_PAYLOAD_PAD) / 4;
    size_t need = 64 + ntiles * HH_NL * 8 + ntiles * HH_KM * 8 + (ntiles + 1) * 16 + 256;
    int rc = ensure_ws(d, need);
    if (rc) return rc;
    uint8_t *w = (uint8_t *)d->ws;
    uint32_t *d_flags = (uint32_t *)w;
    uint64_t *d_rec = (uint64_t *)(w + 64);
    uint64_t *d_tab = d_rec + ntiles * HH_NL;
    uint64_t *d_state = d_tab + ntiles * HH_KM;
    const size_t l2b = sizeof(uint32_t) * d->tab.l2_used;

    HIP_OK(hipMemsetAsync(d_flags, 0, 64, st));
    HIP_OK(hipEventRecord(d->ev[0], st));
    hipLaunchKernelGGL(k_sync, dim3((unsigned)ntiles), dim3(HH_NL), l2b, st, (const uint32_t *)d_data,
                       bits, nwords_ok, S, d->tab, d_rec, d_tab, d_flags);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(d->ev[1], st));
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(HH_SCAN_T), 0, st, d_tab, ntiles, d_state, d_flags);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(d->ev[2], st));
    hipLaunchKernelGGL(k_emit, dim3((unsigned)ntiles), dim3(HH_NL), l2b, st, (const uint32_t *)d_data,
                       bits, nwords_ok, S, d->tab, d_rec, d_state, (uint8_t *)d_out, cap, d_flags);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(d->ev[3], st));
    HIP_OK(hipMemcpyAsync(d->h_flags, d_flags, 16, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    const uint32_t fl = d->h_flags[0];
    const uint64_t total = (uint64_t)d->h_flags[2] | ((uint64_t)d->h_flags[3] << 32);
    float ms[3];
    for (int i = 0; i < 3; i++) hipEventElapsedTime(&ms[i], d->ev[i], d->ev[i + 1]);
    d->stats.ms_sync = ms[0];
    d->stats.ms_scan = ms[1];
    d->stats.ms_emit = ms[2];
    d->stats.ms_total = ms[0] + ms[1] + ms[2];
    d->stats.lanes = ntiles * HH_NL;
    d->stats.out_len = total;
    if (fl & F_FAIL) {
        // A walk found no shared boundary within HH_KM regions: the code does
        // not resynchronise (non-synchronising code) -- take the exact path.
        d->stats.exact_fallback = 1;
        return stage_pipeline(d, d_data, (int64_t)bits, (uint8_t *)d_out, cap, out_len, st);
    }
    if (fl & F_MISMATCH) return HH_ERR_INTERNAL;
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
