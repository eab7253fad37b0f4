/*
 * hh_algo.h -- per-lane building blocks of the O(N) speculative decoder.
 *
 * Everything here is __host__ __device__: the HIP kernels (hh_device.hip)
 * call it on LDS-resident data, and the test-only emulator
 * (tests/emu/hh_emu.cpp) calls it on host arrays to check the stitching
 * logic against the oracle without a GPU.
 *
 * Restatement of the reference pipeline (ReleaseCL/kernels/ *.cl):
 *
 *  decodeallbits  -> a lane decodes its region of S bits speculatively from
 *                    the region start (offset 0): `hh_region_count`.
 *  makebigtable   -> instead of pointer doubling over an int32[25][bits]
 *                    table, chains are stitched directly: the chain leaving
 *                    region j (exact if region j's own chain is exact at its
 *                    exit) is walked in lock-step with region j+1's
 *                    offset-0 chain until the two share a code boundary
 *                    (`hh_walk`).  Sharing a boundary means identical from
 *                    there on, so the merge is exact, never a heuristic.  A
 *                    walk that finds no shared boundary in region j+1 carries
 *                    on into j+2, ... (region j+1 is then "covered").
 *  calcbitsindex  -> the output index of every true boundary follows from a
 *                    prefix sum over per-region symbol counts (hh_orbit_*).
 *  calcresult     -> emission: each live region re-decodes its exact run and
 *                    writes the symbols (`hh_emit_run`).
 *  findmax        -> the total of the prefix sum.
 */
#ifndef HH_ALGO_H_
#define HH_ALGO_H_

#include <stdint.h>
#include "hh_internal.h"

#if defined(__HIPCC__)
#define HH_HD __host__ __device__ __forceinline__
#else
#define HH_HD static inline
#endif
/* This header is C++ (hipcc for the kernels, g++ for the test emulator). */

/* Lanes per tile, max regions a walk may cross (the cross-tile state d is
 * in [0, HH_KM)). */
#define HH_NL 256
#define HH_KM 8

typedef struct {
    const uint32_t *w;      /* tile words; stream bit (tile_bit0 + p) is bit
                               ((p + sh) & 31) of w[(p + sh) >> 5]         */
    uint32_t sh;            /* tile_bit0 & 31                              */
    const uint64_t *l1;     /* HH_L1_SIZE entries                          */
    const uint32_t *l2;
    const uint32_t *tree;   /* compact tree                                */
    const uint8_t *tsym;
    uint32_t bt;            /* end of stream relative to the tile (clamped) */
} hh_ctx;

HH_HD uint32_t hh_read32(const hh_ctx *c, uint32_t p) {
    uint32_t q = p + c->sh;
    uint32_t lo = c->w[q >> 5], hi = c->w[(q >> 5) + 1];
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, q & 31);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (q & 31));
#endif
}

HH_HD uint32_t hh_bit(const hh_ctx *c, uint32_t p) {
    uint32_t q = p + c->sh;
    return (c->w[q >> 5] >> (q & 31)) & 1u;
}

/* The reference's tail rule (decodeallbits.cl:20-31): walking from the root
 * at p, stop at a leaf or at the end of the stream; the node reached gives
 * the symbol byte.  Used only for a code cut off by the end of the stream. */
HH_HD uint32_t hh_tail_symbol(const hh_ctx *c, uint32_t p) {
    uint32_t node = 0;
    while (p < c->bt) {
        uint32_t t = c->tree[node];
        if (t & HH_T_LEAF) break;
        node = hh_bit(c, p) ? (t >> 15) & 0x7fffu : t & 0x7fffu;
        p++;
    }
    return c->tsym[node];
}

/* First code longer than HH_P bits: second-level table, then (very long
 * codes only) a bit-serial walk.  Returns the code length; a walk that hits
 * the end of the stream returns the cut-off length with the internal
 * node's symbol, exactly the tail rule. */
HH_HD uint32_t hh_escape(const hh_ctx *c, uint32_t p, uint32_t win, uint64_t e,
                         uint32_t *sym) {
    uint32_t q = HH_L1_L2Q(e), base = HH_L1_L2BASE(e);
    uint32_t e2 = c->l2[base + ((win >> HH_P) & ((1u << q) - 1u))];
    if (e2 & HH_L2_LEAF) {
        *sym = e2 & 0xffu;
        return (e2 >> 8) & 0xffu;
    }
    uint32_t node = e2 & 0xffffffu, d = HH_P + q;
    for (;;) {
        uint32_t t = c->tree[node];
        if (t & HH_T_LEAF) { *sym = t & 0xffu; return d; }
        if (p + d >= c->bt) { *sym = c->tsym[node]; return d; }
        node = hh_bit(c, p + d) ? (t >> 15) & 0x7fffu : t & 0x7fffu;
        d++;
    }
}

/* Length of the one code starting at p (< bt), cut at the stream end. */
HH_HD uint32_t hh_len1(const hh_ctx *c, uint32_t p) {
    uint32_t win = hh_read32(c, p);
    uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
    uint32_t l;
    if (HH_L1_NSYM(e)) {
        l = HH_L1_LEN0(e);
    } else {
        uint32_t s;
        l = hh_escape(c, p, win, e, &s);
    }
    uint32_t rem = c->bt - p;
    return l < rem ? l : rem;
}

/* One symbol at p (< bt) with its length (tail rule applied). */
HH_HD uint32_t hh_dec1(const hh_ctx *c, uint32_t p, uint32_t *sym) {
    uint32_t win = hh_read32(c, p);
    uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
    uint32_t l, s;
    if (HH_L1_NSYM(e)) {
        l = HH_L1_LEN0(e);
        s = HH_L1_SYMS(e) & 0xffu;
    } else {
        l = hh_escape(c, p, win, e, &s);
    }
    if (l > c->bt - p) {
        s = hh_tail_symbol(c, p);
        l = c->bt - p;
    }
    *sym = s;
    return l;
}

/* Phase A (decodeallbits restated): count the symbols of the chain that
 * starts at p0 and whose starts lie in [p0, lim).  Returns the exit, the
 * first position >= lim on the chain (or bt). */
HH_HD uint32_t hh_region_count(const hh_ctx *c, uint32_t p0, uint32_t lim,
                               uint32_t *count) {
    uint32_t p = p0, n = 0;
    if (lim > c->bt) lim = c->bt;
    while (p < lim) {
        uint32_t win = hh_read32(c, p);
        uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
        uint32_t ns = HH_L1_NSYM(e);
        uint32_t l;
        if (ns) {
            uint32_t nb = HH_L1_NBITS(e);
            if (p + nb <= lim) {
                p += nb;
                n += ns;
                continue;
            }
            l = HH_L1_LEN0(e);
        } else {
            uint32_t s;
            l = hh_escape(c, p, win, e, &s);
        }
        uint32_t rem = c->bt - p;
        p += l < rem ? l : rem;
        n += 1;
    }
    *count = n;
    return p;
}

/* Walk result, packed per lane (u64):
 *   bits  0..15 n      symbols of the lane's own offset-0 chain in its region
 *   bits 16..31 cov    symbols of the walk in covered regions (k > 1)
 *   bits 32..47 delta  (signed) correction for the region the walk merged in:
 *                      walk symbols before the merge minus that region's own
 *                      chain symbols before the merge
 *   bits 48..59 e      entry offset of the walk into the merge region
 *   bits 60..63 k      regions crossed (1 = merged in the next region);
 *                      0 = failed (no merge within HH_KM regions)
 */
typedef struct {
    uint32_t n, cov, e, k;
    int32_t delta;
} hh_rec;

HH_HD uint64_t hh_rec_pack(hh_rec r) {
    return (uint64_t)(r.n & 0xffffu) | ((uint64_t)(r.cov & 0xffffu) << 16) |
           ((uint64_t)((uint32_t)r.delta & 0xffffu) << 32) |
           ((uint64_t)(r.e & 0xfffu) << 48) | ((uint64_t)(r.k & 0xfu) << 60);
}
HH_HD hh_rec hh_rec_unpack(uint64_t v) {
    hh_rec r;
    r.n = (uint32_t)(v & 0xffffu);
    r.cov = (uint32_t)((v >> 16) & 0xffffu);
    r.delta = (int32_t)(int16_t)(uint16_t)((v >> 32) & 0xffffu);
    r.e = (uint32_t)((v >> 48) & 0xfffu);
    r.k = (uint32_t)(v >> 60);
    return r;
}

/* Phase B (makebigtable restated): the chain leaving region `lane` at x
 * (>= region end, <= bt) walked against region lane+1's offset-0 chain,
 * two pointers, always advancing the one behind; a pointer that has left
 * the region stops.  Same position = merged.  Both out of the region and
 * different = region lane+1 is covered by this walk; continue with the next
 * region.  S = region bits. */
HH_HD void hh_walk(const hh_ctx *c, uint32_t lane, uint32_t S, uint32_t x,
                   hh_rec *r) {
    r->k = 1; r->e = 0; r->delta = 0; r->cov = 0;
    uint32_t A = x;
    uint32_t R = lane + 1;
    if (A < R * S) return;      /* stream ended inside this region */
    for (uint32_t it = 0; it < HH_KM; it++, R++) {
        uint32_t Lr = R * S, Le = Lr + S;
        uint32_t eA = A - Lr;
        uint32_t B = Lr, ca = 0, cb = 0;
        for (;;) {
            if (A == B) {
                r->k = it + 1;
                r->e = eA;
                r->delta = (int32_t)ca - (int32_t)cb;
                return;
            }
            uint32_t ad = A >= Le, bd = B >= Le;
            if (ad && bd) break;
            if (!ad && (bd || A < B)) {
                A += hh_len1(c, A);
                ca++;
            } else {
                B += hh_len1(c, B);
                cb++;
            }
        }
        r->cov += ca;
    }
    r->k = 0;   /* no merge within HH_KM regions */
}

/* ------------------------------------------------------------------ */
/* Boundary masks.  Phase A also records, for its region, a bit per     */
/* position that starts a code of its offset-0 chain (mask word w, bit  */
/* i <=> position 32w + i of the region).  A walk then decodes only the */
/* incoming chain, several codes per lookup, and tests each lookup's    */
/* start positions against the next region's mask -- the first common   */
/* start is exactly the two-pointer merge point (hh_walk), found in a   */
/* fraction of the steps.                                               */
/* ------------------------------------------------------------------ */
#define HH_MW_MAX 10   /* mask words per region (S <= 320) */

typedef struct {
    const uint32_t *m;    /* [nreg][mw] region masks            */
    const uint16_t *x;    /* [nreg] exit offset from region start */
    const uint16_t *n;    /* [nreg] own-chain symbol counts        */
    uint32_t nreg;        /* regions with a mask (tile-local 0..)  */
    uint32_t mw;          /* words per region mask                 */
} hh_masks;

/* Phase A with the boundary mask: like hh_region_count, plus
 * sink(w, word) for every mask word w in [0, mw). */
template <class MaskSink>
HH_HD uint32_t hh_region_count_mask(const hh_ctx *c, uint32_t p0, uint32_t lim, uint32_t mw,
                                    uint32_t *count, MaskSink &sink) {
    uint32_t p = p0, n = 0, wdone = 0, mbase = p0;
    uint64_t macc = 0;
    if (lim > c->bt) lim = c->bt;
    while (p < lim) {
        uint32_t win = hh_read32(c, p);
        uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
        uint32_t ns = HH_L1_NSYM(e);
        uint32_t l, bm = 1u;
        if (ns) {
            uint32_t nb = HH_L1_NBITS(e);
            if (p + nb <= lim) {
                l = nb;
                bm = HH_L1_BMASK(e);
            } else {
                l = HH_L1_LEN0(e);
                ns = 1;
            }
        } else {
            uint32_t s;
            l = hh_escape(c, p, win, e, &s);
            ns = 1;
        }
        macc |= (uint64_t)bm << (p - mbase);
        uint32_t rem = c->bt - p;
        p += l < rem ? l : rem;
        n += ns;
        while (p - mbase >= 32 && wdone < mw) {
            sink(wdone++, (uint32_t)macc);
            macc >>= 32;
            mbase += 32;
        }
    }
    while (wdone < mw) {
        sink(wdone++, (uint32_t)macc);
        macc >>= 32;
    }
    *count = n;
    return p;
}

/* Symbols of region r's own chain that start before region offset `off`. */
HH_HD uint32_t hh_mask_rank(const hh_masks *mk, uint32_t r, uint32_t off) {
    const uint32_t *m = mk->m + r * mk->mw;
    uint32_t cnt = 0, w = 0;
    for (; w < (off >> 5); w++) cnt += __builtin_popcount(m[w]);
    if (off & 31u) cnt += __builtin_popcount(m[w] & ((1u << (off & 31u)) - 1u));
    return cnt;
}

/* Phase B with masks: same result as hh_walk.  Regions >= mk->nreg (past
 * the tile's masks) fall back to the two-pointer walk. */
HH_HD void hh_walk_mask(const hh_ctx *c, const hh_masks *mk, uint32_t lane, uint32_t S,
                        uint32_t x, hh_rec *r) {
    r->k = 1; r->e = 0; r->delta = 0; r->cov = 0;
    uint32_t A = x;
    uint32_t R = lane + 1;
    if (A < R * S) return;      /* stream ended inside this region */
    for (uint32_t it = 0; it < HH_KM; it++, R++) {
        const uint32_t Lr = R * S, Le = Lr + S;
        const uint32_t eA = A - Lr;
        uint32_t ca = 0;
        if (R < mk->nreg) {
            const uint32_t *m = mk->m + R * mk->mw;
            const uint32_t lim = Le < c->bt ? Le : c->bt;
            while (A < lim) {
                uint32_t win = hh_read32(c, A);
                uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
                uint32_t ns = HH_L1_NSYM(e), l, bm = 1u;
                if (ns && A + HH_L1_NBITS(e) <= lim) {
                    l = HH_L1_NBITS(e);
                    bm = HH_L1_BMASK(e);
                } else {
                    if (ns) {
                        l = HH_L1_LEN0(e);
                    } else {
                        uint32_t s;
                        l = hh_escape(c, A, win, e, &s);
                    }
                    ns = 1;
                }
                const uint32_t off = A - Lr, wi = off >> 5, sh = off & 31u;
                uint64_t mm = (uint64_t)m[wi];
                if (wi + 1 < mk->mw) mm |= (uint64_t)m[wi + 1] << 32;
                const uint32_t hit = bm & (uint32_t)(mm >> sh);
                if (hit) {
                    const uint32_t t = (uint32_t)__builtin_ctz(hit);
                    const uint32_t a = ca + (uint32_t)__builtin_popcount(bm & ((1u << t) - 1u));
                    const uint32_t b = hh_mask_rank(mk, R, off + t);
                    r->k = it + 1;
                    r->e = eA;
                    r->delta = (int32_t)a - (int32_t)b;
                    return;
                }
                uint32_t rem = c->bt - A;
                A += l < rem ? l : rem;
                ca += ns;
            }
            /* both chains leave the region at the same point -> merged there */
            if (A == Lr + mk->x[R] || A >= c->bt) {
                r->k = it + 1;
                r->e = eA;
                r->delta = (int32_t)ca - (int32_t)mk->n[R];
                return;
            }
        } else {
            uint32_t B = Lr, cb = 0;
            for (;;) {
                if (A == B) {
                    r->k = it + 1;
                    r->e = eA;
                    r->delta = (int32_t)ca - (int32_t)cb;
                    return;
                }
                uint32_t ad = A >= Le, bd = B >= Le;
                if (ad && bd) break;
                if (!ad && (bd || A < B)) {
                    A += hh_len1(c, A);
                    ca++;
                } else {
                    B += hh_len1(c, B);
                    cb++;
                }
            }
        }
        r->cov += ca;
    }
    r->k = 0;
}

/* ------------------------------------------------------------------ */
/* Cross-tile state and tile transfer tables.                          */
/* The state entering a tile: d = first live lane of the tile (lanes    */
/* before it are covered by a walk from the previous tile), e = its     */
/* entry offset, delta = its count correction.  A tile table maps every */
/* d in [0, HH_KM) to the state leaving the tile and the number of      */
/* symbols the tile's live lanes emit (delta of the entering lane not   */
/* included -- it is added when tables are applied).                   */
/* ------------------------------------------------------------------ */
HH_HD uint64_t hh_xf_pack(uint32_t count, int32_t delta, uint32_t e, uint32_t d) {
    return (uint64_t)count | ((uint64_t)((uint32_t)delta & 0xffffu) << 32) |
           ((uint64_t)(e & 0xfffu) << 48) | ((uint64_t)(d & 0xfu) << 60);
}
HH_HD uint32_t hh_xf_count(uint64_t v) { return (uint32_t)v; }
HH_HD int32_t hh_xf_delta(uint64_t v) { return (int32_t)(int16_t)(uint16_t)(v >> 32); }
HH_HD uint32_t hh_xf_e(uint64_t v) { return (uint32_t)(v >> 48) & 0xfffu; }
HH_HD uint32_t hh_xf_d(uint64_t v) { return (uint32_t)(v >> 60); }

/* Tile state: packed (d, e, delta) + 64-bit output base. */
typedef struct {
    uint32_t d, e;
    int32_t delta;
    uint64_t base;
} hh_state;

/* Apply a tile table to the entering state. */
HH_HD hh_state hh_xf_apply(const uint64_t *tab, hh_state s) {
    uint64_t v = tab[s.d];
    hh_state o;
    o.base = s.base + (uint64_t)((int64_t)hh_xf_count(v) + s.delta);
    o.d = hh_xf_d(v);
    o.e = hh_xf_e(v);
    o.delta = hh_xf_delta(v);
    return o;
}

/* Generic composed function over d (64-bit counts): used by the scan. */
typedef struct {
    uint8_t d[HH_KM];
    uint16_t e[HH_KM];
    int16_t delta[HH_KM];
    uint64_t cnt[HH_KM];
} hh_fn;

HH_HD void hh_fn_from_tab(const uint64_t *tab, hh_fn *f) {
    for (int i = 0; i < HH_KM; i++) {
        uint64_t v = tab[i];
        f->d[i] = (uint8_t)hh_xf_d(v);
        f->e[i] = (uint16_t)hh_xf_e(v);
        f->delta[i] = (int16_t)hh_xf_delta(v);
        f->cnt[i] = hh_xf_count(v);
    }
}

/* h = g after f (f applied first). */
HH_HD void hh_fn_compose(const hh_fn *f, const hh_fn *g, hh_fn *h) {
    hh_fn t;
    for (int i = 0; i < HH_KM; i++) {
        uint32_t j = f->d[i];
        uint8_t gd = 0; uint16_t ge = 0; int16_t gdel = 0; uint64_t gc = 0;
        for (int m = 0; m < HH_KM; m++) {   /* select, no dynamic indexing */
            if ((uint32_t)m == j) { gd = g->d[m]; ge = g->e[m]; gdel = g->delta[m]; gc = g->cnt[m]; }
        }
        t.d[i] = gd; t.e[i] = ge; t.delta[i] = gdel;
        t.cnt[i] = (uint64_t)((int64_t)f->cnt[i] + f->delta[i]) + gc;
    }
    *h = t;
}

HH_HD hh_state hh_fn_apply(const hh_fn *f, hh_state s) {
    hh_state o = s;
    for (int m = 0; m < HH_KM; m++) {
        if ((uint32_t)m == s.d) {
            o.base = s.base + (uint64_t)((int64_t)f->cnt[m] + s.delta);
            o.d = f->d[m]; o.e = f->e[m]; o.delta = f->delta[m];
        }
    }
    return o;
}

/* ------------------------------------------------------------------ */
/* Sequential reference forms of the tile resolution (the kernels do   */
/* the same with ballots and LDS; the emulator and the host use these). */
/* ------------------------------------------------------------------ */
HH_HD uint32_t hh_rec_next(uint32_t j, const hh_rec &r) { return j + (r.k ? r.k : 1u); }

/* Tile table over nr regions: for each entering d, follow j -> j + k_j. */
HH_HD void hh_tile_table_seq(const uint64_t *rec, uint32_t nr, uint64_t *tab) {
    for (uint32_t d = 0; d < HH_KM; d++) {
        uint32_t j = d, cnt = 0;
        for (;;) {
            hh_rec r = hh_rec_unpack(rec[j]);
            uint32_t nx = hh_rec_next(j, r);
            cnt += r.n + r.cov;
            if (nx >= nr) { tab[d] = hh_xf_pack(cnt, r.delta, r.e, nx - nr); break; }
            cnt = (uint32_t)((int32_t)cnt + r.delta);
            j = nx;
        }
    }
}

/* Emit one run: decode from *pp while p < pe (a code boundary or bt) and
 * the output index stays below wend.  sink(o, byte) stores a symbol. */
template <class Sink>
HH_HD void hh_emit_run(const hh_ctx *c, uint32_t *pp, uint32_t pe, uint64_t *po,
                       uint64_t wend, Sink &sink) {
    uint32_t p = *pp;
    uint64_t o = *po;
    while (p < pe && o < wend) {
        uint32_t win = hh_read32(c, p);
        uint64_t e = c->l1[win & (HH_L1_SIZE - 1u)];
        uint32_t ns = HH_L1_NSYM(e);
        if (ns && p + HH_L1_NBITS(e) <= pe && o + ns <= wend) {
            uint32_t syms = HH_L1_SYMS(e);
            sink(o, syms & 0xffu);
            if (ns > 1) sink(o + 1, (syms >> 8) & 0xffu);
            if (ns > 2) sink(o + 2, (syms >> 16) & 0xffu);
            if (ns > 3) sink(o + 3, syms >> 24);
            p += HH_L1_NBITS(e);
            o += ns;
        } else {
            uint32_t s;
            uint32_t l = hh_dec1(c, p, &s);
            sink(o, s);
            p += l;
            o++;
        }
    }
    *pp = p;
    *po = o;
}

#endif
