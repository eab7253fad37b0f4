/*
 * hh_algo.h -- per-lane building blocks of the O(N) speculative decoder.
 *
 * Everything here is __host__ __device__: the HIP kernel (hh_device.hip)
 * calls it on LDS-resident data, and the test-only emulator
 * (tests/emu/hh_emu.cpp) calls it on host arrays with the kernel's exact
 * tile geometry and LDS layout, so the stitching logic is checked against
 * the oracle without a GPU.
 *
 * Restatement of the reference pipeline (ReleaseCL/kernels/ *.cl):
 *
 *  decodeallbits  -> lane j decodes its region of S bits speculatively from
 *                    the region start R_j (offset 0): n_j symbols start in
 *                    the region, x_j is the chain's first position at or
 *                    past the region end (`hh_region_count`).
 *  makebigtable   -> instead of pointer doubling over an int32[25][bits]
 *                    table, each region exit is walked against the next
 *                    region's offset-0 chain, two pointers, until the chains
 *                    share a code boundary (`hh_walk`).  A shared boundary
 *                    means identical chains from there on, so the merge is
 *                    exact, never a heuristic.  delta_j = (walk symbols
 *                    before the merge) - (region j+1's own symbols before it).
 *  calcbitsindex  -> output index of every true boundary: prefix sum of the
 *                    CHARGED counts c_j = n_j + delta_j.  The true chain has
 *                    n_j + delta_{j-1} symbols in region j, so the charged
 *                    sum of a tile does not depend on the tile's entry and
 *                    the cross-tile scan is a plain sum.
 *  calcresult     -> each lane re-decodes the exact run [x_{j-1}, x_j) and
 *                    writes its symbols (`hh_emit_step`).
 *  findmax        -> the total of the prefix sum.
 *
 * Chain semantics follow decodeallbits.cl:10-33: from position p, a code of
 * length l ends at p + l; a code cut off by the end of the stream (p + l >
 * bt) is the last symbol, its byte is the sym of the tree node the walk
 * reached (the tail rule), and the chain ends at bt.  Positions are
 * therefore clamped to bt.
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

/* ------------------------------------------------------------------ */
/* Tile geometry.                                                       */
/*   A tile is HH_NR = 64 regions of S bits, one WAVE: lane j owns       */
/*   region j, and everything up to the tile's transfer table happens    */
/*   inside the wave (no workgroup barrier, so a wave with a long walk   */
/*   holds up only itself).  A walk may cross up to HH_KM regions before */
/*   it merges (runs of a repeated symbol keep chains apart for hundreds */
/*   of bits), so a tile stages HH_KM regions of the next tile too, plus */
/*   a halo for codes running past the last one.                         */
/*   The bitstream is staged in LDS TRANSPOSED: tile word g lives at     */
/*   (g % sw) * nls + g / sw, i.e. region r is column r.  Lanes read     */
/*   their own columns, so a wave's reads fall in distinct banks (nls is */
/*   a multiple of 32) however far apart the lanes' chains are.  The     */
/*   emission kernel stages groups of several tiles with its own stride  */
/*   (hh_ctx.nls).                                                       */
/* ------------------------------------------------------------------ */
#define HH_NR 64              /* regions per tile (a wave) */
#define HH_KM 8               /* max regions one walk may cross */
#define HH_NCOL (HH_NR + HH_KM + 1)   /* staged columns */
#ifndef HH_NLS
#define HH_NLS 96             /* column stride of a tile's staging: >= HH_NCOL, multiple of 32 */
#endif
#define HH_SW_MAX 12          /* max words per region (S <= 384) */
#define HH_WALK_MAX 8192      /* iteration cap of one walk (a guard, reported
                                 as a failed walk) */
#ifndef HH_FRONT_WALK
#define HH_FRONT_WALK 0       /* lookups of a walk in k_front; longer walks are
                                 deferred to k_walk (a wave would wait for its
                                 longest walk; 0, 1, 2, 4: kjv front + walks
                                 1.33, 1.37, 1.42, 1.49 ms per GiB) */
#endif

HH_HD uint32_t hh_umulhi(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

HH_HD uint32_t hh_ctz(uint32_t v) {   /* v != 0 */
    return (uint32_t)__builtin_ctz(v);
}
HH_HD uint32_t hh_popc(uint32_t v) { return (uint32_t)__builtin_popcount(v); }
HH_HD uint32_t hh_lowmask(uint32_t o) { return o >= 32 ? 0xffffffffu : ((1u << o) - 1u); }

/* ceil(2^32 / sw): hh_umulhi(g, magic) == g / sw exactly for g < 2^20. */
/* fields of the meta half of an L1 entry (hh_internal.h bits 32..55) */
#define HH_M_NBITS(m) ((m) & 31u)
#define HH_M_NSYM(m) (((m) >> 5) & 7u)
#define HH_M_LEN0(m) (((m) >> 8) & 31u)
#define HH_M_BMASK(m) (((m) >> 13) & ((1u << HH_P) - 1u))
/* escape meta word (nsym == 0): the L2 subtable */
#define HH_M_L2BASE(m) (((m) >> 8) & 0xffffu)
#define HH_M_L2Q(m) (((m) >> 24) & 31u)

HH_HD uint32_t hh_magic(uint32_t sw) { return (uint32_t)((0x100000000ull + sw - 1) / sw); }

typedef struct hh_ctx {
    const uint32_t *w;    /* transposed tile words                        */
    uint32_t sw;          /* words per region                             */
    uint32_t nls;         /* column stride of the staged words            */
    uint32_t magic;       /* hh_magic(sw)                                 */
    const uint32_t *l1m;  /* HH_L1_SIZE entries: the meta half (bits 32..63
                             of the hh_internal.h L1 entry; HH_M_*)      */
    const uint32_t *l1s;  /* the symbol half (bits 0..31; escape: L2 ref) */
    const uint64_t *l1;   /* or both halves interleaved (one 64-bit read per
                             lookup; k_emit), null if split               */
    const uint32_t *l2;
    const uint32_t *tree; /* compact tree (tail symbols, very long codes) */
    const uint8_t *tsym;
    uint32_t bt;          /* end of stream relative to the tile (clamped) */
    uint32_t maxadv;      /* most bits one table step advances:
                             max(HH_P, longest code), <= 32             */
    uint32_t G;           /* overlap: region r's chain starts G bits before
                             the region (r > 0 within a tile), 0 or a
                             multiple of 32 <= 64 (see hh_region_head)   */
    /* the front's table (hh_internal.h F), used by every lookup when pf is
     * HH_PF (k_front, k_walk: no symbol bytes) -- then maxadv must cover
     * HH_PF too */
    const uint16_t *f = nullptr;
    const uint32_t *fdir = nullptr;
    uint32_t pf = 0;
} hh_ctx;

/* The kernel is instantiated per words-per-region (the kernel's hh_ctx has
 * a compile-time sw), so this division folds to shifts / a multiply-high. */
HH_HD uint32_t hh_idx(const hh_ctx *c, uint32_t g) {
    const uint32_t r = g / c->sw;
    return (g - r * c->sw) * c->nls + r;
}
/* LDS index of the word after the one at index a */
HH_HD uint32_t hh_idx_next(const hh_ctx *c, uint32_t a) {
    const uint32_t last = (c->sw - 1) * c->nls;
    return a >= last ? a - last + 1 : a + c->nls;
}
HH_HD uint32_t hh_word(const hh_ctx *c, uint32_t g) { return c->w[hh_idx(c, g)]; }

HH_HD uint32_t hh_funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31));
#endif
}

/* 32 stream bits from tile position p, stream bit p in bit 0 (LSB-first
 * bytes: the reference's window convention, linapproach.c:207-209). */
HH_HD uint32_t hh_win(const hh_ctx *c, uint32_t p) {
    const uint32_t a = hh_idx(c, p >> 5);
    uint32_t lo = c->w[a], hi = c->w[hh_idx_next(c, a)];
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, p & 31);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (p & 31));
#endif
}

HH_HD uint32_t hh_bit(const hh_ctx *c, uint32_t p) {
    return (hh_word(c, p >> 5) >> (p & 31)) & 1u;
}

/* The reference's tail rule (decodeallbits.cl:20-31): walking from the root
 * at p, stop at a leaf or at the end of the stream; the node reached gives
 * the symbol byte.  Used only for a code cut off by the end of the stream. */
/* The tree may live in global memory (k_front): these rare paths end with
 * an explicit wait, so that their loads are complete where the decode loops
 * join them again -- else the compiler waits at every join, i.e. every step,
 * for all memory operations in flight (the symbol stores among them). */
#if defined(__HIP_DEVICE_COMPILE__)
#define HH_LOADS_DONE() __builtin_amdgcn_s_waitcnt(0)
#else
#define HH_LOADS_DONE() do {} while (0)
#endif

HH_HD uint32_t hh_tail_symbol(const hh_ctx *c, uint32_t p) {
    uint32_t node = 0;
    while (p < c->bt) {
        uint32_t t = c->tree[node];
        if (t & HH_T_LEAF) break;
        node = hh_bit(c, p) ? (t >> 15) & 0x7fffu : t & 0x7fffu;
        p++;
    }
    const uint32_t s = c->tsym[node];
    HH_LOADS_DONE();
    return s;
}

/* First code longer than HH_P bits: second-level table, then (very long
 * codes only) a bit-serial walk.  Returns the code length.  A walk that
 * hits the end of the stream returns the cut-off length. */
HH_HD uint32_t hh_escape(const hh_ctx *c, uint32_t p, uint32_t win, uint32_t m, uint32_t *sym) {
    uint32_t q = HH_M_L2Q(m), base = HH_M_L2BASE(m);
    uint32_t e2 = c->l2[base + ((win >> HH_P) & ((1u << q) - 1u))];
    if (e2 & HH_L2_LEAF) {
        *sym = e2 & 0xffu;
        return (e2 >> 8) & 0xffu;
    }
    uint32_t node = e2 & 0xffffffu, d = HH_P + q;
    for (;;) {
        uint32_t t = c->tree[node];
        if (t & HH_T_LEAF) { *sym = t & 0xffu; HH_LOADS_DONE(); return d; }
        if (p + d >= c->bt) { *sym = c->tsym[node]; HH_LOADS_DONE(); return d; }
        node = hh_bit(c, p + d) ? (t >> 15) & 0x7fffu : t & 0x7fffu;
        d++;
    }
}

/* One table lookup at p: up to HH_K whole symbols.
 *   nb   bits of those symbols (next lookup starts at p + nb)
 *   ns   symbols, bm their start offsets (bit 0 always set)
 *   len0 length of the first symbol, syms the bytes (first in bits 0..7) */
typedef struct {
    uint32_t nb, ns, bm, len0, syms;
} hh_look;

HH_HD hh_look hh_lookup_w(const hh_ctx *c, uint32_t p, uint32_t win) {
    if (c->pf) {                                   /* the front's table */
        const uint32_t e = c->f[win & ((1u << c->pf) - 1u)];
        hh_look L;
        L.syms = 0;
        L.nb = e & 15u;
        if (L.nb) {
            const uint32_t r = (e >> 4) << 1;
            L.bm = r | 1u;
            L.ns = hh_popc(L.bm);
            L.len0 = r ? hh_ctz(r) : L.nb;
        } else {
            uint32_t s;
            L.nb = L.len0 = hh_escape(c, p, win, c->fdir[e >> 4], &s);
            L.ns = 1;
            L.bm = 1;
            L.syms = s;
        }
        return L;
    }
    const uint32_t ix = win & (HH_L1_SIZE - 1u);
    const uint64_t e = c->l1 ? c->l1[ix] : 0ull;
    const uint32_t m = c->l1 ? (uint32_t)(e >> 32) : c->l1m[ix];
    hh_look L;
    L.ns = HH_M_NSYM(m);
    if (L.ns) {
        L.nb = HH_M_NBITS(m);
        L.bm = HH_M_BMASK(m);
        L.len0 = HH_M_LEN0(m);
        /* the front kernel stages only the meta half (l1s null): it never
         * needs the symbol bytes */
        L.syms = c->l1 ? (uint32_t)e : c->l1s ? c->l1s[ix] : 0u;
    } else {
        uint32_t s;
        L.nb = L.len0 = hh_escape(c, p, win, m, &s);
        L.ns = 1;
        L.bm = 1;
        L.syms = s;
    }
    return L;
}

HH_HD hh_look hh_lookup(const hh_ctx *c, uint32_t p) { return hh_lookup_w(c, p, hh_win(c, p)); }

/* ------------------------------------------------------------------ */
/* Chain cursor: position p with words p>>5 and p>>5 + 1 in registers and */
/* word p>>5 + 2 preloaded, so a decode step does its table lookup with no */
/* dependent LDS read in front of it.  A step advances <= 32 bits (codes   */
/* of the fast path are <= 32 bits), i.e. crosses at most one word.        */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t p, lo, hi, nx, a;   /* a: LDS index of word p>>5 + 2 (held in nx) */
} hh_cur;

HH_HD hh_cur hh_cur_at(const hh_ctx *c, uint32_t p) {
    hh_cur u;
    const uint32_t a0 = hh_idx(c, p >> 5), a1 = hh_idx_next(c, a0);
    u.p = p;
    u.lo = c->w[a0];
    u.hi = c->w[a1];
    u.a = hh_idx_next(c, a1);
    u.nx = c->w[u.a];
    return u;
}
HH_HD uint32_t hh_cur_win(const hh_cur &u) { return hh_funnel(u.hi, u.lo, u.p & 31); }
HH_HD void hh_cur_adv(const hh_ctx *c, hh_cur &u, uint32_t adv) {
    const uint32_t np = u.p + adv;
    const bool cross = (np >> 5) != (u.p >> 5);
    u.p = np;
    u.lo = cross ? u.hi : u.lo;
    u.hi = cross ? u.nx : u.hi;
    const uint32_t an = hh_idx_next(c, u.a);
    u.a = cross ? an : u.a;
    u.nx = c->w[u.a];
}

/* Offset of the lookup's first boundary at or after offset d (>= 1): a
 * symbol start inside the lookup, or nb (the next lookup's start). */
HH_HD uint32_t hh_first_ge(const hh_look &L, uint32_t d) {
    uint32_t m = d < 32 ? L.bm & ~hh_lowmask(d) : 0u;
    return m ? hh_ctz(m) : L.nb;
}
/* Symbols of the lookup that start before offset o. */
HH_HD uint32_t hh_syms_before(const hh_look &L, uint32_t o) { return hh_popc(L.bm & hh_lowmask(o)); }

/* Pass 1 (decodeallbits restated): the chain from p0 (< lim), counting the
 * symbols that start in [p0, lim) (lim <= bt).  Returns the exit: the
 * chain's first position >= lim (bt if the stream ends first). */
HH_HD uint32_t hh_region_count(const hh_ctx *c, uint32_t p0, uint32_t lim, uint32_t *count,
                               uint32_t *mask = nullptr) {
    hh_cur u = hh_cur_at(c, p0);
    uint32_t n = 0;
    /* Boundary mask of the chain: bit i of mask word g <=> a symbol starts
     * at 32 g + i.  Word g is kept at LDS index hh_idx(g + 2) -- the index
     * the cursor already holds (u.a) while it is in word g -- so recording
     * costs no address arithmetic.  (mlo, mhi) accumulate words p>>5 and
     * p>>5 + 1; the region starts word-aligned. */
    uint32_t mlo = 0, mhi = 0;
    /* main loop: every symbol of a step starts before lim -- a lookup's
     * symbols start within its index bits, an escape's one symbol at p (its
     * code may run past lim, or be cut by the end of the stream: hh_escape) */
    const uint32_t pidx = c->pf ? c->pf : HH_P;
    const uint32_t lf = lim > pidx ? lim - pidx : 0u;
    while (u.p < lf) {
        const uint32_t win = hh_cur_win(u);
        uint32_t ns, nb, bm;
        if (c->pf) {
            const uint32_t e = c->f[win & ((1u << c->pf) - 1u)];
            nb = e & 15u;
            bm = ((e >> 4) << 1) | 1u;
            ns = hh_popc(bm);
            if (nb == 0) {
                uint32_t s;
                nb = hh_escape(c, u.p, win, c->fdir[e >> 4], &s);
                ns = 1;
                bm = 1;
            }
        } else {
            const uint32_t m = c->l1m[win & (HH_L1_SIZE - 1u)];
            ns = HH_M_NSYM(m), nb = HH_M_NBITS(m), bm = HH_M_BMASK(m);
            if (ns == 0) {
                uint32_t s;
                nb = hh_escape(c, u.p, win, m, &s);
                ns = 1;
                bm = 1;
            }
        }
        n += ns;
        if (mask) {
            const uint64_t b = (uint64_t)bm << (u.p & 31);
            mlo |= (uint32_t)b;
            mhi |= (uint32_t)(b >> 32);
            mask[u.a] = mlo;
            const bool cross = ((u.p + nb) >> 5) != (u.p >> 5);
            mlo = cross ? mhi : mlo;
            mhi = cross ? 0u : mhi;
        }
        hh_cur_adv(c, u, nb);
    }
    /* tail: count only the symbols that start before lim */
    while (u.p < lim) {
        hh_look L = hh_lookup_w(c, u.p, hh_cur_win(u));
        const uint32_t o = hh_first_ge(L, lim - u.p);
        n += hh_syms_before(L, o);
        if (mask) {
            const uint64_t b = (uint64_t)(L.bm & hh_lowmask(o)) << (u.p & 31);
            mlo |= (uint32_t)b;
            mhi |= (uint32_t)(b >> 32);
            mask[u.a] = mlo;
            const bool cross = ((u.p + o) >> 5) != (u.p >> 5);
            mlo = cross ? mhi : mlo;
            mhi = cross ? 0u : mhi;
        }
        hh_cur_adv(c, u, o);
    }
    /* the word the chain stopped in, if it is still inside the region */
    if (mask && (u.p >> 5) < (p0 >> 5) + c->sw) mask[u.a] = mlo;
    *count = n;
    return u.p < c->bt ? u.p : c->bt;
}

/* Overlap (c->G > 0).  Region r's chain C_r starts G bits before the
 * region, at s = R - G, so that it has usually merged with its left
 * neighbour's chain before the region starts: the head decode runs from s
 * to y, C_r's first boundary at or past R, and records C_r's boundaries in
 * [s, R) as bits of *head (bit i <=> a symbol starts at s + i).  Pass 1 then
 * counts C_r from y, exactly as a chain started at y (so counts, masks and
 * walks keep the offset-0 semantics with R's entry point y instead of R). */
#ifndef HH_GMAX
#define HH_GMAX 64u           /* largest overlap (k_walk stages G bits before a region) */
#endif
HH_HD uint32_t hh_region_head(const hh_ctx *c, uint32_t s, uint32_t R, uint64_t *head) {
    uint64_t h = 0;
    hh_cur u = hh_cur_at(c, s);
    while (u.p < R && u.p < c->bt) {
        hh_look L = hh_lookup_w(c, u.p, hh_cur_win(u));
        const uint32_t o = hh_first_ge(L, R - u.p);     /* first start >= R, or nb */
        h |= (uint64_t)(L.bm & hh_lowmask(o)) << (u.p - s);
        hh_cur_adv(c, u, o);
    }
    if (head) *head = h;
    return u.p < c->bt ? u.p : c->bt;
}

/* Round 1's boundary-mask merge test and mask walk (below) are no longer on
 * the kernels' path (k_front merges on exit == entry, k_walk compares exits);
 * the emulator keeps them as the reference those are checked against, lane
 * by lane, and k_front's walks with HH_FRONT_WALK > 0 use hh_walk's
 * two-pointer mode.
 *
 * The left chain C_j and the right chain C_{j+1} share a boundary in the
 * overlap window [R - G, R) (R = the start of region j+1) iff C_j's mask
 * bits there meet C_{j+1}'s head bits: then the chains are identical from
 * that boundary on, C_j's exit is C_{j+1}'s entry point y, and the walk
 * from C_j's exit merges at once (k = 1, delta = 0). */
HH_HD bool hh_window_merge(const hh_ctx *c, const uint32_t *mask, uint64_t head_next, uint32_t R) {
    uint64_t mine = 0;
    for (uint32_t w = 0; w < c->G / 32; w++)
        mine |= (uint64_t)mask[hh_idx(c, (R - c->G) / 32 + w + 2)] << (32 * w);
    return (mine & head_next) != 0;
}

/* Symbols of a region's own chain that start before region offset off
 * (popcount of its mask below off). */
HH_HD uint32_t hh_mask_rank(const hh_ctx *c, const uint32_t *mask, uint32_t R, uint32_t off) {
    uint32_t cnt = 0, a = hh_idx(c, (R >> 5) + 2);
    for (uint32_t w = 0; w < (off >> 5); w++) {
        cnt += hh_popc(mask[a]);
        a = hh_idx_next(c, a);
    }
    return cnt + hh_popc(mask[a] & hh_lowmask(off & 31));
}

/* Pass 2 (makebigtable restated).  The chain W leaving region j at its
 * exit x is followed region by region.  In region r (r = j+1, ...) W is
 * tested against r's own offset-0 chain C_r:
 *   - with C_r's boundary mask (regions of this tile): each table step of W
 *     tests its symbol starts against the mask -- the first common start is
 *     the merge;
 *   - without a mask (regions of the next tile): two pointers, the one
 *     behind moves to its first boundary at or past min(other, region end).
 * W reaching its first boundary at or past the region end equal to C_r's
 * exit x_r is a merge there too.  Otherwise region r is COVERED by W, which
 * carries on into region r+1 (up to HH_KM regions).  Any common boundary is
 * a valid merge point: after it the chains are identical, so counts taken
 * there are exact.
 *   k     regions crossed (1 = merged in region j+1), 0 = no merge
 *   e     W's first boundary in the merge region, as an offset from its start
 *   cov   W's symbols from x up to that boundary (the covered regions)
 *   delta W's symbols from there to the merge minus C's symbols before it
 * mask/xs/ns (may be null): masks, exits and counts of regions < nmask.
 * ys (may be null): entry points y of the own chains of regions < nys (the
 * pass-1 heads), so that two-pointer walks need not decode the heads again.
 * maxit < HH_WALK_MAX bounds the lookups: a walk cut there returns more = 1
 * (the front kernel defers it to k_walk, which walks again from x). */
typedef struct {
    uint32_t k, e, cov;
    int32_t delta;
    uint32_t more;   /* 1: stopped after maxit steps, not finished (k == 0) */
    uint32_t steps;  /* table lookups the walk took */
} hh_wk;

HH_HD hh_wk hh_walk(const hh_ctx *c, uint32_t j, uint32_t S, uint32_t x,
                    const uint32_t *mask = nullptr, const uint32_t *xs = nullptr,
                    const uint16_t *ns = nullptr, uint32_t nmask = 0,
                    uint32_t maxit = HH_WALK_MAX, const uint32_t *ys = nullptr,
                    uint32_t nys = 0) {
    hh_wk r = {0u, 0u, 0u, 0, 0u, 0u};
    const uint32_t bt = c->bt;
    uint32_t A = x < bt ? x : bt;
    int32_t ca = 0;
    uint32_t it = 0;
    hh_cur u = {0u, 0u, 0u, 0u, 0u};
    uint32_t ml = 0, mh = 0;
    bool cur_ok = false;
    for (uint32_t k = 1; k <= HH_KM; k++) {
        const uint32_t rg = j + k;
        const uint32_t R = rg * S;
        const uint32_t Ec = R + S < bt ? R + S : bt;
        const int32_t ca0 = ca;
        const uint32_t e = A > R ? A - R : 0u;   /* A == bt <= R: stream ended */
        if (mask && rg < nmask) {
            /* chain cursor, with the mask words p>>5 and p>>5 + 1 (at LDS
             * indices u.a and the next, see hh_region_count) in registers */
            if (!cur_ok) {
                u = hh_cur_at(c, A);
                ml = mask[u.a];
                mh = mask[hh_idx_next(c, u.a)];
                cur_ok = true;
            }
            for (; u.p < Ec && it < maxit; it++) {
                const uint32_t win = hh_cur_win(u);
                const uint32_t m = c->l1m[win & (HH_L1_SIZE - 1u)];
                uint32_t lns = HH_M_NSYM(m), lnb = HH_M_NBITS(m), lbm = HH_M_BMASK(m);
                if (lns == 0) {
                    uint32_t sy;
                    lnb = hh_escape(c, u.p, win, m, &sy);
                    lns = 1;
                    lbm = 1;
                }
                const uint32_t hit = lbm & hh_funnel(mh, ml, u.p & 31) & hh_lowmask(Ec - u.p);
                if (hit) {
                    const uint32_t t = hh_ctz(hit);
                    ca += (int32_t)hh_popc(lbm & hh_lowmask(t));
                    r.k = k;
                    r.e = e;
                    r.cov = (uint32_t)ca0;
                    r.delta = (ca - ca0) - (int32_t)hh_mask_rank(c, mask, R, u.p - R + t);
                    r.steps = it + 1;
                    return r;
                }
                uint32_t adv = lnb;
                if (u.p + lnb <= Ec) {
                    ca += (int32_t)lns;
                } else {
                    adv = lbm & ~hh_lowmask(Ec - u.p) ? hh_ctz(lbm & ~hh_lowmask(Ec - u.p)) : lnb;
                    ca += (int32_t)hh_popc(lbm & hh_lowmask(adv));
                }
                const bool cross = ((u.p + adv) >> 5) != (u.p >> 5);
                hh_cur_adv(c, u, adv);
                const uint32_t nm = mask[hh_idx_next(c, u.a)];
                ml = cross ? mh : ml;
                mh = cross ? nm : mh;
            }
            A = u.p < bt ? u.p : bt;
            const uint32_t xr = xs[rg] < bt ? xs[rg] : bt;
            if (A == xr) {                  /* merged at the region's exit */
                r.k = k;
                r.e = e;
                r.cov = (uint32_t)ca0;
                r.delta = (ca - ca0) - (int32_t)ns[rg];
                r.steps = it;
                return r;
            }
        } else {
            /* the region's own chain, entered at its entry point: the
             * next tile's region 0 starts at R, the others G bits early */
            uint32_t B = R < bt ? R : bt;
            if (rg < nys) B = ys[rg] < bt ? ys[rg] : bt;
            else if (c->G && rg % HH_NR != 0 && R < bt) B = hh_region_head(c, R - c->G, R, nullptr);
            int32_t cb = 0;
            for (; it < maxit; it++) {
                if (A == B) {
                    r.k = k;
                    r.e = e;
                    r.cov = (uint32_t)ca0;
                    r.delta = (ca - ca0) - cb;
                    r.steps = it;
                    return r;
                }
                const bool mvA = A < B;
                const uint32_t P = mvA ? A : B, Q = mvA ? B : A;
                if (P >= Ec) break;              /* both past the region end */
                const uint32_t tgt = Q < Ec ? Q : Ec;
                hh_look L = hh_lookup(c, P);
                const uint32_t o = hh_first_ge(L, tgt - P);
                const int32_t n = (int32_t)hh_syms_before(L, o);
                uint32_t np = P + o;
                if (np > bt) np = bt;
                if (mvA) { A = np; ca += n; } else { B = np; cb += n; }
            }
        }
        if (it >= maxit) break;
    }
    r.more = it >= maxit && maxit < HH_WALK_MAX;
    r.steps = it;
    return r;   /* k == 0: failed (or, with more, not finished yet) */
}

/* The deferred walks (k_walk): the chain W leaving region j at x, followed
 * region by region to its exit only.  W meets region r's own chain C_r iff
 * their exits from r coincide (a shared boundary makes the chains identical
 * from there on; equal exits are a shared boundary), and then W's symbols
 * in r minus C_r's symbols in r equal their difference before the first
 * shared boundary -- so the result is hh_walk's (k, e, cov, delta), given
 * each region's pass-1 exit xr[k] and count nr[k] (k = 1..HH_KM: region
 * j+k).  Every lookup is a cursor step (no second pointer, no heads). */
HH_HD hh_wk hh_walk_exits(const hh_ctx *c, uint32_t j, uint32_t S, uint32_t x, const uint32_t *xr,
                          const uint32_t *nr) {
    hh_wk r = {0u, 0u, 0u, 0, 0u, 0u};
    const uint32_t bt = c->bt;
    uint32_t A = x < bt ? x : bt, ca = 0;
    for (uint32_t k = 1; k <= HH_KM; k++) {
        const uint32_t R = (j + k) * S;
        const uint32_t Ec = R + S < bt ? R + S : bt;
        const uint32_t e = A > R ? A - R : 0u;
        uint32_t n = 0;
        if (A < Ec) A = hh_region_count(c, A, Ec, &n);
        const uint32_t xk = xr[k] < bt ? xr[k] : bt;
        if (A == xk) {
            r.k = k;
            r.e = e;
            r.cov = ca;
            r.delta = (int32_t)n - (int32_t)nr[k];
            return r;
        }
        ca += n;
    }
    return r;   /* k == 0: no merge within HH_KM regions */
}

/* ------------------------------------------------------------------ */
/* Tile transfer table.  The state entering a tile is (d, e, delta):    */
/* regions 0..d-1 are covered by the previous tile's last walk, the     */
/* first live region d is entered e bits past its start, and delta is   */
/* that walk's correction.  Lane j is live for entering d iff d <= j    */
/* and no live walk covers it; its charged count is n + cov + delta.    */
/* For every d in [0, HH_KM) the table gives the charged count of the   */
/* tile's live lanes and the state leaving the tile (from its last live */
/* lane, the one whose walk crosses the tile end).                      */
/* ------------------------------------------------------------------ */
#define HH_DEL_BITS 10
HH_HD uint32_t hh_state_pack(uint32_t d, uint32_t e, int32_t delta) {
    return (d & 0xfu) | ((e & 0x7fu) << 4) | (((uint32_t)delta & ((1u << HH_DEL_BITS) - 1u)) << 11);
}
HH_HD uint32_t hh_state_d(uint32_t s) { return s & 0xfu; }
HH_HD uint32_t hh_state_e(uint32_t s) { return (s >> 4) & 0x7fu; }
HH_HD int32_t hh_state_delta(uint32_t s) {
    return (int32_t)(s << (32 - 11 - HH_DEL_BITS)) >> (32 - HH_DEL_BITS);
}
/* table entry: charged count (signed 20 bits) | state << 20 */
HH_HD uint64_t hh_tab_pack(int32_t count, uint32_t state) {
    return (uint64_t)((uint32_t)count & 0xfffffu) | ((uint64_t)state << 20);
}
HH_HD int32_t hh_tab_count(uint64_t v) { return (int32_t)((uint32_t)v << 12) >> 12; }
HH_HD uint32_t hh_tab_state(uint64_t v) { return (uint32_t)(v >> 20) & 0x1fffffu; }

/* Live masks: bit d of mem[j] <=> lane j is live for entering d.  The
 * exceptions (k > 1), in ascending lane order, clear the lanes they cover
 * for the entering states that reach them. */
HH_HD uint32_t hh_mem_init(uint32_t j) { return j < HH_KM - 1 ? (2u << j) - 1u : (1u << HH_KM) - 1u; }

/* Pass 3 (calcresult restated), one step of a lane's emission: the run is
 * [p, pe) on the true chain (pe a boundary of it, or bt), the output window
 * ends at whi.  Takes a whole lookup when it fits both, else one symbol
 * (with the tail rule at bt).  Returns the symbols taken (k) in *val (first
 * in bits 0..7) and the bits advanced. */
HH_HD uint32_t hh_emit_step(const hh_ctx *c, hh_cur &u, uint32_t pe, uint64_t o, uint64_t whi,
                            uint32_t *val, uint32_t *k) {
    const uint32_t p = u.p;
    hh_look L = hh_lookup_w(c, p, hh_cur_win(u));
    uint32_t adv;
    if (p + L.nb <= pe && o + L.ns <= whi) {
        *val = L.syms;
        *k = L.ns;
        adv = L.nb;
    } else {
        adv = L.len0;
        uint32_t s = L.syms & 0xffu;
        if (adv > c->bt - p) {
            s = hh_tail_symbol(c, p);
            adv = c->bt - p;
        }
        *val = s;
        *k = 1;
    }
    hh_cur_adv(c, u, adv);
    return adv;
}

/* ------------------------------------------------------------------ */
/* Cross-tile granules (64-bit, status in bits 62..63, 0 = not yet).   */
/*   aggregate (status 1): the table entry for d = 0, bit 61 CONST: the  */
/*     leaving state is the same for every entering d.                   */
/*   inclusive (status 2): bits 0..39 charged prefix through the tile,   */
/*     bits 40..60 the tile's resolved leaving state.                    */
/* ------------------------------------------------------------------ */
#define HH_ST_SHIFT 62
#define HH_AGG (1ull << 62)
#define HH_INC (2ull << 62)
#define HH_CST (1ull << 61)
#define HH_INC_MASK ((1ull << 40) - 1ull)

HH_HD uint64_t hh_inc_pack(uint64_t prefix, uint32_t state) {
    return HH_INC | (prefix & HH_INC_MASK) | ((uint64_t)state << 40);
}
HH_HD uint32_t hh_inc_state(uint64_t g) { return (uint32_t)(g >> 40) & 0x1fffffu; }
/* the prefix, sign-extended (a segment's virtual predecessor carries the
 * entry correction, which may be negative) */
HH_HD uint64_t hh_inc_prefix(uint64_t g) { return (uint64_t)((int64_t)(g << 24) >> 24); }

/* Overlap G for a tree (hh_region_head): 64 bits when that keeps chain
 * starts on the code-length lattice (a multiple of the length gcd); none
 * for a fixed-length code (its chains sit on one lattice and merge at
 * once). */
#ifndef HH_OVERLAP_BITS
#define HH_OVERLAP_BITS 64u
#endif
HH_HD uint32_t hh_pick_overlap(const hh_tables *t) {
    const uint32_t g = t->len_gcd > 0 ? (uint32_t)t->len_gcd : 1u;
    return t->fixed_len > 0 || HH_OVERLAP_BITS % g ? 0u : HH_OVERLAP_BITS;
}

/* Region size for a code whose lengths are all multiples of g: a multiple
 * of 32 (whole words per region column) and of g (region starts on the
 * code lattice, or chains of fixed-length codes could never meet), near
 * 256 bits.  0 if none fits HH_SW_MAX words. */
HH_HD uint32_t hh_pick_region_bits(uint32_t g) {
    if (g == 0) g = 1;
    uint32_t a = 32, b = g;
    while (b) { uint32_t t = a % b; a = b; b = t; }
    uint32_t l = 32 / a * g;          /* lcm(32, g) */
    if (l > 32 * HH_SW_MAX) return 0;
    uint32_t S = l;
    while (S + l <= 256) S += l;
    if (S < 128 && S + l <= 32 * HH_SW_MAX) S += l;
    return S;
}

#endif
