/*
 * hh_fsm_algo.h -- per-lane building blocks of the state-machine decode
 * (tables: hh_fsm.h).  __host__ __device__: the kernels (hh_fsm.hip) use
 * them on their rare paths (the stream's last tiles, chains that meet late),
 * and the test-only emulator (tests/emu/hh_emu.cpp) runs the whole tile
 * decomposition with them on the host, against the oracle.
 *
 * Restatement of the reference pipeline (ReleaseCL/kernels/ *.cl) in O(N):
 *
 *  decodeallbits  -> lane j runs the state machine over its region of S bits
 *                    from a GUESSED entering state: the state reached by a
 *                    chain started at the root G bits before the region (a
 *                    code boundary there is the usual case, and chains
 *                    self-synchronise), the root for a tile's region 0.
 *                    It counts the codes completed in the region and ends in
 *                    the region's exit state.
 *  makebigtable   -> the exit state of region j is the true entering state
 *                    of region j+1 (region 0 of a tile: the previous tile's).
 *                    Where it differs from region j+1's guess, lane j WALKS:
 *                    it runs both chains over region j+1 until their states
 *                    are equal at the same position -- from there on they
 *                    are the same chain -- and the difference of their
 *                    counts up to that point corrects region j+1's count.
 *                    A walk that does not meet within its region leaves a
 *                    wrong exit state behind; the regions after it are
 *                    recomputed from the true state until the recorded
 *                    entering state is right again (fsm_fix, rare).
 *  calcbitsindex  -> output index of every region: prefix sum of the counts.
 *  calcresult     -> each lane runs the state machine over its region again
 *                    from the true entering state, emitting the symbols.
 *  findmax        -> the total of the prefix sum.
 *
 * Chain semantics follow decodeallbits.cl:10-33: a code completes at the bit
 * where the walk from the root reaches a leaf; a code cut off by the end of
 * the stream is the last symbol, with the sym byte of the node reached (the
 * tail rule): a chain that is not at the root at the end of the stream adds
 * one symbol there.  A region owns the codes that COMPLETE in it (positions
 * R < end <= R + S); the stream end caps every region.
 */
#ifndef HH_FSM_ALGO_H_
#define HH_FSM_ALGO_H_

#include <stdint.h>
#include "hh_fsm.h"
#include "hh_internal.h"

#if defined(__HIPCC__)
#define HH_FD __host__ __device__ __forceinline__
#else
#define HH_FD static inline
#endif

#define HH_FSM_KM 8           /* regions a late meeting may be followed into */
#ifndef HH_FSM_GMAX
#define HH_FSM_GMAX 128       /* longest head (bits) */
#endif

/* Head bits G (the guess of a region's entering state starts at the root G
 * bits before it): whole count steps (cb bits), on the code-length lattice
 * (a multiple of the gcd of the code lengths: a chain started off it never
 * meets the true one), at most HH_FSM_GMAX and the region bits S; none for
 * a fixed-length code (regions start on its lattice, where the root is
 * always right).  On kjv a 64-bit head leaves 6.7 % of the guesses wrong, a
 * 128-bit head 0.3 %: a wave walks only in 15 % of its tiles. */
HH_FD uint32_t hh_fsm_pick_head(const hh_tables *t, uint32_t S, uint32_t cb) {
    if (t->fixed_len > 0) return 0u;
    const uint32_t g = t->len_gcd > 0 ? (uint32_t)t->len_gcd : 1u;
    uint32_t a = cb, b = g;
    while (b) { const uint32_t x = a % b; a = b; b = x; }
    const uint32_t l = cb / a * g;                 /* lcm(cb, g) */
    const uint32_t gmax = S < HH_FSM_GMAX ? S : HH_FSM_GMAX;   /* (within the region before) */
    return l > gmax ? 0u : gmax / l * l;
}

/* Region bits of the state machine for a tree of ns states whose code
 * lengths share the gcd g: S_default (the byte-stepped default) for ns <=
 * HH_FSM_MAXS8; HH_FSM_S7 (7-bit count steps) for larger trees, when it is
 * on the code lattice; 0: none. */
HH_FD uint32_t hh_fsm_region_bits(uint32_t ns, uint32_t g, uint32_t S_default) {
    if (ns <= HH_FSM_MAXS8) return S_default;
    if (ns > HH_FSM_MAXS) return 0u;
    return g == 0 || HH_FSM_S7 % g == 0 ? HH_FSM_S7 : 0u;
}

typedef struct {
    const uint16_t *ct;      /* cb-bit steps: next << (cb + 1) | completed */
    const uint32_t *b1;      /* 1-bit steps: next | completed << 8 | sym << 16 */
    const uint8_t *tsym;     /* tail-rule symbol of a state */
    uint32_t cb;             /* count step bits (8 or 7) */
} hh_fsm_view;

/* stream bits [p, p + n), n <= 25, p + n <= the readable bits (the word
 * after p's is read only when the bits reach into it) / a single bit */
HH_FD uint32_t fsm_win(const uint32_t *w, uint64_t p, uint32_t n) {
    const uint32_t o = (uint32_t)(p & 31), lo = w[p >> 5] >> o;
    const uint32_t v = o + n > 32 ? lo | (w[(p >> 5) + 1] << (32 - o)) : lo;
    return v & ((1u << n) - 1u);
}
HH_FD uint32_t fsm_bit(const uint32_t *w, uint64_t p) { return (w[p >> 5] >> (p & 31)) & 1u; }

/* The state machine from state s over stream bits [p, e): whole count steps
 * (cb bits, at any position: a step's result does not depend on where codes
 * start), then single bits.  *n += the codes completed. */
HH_FD uint32_t fsm_run(const hh_fsm_view *F, const uint32_t *w, uint64_t p, uint64_t e, uint32_t s,
                       uint32_t *n) {
    uint32_t c = 0;
    const uint32_t cb = F->cb;
    while (p + cb <= e) {
        const uint32_t v = F->ct[(s << cb) | fsm_win(w, p, cb)];
        s = HH_FSM_CT_NEXT(v, cb);
        c += HH_FSM_CT_CNT(v);
        p += cb;
    }
    while (p < e) {
        const uint32_t v = F->b1[s * 2 + fsm_bit(w, p)];
        s = v & 255u;
        c += (v >> 8) & 255u;
        p++;
    }
    *n += c;
    return s;
}

/* A region [R, Re) of a stream of `bits` bits entered in state s: its count
 * (codes completing in it, plus the tail-rule symbol when the stream ends
 * inside it) and its exit state. */
HH_FD uint32_t fsm_region(const hh_fsm_view *F, const uint32_t *w, uint64_t R, uint64_t Re, uint64_t bits,
                          uint32_t s, uint32_t *n) {
    const uint64_t e = Re < bits ? Re : bits;
    *n = 0;
    if (R >= e) return s;
    s = fsm_run(F, w, R, e, s, n);
    if (Re >= bits && s != 0) *n += 1;
    return s;
}

/* Two chains in states *A and *B over the region [R, Re) (capped by the
 * stream end): stepped together, a count step at a time (a bit at a time
 * past the last whole step), until they are in the same state at the same
 * position.  Returns 1 if they met; *d += (A's codes - B's codes) up to
 * there, or over the whole region (tail rule included) if they did not. */
HH_FD int fsm_walk2(const hh_fsm_view *F, const uint32_t *w, uint64_t R, uint64_t Re, uint64_t bits,
                    uint32_t *A, uint32_t *B, int32_t *d) {
    const uint64_t e = Re < bits ? Re : bits;
    const uint32_t cb = F->cb;
    uint32_t a = *A, b = *B;
    int32_t dd = 0;
    uint64_t p = R;
    while (p < e && a != b) {
        uint32_t va, vb;
        if (p + cb <= e) {
            const uint32_t x = fsm_win(w, p, cb);
            va = F->ct[(a << cb) | x];
            vb = F->ct[(b << cb) | x];
            p += cb;
            dd += (int32_t)HH_FSM_CT_CNT(va) - (int32_t)HH_FSM_CT_CNT(vb);
            a = HH_FSM_CT_NEXT(va, cb);
            b = HH_FSM_CT_NEXT(vb, cb);
            continue;
        } else {
            const uint32_t x = fsm_bit(w, p);
            va = F->b1[a * 2 + x];
            vb = F->b1[b * 2 + x];
            p++;
            dd += (int32_t)((va >> 8) & 255u) - (int32_t)((vb >> 8) & 255u);
        }
        a = va & 255u;
        b = vb & 255u;
    }
    const int met = a == b;
    if (!met && Re >= bits && R < bits) dd += (int32_t)(a != 0) - (int32_t)(b != 0);
    *A = a;
    *B = b;
    *d += dd;
    return met;
}

/* Emission of a region [R, Re) entered in state s, bit-serial (the rare
 * paths; the kernels' fast path takes K-bit steps): the symbols to out[],
 * the tail-rule symbol when the stream ends inside the region.  Returns the
 * symbols written. */
HH_FD uint32_t fsm_emit_serial(const hh_fsm_view *F, const uint32_t *w, uint64_t R, uint64_t Re,
                               uint64_t bits, uint32_t s, uint8_t *out) {
    const uint64_t e = Re < bits ? Re : bits;
    uint32_t o = 0;
    for (uint64_t p = R; p < e; p++) {
        const uint32_t v = F->b1[s * 2 + fsm_bit(w, p)];
        s = v & 255u;
        if ((v >> 8) & 255u) out[o++] = (uint8_t)(v >> 16);
    }
    if (R < e && Re >= bits && s != 0) out[o++] = F->tsym[s];
    return o;
}

/* Record of a region for the emission pass: entering state | count << 8. */
HH_FD uint32_t fsm_rec(uint32_t ent, uint32_t cnt) { return ent | (cnt << 8); }
HH_FD uint32_t fsm_rec_ent(uint32_t r) { return r & 255u; }
HH_FD uint32_t fsm_rec_cnt(uint32_t r) { return r >> 8; }

/* Correction of a region of the NEXT tile, written by the tile before it
 * when its true exit state differs from that tile's assumption (the root):
 * valid | true entering state << 1 | (count correction, 16-bit) << 16. */
HH_FD uint32_t fsm_fx(uint32_t ent, int32_t d) { return 1u | (ent << 1) | ((uint32_t)d << 16); }
HH_FD uint32_t fsm_fx_ok(uint32_t f) { return f & 1u; }
HH_FD uint32_t fsm_fx_ent(uint32_t f) { return (f >> 1) & 255u; }
HH_FD int32_t fsm_fx_d(uint32_t f) { return (int32_t)f >> 16; }

/* The chain leaving tile t in state x (its true exit) against tile t+1's
 * assumption (region 0 entered in state h -- the head guess, from the root G
 * bits before the tile -- each later region in the state its predecessor
 * left it in): followed region by region from tile t+1's start until they
 * meet.  fx[r] (r < HH_FSM_KM) receives the corrections of tile t+1's
 * regions; returns 0 if they did not meet within HH_FSM_KM regions.  T1 =
 * tile t+1's first bit, S region bits. */
HH_FD int fsm_fix_next(const hh_fsm_view *F, const uint32_t *w, uint64_t T1, uint32_t S, uint64_t bits,
                       uint32_t x, uint32_t h, uint32_t *fx) {
    for (int r = 0; r < HH_FSM_KM; r++) fx[r] = 0;
    uint32_t a = x, b = h;
    for (int r = 0; r < HH_FSM_KM; r++) {
        const uint64_t R = T1 + (uint64_t)r * S;
        if (a == b || R >= bits) return 1;   /* met, or past the end: nothing more to correct */
        const uint32_t ent = a;
        int32_t d = 0;
        fsm_walk2(F, w, R, R + S, bits, &a, &b, &d);   /* (not met: a, b enter region r+1) */
        fx[r] = fsm_fx(ent, d);
    }
    return a == b;
}

#endif
