// hh_one.hip -- the single-pass state-machine decode (gfx950): ONE launch,
// the payload read once, each symbol decoded by one table walk.
//
// The reference decodes speculatively from every bit (decodeallbits.cl:10-33)
// and resolves which speculative chain is the true one by pointer doubling
// (makebigtable.cl:10-40, calcbitsindex.cl:5-22) before it scatters the
// symbols it already decoded (calcresult.cl:14-16).  The same here, in O(N):
//
//   * decodeallbits -> heads + speculative emission.  A tile is 64 regions of
//     S bits, lane j owns region j.  Lane j guesses the state entering region
//     j+1 by a chain from the root over the last G bits of its own region
//     (hh_fsm_pick_head; the emission table's K-bit steps, row only), and
//     every lane emits its region from the guess made for it -- each step's
//     symbols go to the lane's own column in LDS (dword k of lane j at
//     column row k: conflict-free stores).  The symbol count and the exit
//     state fall out of the same lookups; there is no count pass.
//   * makebigtable -> fix rounds.  Where lane j-1's exit differs from lane
//     j's guess, lane j emits its region again from that exit (its column
//     overwritten); a round that changes an exit is followed by another
//     (the chains of a resynchronising code meet within a region or two;
//     ONE_RMAX rounds bound it -- beyond, the decode is handed to the
//     two-pass pipeline).
//   * calcbitsindex / findmax -> a decoupled look-back.  The tile publishes
//     (its lane-0 guess, its exit state, its symbol count) as one epoch-tagged
//     64-bit word, then reads its predecessors' words: a run of published
//     aggregates whose exits and guesses chain up to an inclusive word gives
//     the tile's true entry state and output base.  Lane 0's guess wrong
//     (about 1 % of tiles): lane 0 emits again from the true entry, the fix
//     rounds follow.  The tile then publishes its inclusive word (exit state,
//     base + count).
//   * calcresult -> the wave's prefix of the lanes' counts places every
//     lane's run: the columns are read into registers and written back into
//     the same LDS as the tile's contiguous output (aligned dwords; a dword
//     two runs share is ORed), which the wave copies out with 16-B stores.
//
// Tiles go to waves in order: each workgroup claims blocks of NB consecutive
// tiles from a device-scope counter (one block ahead), its waves take the
// block's tiles one at a time from an LDS ticket -- a tile's predecessors are
// always held by running waves, so the look-back never waits on a tile no
// wave will decode (whatever the residency of the grid).  Every wait is
// bounded (ONE_SPIN polls): a wait that runs out marks the decode for the
// two-pass pipeline instead of hanging the GPU.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "hh_fsm_kern.h"

#define ONE_WMAX 16           // waves per workgroup at most
#define ONE_RING 32           // local block -> global block map (LDS ring)
#define ONE_CAPMAX 32         // column dwords per lane at most (128 B)
#define ONE_RMAX 8            // fix rounds per tile before the decode is handed to the two-pass pipeline
#define ONE_SPIN (1u << 20)   // polls before a wait gives up
#define ONE_CTL 288           // LDS control block: ticket (16 B), block map ring (ONE_RING x 8 B)
#define ONE_NONE 0xffffffffu
#define FF_RETRY 4            // result flag: hand the decode to the two-pass pipeline
#define ONE_DEFAULT 0         // the single pass decodes unless HH_ONE=0 (1) / only with HH_ONE=1 (0)

// A tile's published word: epoch << 56 | kind << 54 | guess << 46 | exit << 38 | value.
// kind 1: aggregate (value: the tile's symbols, valid if the tile was entered
// in `guess`); 2: inclusive (value: the symbols up to and including the
// tile; exit exact); 3: inclusive of a failed decode.
#define ST_VMASK ((1ull << 38) - 1ull)
__device__ __forceinline__ uint64_t st_make(uint32_t epoch, uint32_t kind, uint32_t g, uint32_t x, uint64_t v) {
    return (uint64_t)epoch << 56 | (uint64_t)kind << 54 | (uint64_t)g << 46 | (uint64_t)x << 38 | (v & ST_VMASK);
}

struct OneGeo {
    uint64_t bits;        // stream length of the segment
    uint64_t nwords;      // readable payload words
    uint32_t ntiles;
    uint32_t ne;          // tiles [0, ne) end before the stream's last bit (no end checks)
    uint32_t emit_from;   // tiles before it are a prologue: decoded, nothing emitted
    uint32_t in_state;    // the state entering tile 0
    uint32_t ns, r;       // states, remainder step bits
    uint32_t gs;          // head steps (K bits each; 0: every guess the root)
    uint32_t capd;        // column dwords per lane
    uint32_t nb;          // tiles per claimed block
    uint32_t nblocks;     // blocks
    uint32_t epoch;       // this decode's tag (1..255)
    uint32_t test_retry;  // tests only (HH_TEST_ONE_RETRY=1): the decode is handed back to the two passes
};
struct OneWork {
    uint64_t *st;         // [ntiles] published words
    uint32_t *ctr;        // [2] block counters (by epoch parity)
    uint32_t *res;        // the result slot (host-mapped): [0] flags, [2..3] total, [4] leave, [5] entry
    uint64_t *dbg;        // (HH_ONE_DBG=1 at set_tree) counters, OneDbg; else null
};
// Counters of a decode (HH_ONE_DBG; hh_debug_counters): per wave in
// registers, added once at the wave's end.  Cycles: s_memtime.
enum { OD_TILES, OD_POLLS, OD_RESTARTS, OD_FIXTILES, OD_FIXROUNDS, OD_REDO0, OD_OVF, OD_RINGSPIN,
       OD_CYC_EMIT, OD_CYC_LB, OD_CYC_OUT, OD_CYC_TAKE, OD_CYC_ALL, OD_N };
// (a diagnostic build: make variant V=odbg HIPEXTRA=-DHH_ONE_DBG, run with
// HH_ONE_DBG=1; in the product build the counters compile to nothing)
#ifdef HH_ONE_DBG
struct OneDbg {
    uint64_t c[OD_N];
    __device__ __forceinline__ void inc(uint32_t i) { c[i]++; }
    __device__ __forceinline__ void stamp(bool on, uint32_t i, uint64_t &t) {
        if (on) {
            const uint64_t n = __builtin_amdgcn_s_memtime();
            c[i] += n - t;
            t = n;
        }
    }
    __device__ __forceinline__ void flush(uint64_t *dbg, uint64_t t0) {
        if (dbg && (threadIdx.x & 63u) == 0) {
            c[OD_CYC_ALL] = __builtin_amdgcn_s_memtime() - t0;
            for (uint32_t i = 0; i < OD_N; i++) atomicAdd((unsigned long long *)&dbg[i], (unsigned long long)c[i]);
        }
    }
};
#define ONE_DBG_ON(wk) ((wk).dbg != nullptr)
#else
struct OneDbg {
    __device__ __forceinline__ void inc(uint32_t) {}
    __device__ __forceinline__ void stamp(bool, uint32_t, uint64_t &) {}
    __device__ __forceinline__ void flush(uint64_t *, uint64_t) {}
};
#define ONE_DBG_ON(wk) false
#endif

// Head steps of the emission table at most: G <= HH_FSM_GMAX bits, whole steps.
__host__ __device__ constexpr uint32_t one_hs(uint32_t SW, uint32_t K) {
    return (32 * SW) / K < HH_FSM_GMAX / K ? (32 * SW) / K : HH_FSM_GMAX / K;
}

// The state a chain from the root reaches over the last gs K-bit steps (of
// at most HS) of the NW words w (the bits just before the guessed region),
// as an emission-table row.  Only the row of each entry is read (its high
// word: row | 8 x symbols, whose low bits et_addr replaces).
template <uint32_t NW, uint32_t K, uint32_t HS>
__device__ __forceinline__ uint32_t head_row(const uint32_t *w, uint32_t gs) {
    constexpr uint32_t B = 32 * NW;
    static_assert(K * HS <= B, "the head within the words");
    uint32_t h = 0;
#pragma unroll
    for (uint32_t i = 0; i < HS; i++)
        if (i >= HS - gs) h = *(lds_cu32p)(uintptr_t)(et_addr<NW, K>(h, w, B - K * (HS - i)) + 4u);
    return h & ~255u;
}

// The emission chain of one region into the lane's column: a step's symbols
// are shifted into the current dword, stored at its column row when full
// (rows 256 B apart: lane j's dword at byte 4 j of the row).  Rows past the
// column go to the wave's sink row (a region emitting more than the column
// holds is decoded again straight to HBM, one_direct).
template <uint32_t K>
struct ColChain {
    uint32_t row, wd, sh, a;
    __device__ __forceinline__ void put(uint64_t e, uint32_t sink) {
        const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
        const uint32_t u = sh + (hi & 255u);          // 8 x the symbols
        const uint64_t t = (uint64_t)lo << sh;
        const uint32_t an = (uint32_t)t | a;
        const bool full = u >= 32;
        if (full) *(lds_u32p)(uintptr_t)min(wd, sink) = an;
        a = full ? (uint32_t)(t >> 32) : an;
        wd += full ? 256u : 0u;
        sh = u & 31u;
    }
};

// Region emission from entry row row0 into the column at LDS byte address
// base: *nb the bytes (symbols), *xr the exit row.  TAIL: the region may be
// cut by the stream's end (lim readable bits; steps while whole, then bit by
// bit); at_end: the stream ends in (or at the end of) this region -- the
// reference's tail rule (decodeallbits.cl:20-31) emits the symbol of a chain
// cut mid-code.
template <uint32_t SW, uint32_t K, bool TAIL>
__device__ __forceinline__ void col_emit(const uint8_t *lds, uint32_t er_off, const uint32_t *b1, const uint8_t *ts,
                                         const uint32_t *w, uint32_t row0, uint32_t lim, bool at_end, uint32_t base,
                                         uint32_t sink, uint32_t &nb, uint32_t &xr) {
    constexpr uint32_t S = 32 * SW, r = S % K, NST = S / K, RSH = HH_FSM_ET_RSH(K);
    ColChain<K> ch;
    ch.row = row0;
    ch.wd = base;
    ch.sh = 0;
    ch.a = 0;
    if (!TAIL) {
        // step k+1's read issued before step k's store logic (k_emf's order)
        uint64_t e = *(lds_u64p)(uintptr_t)et_addr<SW, K>(ch.row, w, 0);
#pragma unroll
        for (uint32_t k = 0; k < NST; k++) {
            const uint32_t hi = (uint32_t)(e >> 32);
            uint64_t en = 0;
            if (k + 1 < NST) en = *(lds_u64p)(uintptr_t)et_addr<SW, K>(hi, w, (k + 1) * K);
            else if (r)
                en = *(lds_u64p)(uintptr_t)(er_off + (HH_FSM_ET_ROW(e) >> (HH_FSM_ET_LG(K) - r)) + (rbits<SW>(w, S - r, r) << 3));
            ch.row = HH_FSM_ET_ROW(e);
            ch.put(e, sink);
            e = en;
        }
        if (r) {
            ch.put(e, sink);
            ch.row = HH_FSM_ET_ROW(e);
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < NST; k++) {
            const uint32_t q = k * K;
            if (q + K <= lim) {
                const uint64_t e = *(const uint64_t *)(lds + ch.row + win8<SW, K>(w, q));
                ch.put(e, sink);
                ch.row = HH_FSM_ET_ROW(e);
            }
        }
        uint32_t st = ch.row >> RSH;
        for (uint32_t q = lim / K * K; q < lim; q++) {
            const uint32_t v = b1[st * 2 + rbit_dyn<SW>(w, q)];
            st = v & 255u;
            ch.put(HH_FSM_ET_MAKE((v >> 16) & 255u, 0u, (v >> 8) & 255u), sink);
        }
        ch.row = st << RSH;
    }
    if (at_end && ch.row != 0) ch.put(HH_FSM_ET_MAKE(ts[ch.row >> RSH], 0u, 1u), sink);   // the tail rule
    if (ch.sh) *(lds_u32p)(uintptr_t)min(ch.wd, sink) = ch.a;   // the last, partial dword (unused bytes zero)
    nb = (ch.wd - base) / 64u + ch.sh / 8u;          // (rows of 256 B: 4 bytes each)
    xr = ch.row;
}

// The same, out of line: the rare emissions (fix rounds, a wrong lane-0
// guess) -- kept out of the main chain's register allocation.
// (words by value: a pointer would put the caller's words in scratch)
struct ColRes {
    uint32_t nb, xr;
};
template <uint32_t SW>
struct Words {
    uint32_t v[SW];
};
template <uint32_t SW, uint32_t K, bool TAIL>
__device__ __noinline__ ColRes col_emit_rare(const uint8_t *lds, uint32_t er_off, const uint32_t *b1, const uint8_t *ts,
                                            Words<SW> w, uint32_t row0, uint32_t lim, bool at_end, uint32_t base,
                                            uint32_t sink) {
    ColRes o;
    col_emit<SW, K, TAIL>(lds, er_off, b1, ts, w.v, row0, lim, at_end, base, sink, o.nb, o.xr);
    return o;
}

// A region straight to HBM, bit by bit (a tile whose columns overflowed; rare).
template <uint32_t SW>
__device__ __forceinline__ void one_direct(const uint32_t *b1, const uint8_t *ts, const uint32_t *w, uint32_t s,
                                           uint32_t lim, bool at_end, uint8_t *dst) {
    uint32_t o = 0;
    for (uint32_t q = 0; q < lim; q++) {
        const uint32_t v = b1[s * 2 + rbit_dyn<SW>(w, q)];
        s = v & 255u;
        if ((v >> 8) & 255u) dst[o++] = (uint8_t)(v >> 16);
    }
    if (at_end && s != 0) dst[o] = ts[s];
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((long long)v, o, 64);
    return v;
}

// The look-back of tile t (t >= 1): lane i reads the word of tile k0 - i.
// v: the first window's words (the poll issued early).  Returns the state
// entering tile t, the symbols before it, and whether a predecessor failed;
// ok = 0 when the polls ran out.
//
// An aggregate of tile k is valid when k was entered in its guess, i.e. when
// tile k-1 (valid) left that state.  Scanning back from tile t-1, the words
// are taken while each aggregate's guess is the state its older neighbour
// left; the first inclusive word ends the scan.  A tile not published yet --
// or an aggregate whose guess its neighbour did not leave (that tile waits
// for its own look-back and publishes an inclusive word) -- stops the scan:
// the aggregates before it are kept (all but the last, whose link is not
// checked yet: `need`, the state the next tile scanned must leave) and the
// scan resumes there, never from t-1 again unless a kept link turns out
// broken.  A scan that ends publishes inclusive words for the aggregates of
// its last window (their prefixes are known now), so that the tiles after
// them find an inclusive word near (with ~3,000 tiles in flight, scans
// that waited for the owners' own look-backs walked thousands of tiles).
struct OneLB {
    uint32_t E, fail, ok;
    uint64_t B;
};
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ OneLB one_lookback(uint64_t *st, uint32_t t, uint32_t epoch, uint64_t v, OneDbg &dg) {
    const uint32_t j = threadIdx.x & 63u;
    uint32_t k0 = t - 1, need = ONE_NONE, E = ONE_NONE;
    uint64_t acc = 0;
    for (uint32_t spin = 0; spin < ONE_SPIN; spin++) {
        dg.inc(OD_POLLS);
        const bool in = j <= k0;
        const uint32_t kind = in && (uint32_t)(v >> 56) == epoch ? (uint32_t)(v >> 54) & 3u : 0u;
        const uint32_t gin = (uint32_t)(v >> 46) & 255u, x = (uint32_t)(v >> 38) & 255u;
        const uint64_t val = v & ST_VMASK;
        const uint32_t kn = shfl_down1(kind), xn = shfl_down1(x);   // (the tile before lane j's)
        // lane j stops the scan: not published, or an aggregate whose guess
        // its (published) older neighbour did not leave
        const bool blk = kind == 0u || (kind == 1u && j < 63u && kn != 0u && xn != gin);
        const uint64_t bm = __ballot(blk), im = __ballot(kind >= 2u);
        const uint32_t i0 = bm ? (uint32_t)__builtin_ctzll(bm) : 64u, p = im ? (uint32_t)__builtin_ctzll(im) : 64u;
        const uint32_t x0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
        const uint32_t kind0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)kind);
        if (need != ONE_NONE && kind0 != 0u && x0 != need) {
            // a kept aggregate's guess is not the state this tile left: it
            // was entered wrongly after all -- scan again from t-1
            dg.inc(OD_RESTARTS);
            acc = 0;
            need = ONE_NONE;
            E = ONE_NONE;
            k0 = t - 1;
            __builtin_amdgcn_s_sleep(2);
        } else if (p < i0) {
            // an inclusive word with every aggregate before it chaining to it
            if (E == ONE_NONE) E = x0;
            const uint64_t pre = j < p ? val : 0ull;
            uint64_t incl = pre;                      // (inclusive scan of the aggregates before p)
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint64_t y = (uint64_t)__shfl_up((long long)incl, o, 64);
                if (j >= (uint32_t)o) incl += y;
            }
            const uint64_t Tp = readlane64(incl, 63u), vp = readlane64(val, p);
            const uint32_t kp = (uint32_t)__builtin_amdgcn_readlane((int)kind, p);
            // the aggregates of this window, now inclusive (kind 3: a failure
            // behind them travels on)
            if (j < p && kind == 1u)
                __hip_atomic_store(&st[k0 - j], st_make(epoch, kp, 0u, x, vp + Tp - (incl - pre)), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            return OneLB{E, kp == 3u ? 1u : 0u, 1u, acc + vp + Tp};
        } else {
            // keep the aggregates that chain up to the stop (or the whole
            // window), the last one's link left to the next window
            const uint32_t c = i0 == 64u ? 64u : (i0 > 0u ? i0 - 1u : 0u);
            if (c > 0u) {
                if (E == ONE_NONE) E = x0;
                uint64_t s = j < c ? val : 0ull;
                acc += wave_sum64(s);
                need = (uint32_t)__builtin_amdgcn_readlane((int)gin, c - 1u);
                k0 -= c;
            } else {
                dg.inc(OD_RESTARTS);
                __builtin_amdgcn_s_sleep(2);
            }
        }
        v = j <= k0 ? __hip_atomic_load(&st[k0 - j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    }
    return OneLB{0u, 1u, 0u, 0ull};
}

// One tile t (uniform) with its words w (region j's, lane j) and pv (the 16
// bytes before the tile, uniform).  colb: the wave's column area.
// The tile's guesses (decodeallbits' heads): gn, lane j's for region j+1
// (over the last G bits of its own region), and g0, lane 0's for region 0
// (over the 16 bytes before the tile), as emission-table rows.
template <uint32_t SW, uint32_t K>
__device__ __forceinline__ void one_heads(const OneGeo &geo, uint32_t t, const uint32_t *w, const uint32_t *pv, uint32_t &gn,
                                          uint32_t &g0) {
    constexpr uint32_t RSH = HH_FSM_ET_RSH(K), HS = one_hs(SW, K);
    gn = geo.gs ? head_row<SW, K, HS>(w, geo.gs) : 0u;
    g0 = t == 0 ? geo.in_state << RSH : (geo.gs ? head_row<4, K, HS>(pv, geo.gs) : 0u);
}

// One tile t (uniform) with its words w (region j's, lane j) and its
// guesses (one_heads).  colb: the wave's column area.  between(): called
// once the tile's look-back is done, before its output is staged and
// copied out (the wave takes its next tile there and issues its loads: a
// wave holds no ticket while it may wait -- a ticket taken a tile ahead,
// by a wave then waiting in its look-back, held up the tile every later
// look-back waited for, and the decode ran tile by tile).
template <uint32_t SW, uint32_t K, bool TAIL, uint32_t COI, typename Between>
__device__ __forceinline__ void one_tile(uint8_t *smem, const OneGeo &geo, const OneWork &wk, uint8_t *__restrict__ out,
                                         uint64_t cap, uint32_t t, const uint32_t *w, uint32_t gn, uint32_t g0,
                                         uint32_t er_off, const uint32_t *b1, const uint8_t *ts, uint32_t colb, OneDbg &dg,
                                         Between between) {
    constexpr uint32_t S = 32 * SW, RSH = HH_FSM_ET_RSH(K);
    const bool don = ONE_DBG_ON(wk);
    uint64_t tdg = don ? __builtin_amdgcn_s_memtime() : 0;
    dg.inc(OD_TILES);
    const uint32_t j = threadIdx.x & 63u;
    const uint64_t TB = (uint64_t)NR * S, R = (uint64_t)t * TB + (uint64_t)j * S;
    uint32_t lim = S;
    bool at_end = R + S == geo.bits;
    if (TAIL) {
        lim = R >= geo.bits ? 0u : (geo.bits - R < S ? (uint32_t)(geo.bits - R) : S);
        at_end = R < geo.bits && R + S >= geo.bits;
    }
    const uint32_t base = colb + 4u * j, sink = colb + 256u * geo.capd + 4u * j;
    Words<SW> wv;
#pragma unroll
    for (uint32_t k = 0; k < SW; k++) wv.v[k] = w[k];

    // decodeallbits: the speculative emission from the guesses
    const uint32_t gup = shfl_up1(gn);
    uint32_t gr = j ? gup : g0;                       // the entry row of the lane's chain
    uint32_t n, x;
    col_emit<SW, K, TAIL>(smem, er_off, b1, ts, w, gr, lim, at_end, base, sink, n, x);

    // makebigtable: lanes whose predecessor left another state emit again
    // (lanes past the stream's end, TAIL, emit nothing and take no part)
    bool fail = false;
    auto fix = [&]() {
        for (uint32_t round = 0;; round++) {
            const uint32_t xm = shfl_up1(x);
            const bool bad = j > 0 && (!TAIL || lim > 0) && xm != gr;
            if (__ballot(bad) == 0) return;
            dg.inc(OD_FIXROUNDS);
            if (round == 0) dg.inc(OD_FIXTILES);
            if (round >= ONE_RMAX) {
                fail = true;
                return;
            }
            if (bad) {
                gr = xm;
                const ColRes c = col_emit_rare<SW, K, TAIL>(smem, er_off, b1, ts, wv, gr, lim, at_end, base, sink);
                n = c.nb;
                x = c.xr;
            }
        }
    };
    fix();
    const bool pro = t < geo.emit_from;              // (a prologue tile emits nothing)
    uint32_t T = pro ? 0u : (uint32_t)wave_sum((int32_t)n);
    // the state leaving the tile: lane 63's, or (TAIL) that of the lane in
    // which the stream ends
    const uint32_t xl = TAIL ? (uint32_t)std::min<uint64_t>(63u, (geo.bits - 1 - (uint64_t)t * TB) / S) : 63u;
    uint32_t x63 = (uint32_t)__builtin_amdgcn_readlane((int)x, xl) >> RSH;

    dg.stamp(don, OD_CYC_EMIT, tdg);
    // calcbitsindex: the tile's true entry and output base
    uint32_t E = g0 >> RSH;
    uint64_t B = 0;
    uint64_t *stp = wk.st;
    if (t > 0) {
        // (a tile whose fix rounds ran out publishes a failed inclusive word
        // at once: no later scan may take it for a valid aggregate)
        if (j == 0)
            __hip_atomic_store(&stp[t], fail ? st_make(geo.epoch, 3u, 0u, x63, 0u) : st_make(geo.epoch, 1u, g0 >> RSH, x63, T),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t v0 = j < t ? __hip_atomic_load(&stp[t - 1 - j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const OneLB lb = one_lookback(stp, t, geo.epoch, v0, dg);
        dg.stamp(don, OD_CYC_LB, tdg);
        B = lb.B;
        if (lb.fail || !lb.ok) fail = true;
        if (lb.ok && lb.E != E) {
            // lane 0's guess was wrong: lane 0 emits again from the true entry
            E = lb.E;
            dg.inc(OD_REDO0);
            if (j == 0) {
                gr = E << RSH;
                const ColRes c = col_emit_rare<SW, K, TAIL>(smem, er_off, b1, ts, wv, gr, lim, at_end, base, sink);
                n = c.nb;
                x = c.xr;
            }
            fix();
            T = pro ? 0u : (uint32_t)wave_sum((int32_t)n);
            x63 = (uint32_t)__builtin_amdgcn_readlane((int)x, xl) >> RSH;
        }
    }
    if (j == 0) __hip_atomic_store(&stp[t], st_make(geo.epoch, fail ? 3u : 2u, 0u, x63, B + T), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    between();
    if (j == 0 && t == geo.ntiles - 1) {
        wk.res[0] = fail || geo.test_retry ? (uint32_t)FF_RETRY : 0u;
        wk.res[2] = (uint32_t)(B + T);
        wk.res[3] = (uint32_t)((B + T) >> 32);
        wk.res[4] = x63;
        if (geo.emit_from >= geo.ntiles) wk.res[5] = geo.in_state;
    }
    if (j == 0 && t == geo.emit_from) wk.res[5] = E;
    if (pro || fail || B + T > cap) return;          // (over the capacity: the host sees total > cap)

    // calcresult: the lanes' runs placed by the wave's prefix of their counts
    const uint32_t capb = 4u * geo.capd;
    const uint32_t a0 = (uint32_t)(B & 15u);
    const bool ovf = __ballot(n > capb) != 0 || a0 + T + 8u > 64u * capb;
    const uint32_t L = (uint32_t)wave_incl_scan((int32_t)n) - n;
    if (ovf) {
        dg.inc(OD_OVF);
        // (rare) every lane's region straight to HBM from its true entry
        one_direct<SW>(b1, ts, w, gr >> RSH, lim, at_end, out + B + L);
        return;
    }
    // the columns into registers (rows up to the wave's longest run)
    uint32_t nmax = n;
#pragma unroll
    for (int oo = 32; oo > 0; oo >>= 1) nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, oo, 64));
    const uint32_t kmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)((nmax + 3u) / 4u));
    constexpr uint32_t CAPR = 4u * COI;               // (column dwords at most: one_coi)
    uint32_t v[CAPR];
#pragma unroll
    for (uint32_t k = 0; k < CAPR; k++) v[k] = k < kmax ? *(lds_u32p)(uintptr_t)(base + 256u * k) : 0u;
    WAVE_SYNC();                                      // (every lane's column read before the staging writes)
    // the tile's output, contiguous from the column area's byte a0: lane j's
    // bytes at o = a0 + L.  A dword is stored by the run holding its last byte
    // (zeros where earlier runs' bytes go); a run ending inside a dword ORs
    // its bytes in afterwards (the tile's last run stores its partial dword).
    const uint32_t o = a0 + L, e = o + n, d0 = o >> 2, sb = 8u * (o & 3u);
    const uint32_t mcnt = e / 4u > d0 ? e / 4u - d0 : 0u;   // dwords this run stores whole
    const uint64_t ne_mask = __ballot(n > 0u);
    const uint32_t lastl = ne_mask ? 63u - (uint32_t)__builtin_clzll(ne_mask) : 0u;
    uint32_t vl = 0, prev = 0;
#pragma unroll
    for (uint32_t m = 0; m <= CAPR; m++) {
        if (m <= kmax) {
            const uint32_t cur = m < CAPR ? v[m] : 0u;
            const uint32_t V = (uint32_t)((((uint64_t)cur << 32) | prev) >> (32u - sb));
            if (m < mcnt) *(lds_u32p)(uintptr_t)(colb + 4u * (d0 + m)) = V;
            vl = m == mcnt ? V : vl;
            prev = cur;
        }
    }
    const uint32_t part = e & 3u;
    vl &= (1u << (8u * part)) - 1u;                  // (part 0: nothing; the mask is 0)
    const bool tail_dw = n > 0u && part != 0u;
    if (tail_dw && j == lastl) *(lds_u32p)(uintptr_t)(colb + 4u * (e >> 2)) = vl;
    WAVE_SYNC();
    if (tail_dw && j != lastl)
        __hip_atomic_fetch_or((uint32_t *)__builtin_assume_aligned(smem + colb + 4u * (e >> 2), 4), vl, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WAVEFRONT);
    WAVE_SYNC();
    // copy-out: whole 16-B blocks through a buffer resource spanning the
    // tile's bytes [0, end) (stores past it are dropped: a compile-time
    // number of stores), the partial first and last blocks byte by byte
    uint8_t *gb = out + (B - a0);
    const uint32_t end = a0 + T;
    const bool part0 = a0 != 0 || end < 16, partl = (end & 15u) != 0 && end > 16;
    const uint32_t q = j < 16 ? j : (end & ~15u) + (j - 16);
    const bool pb = j < 32 && (j < 16 ? part0 : partl) && q >= a0 && q < end;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(gb, 0, (int)end, 0x00020000);
#pragma unroll
    for (uint32_t ii = 0; ii < COI; ii++) {
        const uint32_t lo = 16 * (j + 64 * ii);
        u32x4 vv = {0u, 0u, 0u, 0u};
        if (lo < end) vv = *(const u32x4 *)(smem + colb + lo);
        __builtin_amdgcn_raw_buffer_store_b128(vv, ors, (int)(lo >= a0 ? lo : 0x40000000u), 0, 2);
    }
    __builtin_amdgcn_raw_buffer_store_b8(smem[colb + q], ors, (int)(pb ? q : 0x40000000u), 0, 0);
    WAVE_SYNC();
    dg.stamp(don, OD_CYC_OUT, tdg);                                      // (the copy-out has read the area before the next tile's columns)
}

// The tiles in which the stream ends (at most two per decode), out of line.
// (the stream's last tile: its wave takes its next ticket after it)
template <uint32_t SW, uint32_t K, uint32_t COI>
__device__ __noinline__ void one_tile_tail(uint8_t *smem, OneGeo geo, OneWork wk, uint8_t *__restrict__ out, uint64_t cap,
                                           uint32_t t, Words<SW> w, uint32_t gn, uint32_t g0, uint32_t er_off,
                                           const uint32_t *b1, const uint8_t *ts, uint32_t colb) {
    OneDbg dg = {};
    one_tile<SW, K, true, COI>(smem, geo, wk, out, cap, t, w.v, gn, g0, er_off, b1, ts, colb, dg, [] {});
}

// k_one: the whole decode of tiles [0, ntiles).  Workgroups of nw waves (the
// LDS beside the tables holds nw column areas), one per CU.
template <uint32_t SW, uint32_t K, uint32_t COI>
__global__ __launch_bounds__(64 * ONE_WMAX) void k_one(const uint32_t *__restrict__ g, OneGeo geo, FsmTab tab, OneWork wk,
                                                       uint8_t *__restrict__ out, uint64_t cap) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t S = 32 * SW;
    const uint32_t ns = geo.ns, r = geo.r, tid = threadIdx.x, j = tid & 63u;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t er_off = (ns << HH_FSM_ET_LG(K)) * 8u;
    uint32_t *s_b1 = (uint32_t *)(smem + er_off + (r ? (ns << r) * 8u : 0u));
    uint8_t *s_ts = (uint8_t *)(s_b1 + 2 * ns);
    const uint32_t tabb = emf_tab_bytes(ns, K, r);
    const uint32_t ctl = tabb, ring = ctl + 16u, col0 = ctl + ONE_CTL;
    const uint32_t par = geo.epoch & 1u, NB = geo.nb;
    uint32_t *tkt = (uint32_t *)__builtin_assume_aligned(smem + ctl, 16);        // the ticket counter
    uint64_t *rng = (uint64_t *)__builtin_assume_aligned(smem + ring, 16);       // the block map
    lds_fill16(smem, tab.et, (ns << HH_FSM_ET_LG(K)) * 8u);
    for (uint32_t i = tid; r && i < (ns << r); i += blockDim.x) ((uint64_t *)(smem + er_off))[i] = tab.er[i];
    for (uint32_t i = tid; i < 2 * ns; i += blockDim.x) s_b1[i] = tab.b1[i];
    for (uint32_t i = tid; i < ns; i += blockDim.x) s_ts[i] = tab.tsym[i];
    if (tid < ONE_RING) rng[tid] = 0xffffffff00000000ull;
    __syncthreads();
    if (tid == 0) {
        if (!lds_base_is_zero(smem)) wk.res[0] = FF_RETRY;   // (see hh_fsm_kern.h: nothing decoded then)
        *tkt = 0u;
        const uint32_t gb = __hip_atomic_fetch_add(&wk.ctr[par], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(rng, (uint64_t)gb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (blockIdx.x == 0) __hip_atomic_store(&wk.ctr[par ^ 1u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (the next decode's)
    }
    __syncthreads();
    if (!lds_base_is_zero(smem)) return;
    const uint32_t colb = col0 + wv * 256u * (geo.capd + 1u);
    const bool don = ONE_DBG_ON(wk);
    OneDbg dg = {};
    const uint64_t t_start = don ? __builtin_amdgcn_s_memtime() : 0;

    // the next tile: a ticket from the workgroup's counter; the wave whose
    // ticket opens a local block claims the global block of the next one
    auto take = [&]() -> uint32_t {
        uint32_t u = 0;
        if (j == 0) u = __hip_atomic_fetch_add(tkt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        u = (uint32_t)__builtin_amdgcn_readfirstlane((int)u);
        const uint32_t k = u / NB, i = u - k * NB;
        if (i == 0 && j == 0) {
            const uint32_t gb = __hip_atomic_fetch_add(&wk.ctr[par], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(rng + (k + 1u) % ONE_RING, (uint64_t)(k + 1u) << 32 | gb, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        uint64_t m = 0;
        for (uint32_t spin = 0; spin < ONE_SPIN; spin++) {
            m = __hip_atomic_load(rng + k % ONE_RING, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            m = uni64(m);
            if ((uint32_t)(m >> 32) == k) break;
            dg.inc(OD_RINGSPIN);
            __builtin_amdgcn_s_sleep(1);
        }
        if ((uint32_t)(m >> 32) != k) {
            if (j == 0) wk.res[0] = FF_RETRY;         // (never expected: the claim is made before any wait)
            return ONE_NONE;
        }
        const uint32_t gb = (uint32_t)m;
        if (gb >= geo.nblocks) return ONE_NONE;
        const uint32_t tt = gb * NB + i;
        return tt < geo.ntiles ? tt : ONE_NONE;
    };
    const uint64_t TB = (uint64_t)NR * S;
    uint32_t pw[SW], ppv = 0;
    auto prefetch = [&](uint32_t tt) {
        if (tt == ONE_NONE) return;
        const uint64_t tw = (uint64_t)tt * TB / 32;
        fs_load<SW>(pw, fs_rsrc(g, tw, geo.nwords), lane_id() * SW);
        const uint64_t pa = tw >= 4 ? tw - 4 : 0u;   // (tile 0: unused)
        ppv = __builtin_amdgcn_raw_buffer_load_b32(fs_rsrc(g, pa, geo.nwords), (int)(4u * (lane_id() & 3u)), 0, 0);
    };
    // the tile loop: a tile's heads once its words are in, its emission and
    // look-back, then (between) the next ticket and its loads, then this
    // tile's output while they are in flight
    uint32_t t = take();
    prefetch(t);
    while (t != ONE_NONE) {
        uint32_t w[SW], pv[4], gn, g0;
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) w[k] = pw[k];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) pv[i] = (uint32_t)__builtin_amdgcn_readlane((int)ppv, i);
        one_heads<SW, K>(geo, t, w, pv, gn, g0);
        uint32_t tn = ONE_NONE;
        auto between = [&] {
            uint64_t tk = don ? __builtin_amdgcn_s_memtime() : 0;
            tn = take();
            prefetch(tn);
            dg.stamp(don, OD_CYC_TAKE, tk);
        };
        if (t < geo.ne) {
            one_tile<SW, K, false, COI>(smem, geo, wk, out, cap, t, w, gn, g0, er_off, s_b1, s_ts, colb, dg, between);
        } else {
            Words<SW> ww;
#pragma unroll
            for (uint32_t k = 0; k < SW; k++) ww.v[k] = w[k];
            one_tile_tail<SW, K, COI>(smem, geo, wk, out, cap, t, ww, gn, g0, er_off, s_b1, s_ts, colb);
            between();
        }
        t = tn;
    }
    dg.flush(wk.dbg, t_start);
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
typedef void (*kone_t)(const uint32_t *, OneGeo, FsmTab, OneWork, uint8_t *, uint64_t);

// (the region geometries of the state machine: 256-bit regions with 7-bit
// steps for trees of <= 127 states, 224-bit regions with 5- or 6-bit steps
// for larger ones, 4-bit steps for a tree with a 1-bit code; others keep the
// two-pass pipeline)
static kone_t kone_for(uint32_t sw, uint32_t K, uint32_t coi) {
#define ONE_K(n, k) (coi <= 4 ? k_one<n, k, 4> : coi <= 6 ? k_one<n, k, 6> : k_one<n, k, 8>)
    if (sw == 8) return K == 7 ? ONE_K(8, 7) : K == 6 ? ONE_K(8, 6) : K == 5 ? ONE_K(8, 5) : K == 4 ? ONE_K(8, 4) : nullptr;
    if (sw == 7) return K == 7 ? ONE_K(7, 7) : K == 6 ? ONE_K(7, 6) : K == 5 ? ONE_K(7, 5) : K == 4 ? ONE_K(7, 4) : nullptr;
#undef ONE_K
    return nullptr;
}
// copy-out stores per lane for a tile of less than 64 x 4 capd bytes, in the
// instantiated steps (4, 6, 8: the column registers are 4 x COI)
static uint32_t one_coi(uint32_t capd) {
    const uint32_t c = (capd + 3u) / 4u;             // (a tile's output stays below 256 capd bytes: see ovf)
    return c <= 4 ? 4u : c <= 6 ? 6u : 8u;
}

#define ONE_LDS (160u * 1024u)

// The single pass's geometry for the tables in fd: head steps, column
// dwords, waves per workgroup.  avg: expected bits per symbol; HH_ONE=0
// keeps the two-pass pipeline (experiments and tests).
void one_setup(FsmDev *fd, uint32_t G, double avg, uint32_t minlen) {
    fd->one_ok = 0;
    const char *on = getenv("HH_ONE");
    if (!fd->ok || !(on ? atoi(on) != 0 : ONE_DEFAULT)) return;
    const uint32_t sw = fd->S / 32, K = fd->K;
    if (fd->S % 32 || G % K || G > HH_FSM_GMAX) return;
    const uint32_t gs = G / K;
    if (gs > one_hs(sw, K)) return;
    // columns: 1.25 x the expected bytes of a region, at most the most a
    // region can emit (S / minlen, + the tail-rule symbol) and ONE_CAPMAX
    const double est = avg > 0.0 ? fd->S / avg : (double)fd->S;
    uint32_t capd = (uint32_t)(est * 1.25 / 4.0) + 2u;
    const uint32_t worst = (fd->S / (minlen ? minlen : 1u) + 1u + 3u) / 4u;
    if (capd > worst) capd = worst;
    if (capd > ONE_CAPMAX) capd = ONE_CAPMAX;        // (short codes: regions past the columns go straight to HBM)
    if (getenv("HH_ONE_CAPD")) capd = (uint32_t)atoi(getenv("HH_ONE_CAPD"));   // (tests: forced overflows)
    if (capd < 2u || capd > ONE_CAPMAX) return;
    const uint32_t tabb = emf_tab_bytes(fd->ns, K, fd->r);
    const uint32_t per = 256u * (capd + 1u);
    if (tabb + ONE_CTL + 4u * per > ONE_LDS) return;   // (fewer than 4 waves: the two passes)
    uint32_t nw = (ONE_LDS - tabb - ONE_CTL) / per;
    if (nw > ONE_WMAX) nw = ONE_WMAX;
    if (getenv("HH_ONE_WAVES")) nw = std::max(1u, std::min(nw, (uint32_t)atoi(getenv("HH_ONE_WAVES"))));
    if (!kone_for(sw, K, one_coi(capd))) return;
    fd->one_gs = gs;
    fd->one_capd = capd;
    fd->one_nw = nw;
    fd->one_lds = tabb + ONE_CTL + nw * per;
    fd->one_grid = 0;
    fd->one_test_retry = getenv("HH_TEST_ONE_RETRY") && atoi(getenv("HH_TEST_ONE_RETRY")) != 0;
    fd->one_dbg = getenv("HH_ONE_DBG") && atoi(getenv("HH_ONE_DBG")) != 0;   // (counters: hh_debug_counters)
    fd->one_nbm = getenv("HH_ONE_NBM") ? std::max(1, atoi(getenv("HH_ONE_NBM"))) : 1u;   // (experiments)
    fd->one_ok = 1;
}

static int one_status(FsmWs *ws, uint64_t nt, hipStream_t st) {
    // the published words (and the two block counters in front of them):
    // their own allocation, zeroed when made and when the epoch wraps
    const uint64_t need = nt + 8u;
    if (ws->st_cap < need) {
        if (ws->st) {
            FS_OK(hipDeviceSynchronize());           // (an asynchronous decode may still use it)
            FS_OK(hipFree(ws->st));
        }
        ws->st = nullptr;
        ws->st_cap = 0;
        const uint64_t cap = need + need / 8u;
        if (hipMalloc(&ws->st, cap * 8u) != hipSuccess) {
            ws->st = nullptr;
            return HH_ERR_NOMEM;
        }
        ws->st_cap = cap;
        ws->epoch = 0;
    }
    if (++ws->epoch > 255u || ws->epoch == 1u) {
        FS_OK(hipMemsetAsync(ws->st, 0, ws->st_cap * 8u, st));
        ws->epoch = 1;
    }
    return HH_OK;
}

int one_launch(FsmDev *fd, FsmWs *ws, uint32_t slot, hipEvent_t *ev, const void *d_data, uint64_t bits, uint64_t ntiles,
               uint32_t in_state, uint64_t emit_from, void *d_out, uint64_t cap, hipStream_t st, FsmPend *pd) {
    if (!fd->one_ok) return HH_ERR_UNSUPPORTED;
    if (slot >= FSM_RES_SLOTS) return HH_ERR_ARG;
    if (in_state >= fd->ns) return HH_ERR_ARG;
    const uint32_t sw = fd->S / 32;
    const uint64_t TB = (uint64_t)NR * fd->S;
    const uint64_t all = (bits + TB - 1) / TB;
    const uint64_t nt = ntiles && ntiles < all ? ntiles : all;
    if (nt == 0 || nt >= 0xffffffffull / 64u) return HH_ERR_UNSUPPORTED;
    const kone_t kf = kone_for(sw, fd->K, one_coi(fd->one_capd));
    if (!kf) return HH_ERR_UNSUPPORTED;
    if (!fd->one_grid) {
        int pe = 0, ncu = 0, dev = 0;
        FS_OK(hipGetDevice(&dev));
        FS_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pe, kf, 64 * fd->one_nw, fd->one_lds));
        FS_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        if (pe < 1) return HH_ERR_UNSUPPORTED;
        hipFuncAttributes fa;                        // (no static LDS: hh_fsm_kern.h)
        if (hipFuncGetAttributes(&fa, (const void *)kf) != hipSuccess || fa.sharedSizeBytes != 0) return HH_ERR_INTERNAL;
        fd->one_grid = (uint32_t)(pe * ncu);
    }
    int rc = one_status(ws, nt, st);
    if (rc) return rc;
    if (!ws->h_res) {
        if (hipHostMalloc((void **)&ws->h_res, FSM_RES_SLOTS * 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            ws->h_res = nullptr;
            return HH_ERR_NOMEM;
        }
        FS_OK(hipHostGetDevicePointer((void **)&ws->d_res, ws->h_res, 0));
    }
    OneGeo geo;
    geo.bits = bits;
    geo.nwords = ((bits + 7) / 8 + HH_PAYLOAD_PAD) / 4;
    geo.ntiles = (uint32_t)nt;
    geo.ne = (uint32_t)std::min<uint64_t>(bits / TB, nt);
    geo.emit_from = (uint32_t)std::min<uint64_t>(emit_from, nt);
    geo.in_state = in_state;
    geo.ns = fd->ns;
    geo.r = fd->r;
    geo.gs = fd->one_gs;
    geo.capd = fd->one_capd;
    // a claimed block is one round of the workgroup's waves: a tile's
    // predecessor is then decoded beside it, not rounds later (blocks of
    // 4 rounds made every workgroup's first round wait for the last round of
    // the workgroup before it: the decode ran tile by tile)
    geo.nb = fd->one_nbm * fd->one_nw;
    geo.nblocks = (uint32_t)((nt + geo.nb - 1) / geo.nb);
    geo.epoch = ws->epoch;
    geo.test_retry = fd->one_test_retry;
    OneWork wk;
    wk.ctr = (uint32_t *)ws->st;
    wk.st = ws->st + 8;
    wk.res = ws->d_res + 16 * slot;
    wk.dbg = fd->one_dbg ? fd->dbg : nullptr;
    if (wk.dbg) FS_OK(hipMemsetAsync(wk.dbg, 0, 16 * sizeof(uint64_t), st));
    FsmTab tab = {fd->ct, fd->b1, fd->tsym, fd->et, fd->er};
    const uint32_t grid = (uint32_t)std::min<uint64_t>(fd->one_grid, geo.nblocks);
    // (the slot's flags word: the kernel only ever sets it)
    memset((void *)(ws->h_res + 16 * slot), 0, 64);
    FS_OK(hipEventRecord(ev[0], st));
    hipLaunchKernelGGL(kf, dim3(grid), dim3(64 * fd->one_nw), fd->one_lds, st, (const uint32_t *)d_data, geo, tab, wk,
                       (uint8_t *)d_out, cap);
    FS_OK(hipGetLastError());
    FS_OK(hipEventRecord(ev[3], st));
    pd->phases = 0;
    pd->nt = nt;
    pd->emit_from = emit_from;
    pd->cap = cap;
    pd->slot = slot;
    pd->test_nosync = fd->test_nosync;
    pd->one = 1;
    return HH_OK;
}
