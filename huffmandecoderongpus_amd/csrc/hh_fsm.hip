// hh_fsm.hip -- the state-machine decode (gfx950), the decoder's main path.
//
// Three kernels on one stream (tables and per-lane rules: hh_fsm.h,
// hh_fsm_algo.h):
//
//   k_cnt     one tile (64 regions of S bits) per WAVE, persistent grid:
//             lane j holds region j's words and region j+1's in registers;
//             (decodeallbits) the guess for region j+1 from a G-bit head,
//             the region's count and exit state in 8-bit steps of the count
//             table; (makebigtable) walks where an exit state differs from
//             the next region's guess, repeated while a walk does not meet
//             within its region; the next tile's corrections (lane 63);
//             per region (entering state, count) -> HBM
//   k_fscan1/2 the exclusive prefix of the tiles' counts (calcbitsindex /
//             findmax)
//   k_emf     one tile per wave again: each lane runs the state machine over
//             its region from its true entering state in K-bit steps of the
//             emission table, storing each step's symbols (up to 4 bytes) with
//             one 4-byte LDS store at its output offset in the wave's staging
//             buffer; the wave copies the tile's output out with 16-B stores
//             (calcresult)
//
// No step needs a bit cursor: the step positions are compile-time, only the
// state chains through the table lookups.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "hh_fsm_kern.h"

#define CW 16                 // k_cnt: waves per workgroup
__host__ __device__ constexpr uint32_t emf_waves() { return 16u; }   // k_emf: waves per workgroup (at most)
#define SCAN_TB 1024          // tiles per k_fscan1 block
#define FX_W 8                // corrections per tile (HH_FSM_KM)
static_assert(FX_W == HH_FSM_KM, "corrections per tile");

enum { FF_FAIL = 1, FF_OVER = 2 };

struct FsmGeo {
    uint64_t bits;        // stream length of the segment
    uint64_t nwords;      // readable payload words
    uint64_t ntiles;
    uint64_t emit_from;   // tiles before it are a prologue
    uint32_t S, G, in_state, ns, r;
};

// Workspace (fsm_decode).  Nothing needs zeroing but `flags`.
struct FsmWork {
    uint32_t *flags;      // [0] status, [2..3] total, [4] leave state, [5] entry state,
                          // [6] the largest tile output
    uint32_t *rec;        // [ntiles][NR] entering state | count << 8
    int32_t *tsum;        // [ntiles] the tile's count (its own view of region 0)
    uint32_t *xs;         // [ntiles] the state leaving the tile
    uint32_t *fx;         // [ntiles + 1][FX_W] corrections of a tile's first regions
    int32_t *fxs;         // [ntiles + 1] the sum of a tile's corrections (k_fscan1's view of fx)
    int32_t *lex;         // [ntiles + 1] exclusive prefix within the scan block
    int64_t *blk;         // [nblk] block totals, then block bases
    int32_t *bmax;        // [nblk] the block's largest tile count (k_emf sizes its staging by it)
};

// The count table at LDS address 0: CB-bit steps (8 for trees of <= 127
// states, 7 above: hh_fsm.h).  A state is carried as its row's byte offset
// (state << (CB + 1)), an entry is the next row | the codes completed, so
// the next lookup's address is one AND-OR of the entry and the step's bits
// (times 2: u16 entries).
template <uint32_t CB>
struct CntFmt {
    static constexpr uint32_t RS = CB + 1;                          // row = state << RS
    static constexpr uint32_t RM = CB == 8 ? 0xfe00u : 0xff00u;     // the row bits of an entry
    // the counts of a sum of entries: bits 4 .. RS - 1 of an entry (between
    // its count and its row) are 0, so the low RS bits of a sum of entries
    // are the sum of their counts while that is below 2^RS (a region's count
    // steps complete at most S < 2^RS codes)
    static constexpr uint32_t CM = (1u << RS) - 1u;
};
// (the kernels using the count table declare no static LDS: the dynamic
// LDS, and with it the table, starts at address 0, and the lookup address
// is the AND-OR alone -- v_and_or_b32, no base add)
template <uint32_t CB>
__device__ __forceinline__ uint32_t ct_at(const uint8_t *, uint32_t row, uint32_t off) {
    return *(lds_u16p)(uintptr_t)((row & CntFmt<CB>::RM) | off);
}
// step k's table offset (its CB bits << 1) in a region held in registers
template <uint32_t SW, uint32_t CB>
__device__ __forceinline__ uint32_t cstep(const uint32_t *w, uint32_t k) {
    if (CB == 8) return rbyte<SW>(w, k) << 1;
    return winsh<SW, CB, 1>(w, CB * k);
}
template <uint32_t CB>
__device__ __forceinline__ uint32_t b1_row(const uint32_t *b1, uint32_t row, uint32_t bit, uint32_t *c) {
    const uint32_t v = b1[(row >> CntFmt<CB>::RS) * 2 + bit];
    *c += (v >> 8) & 255u;
    return (v & 255u) << CntFmt<CB>::RS;
}

// ---------------------------------------------------------------------------
// Region passes of k_cnt on words in registers (states as rows).  lim: the
// region's readable bits (S unless the stream ends inside it); only the TAIL
// instantiations check it.
// ---------------------------------------------------------------------------
// Head steps: the last HS count steps of a region (at most HH_FSM_GMAX bits);
// a head reads the region's words from HWL on.
template <uint32_t SW, uint32_t CB>
struct HeadGeo {
    static constexpr uint32_t S = 32 * SW, NS = S / CB;
    static constexpr uint32_t HS = NS < HH_FSM_GMAX / CB ? NS : HH_FSM_GMAX / CB;
    static constexpr uint32_t HWL = (S - CB * HS) / 32;
};

// The count chain of region j from state s.
template <uint32_t SW, bool TAIL, uint32_t CB>
__device__ __forceinline__ uint32_t cnt_region(const uint8_t *lds, const uint32_t *b1, const uint32_t *w,
                                               uint32_t s, uint32_t lim, uint32_t *n) {
    uint32_t c = 0, ep = 0;
#pragma unroll
    for (uint32_t k = 0; k < 32 * SW / CB; k++) {
        if (!TAIL || CB * k + CB <= lim) {
            const uint32_t e = ct_at<CB>(lds, s, cstep<SW, CB>(w, k));
            s = e;
            // (the counts: c's low RS bits, CntFmt::CM.  Each entry is added
            // one step late, after the next read is issued: the add is then
            // off the chain's read -> AND-OR -> read path.  Added at its
            // step but left to the scheduler, the adds sink to the end of
            // the chain and every step's entry stays live -- 32 registers,
            // the difference between 24 and 32 waves per CU)
            c += ep;
            asm volatile("" : "+v"(c));
            ep = e;
        }
    }
    c += ep;
    c &= CntFmt<CB>::CM;
    s &= CntFmt<CB>::RM;
    if (TAIL)
        for (uint32_t q = lim / CB * CB; q < lim; q++) s = b1_row<CB>(b1, s, rbit_dyn<SW>(w, q), &c);   // the last partial step
    *n = c;
    return s;
}

// Walk: chains A and B stepped together over a region until they meet
// (their count difference stops changing then); lanes not walking carry
// A == B.  Only the lanes whose chains have not met yet look up (the others
// are masked off: a table read costs LDS cycles per distinct bank address of
// its ACTIVE lanes, and most lanes do not walk).  Stops when every lane has
// met.
template <uint32_t SW, bool TAIL, uint32_t CB>
__device__ __forceinline__ void walk_region(const uint8_t *lds, const uint32_t *b1, const uint32_t *w,
                                            uint32_t &A, uint32_t &B, int32_t &d, uint32_t lim) {
    constexpr uint32_t RM = CntFmt<CB>::RM;
    bool go = true;                                   // (uniform) some lane has not met yet
#pragma unroll
    for (uint32_t k = 0; k < 32 * SW / CB; k++) {
        if (go && (!TAIL || CB * k + CB <= lim)) {
            if (A != B) {
                const uint32_t x = cstep<SW, CB>(w, k);
                const uint32_t ea = ct_at<CB>(lds, A, x), eb = ct_at<CB>(lds, B, x);
                A = ea & RM;
                B = eb & RM;
                d += (int32_t)(ea & 15u) - (int32_t)(eb & 15u);
            }
        }
        if ((k & 1u) == 1u && go) go = __ballot(A != B) != 0;   // (every second step)
    }
    if (TAIL) {
        for (uint32_t q = lim / CB * CB; q < lim && A != B; q++) {
            const uint32_t x = rbit_dyn<SW>(w, q);
            uint32_t ca = 0, cb = 0;
            A = b1_row<CB>(b1, A, x, &ca);
            B = b1_row<CB>(b1, B, x, &cb);
            d += (int32_t)ca - (int32_t)cb;
        }
    }
}

// The rare cross-tile fixer (the chains leaving a tile meet beyond the next
// tile's region 0): the true chain (state x) and the assumed one (h) walked
// on through the next tile's regions 1, 2, ... until they meet, at most
// HH_FSM_KM regions, each region's corrections into f -- fsm_fix_next's rule
// (hh_fsm_algo.h), run by the whole wave on uniform chains with the region's
// words in registers, the next region's loaded during the walk.  (Lane 0
// alone reading every window from global memory: ~25 us per fix, the
// slowest waves of a 64 MiB count -- round 5's per-wave end-time stamps.)
// T1: the next tile's first bit (a whole word).  Out of line, by value.
struct CntFix {
    uint32_t f[FX_W];
    uint32_t ok;
};
template <uint32_t SW, uint32_t CB>
__device__ __noinline__ CntFix cnt_fix_wave(const uint32_t *b1, const uint32_t *__restrict__ g, uint64_t nwords, uint64_t bits,
                                            uint64_t T1, uint32_t x, uint32_t h) {
    static_assert(FX_W == HH_FSM_KM, "a correction per region a late meeting may be followed into");
    constexpr uint32_t S = 32 * SW, RS = CntFmt<CB>::RS;
    CntFix o;
    for (uint32_t r = 0; r < FX_W; r++) o.f[r] = 0u;
    uint32_t A = x << RS, B = h << RS, nv[SW], nn[SW];
    fs_load<SW>(nv, fs_rsrc(g, T1 / 32, nwords), 0);
    uint32_t r = 0;
    for (; r < HH_FSM_KM; r++) {
        const uint64_t R = T1 + (uint64_t)r * S;
        if (A == B || R >= bits) break;
        if (r + 1 < HH_FSM_KM) fs_load<SW>(nn, fs_rsrc(g, (R + S) / 32, nwords), 0);   // (the next region's words)
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) asm volatile("" : "+v"(nv[k]));
        const uint32_t ent = A >> RS;
        int32_t dd = 0;
        if (bits - R < S) {
            walk_region<SW, true, CB>(nullptr, b1, nv, A, B, dd, (uint32_t)(bits - R));
            if (A != B) dd += (int32_t)(A != 0) - (int32_t)(B != 0);   // (the tail rule)
        } else {
            walk_region<SW, false, CB>(nullptr, b1, nv, A, B, dd, S);
            if (R + S == bits && A != B) dd += (int32_t)(A != 0) - (int32_t)(B != 0);
        }
        o.f[r] = fsm_fx(ent, dd);
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) nv[k] = nn[k];
    }
    o.ok = r < HH_FSM_KM || A == B ? 1u : 0u;
    return o;
}

// ---------------------------------------------------------------------------
// k_cnt: the count pass of tiles [t0, t1), one tile per wave.  TAIL: the
// tiles in which the stream ends (or whose next tile's region 0 holds the
// end), launched on their own.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr uint32_t cnt_tab_bytes(uint32_t ns, uint32_t cb) {
    return (((ns << (cb + 1)) + ns * 8u + ns) + 15u) & ~15u;
}
// The count launches' LDS: the tables, then k_cntm's chunk counter (16 B)
__host__ __device__ constexpr uint32_t cnt_ctr_off(uint32_t ns, uint32_t cb) { return cnt_tab_bytes(ns, cb); }

// One tile: w = region j's words; region j+1's are loaded here when some
// lane walks -- with a 128-bit head most tiles have no walk, and registers
// held across the count for the rare walk cost occupancy.
// hin: lane 0's guess for region 0 when the caller has it (the previous
// tile's lane-63 head, same wave: tiles in order), else HIN_NONE (computed
// here from pv, the 16 bytes before the tile).  Returns lane 63's head (the
// next tile's region-0 guess), as a row.
#define HIN_NONE 0xffffffffu
// decodeallbits: lane j's guess gs for region j+1's entering state (a chain
// from the root over the last G bits of region j) and (hin == HIN_NONE) lane
// 0's guess hp for its own region 0: the same head over the previous
// region's last G bits -- pv, the HB bytes before the tile: uniform words, a
// chain every lane runs alike (broadcast reads), interleaved with its own
// head.  Both as rows; hp = hin when given.
// (PV = false: hin is always given, pv never read)
template <uint32_t SW, uint32_t CB, bool PV = true>
__device__ __forceinline__ void cnt_heads(const uint8_t *lds, const uint32_t *w, const uint32_t *pv, uint32_t G,
                                          uint32_t hin, uint32_t &gs, uint32_t &hp) {
    constexpr uint32_t S = 32 * SW, RM = CntFmt<CB>::RM;
    constexpr uint32_t NS = S / CB;
    constexpr uint32_t HB = 4 * SW < HH_FSM_GMAX / 8 ? 4 * SW : HH_FSM_GMAX / 8;
    constexpr uint32_t HS = HeadGeo<SW, CB>::HS;   // head steps at most
    static_assert(HB % 4 == 0, "head bytes in whole words");
    static_assert(CB * HS <= 8 * HB, "the head of region 0 within the bytes before the tile");
    const uint32_t GS = G / CB;                       // (uniform)
    gs = 0;
    hp = 0;
    if (PV && hin == HIN_NONE) {
#pragma unroll
        for (uint32_t k = NS - HS; k < NS; k++)
            if (k >= NS - GS) {
                gs = ct_at<CB>(lds, gs, cstep<SW, CB>(w, k));
                hp = ct_at<CB>(lds, hp, CB == 8 ? __builtin_amdgcn_ubfe(pv[(k - (NS - HS)) >> 2], 8 * ((k - (NS - HS)) & 3), 8) << 1
                                                : winsh<HB / 4, CB, 1>(pv, 8 * HB + CB * k - S));
            }
        hp &= RM;
    } else {
#pragma unroll
        for (uint32_t k = NS - HS; k < NS; k++)
            if (k >= NS - GS) gs = ct_at<CB>(lds, gs, cstep<SW, CB>(w, k));
        hp = hin;
    }
    gs &= RM;
}
template <uint32_t SW, bool TAIL, uint32_t CB>
__device__ __forceinline__ uint32_t cnt_tile(const uint8_t *lds, const hh_fsm_view &F, const uint32_t *__restrict__ g,
                                             const FsmGeo &geo, const FsmWork &wk, uint64_t t, const uint32_t *w,
                                             const uint32_t *pv, uint32_t hin) {
    constexpr uint32_t S = 32 * SW, RS = CntFmt<CB>::RS;
    const uint32_t j = threadIdx.x & 63u;
    const uint64_t TB = (uint64_t)NR * S, T0 = t * TB;
    const uint64_t R = T0 + (uint64_t)j * S;
    // readable bits of region j and of region j+1
    uint32_t lim = S, limn = S;
    if (TAIL) {
        lim = R >= geo.bits ? 0u : (geo.bits - R < S ? (uint32_t)(geo.bits - R) : S);
        limn = R + S >= geo.bits ? 0u : (geo.bits - R - S < S ? (uint32_t)(geo.bits - R - S) : S);
    }
    const bool has_next = t + 1 < geo.ntiles;

    // decodeallbits: the guess for region j+1 (a chain started at the root G
    // bits before it), then region j from the guess lane j-1 made for it
    uint32_t gs = 0, hp = 0;
    if (geo.G) cnt_heads<SW, CB>(lds, w, pv, geo.G, hin, gs, hp);
    const uint32_t gup = shfl_up1(gs);              // (cross-lane ops with every lane active)
    const uint32_t sp = j ? gup : (t == 0 ? geo.in_state << RS : hp);
    uint32_t n;
    uint32_t X = cnt_region<SW, TAIL, CB>(lds, F.b1, w, sp, lim, &n);   // region j's exit (given its entry)
    // the stream ends in region j / in region j+1: the tail rule counts a
    // chain that is not at the root there (fsm_region, fsm_walk2)
    const bool endj = TAIL && lim > 0 && R + lim == geo.bits;
    const bool endn = TAIL && limn > 0 && R + S + limn == geo.bits;
    if (endj && X != 0) n += 1;

    // makebigtable: where region j's exit differs from the entry assumed for
    // region j+1 (E), lane j walks region j+1 with both chains; their count
    // difference up to where they meet corrects region j+1's count, and E
    // becomes the exit.  A walk that does not meet in its region changes that
    // region's exit: the next lane walks again in the next round.  The
    // corrections telescope: d = count(true chain) - count(first assumption).
    uint32_t E = gs;                                // (lane 63: the next tile's region 0, guessed alike)
    int32_t d = 0;
    bool lost = false;                              // lane 63: not met in the next tile's region 0
    uint32_t nv[SW];
    bool have_nv = false;
    for (int round = 0; round < NR; round++) {
        const bool want = X != E && limn > 0 && (j < 63 || has_next);
        if (__ballot(want) == 0) break;
        uint32_t A = X, B = want ? E : X;           // (not walking: A == B, no change)
        int32_t dd = 0;
        if (round == 0) {
#pragma unroll
            for (uint32_t k = 0; k < SW; k++) nv[k] = 0u;
        }
        if (want && !have_nv) {
            // region j+1's words, loaded by the walking lanes only (the
            // others' lookups are masked off; their words are not used)
            fs_load<SW>(nv, fs_rsrc(g, uni64(t) * TB / 32, geo.nwords), (j + 1) * SW);
            have_nv = true;
        }
        // (opaque per round: the byte offsets of the walk are not hoisted out
        // of the rounds loop into 4 x SW live registers)
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) asm volatile("" : "+v"(nv[k]));
        walk_region<SW, TAIL, CB>(lds, F.b1, nv, A, B, dd, limn);
        bool deep = false;
        if (want) {
            if (endn && A != B) dd += (int32_t)(A != 0) - (int32_t)(B != 0);   // tail rule
            d += dd;
            E = X;
            deep = A != B && !endn;
            if (j == 63 && deep) {
                lost = true;
                deep = false;
            }
        }
        const uint32_t dp = shfl_up1(deep ? 1u : 0u), xa = shfl_up1(A);
        if (j > 0 && dp) X = xa;
    }

    // records: region j entered in the state lane j-1 assumed last
    const uint32_t Eup = shfl_up1(E), dup = shfl_up1((uint32_t)d);
    const uint32_t ent = (j ? Eup : sp) >> RS;
    const uint32_t cnt = (uint32_t)((int32_t)n + (j ? (int32_t)dup : 0));
    // the tile's stores are unconditional (every lane the same value where a
    // word is the tile's: one store instruction, no branch), so that the
    // compiler can count them and the next tile waits only for its prefetched
    // words, not for these stores to reach memory
    wk.rec[t * NR + j] = fsm_rec(ent, cnt);
    const int32_t sum = wave_sum((int32_t)cnt);
    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)X, 63) >> RS;
    wk.tsum[t] = sum;
    // the next tile's corrections (its region 0 assumed entered in the head
    // guess, lane 63's gs); lanes j and j + 8k store the same word
    uint32_t fxv = 0, fail = 0;
    int32_t fsum = 0;                               // (the corrections' sum: k_fscan1 reads it alone)
    if (has_next) {
        const bool lst = __builtin_amdgcn_readlane((int)lost, 63) != 0;
        if (!lst) {
            const uint32_t E63 = (uint32_t)__builtin_amdgcn_readlane((int)E, 63) >> RS;
            const int32_t d63 = __builtin_amdgcn_readlane(d, 63);
            const uint32_t g63 = (uint32_t)__builtin_amdgcn_readlane((int)gs, 63) >> RS;
            const bool walked = E63 != g63 || d63 != 0;      // (lane 63 walked into the next tile)
            fxv = (j & (FX_W - 1)) == 0 && walked ? fsm_fx(E63, d63) : 0u;
            fsum = walked ? d63 : 0;
        } else {
            // rare: the chains meet beyond the next tile's region 0
            const uint32_t h63 = (uint32_t)__builtin_amdgcn_readlane((int)gs, 63) >> RS;
            const CntFix fo = cnt_fix_wave<SW, CB>(F.b1, g, geo.nwords, geo.bits, T0 + TB, x, h63);
            const uint32_t *f = fo.f, ok = fo.ok;
#pragma unroll
            for (int i = 0; i < FX_W; i++) {
                const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)f[i], 0);
                fxv = (j & (FX_W - 1)) == (uint32_t)i ? v : fxv;
                fsum += fsm_fx_d(v);
            }
            fail = __builtin_amdgcn_readlane((int)ok, 0) ? 0u : 1u;
        }
    }
    wk.fx[(t + 1) * FX_W + (j & (FX_W - 1))] = fxv;   // ((ntiles + 1) x FX_W words: the last tile's too)
    wk.fxs[t + 1] = fsum;
    wk.xs[t] = x | fail << 31;                        // (bit 31: chains that did not meet, k_fscan reports it)
    return (uint32_t)__builtin_amdgcn_readlane((int)gs, 63);
}

#define CNT_WAVES 8           // k_cnt: waves per SIMD the register budget is cut for (32 per CU: 2 workgroups of 16)
// The count pass over tiles [t0, t1) as workgroup blk of nblk with CWX waves
// each (k_cnt; and the tail tiles run by the last workgroups of k_cntm's
// launch, instead of a launch of their own after it).
template <uint32_t SW, bool TAIL, uint32_t CB, uint32_t CWX>
__device__ __forceinline__ void cnt_run(const uint32_t *__restrict__ g, const FsmGeo &geo, const FsmTab &tab,
                                        const FsmWork &wk, uint64_t t0, uint64_t t1, uint32_t blk, uint32_t nblk) {
    static_assert((32 * SW) % CB == 0, "whole count steps per region");
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t S = 32 * SW;
    const uint32_t ns = geo.ns, tid = threadIdx.x, j = tid & 63u;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));   // (uniform: scalar tile index)
    uint32_t *s_b1 = (uint32_t *)(smem + (ns << (CB + 1)));
    uint8_t *s_ts = (uint8_t *)(s_b1 + 2 * ns);
    lds_fill16(smem, tab.ct, ns << (CB + 1));            // (ns x 2^CB u16: a multiple of 16 B)
    for (uint32_t i = tid; i < 2 * ns; i += blockDim.x) s_b1[i] = tab.b1[i];
    for (uint32_t i = tid; i < ns; i += blockDim.x) s_ts[i] = tab.tsym[i];
    __syncthreads();
    const hh_fsm_view F = {(const uint16_t *)smem, s_b1, s_ts, CB};
    const uint64_t TB = (uint64_t)NR * S;
    // tile indices fit 32 bits (2^32 tiles of >= 512 bytes); uniform, kept
    // in scalar registers
    // each wave counts a contiguous run of tiles, in order (TAIL launches: a
    // tile per wave): lane 0's region-0 guess of a tile is then the previous
    // tile's lane-63 head, so only a run's first tile computes it
    const uint32_t nwv = nblk * CWX, te = (uint32_t)t1, gw = blk * CWX + wv;
    const uint32_t run = TAIL ? 1u : ((uint32_t)(t1 - t0) + nwv - 1) / nwv;
    uint32_t t = TAIL ? (uint32_t)t0 + gw : (uint32_t)t0 + gw * run;
    const uint32_t tend = TAIL ? te : (t + run < te ? t + run : te);
    const uint32_t tstep = TAIL ? nwv : 1u;
    // the next tile's words are loaded one tile ahead
    // (and the HB bytes before the tile, for lane 0's head: lane i loads word
    // i -- a scalar load would be waited for by every LDS wait of the tile,
    // since scalar loads return out of order and share the LDS counter)
    constexpr uint32_t HB = 4 * SW < HH_FSM_GMAX / 8 ? 4 * SW : HH_FSM_GMAX / 8;
    uint32_t pw[SW], ppv = 0;
    auto prefetch = [&](uint32_t tt, bool with_pv) {
        tt = (uint32_t)__builtin_amdgcn_readfirstlane((int)tt);
        const uint64_t tw = (uint64_t)tt * TB / 32, pa = tw >= HB / 4 ? tw - HB / 4 : 0u;   // (tile 0: unused)
        const __amdgpu_buffer_rsrc_t rs = fs_rsrc(g, tw, geo.nwords);
        // (the lane id recomputed here: the register budget has no room to
        // keep the load offsets live across the tile)
        const uint32_t ln = lane_id();
        fs_load<SW>(pw, rs, ln * SW);
        if (with_pv) ppv = __builtin_amdgcn_raw_buffer_load_b32(fs_rsrc(g, pa, geo.nwords), (int)(4u * (ln % (HB / 4))), 0, 0);
    };
    if (t == 0 && j < FX_W) wk.fx[j] = 0u;           // (tile 0 has no predecessor to correct it)
    if (t == 0 && j == 0) wk.fxs[0] = 0;
    // The bytes before a tile (pv) are needed by the first tile of a run only
    // (TAIL: every tile): read once before the loop, the loop's loads are the
    // words alone -- reading pv in the loop had every tile wait for all of
    // its memory operations (vmcnt(0)), the previous tile's stores included.
    if (t < tend) prefetch(t, true);
    uint32_t hin = HIN_NONE, pv[HB / 4];
    if (!TAIL) {
#pragma unroll
        for (uint32_t i = 0; i < HB / 4; i++) pv[i] = (uint32_t)__builtin_amdgcn_readlane((int)ppv, i);
    }
    for (; t < tend; t += tstep) {
        t = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
        uint32_t w[SW];
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) w[k] = pw[k];
        if (TAIL) {
#pragma unroll
            for (uint32_t i = 0; i < HB / 4; i++) pv[i] = (uint32_t)__builtin_amdgcn_readlane((int)ppv, i);
        }
        prefetch(t + tstep < tend ? t + tstep : t, TAIL);
        const uint32_t h63 = cnt_tile<SW, TAIL, CB>(smem, F, g, geo, wk, (uint64_t)t, w, pv, hin);
        hin = TAIL ? HIN_NONE : (uint32_t)__builtin_amdgcn_readfirstlane((int)h63);
    }
}

template <uint32_t SW, bool TAIL, uint32_t CB>
__global__ __launch_bounds__(64 * CW) __attribute__((amdgpu_waves_per_eu(CNT_WAVES, 8))) void k_cnt(const uint32_t *__restrict__ g, FsmGeo geo, FsmTab tab, FsmWork wk,
                                                 uint64_t t0, uint64_t t1) {
    cnt_run<SW, TAIL, CB, CW>(g, geo, tab, wk, t0, t1, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// k_cntm: the count pass with M consecutive regions per lane.  A count tile
// is 64 x M regions (M emission tiles); lane j counts regions j M .. j M +
// M - 1 in order, its chain carried from one region into the next, so a head
// (16 lookups) guesses only the entry of a lane's first region: a region
// costs 32 + 16 / M count-table lookups instead of 48.  The head of lane j
// runs over the last G bits of its own last region and guesses lane j+1's
// first entry (lane 63's: the next tile's, as in k_cnt).  Where a lane's exit
// differs from that guess, the lane walks its successor's regions in order
// -- each region's assumed entry read back from the record its owner wrote,
// the record rewritten with the true entry and the corrected count -- until
// the chains meet; a walk that crosses all M regions changes the
// successor's exit, and the successor walks in the next round.  Tile sums
// and states per emission tile (64 regions: 64 / M lanes), corrections of
// the next tile's first regions as in k_cnt.
// ---------------------------------------------------------------------------
// k_cntm's workgroups: cntm_cw(M) waves each, the register budget of
// cntm_waves(M) waves per SIMD (a lane holds its whole span of M regions:
// more than k_cnt's 64 VGPRs).  M = 2: 24 waves per CU in 3 workgroups of 8
// (80 VGPRs); M = 4: 20 in 2 of 10 (96 VGPRs); each workgroup its tables.
// (cb 7: 65 KB count tables for 255 states -- two workgroups per CU, of 12
// waves: byte alphabet count 0.51 -> 0.43 ms against 8)
__host__ __device__ constexpr uint32_t cntm_cw(uint32_t m, uint32_t cb = 8) {
    return m >= 4 ? 10u : cb == 7 ? 12u : 8u;
}
__host__ __device__ constexpr uint32_t cntm_waves(uint32_t m) { return m >= 4 ? 5u : 6u; }
#define CNT_CKDIV 4           // chunks of at most wrun / (waves x CKDIV) tiles, at least 1
#define CNT_CHUNK 4           // k_cntm: count tiles per chunk a wave takes from its workgroup's counter
#ifndef HH_CNT_M
#define HH_CNT_M 2            // regions per lane of the count pass: 2, 4 (k_cntm) or 1 (k_cnt; HH_CNT_M=n overrides)
#endif

// Lane j walks lane j+1's regions, q0 the first (want: this lane walks; A:
// the true state entering them, B0: the entry lane j+1 assumed for its
// first region, both rows).  Out of line (rare; everything by value, so
// that the kernel's argument structures stay in scalar registers).
struct CntmWalk {
    uint32_t A;          // the true state leaving the last region walked (row)
    int32_t d;           // the count corrections applied
    uint32_t met;        // the chains met within the regions
};
template <uint32_t SW, uint32_t CB, uint32_t M>
__device__ __noinline__ CntmWalk cntm_walk(const uint32_t *b1, const uint32_t *__restrict__ g, uint64_t nwords,
                                           uint32_t *rec, uint64_t q0, bool want, uint32_t A, uint32_t B0) {
    constexpr uint32_t S = 32 * SW, RS = CntFmt<CB>::RS;
    bool met = !want;
    uint32_t a = A, b = B0;
    int32_t dsum = 0;
    for (uint32_t r = 0; r < M; r++) {
        if (__ballot(!met) == 0) break;
        const uint64_t q = q0 + r;                       // (lane j+1's region r)
        uint32_t nv[SW], rc = 0;
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) nv[k] = 0u;
        if (!met) {
            fs_load<SW>(nv, fs_rsrc(g, q * SW, nwords), 0);
            // the record as it stands (written by its owner, or by this
            // walk's earlier round): the entry of the chain it counts
            rc = __hip_atomic_load(&rec[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (r > 0) b = fsm_rec_ent(rc) << RS;
        }
#pragma unroll
        for (uint32_t k = 0; k < SW; k++) asm volatile("" : "+v"(nv[k]));
        uint32_t aa = met ? 0u : a, bb = met ? 0u : b;
        int32_t dd = 0;
        walk_region<SW, false, CB>(nullptr, b1, nv, aa, bb, dd, S);
        if (!met) {
            rec[q] = fsm_rec(a >> RS, (uint32_t)((int32_t)fsm_rec_cnt(rc) + dd));
            dsum += dd;
            met = aa == bb;
            a = aa;
        }
    }
    return CntmWalk{a, dsum, met ? 1u : 0u};
}


template <uint32_t SW, uint32_t CB, uint32_t M>
__global__ __launch_bounds__(64 * cntm_cw(M, CB)) __attribute__((amdgpu_waves_per_eu(cntm_waves(M), 8))) void k_cntm(const uint32_t *__restrict__ g, FsmGeo geo, FsmTab tab, FsmWork wk,
                                                  uint64_t c0, uint64_t c1, uint64_t u0, uint64_t u1, uint32_t ntb) {
    static_assert((32 * SW) % CB == 0 && 64 % M == 0, "whole count steps per region, lanes in whole emission tiles");
    constexpr uint32_t CWM = cntm_cw(M, CB);
    // the first ntb workgroups (dispatched first, resident beside the rest):
    // the emission tiles [u0, u1) after the count tiles, one per wave with
    // the stream-end checks (TAIL) -- a launch of their own after this one
    // cost a tile's time at the end of every decode
    if (blockIdx.x < ntb) {
        cnt_run<SW, true, CB, CWM>(g, geo, tab, wk, u0, u1, blockIdx.x, ntb);
        return;
    }
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t S = 32 * SW, RS = CntFmt<CB>::RS, LG = 64 / M;   // LG: lanes per emission tile
    constexpr uint32_t HB = 4 * SW < HH_FSM_GMAX / 8 ? 4 * SW : HH_FSM_GMAX / 8;
    const uint32_t ns = geo.ns, tid = threadIdx.x, j = tid & 63u;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    uint32_t *s_b1 = (uint32_t *)(smem + (ns << (CB + 1)));
    uint8_t *s_ts = (uint8_t *)(s_b1 + 2 * ns);
    lds_fill16(smem, tab.ct, ns << (CB + 1));            // (ns x 2^CB u16: a multiple of 16 B)
    for (uint32_t i = tid; i < 2 * ns; i += blockDim.x) s_b1[i] = tab.b1[i];
    for (uint32_t i = tid; i < ns; i += blockDim.x) s_ts[i] = tab.tsym[i];
    // the workgroup's chunk counter, after the tables
    const uint32_t ctr = cnt_ctr_off(ns, CB);
    if (tid == 0) *(lds_u32p)(uintptr_t)ctr = 0u;
    __syncthreads();
    const hh_fsm_view F = {(const uint16_t *)smem, s_b1, s_ts, CB};
    // Each workgroup counts a contiguous range of count tiles, its waves
    // taking chunks of ck tiles in turn from the workgroup's LDS counter; a
    // wave counts a chunk's tiles in order -- lane 0's entry guess of a tile:
    // the previous tile's lane-63 head; of a chunk's first, a head over the
    // bytes before it.  (Equal runs per wave: the workgroup's waves ended up
    // to 50 us apart in round 5's per-wave end-time stamps.  Chunks from
    // one device-scope counter per XCD instead: count 0.40 -> 0.42 ms.)
    // ck: CNT_CHUNK tiles, or fewer where a workgroup's range holds fewer
    // than CNT_CKDIV chunks per wave (small streams: 128 MiB count 0.070
    // -> 0.063 ms against one chunk per wave)
    const uint32_t nwg = gridDim.x - ntb, wgi = blockIdx.x - ntb, ce = (uint32_t)c1;
    const uint32_t wrun = ((uint32_t)(c1 - c0) + nwg - 1) / nwg;
    const uint32_t ck = max(1u, min((uint32_t)CNT_CHUNK, wrun / (CWM * CNT_CKDIV)));
    const uint32_t wc0 = (uint32_t)c0 + wgi * wrun < ce ? (uint32_t)c0 + wgi * wrun : ce;
    const uint32_t wc1 = wc0 + wrun < ce ? wc0 + wrun : ce;
    const uint32_t nchunk = (wc1 - wc0 + ck - 1) / ck;
    auto claim = [&]() -> uint32_t {
        uint32_t u = 0;
        if (j == 0) u = __hip_atomic_fetch_add((lds_u32p)(uintptr_t)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return (uint32_t)__builtin_amdgcn_readlane((int)u, 0);
    };
    if (c0 == 0 && wgi == 0 && wv == 0) {
        if (j < FX_W) wk.fx[j] = 0u;                  // (tile 0 has no predecessor to correct it)
        if (j == 0) wk.fxs[0] = 0;
    }
    uint32_t kc = claim();
    if (kc >= nchunk) {
        return;
    }
    uint32_t c = wc0 + kc * ck, cend = c + ck < wc1 ? c + ck : wc1;
    // region words a region ahead (the next tile's first after a tile's
    // last), the head words (the last region's [HWL, SW)) a tile ahead
    auto load_region = [&](uint32_t *v, uint32_t cc, uint32_t r, uint32_t a, uint32_t b) {
        cc = (uint32_t)__builtin_amdgcn_readfirstlane((int)cc);
        const __amdgpu_buffer_rsrc_t rs = fs_rsrc(g, (uint64_t)cc * (64u * M) * SW, geo.nwords);
        uint32_t ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        const uint32_t wo = (ln * M + r) * SW;
        if (SW % 4 == 0 && a % 4 == 0 && b % 4 == 0) {
#pragma unroll
            for (uint32_t k = 0; k < SW; k += 4)
                if (k >= a && k < b) {
                    const u32x4 q = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(4u * (wo + k)), 0, 0));
                    v[k] = q.x; v[k + 1] = q.y; v[k + 2] = q.z; v[k + 3] = q.w;
                }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < SW; k++)
                if (k >= a && k < b) v[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * (wo + k)), 0, 0);
        }
    };
    // a lane's M regions are adjacent in memory (M * SW words): loaded in one
    // burst, so that every cache line is read once and at once -- loaded a
    // region at a time, the lines of 64 lanes' spans left L1 between their
    // loads (5x the L2 reads of k_cnt at M = 4).  The heads read the last
    // region's words from the same burst.  The next tile's burst is issued
    // when the last region's words are the only ones still in use.
    uint32_t span[M * SW];
#pragma unroll
    for (uint32_t r = 0; r < M; r++) load_region(span + r * SW, c, r, 0, SW);
    // the HB bytes before a chunk's first tile (lane i: word i), for lane 0's
    // entry guess there
    auto load_pv = [&](uint32_t cc) {
        const uint64_t tw = (uint64_t)cc * (64u * M) * SW, pa = tw >= HB / 4 ? tw - HB / 4 : 0u;   // (tile 0: unused)
        uint32_t ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        return __builtin_amdgcn_raw_buffer_load_b32(fs_rsrc(g, pa, geo.nwords), (int)(4u * (ln % (HB / 4))), 0, 0);
    };
    uint32_t ppv = load_pv(c), hin = HIN_NONE;
    __builtin_amdgcn_s_waitcnt(VMCNT0);
    for (;;) {
        c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
        const uint64_t Q0 = (uint64_t)c * (64u * M);     // the tile's first region
        // the next tile: this chunk's next, else the next chunk's first
        const bool last = c + 1 >= cend;
        if (last) kc = claim();
        const bool more = !last || kc < nchunk;
        const uint32_t cn = !last ? c + 1 : more ? wc0 + kc * ck : c;
        const bool has_next = (uint64_t)(c + 1) * M < geo.ntiles;
        // decodeallbits: lane j's guess for lane j+1's first region, lane 0's
        // for its own (the previous tile's lane-63 head, or -- a chunk's first
        // tile -- a head over the bytes before it, beside lane j's)
        uint32_t gs = 0, hp = hin == HIN_NONE ? 0u : hin;   // (G = 0: every guess the root)
        if (geo.G) {
            if (hin == HIN_NONE) {
                uint32_t pv[HB / 4];
#pragma unroll
                for (uint32_t i = 0; i < HB / 4; i++) pv[i] = (uint32_t)__builtin_amdgcn_readlane((int)ppv, i);
                cnt_heads<SW, CB>(smem, span + (M - 1) * SW, pv, geo.G, HIN_NONE, gs, hp);
                hp = (uint32_t)__builtin_amdgcn_readfirstlane((int)hp);
            } else {
                cnt_heads<SW, CB, false>(smem, span + (M - 1) * SW, nullptr, geo.G, hin, gs, hp);
            }
        }
        const uint32_t gup = shfl_up1(gs);
        const uint32_t sp = j ? gup : (c == 0 ? geo.in_state << RS : hp);
        // the lane's regions in order (records through a buffer resource on
        // the tile's: a scalar base, a 32-bit lane offset)
        const __amdgpu_buffer_rsrc_t rrs =
            __builtin_amdgcn_make_buffer_rsrc((void *)(wk.rec + Q0), 0, (int)(64u * M * 4u), 0x00020000);
        uint32_t s = sp, nsum = 0;
#pragma unroll
        for (uint32_t r = 0; r < M; r++) {
            uint32_t w[SW];
#pragma unroll
            for (uint32_t k = 0; k < SW; k++) w[k] = span[r * SW + k];
            if (r + 1 == M) {
#pragma unroll
                for (uint32_t q = 0; q < M; q++) load_region(span + q * SW, cn, q, 0, SW);   // (the next tile's burst)
                if (last && more) ppv = load_pv(cn);
            }
            uint32_t n;
            const uint32_t X = cnt_region<SW, false, CB>(smem, F.b1, w, s, S, &n);
            __builtin_amdgcn_raw_buffer_store_b32(fsm_rec(s >> RS, n), rrs, (int)(4u * (j * M + r)), 0, 0);
            nsum += n;
            s = X;
        }
        uint32_t X = s, E = gs;

        // makebigtable: walks into the successor's regions (lane 63: into the
        // next tile's region 0, its corrections in fx as in k_cnt)
        int32_t d = 0, dsum = 0;
        bool lost = false;
        for (int round = 0; round < NR; round++) {
            const bool want = X != E && (j < 63 || has_next);
            if (__ballot(want) == 0) break;
            // (the tile's records -- and the last round's rewrites -- reached
            // memory: walks read them back)
            __builtin_amdgcn_s_waitcnt(VMCNT0);
            uint32_t A = X;
            bool met;
            if (j < 63) {
                const CntmWalk cw = cntm_walk<SW, CB, M>(F.b1, g, geo.nwords, wk.rec, Q0 + (uint64_t)(j + 1) * M, want, A, E);
                A = cw.A;
                dsum += cw.d;
                met = cw.met != 0;
            } else {
                // lane 63: the next tile's region 0 (its own record not written yet)
                uint32_t nv[SW];
#pragma unroll
                for (uint32_t k = 0; k < SW; k++) nv[k] = 0u;
                if (want) fs_load<SW>(nv, fs_rsrc(g, (Q0 + 64u * M) * SW, geo.nwords), 0);
#pragma unroll
                for (uint32_t k = 0; k < SW; k++) asm volatile("" : "+v"(nv[k]));
                uint32_t B = want ? E : X;
                int32_t dd = 0;
                walk_region<SW, false, CB>(smem, F.b1, nv, A, B, dd, S);
                if (want) d += dd;
                met = !want || A == B;
            }
            if (want) E = X;
            bool deep = want && !met;
            if (j == 63 && deep) {
                lost = true;
                deep = false;
            }
            const uint32_t dp = shfl_up1(deep ? 1u : 0u), xa = shfl_up1(A);
            if (j > 0 && dp) X = xa;
        }
        // per emission tile (LG lanes): counts with the walks' corrections
        const uint32_t recv = shfl_up1((uint32_t)dsum);
        int32_t v = (int32_t)nsum + (j ? (int32_t)recv : 0);
#pragma unroll
        for (uint32_t o = LG / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        const uint32_t grp = j / LG;
        wk.tsum[(uint64_t)c * M + grp] = v;
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)X, 63) >> RS;
        uint32_t fxv = 0, fail = 0;
        int32_t fsum = 0;
        if (has_next) {
            const bool lst = __builtin_amdgcn_readlane((int)lost, 63) != 0;
            if (!lst) {
                const uint32_t E63 = (uint32_t)__builtin_amdgcn_readlane((int)E, 63) >> RS;
                const int32_t d63 = __builtin_amdgcn_readlane(d, 63);
                const uint32_t g63 = (uint32_t)__builtin_amdgcn_readlane((int)gs, 63) >> RS;
                const bool walked = E63 != g63 || d63 != 0;
                fxv = (j & (FX_W - 1)) == 0 && walked ? fsm_fx(E63, d63) : 0u;
                fsum = walked ? d63 : 0;
            } else {
                const uint32_t h63 = (uint32_t)__builtin_amdgcn_readlane((int)gs, 63) >> RS;
                const CntFix fo = cnt_fix_wave<SW, CB>(F.b1, g, geo.nwords, geo.bits, (Q0 + 64u * M) * S, x, h63);
                const uint32_t *f = fo.f, ok = fo.ok;
#pragma unroll
                for (int i = 0; i < FX_W; i++) {
                    const uint32_t fv = (uint32_t)__builtin_amdgcn_readlane((int)f[i], 0);
                    fxv = (j & (FX_W - 1)) == (uint32_t)i ? fv : fxv;
                    fsum += fsm_fx_d(fv);
                }
                fail = __builtin_amdgcn_readlane((int)ok, 0) ? 0u : 1u;
            }
        }
        // the next tile's first regions' corrections; none for this tile's
        // emission tiles after its first (lanes 8 .. 8 M - 1)
        wk.fx[((uint64_t)c + 1) * M * FX_W + (j & (FX_W - 1))] = fxv;
        if (j < (M - 1) * FX_W) wk.fx[((uint64_t)c * M + 1) * FX_W + j] = 0u;
        // (the sums: the next count tile's first emission tile, zero for this
        // count tile's later ones)
        wk.fxs[j < M ? (j == 0 ? ((uint64_t)c + 1) * M : (uint64_t)c * M + j) : ((uint64_t)c + 1) * M] = j == 0 || j >= M ? fsum : 0;
        // states leaving the emission tiles (the last one's is the tile's)
        wk.xs[(uint64_t)c * M + grp] = (grp == M - 1 ? x : 0u) | fail << 31;
        hin = (uint32_t)__builtin_amdgcn_readlane((int)gs, 63);
        if (!more) break;
        if (last) {
            c = cn;
            cend = c + ck < wc1 ? c + ck : wc1;
            hin = HIN_NONE;
        } else {
            c++;
        }
    }
}

// ---------------------------------------------------------------------------
// k_fscan1: output base of every tile
// ---------------------------------------------------------------------------
#define BMAX_FAIL 0x40000000    // bmax[b]: a tile of block b whose last chain met no other
// The block totals -> exclusive block bases; totals and states into the
// result slot (k_fscan1's last block; blk / bmax were stored sc1 by every
// block, so they are read with sc1 loads -- agent-scope atomic loads -- and
// no cache write-back or invalidate is needed on either side).  s_w, s_mx2,
// s_fl: 16 words of LDS each.
__device__ __forceinline__ void fscan_final(const FsmGeo &geo, const FsmWork &wk, uint32_t nblk, uint32_t *res, int64_t *s_w,
                                            int32_t *s_mx2, uint32_t *s_fl) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    int64_t carry = 0;
    int32_t mx = 0;
    uint32_t fail = 0;
    for (uint32_t b0 = 0; b0 < nblk; b0 += 1024) {
        int64_t v = 0;
        if (b0 + tid < nblk) {
            v = __hip_atomic_load(&wk.blk[b0 + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int32_t bm = __hip_atomic_load(&wk.bmax[b0 + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            mx = max(mx, bm & ~BMAX_FAIL);
            fail |= (uint32_t)bm & BMAX_FAIL;
        }
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
        if (b0 + tid < nblk) {
            wk.blk[b0 + tid] = carry + base + x - v;   // (read by k_emf, after this kernel)
        }
        carry += tot;
        __syncthreads();
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mx = max(mx, __shfl_xor(mx, o, 64));
        fail |= (uint32_t)__shfl_xor((int)fail, o, 64);
    }
    if (lane == 0) {
        s_mx2[wv] = mx;
        s_fl[wv] = fail;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t fl = 0;
        for (uint32_t i = 0; i < 16; i++) {
            mx = max(mx, s_mx2[i]);
            fl |= s_fl[i] ? (uint32_t)FF_FAIL : 0u;
        }
        wk.flags[6] = (uint32_t)mx;       // the largest tile output (symbols)
        wk.flags[8] = 0u;                 // (the block ticket, for the next decode's k_fscan1)
        const uint32_t lv = geo.ntiles ? wk.xs[geo.ntiles - 1] & 255u : geo.in_state;
        uint32_t en = geo.in_state;
        if (geo.emit_from < geo.ntiles) {
            const uint32_t f = wk.fx[geo.emit_from * FX_W];
            en = fsm_fx_ok(f) ? fsm_fx_ent(f) : fsm_rec_ent(wk.rec[geo.emit_from * NR]);
        }
        // the host's copy (mapped memory), read after the stream's sync
        res[0] = fl;
        res[2] = (uint32_t)carry;
        res[3] = (uint32_t)((uint64_t)carry >> 32);
        res[4] = lv;
        res[5] = en;
        res[6] = (uint32_t)mx;
    }
}

// One thread per tile t in [0, ntiles]: the tile's count (its own view plus
// the sum of the corrections its predecessor wrote; prologue tiles emit
// nothing), the exclusive prefix within the block -> lex, the block total ->
// blk.  The block that finishes last then scans the block totals
// (fscan_final): one launch for the whole scan.  The hand-off without fences
// is row 1 of MI355X_MICROARCH.md's measured sc1 hand-off table, cell for
// cell (gfx950 only: hh_fsm_kern.h refuses other targets): each block's
// totals stored sc1 (agent-scope relaxed atomic stores) by ONE lane, that
// lane's s_waitcnt vmcnt(0), then its agent-scope add to ONE ticket word
// (flags[8]); the block whose add returns nblk - 1 -- the last adder, told
// by the value its add returned -- reads them with sc1 loads (agent-scope
// atomic loads), its other waves after a workgroup barrier.
// (test_gpu_parity.py::test_scan_blocks_against_host_prefix checks the bases
// of a many-block scan.)  Block b's part (SCAN_TB threads); returns (uniform)
// whether it drew the last ticket.  s_tmp, s_mx: SCAN_TB / 64 words of LDS
// each, s_last one.
__device__ __forceinline__ bool fscan_block(const FsmGeo &geo, const FsmWork &wk, uint32_t b, uint32_t nblk, int32_t *s_tmp,
                                            int32_t *s_mx, uint32_t *s_last) {
    const uint64_t t = (uint64_t)b * SCAN_TB + threadIdx.x;
    int32_t c = 0;
    if (t < geo.ntiles && t >= geo.emit_from) c = wk.tsum[t] + wk.fxs[t];
    // a tile whose last chain met no other within HH_FSM_KM regions (k_cnt
    // marks its leaving state)
    const bool fl = __ballot(t < geo.ntiles && (wk.xs[t] >> 31)) != 0;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const int32_t x = wave_incl_scan(c);
    int32_t m = c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if (lane == 63) s_tmp[wv] = x;
    if (lane == 0) s_mx[wv] = m | (fl ? BMAX_FAIL : 0);
    __syncthreads();
    int32_t base = 0, tot = 0, mx = 0;
#pragma unroll
    for (uint32_t i = 0; i < SCAN_TB / 64; i++) {
        const int32_t v = s_tmp[i];
        base += i < wv ? v : 0;
        tot += v;
        mx = max(mx & ~BMAX_FAIL, s_mx[i] & ~BMAX_FAIL) | ((mx | s_mx[i]) & BMAX_FAIL);
    }
    if (t <= geo.ntiles) wk.lex[t] = base + x - c;   // (read by k_emf, after this kernel)
    if (threadIdx.x == 0) {
        __hip_atomic_store(&wk.blk[b], (int64_t)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&wk.bmax[b], mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (this thread's stores, before its ticket)
        *s_last = __hip_atomic_fetch_add(&wk.flags[8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1u;
    }
    __syncthreads();
    return *s_last != 0;
}
__global__ __launch_bounds__(SCAN_TB) void k_fscan1(FsmGeo geo, FsmWork wk, uint32_t nblk, uint32_t *res) {
    __shared__ int32_t s_tmp[SCAN_TB / 64], s_mx[SCAN_TB / 64];
    __shared__ uint32_t s_last;
    __shared__ int64_t s_w[16];
    __shared__ int32_t s_mx2[16];
    __shared__ uint32_t s_fl[16];
    if (fscan_block(geo, wk, blockIdx.x, nblk, s_tmp, s_mx, &s_last)) fscan_final(geo, wk, nblk, res, s_w, s_mx2, s_fl);
}

// ---------------------------------------------------------------------------
// k_emf: emission of tiles [t0, t1), one tile per wave.
// ---------------------------------------------------------------------------

// The emission chain of one region (state, output dword, shift) while it
// stores each step's symbols into the staging: every step's symbols are
// shifted into the current dword, which is stored to its aligned LDS address
// when it is full (the last, partial one after the last step).  The unused
// bytes of every stored dword are zero: a dword shared with the
// neighbouring runs is repaired by OR afterwards (emf_edges).
#define EMF_CPOL 2            // k_emf's static copy-out stores: cache policy bits (2: nt -- 1 GiB kjv -3 % against plain)
// Staging swizzle (SWZ, near-uniform codes): the dword at LDS byte address a
// is kept at a ^ (((a >> 7) & 31) << 2), i.e. dwords are permuted within
// each aligned 128-B chunk by the chunk's index.  Where every region emits
// the same number of bytes (2-bit codes: 128 B per 256-bit region) the 64
// lanes' runs start 32 dwords apart and every step's stores would fall in
// one bank; swizzled, lane j's dword p is in bank p ^ j.  The copy-out reads
// a chunk's 16-B blocks back in order (emf_unswz).
template <bool SWZ>
__device__ __forceinline__ uint32_t emf_swz(uint32_t a) { return SWZ ? a ^ ((a >> 5) & 0x7cu) : a; }

// The 16 bytes at LDS offset a (a multiple of 16) in order: with SWZ the
// 128-B chunk's key moves the block (key bits 2..4) and permutes its dwords
// (bits 0..1).
template <bool SWZ>
__device__ __forceinline__ u32x4 emf_read16(const uint8_t *lds, uint32_t a) {
    if (!SWZ) return *(const u32x4 *)(lds + a);
    const uint32_t key = (a >> 7) & 31u;
    const u32x4 v = *(const u32x4 *)(lds + (a ^ ((key & 28u) << 2)));
    const bool s1 = key & 1u, s2 = key & 2u;
    // logical dword t is at position t ^ (key & 3)
    const uint32_t x0 = s1 ? v.y : v.x, x1 = s1 ? v.x : v.y, x2 = s1 ? v.w : v.z, x3 = s1 ? v.z : v.w;
    u32x4 o;
    o.x = s2 ? x2 : x0;
    o.y = s2 ? x3 : x1;
    o.z = s2 ? x0 : x2;
    o.w = s2 ? x1 : x3;
    return o;
}

template <uint32_t K, bool SWZ = false>
struct EmfChain {
    uint32_t row, wd, sh, a;
    __device__ __forceinline__ void init(uint32_t s, uint32_t oa) {
        row = s << HH_FSM_ET_RSH(K);
        wd = oa & ~3u;
        sh = (oa & 3u) * 8u;
        a = 0;                                      // the current dword's bytes so far
    }
    __device__ __forceinline__ uint32_t put(uint8_t *lds, uint64_t e) {
        const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
        const uint32_t u = sh + (hi & 255u);          // 8 x the symbols: one SDWA add
        // one 64-bit shift gives both the bytes that fit the current dword
        // and those that spill into the next (none at sh = 0): 2 VALU
        // instead of 5 (shift-or, negate, alignbit, compare, select); the
        // store through an LDS-space pointer (the staging's byte address is
        // its LDS address: no base add).  A dword is stored once it is full
        // (the run's last, partial one at the end): an exec-masked store's
        // LDS cycles count its active lanes' addresses only.
        const uint64_t t = (uint64_t)lo << sh;
        const uint32_t an = (uint32_t)t | a;
        const bool full = u >= 32;
        if (full) *(lds_u32p)(uintptr_t)emf_swz<SWZ>(wd) = an;
        a = full ? (uint32_t)(t >> 32) : an;
        wd += full ? 4u : 0u;
        sh = u & 31u;
        return an;
    }
    // a step's entry e: store its symbols, advance
    __device__ __forceinline__ void step(uint8_t *lds, uint64_t e) {
        put(lds, e);
        row = HH_FSM_ET_ROW(e);
    }
};

// NCH independent regions (one per chain: region j of NCH tiles) entered in
// states s[c], their symbols to the staging from LDS byte address oa[c] on:
// K-bit steps, the NCH chains' table reads issued together (each chain is a
// dependent sequence of LDS reads; interleaving them hides the latency), then
// the r-bit step (r = S mod K); TAIL (NCH = 1): steps while whole, the rest
// bit by bit, and the tail rule.
//
// Dwords shared between runs: a dword is stored, during the steps, only by
// the run that fills its last byte (its value holds that run's bytes, zeros
// where earlier runs' bytes go); the run that ends the tile stores its last,
// partial dword at the end; every other run that ends inside a dword ORs its
// bytes there after every lane's stores (emf_edges: *lastw at *lastwd when
// *lastpart).  So every dword of the tile's output is stored exactly once
// before the ORs, and no run's first dword needs capturing.
template <uint32_t SW, uint32_t K, bool TAIL, uint32_t NCH, bool SWZ = false>
__device__ __forceinline__ void emf_region(uint8_t *lds, uint32_t er_off, const uint32_t *b1, const uint8_t *ts,
                                           const uint32_t (*w)[SW], const uint32_t *s, uint32_t lim,
                                           const bool *at_end, const uint32_t *oa, const bool *tlast,
                                           uint32_t *lastw, uint32_t *lastwd, bool *lastpart) {
    constexpr uint32_t S = 32 * SW, r = S % K;
    EmfChain<K, SWZ> ch[NCH];
#pragma unroll
    for (uint32_t c = 0; c < NCH; c++) ch[c].init(s[c], oa[c]);
    constexpr uint32_t NST = S / K;
    if (!TAIL) {
        // The chain's critical path is read -> next row -> next read; the
        // symbols' shifts, the full-dword test and the exec-masked store are
        // off it.  Step k+1's read (and after the last step the remainder
        // step's) is issued as soon as step k's entry is back, before step
        // k's store logic: one wait per step, and the store work of a step
        // overlaps the next read's latency (in program order the compiler
        // put the whole store block between a read's return and the next read).
        uint64_t e[NCH];
#pragma unroll
        for (uint32_t c = 0; c < NCH; c++) e[c] = *(const uint64_t *)(lds + et_addr<SW, K>(ch[c].row, w[c], 0));
#pragma unroll
        for (uint32_t k = 0; k < NST; k++) {
            uint64_t en[NCH];
#pragma unroll
            for (uint32_t c = 0; c < NCH; c++) {
                const uint32_t hi = (uint32_t)(e[c] >> 32);
                if (k + 1 < NST) {
                    en[c] = *(const uint64_t __attribute__((address_space(3))) *)(uintptr_t)et_addr<SW, K>(hi, w[c], (k + 1) * K);
                } else if (r) {
                    en[c] = *(const uint64_t *)(lds + er_off + (HH_FSM_ET_ROW(e[c]) >> (HH_FSM_ET_LG(K) - r)) +
                                                (rbits<SW>(w[c], S - r, r) << 3));
                } else {
                    en[c] = 0;
                }
                ch[c].row = HH_FSM_ET_ROW(e[c]);
            }
#pragma unroll
            for (uint32_t c = 0; c < NCH; c++) {
                ch[c].put(lds, e[c]);
                e[c] = en[c];
            }
        }
        if (r) {
#pragma unroll
            for (uint32_t c = 0; c < NCH; c++) {
                ch[c].put(lds, e[c]);
                ch[c].row = HH_FSM_ET_ROW(e[c]);
            }
        }
    } else {
#pragma unroll
    for (uint32_t k = 0; k < S / K; k++) {
        const uint32_t q = k * K;
        if (!TAIL || q + K <= lim) {
            uint64_t e[NCH];
#pragma unroll
            for (uint32_t c = 0; c < NCH; c++) e[c] = *(const uint64_t *)(lds + ch[c].row + win8<SW, K>(w[c], q));
#pragma unroll
            for (uint32_t c = 0; c < NCH; c++) ch[c].step(lds, e[c]);
        }
    }
    }
#pragma unroll
    for (uint32_t c = 0; c < NCH; c++) {
        EmfChain<K, SWZ> &x = ch[c];
        if (!TAIL) {
        } else {
            uint32_t st = x.row >> HH_FSM_ET_RSH(K);
            for (uint32_t q = lim / K * K; q < lim; q++) {
                const uint32_t v = b1[st * 2 + rbit_dyn<SW>(w[c], q)];
                st = v & 255u;
                x.put(lds, HH_FSM_ET_MAKE((v >> 16) & 255u, 0u, (v >> 8) & 255u));
            }
            x.row = st << HH_FSM_ET_RSH(K);
        }
        if (at_end[c] && (x.row >> HH_FSM_ET_RSH(K)) != 0) x.put(lds, HH_FSM_ET_MAKE(ts[x.row >> HH_FSM_ET_RSH(K)], 0u, 1u));   // the tail rule
        if (tlast[c] && x.sh) *(uint32_t *)(lds + emf_swz<SWZ>(x.wd)) = x.a;   // the tile's last, partial dword
        lastw[c] = x.a;
        lastwd[c] = x.wd;
        lastpart[c] = x.sh != 0 && !tlast[c];
    }
}

// After every lane's stores (emf_region): a run that ends inside a dword ORs
// its bytes into it (the run that fills the dword stored it with zeros there).
template <bool SWZ = false>
__device__ __forceinline__ void emf_edges(uint8_t *lds, uint32_t lastw, uint32_t lastwd, bool lastpart) {
    if (lastpart) atomicOr((uint32_t *)(lds + emf_swz<SWZ>(lastwd)), lastw);
}

// A region whose tile's output does not fit the staging buffer: its symbols
// straight to HBM, bit by bit (rare).
template <uint32_t SW>
__device__ __forceinline__ void emf_direct(const uint32_t *b1, const uint8_t *ts, const uint32_t *w, uint32_t s,
                                           uint32_t lim, bool at_end, uint8_t *dst) {
    uint32_t o = 0;
    for (uint32_t q = 0; q < lim; q++) {
        const uint32_t v = b1[s * 2 + rbit_dyn<SW>(w, q)];
        s = v & 255u;
        if ((v >> 8) & 255u) dst[o++] = (uint8_t)(v >> 16);
    }
    if (at_end && s != 0) dst[o] = ts[s];
}

// k_emf: emission of tiles [t0, t1).  Each wave takes NCH tiles at a time
// (tiles t, t + W, ..., W = the grid's active waves), one region of each per
// lane.  The staging is sized from the largest tile output of this decode
// (flags[6], k_fscan1's last block): as many waves of the workgroup are active as the
// LDS beside the tables holds NCH tile stagings for (up to EW), so that
// typical streams keep more chains in flight than a worst-case size allows.
// SCO (static copy-out): the copy-out is COI unrolled lane-masked 16-B
// stores per lane, COI in {4, 8, 16} KiB per tile chosen from this decode's
// largest tile output (flags[6]) -- the number of stores per tile is a
// compile-time constant, so the next tile's wait for its prefetched words
// (vmcnt counts loads and stores in order) need not wait for this tile's
// stores to reach memory.  With a data-dependent store loop it must: the
// compiler waits vmcnt(0) at every tile's start (30 % of the kernel's wave
// cycles in round 3's cycle-stamp build).  (Round 3 measured a fixed COI of 16 no
// faster: three quarters of its stores were empty.)
// The emission of tiles [t0, t1) as workgroup blk of nblk (k_emf; and the
// tail tiles run by k_emf's first workgroups).
template <uint32_t SW, uint32_t K, bool TAIL, uint32_t NCH, bool SCO, bool SWZ>
__device__ __forceinline__ void emf_run(const uint32_t *__restrict__ g, const FsmGeo &geo, const FsmTab &tab,
                                        const FsmWork &wk, uint8_t *__restrict__ out, uint64_t cap, uint64_t t0,
                                        uint64_t t1, uint32_t lds_bytes, uint32_t blk, uint32_t nblk) {
    static_assert(!TAIL || NCH == 1, "the tail tiles take one chain per lane");
    static_assert(!SWZ || !TAIL, "the tail tiles' staging is not swizzled");
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr uint32_t S = 32 * SW;
    const uint32_t ns = geo.ns, r = geo.r, tid = threadIdx.x, j = tid & 63u;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));   // (uniform: scalar tile index)
    const uint32_t er_off = (ns << HH_FSM_ET_LG(K)) * 8u;
    uint32_t *s_b1 = (uint32_t *)(smem + er_off + (r ? (ns << r) * 8u : 0u));
    uint8_t *s_ts = (uint8_t *)(s_b1 + 2 * ns);
    constexpr uint32_t EW = emf_waves();
    lds_fill16(smem, tab.et, (ns << HH_FSM_ET_LG(K)) * 8u);   // (ns x 2^LG u64: a multiple of 16 B)
    for (uint32_t i = tid; r && i < (ns << r); i += blockDim.x) ((uint64_t *)(smem + er_off))[i] = tab.er[i];
    for (uint32_t i = tid; i < 2 * ns; i += blockDim.x) s_b1[i] = tab.b1[i];
    for (uint32_t i = tid; i < ns; i += blockDim.x) s_ts[i] = tab.tsym[i];
    // the workgroup's tile counter (DYN), in the LDS's last 16 bytes
    constexpr bool DYN = !TAIL && NCH == 1;
    const uint32_t ctr = lds_bytes - 16u;
    if (DYN && tid == 0) *(lds_u32p)(uintptr_t)ctr = 0u;
    __syncthreads();
    // staging per tile: the largest tile output + its 16-B misalignment + the
    // last step's overflow dword; the active waves share the rest of the LDS
    const uint32_t tabb = SWZ ? (emf_tab_bytes(ns, K, r) + 127u) & ~127u : emf_tab_bytes(ns, K, r);   // (SWZ: 128-B chunks)
    const uint32_t pool = lds_bytes > tabb + 16u ? lds_bytes - tabb - 16u : 0u;
    const uint32_t mx = __builtin_amdgcn_readfirstlane((int)wk.flags[6]);
    constexpr uint32_t SU = SWZ ? 128u : 16u;         // staging slot unit (SWZ: whole 128-B chunks)
    const uint32_t need = (mx + 16u + 8u + SU - 1u) & ~(SU - 1u);
    uint32_t nact = pool / (NCH * need);
    nact = nact > EW ? EW : nact < 1u ? 1u : nact;
    if (nact > blockDim.x / 64u) nact = blockDim.x / 64u;
    if (wv >= nact) return;                          // (no workgroup barrier after this point)
    const uint32_t obw = pool / (NCH * nact) & ~(SU - 1u);   // (>= need: need is a multiple of SU)

    // the tile loop, with COI unrolled 16-B copy-out stores per lane (a
    // compile-time count: see above) or (COI = 0) a loop over the tile's bytes
    auto tiles = [&](auto coi) {
    constexpr uint32_t COI = decltype(coi)::value;
        const uint64_t TB = (uint64_t)NR * S, nwv = (uint64_t)nblk * nact;
        // next tiles' words, records, corrections and bases, loaded one step
        // ahead (the base words by lanes 0..2, read out with readlane where consumed)
        uint32_t pw[NCH][SW], prec[NCH], pfx[NCH], pmeta[NCH];
        auto prefetch = [&](uint64_t tt0) {
    #pragma unroll
            for (uint32_t c = 0; c < NCH; c++) {
                uint64_t tt = tt0 + c * nwv;
                tt = uni64(tt < t1 ? tt : tt0);
                const uint64_t tw = tt;
                const __amdgpu_buffer_rsrc_t rs = fs_rsrc(g, tw * TB / 32, geo.nwords);
                prec[c] = wk.rec[tw * NR + j];
                pfx[c] = wk.fx[tw * FX_W + (j & (FX_W - 1))];
                const uint32_t *blk32 = (const uint32_t *)wk.blk + 2 * (tt / SCAN_TB);
                const uint32_t ln = j & 3u;
                pmeta[c] = *(ln == 0 ? blk32 : ln == 1 ? blk32 + 1 : (const uint32_t *)&wk.lex[tt]);
                fs_load<SW>(pw[c], rs, j * SW);
            }
        };
        // DYN: the workgroup's tiles t0 + k nwv + blk nact + v (v < nact), in
        // the order u = k nact + v, go to its waves one at a time from the
        // LDS counter -- with equal shares the workgroup's younger waves,
        // behind the older ones in the SIMDs' issue order, ended up to 25 %
        // later (round 5's per-wave end-time stamps)
        auto tile_of = [&](uint32_t u) -> uint64_t {
            const uint32_t k = u / nact;
            return t0 + (uint64_t)k * nwv + (uint64_t)blk * nact + (u - k * nact);
        };
        auto claim = [&]() -> uint64_t {
            uint32_t u = 0;
            if (j == 0) u = __hip_atomic_fetch_add((lds_u32p)(uintptr_t)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return tile_of((uint32_t)__builtin_amdgcn_readlane((int)u, 0));
        };
        uint64_t t = DYN ? claim() : t0 + (uint64_t)blk * nact + wv, tn = t;
        if (t < t1) prefetch(t);
        // (the first tile's loads complete here, once per wave: the compiler
        // orders them differently before the loop than inside it, and its
        // wait at the loop head, merged over both paths, was vmcnt(0) --
        // every tile waiting for the previous tile's stores)
        __builtin_amdgcn_s_waitcnt(VMCNT0);
        for (; t < t1; t = tn) {
            uint32_t w[NCH][SW], ent[NCH], c[NCH], L[NCH], Tout[NCH], a0[NCH], oa[NCH], lim = S;
            uint64_t P0[NCH];
            bool at_end[NCH], fit[NCH], live[NCH];
    #pragma unroll
            for (uint32_t x = 0; x < NCH; x++) {
    #pragma unroll
                for (uint32_t k = 0; k < SW; k++) w[x][k] = pw[x][k];
                const uint64_t tx = t + x * nwv;
                live[x] = tx < t1;
                const uint32_t rc = prec[x], fx = j < FX_W ? pfx[x] : 0u;
                const uint32_t blo = (uint32_t)__builtin_amdgcn_readlane((int)pmeta[x], 0);
                const uint32_t bhi = (uint32_t)__builtin_amdgcn_readlane((int)pmeta[x], 1);
                const int32_t lx = __builtin_amdgcn_readlane((int)pmeta[x], 2);
                ent[x] = fsm_rec_ent(rc);
                int32_t cn = (int32_t)fsm_rec_cnt(rc);
                if (fsm_fx_ok(fx)) {
                    ent[x] = fsm_fx_ent(fx);
                    cn += fsm_fx_d(fx);
                }
                c[x] = live[x] ? (uint32_t)cn : 0u;
                const int32_t incl = wave_incl_scan((int32_t)c[x]);
                L[x] = (uint32_t)incl - c[x];
                Tout[x] = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
                P0[x] = (uint64_t)((int64_t)(((uint64_t)bhi << 32) | blo) + lx);
                const bool inside = P0[x] <= cap && Tout[x] <= cap - P0[x];
                // (a tile past the capacity: the host reports it, total > cap)
                live[x] = live[x] && inside;
                const uint64_t R = tx * TB + (uint64_t)j * S;
                at_end[x] = R + S == geo.bits;
                if (TAIL) {
                    lim = R >= geo.bits ? 0u : (geo.bits - R < S ? (uint32_t)(geo.bits - R) : S);
                    at_end[x] = R < geo.bits && R + S >= geo.bits;
                }
                a0[x] = (uint32_t)(P0[x] & 15u);
                fit[x] = a0[x] + Tout[x] + 8 <= obw;
                // (a chain that does not write its staging still runs: its lanes
                // all store at the slot's start, inside the slot)
                oa[x] = tabb + (wv * NCH + x) * obw + (live[x] && fit[x] ? a0[x] + L[x] : 0u);
            }
            tn = DYN ? claim() : t + NCH * nwv;
            prefetch(tn < t1 ? tn : t);
            uint32_t lw[NCH], lwd[NCH];
            bool lpart[NCH], tl[NCH];
    #pragma unroll
            for (uint32_t x = 0; x < NCH; x++) tl[x] = live[x] && fit[x] && c[x] > 0 && L[x] + c[x] == Tout[x];
            WAVE_SYNC();                                  // the previous tiles' copy-out has read the staging
            emf_region<SW, K, TAIL, NCH, SWZ>(smem, er_off, s_b1, s_ts, w, ent, lim, at_end, oa, tl, lw, lwd, lpart);
            WAVE_SYNC();
    #pragma unroll
            for (uint32_t x = 0; x < NCH; x++)
                if (live[x] && fit[x]) emf_edges<SWZ>(smem, lw[x], lwd[x], lpart[x]);
            WAVE_SYNC();
    #pragma unroll
            for (uint32_t x = 0; x < NCH; x++) {
                if (!(COI != 0) && !live[x]) continue;      // ((COI != 0): no branch around the stores; a dead tile's resource is empty)
                if ((COI != 0) || fit[x]) {
                    // copy-out: whole 16-B blocks; the bytes of the partial first
                    // and last blocks one per lane (lanes 0..15, 16..31)
                    uint8_t *gb = out + (P0[x] - a0[x]);
                    const uint8_t *sb = smem + tabb + (wv * NCH + x) * obw;
                    const uint32_t end = a0[x] + Tout[x], nq = (end + 15u) / 16u;
                    const bool part0 = a0[x] != 0 || end < 16, partl = (end & 15u) != 0 && end > 16;
                    const uint32_t q = j < 16 ? j : (end & ~15u) + (j - 16);
                    const bool pb = j < 32 && (j < 16 ? part0 : partl) && q >= a0[x] && q < end;
                    if ((COI != 0)) {
                        // unconditional buffer stores: the resource spans the
                        // tile's bytes [0, end), so the hardware drops a store
                        // past it; lanes with nothing to store get an offset
                        // past it too -- no branch, a fixed number of stores
                        const __amdgpu_buffer_rsrc_t ors =
                            __builtin_amdgcn_make_buffer_rsrc(gb, 0, (int)(live[x] ? end : 0u), 0x00020000);
    #pragma unroll
                        for (uint32_t ii = 0; ii < COI; ii++) {
                            const uint32_t lo = 16 * (j + 64 * ii);
                            u32x4 v = {0u, 0u, 0u, 0u};
                            if (lo < end) v = emf_read16<SWZ>(smem, (uint32_t)(sb - smem) + lo);   // (LDS reads only where the tile has bytes)
                            __builtin_amdgcn_raw_buffer_store_b128(v, ors, (int)(lo >= a0[x] ? lo : 0x40000000u), 0, EMF_CPOL);
                        }
                        __builtin_amdgcn_raw_buffer_store_b8(smem[emf_swz<SWZ>((uint32_t)(sb - smem) + q)], ors, (int)(pb ? q : 0x40000000u), 0, 0);
                    } else {
                        // four blocks per lane per pass: their LDS reads issued
                        // together, one wait, then their stores
                        for (uint32_t i0 = j; i0 < nq; i0 += 256) {
                            u32x4 v[4];
    #pragma unroll
                            for (uint32_t u = 0; u < 4; u++)   // (unconditional: past the tile's bytes they read
                                v[u] = emf_read16<SWZ>(smem, (uint32_t)(sb - smem) + 16 * (i0 + 64 * u));   // what is never stored)
    #pragma unroll
                            for (uint32_t u = 0; u < 4; u++) {
                                const uint32_t lo = 16 * (i0 + 64 * u);
                                if (lo >= a0[x] && lo + 16 <= end) __builtin_nontemporal_store(v[u], (u32x4 *)(gb + lo));
                            }
                        }
                        if (pb) gb[q] = smem[emf_swz<SWZ>((uint32_t)(sb - smem) + q)];
                    }
                } else {
                    emf_direct<SW>(s_b1, s_ts, w[x], ent[x], lim, at_end[x], out + P0[x] + L[x]);
                }
            }
        }
    };
    // COI from this decode's largest tile output: the copy-out of a tile of
    // mx symbols at a 16-B misalignment < 16 is at most (mx + 15) / 16 blocks
    const uint32_t per = (mx + 15u + 16u * 64u - 1u) / (16u * 64u);
    if (!TAIL && SCO && per <= 4) tiles(std::integral_constant<uint32_t, 4>{});
    else if (!TAIL && SCO && per <= 8) tiles(std::integral_constant<uint32_t, 8>{});
    else if (!TAIL && SCO && per <= 16) tiles(std::integral_constant<uint32_t, 16>{});
    else tiles(std::integral_constant<uint32_t, 0>{});
}

// k_emf: the emission of tiles [t0, t1); its first ntb workgroups (dispatched
// first, resident beside the rest) emit the stream's last tiles [u0, u1)
// with the stream-end checks (TAIL) -- a launch of their own after this one
// cost a tile's time at the end of every decode.
template <uint32_t SW, uint32_t K, bool TAIL, uint32_t NCH, bool SCO, bool SWZ = false>
__global__ __launch_bounds__(64 * emf_waves()) void k_emf(const uint32_t *__restrict__ g, FsmGeo geo, FsmTab tab, FsmWork wk,
                                                 uint8_t *__restrict__ out, uint64_t cap, uint64_t t0, uint64_t t1,
                                                 uint32_t lds_bytes, uint64_t u0, uint64_t u1, uint32_t ntb) {
    if (!TAIL && blockIdx.x < ntb) {
        emf_run<SW, K, true, 1, false, false>(g, geo, tab, wk, out, cap, u0, u1, lds_bytes, blockIdx.x, ntb);
        return;
    }
    emf_run<SW, K, TAIL, NCH, SCO, SWZ>(g, geo, tab, wk, out, cap, t0, t1, lds_bytes, blockIdx.x - ntb, gridDim.x - ntb);
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
typedef void (*kcnt_t)(const uint32_t *, FsmGeo, FsmTab, FsmWork, uint64_t, uint64_t);
typedef void (*kcntm_t)(const uint32_t *, FsmGeo, FsmTab, FsmWork, uint64_t, uint64_t, uint64_t, uint64_t, uint32_t);
typedef void (*kemf_t)(const uint32_t *, FsmGeo, FsmTab, FsmWork, uint8_t *, uint64_t, uint64_t, uint64_t, uint32_t, uint64_t,
                       uint64_t, uint32_t);

#define FSM_SW_CASES(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12)
// k_cntm for regions of S = 32 sw bits with count steps of cb bits (M =
// HH_CNT_M regions per lane): the byte-stepped regions of 256 bits, and the
// 224-bit regions of trees of more than 127 states
static kcntm_t kcntm_for(uint32_t sw, uint32_t cb, uint32_t m) {
    if (cb == 8 && sw == 8) return m == 2 ? k_cntm<8, 8, 2> : m == 4 ? k_cntm<8, 8, 4> : nullptr;
    if (cb == 8 && sw == 7) return m == 2 ? k_cntm<7, 8, 2> : nullptr;   // 224-bit regions: 7-bit emission steps without a remainder
    if (cb == 7 && sw == HH_FSM_S7 / 32)
        return m == 2 ? k_cntm<HH_FSM_S7 / 32, 7, 2> : m == 4 ? k_cntm<HH_FSM_S7 / 32, 7, 4> : nullptr;
    return nullptr;
}
static kcnt_t kcnt_for(uint32_t sw, bool tail, uint32_t cb) {
    // 7-bit count steps: trees of more than 127 states, 224-bit regions only
    if (cb == 7) return sw == HH_FSM_S7 / 32 ? (tail ? k_cnt<HH_FSM_S7 / 32, true, 7> : k_cnt<HH_FSM_S7 / 32, false, 7>) : nullptr;
    if (cb != 8) return nullptr;
    switch (sw) {
#define X(n) case n: return tail ? k_cnt<n, true, 8> : k_cnt<n, false, 8>;
        FSM_SW_CASES(X)
#undef X
    default: return nullptr;
    }
}
// (swz: the swizzled staging, with the static copy-out)
static kemf_t kemf_for(uint32_t sw, uint32_t K, bool tail, bool sco, bool swz = false) {
    switch (sw) {
#define EMF_K(n, k)                                                                                       \
    (tail ? k_emf<n, k, true, 1, false> : swz ? k_emf<n, k, false, 1, true, true>                         \
                                        : sco ? k_emf<n, k, false, 1, true> : k_emf<n, k, false, 1, false>)
#define X(n)                                                                            \
    case n:                                                                             \
        return K == 7 ? EMF_K(n, 7) : K == 6 ? EMF_K(n, 6) : K == 5 ? EMF_K(n, 5) : K == 4 ? EMF_K(n, 4) : nullptr;
        FSM_SW_CASES(X)
#undef X
#undef EMF_K
    default: return nullptr;
    }
}

static size_t lds_cnt(const FsmDev *fd) { return cnt_ctr_off(fd->ns, fd->cb) + 16u; }   // (+ k_cntm's chunk counter)
// k_emf takes the whole LDS (one workgroup per CU) and sizes its stagings
// from the largest tile output at run time
#define EMF_LDS (160u * 1024u)
static size_t lds_emf(const FsmDev *) { return EMF_LDS; }
static_assert(EMF_LDS <= 160u * 1024u, "k_emf's LDS");

// the emission tables of F leave room for 16 stagings of the expected tile
// output (k_emf sizes them at run time)
bool fsm_k_fits(const hh_fsm_tables *F, uint32_t est_tile) {
    const uint64_t need = ((uint64_t)est_tile + 16u + 8u + 15u) & ~15ull;
    return emf_tab_bytes(F->ns, F->K, F->r) + 16u * need + 16u <= EMF_LDS;   // (+ k_emf's tile counter)
}

void fsm_free(FsmDev *fd) {
    if (fd->ct) (void)hipFree(fd->ct);
    if (fd->b1) (void)hipFree(fd->b1);
    if (fd->tsym) (void)hipFree(fd->tsym);
    if (fd->et) (void)hipFree(fd->et);
    if (fd->er) (void)hipFree(fd->er);
    memset(fd, 0, sizeof(*fd));
}

int fsm_upload(FsmDev *fd, const hh_fsm_tables *F, uint32_t G, uint32_t minlen, uint32_t maxlen) {
    fsm_free(fd);
    const uint32_t ns = F->ns;
    const uint32_t sw = F->S / 32;
    if (F->S % 32 || sw < 2 || sw > 12 || (F->cb != 8 && F->cb != 7) || G % F->cb || G > HH_FSM_GMAX || G > F->S)
        return HH_ERR_UNSUPPORTED;
    if (!kcnt_for(sw, false, F->cb)) return HH_ERR_UNSUPPORTED;
    // the tables in LDS: k_cnt's count table; k_emf's emission tables plus
    // at least one staging of the largest tile output the tree allows
    // (k_emf sizes its stagings at run time, from this decode's largest)
    const uint64_t tmax = (uint64_t)NR * F->S / (minlen ? minlen : 1u) + 1u;
    if (cnt_tab_bytes(ns, F->cb) > 160u * 1024u / 2u ||
        (uint64_t)emf_tab_bytes(ns, F->K, F->r) + ((tmax + 16u + 8u + 15u) & ~15ull) > EMF_LDS)
        return HH_ERR_UNSUPPORTED;
    fd->ns = ns;
    fd->cb = F->cb;
    fd->K = F->K;
    fd->r = F->r;
    fd->S = F->S;
    fd->G = G;
    // the static copy-out (k_emf, SCO) unless HH_EMF_SCO=0; k_emf falls back
    // to the store loop itself for tiles of more than 16 KiB
    fd->sco = !(getenv("HH_EMF_SCO") && atoi(getenv("HH_EMF_SCO")) == 0);
    // the count pass with HH_CNT_M regions per lane unless HH_CNT_M=1 is set
    fd->cm = getenv("HH_CNT_M") ? (uint32_t)atoi(getenv("HH_CNT_M")) : (uint32_t)HH_CNT_M;
    if (fd->cm != 2 && fd->cm != 4) fd->cm = 1;
    // regions of a code whose lengths differ by at most one bit emit nearly
    // the same number of bytes each: lanes' runs start a fixed stride apart
    // and their stores collide in one bank unless the staging is swizzled
    // (HH_EMF_SWZ=0/1 overrides)
    fd->swz = maxlen <= minlen + 1;
    if (getenv("HH_EMF_SWZ")) fd->swz = atoi(getenv("HH_EMF_SWZ")) != 0;
    // (the swizzled staging rounds the tables and a tile's staging up to
    // 128 B: one staging of the largest tile output must still fit)
    fd->test_nosync = getenv("HH_TEST_NOSYNC") && atoi(getenv("HH_TEST_NOSYNC")) != 0;
    if (fd->swz && ((uint64_t)((emf_tab_bytes(ns, F->K, F->r) + 127u) & ~127u) + ((tmax + 16u + 8u + 127u) & ~127ull) >
                    EMF_LDS || !fd->sco))
        fd->swz = 0;
    FS_OK(hipMalloc(&fd->ct, (size_t)ns << (F->cb + 1)));
    FS_OK(hipMalloc(&fd->b1, (size_t)ns * 8));
    FS_OK(hipMalloc(&fd->tsym, (size_t)ns + 1));
    FS_OK(hipMalloc(&fd->et, (size_t)(ns << HH_FSM_ET_LG(F->K)) * 8));
    FS_OK(hipMalloc(&fd->er, (size_t)(ns << (F->r ? F->r : 1)) * 8));
    FS_OK(hipMemcpy(fd->ct, F->ct, (size_t)ns << (F->cb + 1), hipMemcpyHostToDevice));
    FS_OK(hipMemcpy(fd->b1, F->b1, (size_t)ns * 8, hipMemcpyHostToDevice));
    FS_OK(hipMemcpy(fd->tsym, F->tsym, (size_t)ns, hipMemcpyHostToDevice));
    FS_OK(hipMemcpy(fd->et, F->et, (size_t)(ns << HH_FSM_ET_LG(F->K)) * 8, hipMemcpyHostToDevice));
    if (F->r) FS_OK(hipMemcpy(fd->er, F->er, (size_t)(ns << F->r) * 8, hipMemcpyHostToDevice));
    fd->ok = 1;
    return HH_OK;
}

static int fsm_grids(FsmDev *fd) {
    if (fd->grid_c && fd->sized_S == fd->S && fd->sized_ns == fd->ns && fd->sized_K == fd->K && fd->sized_sco == fd->sco &&
        fd->sized_cb == fd->cb && fd->sized_swz == fd->swz && fd->sized_cm == fd->cm)
        return HH_OK;
    const uint32_t sw = fd->S / 32;
    const kcnt_t kc = kcnt_for(sw, false, fd->cb);
    const kemf_t ke = kemf_for(sw, fd->K, false, fd->sco, fd->swz);
    if (!kc || !ke) return HH_ERR_UNSUPPORTED;
    int pc = 0, pe = 0, ncu = 0, dev = 0;
    FS_OK(hipGetDevice(&dev));
    // the table lookups address LDS from 0 (hh_fsm_kern.h): the kernels may
    // declare no static LDS
    const void *kst[3] = {(const void *)kc, (const void *)ke,
                          (const void *)(fd->cm > 1 ? kcntm_for(sw, fd->cb, fd->cm) : nullptr)};
    for (const void *k : kst) {
        hipFuncAttributes fa;
        if (k && (hipFuncGetAttributes(&fa, k) != hipSuccess || fa.sharedSizeBytes != 0)) return HH_ERR_INTERNAL;
    }
    FS_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kc, 64 * CW, lds_cnt(fd)));
    FS_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pe, ke, 64 * emf_waves(), lds_emf(fd)));
    FS_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (pc < 1 || pe < 1) return HH_ERR_UNSUPPORTED;
    fd->grid_c = (uint32_t)(pc * ncu);
    fd->grid_cm = 0;
    const kcntm_t km = fd->cm > 1 ? kcntm_for(sw, fd->cb, fd->cm) : nullptr;
    if (km) {
        int pm = 0;
        FS_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pm, km, 64 * cntm_cw(fd->cm, fd->cb), lds_cnt(fd)));
        fd->grid_cm = pm > 0 ? (uint32_t)(pm * ncu) : 0u;
    }
    fd->grid_e = (uint32_t)(pe * ncu);
    fd->sized_S = fd->S;
    fd->sized_ns = fd->ns;
    fd->sized_K = fd->K;
    fd->sized_sco = fd->sco;
    fd->sized_swz = fd->swz;
    fd->sized_cb = fd->cb;
    fd->sized_cm = fd->cm;
    return HH_OK;
}

static int ws_need(FsmWs *ws, size_t need, hipStream_t st) {
    if (ws->size >= need) return HH_OK;
    if (ws->p) {
        FS_OK(hipDeviceSynchronize());   // (an asynchronous decode may still use it)
        FS_OK(hipFree(ws->p));
    }
    ws->p = nullptr;
    ws->size = 0;
    const size_t sz = need + need / 8;
    if (hipMalloc(&ws->p, sz) != hipSuccess) return HH_ERR_NOMEM;
    ws->size = sz;
    // the status word and the scan's block ticket (the scan's last block
    // clears it), zeroed on the decode's stream: a plain hipMemset goes to
    // the null stream, which a non-blocking decode stream does not wait
    // for -- it could land while the first decode's scan counts its tickets
    FS_OK(hipMemsetAsync(ws->p, 0, 64, st));
    return HH_OK;
}

void fsm_ws_free(FsmWs *ws) {
    if (ws->p) (void)hipFree(ws->p);
    if (ws->st) (void)hipFree(ws->st);
    if (ws->h_res) (void)hipHostFree(ws->h_res);
    memset(ws, 0, sizeof(*ws));
}

static int ws_side(FsmWs *ws) {
    if (ws->h_res) return HH_OK;
    if (hipHostMalloc((void **)&ws->h_res, FSM_RES_SLOTS * 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        ws->h_res = nullptr;
        return HH_ERR_NOMEM;
    }
    FS_OK(hipHostGetDevicePointer((void **)&ws->d_res, ws->h_res, 0));
    return HH_OK;
}

// The launch half: every kernel of the decode enqueued on st, the results
// to be written by k_fscan1's last block into result slot `slot` of the host-mapped
// memory; *pd keeps what fsm_collect needs.
int fsm_launch(FsmDev *fd, FsmWs *ws, uint32_t slot, hipEvent_t *ev, const void *d_data, uint64_t bits,
               uint64_t ntiles, uint32_t in_state, uint64_t emit_from, void *d_out, uint64_t cap, hipStream_t st,
               FsmPend *pd, bool force_two) {
    if (!fd->ok) return HH_ERR_UNSUPPORTED;
    // the single pass (hh_one.hip) unless the tree's tables leave it no room,
    // the decoder asks for the two passes, or a single-pass decode of this
    // stream handed it back
    pd->nt_arg = ntiles;
    pd->in_state = in_state;
    if (fd->one_ok && !fd->two_pass && !fd->phases && !force_two) {
        const int orc = one_launch(fd, ws, slot, ev, d_data, bits, ntiles, in_state, emit_from, d_out, cap, st, pd);
        if (orc != HH_ERR_UNSUPPORTED) return orc;
    }
    pd->one = 0;
    if (slot >= FSM_RES_SLOTS) return HH_ERR_ARG;
    int rc = fsm_grids(fd);
    if (rc) return rc;
    if (in_state >= fd->ns) return HH_ERR_ARG;
    FsmGeo geo;
    geo.bits = bits;
    geo.nwords = ((bits + 7) / 8 + HH_PAYLOAD_PAD) / 4;
    geo.S = fd->S;
    geo.G = fd->G;
    geo.in_state = in_state;
    geo.ns = fd->ns;
    geo.r = fd->r;
    const uint64_t TB = (uint64_t)NR * fd->S;
    const uint64_t all = (bits + TB - 1) / TB;
    geo.ntiles = ntiles && ntiles < all ? ntiles : all;
    geo.emit_from = emit_from;
    const uint64_t nt = geo.ntiles;
    const uint32_t nblk = (uint32_t)((nt + 1 + SCAN_TB - 1) / SCAN_TB);
    // workspace: flags 64 B | rec | tsum | xs | fx | lex | fxs | blk
    const size_t o_rec = 64, o_tsum = o_rec + nt * NR * 4, o_xs = o_tsum + nt * 4, o_fx = o_xs + nt * 4;
    const size_t o_lex = o_fx + (nt + 1) * FX_W * 4, o_fxs = o_lex + (nt + 1) * 4;
    const size_t o_blk = (o_fxs + (nt + 1) * 4 + 7) & ~(size_t)7;
    const size_t o_bmax = o_blk + (size_t)nblk * 8;
    rc = ws_need(ws, o_bmax + (size_t)nblk * 4, st);
    if (rc) return rc;
    uint8_t *w = (uint8_t *)ws->p;
    FsmWork wk;
    wk.flags = (uint32_t *)w;
    wk.rec = (uint32_t *)(w + o_rec);
    wk.tsum = (int32_t *)(w + o_tsum);
    wk.xs = (uint32_t *)(w + o_xs);
    wk.fx = (uint32_t *)(w + o_fx);
    wk.lex = (int32_t *)(w + o_lex);
    wk.fxs = (int32_t *)(w + o_fxs);
    wk.blk = (int64_t *)(w + o_blk);
    wk.bmax = (int32_t *)(w + o_bmax);
    FsmTab tab = {fd->ct, fd->b1, fd->tsym, fd->et, fd->er};
    const uint32_t sw = fd->S / 32;
    rc = ws_side(ws);
    if (rc) return rc;
    FS_OK(hipEventRecord(ev[0], st));
    {
        // tiles [0, nc) whose regions and next region end before the stream,
        // then the last ones (TAIL).  (The tail launches on a second stream
        // beside the main ones measured slower: the cross-stream waits cost
        // more than the overlap saved, 0.155 -> 0.18 ms at 64 MiB.)
        const uint64_t S = fd->S;
        uint64_t nc = bits > TB + S ? std::min<uint64_t>((bits - S - 1) / TB, nt) : 0;
        // k_cntm (M regions per lane) over the whole count tiles in [0, nc),
        // the tiles after them (fewer than M, and the stream's last) by the
        // TAIL launch
        const uint64_t nct = fd->grid_cm ? nc / fd->cm : 0;
        if (nct) {
            // (the tiles after the count tiles: the launch's first workgroups)
            const uint32_t cwm = cntm_cw(fd->cm, fd->cb);
            const uint64_t nu = nt - nct * fd->cm;
            const uint32_t ntb = (uint32_t)((nu + cwm - 1) / cwm);
            const uint64_t nwg = (nct + cwm - 1) / cwm;
            const uint32_t gm = fd->grid_cm > ntb + 1 ? fd->grid_cm - ntb : 1u;
            const uint32_t gc = (uint32_t)(nwg < gm ? nwg : gm) + ntb;
            hipLaunchKernelGGL(kcntm_for(sw, fd->cb, fd->cm), dim3(gc), dim3(64 * cwm), lds_cnt(fd), st, (const uint32_t *)d_data, geo,
                               tab, wk, (uint64_t)0, nct, nct * fd->cm, nt, ntb);
            FS_OK(hipGetLastError());
            nc = nt;
        } else if (nc) {
            const uint64_t nwg = (nc + CW - 1) / CW;
            const uint32_t gc = (uint32_t)(nwg < fd->grid_c ? nwg : fd->grid_c);
            hipLaunchKernelGGL(kcnt_for(sw, false, fd->cb), dim3(gc), dim3(64 * CW), lds_cnt(fd), st, (const uint32_t *)d_data,
                               geo, tab, wk, (uint64_t)0, nc);
            FS_OK(hipGetLastError());
        }
        if (nc < nt) {
            hipLaunchKernelGGL(kcnt_for(sw, true, fd->cb), dim3((unsigned)((nt - nc + CW - 1) / CW)), dim3(64 * CW), lds_cnt(fd),
                               st, (const uint32_t *)d_data, geo, tab, wk, nc, nt);
            FS_OK(hipGetLastError());
        }
    }
    if (fd->phases) FS_OK(hipEventRecord(ev[1], st));
    // tiles that end before the stream, then the last one(s) (TAIL: the main
    // emission launch's first workgroups; a launch of their own without
    // tiles before them)
    const uint64_t ne = std::max<uint64_t>(emit_from, std::min<uint64_t>(bits / TB, nt));
    hipLaunchKernelGGL(k_fscan1, dim3(nblk), dim3(SCAN_TB), 0, st, geo, wk, nblk, ws->d_res + 16 * slot);
    FS_OK(hipGetLastError());
    if (fd->phases) FS_OK(hipEventRecord(ev[2], st));
    if (emit_from < nt) {
        const uint32_t ew = emf_waves(), ew1 = emf_waves();
        const uint32_t ntb = (uint32_t)((nt - ne + ew1 - 1) / ew1);
        if (ne > emit_from) {
            const uint64_t nwg = (ne - emit_from + ew - 1) / ew;
            const uint32_t gm = fd->grid_e > ntb + 1 ? fd->grid_e - ntb : 1u;
            const uint32_t ge = (uint32_t)(nwg < gm ? nwg : gm) + ntb;
            hipLaunchKernelGGL(kemf_for(sw, fd->K, false, fd->sco, fd->swz), dim3(ge), dim3(64 * ew), lds_emf(fd), st,
                               (const uint32_t *)d_data, geo, tab, wk, (uint8_t *)d_out, cap, emit_from, ne,
                               (uint32_t)lds_emf(fd), ne, nt, ntb);
            FS_OK(hipGetLastError());
        } else if (ne < nt) {
            hipLaunchKernelGGL(kemf_for(sw, fd->K, true, false), dim3(ntb), dim3(64 * ew1), lds_emf(fd), st,
                               (const uint32_t *)d_data, geo, tab, wk, (uint8_t *)d_out, cap, ne, nt,
                               (uint32_t)lds_emf(fd), (uint64_t)0, (uint64_t)0, 0u);
            FS_OK(hipGetLastError());
        }
    }
    FS_OK(hipEventRecord(ev[3], st));
    pd->phases = fd->phases;
    pd->nt = nt;
    pd->emit_from = emit_from;
    pd->cap = cap;
    pd->slot = slot;
    pd->test_nosync = fd->test_nosync;
    return HH_OK;
}

// The collect half: waits for the decode's last kernel (its end event) and
// reads its results from its slot.
int fsm_collect(FsmWs *ws, hipEvent_t *ev, const FsmPend *pd, uint64_t *total, uint32_t *leave, uint32_t *entry,
                float *ms) {
    FS_OK(hipEventSynchronize(ev[3]));
    const uint64_t nt = pd->nt, emit_from = pd->emit_from, cap = pd->cap;
    const volatile uint32_t *res = ws->h_res + 16 * pd->slot;
    const uint32_t fl = res[0];
    if (pd->one && (fl & ~(uint32_t)FF_FAIL)) return HH_ONE_RETRY;   // (the single pass handed it back)
    *total = (uint64_t)res[2] | ((uint64_t)res[3] << 32);
    *leave = res[4];
    *entry = res[5];
    if (emit_from >= nt) *total = 0;
    if (pd->phases) {
        (void)hipEventElapsedTime(&ms[0], ev[0], ev[1]);
        (void)hipEventElapsedTime(&ms[1], ev[1], ev[2]);
        (void)hipEventElapsedTime(&ms[2], ev[2], ev[3]);
        ms[3] = ms[0] + ms[1] + ms[2];
    } else {
        // (no events between the kernels: each costs ~6 us of idle GPU)
        ms[0] = ms[1] = ms[2] = 0.0f;
        (void)hipEventElapsedTime(&ms[3], ev[0], ev[3]);
    }
    if ((fl & FF_FAIL) || pd->test_nosync) return HH_NOSYNC;
    if (*total > cap) return HH_ERR_CAPACITY;
    return HH_OK;
}

int fsm_decode(FsmDev *fd, FsmWs *ws, uint32_t *h_flags, hipEvent_t *ev, const void *d_data, uint64_t bits,
               uint64_t ntiles, uint32_t in_state, uint64_t emit_from, void *d_out, uint64_t cap,
               hipStream_t st, uint64_t *total, uint32_t *leave, uint32_t *entry, float *ms) {
    (void)h_flags;
    FsmPend pd;
    int rc = fsm_launch(fd, ws, 0, ev, d_data, bits, ntiles, in_state, emit_from, d_out, cap, st, &pd);
    if (rc) return rc;
    rc = fsm_collect(ws, ev, &pd, total, leave, entry, ms);
    ws->last_one = pd.one;
    if (rc != HH_ONE_RETRY) return rc;
    ws->last_one = 0;
    rc = fsm_launch(fd, ws, 0, ev, d_data, bits, ntiles, in_state, emit_from, d_out, cap, st, &pd, true);
    if (rc) return rc;
    return fsm_collect(ws, ev, &pd, total, leave, entry, ms);
}

// Diagnostic: the count pass's arrays of the last decode (tests, tools).
int fsm_debug_arrays(const FsmWs *ws, uint64_t nt, uint32_t *rec, uint32_t *fx, int32_t *tsum, uint32_t *xs) {
    if (!ws->p) return HH_ERR_ARG;
    const size_t o_rec = 64, o_tsum = o_rec + nt * NR * 4, o_xs = o_tsum + nt * 4, o_fx = o_xs + nt * 4;
    const uint8_t *w = (const uint8_t *)ws->p;
    if (o_fx + (nt + 1) * FX_W * 4 > ws->size) return HH_ERR_ARG;
    FS_OK(hipDeviceSynchronize());
    if (rec) FS_OK(hipMemcpy(rec, w + o_rec, nt * NR * 4, hipMemcpyDeviceToHost));
    if (tsum) FS_OK(hipMemcpy(tsum, w + o_tsum, nt * 4, hipMemcpyDeviceToHost));
    if (xs) FS_OK(hipMemcpy(xs, w + o_xs, nt * 4, hipMemcpyDeviceToHost));
    if (fx) FS_OK(hipMemcpy(fx, w + o_fx, (nt + 1) * FX_W * 4, hipMemcpyDeviceToHost));
    return HH_OK;
}
