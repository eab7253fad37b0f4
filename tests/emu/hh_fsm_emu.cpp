// hh_fsm_emu.cpp -- TEST-ONLY host emulation of the state-machine decode
// (hh_fsm.hip).  Runs the kernels' tile decomposition lane by lane with the
// same tables (hh_fsm_build) and the same per-lane helpers (hh_fsm_algo.h):
// guesses from G-bit heads, region counts, walks where a region's exit state
// differs from the next region's guess, the in-tile fixer for walks that do
// not meet within their region, the next tile's corrections, the prefix of
// tile counts, and emission with the kernels' K-bit steps -- so that the
// decomposition is checked against the oracle without a GPU.  Every region's
// emitted symbols are checked against its recorded count.  Nothing in the
// product links this file (tests/emu/libhh_emu.so).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hh_algo.h"
#include "hh_fsm_algo.h"
#include "hh_internal.h"
#include "hiphuff.h"

#define NR 64   // regions per tile (the kernels' wave)

static hh_tables g_T;
static hh_fsm_tables g_F;
static uint32_t g_K = 0;                            // emission step bits asked for (hh_fsm_emu_set_k)
static uint32_t g_M = 1;                            // regions per lane of the count pass (hh_fsm_emu_set_m)
static std::vector<uint32_t> g_rec, g_xs, g_fx;   // the last decode's count-pass arrays
static std::vector<int64_t> g_tsum;

extern "C" {

// The emission step the next decodes build their tables for (0, 6, 7).
void hh_fsm_emu_set_k(uint32_t K) { g_K = K; }
// Regions per lane of the count pass (the kernels' k_cnt with M > 1: a lane
// counts M consecutive regions, its chain carried from one to the next; a
// head guesses only a lane's first region): tiles of 64 M regions.
void hh_fsm_emu_set_m(uint32_t M) { g_M = M ? M : 1u; }

// stats[0] tiles  [1] walks  [2] walks not met in their region  [3] S
// [4] G  [5] next-tile corrections  [6] corrections over > 1 region
// [7] K-step regions emitted  [8] serial regions emitted
int64_t hh_fsm_emu_decode(const int32_t *izero, const int32_t *ione, const uint8_t *sym, int32_t nodes,
                          const uint8_t *data, uint64_t bits, uint32_t S, int32_t G_req,
                          uint64_t ntiles_req, uint64_t prologue, uint32_t in_state, uint8_t *out,
                          uint64_t cap, int64_t *stats, uint32_t *leave, uint32_t *entry) {
    hh_tree tree = {nodes, izero, ione, sym};
    int rc = hh_tables_build(&tree, &g_T);
    if (rc) return rc;
    for (int i = 0; i < 9; i++) stats[i] = 0;
    if (S == 0)
        S = hh_fsm_region_bits(hh_fsm_nstates(&g_T), (uint32_t)g_T.len_gcd,
                               hh_pick_region_bits((uint32_t)g_T.len_gcd));
    if (S < 32 || S % 32) return HH_ERR_ARG;
    rc = hh_fsm_build(&g_T, S, g_K, &g_F);
    if (rc) return rc;
    uint32_t G = G_req >= 0 ? (uint32_t)G_req : hh_fsm_pick_head(&g_T, S, g_F.cb);
    if (G % g_F.cb || G > HH_FSM_GMAX || G > S) return HH_ERR_ARG;
    stats[3] = S;
    stats[4] = G;
    if (leave) *leave = in_state;
    if (entry) *entry = in_state;
    if (bits == 0) return 0;
    const hh_fsm_view F = {g_F.ct, g_F.b1, g_F.tsym, g_F.cb};
    const uint64_t nw = (bits + 7) / 8 / 4 + 24;
    std::vector<uint32_t> wv(nw, 0u);
    memcpy(wv.data(), data, (bits + 7) / 8);
    // (bits past the end are never read as stream bits)
    const uint32_t *w = wv.data();
    // (a tile here: 64 lanes x M regions; region j of a tile is lane j / M's)
    const uint32_t M = g_M, NRT = NR * M;
    const uint64_t TB = (uint64_t)NRT * S;
    const uint64_t all = (bits + TB - 1) / TB;
    const uint64_t nt = ntiles_req && ntiles_req < all ? ntiles_req : all;
    std::vector<uint32_t> rec(nt * NRT), xs(nt), fx((nt + 1) * HH_FSM_KM, 0u);
    std::vector<int64_t> tsum(nt);
    std::vector<uint32_t> g(NRT), sp(NRT), n(NRT), tx(NRT), mm(NRT), dp(NRT), u(NRT), ent(NRT), cnt(NRT), xv(NRT);
    std::vector<int32_t> dl(NRT);
    for (uint64_t t = 0; t < nt; t++) {
        const uint64_t T0 = t * TB;
        // g[j]: the entry region j+1 is assumed in -- a head guess where
        // region j+1 starts a lane, else the exit region j's chain reaches
        for (uint32_t j = 0; j < NRT; j++) {
            const uint64_t R1 = T0 + (uint64_t)(j + 1) * S;
            uint32_t c = 0;
            g[j] = 0;
            if ((j + 1) % M == 0 && G && R1 - G < bits) g[j] = fsm_run(&F, w, R1 - G, R1 < bits ? R1 : bits, 0u, &c);
        }
        // region 0 of a later tile: the head guess from the G bits before it
        // (the same chain the previous tile's last lane computed as g[NRT-1])
        uint32_t h0 = 0;
        if (t > 0 && G) {
            uint32_t c = 0;
            h0 = fsm_run(&F, w, T0 - G, T0, 0u, &c);
        }
        for (uint32_t j = 0; j < NRT; j++) {
            if (j % M != 0) g[j - 1] = tx[j - 1];     // (a lane's chain carried into its next region)
            sp[j] = j ? g[j - 1] : (t == 0 ? in_state : h0);
            const uint64_t R = T0 + (uint64_t)j * S;
            tx[j] = fsm_region(&F, w, R, R + S, bits, sp[j], &n[j]);
        }
        for (uint32_t j = 0; j < NRT; j++) {
            mm[j] = dp[j] = 0;
            dl[j] = 0;
            u[j] = tx[j];
            if (j == NRT - 1) continue;                // (the next tile: fsm_fix_next)
            const uint64_t R = T0 + (uint64_t)(j + 1) * S;
            if (tx[j] == g[j] || R >= bits) continue;
            mm[j] = 1;
            stats[1]++;
            uint32_t A = tx[j], B = g[j];
            const int met = fsm_walk2(&F, w, R, R + S, bits, &A, &B, &dl[j]);
            dp[j] = !met && R + S < bits;
            u[j] = A;
            stats[2] += dp[j];
        }
        for (uint32_t j = 0; j < NRT; j++) {
            ent[j] = j ? tx[j - 1] : sp[0];
            cnt[j] = n[j] + (j && mm[j - 1] ? (uint32_t)dl[j - 1] : 0u);
            xv[j] = j && mm[j - 1] && dp[j - 1] ? u[j - 1] : tx[j];
        }
        uint32_t x = xv[NRT - 1];
        bool deep = false;
        for (uint32_t j = 0; j < NRT; j++) deep = deep || dp[j];
        if (deep) {
            // the in-tile fixer (the kernel's rare serial path)
            uint32_t st = xv[0];
            for (uint32_t r = 1; r < NRT; r++) {
                if (st == ent[r]) {
                    st = xv[r];
                    continue;
                }
                const uint64_t R = T0 + (uint64_t)r * S;
                uint32_t c;
                const uint32_t e = fsm_region(&F, w, R, R + S, bits, st, &c);
                ent[r] = st;
                cnt[r] = c;
                st = e;
            }
            x = st;
        }
        xs[t] = x;
        int64_t sum = 0;
        for (uint32_t j = 0; j < NRT; j++) {
            rec[t * NRT + j] = fsm_rec(ent[j], cnt[j]);
            sum += cnt[j];
        }
        tsum[t] = sum;
        if (t + 1 < nt && x != g[NRT - 1]) {
            stats[5]++;
            if (!fsm_fix_next(&F, w, T0 + TB, S, bits, x, g[NRT - 1], &fx[(t + 1) * HH_FSM_KM])) return HH_ERR_UNSUPPORTED;
            stats[6] += fsm_fx_ok(fx[(t + 1) * HH_FSM_KM + 1]) != 0;
        }
        stats[0]++;
    }
    // scan (prologue tiles emit nothing) and emission
    uint64_t o = 0;
    const uint32_t K = g_F.K, r = g_F.r;
    uint8_t buf[8192];
    for (uint64_t t = prologue; t < nt; t++) {
        const uint64_t T0 = t * TB;
        for (uint32_t j = 0; j < NRT; j++) {
            uint32_t e = fsm_rec_ent(rec[t * NRT + j]);
            int64_t c = fsm_rec_cnt(rec[t * NRT + j]);
            if (j < HH_FSM_KM && fsm_fx_ok(fx[t * HH_FSM_KM + j])) {
                e = fsm_fx_ent(fx[t * HH_FSM_KM + j]);
                c += fsm_fx_d(fx[t * HH_FSM_KM + j]);
            }
            if (t == prologue && j == 0 && entry) *entry = e;
            const uint64_t R = T0 + (uint64_t)j * S;
            uint32_t k = 0;
            if (R + S <= bits) {
                // the kernels' fast path: K-bit steps, then the r-bit step
                uint32_t row = e << HH_FSM_ET_RSH(K);
                for (uint32_t q = 0; q + K <= S; q += K) {
                    const uint32_t v = (uint32_t)(((uint64_t)w[(R + q) >> 5] | (uint64_t)w[((R + q) >> 5) + 1] << 32) >>
                                                  ((R + q) & 31)) & ((1u << K) - 1u);
                    const uint64_t en = g_F.et[(row >> 3) + v];
                    for (uint32_t i = 0; i < HH_FSM_ET_NSYM(en); i++) buf[k++] = (uint8_t)(HH_FSM_ET_SYMS(en) >> (8 * i));
                    row = HH_FSM_ET_ROW(en);
                }
                if (r) {
                    const uint64_t q = R + S - r;
                    const uint32_t v = (uint32_t)(((uint64_t)w[q >> 5] | (uint64_t)w[(q >> 5) + 1] << 32) >> (q & 31)) &
                                       ((1u << r) - 1u);
                    const uint64_t en = g_F.er[((row >> HH_FSM_ET_RSH(K)) << r) + v];
                    for (uint32_t i = 0; i < HH_FSM_ET_NSYM(en); i++) buf[k++] = (uint8_t)(HH_FSM_ET_SYMS(en) >> (8 * i));
                    row = HH_FSM_ET_ROW(en);
                }
                if (R + S == bits && (row >> HH_FSM_ET_RSH(K)) != 0) buf[k++] = g_F.tsym[row >> HH_FSM_ET_RSH(K)];   // tail rule
                stats[7]++;
            } else {
                k = fsm_emit_serial(&F, w, R, R + S, bits, e, buf);
                stats[8]++;
            }
            if ((int64_t)k != c) {
                fprintf(stderr, "fsm emu: tile %llu region %d emitted %u, counted %lld\n", (unsigned long long)t, j, k,
                        (long long)c);
                return HH_ERR_INTERNAL;
            }
            if (o + k > cap) return HH_ERR_CAPACITY;
            memcpy(out + o, buf, k);
            o += k;
        }
    }
    if (leave) *leave = xs[nt - 1];
    g_rec = rec;
    g_xs = xs;
    g_fx = fx;
    g_tsum = tsum;
    return (int64_t)o;
}

// The count-pass arrays of the last hh_fsm_emu_decode (the kernels' layout).
int64_t hh_fsm_emu_arrays(uint32_t *rec, uint32_t *fx, int32_t *tsum, uint32_t *xs) {
    for (size_t i = 0; i < g_rec.size(); i++) rec[i] = g_rec[i];
    for (size_t i = 0; i < g_fx.size(); i++) fx[i] = g_fx[i];
    for (size_t i = 0; i < g_tsum.size(); i++) tsum[i] = (int32_t)g_tsum[i];
    for (size_t i = 0; i < g_xs.size(); i++) xs[i] = g_xs[i];
    return (int64_t)g_xs.size();
}

int64_t hh_fsm_emu_tables(const int32_t *izero, const int32_t *ione, const uint8_t *sym, int32_t nodes,
                          uint32_t S, uint32_t *info) {
    hh_tree tree = {nodes, izero, ione, sym};
    int rc = hh_tables_build(&tree, &g_T);
    if (rc) return rc;
    if (S == 0)
        S = hh_fsm_region_bits(hh_fsm_nstates(&g_T), (uint32_t)g_T.len_gcd,
                               hh_pick_region_bits((uint32_t)g_T.len_gcd));
    rc = hh_fsm_build(&g_T, S, g_K, &g_F);
    if (rc) return rc;
    info[0] = g_F.ns;
    info[1] = g_F.K;
    info[2] = g_F.r;
    info[3] = hh_fsm_pick_head(&g_T, S, g_F.cb);
    info[4] = g_F.cb;
    return HH_OK;
}

}  // extern "C"
