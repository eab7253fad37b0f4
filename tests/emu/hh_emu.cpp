// hh_emu.cpp -- TEST-ONLY host emulation of the decode kernel.
//
// Runs the kernel's per-lane building blocks (hh_algo.h) on host arrays with
// the kernel's geometry and LDS layout -- tiles of HH_NR regions staged as
// transposed word columns (plus HH_KM regions of the next tile), two-pointer
// walks across up to HH_KM regions, live masks and exceptions, the tile
// transfer table over the entering state, the resolved state chain between
// tiles and per-lane emission at the kernel's local offsets -- so the
// stitching logic is checked against the oracle without a GPU.  Every lane's
// emitted run is checked against its predicted count, every tile's output
// size against its table entry and every tile's base against the charged
// prefix.  Nothing in the product links this file; it builds into
// tests/emu/libhh_emu.so.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "hh_algo.h"
#include "hiphuff.h"


extern "C" {

// regions per tile of the emulated (and the kernel's) geometry
uint32_t hh_emu_regions(void) { return HH_NR; }


// stats[0]=tiles stats[1]=walks with k > 1 stats[2]=failed walks
// stats[3]=region bits used stats[4]=max k stats[5]=non-CONST tiles
// stats[6]=CONST prologue tiles stats[7]=CONST emitted tiles
// A segment: tiles [0, ntiles) (0 = all) of the bits at data, entered at
// in_state; *leave receives the state leaving the last tile (the kernel's
// hh_decode_device_range).
int64_t hh_emu_decode_range(const int32_t *izero, const int32_t *ione, const uint8_t *sym,
                            int32_t nodes, const uint8_t *data, uint64_t bits, uint32_t S,
                            uint64_t ntiles_req, uint64_t prologue, uint32_t in_state,
                            uint8_t *out, uint64_t cap, int64_t *stats, uint32_t *leave,
                            uint32_t *entry) {
    hh_tree tree = {nodes, izero, ione, sym};
    static hh_tables T;   // large; not reentrant (test helper)
    int rc = hh_tables_build(&tree, &T);
    if (rc) return rc;
    for (int i = 0; i < 8; i++) stats[i] = 0;
    if (S == 0) S = hh_pick_region_bits((uint32_t)T.len_gcd);
    stats[3] = S;
    uint32_t G = hh_pick_overlap(&T);
    if (getenv("HH_EMU_G") && !T.fixed_len) G = (uint32_t)atoi(getenv("HH_EMU_G"));
    if (G > HH_GMAX || G + 32 > S) G = 0;          // (the kernel's rule)
    if (leave) *leave = in_state;
    if (entry) *entry = in_state;
    if (bits == 0) return 0;
    if (S < 32 || S % 32 || S > 32 * HH_SW_MAX) return HH_ERR_ARG;
    const uint32_t sw = S / 32;
    const uint64_t TB = (uint64_t)HH_NR * S;
    const uint64_t all = (bits + TB - 1) / TB;
    const uint64_t ntiles = ntiles_req && ntiles_req < all ? ntiles_req : all;
    const uint64_t nbytes = (bits + 7) / 8;
    const uint32_t span = HH_NCOL * S;
    std::vector<uint32_t> w((size_t)sw * HH_NLS);
    std::vector<uint32_t> xs(HH_NR), ys(HH_NR), ns(HH_NR), mem(HH_NR), ent(HH_NR);
    // k_walk's staging of a deferred walk: words g0 .. g0 + nwin of the tile
    // at LDS index (g - g0) * 64 + lane (emulated for lane 0)
    const uint32_t fw = getenv("HH_FRONT_WALK") ? (uint32_t)atoi(getenv("HH_FRONT_WALK")) : HH_FRONT_WALK;
    std::vector<uint32_t> win((size_t)(HH_NCOL * HH_SW_MAX + 8) * 64);
    int64_t ndefer = 0;
    std::vector<uint16_t> n16(HH_NR);
    std::vector<uint32_t> l1m(HH_L1_SIZE), l1s(HH_L1_SIZE);   // split L1, as staged in LDS
    for (uint32_t i = 0; i < HH_L1_SIZE; i++) {
        l1m[i] = (uint32_t)(T.l1[i] >> 32);
        l1s[i] = (uint32_t)T.l1[i];
    }
    std::vector<uint32_t> mk((size_t)sw * HH_NLS);   // boundary masks (transposed like w)
    std::vector<uint64_t> hd(HH_NR);                 // overlap heads (hh_region_head)
    std::vector<int32_t> din(HH_NR);
    std::vector<hh_wk> wk(HH_NR);
    stats[0] = (int64_t)ntiles;
    // HH_EMU_HIST: walk-length statistics (lookups per lane, longest per tile)
    const bool hist = getenv("HH_EMU_HIST") != nullptr;
    std::vector<uint64_t> hl(1025, 0), ht(1025, 0);

    auto word_at = [&](uint64_t gw) -> uint32_t {
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) {
            uint64_t byte = gw * 4 + k;
            if (byte < nbytes) v |= (uint32_t)data[byte] << (8 * k);
        }
        return v;
    };

    uint64_t base = 0;                            // P_0 of the tile
    uint32_t st_in = in_state;                    // resolved entering state
    // charged prefix of tiles < t, + the entry correction (carried by the
    // last prologue tile's counts when there is a prologue)
    int64_t excl = prologue ? 0 : hh_state_delta(in_state);
    for (uint64_t t = 0; t < ntiles; t++) {
        hh_ctx c;
        const uint64_t tw0 = t * TB / 32;
        for (uint32_t col = 0; col < HH_NCOL; col++)          // the kernel's staging
            for (uint32_t k = 0; k < sw; k++) w[k * HH_NLS + col] = word_at(tw0 + (uint64_t)col * sw + k);
        c.w = w.data();
        c.sw = sw;
        c.nls = HH_NLS;
        c.magic = hh_magic(sw);
        c.l1m = l1m.data();
        c.l1s = l1s.data();
        c.l1 = nullptr;
        c.l2 = T.l2;
        c.tree = T.tree;
        c.tsym = T.tsym;
        c.maxadv = T.maxlen > HH_P ? (uint32_t)T.maxlen : HH_P;
        c.G = G;
        const uint64_t rem = bits - t * TB;
        c.bt = rem < span ? (uint32_t)rem : span;
        const uint32_t bt = c.bt;
        // the front kernels' context: lookups through F (no symbol bytes)
        hh_ctx cf = c;
        cf.f = T.f;
        cf.fdir = T.fdir;
        cf.pf = HH_PF;
        if (cf.maxadv < HH_PF) cf.maxadv = HH_PF;

        for (size_t i = 0; i < mk.size(); i++)          // words pass 1 leaves unwritten
            mk[i] = (uint32_t)(0x9e3779b9u * (uint32_t)(i + t * 7919u + 1));   // hold junk
        for (uint32_t j = 0; j < HH_NR; j++) {            // pass 1 (head, then count)
            uint32_t p0 = j * S, n = 0, x = bt, y = p0;
            hd[j] = 0;
            if (p0 < bt) {
                if (j > 0 && G) y = hh_region_head(&cf, p0 - G, p0, &hd[j]);
                uint32_t lim = p0 + S < bt ? p0 + S : bt;
                x = y < lim ? hh_region_count(&cf, y, lim, &n, mk.data()) : y;
            }
            xs[j] = x;
            ys[j] = p0 < bt ? y : bt;
            ns[j] = n;
            n16[j] = (uint16_t)n;
        }
        for (uint32_t j = 0; j < HH_NR; j++) {            // merges at the exit, else walks
            const uint32_t R1 = (j + 1) * S;
            // the kernel's rule: chain j's exit is chain j+1's entry point
            const uint32_t ynext = j + 1 < HH_NR ? ys[j + 1] : R1;
            const bool merged = R1 < bt && xs[j] == ynext;
            // the round-1 rule it replaces (boundary masks in the overlap window)
            const bool wmerged = G && j + 1 < HH_NR && R1 < bt && hh_window_merge(&c, mk.data(), hd[j + 1], R1);
            if (wmerged && !merged) return HH_ERR_INTERNAL - 501;
            // reference result: the mask walk over the whole tile
            const hh_wk ref = merged ? hh_wk{1u, xs[j] - R1, 0u, 0, 0u, 0u}
                                     : hh_walk(&c, j, S, xs[j], mk.data(), xs.data(), n16.data(), HH_NR);
            if (merged) {
                wk[j] = ref;
                continue;
            }
            // the kernel's: a two-pointer walk of at most fw lookups in k_front,
            // else again from the exit in k_walk over its own staging
            wk[j] = hh_walk(&cf, j, S, xs[j], nullptr, nullptr, nullptr, 0, fw, ys.data(), HH_NR);
            {
                // k_walk's form of every walk: exits and counts of the regions
                // it may reach (pass 1 of this tile; regions of the next tile
                // from their own heads), then exit comparisons over k_walk's
                // staging of the lane's words
                uint32_t xr[HH_KM + 1], nr[HH_KM + 1];
                for (uint32_t k = 1; k <= HH_KM; k++) {
                    const uint32_t rg = j + k, R = rg * S;
                    if (rg < HH_NR) { xr[k] = xs[rg]; nr[k] = ns[rg]; continue; }
                    uint32_t yy = R < bt ? R : bt, nn = 0, xx = yy;
                    if (R < bt && G && rg % HH_NR) yy = hh_region_head(&cf, R - G, R, nullptr);
                    const uint32_t lim = R + S < bt ? R + S : bt;
                    if (yy < lim) xx = hh_region_count(&cf, yy, lim, &nn);
                    xr[k] = xx;
                    nr[k] = nn;
                }
                const uint32_t g0 = (j + 1) * sw >= 2 ? (j + 1) * sw - 2 : 0;
                const uint32_t nwin = 2 + HH_KM * sw + 4;
                for (uint32_t q = 0; q < nwin; q++) win[(size_t)(g0 + q) * 64] = word_at(tw0 + g0 + q);
                hh_ctx cw = cf;
                cw.w = win.data();
                cw.sw = 1024;
                cw.nls = 64;
                const hh_wk we = hh_walk_exits(&cw, j, S, xs[j], xr, nr);
                if (we.k != ref.k || (ref.k && (we.e != ref.e || we.cov != ref.cov || we.delta != ref.delta))) {
                    fprintf(stderr, "emu: tile %lu lane %u exit walk (k %u e %u cov %u delta %d) vs mask walk (k %u e %u cov %u delta %d)\n",
                            (unsigned long)t, j, we.k, we.e, we.cov, we.delta, ref.k, ref.e, ref.cov, ref.delta);
                    return HH_ERR_INTERNAL - 502;
                }
                if (wk[j].more) {
                    ndefer++;
                    wk[j] = we;
                }
            }
            if (wk[j].k != ref.k || (ref.k && (wk[j].e != ref.e || wk[j].cov != ref.cov || wk[j].delta != ref.delta))) {
                fprintf(stderr, "emu: tile %lu lane %u walk (k %u e %u cov %u delta %d) vs mask walk (k %u e %u cov %u delta %d)\n",
                        (unsigned long)t, j, wk[j].k, wk[j].e, wk[j].cov, wk[j].delta, ref.k, ref.e, ref.cov, ref.delta);
                return HH_ERR_INTERNAL - 500;
            }
            if (wk[j].k == 0) stats[2]++;
            if (wk[j].k > 1) stats[1]++;
            if ((int64_t)wk[j].k > stats[4]) stats[4] = wk[j].k;
        }
        if (stats[2]) return HH_ERR_UNSUPPORTED;
        if (hist) {
            uint32_t mx = 0;
            for (uint32_t j = 0; j < HH_NR; j++) {
                const uint32_t s = wk[j].steps < 1024 ? wk[j].steps : 1024;
                hl[s]++;
                mx = s > mx ? s : mx;
            }
            ht[mx]++;
        }
        // transfer table
        for (uint32_t j = 0; j < HH_NR; j++) mem[j] = hh_mem_init(j);
        for (uint32_t j = 0; j < HH_NR; j++)              // exceptions, ascending
            for (uint32_t q = j + 1; q < j + wk[j].k && q < HH_NR; q++) mem[q] &= ~mem[j];
        int32_t cnt[HH_KM];
        uint32_t ost[HH_KM];
        int nlast[HH_KM];
        for (uint32_t d = 0; d < HH_KM; d++) { cnt[d] = 0; nlast[d] = 0; ost[d] = 0; }
        for (uint32_t j = 0; j < HH_NR; j++) {
            const int32_t ch = (int32_t)(ns[j] + wk[j].cov) + wk[j].delta;
            for (uint32_t d = 0; d < HH_KM; d++) {
                if (!((mem[j] >> d) & 1u)) continue;
                cnt[d] += ch;
                if (j + wk[j].k >= HH_NR) {
                    ost[d] = hh_state_pack(j + wk[j].k - HH_NR, wk[j].e, wk[j].delta);
                    nlast[d]++;
                }
            }
        }
        bool cst = true;
        for (uint32_t d = 0; d < HH_KM; d++) {
            if (nlast[d] != 1) return HH_ERR_INTERNAL - 400;
            if (hh_tab_state(hh_tab_pack(cnt[d], ost[d])) != ost[d] ||
                hh_tab_count(hh_tab_pack(cnt[d], ost[d])) != cnt[d])
                return HH_ERR_INTERNAL - 401;                // field overflow
            if (ost[d] != ost[0]) cst = false;
        }
        if (!cst) stats[5]++;
        if (cst) stats[t < prologue ? 6 : 7]++;
        if (t < prologue) {                               // prologue tile: state only
            const uint32_t so = ost[hh_state_d(st_in)];
            excl += t + 1 == prologue ? hh_state_delta(so) : 0;
            st_in = so;
            continue;
        }
        if (t == prologue && entry) *entry = st_in;
        // entering state -> live lanes, entries, run counts
        const uint32_t d_t = hh_state_d(st_in), e_t = hh_state_e(st_in);
        const int32_t dprev = hh_state_delta(st_in);
        if ((int64_t)base != excl - dprev) return HH_ERR_INTERNAL - 300;
        for (uint32_t j = 0; j < HH_NR; j++) { ent[j] = 0; din[j] = 0; }
        ent[d_t] = d_t * S + e_t;
        din[d_t] = dprev;
        for (uint32_t j = 0; j < HH_NR; j++)
            if (((mem[j] >> d_t) & 1u) && j + wk[j].k < HH_NR) {
                ent[j + wk[j].k] = (j + wk[j].k) * S + wk[j].e;
                din[j + wk[j].k] = wk[j].delta;
            }
        uint64_t o = base;
        for (uint32_t j = 0; j < HH_NR; j++) {            // emission
            if (!((mem[j] >> d_t) & 1u)) continue;
            const uint32_t pe0 = (j + wk[j].k) * S + wk[j].e;
            const uint32_t pe = pe0 < bt ? pe0 : bt;
            const uint64_t want = (uint64_t)((int64_t)ns[j] + wk[j].cov + din[j]);
            hh_cur cu = hh_cur_at(&c, ent[j]);
            const uint64_t o0 = o;
            while (cu.p < pe) {
                uint32_t val, k;
                hh_emit_step(&c, cu, pe, o, ~0ull, &val, &k);
                for (uint32_t i = 0; i < k; i++) {
                    if (o + i >= cap) return HH_ERR_CAPACITY;
                    out[o + i] = (uint8_t)(val >> (8 * i));
                }
                o += k;
            }
            if (o - o0 != want || (cu.p != pe && !(cu.p >= pe && ent[j] >= pe))) {
                fprintf(stderr, "emu: tile %lu lane %u emitted %lu, predicted %lu (e=%u pe=%u p=%u)\n",
                        (unsigned long)t, j, (unsigned long)(o - o0), (unsigned long)want, ent[j], pe, cu.p);
                return HH_ERR_INTERNAL;
            }
        }
        const uint32_t so = ost[d_t];
        const int64_t tout = (int64_t)cnt[d_t] - hh_state_delta(so) + dprev;
        if (getenv("HH_EMU_TILE") && (uint64_t)atoll(getenv("HH_EMU_TILE")) == t) {
            fprintf(stderr, "tile %lu: in 0x%x base %lu excl %ld cnt0 %d out0 0x%x tout %ld\n",
                    (unsigned long)t, st_in, (unsigned long)base, (long)excl, cnt[0], ost[0], (long)tout);
            for (uint32_t j = HH_NR - 10; j < HH_NR; j++)
                fprintf(stderr, "  lane %u n %u x %u k %u e %u cov %u delta %d mem %x\n", j, ns[j], xs[j],
                        wk[j].k, wk[j].e, wk[j].cov, wk[j].delta, mem[j]);
        }
        if ((int64_t)(o - base) != tout) return HH_ERR_INTERNAL - 2;
        excl += cnt[d_t];
        base = o;
        st_in = so;
    }
    if (leave) *leave = st_in;
    if (hist) {
        fprintf(stderr, "deferred %ld of %lu lanes\n", (long)ndefer, (unsigned long)(ntiles * HH_NR));
        for (uint32_t b = 0; b <= 1024; b++)
            if (hl[b] || ht[b]) fprintf(stderr, "hist %u lanes %lu tiles %lu\n", b, (unsigned long)hl[b], (unsigned long)ht[b]);
    }
    return (int64_t)base;
}

int64_t hh_emu_decode(const int32_t *izero, const int32_t *ione, const uint8_t *sym,
                      int32_t nodes, const uint8_t *data, uint64_t bits, uint32_t S,
                      uint8_t *out, uint64_t cap, int64_t *stats) {
    return hh_emu_decode_range(izero, ione, sym, nodes, data, bits, S, 0, 0, hh_state_pack(0, 0, 0),
                               out, cap, stats, nullptr, nullptr);
}

}  // extern "C"
