// hh_emu.cpp -- TEST-ONLY host emulation of the fused decode kernel.
//
// Runs the kernel's per-lane building blocks (hh_algo.h) on host arrays with
// the kernel's geometry -- tiles of HH_NL-1 regions, one auxiliary lane that
// decodes the next tile's first region, boundary masks, mask walks, tile
// transfer tables, ordered state application, the look-back's charged
// counts, emission -- so the stitching
// logic is checked against the oracle without a GPU.  Every lane's mask walk
// is also cross-checked against the plain two-pointer walk.  Nothing in the
// product links this file; it builds into tests/emu/libhh_emu.so.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hh_algo.h"
#include "hiphuff.h"

extern "C" {

// stats[0]=tiles stats[1]=walks with k>1 stats[2]=failed walks stats[3]=max k
int64_t hh_emu_decode(const int32_t *izero, const int32_t *ione, const uint8_t *sym,
                      int32_t nodes, const uint8_t *data, uint64_t bits, uint32_t S,
                      uint8_t *out, uint64_t cap, int64_t *stats) {
    const uint32_t NR = HH_NL - 1;
    hh_tree tree = {nodes, izero, ione, sym};
    static hh_tables T;   // large; not reentrant (test helper)
    int rc = hh_tables_build(&tree, &T);
    if (rc) return rc;
    for (int i = 0; i < 4; i++) stats[i] = 0;
    if (bits == 0) return 0;
    if (S < 2 || S > 32 * HH_MW_MAX) return HH_ERR_ARG;
    const uint64_t TB = (uint64_t)NR * S;
    const uint64_t ntiles = (bits + TB - 1) / TB;
    const uint64_t nbytes = (bits + 7) / 8;
    const uint32_t span = (HH_NL + HH_KM + 1) * S + 320;  // bits a tile may touch
    const uint32_t nw = span / 32 + 3;
    const uint32_t mw = (S + 31) / 32;
    std::vector<uint32_t> w(nw);
    std::vector<uint64_t> rec((size_t)ntiles * NR), tab((size_t)ntiles * HH_KM);
    std::vector<uint32_t> mask(HH_NL * mw);
    std::vector<uint16_t> mx(HH_NL), mn(HH_NL);
    std::vector<uint32_t> xs(HH_NL), ns(HH_NL);
    stats[0] = (int64_t)ntiles;

    auto load_tile = [&](uint64_t t, hh_ctx &c) {
        uint64_t b0 = t * TB;
        uint64_t w0 = b0 >> 5;
        for (uint32_t i = 0; i < nw; i++) {
            uint64_t byte = (w0 + i) * 4;
            uint32_t v = 0;
            for (int k = 0; k < 4; k++)
                if (byte + k < nbytes) v |= (uint32_t)data[byte + k] << (8 * k);
            w[i] = v;
        }
        c.w = w.data();
        c.sh = (uint32_t)(b0 & 31);
        c.l1 = T.l1;
        c.l2 = T.l2;
        c.tree = T.tree;
        c.tsym = T.tsym;
        uint64_t rem = bits - b0;
        c.bt = rem < span ? (uint32_t)rem : span;
    };

    for (uint64_t t = 0; t < ntiles; t++) {
        hh_ctx c;
        load_tile(t, c);
        for (uint32_t lane = 0; lane < HH_NL; lane++) {   // incl. the aux lane
            uint32_t p0 = lane * S;
            uint32_t n = 0, x = p0, n2 = 0;
            struct MS {
                uint32_t *m;
                void operator()(uint32_t wi, uint32_t v) { m[wi] = v; }
            } ms{&mask[lane * mw]};
            for (uint32_t w2 = 0; w2 < mw; w2++) mask[lane * mw + w2] = 0;
            if (p0 < c.bt) {
                x = hh_region_count(&c, p0, p0 + S, &n);
                uint32_t x2 = hh_region_count_mask(&c, p0, p0 + S, mw, &n2, ms);
                if (x2 != x || n2 != n) return HH_ERR_INTERNAL;
            }
            xs[lane] = x;
            ns[lane] = n;
            mx[lane] = (uint16_t)(x - p0);
            mn[lane] = (uint16_t)n;
        }
        hh_masks mk = {mask.data(), mx.data(), mn.data(), HH_NL, mw};
        for (uint32_t lane = 0; lane < NR; lane++) {
            hh_rec r, r2;
            hh_walk(&c, lane, S, xs[lane], &r);
            hh_walk_mask(&c, &mk, lane, S, xs[lane], &r2);
            if (r.k != r2.k || r.e != r2.e || r.delta != r2.delta || r.cov != r2.cov) {
                fprintf(stderr, "walk mismatch tile %lu lane %u: 2ptr k=%u e=%u d=%d cov=%u | mask k=%u e=%u d=%d cov=%u\n",
                        (unsigned long)t, lane, r.k, r.e, r.delta, r.cov, r2.k, r2.e, r2.delta, r2.cov);
                return HH_ERR_INTERNAL - 100;
            }
            r2.n = ns[lane];
            if (r2.k == 0) stats[2]++;
            if (r2.k > 1) stats[1]++;
            if ((int64_t)r2.k > stats[3]) stats[3] = r2.k;
            rec[t * NR + lane] = hh_rec_pack(r2);
        }
        hh_tile_table_seq(&rec[t * NR], NR, &tab[t * HH_KM]);
    }
    if (stats[2]) return HH_ERR_UNSUPPORTED;

    // ordered application of the tile tables (the kernel's look-back)
    std::vector<hh_state> st(ntiles + 1);
    st[0] = hh_state{0, 0, 0, 0};
    for (uint64_t t = 0; t < ntiles; t++) st[t + 1] = hh_xf_apply(&tab[t * HH_KM], st[t]);
    uint64_t total = st[ntiles].base;
    if (total > cap) return HH_ERR_CAPACITY;

    // The kernel's look-back sums CHARGED counts (each walk's delta charged
    // to the walker's tile: count_t(d) = sum over live lanes of n+cov+delta)
    // and starts tile t's first run delta_in(t) symbols before that prefix.
    {
        int64_t charged = 0;
        for (uint64_t t = 0; t < ntiles; t++) {
            if ((int64_t)st[t].base != charged - st[t].delta) return HH_ERR_INTERNAL - 200;
            for (uint32_t j = st[t].d; j < NR;) {
                hh_rec r = hh_rec_unpack(rec[t * NR + j]);
                charged += (int64_t)r.n + r.cov + r.delta;
                j = hh_rec_next(j, r);
            }
        }
        if (charged != (int64_t)total) return HH_ERR_INTERNAL - 201;
    }

    struct Sink {
        uint8_t *out;
        void operator()(uint64_t o, uint32_t b) { out[o] = (uint8_t)b; }
    } sink{out};
    for (uint64_t t = 0; t < ntiles; t++) {
        hh_ctx c;
        load_tile(t, c);
        hh_state s = st[t];
        uint32_t j = s.d, e_in = s.e;
        int32_t del_in = s.delta;
        uint64_t o = s.base;
        while (j < NR) {
            hh_rec r = hh_rec_unpack(rec[t * NR + j]);
            uint32_t nx = hh_rec_next(j, r);
            uint32_t start = j * S + e_in, end = nx * S + r.e;
            uint32_t pe = end < c.bt ? end : c.bt;
            uint64_t cnt = (uint64_t)((int64_t)r.n + r.cov + del_in);
            uint32_t p = start;
            uint64_t o0 = o;
            if (p < pe) hh_emit_run(&c, &p, pe, &o, total, sink);
            if (o - o0 != cnt) return HH_ERR_INTERNAL;   // count/emission disagree
            e_in = r.e;
            del_in = r.delta;
            j = nx;
        }
        if (o != st[t + 1].base) return HH_ERR_INTERNAL;
    }
    return (int64_t)total;
}

}  // extern "C"
