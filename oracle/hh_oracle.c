/*
 * hh_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY; see hh_oracle.h).
 *
 * Clean-room restatements of the reference's serial decoders.  Citations are
 * BeauJoh/HuffmanDecoderOnGPUs framework/<file>:<line>.
 */
#define _GNU_SOURCE
#include "hh_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

double or_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ------------------------------------------------------------------ */
/* Loader: huffdata.c:27-68 (HUFF, big-endian int32 header fields).    */
/* "HUFX" is the 64-bit sibling defined in DESIGN.md: int32 nodes,     */
/* int64 bits, int64 uncompressedsize; tree and payload unchanged.     */
/* ------------------------------------------------------------------ */
static int rd_be32(FILE *f, int32_t *v) {
    unsigned char b[4];
    if (fread(b, 1, 4, f) != 4) return -1;
    *v = (int32_t)(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) |
                   ((uint32_t)b[2] << 8) | (uint32_t)b[3]);
    return 0;
}
static int rd_be64(FILE *f, int64_t *v) {
    int32_t hi, lo;
    if (rd_be32(f, &hi) || rd_be32(f, &lo)) return -1;
    *v = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
    return 0;
}

void or_free_huff(or_huff *h) {
    if (!h) return;
    free(h->izero); free(h->ione); free(h->sym); free(h->data);
    memset(h, 0, sizeof(*h));
}

int or_load_huff(const char *path, or_huff *h) {
    memset(h, 0, sizeof(*h));
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char magic[4];
    int wide = 0;
    if (fread(magic, 1, 4, f) != 4) goto bad;
    if (memcmp(magic, "HUFF", 4) == 0) wide = 0;
    else if (memcmp(magic, "HUFX", 4) == 0) wide = 1;
    else goto bad;
    int32_t nodes;
    if (rd_be32(f, &nodes) || nodes <= 0) goto bad;
    if (wide) {
        if (rd_be64(f, &h->bits) || rd_be64(f, &h->uncompressedsize)) goto bad;
    } else {
        int32_t b, u;
        if (rd_be32(f, &b) || rd_be32(f, &u)) goto bad;
        h->bits = b; h->uncompressedsize = u;
    }
    if (h->bits < 0 || h->uncompressedsize < 0) goto bad;
    h->nodes = nodes;
    h->izero = (int32_t *)malloc(sizeof(int32_t) * (size_t)nodes);
    h->ione = (int32_t *)malloc(sizeof(int32_t) * (size_t)nodes);
    h->sym = (uint8_t *)malloc((size_t)nodes);
    for (int32_t i = 0; i < nodes; i++) {               /* huffdata.c:50-54 */
        if (fread(&h->sym[i], 1, 1, f) != 1) goto bad;
        if (rd_be32(f, &h->izero[i]) || rd_be32(f, &h->ione[i])) goto bad;
    }
    int64_t cb = (h->bits + 7) / 8;                      /* huffdata.c:55 */
    h->data = (uint8_t *)calloc((size_t)cb + 8, 1);      /* +pad, :58-61 */
    if (cb && fread(h->data, 1, (size_t)cb, f) != (size_t)cb) goto bad;
    fclose(f);
    return 0;
bad:
    fclose(f);
    or_free_huff(h);
    return -2;
}

static inline int bit_at(const uint8_t *d, int64_t p) {
    return (d[p >> 3] >> (p & 7)) & 1;   /* decodeallbits.cl:23, LSB-first */
}
static inline int is_leaf(const or_huff *h, int32_t n) {
    return h->izero[n] == -1;            /* decodeallbits.cl:21 */
}

/* ------------------------------------------------------------------ */
/* simpleDecode: mainrun.c:38-55.                                      */
/* ------------------------------------------------------------------ */
int64_t or_simple_decode(const or_huff *h, uint8_t *out, int64_t cap) {
    int64_t n = 0;
    int32_t node = 0;
    for (int64_t p = 0; p < h->bits; p++) {
        node = bit_at(h->data, p) ? h->ione[node] : h->izero[node];
        if (node < 0 || node >= h->nodes) return -1;
        if (h->izero[node] == -1 && h->ione[node] == -1) {
            if (n >= cap) return -1;
            out[n++] = h->sym[node];
            node = 0;
        }
    }
    return n;
}

/* ------------------------------------------------------------------ */
/* The pipeline's observable result, serially (pes.c:30-46 decodes    */
/* every bit; calcbitsindex/calcresult keep exactly the chain from bit */
/* 0; findmax sets the length).  A walk stops at a leaf or at the end  */
/* of the stream; in the latter case the internal node's sym byte is   */
/* the symbol (decodeallbits.cl:20-31).                                */
/* ------------------------------------------------------------------ */
int64_t or_chain_decode(const or_huff *h, uint8_t *out, int64_t cap) {
    if (h->nodes < 1 || is_leaf(h, 0)) return h->bits ? -1 : 0;
    int64_t n = 0, p = 0;
    while (p < h->bits) {
        int32_t node = 0;
        while (!is_leaf(h, node) && p < h->bits) {
            node = bit_at(h->data, p) ? h->ione[node] : h->izero[node];
            if (node < 0 || node >= h->nodes) return -1;
            p++;
        }
        if (n >= cap) return -1;
        out[n++] = h->sym[node];
    }
    return n;
}

/* ------------------------------------------------------------------ */
/* Stage oracle: pes.c:22-209, every array kept.                       */
/* ------------------------------------------------------------------ */
int64_t or_pes(const or_huff *h, uint8_t *bitdecode, int32_t *steps,
               int32_t *bitsindex, uint8_t *result, int32_t *nlevels) {
    const int64_t B = h->bits;
    if (B <= 0 || B > 0x7fffffff || is_leaf(h, 0)) return -1;
    /* initbitsindex: pes.c:22-28 */
    for (int64_t b = 0; b < B; b++) bitsindex[b] = -1;
    /* decodeAllBits: pes.c:30-46 (level 0 of steps = code length) */
    for (int64_t b = 0; b < B; b++) {
        int64_t p = b;
        int32_t node = 0;
        while (!is_leaf(h, node) && p < B) {
            node = bit_at(h->data, p) ? h->ione[node] : h->izero[node];
            p++;
        }
        bitdecode[b] = h->sym[node];
        steps[b] = (int32_t)(p - b);
    }
    /* makebigtable loop: pes.c:48-71, 146-161.  Serial order matters for
     * the one aliased read at b + s == B (it reads row step+1, entry 0,
     * already written in this pass), so keep ascending b. */
    int32_t step = 0, flag;
    do {
        if (step + 1 >= 25) return -1;            /* 25 rows, pes.c:131 */
        int32_t *cur = steps + (int64_t)step * B;
        int32_t *nxt = steps + (int64_t)(step + 1) * B;
        for (int64_t b = 0; b < B; b++) {
            int32_t s = cur[b];
            int32_t v;
            if (s == -1 || b + s > B) {
                v = -1;
            } else {
                int32_t w = cur[b + s];           /* may alias nxt[0] */
                v = (w == -1 || b + s + w > B) ? -1 : s + w;
            }
            nxt[b] = v;
        }
        flag = cur[0];                            /* pes.c:70 */
        step++;
    } while (flag != -1);
    *nlevels = step;
    /* calcbitsindex: pes.c:73-85, 174-185 */
    int32_t pw = 1 << (step - 1);
    bitsindex[0] = 0;
    while (step > 0) {
        const int32_t *lv = steps + (int64_t)(step - 1) * B;
        for (int64_t b = 0; b < B; b++) {
            int32_t off = lv[b], cv = bitsindex[b];
            if (off != -1 && cv != -1 && b + off < B) bitsindex[b + off] = cv + pw;
        }
        step--;
        pw >>= 1;
    }
    /* calcresult: pes.c:87-96 */
    for (int64_t b = 0; b < B; b++)
        if (bitsindex[b] != -1) result[bitsindex[b]] = bitdecode[b];
    /* findmax: pes.c:98-104 (the reference overwrites bitsindex[0]; we
     * report the value instead so the array stays inspectable) */
    int64_t b = B - 1;
    while (b > 0 && bitsindex[b] == -1) b--;
    return (int64_t)bitsindex[b] + 1;
}

/* ------------------------------------------------------------------ */
/* linApproach restatement: linapproach.c:110-282.                     */
/* Tables: one 2^J-entry table per "root": the tree root, every        */
/* internal node at a depth that is a positive multiple of J           */
/* (findroots, :16-30), and every internal node at depth 1..J-1        */
/* (findteleroots, :32-47).  An entry walks J bits from its root,      */
/* restarting at the tree root after each leaf (traverseLinTree,       */
/* :49-87).                                                            */
/* ------------------------------------------------------------------ */
typedef struct {
    union { int32_t val; uint8_t syms[8]; } u;
    int32_t l;
    uint8_t nsym;
} lin_elem;   /* sElement8, linapproach.h:13-21 (same 16-byte layout) */

typedef struct { int32_t *roots; int32_t *lev; int n, cap; } rootlist;

static void rl_push(rootlist *r, int32_t node, int32_t lev) {
    if (r->n == r->cap) {
        r->cap = r->cap ? 2 * r->cap : 64;
        r->roots = (int32_t *)realloc(r->roots, sizeof(int32_t) * (size_t)r->cap);
        r->lev = (int32_t *)realloc(r->lev, sizeof(int32_t) * (size_t)r->cap);
    }
    r->roots[r->n] = node;
    r->lev[r->n] = lev;
    r->n++;
}

/* nodes at depth k*J (k>=1) below `node`, pre-order, zero-branch first */
static void lin_deep_roots(const or_huff *h, int32_t node, int down, int J,
                           rootlist *r) {
    if (is_leaf(h, node)) return;
    if (down == 0) {
        rl_push(r, node, 0);
        down = J;
    }
    lin_deep_roots(h, h->izero[node], down - 1, J, r);
    lin_deep_roots(h, h->ione[node], down - 1, J, r);
}

/* internal nodes at depth 1..J-1 below the root, pre-order */
static void lin_tele_roots(const or_huff *h, int32_t node, int level, int down,
                           rootlist *r) {
    if (is_leaf(h, node) || down == 0) return;
    rl_push(r, node, level);
    lin_tele_roots(h, h->izero[node], level + 1, down - 1, r);
    lin_tele_roots(h, h->ione[node], level + 1, down - 1, r);
}

int64_t or_lin_decode(const or_huff *h, int J, uint8_t *out, int64_t cap) {
    if (J < 1 || J > 15 || is_leaf(h, 0)) return -1;
    const int32_t tsize = 1 << J;
    rootlist r = {0};
    rl_push(&r, 0, 0);
    lin_deep_roots(h, 0, J, J, &r);
    const int ndeep = r.n;
    lin_tele_roots(h, h->izero[0], 1, J - 1, &r);
    lin_tele_roots(h, h->ione[0], 1, J - 1, &r);

    int32_t *inv = (int32_t *)malloc(sizeof(int32_t) * (size_t)h->nodes);
    for (int i = 0; i < h->nodes; i++) inv[i] = 0;
    for (int i = 0; i < r.n; i++) inv[r.roots[i]] = i * tsize;

    lin_elem *tab = (lin_elem *)malloc(sizeof(lin_elem) * (size_t)r.n * (size_t)tsize);
    for (int t = 0; t < r.n; t++) {
        const int tele = t >= ndeep;
        const int tl = r.lev[t];
        for (int32_t code = 0; code < tsize; code++) {
            lin_elem *e = &tab[(int64_t)t * tsize + code];
            int32_t node = r.roots[t], back = 0, backnode = 0;
            int ns = 0;
            for (int pos = 0; pos < J;) {
                node = ((code >> pos) & 1) ? h->ione[node] : h->izero[node];
                pos++;
                if (tele && tl + pos == J) { back = J - pos; backnode = node; }
                if (is_leaf(h, node)) {
                    if (ns >= 8) { free(tab); free(inv); free(r.roots); free(r.lev); return -1; }
                    e->u.syms[ns++] = h->sym[node];
                    node = 0;
                }
            }
            if (ns > 0) {
                e->nsym = (uint8_t)ns;
                e->l = inv[node];
            } else {
                e->nsym = 0;
                e->l = tele ? back : 0;
                e->u.val = inv[tele ? backnode : node];
            }
        }
    }

    /* decode loop: linapproach.c:198-273 */
    const uint8_t *d = h->data;
    const uint32_t mask = (1u << J) - 1;
    int64_t cp = 0, n = 0;
    int64_t ap = 0;
    while (cp < h->bits) {
        uint32_t w = (uint32_t)d[cp >> 3] | ((uint32_t)d[(cp >> 3) + 1] << 8);
        if (J >= 8) w |= (uint32_t)d[(cp >> 3) + 2] << 16;
        ap += (w >> (cp & 7)) & mask;
        const lin_elem *e = &tab[ap];
        if (e->nsym == 0) {
            cp += J - e->l;
            ap = e->u.val;
        } else {
            if (n + e->nsym > cap) { n = -1; break; }
            for (int i = 0; i < e->nsym; i++) out[n++] = e->u.syms[i];
            ap = e->l;
            cp += J;
        }
    }
    free(tab); free(inv); free(r.roots); free(r.lev);
    return n;
}
