/*
 * hh_huff.c -- .huff container, tree validation, encoder and decode-table
 * construction (host C).
 *
 * Container: the reference's loadHuffFile (framework/huffdata.c:27-68) reads
 * "HUFF", big-endian int32 nodes/bits/uncompressedsize, nodes x 9-byte
 * {u8 sym, be-i32 izero, be-i32 ione} and ceil(bits/8) payload bytes.  The
 * int32 bit count caps a file at 256 MiB of payload (huffdata.c:41-43), so
 * "HUFX" widens bits and uncompressedsize to be-i64 and keeps the rest.
 */
#include "hiphuff.h"
#include "hh_internal.h"
#include "hh_fsm.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

const char *hh_strerror(int s) {
    switch (s) {
    case HH_OK: return "ok";
    case HH_ERR_ARG: return "bad argument";
    case HH_ERR_IO: return "i/o error";
    case HH_ERR_FORMAT: return "not a HUFF/HUFX file";
    case HH_ERR_TREE: return "invalid code tree";
    case HH_ERR_CAPACITY: return "output buffer too small";
    case HH_ERR_DEVICE: return "HIP runtime error";
    case HH_ERR_NOMEM: return "out of memory";
    case HH_ERR_INTERNAL: return "internal error";
    case HH_ERR_TIMEOUT: return "in-kernel wait timed out";
    case HH_ERR_UNSUPPORTED: return "unsupported input";
    default: return "unknown status";
    }
}

/* ------------------------------------------------------------------ */
/* container                                                           */
/* ------------------------------------------------------------------ */
static int rd32(FILE *f, uint32_t *v) {
    unsigned char b[4];
    if (fread(b, 1, 4, f) != 4) return -1;
    *v = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
    return 0;
}
static int rd64(FILE *f, uint64_t *v) {
    uint32_t hi, lo;
    if (rd32(f, &hi) || rd32(f, &lo)) return -1;
    *v = ((uint64_t)hi << 32) | lo;
    return 0;
}
static int wr32(FILE *f, uint32_t v) {
    unsigned char b[4] = {(unsigned char)(v >> 24), (unsigned char)(v >> 16),
                          (unsigned char)(v >> 8), (unsigned char)v};
    return fwrite(b, 1, 4, f) == 4 ? 0 : -1;
}
static int wr64(FILE *f, uint64_t v) {
    return wr32(f, (uint32_t)(v >> 32)) || wr32(f, (uint32_t)v) ? -1 : 0;
}

void hh_huff_free(hh_huff *h) {
    if (!h) return;
    free(h->izero);
    free(h->ione);
    free(h->sym);
    free(h->data);
    memset(h, 0, sizeof(*h));
}

hh_tree hh_huff_tree(const hh_huff *h) {
    hh_tree t = {h->nodes, h->izero, h->ione, h->sym};
    return t;
}

int hh_huff_load(const char *path, hh_huff *h) {
    if (!path || !h) return HH_ERR_ARG;
    memset(h, 0, sizeof(*h));
    FILE *f = fopen(path, "rb");
    if (!f) return HH_ERR_IO;
    int rc = HH_ERR_FORMAT;
    char magic[4];
    uint32_t nodes;
    if (fread(magic, 1, 4, f) != 4) goto out;
    if (!memcmp(magic, "HUFF", 4)) {
        uint32_t b, u;
        if (rd32(f, &nodes) || rd32(f, &b) || rd32(f, &u)) goto out;
        if ((int32_t)b < 0 || (int32_t)u < 0) goto out;
        h->bits = b;
        h->uncompressedsize = u;
        h->wide = 0;
    } else if (!memcmp(magic, "HUFX", 4)) {
        if (rd32(f, &nodes) || rd64(f, &h->bits) || rd64(f, &h->uncompressedsize)) goto out;
        if ((int64_t)h->bits < 0 || (int64_t)h->uncompressedsize < 0) goto out;
        h->wide = 1;
    } else {
        goto out;
    }
    if ((int32_t)nodes <= 0) goto out;
    h->nodes = (int32_t)nodes;
    h->izero = (int32_t *)malloc(sizeof(int32_t) * nodes);
    h->ione = (int32_t *)malloc(sizeof(int32_t) * nodes);
    h->sym = (uint8_t *)malloc(nodes);
    if (!h->izero || !h->ione || !h->sym) { rc = HH_ERR_NOMEM; goto out; }
    for (uint32_t i = 0; i < nodes; i++) {
        uint32_t a, b;
        if (fread(&h->sym[i], 1, 1, f) != 1 || rd32(f, &a) || rd32(f, &b)) goto out;
        h->izero[i] = (int32_t)a;
        h->ione[i] = (int32_t)b;
    }
    uint64_t cb = (h->bits + 7) / 8;
    h->data = (uint8_t *)calloc(cb + HH_PAYLOAD_PAD, 1);
    if (!h->data) { rc = HH_ERR_NOMEM; goto out; }
    if (cb && fread(h->data, 1, cb, f) != cb) goto out;
    rc = HH_OK;
out:
    fclose(f);
    if (rc != HH_OK) hh_huff_free(h);
    return rc;
}

int hh_huff_save(const char *path, const hh_huff *h) {
    if (!path || !h || h->nodes <= 0) return HH_ERR_ARG;
    FILE *f = fopen(path, "wb");
    if (!f) return HH_ERR_IO;
    int wide = h->wide || h->bits > 0x7fffffffull || h->uncompressedsize > 0x7fffffffull;
    int bad = 0;
    bad |= fwrite(wide ? "HUFX" : "HUFF", 1, 4, f) != 4;
    bad |= wr32(f, (uint32_t)h->nodes);
    if (wide) {
        bad |= wr64(f, h->bits);
        bad |= wr64(f, h->uncompressedsize);
    } else {
        bad |= wr32(f, (uint32_t)h->bits);
        bad |= wr32(f, (uint32_t)h->uncompressedsize);
    }
    for (int32_t i = 0; i < h->nodes && !bad; i++) {
        bad |= fwrite(&h->sym[i], 1, 1, f) != 1;
        bad |= wr32(f, (uint32_t)h->izero[i]);
        bad |= wr32(f, (uint32_t)h->ione[i]);
    }
    uint64_t cb = (h->bits + 7) / 8;
    if (!bad && cb) bad |= fwrite(h->data, 1, cb, f) != cb;
    bad |= fclose(f) != 0;
    return bad ? HH_ERR_IO : HH_OK;
}

/* ------------------------------------------------------------------ */
/* tree                                                                */
/* ------------------------------------------------------------------ */
static int gcd_i(int a, int b) {
    while (b) { int t = a % b; a = b; b = t; }
    return a;
}

/* Iterative DFS from the root: every reachable node is a leaf (both
 * children -1) or has two in-range children; no node is reached twice. */
int hh_tree_check(const hh_tree *t, hh_tree_info *info) {
    if (!t || t->nodes <= 0 || !t->izero || !t->ione || !t->sym) return HH_ERR_ARG;
    const int32_t n = t->nodes;
    uint8_t *seen = (uint8_t *)calloc((size_t)n, 1);
    /* every pop of an unseen node pushes two: at most 2n + 1 entries */
    int32_t *stk = (int32_t *)malloc(sizeof(int32_t) * 2 * (2 * (size_t)n + 2));
    int32_t *dep = stk + 2 * (size_t)n + 2;
    if (!seen || !stk) { free(seen); free(stk); return HH_ERR_NOMEM; }
    hh_tree_info in = {0, 0, 1 << 30, 0, 0};
    int sp = 0, rc = HH_OK;
    stk[sp] = 0; dep[sp] = 0; sp++;
    while (sp) {
        sp--;
        int32_t v = stk[sp], d = dep[sp];
        if (v < 0 || v >= n || seen[v]) { rc = HH_ERR_TREE; break; }
        seen[v] = 1;
        in.reachable++;
        int32_t a = t->izero[v], b = t->ione[v];
        if (a == -1 && b == -1) {
            in.leaves++;
            if (d < in.minlen) in.minlen = d;
            if (d > in.maxlen) in.maxlen = d;
            in.len_gcd = gcd_i(in.len_gcd, d);
            continue;
        }
        if (a < 0 || b < 0 || a >= n || b >= n) { rc = HH_ERR_TREE; break; }
        stk[sp] = a; dep[sp] = d + 1; sp++;
        stk[sp] = b; dep[sp] = d + 1; sp++;
    }
    free(seen);
    free(stk);
    if (rc == HH_OK && in.minlen == 0) rc = HH_ERR_TREE;   /* root is a leaf */
    if (info) *info = in;
    return rc;
}

/* ------------------------------------------------------------------ */
/* encoder                                                             */
/* ------------------------------------------------------------------ */
typedef struct { uint64_t code[256]; uint8_t len[256]; uint8_t have[256]; } codebook;

static int build_codebook(const hh_tree *t, codebook *cb) {
    hh_tree_info in;
    int rc = hh_tree_check(t, &in);
    if (rc) return rc;
    if (in.maxlen > 64) return HH_ERR_UNSUPPORTED;
    memset(cb, 0, sizeof(*cb));
    int32_t *stk = (int32_t *)malloc(sizeof(int32_t) * (size_t)t->nodes);
    uint64_t *cs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)t->nodes);
    uint8_t *ls = (uint8_t *)malloc((size_t)t->nodes);
    if (!stk || !cs || !ls) { free(stk); free(cs); free(ls); return HH_ERR_NOMEM; }
    int sp = 0;
    stk[sp] = 0; cs[sp] = 0; ls[sp] = 0; sp++;
    while (sp) {
        sp--;
        int32_t v = stk[sp];
        uint64_t c = cs[sp];
        uint8_t l = ls[sp];
        if (t->izero[v] == -1) {
            uint8_t s = t->sym[v];
            /* first (shallowest-visited) leaf wins for duplicate syms */
            if (!cb->have[s] || l < cb->len[s]) {
                cb->have[s] = 1; cb->code[s] = c; cb->len[s] = l;
            }
            continue;
        }
        stk[sp] = t->ione[v]; cs[sp] = c | (1ull << l); ls[sp] = (uint8_t)(l + 1); sp++;
        stk[sp] = t->izero[v]; cs[sp] = c; ls[sp] = (uint8_t)(l + 1); sp++;
    }
    free(stk); free(cs); free(ls);
    return HH_OK;
}

/* The code table for the device encoder (csrc/hh_encode.hip): len 0 for a
 * symbol absent from the tree. */
int hh_codebook(const void *tv, uint64_t code[256], uint8_t len[256]) {
    codebook cb;
    int rc = build_codebook((const hh_tree *)tv, &cb);
    if (rc) return rc;
    for (int i = 0; i < 256; i++) {
        if (cb.have[i] && cb.len[i] == 0) return HH_ERR_UNSUPPORTED;   /* (a one-leaf tree: codes of no bits) */
        code[i] = cb.code[i];
        len[i] = cb.have[i] ? cb.len[i] : 0;
    }
    return HH_OK;
}

uint64_t hh_encode_bound(const hh_tree *t, uint64_t n) {
    hh_tree_info in;
    if (hh_tree_check(t, &in)) return 0;
    return (n * (uint64_t)in.maxlen + 7) / 8 + 16;
}

int hh_encode(const hh_tree *t, const uint8_t *syms, uint64_t n, uint8_t *out,
              uint64_t *bits) {
    if (!t || (!syms && n) || !out || !bits) return HH_ERR_ARG;
    codebook cb;
    int rc = build_codebook(t, &cb);
    if (rc) return rc;
    uint64_t acc = 0, pos = 0;   /* acc holds `fill` pending bits */
    unsigned fill = 0;
    uint64_t ob = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint8_t s = syms[i];
        if (!cb.have[s]) return HH_ERR_ARG;
        uint64_t c = cb.code[s];
        unsigned l = cb.len[s];
        /* split codes so the accumulator never overflows */
        while (l) {
            unsigned take = l < 32 ? l : 32;
            acc |= (c & ((1ull << take) - 1)) << fill;
            fill += take;
            c >>= take;
            l -= take;
            pos += take;
            while (fill >= 8) {
                out[ob++] = (uint8_t)acc;
                acc >>= 8;
                fill -= 8;
            }
        }
    }
    if (fill) out[ob++] = (uint8_t)acc;
    *bits = pos;
    return HH_OK;
}

/* ------------------------------------------------------------------ */
/* decode tables (layout in hh_internal.h)                             */
/* ------------------------------------------------------------------ */
typedef struct {
    const hh_tree *t;
    int32_t *cid;     /* original node -> compact id, -1 unvisited */
    hh_tables *out;
} tb_ctx;

/* compact ids in BFS order so the root is 0 */
static int compact_tree(tb_ctx *c) {
    const hh_tree *t = c->t;
    int32_t *q = (int32_t *)malloc(sizeof(int32_t) * (size_t)t->nodes);
    if (!q) return HH_ERR_NOMEM;
    for (int32_t i = 0; i < t->nodes; i++) c->cid[i] = -1;
    int32_t qh = 0, qt = 0, next = 0;
    q[qt++] = 0;
    c->cid[0] = next++;
    while (qh < qt) {
        int32_t v = q[qh++];
        if (t->izero[v] == -1) continue;
        int32_t ch[2] = {t->izero[v], t->ione[v]};
        for (int k = 0; k < 2; k++) {
            if (c->cid[ch[k]] < 0) {
                if (next > HH_TREE_MAX) { free(q); return HH_ERR_UNSUPPORTED; }
                c->cid[ch[k]] = next++;
                q[qt++] = ch[k];
            }
        }
    }
    for (int32_t i = 0; i < qt; i++) {
        int32_t v = q[i], id = c->cid[v];
        c->out->tsym[id] = t->sym[v];
        if (t->izero[v] == -1) {
            c->out->tree[id] = HH_T_LEAF | t->sym[v];
        } else {
            c->out->tree[id] = (uint32_t)c->cid[t->izero[v]] |
                               ((uint32_t)c->cid[t->ione[v]] << 15);
        }
    }
    c->out->tree_used = (uint32_t)qt;
    free(q);
    return HH_OK;
}

static inline int tleaf(const hh_tables *T, uint32_t id) { return (T->tree[id] & HH_T_LEAF) != 0; }
static inline uint32_t tchild(const hh_tables *T, uint32_t id, unsigned bit) {
    return bit ? (T->tree[id] >> 15) & 0x7fff : T->tree[id] & 0x7fff;
}

static int subtree_height(const hh_tables *T, uint32_t id, int cap) {
    if (tleaf(T, id) || cap == 0) return 0;
    int a = subtree_height(T, tchild(T, id, 0), cap - 1);
    int b = subtree_height(T, tchild(T, id, 1), cap - 1);
    return 1 + (a > b ? a : b);
}

int hh_tables_build(const void *tree_v, hh_tables *T) {
    const hh_tree *t = (const hh_tree *)tree_v;
    hh_tree_info in;
    int rc = hh_tree_check(t, &in);
    if (rc) return rc;
    memset(T, 0, sizeof(*T));
    T->minlen = in.minlen;
    T->maxlen = in.maxlen;
    T->len_gcd = in.len_gcd;
    T->fixed_len = in.minlen == in.maxlen ? in.minlen : 0;
    tb_ctx c = {t, (int32_t *)malloc(sizeof(int32_t) * (size_t)t->nodes), T};
    if (!c.cid) return HH_ERR_NOMEM;
    rc = compact_tree(&c);
    free(c.cid);
    if (rc) return rc;

    /* L1: walk HH_P bits of the index, collect up to HH_K complete symbols */
    for (uint32_t w = 0; w < HH_L1_SIZE; w++) {
        uint32_t node = 0, syms = 0, nsym = 0, nbits = 0, len0 = 0, bmask = 0;
        unsigned pos = 0, start = 0;
        while (pos < HH_P && nsym < HH_K) {
            node = tchild(T, node, (w >> pos) & 1);
            pos++;
            if (tleaf(T, node)) {
                syms |= (uint32_t)T->tsym[node] << (8 * nsym);
                bmask |= 1u << start;
                if (nsym == 0) len0 = pos - start;
                nsym++;
                nbits = pos;
                node = 0;
                start = pos;
            }
        }
        uint64_t e;
        if (nsym) {
            e = (uint64_t)syms | ((uint64_t)nbits << 32) | ((uint64_t)nsym << 37) |
                ((uint64_t)len0 << 40) | ((uint64_t)bmask << 45);
        } else {
            /* node is the internal node at depth HH_P on the path of w */
            int q = subtree_height(T, node, HH_Q_MAX);
            uint32_t base = T->l2_used;
            if (base + (1u << q) > HH_L2_MAX) {
                /* out of L2 room: q = 0 subtable = one "walk from node" entry */
                q = 0;
                if (base + 1 > HH_L2_MAX) return HH_ERR_UNSUPPORTED;
            }
            for (uint32_t j = 0; j < (1u << q); j++) {
                uint32_t v = node, d = 0;
                while (d < (uint32_t)q && !tleaf(T, v)) {
                    v = tchild(T, v, (j >> d) & 1);
                    d++;
                }
                if (tleaf(T, v)) {
                    T->l2[base + j] = HH_L2_LEAF | T->tsym[v] | ((HH_P + d) << 8);
                } else {
                    T->l2[base + j] = v;   /* walk from v at depth HH_P+q */
                }
            }
            T->l2_used = base + (1u << q);
            /* the subtable reference sits in both halves: the meta half's
             * nsym field stays 0 (escape), so a pass that stages only the
             * meta half (the front kernel) still finds its subtable */
            e = (uint64_t)base | ((uint64_t)q << 16) |
                ((uint64_t)(((uint32_t)base << 8) | ((uint32_t)q << 24)) << 32);
        }
        T->l1[w] = e;
    }

    /* F (the front kernel's table): every complete symbol of HH_PF bits */
    int16_t slot[HH_L1_SIZE];
    for (uint32_t i = 0; i < HH_L1_SIZE; i++) slot[i] = -1;
    for (uint32_t w = 0; w < HH_F_SIZE; w++) {
        uint32_t node = 0, nbits = 0, bm = 0;
        unsigned pos = 0, start = 0;
        while (pos < HH_PF) {
            node = tchild(T, node, (w >> pos) & 1);
            pos++;
            if (tleaf(T, node)) {
                bm |= 1u << start;
                nbits = pos;
                node = 0;
                start = pos;
            }
        }
        if (nbits) {
            T->f[w] = (uint16_t)(nbits | ((bm >> 1) << 4));
        } else {
            /* first code longer than HH_PF (>= HH_P) bits: its first HH_P
             * bits index an L1 escape entry; F points at a copy of its
             * meta half */
            const uint32_t i1 = w & (HH_L1_SIZE - 1u);
            if (slot[i1] < 0) {
                if (T->fdir_used >= HH_L2_MAX) return HH_ERR_UNSUPPORTED;
                slot[i1] = (int16_t)T->fdir_used;
                T->fdir[T->fdir_used++] = (uint32_t)(T->l1[i1] >> 32);
            }
            T->f[w] = (uint16_t)((uint32_t)slot[i1] << 4);
        }
    }
    return HH_OK;
}

/* ------------------------------------------------------------------ */
/* decode state machine (layout in hh_fsm.h)                           */
/* ------------------------------------------------------------------ */
/* One step of `nb` stream bits v (first bit in bit 0) from the internal node
 * `node`: the node reached, the symbols completed (up to `cap` kept, first in
 * bits 0..7) and their number. */
static uint32_t fsm_walk(const hh_tables *T, uint32_t node, uint32_t v, unsigned nb, unsigned cap,
                         uint32_t *syms, uint32_t *nsym) {
    uint32_t s = 0, n = 0;
    for (unsigned i = 0; i < nb; i++) {
        node = tchild(T, node, (v >> i) & 1u);
        if (tleaf(T, node)) {
            if (n < cap) s |= (uint32_t)T->tsym[node] << (8 * n);
            n++;
            node = 0;
        }
    }
    *syms = s;
    *nsym = n;
    return node;
}

uint32_t hh_fsm_nstates(const void *tv) {
    const hh_tables *T = (const hh_tables *)tv;
    uint32_t ns = 0;
    for (uint32_t i = 0; i < T->tree_used; i++) ns += !tleaf(T, i);
    return ns;
}

int hh_fsm_build(const void *tv, uint32_t S, uint32_t Kreq, hh_fsm_tables *F) {
    const hh_tables *T = (const hh_tables *)tv;
    /* states: the internal nodes, in compact (BFS) order, root = 0 */
    int32_t *st = (int32_t *)malloc(sizeof(int32_t) * T->tree_used);
    uint32_t *node = (uint32_t *)malloc(sizeof(uint32_t) * (HH_FSM_MAXS + 1));
    if (!st || !node) { free(st); free(node); return HH_ERR_NOMEM; }
    uint32_t ns = 0;
    int rc = HH_OK;
    for (uint32_t i = 0; i < T->tree_used; i++) {
        st[i] = -1;
        if (!tleaf(T, i)) {
            if (ns >= HH_FSM_MAXS) { rc = HH_ERR_UNSUPPORTED; goto out; }
            st[i] = (int32_t)ns;
            node[ns++] = i;
        }
    }
    if (ns == 0 || st[0] != 0) { rc = HH_ERR_UNSUPPORTED; goto out; }
    if (Kreq != 0 && (Kreq < 4 || Kreq > 7)) { rc = HH_ERR_ARG; goto out; }
    {
        /* the count step: a 16-bit entry holds the next row (state << (CB + 1)) */
        const uint32_t cb = ns <= HH_FSM_MAXS8 && S % 8 == 0 ? 8u : 7u;
        if (S == 0 || S % cb) { rc = HH_ERR_UNSUPPORTED; goto out; }
        memset(F, 0, sizeof(*F));
        F->ns = ns;
        F->cb = cb;
        F->K = T->minlen >= 2 ? (Kreq ? Kreq : 6u) : 4u;
        if (ns > HH_FSM_MAXS8 && F->K == 7) F->K = 6;   /* (the et row field is 17 bits) */
        F->S = S;
        F->r = S % F->K;
    }
    for (uint32_t s = 0; s < ns; s++) {
        const uint32_t nd = node[s];
        const uint32_t cb = F->cb;
        F->tsym[s] = T->tsym[nd];
        uint32_t sy, n;
        for (uint32_t v = 0; v < (1u << cb); v++) {
            const uint32_t to = fsm_walk(T, nd, v, cb, 0, &sy, &n);
            F->ct[(s << cb) | v] = (uint16_t)(((uint32_t)st[to] << (cb + 1)) | n);
        }
        for (uint32_t bit = 0; bit < 2; bit++) {
            const uint32_t to = fsm_walk(T, nd, bit, 1, 1, &sy, &n);
            F->b1[s * 2 + bit] = (uint32_t)st[to] | (n << 8) | (sy << 16);
        }
        const uint32_t K = F->K, LG = HH_FSM_ET_LG(K), RSH = HH_FSM_ET_RSH(K);
        for (uint32_t v = 0; v < (1u << K); v++) {
            const uint32_t to = fsm_walk(T, nd, v, K, 4, &sy, &n);
            F->et[(s << LG) | v] = HH_FSM_ET_MAKE(sy, (uint32_t)st[to] << RSH, n);
        }
        for (uint32_t v = 0; F->r && v < (1u << F->r); v++) {
            const uint32_t to = fsm_walk(T, nd, v, F->r, 4, &sy, &n);
            F->er[(s << F->r) | v] = HH_FSM_ET_MAKE(sy, (uint32_t)st[to] << RSH, n);
        }
    }
out:
    free(st);
    free(node);
    return rc;
}
