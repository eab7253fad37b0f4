/*
 * hh_plugin.c -- hipHuffApproach: the HIP decoder behind the reference's
 * decoder-plugin signature (see include/hiphuff_plugin.h).
 */
#include "hiphuff.h"
#include "hiphuff_plugin.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Layout mirrors of the reference's structs (framework/huffdata.h:12-37). */
struct HuffNode {
    unsigned char sym;
    int izero;
    int ione;
};
struct CompressedData {
    int bits;
    int nodes;
    int uncompressedsize;
    struct HuffNode *tree;
    unsigned char *data;
};
struct UnCompressedData {
    int uncompressedsize;
    unsigned char *data;
};

static hh_decoder *g_dec;
static int32_t *g_iz, *g_io;
static uint8_t *g_sym;
static int32_t g_nodes;

static void plugin_release(void) {
    hh_decoder_destroy(g_dec);
    g_dec = NULL;
    free(g_iz); free(g_io); free(g_sym);
    g_iz = g_io = NULL; g_sym = NULL; g_nodes = 0;
}

static void die(const char *what, int rc) {
    fprintf(stderr, "hipHuffApproach: %s: %s\n", what, hh_strerror(rc));
    exit(1);
}

/* Rebuild the tables only when the tree differs from the cached one. */
static void ensure_tree(const struct CompressedData *cd) {
    int same = g_dec && g_nodes == cd->nodes;
    for (int i = 0; same && i < cd->nodes; i++)
        same = g_iz[i] == cd->tree[i].izero && g_io[i] == cd->tree[i].ione &&
               g_sym[i] == cd->tree[i].sym;
    if (same) return;
    if (!g_dec) {
        hh_config cfg = {0, 0, 0};
        const char *dev = getenv("HIPHUFF_DEVICE");
        if (dev) cfg.device = atoi(dev);
        int rc = hh_decoder_create(&g_dec, &cfg);
        if (rc) die("device init", rc);
        atexit(plugin_release);
    }
    free(g_iz); free(g_io); free(g_sym);
    g_nodes = cd->nodes;
    g_iz = (int32_t *)malloc(sizeof(int32_t) * (size_t)cd->nodes);
    g_io = (int32_t *)malloc(sizeof(int32_t) * (size_t)cd->nodes);
    g_sym = (uint8_t *)malloc((size_t)cd->nodes);
    if (!g_iz || !g_io || !g_sym) die("tree copy", HH_ERR_NOMEM);
    for (int i = 0; i < cd->nodes; i++) {
        g_iz[i] = cd->tree[i].izero;
        g_io[i] = cd->tree[i].ione;
        g_sym[i] = cd->tree[i].sym;
    }
    hh_tree t = {g_nodes, g_iz, g_io, g_sym};
    int rc = hh_decoder_set_tree(g_dec, &t);
    if (rc) { g_nodes = 0; die("tree", rc); }
}

void hipHuffApproach(struct CompressedData *cd, struct UnCompressedData *uncompressed,
                     void *paramdata) {
    (void)paramdata;
    if (!cd || !uncompressed || cd->bits < 0) die("arguments", HH_ERR_ARG);
    ensure_tree(cd);
    uint64_t n = 0;
    /* the caller's buffer is uncompressedsize + 3 bytes (huffdata.c:166-173) */
    uint64_t cap = (uint64_t)uncompressed->uncompressedsize + 3;
    int rc = hh_decode_host(g_dec, cd->data, (uint64_t)cd->bits, uncompressed->data, cap, &n);
    if (rc) die("decode", rc);
}
