/*
 * hh_cli.c -- HuffFramework, the reference's CLI driver restated for the HIP
 * decoder (framework/mainrun.c:467-657 + decodeUtil.c:30-70).
 *
 *   HuffFramework <test> [--files DIR] [--reps N]
 *
 * Test names follow mainrun.c: hello, bigtable, kjvprof, quickgraph2, graph2,
 * plus `file <name>` (any DIR/<name> + DIR/<name>.huff pair) and `stages
 * <name>` (the reference-shaped six-kernel pipeline).  Every run is checked
 * byte-for-byte against the original file first (decodeUtil.c:47-52: a
 * mismatch prints the first differences and exits 1), then timed REPEATS
 * more times; the minimum is printed in the reference's format
 * "%17s %8s     %.9f ms" (mainrun.c:412-420).  DIR defaults to
 * $HIPHUFF_FILES or ./files.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hiphuff.h"

#define REPEATS 25   /* decodeUtil.h:26 */

static const char *g_dir = "files";
static int g_reps = REPEATS;
static hh_decoder *g_dec;

typedef struct {
    char name[64];
    hh_huff h;
    uint8_t *orig;
    uint64_t orig_len;
} testdata;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts);   /* framework/time.h:20 */
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int load_test(testdata *td, const char *file, const char *name) {
    char path[4096];
    memset(td, 0, sizeof(*td));
    snprintf(td->name, sizeof td->name, "%s", name);
    snprintf(path, sizeof path, "%s/%s.huff", g_dir, file);
    int rc = hh_huff_load(path, &td->h);
    if (rc) {
        fprintf(stderr, "cannot load %s: %s\n", path, hh_strerror(rc));
        return rc;
    }
    snprintf(path, sizeof path, "%s/%s", g_dir, file);
    FILE *f = fopen(path, "rb");
    if (f) {
        fseek(f, 0, SEEK_END);
        long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        td->orig = (uint8_t *)malloc((size_t)n + 3);
        td->orig_len = (uint64_t)n;
        if (fread(td->orig, 1, (size_t)n, f) != (size_t)n) td->orig_len = 0;
        fclose(f);
    } else {
        fprintf(stderr, "note: %s absent, checking against the header size only\n", path);
    }
    return 0;
}

static void free_test(testdata *td) {
    hh_huff_free(&td->h);
    free(td->orig);
}

/* huffdata.c:183-203 message format */
static int compare(const uint8_t *a, uint64_t na, const uint8_t *b, uint64_t nb) {
    if (na != nb) {
        printf("different size! : %llu %llu\n", (unsigned long long)na, (unsigned long long)nb);
        return -1;
    }
    uint64_t diff = 0;
    for (uint64_t i = 0; i < na; i++) {
        if (a[i] != b[i]) {
            if (diff < 10) printf("different at: %llu  val1: %d  val2: %d\n", (unsigned long long)i, a[i], b[i]);
            diff++;
        }
    }
    if (!diff) return 0;
    printf("differences %llu / %llu\n", (unsigned long long)diff, (unsigned long long)na);
    return -1;
}

typedef int (*decode_fn)(const testdata *, uint64_t bits, uint8_t *out, uint64_t cap, uint64_t *n);

static int dec_hip(const testdata *td, uint64_t bits, uint8_t *out, uint64_t cap, uint64_t *n) {
    return hh_decode_host(g_dec, td->h.data, bits, out, cap, n);
}

static int ensure_tree(const testdata *td) {
    hh_tree t = hh_huff_tree(&td->h);
    return hh_decoder_set_tree(g_dec, &t);
}

/* evaluate(): one checked run, then g_reps timed runs; returns min seconds */
static double evaluate(decode_fn fn, const char *dname, const testdata *td, uint64_t bits,
                       uint64_t expect_len, const uint8_t *expect) {
    if (ensure_tree(td)) { fprintf(stderr, "tree rejected\n"); exit(1); }
    uint64_t cap = expect_len + 3;
    uint8_t *out = (uint8_t *)calloc(cap, 1);
    uint64_t n = 0;
    double t0 = now_s();
    int rc = fn(td, bits, out, cap, &n);
    double best = now_s() - t0;
    if (rc) {
        fprintf(stderr, "problem with : %s (%s)\n", dname, hh_strerror(rc));
        exit(1);
    }
    if (expect && compare(out, n, expect, expect_len) != 0) {
        fprintf(stderr, "problem with : %s\n", dname);
        fprintf(stderr, "decode problem\n");
        exit(1);
    }
    if (!expect && n != expect_len) {
        fprintf(stderr, "problem with : %s (length %llu != %llu)\n", dname,
                (unsigned long long)n, (unsigned long long)expect_len);
        exit(1);
    }
    for (int i = 0; i < g_reps; i++) {
        memset(out, 0, cap);
        t0 = now_s();
        fn(td, bits, out, cap, &n);
        double t = now_s() - t0;
        if (t < best) best = t;
    }
    free(out);
    return best;
}

static void evalandshow(decode_fn fn, const char *dname, const testdata *td) {
    double s = evaluate(fn, dname, td, td->h.bits, td->orig ? td->orig_len : td->h.uncompressedsize,
                        td->orig);
    hh_stats st;
    hh_decoder_stats(g_dec, &st);
    printf("%17s %8s     %.9f ms\n", dname, td->name, s * 1000.0);
    printf("%17s %8s     %.9f ms device (sync %.4f scan %.4f emit %.4f)%s\n", "", "", st.ms_total,
           st.ms_sync, st.ms_scan, st.ms_emit, st.exact_fallback ? " [exact path]" : "");
}

/* setTargetSizes (mainrun.c:361-385): cut at the last whole symbol before
 * `target` bits; returns bits and the symbol count through *syms. */
static uint64_t target_bits(const testdata *td, uint64_t target, uint64_t *syms) {
    const hh_huff *h = &td->h;
    uint64_t pos = 0, nsym = 0, lastok = 0;
    int32_t node = 0;
    while (pos < target && pos < h->bits) {
        int bit = (h->data[pos >> 3] >> (pos & 7)) & 1;
        node = bit ? h->ione[node] : h->izero[node];
        if (h->izero[node] == -1) {
            nsym++;
            node = 0;
            lastok = pos;
        }
        pos++;
    }
    *syms = nsym;
    return lastok + 1;
}

/* graphtest (mainrun.c:387-410) */
static void graphtest(decode_fn fn, const char *dname, const testdata *td, uint64_t incs) {
    for (uint64_t size = incs; size < td->h.bits; size += incs) {
        uint64_t syms;
        uint64_t b = target_bits(td, size, &syms);
        double s = evaluate(fn, dname, td, b, syms, td->orig);
        printf("%8llu  %.9f\n", (unsigned long long)size, s);
    }
}

static int dec_stages(const testdata *td, uint64_t bits, uint8_t *out, uint64_t cap, uint64_t *n);

int main(int argc, char **argv) {
    const char *test = argc > 1 ? argv[1] : "hello";
    const char *arg2 = NULL;
    for (int i = 2; i < argc; i++) {
        if (!strcmp(argv[i], "--files") && i + 1 < argc) g_dir = argv[++i];
        else if (!strcmp(argv[i], "--reps") && i + 1 < argc) g_reps = atoi(argv[++i]);
        else arg2 = argv[i];
    }
    const char *env = getenv("HIPHUFF_FILES");
    if (env && strcmp(g_dir, "files") == 0) g_dir = env;
    fprintf(stderr, "running test: %s\n", test);
    hh_config cfg = {0, 0, 0};
    int rc = hh_decoder_create(&g_dec, &cfg);
    if (rc) { fprintf(stderr, "no HIP device: %s\n", hh_strerror(rc)); return 1; }

    testdata td;
    if (!strcmp(test, "hello")) {
        if (load_test(&td, "hello", "hello")) return 1;
        evalandshow(dec_hip, "hip", &td);
        free_test(&td);
    } else if (!strcmp(test, "bigtable")) {
        const char *files[] = {"paper1", "hello", "news", "kjv.txt", "book2"};
        const char *names[] = {"paper1", "hello", "news", "kjv", "book2"};
        testdata t[5];
        for (int i = 0; i < 5; i++) {
            if (load_test(&t[i], files[i], names[i])) return 1;
            printf("%s nodes %d, bits %llu, uncompressedsize %llu\n", names[i], t[i].h.nodes,
                   (unsigned long long)t[i].h.bits, (unsigned long long)t[i].h.uncompressedsize);
        }
        for (int i = 0; i < 5; i++) evalandshow(dec_hip, "hip", &t[i]);
        for (int i = 0; i < 5; i++) free_test(&t[i]);
    } else if (!strcmp(test, "kjvprof")) {
        if (load_test(&td, "kjv.txt", "kjv")) return 1;
        evalandshow(dec_hip, "hip", &td);
        free_test(&td);
    } else if (!strcmp(test, "quickgraph2")) {
        if (load_test(&td, "paper1", "paper1")) return 1;
        graphtest(dec_hip, "hip", &td, 10000);
        free_test(&td);
    } else if (!strcmp(test, "graph2")) {
        if (load_test(&td, "kjv.txt", "kjv")) return 1;
        graphtest(dec_hip, "hip", &td, 500000);
        free_test(&td);
    } else if (!strcmp(test, "file") && arg2) {
        if (load_test(&td, arg2, arg2)) return 1;
        evalandshow(dec_hip, "hip", &td);
        free_test(&td);
    } else if (!strcmp(test, "stages") && arg2) {
        if (load_test(&td, arg2, arg2)) return 1;
        evalandshow(dec_stages, "hipstages", &td);
        free_test(&td);
    } else {
        fprintf(stderr, "unknown test %s\n", test);
        hh_decoder_destroy(g_dec);
        return 2;
    }
    hh_decoder_destroy(g_dec);
    return 0;
}

#include <hip/hip_runtime_api.h>
static int dec_stages(const testdata *td, uint64_t bits, uint8_t *out, uint64_t cap, uint64_t *n) {
    void *dd = NULL, *dout = NULL;
    uint64_t nb = (bits + 7) / 8;
    if (hipMalloc(&dd, nb + HH_PAYLOAD_PAD) != hipSuccess) return HH_ERR_NOMEM;
    if (hipMalloc(&dout, cap) != hipSuccess) { (void)hipFree(dd); return HH_ERR_NOMEM; }
    int rc = HH_OK;
    if (hipMemcpy(dd, td->h.data, nb + HH_PAYLOAD_PAD, hipMemcpyHostToDevice) != hipSuccess) rc = HH_ERR_DEVICE;
    if (!rc) rc = hh_stage_pipeline(g_dec, dd, (int64_t)bits, (uint8_t *)dout, cap, n, NULL);
    if (!rc && *n && hipMemcpy(out, dout, *n, hipMemcpyDeviceToHost) != hipSuccess) rc = HH_ERR_DEVICE;
    (void)hipFree(dd);
    (void)hipFree(dout);
    return rc;
}
