/*
 * hh_oracle.h -- CPU oracle for the hiphuff parity tests.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path
 * (huffmandecoderongpus_amd/, include/) links, loads or calls this code.
 * It is imported only by tests/, by __graft_entry__.smoke() and by the
 * cpu_baseline leg of bench.py, always as the checker (or as the timed CPU
 * baseline), never as the thing being measured or shipped.
 *
 * Each function is a clean-room restatement of one routine of the
 * reference (BeauJoh/HuffmanDecoderOnGPUs, paths relative to framework/):
 *
 *   or_load_huff       huffdata.c:27-68      (loadHuffFile, big-endian HUFF)
 *   or_simple_decode   mainrun.c:38-55       (simpleDecode, bit-serial walk)
 *   or_chain_decode    pes.c:30-46 + 87-104  (the every-bit pipeline's
 *                                              observable result, serially)
 *   or_pes_*           pes.c:22-209          (stage oracle, every array)
 *   or_lin_decode      linapproach.c:110-282 (linApproach, CPU baseline)
 *
 * Parity is pinned by tests/test_oracle.py: or_simple_decode / or_lin_decode
 * reproduce the six shipped originals byte-exactly, the regenerated kjv.txt
 * and E.coli match the sha256 digests recorded in BASELINE.md, and the pes
 * stage arrays reproduce the hello.huff known-answer trace.
 * When oracle/_ref (the reference's own C sources, compiled by
 * oracle/Makefile) is present the tests also compare against it directly.
 */
#ifndef HH_ORACLE_H_
#define HH_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A loaded .huff file (the reference's struct CompressedData, huffdata.h:26-32,
 * with 64-bit sizes).  data has ceil(bits/8) payload bytes + 8 zero pad bytes. */
typedef struct {
    int64_t bits;
    int64_t uncompressedsize;
    int32_t nodes;
    int32_t *izero;   /* [nodes] child on bit 0, -1 for a leaf   */
    int32_t *ione;    /* [nodes] child on bit 1, -1 for a leaf   */
    uint8_t *sym;     /* [nodes] symbol byte (internal nodes too) */
    uint8_t *data;    /* payload, LSB-first bit order             */
} or_huff;

/* Returns 0 on success, negative on error.  Accepts the reference's "HUFF"
 * container and the 64-bit "HUFX" sibling (File format). */
int or_load_huff(const char *path, or_huff *out);
void or_free_huff(or_huff *h);

/* simpleDecode (mainrun.c:38-55): emits a symbol at every leaf; a partial
 * code at the end of the stream is dropped.  Returns symbols written. */
int64_t or_simple_decode(const or_huff *h, uint8_t *out, int64_t cap);

/* The every-bit pipeline's result (pes.c): decode along the chain from bit 0,
 * a code cut off by the end of the stream yields the symbol byte of the
 * internal node the walk stopped at (decodeallbits.cl:22-30).  This is the
 * exact specification the GPU path must meet.  Returns symbols written or -1
 * if cap is too small. */
int64_t or_chain_decode(const or_huff *h, uint8_t *out, int64_t cap);

/* Stage oracle (pes.c).  Arrays are caller-allocated:
 *   bitdecode[bits], steps[25*bits] (row k = makebigtable level k),
 *   bitsindex[bits] (after the last calcbitsindex step), result[bits].
 * Returns the output length (findmax + 1) or -1 on error.
 * *nlevels receives the number of makebigtable launches. */
int64_t or_pes(const or_huff *h, uint8_t *bitdecode, int32_t *steps,
               int32_t *bitsindex, uint8_t *result, int32_t *nlevels);

/* linApproach restatement (linapproach.c:110-282).  out must have at least
 * uncompressedsize + 64 bytes (the reference overruns the logical end by
 * up to one window of garbage symbols, which land in caller slack).
 * Returns the number of symbols the decoder wrote, or -1 on error. */
int64_t or_lin_decode(const or_huff *h, int jumpbits, uint8_t *out, int64_t cap);

/* Monotonic seconds (CLOCK_MONOTONIC_RAW, as framework/time.h:20). */
double or_now(void);

#ifdef __cplusplus
}
#endif
#endif
