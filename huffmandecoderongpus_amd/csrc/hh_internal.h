/*
 * hh_internal.h -- layouts shared by the host table builder (C) and the
 * HIP kernels.  Not part of the public ABI.
 *
 * Decode tables (built on the host from the tree, staged in LDS per
 * workgroup):
 *
 *   L1[2^HH_P]  u64, indexed by the next HH_P stream bits (LSB-first, i.e.
 *               stream bit p is bit 0 of the index -- the reference's window
 *               convention, linapproach.c:207-209, mainrun.c:176-178).
 *     bits  0..31  up to 4 symbol bytes, first symbol in bits 0..7
 *     bits 32..36  nbits: total code bits of the nsym complete symbols
 *     bits 37..39  nsym:  0 = escape (first code longer than HH_P bits)
 *     bits 40..44  len0:  code length of the first symbol (nsym > 0)
 *     bits 45..    bmask: start offsets of the nsym symbols (bit 0 = first),
 *                  HH_P bits
 *     escape entries (nsym == 0):
 *     bits  0..15  L2 base index of the subtable for the depth-HH_P node
 *     bits 16..20  q: index bits of that subtable (<= HH_Q_MAX)
 *     bits 40..55  the same L2 base, bits 56..60 the same q (so the meta
 *                  half alone -- all the front kernel stages -- resolves
 *                  an escape; bits 37..39 stay 0)
 *   A multi-symbol entry is the reference's bigTableMulti idea
 *   (mainrun.c:197-201, 229-247) restricted to the bits in the window.
 *
 *   L2[]        u32 second-level entries, indexed by base + next q bits
 *               (stream bits p+HH_P .. p+HH_P+q-1):
 *     bit  31      1 = leaf found
 *     leaf:     bits 0..7 sym, bits 8..15 total code length
 *     no leaf:  bits 0..23 compact node id at depth HH_P+q (continue with a
 *               bit-serial walk -- only for codes longer than HH_P+HH_Q_MAX)
 *
 *   F[2^HH_PF]  u16, the front kernel's table (it needs no symbol bytes):
 *               indexed by the next HH_PF stream bits like L1, every complete
 *               symbol in the window (no HH_K cap)
 *     bits  0..3   nbits of those symbols (0 = escape: first code longer
 *                  than HH_PF bits)
 *     bits  4..15  start offsets 1..12 of the symbols after the first
 *                  (bit i <=> a symbol starts at offset i + 1)
 *     escape:      bits 4..15 index FDIR[], the meta half of the L1 escape
 *                  entry of the first HH_P bits (its L2 subtable)
 *
 *   tree[]      compact tree for walks (tail symbols, very long codes):
 *               u32 per compact node: bit 31 leaf; leaf -> bits 0..7 sym;
 *               internal -> bits 0..14 child0, bits 15..29 child1; internal
 *               nodes also keep their own sym byte in tsym[] (the reference
 *               emits an internal node's sym for a code cut off by the end of
 *               the stream, decodeallbits.cl:20-31).
 */
#ifndef HH_INTERNAL_H_
#define HH_INTERNAL_H_

#include <stdint.h>

#ifndef HH_P
#define HH_P 12                 /* L1 index bits (11: k_emit 17 % slower on
                                   kjv, with half the table in LDS)    */
#endif
#define HH_L1_SIZE (1u << HH_P)
#ifndef HH_PF
#define HH_PF 13                /* F index bits (HH_P <= HH_PF <= 13; 13:
                                   11.0 bits per lookup on kjv, 12: 10.1) */
#endif
/* an F entry packs nbits and the start mask into 4 + 12 bits, and a code that
 * escapes F must also escape L1 (its fdir word is an L1 escape word) */
#if HH_PF < HH_P || HH_PF > 13
#error "HH_PF must lie in [HH_P, 13]"
#endif
#define HH_F_SIZE (1u << HH_PF)
/* Internal status (never returned through the C ABI): chains that did not
 * meet within the bounded walk -- a code that does not resynchronise; the
 * callers fall back to the exact segment path.  Configuration failures keep
 * their own codes and propagate. */
#define HH_NOSYNC (-100)
#define HH_Q_MAX 9              /* max L2 subtable index bits         */
#define HH_L2_MAX 4096          /* L2 entries kept (LDS budget 16 KB) */
#define HH_TREE_MAX 32767       /* compact nodes (15-bit ids)         */
#define HH_K 4                  /* max symbols per L1 entry           */

#define HH_L1_NBITS(e) ((uint32_t)((e) >> 32) & 31u)
#define HH_L1_NSYM(e) ((uint32_t)((e) >> 37) & 7u)
#define HH_L1_LEN0(e) ((uint32_t)((e) >> 40) & 31u)
#define HH_L1_BMASK(e) ((uint32_t)((e) >> 45) & ((1u << HH_P) - 1u))
#define HH_L1_SYMS(e) ((uint32_t)(e))
#define HH_L1_L2BASE(e) ((uint32_t)(e) & 0xffffu)
#define HH_L1_L2Q(e) (((uint32_t)(e) >> 16) & 31u)

#define HH_L2_LEAF 0x80000000u
#define HH_T_LEAF 0x80000000u

typedef struct {
    uint64_t l1[HH_L1_SIZE];
    uint32_t l2[HH_L2_MAX];
    uint32_t l2_used;
    uint16_t f[HH_F_SIZE];
    uint32_t fdir[HH_L2_MAX];
    uint32_t fdir_used;
    uint32_t tree[HH_TREE_MAX + 1];
    uint8_t tsym[HH_TREE_MAX + 1];
    uint32_t tree_used;
    int32_t minlen, maxlen, len_gcd;
    int32_t fixed_len;          /* >0 if every code has this length   */
} hh_tables;

#ifdef __cplusplus
extern "C" {
#endif
/* Builds the tables; returns HH_OK or an hh_status. */
int hh_tables_build(const void *tree /* const hh_tree* */, hh_tables *t);
/* The encoder's code table (first stream bit in bit 0; len 0: absent). */
int hh_codebook(const void *tree /* const hh_tree* */, uint64_t code[256], uint8_t len[256]);
#ifdef __cplusplus
}
#endif

#endif
