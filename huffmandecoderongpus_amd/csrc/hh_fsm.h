/*
 * hh_fsm.h -- the decode state machine (round 3's decode path).  Not part
 * of the public ABI; shared by the host table builder (hh_huff.c), the HIP
 * kernels (hh_fsm.hip) and the test emulator (tests/emu/hh_emu.cpp).
 *
 * The reference decodes bit by bit down the tree from every offset
 * (decodeallbits.cl:10-33).  A chain's position inside the tree at a bit
 * position p is a STATE: the internal node it has reached (0 = the root, i.e.
 * p is a code boundary).  Stepping a state over the next k stream bits is a
 * table lookup, independent of where codes start, so a decode step needs no
 * data-dependent bit cursor: the step positions are fixed, only the state
 * chains through the lookups.  Two chains that are in the same state at the
 * same position are identical from there on, so "the speculative chain has
 * met the true one" is a state comparison (the FSM form of makebigtable's
 * pointer doubling, makebigtable.cl:10-40).
 *
 * States are numbered 0..ns-1 (internal nodes of the compact tree, BFS
 * order, root first), ns <= HH_FSM_MAXS (255: any tree over a byte alphabet
 * has at most 255 internal nodes).  The count table's step width CB depends
 * on ns so that an entry (next state's row offset | count) stays 16 bits:
 * CB = 8 for ns <= 127 (row = state << 9), CB = 7 for larger trees (row =
 * state << 8; regions of S = 224 bits, 32 steps).
 *
 *   ct[s << CB | v]   u16: CB-bit steps (count pass): the state after the CB
 *                     stream bits v (stream bit p in bit 0, the reference's
 *                     LSB-first order, decodeallbits.cl:23) << (CB + 1),
 *                     i.e. its row's byte offset | the codes completed on the
 *                     way (bits 0..3): the next lookup's address is
 *                     (entry & row mask) | v << 1
 *   b1[s * 2 + bit]   u32: 1-bit steps (the stream's last partial step):
 *                     next state | completed << 8 | the symbol << 16
 *   tsym[s]           the sym byte of the state's node: the symbol the
 *                     reference emits for a code cut off by the end of the
 *                     stream (its tail rule, decodeallbits.cl:20-31)
 *   et[s << LG | v]   u64: K-bit steps (emission), v = the next K bits;
 *                     LG = HH_FSM_ET_LG(K) = max(K, 5) entries per state (K =
 *                     4 rows are padded to 32 entries)
 *       bits  0..31   the symbols completed (first in bits 0..7, unused
 *                     bytes 0): K = 4..7 for codes of >= 2 bits, K = 4
 *                     when a code has 1 bit; a step from inside a code
 *                     completes up to 3 (K = 6) or 4 (K = 7, 4) symbols
 *       bits 32..37   8 x the number of symbols (the output shift; bits
 *                     38..39 are 0)
 *       bits 40..63   the next state's row in et, in bytes: next <<
 *                     HH_FSM_ET_RSH(K) (= LG + 3 >= 8: the row bits of the
 *                     high word start at bit 8, above the shift, so that the
 *                     next entry's LDS address is one bit-field insert of the
 *                     step's K bits, at bit 3, into the high word)
 *   er[s << r | v]    u64: the r-bit step that ends a region of S bits when K
 *                     does not divide S (r = S mod K, 0: none); same layout,
 *                     rows in et units
 */
#ifndef HH_FSM_H_
#define HH_FSM_H_

#include <stdint.h>

#define HH_FSM_MAXS 255
#define HH_FSM_MAXS8 127    /* largest ns with 8-bit count steps */
#define HH_FSM_S7 224       /* region bits with 7-bit count steps */

typedef struct {
    uint32_t ns;              /* states (internal nodes)                      */
    uint32_t K;               /* emission step bits                           */
    uint32_t r;               /* remainder step bits of a region (S mod K)    */
    uint32_t S;               /* region bits the remainder table is built for */
    uint32_t cb;              /* count step bits: 8 (ns <= 127) or 7          */
    uint16_t ct[HH_FSM_MAXS * 256];
    uint32_t b1[HH_FSM_MAXS * 2];
    uint8_t tsym[HH_FSM_MAXS + 1];
    uint64_t et[HH_FSM_MAXS * 128];
    uint64_t er[HH_FSM_MAXS * 64];
} hh_fsm_tables;

#define HH_FSM_ET_LG(K) ((K) < 5u ? 5u : (K))          /* log2 entries per state row */
#define HH_FSM_ET_RSH(K) (HH_FSM_ET_LG(K) + 3u)          /* log2 bytes per state row   */
#define HH_FSM_ET_SYMS(e) ((uint32_t)(e))
#define HH_FSM_ET_ROW(e) ((uint32_t)((e) >> 32) & ~255u)
#define HH_FSM_ET_NSYM(e) (((uint32_t)((e) >> 32) & 255u) >> 3)
#define HH_FSM_ET_MAKE(syms, row, n) \
    ((uint64_t)(uint32_t)(syms) | (uint64_t)((uint32_t)(row) | 8u * (uint32_t)(n)) << 32)
#define HH_FSM_CT_NEXT(v, cb) ((uint32_t)(v) >> ((cb) + 1))
#define HH_FSM_CT_CNT(v) ((uint32_t)(v) & 15u)

#ifdef __cplusplus
extern "C" {
#endif
/* Builds the state machine of the compact tree in T (hh_tables_build) for
 * regions of S bits, emission steps of K bits (4..7; 0: 6; a code of 1 bit
 * takes K = 4 whatever is asked; trees of more than HH_FSM_MAXS8 internal
 * nodes take at most 6).  Count steps of 8 bits when ns <= HH_FSM_MAXS8 and
 * S is whole bytes, else of 7 bits (S a multiple of 7).  HH_ERR_UNSUPPORTED
 * when the tree has more than HH_FSM_MAXS internal nodes or S does not fit
 * the count step. */
int hh_fsm_build(const void *T /* const hh_tables* */, uint32_t S, uint32_t K, hh_fsm_tables *F);
/* The number of states (internal nodes) of the compact tree in T. */
uint32_t hh_fsm_nstates(const void *T /* const hh_tables* */);
#ifdef __cplusplus
}
#endif

#endif
