/*
 * hiphuff.h -- C ABI of the MI355X-native parallel Huffman decoder.
 *
 * Plain C types only (pointers, sizes, status codes): this is the drop-in
 * boundary a host program links against (libhiphuff.so).  Each entry point
 * names the reference interface it replaces (BeauJoh/HuffmanDecoderOnGPUs,
 * paths relative to framework/).
 *
 * Layering
 *   hh_huff_*      .huff container (HUFF + 64-bit HUFX)     replaces huffdata.c:27-68
 *   hh_decoder_*   device decoder state (tables, workspace)  replaces the lazy CL/CUDA
 *                                                             globals, openclapproach.c:231-234
 *   hh_decode_*    the hot path                               replaces openclApproach
 *                                                             (openclapproach.c:236-1047) and
 *                                                             fastgpuApproach (fastgpu.cu:140-332)
 *   hh_stage_*     reference-shaped stage kernels             replaces the six kernels of
 *                                                             ReleaseCL/kernels/ *.cl one by one
 *   hipHuffApproach  plugin with the reference's decoder       decodeUtil.h:14-19 function-pointer
 *                    signature (see hiphuff_plugin.h)          type, registered like mainrun.c:480-488
 *
 * Every function returns HH_OK (0) or a negative hh_status; nothing aborts
 * the process (the plugin wrapper converts errors to the reference's
 * exit(1) behaviour, decodeUtil.c:47-52).
 */
#ifndef HIPHUFF_H_
#define HIPHUFF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HIPHUFF_VERSION_MAJOR 0
#define HIPHUFF_VERSION_MINOR 1

typedef enum {
    HH_OK = 0,
    HH_ERR_ARG = -1,          /* bad argument (null pointer, size)            */
    HH_ERR_IO = -2,           /* file could not be opened / read / written    */
    HH_ERR_FORMAT = -3,       /* not a HUFF/HUFX container, truncated         */
    HH_ERR_TREE = -4,         /* tree is not a proper binary tree from node 0,
                                 or the root is a leaf (the reference loops
                                 forever on such a tree, pes.c:151-161)       */
    HH_ERR_CAPACITY = -5,     /* output buffer too small for the decode       */
    HH_ERR_DEVICE = -6,       /* HIP runtime error                            */
    HH_ERR_NOMEM = -7,        /* host or device allocation failed             */
    HH_ERR_INTERNAL = -8,     /* internal consistency check failed            */
    HH_ERR_TIMEOUT = -9,      /* bounded in-kernel wait expired               */
    HH_ERR_UNSUPPORTED = -10  /* input outside what this entry point handles  */
} hh_status;

const char *hh_strerror(int status);

/* ---------------------------------------------------------------------- */
/* Code tree.  Same information as struct HuffNode (huffdata.h:12-16):    */
/* node 0 is the root, a leaf has izero == ione == -1, bit 0 follows      */
/* izero, bit 1 follows ione.  Structure-of-arrays, no padding games.     */
/* ---------------------------------------------------------------------- */
typedef struct {
    int32_t nodes;
    const int32_t *izero;
    const int32_t *ione;
    const uint8_t *sym;
} hh_tree;

/* Static facts about a tree (validated: reachable part is a full binary
 * tree rooted at 0, no cycles). */
typedef struct {
    int32_t reachable;   /* nodes reachable from the root                 */
    int32_t leaves;      /* reachable leaves                              */
    int32_t minlen;      /* shortest code (tableMinDepth, huffdata.c:272) */
    int32_t maxlen;      /* longest code  (tableHeight,  huffdata.c:224)  */
    int32_t len_gcd;     /* gcd of all code lengths                       */
} hh_tree_info;

int hh_tree_check(const hh_tree *tree, hh_tree_info *info);

/* ---------------------------------------------------------------------- */
/* Container: loadHuffFile (huffdata.c:27-68) with 64-bit sizes.          */
/*   "HUFF": be-i32 nodes, be-i32 bits, be-i32 uncompressedsize,          */
/*           nodes x {u8 sym, be-i32 izero, be-i32 ione}, ceil(bits/8) B  */
/*   "HUFX": be-i32 nodes, be-i64 bits, be-i64 uncompressedsize, then the */
/*           same tree and payload (the 64-bit sibling for > 2^31 bits).  */
/* The loaded payload is followed by HH_PAYLOAD_PAD zero bytes.           */
/* ---------------------------------------------------------------------- */
#define HH_PAYLOAD_PAD 64

typedef struct {
    int32_t nodes;
    int32_t *izero;
    int32_t *ione;
    uint8_t *sym;
    uint64_t bits;
    uint64_t uncompressedsize;
    uint8_t *data;           /* ceil(bits/8) + HH_PAYLOAD_PAD bytes       */
    int wide;                /* 1 if read from / to be written as HUFX    */
} hh_huff;

int hh_huff_load(const char *path, hh_huff *out);
/* Writes HUFF when bits and size fit int32 (and !h->wide), else HUFX.    */
int hh_huff_save(const char *path, const hh_huff *h);
void hh_huff_free(hh_huff *h);
hh_tree hh_huff_tree(const hh_huff *h);

/* ---------------------------------------------------------------------- */
/* Encoder (the reference ships none).  Builds the    */
/* canonical bit strings of `tree` and packs `n` symbols LSB-first.       */
/* out must hold hh_encode_bound(tree, n) bytes; *bits gets the length.   */
/* Symbols absent from the tree are an HH_ERR_ARG.                        */
/* ---------------------------------------------------------------------- */
uint64_t hh_encode_bound(const hh_tree *tree, uint64_t n);
int hh_encode(const hh_tree *tree, const uint8_t *syms, uint64_t n,
              uint8_t *out, uint64_t *bits);
/* The same on the GPU through an encoder (its device's workspace, kept
 * across calls): n symbols at device pointer d_syms packed into device
 * buffer d_out (cap bytes, 4-byte aligned; it must hold the stream rounded
 * up to whole 32-bit words -- hh_encode_bound always does).  The same bytes
 * as hh_encode.  *bits gets the length (also with HH_ERR_CAPACITY).
 * Enqueued on hip_stream; returns when done.  One call at a time per
 * encoder; encoders are independent (one per stream encodes at once).  At
 * most about 2^36 symbols per call (HH_ERR_UNSUPPORTED beyond: the launch's
 * grid limit). */
typedef struct hh_encoder hh_encoder;
int hh_encoder_create(hh_encoder **enc, int device);
void hh_encoder_destroy(hh_encoder *enc);
int hh_encoder_encode(hh_encoder *enc, const hh_tree *tree, const void *d_syms, uint64_t n,
                      void *d_out, uint64_t cap, uint64_t *bits, void *hip_stream);
/* hh_encoder_encode on a process-wide encoder of the current device (calls
 * serialised on it). */
int hh_encode_device(const hh_tree *tree, const void *d_syms, uint64_t n,
                     void *d_out, uint64_t cap, uint64_t *bits, void *hip_stream);

/* ---------------------------------------------------------------------- */
/* Device decoder.                                                        */
/* ---------------------------------------------------------------------- */
typedef struct hh_decoder hh_decoder;

typedef struct {
    int device;              /* HIP device ordinal                           */
    int lane_bits;           /* bits per lane region, 0 = default            */
    int flags;               /* HH_FLAG_*                                    */
} hh_config;

#define HH_FLAG_FORCE_EXACT 1   /* skip the fast path and decode with the
                                   reference-shaped stage pipeline (the six
                                   hh_stage_* kernels: exact, O(25 * bits)
                                   memory, bits < 2^31) */
#define HH_FLAG_FORCE_SEGMENT 2 /* skip the fast path and decode with the
                                   segment path (exact, O(N), any length;
                                   the path codes that do not resynchronise
                                   take, codes <= 32 bits) */
#define HH_FLAG_NO_FIXED 4      /* a complete fixed-length code (2^L symbols,
                                   every code L <= 8 bits, e.g. E.coli's) is
                                   unpacked directly (k_fixed) unless this is
                                   set: then it takes the general pipeline */
#define HH_FLAG_LEGACY 8        /* decode with round 2's pipeline (k_front,
                                   k_walk, k_table, k_scan, k_emit) instead of
                                   the state-machine decode (k_cnt, k_fscan,
                                   k_emf) */
#define HH_FLAG_PHASE_TIMING 16 /* record a HIP event between the count, scan
                                   and emission kernels of every decode, for
                                   ms_sync / ms_scan / ms_emit (each event
                                   adds ~6 us of idle GPU time between the
                                   kernels it separates; without the flag
                                   only ms_total is measured, the phase times
                                   read 0) */
#define HH_FLAG_KEEP_HOST_PINNED 32 /* hh_decode_host keeps the caller's payload
                                   and output buffers page-locked across calls
                                   (hipHostRegister once per buffer: a call
                                   with another pointer or a longer length
                                   re-registers) instead of registering and
                                   releasing them in every call.  The caller
                                   must not free or unmap a buffer the decoder
                                   holds: release it first with
                                   hh_decoder_release_host (hh_decoder_destroy
                                   releases them too).  For a harness that
                                   decodes the same buffers again and again,
                                   as the reference's evaluate() does
                                   (decodeUtil.c:41-43, 54-68). */
#define HH_FLAG_TWO_PASS 64     /* the state-machine decode in its two-pass
                                   form (k_cntm count pass, k_fscan1 scan,
                                   k_emf emission) instead of the single pass
                                   (k_one: speculative emission, decoupled
                                   look-back); HH_FLAG_PHASE_TIMING implies
                                   it (the split is between its kernels) */

int hh_decoder_create(hh_decoder **dec, const hh_config *cfg);
void hh_decoder_destroy(hh_decoder *dec);

/* Upload / replace the code tree (builds the lookup tables on the host,
 * copies them to the device).  The tree may be reused across decodes. */
int hh_decoder_set_tree(hh_decoder *dec, const hh_tree *tree);

/* Statistics of the last decode (device time of each phase, in ms). */
typedef struct {
    double ms_total;         /* hipEvent time of the whole device pipeline  */
    double ms_sync;          /* count kernels: heads, region counts, walks
                                (state machine: HH_FLAG_PHASE_TIMING only)  */
    double ms_scan;          /* scan kernels: tile bases, total (idem)      */
    double ms_emit;          /* emission kernels: symbols to HBM (idem)     */
    uint64_t out_len;        /* symbols decoded                              */
    uint64_t lanes;          /* lane regions                                 */
    uint64_t repairs;        /* 1: a tile-state chain was composed on the
                                host (or the stage pipeline ran)            */
    int exact_fallback;      /* 0: the fast path decoded; 1: the stage
                                pipeline (codes longer than 32 bits); 2: the
                                segment path (a walk found no merge: a code
                                that does not resynchronise)                */
    int fixed_length;        /* 1: a complete fixed-length code, unpacked
                                by k_fixed (HH_FLAG_NO_FIXED: 0)            */
    int state_machine;       /* the state-machine decode ran: 1 its two
                                passes (k_cntm, k_fscan1, k_emf), 2 its
                                single pass (k_one)                         */
} hh_stats;

int hh_decoder_stats(const hh_decoder *dec, hh_stats *st);

/* Decode `bits` bits at device pointer d_data (it must be readable for
 * ceil(bits/8) + HH_PAYLOAD_PAD bytes; the pad content is ignored) into
 * device buffer d_out (cap bytes).  *out_len receives the number of
 * symbols, i.e. the length the reference computes with findmax + 1
 * (findmax.cl:2-8).  Enqueued on `hip_stream` (a hipStream_t, NULL = the
 * default stream); the call returns after the output length is known.
 * HH_ERR_CAPACITY (the decode needs more than cap bytes): *out_len is still
 * the stream's full symbol count -- the size to retry with -- here and in
 * hh_decode_host; the output buffer's content is then unspecified.       */
int hh_decode_device(hh_decoder *dec, const void *d_data, uint64_t bits,
                     void *d_out, uint64_t cap, uint64_t *out_len,
                     void *hip_stream);

/* Asynchronous form of hh_decode_device for a stream of decodes: enqueues
 * the decode on `hip_stream` and returns before it has run, then checks the
 * decode issued before it (its length into the out_len pointer passed with
 * it), so that the GPU has the next decode queued while the host reads the
 * last one's results instead of idling between synchronous calls.
 * hh_decode_wait checks the last one and returns the first failure of the
 * asynchronous decodes since the previous wait (HH_OK if none), as
 * hh_decode_device would have returned it; a stream that does not
 * resynchronise is decoded again on the exact path there.  Every out_len
 * pointer and output buffer must stay valid until hh_decode_wait returns.
 * The call itself returns HH_OK, or the argument / launch failure of this
 * decode.  Paths other than the state machine and k_fixed decode
 * synchronously inside the call.  Other entry points (hh_decode_device,
 * ranges, host decodes) first check a pending asynchronous decode.
 * Consecutive asynchronous decodes may use different streams: the decoder's
 * workspace is shared, so a decode on another stream than the pending one
 * is ordered after that one's last kernel (hipStreamWaitEvent). */
int hh_decode_device_async(hh_decoder *dec, const void *d_data, uint64_t bits,
                           void *d_out, uint64_t cap, uint64_t *out_len,
                           void *hip_stream);
int hh_decode_wait(hh_decoder *dec);

/* ---------------------------------------------------------------------- */
/* Segments (multi-GPU shards).  The stream is cut into tiles of           */
/* hh_decoder_tile_bits() bits; a segment is a run of whole tiles.  The    */
/* chain enters a segment in a STATE that is the state leaving the       */
/* previous segment; the stream starts in state 0.  States are opaque     */
/* 32-bit values of the decoder's (a node of the code tree on the state-  */
/* machine path): pass a predecessor's leave_state on unchanged, for the  */
/* same tree.  A segment's output is the symbols from its entry point up to */
/* its successor's, i.e. the segments' outputs concatenate to the stream's */
/* (the reference has no multi-device path).              */
/* ---------------------------------------------------------------------- */
int hh_decoder_tile_bits(const hh_decoder *dec, uint64_t *tile_bits);

typedef struct {
    uint64_t bits_avail;     /* readable stream bits at d_data: the segment's
                                tiles plus at least one tile after them (the
                                next segment's first regions), or up to the
                                end of the stream for the last segment     */
    uint64_t ntiles;         /* tiles to decode (prologue included; at most */
                             /* the tiles of bits_avail).  0 decodes none:  */
                             /* out_len 0, leave_state = entry_state =      */
                             /* in_state, entry_exact = (prologue == 0)     */
    uint64_t prologue;       /* the first `prologue` tiles are the end of   */
                             /* the PREVIOUS segment: decoded only to find  */
                             /* the state entering tile `prologue`, where   */
                             /* output starts (0: start at tile 0)          */
    uint32_t in_state;       /* state entering tile 0                       */
} hh_range;

typedef struct {
    uint64_t out_len;        /* symbols written                             */
    uint32_t leave_state;    /* state leaving the last tile                 */
    uint32_t const_seen;     /* 1: leave_state does not depend on the entry */
                             /* (some emitted tile's table is CONST; on the */
                             /* state machine: the entry's chain was seen   */
                             /* to meet a head's, i.e. a segment of more    */
                             /* than one count tile)                        */
    uint32_t entry_state;    /* state entering the first emitted tile       */
    uint32_t entry_exact;    /* 1: the entry state of the first emitted     */
                             /* tile is exact (no prologue, or some         */
                             /* prologue tile's table is CONST)             */
} hh_range_out;

/* Decode a segment (device pointers, stream as hh_decode_device).  A
 * shard that holds the last tiles of its predecessor before its own decodes
 * them as a prologue (in_state 0) and so finds its own entry state locally
 * (exact whenever one of those tiles is CONST, which real codes almost
 * always are); hh_range_out lets the caller check the entries against the
 * predecessors' leave_state and redo a segment entered wrongly.  Trees
 * the fused path does not handle (codes longer than 32 bits, codes that
 * never resynchronise) return HH_ERR_UNSUPPORTED: decode those whole. */
int hh_decode_device_range(hh_decoder *dec, const void *d_data, const hh_range *rg,
                           void *d_out, uint64_t cap, hh_range_out *out,
                           void *hip_stream);
/* Asynchronous form (as hh_decode_device_async): enqueues the segment's
 * decode and returns; *out is complete once the decode has been checked --
 * by the next asynchronous decode on this decoder or by hh_decode_wait,
 * which returns the first failure (HH_ERR_UNSUPPORTED for a code that does
 * not resynchronise).  const_seen and entry_exact are set at once.  *out
 * and the buffers must stay valid until hh_decode_wait returns. */
int hh_decode_device_range_async(hh_decoder *dec, const void *d_data, const hh_range *rg,
                                 void *d_out, uint64_t cap, hh_range_out *out,
                                 void *hip_stream);

/* Host-to-host convenience: H2D, hh_decode_device, D2H.  This is the scope
 * the reference times in evaluate() (decodeUtil.c:41-43). */
int hh_decode_host(hh_decoder *dec, const uint8_t *data, uint64_t bits,
                   uint8_t *out, uint64_t cap, uint64_t *out_len);
/* Releases the host buffers HH_FLAG_KEEP_HOST_PINNED kept page-locked
 * (nothing to do without the flag). */
int hh_decoder_release_host(hh_decoder *dec);

/* ---------------------------------------------------------------------- */
/* Measurement helper (not on the decode path): a streaming device-to-    */
/* device copy of nbytes (a multiple of 16, 16-B aligned pointers), 16 B  */
/* per lane, plain (nt = 0) or nontemporal (nt = 1) loads and stores; *ms */
/* gets its device time.  bench.py's reference for the HBM rate a plain  */
/* stream reaches on the same GPU (roofline.frac_vs_copy).  Returns when  */
/* done.                                                                  */
/* ---------------------------------------------------------------------- */
int hh_copy_device(const void *d_src, void *d_dst, uint64_t nbytes, int nt,
                   void *hip_stream, float *ms);

/* ---------------------------------------------------------------------- */
/* Reference-shaped stage kernels (one HIP kernel per reference kernel,   */
/* int32 arrays exactly as pes.c / the .cl kernels lay them out).  For    */
/* parity of intermediate arrays; O(25 * bits) memory, bits < 2^31.       */
/* All pointers are device pointers.                                      */
/* ---------------------------------------------------------------------- */
/* initbitsindex.cl:4-12 */
int hh_stage_initbitsindex(hh_decoder *dec, int32_t *d_bitsindex, int64_t bits,
                           void *hip_stream);
/* decodeallbits.cl:10-33: sym per bit, level-0 lengths into d_steps[0..bits) */
int hh_stage_decodeallbits(hh_decoder *dec, const void *d_data, int64_t bits,
                           uint8_t *d_bitdecode, int32_t *d_steps, void *hip_stream);
/* makebigtable.cl:10-40: level `step` -> step+1; *flag gets steps[step][0] */
int hh_stage_makebigtable(hh_decoder *dec, int64_t bits, int32_t *d_steps,
                          int32_t step, int32_t *flag, void *hip_stream);
/* calcbitsindex.cl:5-22 */
int hh_stage_calcbitsindex(hh_decoder *dec, int64_t bits, int32_t *d_bitsindex,
                           const int32_t *d_steps, int32_t step, int32_t powertwo,
                           void *hip_stream);
/* calcresult.cl:5-19 */
int hh_stage_calcresult(hh_decoder *dec, int64_t bits, const int32_t *d_bitsindex,
                        const uint8_t *d_bitdecode, uint8_t *d_result,
                        void *hip_stream);
/* findmax.cl:2-8 (parallel max-reduction instead of one work-item) */
int hh_stage_findmax(hh_decoder *dec, int64_t bits, const int32_t *d_bitsindex,
                     int32_t *maxvalue, void *hip_stream);
/* The six stages driven like openclApproach; returns the output length. */
int hh_stage_pipeline(hh_decoder *dec, const void *d_data, int64_t bits,
                      uint8_t *d_out, uint64_t cap, uint64_t *out_len,
                      void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
