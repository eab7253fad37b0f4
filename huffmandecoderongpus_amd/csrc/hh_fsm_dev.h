// hh_fsm_dev.h -- host interface of the state-machine decode kernels
// (hh_fsm.hip), used by the decoder's host side (hh_device.hip).  C++ only,
// not part of the public ABI.
#ifndef HH_FSM_DEV_H_
#define HH_FSM_DEV_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hh_fsm.h"

// Device copies of a tree's state-machine tables (hh_fsm_tables) and the
// launch shapes that go with them.
struct FsmDev {
    uint32_t ok;             // tables built and uploaded
    uint32_t ns, K, r, S, G, cb;   // cb: count step bits (8, or 7 for trees of > 127 states)
    uint16_t *ct;
    uint32_t *b1;
    uint8_t *tsym;
    uint64_t *et, *er;
    // persistent grids (workgroups), sized by the occupancy API for S / ns
    uint32_t grid_c, grid_e, sized_S, sized_ns, sized_K, sized_sco, sized_cb, sized_swz;
    uint32_t grid_cm;        // k_cntm's grid (0: no k_cntm for this tree / HH_CNT_M=1)
    uint32_t cm;             // regions per lane of the count pass (k_cntm, 2 or 4; 1: k_cnt only)
    uint32_t phases;         // events between the count, scan and emission kernels (HH_FLAG_PHASE_TIMING)
    uint32_t sized_cm;
    uint32_t sco;            // k_emf's static copy-out (the default; HH_EMF_SCO=0: the store loop)
    uint32_t swz;            // k_emf's swizzled staging: codes whose lengths differ by at most 1 bit
    uint64_t *dbg;           // HH_DIAG builds: phase cycles of k_cnt (16 x u64, the decoder's)
    uint32_t test_nosync;    // tests only (HH_TEST_NOSYNC=1 at set_tree): every decode reports chains
                             // that did not meet, so that the callers' exact fallbacks run
    // the single-pass decode (hh_one.hip; one_setup): usable, head steps,
    // column dwords per lane, waves per workgroup, LDS bytes, grid
    uint32_t one_ok, one_gs, one_capd, one_nw, one_lds, one_grid;
    uint32_t one_nbm;        // rounds of the workgroup's waves per claimed block
    uint32_t one_dbg;        // counters of every decode into dbg (HH_ONE_DBG=1)
    uint32_t one_test_retry; // tests only (HH_TEST_ONE_RETRY=1 at set_tree): every single-pass decode hands
                             // itself back to the two passes, so that the callers' retries run
    uint32_t two_pass;       // the two-pass pipeline only (HH_FLAG_TWO_PASS)
};

// One decode of tiles [0, ntiles) of the segment at d_data (bits readable
// stream bits), the first `emit_from` a prologue, tile 0 entered in state
// in_state.  Outputs: *total symbols written to d_out, *leave (state after
// the last tile), *entry (state entering tile emit_from).  ms[0..3]: count,
// scan, emission device time (fd->phases; else 0), the whole pipeline's.  Returns HH_OK, HH_ERR_CAPACITY, HH_ERR_DEVICE,
// HH_ERR_NOMEM, HH_ERR_UNSUPPORTED (no tables) or the internal HH_NOSYNC
// (chains that did not meet within HH_FSM_KM regions: a code that does not
// resynchronise; never returned through the C ABI -- the callers take the
// segment path or report HH_ERR_UNSUPPORTED).
struct FsmWs {
    void *p;
    size_t size;
    // the decode's results (status, total, leave / entry state), written by
    // k_fscan1 (its last block) straight into host-mapped memory: no copy, no memset per
    // decode.  FSM_RES_SLOTS slots of 16 words: a decode in flight and the
    // next one enqueued behind it (hh_decode_device_async) keep theirs apart.
    uint32_t *h_res, *d_res;
    uint32_t epoch;           // the last single-pass decode's tag (hh_one.hip: its tile states)
    uint64_t *st;             // the single pass's published tile words (+ its block counters), st_cap words
    uint64_t st_cap;
    uint32_t last_one;        // the last decode fsm_decode finished ran the single pass
};
#define FSM_RES_SLOTS 2
// What fsm_collect needs of a decode fsm_launch enqueued.
struct FsmPend {
    uint64_t nt, emit_from, cap;
    uint32_t slot, phases, test_nosync;
    uint32_t one;             // the single pass (k_one) decoded
    uint64_t nt_arg;          // the launch's ntiles and in_state arguments (a retry's)
    uint32_t in_state;
};
// fsm_collect: the single pass handed the decode back (a wait that ran out,
// more fix rounds than it allows): decode it again with the two passes
#define HH_ONE_RETRY (-101)
void fsm_ws_free(FsmWs *ws);
int fsm_decode(FsmDev *fd, FsmWs *ws, uint32_t *h_flags, hipEvent_t *ev, const void *d_data, uint64_t bits,
               uint64_t ntiles, uint32_t in_state, uint64_t emit_from, void *d_out, uint64_t cap,
               hipStream_t st, uint64_t *total, uint32_t *leave, uint32_t *entry, float *ms);
// fsm_decode in two halves: fsm_launch enqueues the decode (results into
// slot `slot`, events ev[0..3]) and returns; fsm_collect waits for its end
// event and returns what fsm_decode would.
int fsm_launch(FsmDev *fd, FsmWs *ws, uint32_t slot, hipEvent_t *ev, const void *d_data, uint64_t bits,
               uint64_t ntiles, uint32_t in_state, uint64_t emit_from, void *d_out, uint64_t cap, hipStream_t st,
               FsmPend *pd, bool force_two = false);
int fsm_collect(FsmWs *ws, hipEvent_t *ev, const FsmPend *pd, uint64_t *total, uint32_t *leave, uint32_t *entry,
                float *ms);
int fsm_upload(FsmDev *fd, const hh_fsm_tables *F, uint32_t G, uint32_t minlen, uint32_t maxlen);
bool fsm_k_fits(const hh_fsm_tables *F, uint32_t est_tile);   // F's emission tables leave room for 16 stagings
void fsm_free(FsmDev *fd);
// the single pass (hh_one.hip): its geometry for the tables in fd (G: head
// bits, avg: expected bits per symbol), and the launch half (fsm_launch's
// contract; fsm_launch calls it unless fd->two_pass or force_two)
void one_setup(FsmDev *fd, uint32_t G, double avg, uint32_t minlen);
int one_launch(FsmDev *fd, FsmWs *ws, uint32_t slot, hipEvent_t *ev, const void *d_data, uint64_t bits, uint64_t ntiles,
               uint32_t in_state, uint64_t emit_from, void *d_out, uint64_t cap, hipStream_t st, FsmPend *pd);
int fsm_debug_arrays(const FsmWs *ws, uint64_t nt, uint32_t *rec, uint32_t *fx, int32_t *tsum, uint32_t *xs);

#endif
