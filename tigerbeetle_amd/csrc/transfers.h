// transfers.h — per-call arguments of the create_transfers kernels.
#pragma once
#include "engine.h"

// What the fixed point's evaluation reads of a transfer on every pass, compact
// (the 128-byte event is read again only for an `exists` comparison or a post/void).
struct alignas(16) EvCore {
    u128 amount;
    u64 ts;       // the event's timestamp
    u32 timeout;
    u16 flags;    // transfer flags
    u8 aflags;    // debit account flags | credit account flags << 4 (limits, history)
    u8 pad;
};
static_assert(sizeof(EvCore) == 32, "EvCore");

struct TrArgs {
    const Transfer* ev;   // events of the call (all batches), in HBM
    u32 n;                // event count
    u32 nb;               // batch count
    const u32* b_start;   // [nb + 1] event offset of each batch
    const u64* b_ts;      // [nb] prepare timestamp of each batch
    const u64* ev_ts;     // [n] event timestamps (routed sub-batches) or null
    const u8* ctl;        // [n] TBGPU_CTL_* bits (chains spanning shards) or null
    u64* commit_ts;       // commit_timestamp sink (T.commit_ts, or a scratch word when dry)
    u32 dry;              // dry run: replies only, no state change
    u64* ts;              // assigned event timestamps
    EvCore* core;         // compact per-event record (classify)
    u32* cs;              // linked-chain start (== index for standalone events)
    u32* ce;              // linked-chain end (inclusive)
    u8* sres;             // static result or SRES_DYN
    u32* dslot;           // debit / credit account slots (regular transfers)
    u32* cslot;
    u32* pre_e;           // committed row with the same id, or NONE32
    u32* pre_p;           // committed row with id == pending_id, or NONE32
    u32* pp_dslot;        // account slots of that committed pending transfer
    u32* pp_cslot;
    u32* gslot;           // group-table slot of the id / of the pending_id
    u32* pslot;
    u32* prev_id;         // previous dynamic event with the same id
    u32* pend_last;       // last earlier dynamic event whose id == pending_id
    u32* pend_first;      // first such event (the one that can succeed: the later ones repeat its id)
    u32* prev_pend;       // previous dynamic post/void with the same pending_id
    u32* gclaim;          // group table: claim words, member counts, ranges
    u32* gcnt_id;
    u32* gcnt_pd;
    u32* gmem;
    u32* gbeg;            // id groups of 2+ members: [gbeg, gend) of gmembers, ascending
    u32* gend;
    u32* gmembers;        // id-group members by index (valid when FL_MULTI_ID)
    u32* gfill;           // per slot: members placed so far (id groups), then pending groups
    u32* pfill;
    u32* pbeg;            // pending groups of 2+ members: their range in plist
    u32* glist;           // scratch: id-group members in arrival order
    u32* plist;           // scratch: pending-group members in arrival order
    u64 gmask;
    u32* counters;
    // Per-pass work lists (tr_lists, once per chunk): `simple` holds the transfers whose
    // id nothing before them in the call or the state holds (their pass is create_transfer's
    // balance tail alone) and the static failures inside chains (their failure breaks the
    // chain every pass); `complex` the post/voids and possible `exists`.  Static failures
    // outside chains are final after tr_init and never re-evaluated.
    u32* lst_simple;
    u32* lst_complex;
    Dirty dt;             // dirty tracking of the passes (engine.h)
    const u128* bh;       // headroom passes: the side's balance figure (balances.hip), or null (Bal4)
    const u64* bh64;      // 64-bit headroom passes (side_scan_fused_h64): the same figure, or null
    u32 debug;            // diagnostics: count changed events by kind (TBGPU_TRACE_PASSES)
    u32 sparse;           // a pass whose previous pass changed fewer than n >> sparse events checks
                          // each event's due stamp before issuing its loads (0: never)
    u32 probe;            // timing probes only (TBGPU_EVAL_PROBE, after convergence): 1 skip post/void, 2 no side records
    Sides sd;             // the account sides of the call's events (engine.h)
    // The apply kernels' gate (tr_launch_converged): they run only when *epi != 0, so the
    // host enqueues them behind a pass group before it knows whether the group converged
    // (null: ungated).  *epi == 1: the converged state is the kernel's EvalState argument
    // (st[0]), 2: epi_alt (st[1]).
    const u32* epi;
    EvalState epi_alt;
};
// epi = 1 + ((q + 1) & 1) for the first pass q of p0 .. p1 - 1 that changed nothing
// (its result state is st[(q + 1) & 1]), when no pass halted (a re-sort or a long
// account segment); 0 otherwise.  One thread.
void tr_launch_converged(const u32* ring, u32 ring_len, u32 p0, u32 p1, const u32* counters, u32* epi,
                         hipStream_t stream);

void tr_launch_classify(const Tables& T, const TrArgs& C, hipStream_t stream);
// Events sharing an id (kind 0: prev_id, ranges) or a pending id (kind 1: prev_pend),
// without a sort: ranges reserved per group, members placed, then ranked in it.
void tr_launch_group(const TrArgs& C, u32 kind, hipStream_t stream);
void tr_launch_group2(const TrArgs& C, hipStream_t stream);
// D: the first pass's input state; D2 (the other buffer) also receives the static
// failures outside chains, which no pass evaluates again
void tr_launch_init_lists(const Tables& T, const TrArgs& C, const EvalState& D, const EvalState& D2, hipStream_t stream);
void tr_launch_side_count(const TrArgs& C, u32 kmax, u8* mask, hipStream_t stream);
void tr_launch_side_build(const TrArgs& C, const EvalState& S, u32 kmax, const uint4* pairs, u32 invalid, u32* skey,
                          u32* sval, hipStream_t stream);
void tr_launch_side_pos(const TrArgs& C, const u32* sval_s, u64 m, hipStream_t stream);
void tr_launch_side_rec(const TrArgs& C, const EvalState& S, hipStream_t stream);
void tr_launch_evaluate(const Tables& T, const TrArgs& C, const EvalState& S, const EvalState& D, const Bal4* bb,
                        const PassGate& g, u32* chg, u32* chg_next, u32* front, u32* front_next, hipStream_t stream);
// One pass over the work lists (tr_lists): the simple list's kernel, then evaluate_one
// over the complex list (counts from the host's copy of CNT_NSIMPLE / CNT_NCOMPLEX).
void tr_launch_evaluate_lists(const Tables& T, const TrArgs& C, const EvalState& S, const EvalState& D, const Bal4* bb,
                              const PassGate& g, u32* chg, u32* chg_next, u32* front, u32* front_next, u32 n_simple,
                              u32 n_complex, hipStream_t stream);
void tr_launch_mask(const Tables& T, const TrArgs& C, const EvalState& S, u8* fres, u8* mask, hipStream_t stream);
// The bounded worst case (transfers.hip tr_walk): the events from `start` (a chain
// start; every earlier event final in D) walked in execute's order.  out[0]: the
// chain start to resume from after a side rebuild (NONE32: done), out[1]: error.
void tr_launch_walk_prep(const TrArgs& C, u64 m, u32 start, u32* sstart, u32* cfail, hipStream_t stream);
void tr_launch_walk(const Tables& T, const TrArgs& C, const EvalState& D, Bal4* bb, u64 m, const u32* sstart,
                    Bal4* wbal, u32* undo_slot, Bal4* undo_val, u32 undo_cap, u32 start, u32* out, hipStream_t stream);
void tr_launch_apply(const Tables& T, const TrArgs& C, const EvalState& S, const u8* fres, const uint4* rk,
                     const Bal4* bb, tbgpu_create_transfers_result_t* results, u32* counts, u64* part,
                     hipStream_t stream);
void tr_launch_advance(const Tables& T, const TrArgs& C, const uint4* rk, const u64* part, hipStream_t stream);
u64 tr_range_part_words(u64 n);
void tr_launch_prep(const TrArgs& C, u32* cfail0, u32* pc, u32 ring, hipStream_t stream);

// create_accounts (accounts.hip)
struct AcArgs {
    const Account* ev;
    u32 n;
    u32 nb;
    const u32* b_start;
    const u64* b_ts;
    u64* ts;
    u32* cs;
    u32* ce;
    u8* sres;
    u32* pre;       // slot of an existing account with the same id
    u64* ts_part;   // ac_mask's per-workgroup max accepted timestamp (GRID(n) words)
    u32* gslot;
    u32* prev_id;
    u32* gclaim;
    u32* gcnt_id;
    u64 gmask;
    u32* counters;
    u32* counts_out;  // per-batch reply counts (the clean two-pass call writes zeros)
    // the clean call's repeats of a hashed id: a call-local claim table (event + 1 per
    // slot, all-zero between calls: the fast path's transfer-id claim table) finds a
    // repeated id, and each event's claimed slot to clear again
    u32* ftab;
    u32* fpos;
    u64 fmask;
    // the clean call's outcome: its flags and ac_fast_index's ticket in fast_words[0..1]
    // (a pair of its own, all-zero between calls); for a small call (flags_out set) the
    // last workgroup stores the flags to flags_out (page-locked host memory, its device
    // address) and zeroes the pair, otherwise the host copies and zeroes them
    u32* fast_words;
    u32* flags_out;
};
// The clean call (accounts.hip ac_fast_*): raises FL_SLOW in counters[CNT_FLAGS] and
// changes nothing visible when the call is not clean (no repeated id, all fields valid,
// no chain, no existing id); otherwise commits it.  The caller ensures row capacity.
// A small call's batch block travels in the kernels' arguments (fast.h BlockInline:
// ac_fast_check reads it there, ac_fast_index writes it for the general path).
struct BlockInline;
void ac_launch_fast(const Tables& T, const AcArgs& C, u64 row_base, const BlockInline& bi, hipStream_t stream);
u32 ac_fast_index_grid(const AcArgs& C);
constexpr u32 AC_TICKET_GRID_MAX = 64;  // ac_fast_index grids up to this size report by ticket
void ac_launch_classify(const Tables& T, const AcArgs& C, hipStream_t stream);
void ac_launch_group_sort(const AcArgs& C, u32 invalid, int bits, u32* k_in, u32* v_in, u32* k_out, u32* v_out,
                          SortScratch& ss, hipStream_t stream);
void ac_launch_init(const AcArgs& C, u8* res, u8* ok, u32* cfail, hipStream_t stream);
void ac_launch_evaluate(const Tables& T, const AcArgs& C, const u8* res_s, const u8* ok_s, u8* res_d, u8* ok_d,
                        u32* cfail_d, hipStream_t stream);
// gate: run only while *gate != 0 (null: always); apply writes no row at or past `cap`
// (it raises FL_ERROR instead)
void ac_launch_mask(const Tables& T, const AcArgs& C, const u8* res, const u8* ok, const u32* cfail, u8* fres,
                    u8* mask, hipStream_t stream, const u32* gate = nullptr);
void ac_launch_apply(const Tables& T, const AcArgs& C, const u8* ok, const u8* fres, const uint4* rk, u64 row_base,
                     u64 cap, tbgpu_create_accounts_result_t* results, u32* counts, hipStream_t stream,
                     const u32* gate = nullptr);
// *gate = 1 when classify found no chain and no repeated id (one evaluation is final)
void ac_launch_gate(const AcArgs& C, u32* gate, hipStream_t stream);

// lookups / maintenance (accounts.hip)
void launch_lookup_accounts(const Tables& T, const u128* ids, u32 n, Account* out, u8* found, hipStream_t stream);
void launch_lookup_transfers(const Tables& T, const u128* ids, u32 n, Transfer* out, u8* found, hipStream_t stream);
void launch_set_balances(const Tables& T, u128 id, Bal4 b, int* status, hipStream_t stream);
void launch_import_transfers(const Tables& T, const Transfer* rows, u32 n, u64 row_base, hipStream_t stream);
void launch_rehash_xidx(const Tables& T, u64 n, hipStream_t stream);
void launch_get_posted(const Tables& T, u128 id, int* status, hipStream_t stream);
void launch_rebuild_accounts(const Tables& T, u64 n, hipStream_t stream);
// ledger shards: other shards' accounts into / out of the directory
void launch_insert_foreign(const Tables& T, const ForeignAccount* f, u64 n, hipStream_t stream);
void launch_collect_foreign(const Tables& T, ForeignAccount* out, u32* cursor, u64 cap, hipStream_t stream);
