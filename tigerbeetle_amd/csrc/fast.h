// fast.h — arguments of the single-pass create_transfers kernels (fast.hip).
#pragma once
#include "engine.h"

struct FastArgs {
    const Transfer* ev;
    u32 n;
    u32 nb;
    const u32* b_start;
    const u64* b_ts;
    const u64* ev_ts;   // [n] event timestamps (routed sub-batches) or null
    u32* gtab;          // duplicate-id claims (event + 1), all-zero between calls
    u32* gpos;          // slot each event claimed (cleared again by fp_index)
    u64 gmask;
    u8* fres;           // per-event result (0 = accepted, deltas applied)
    u32* counters;
    u32* batch_counts;  // failures per batch
    tbgpu_create_transfers_result_t* results;  // replies, concatenated across batches
    u64 row_base;       // host copy of T.base[BASE_ROWS] (timing ablations only; kernels read T.base)
    u128* keys;         // accepted ids, for fp_index
    u32* rows;          // stored row per accepted event (written by fp_fix only)
    u64* tile_idr;      // per tile (TILE_WORDS): componentwise max lo, max hi, min lo, min hi of the
                        // accepted ids; max accepted timestamp; accepted count
    const u8* ctl;      // [n] TBGPU_CTL_* bits (routed calls) or null
    u8* fres2;          // chain members' final results (fp_chains), scratch
    u64* commit_ts;     // commit_timestamp sink (T.commit_ts, or a scratch word when dry)
    u32 dry;            // dry run: replies only, no state change
    Transfer* ev_copy;  // ev is in host memory (zero copy): fp_commit leaves an HBM copy here, or null
    u32 tile;           // events per fp_commit workgroup (FP_SMALL_TILE for a small call, else fp_tiles')
    u32 small;          // fp_commit_small ran: no fp_prep; fp_tail sets the counters from the tile records
    // Eager id claims (a call predicted not to rise: random or reversed ids): fp_commit
    // claims each accepted id's slot of the transfer-id index at its optimistic row by CAS,
    // which also finds a repeat within the call (-> FL_SLOW); gpos[i] is the slot.  No
    // fp_dupcheck, no inserts after; the fix moves a slot to its row's rank, a broken
    // chain withdraws its members' claims (XIDX_TOMB), a fallback clears every claim.
    u32 eager;
    // A prepared drop-in commit (tbgpu_prefetch_transfers): fp_commit_small is enqueued at
    // prefetch time and classifies every event against the pre-call state right away
    // (reads only; the timestamp enters only the last check, overflows_timeout, which is
    // patched after); then each tile waits for the commit call's word in pinned memory
    // (gate_go: gate_seq, or gate_seq | GATE_CANCEL_BIT; the timestamp in gate_ts), and
    // the tiles agree on one verdict through the device word `gate` (tagged gate_seq << 2 |
    // GATE_GO / GATE_OFF, set by the first tile to decide; an OFF winner also stores
    // gate_seq into gate_ack).  Nothing changes state before GO.  fp_tail does nothing
    // unless the tag is GO.  Null: ungated.
    u32* gate;
    u32 gate_seq;
    // fp_commit_small's last tile ends a simple small call itself (no failure, no chain,
    // no repeat check left, the rows taken by the sorted run or already claimed): the
    // counters, cursors and the report with its sequence word, so the host's wait ends
    // there; fp_tail, enqueued behind it as always, then returns at once.
    u32 fuse;
};
constexpr u32 GATE_GO = 1, GATE_OFF = 2;
constexpr u32 GATE_CANCEL_BIT = 0x80000000u;
__host__ __device__ inline u32 gate_tag(u32 seq, u32 verdict) { return (seq << 2) | verdict; }
// per tile: max lo, max hi, min lo, min hi of the accepted ids; max accepted timestamp;
// accepted count; (fp_commit_small) failures and FL_* flags
constexpr u32 TILE_WORDS = 8;
// a drop-in call's tile: 64 events (one wave) per workgroup, so one 8190-event
// prepare spans 128 workgroups instead of 16
constexpr u32 FP_SMALL_TILE = 64;
// calls of at most FP_TAIL_MAX events run fp_launch_tail (one workgroup) instead of
// fp_launch_index + fp_launch_fix + fp_launch_advance
constexpr u32 FP_TAIL_THREADS = 1024, FP_TAIL_MAX = 16384;
enum { ABL_DUP = 1, ABL_BALANCES = 2, ABL_ROWS = 4, ABL_LOOKBACK = 8, ABL_EVENT = 16, ABL_PROBE = 32, ABL_IDS = 64,
       ABL_XREAD = 128, ABL_CLAIM_STORE = 256 };
// Timing-only ablations exist only in variant builds (build.build_variant with
// FP_ABLATE=<mask>, profiles/ablate.py): the product library compiles them out, so no
// environment setting can make it skip work.
#ifndef FP_ABLATE
#define FP_ABLATE 0
#endif
// Variants whose results are wrong (ablations that skip work, for timing only) build
// only with TBGPU_TIMING_VARIANTS, which build.py never passes to the product library.
#if (FP_ABLATE != 0 || defined(FP_NOFLUSH) || defined(FP_SKIP_HOT)) && !defined(TBGPU_TIMING_VARIANTS)
#error "results-changing timing variant without TBGPU_TIMING_VARIANTS (never the product build)"
#endif

// A small call's batch block (starts, then timestamps: engine.hip upload_batches)
// written by fp_prep from its arguments instead of by a launch of its own.
constexpr u32 BLOCK_INLINE_WORDS = 8;
struct BlockInline {
    u32* block;          // c->b_start
    u64* base;           // T.base (the reply cursor's reset)
    u32 words;           // 0: nothing to write
    u32 reset_replies;
    u32 w[BLOCK_INLINE_WORDS];
};
void fp_launch_prep(const FastArgs& F, hipStream_t stream, const BlockInline& bi = BlockInline{});
struct TailReport;
// The prepared commit's words in pinned memory (FastArgs::gate), fp_commit_small's own
// argument (fp_commit's arguments stay as they are: their size is its SGPR budget).
struct GateArgs {
    const u32* go;
    const u64* ts;
    u32* ack;
    u64 budget;  // wall-clock ticks a tile waits before deciding OFF
};
void fp_launch_commit(const Tables& T, const FastArgs& F, hipStream_t stream, const BlockInline& bi,
                      const TailReport& rp, const GateArgs& ga = GateArgs{});
void fp_launch_index(const Tables& T, const FastArgs& F, hipStream_t stream);
void fp_launch_fix(const Tables& T, const FastArgs& F, u8* mask, uint4* ranks, Scan3Scratch& sc, hipStream_t stream);
void fp_launch_undo(const Tables& T, const FastArgs& F, hipStream_t stream);
// k_report's stores made by fp_tail at its end (a small one-chunk call): counters,
// T.base and the reply counts into out (pinned host memory), the replies when
// out_replies is set
struct TailReport {
    u32* out;
    u32 nb;
    const u64* replies;
    u64* out_replies;
    u32* seq_out;  // pinned host word: `seq` stored last, after every other store is visible
    u32 seq;
};
void fp_launch_tail(const Tables& T, const FastArgs& F, hipStream_t stream, const BlockInline& bi = BlockInline{},
                    const TailReport& rp = TailReport{});
void fp_launch_advance(const Tables& T, const FastArgs& F, hipStream_t stream);
u64 fp_tiles(u64 n);
u32 fp_tile_events();  // events per fp_commit workgroup (streamed calls)
