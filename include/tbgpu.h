/*
 * tbgpu.h — C ABI of the MI355X-native TigerBeetle commit engine.
 *
 * This is the drop-in boundary for the `create_accounts` / `create_transfers`
 * arms of `StateMachine.commit` (reference: src/state_machine.zig:894-928,
 * `execute` :1002-1088).  A thin Zig `extern "C"` shim in
 * src/state_machine.zig binds these symbols.
 *
 * Plain C: fixed-layout structs, pointers and sizes.  No torch, no HIP types.
 *
 * Struct layouts are byte-identical to the reference's extern structs
 *   Account               src/tigerbeetle.zig:7-40      (tb_client.h:26-40)
 *   Transfer              src/tigerbeetle.zig:80-105    (tb_client.h:51-65)
 *   CreateAccountsResult  src/tigerbeetle.zig:247-255   (tb_client.h:150-153)
 *   CreateTransfersResult src/tigerbeetle.zig:257-265   (tb_client.h:155-158)
 * and the result codes are the reference enums (src/tigerbeetle.zig:125-245),
 * whose numeric value equals their precedence index.
 */
#ifndef TBGPU_H
#define TBGPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* u128 as two little-endian u64 words (the reference targets little-endian only,
 * src/tigerbeetle.zig:306-309). */
typedef struct tbgpu_uint128_t { uint64_t lo, hi; } tbgpu_uint128_t;

typedef struct tbgpu_account_t {
    tbgpu_uint128_t id;
    tbgpu_uint128_t debits_pending;
    tbgpu_uint128_t debits_posted;
    tbgpu_uint128_t credits_pending;
    tbgpu_uint128_t credits_posted;
    tbgpu_uint128_t user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t reserved;
    uint32_t ledger;
    uint16_t code;
    uint16_t flags;
    uint64_t timestamp;
} tbgpu_account_t;

typedef struct tbgpu_transfer_t {
    tbgpu_uint128_t id;
    tbgpu_uint128_t debit_account_id;
    tbgpu_uint128_t credit_account_id;
    tbgpu_uint128_t amount;
    tbgpu_uint128_t pending_id;
    tbgpu_uint128_t user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t timeout;
    uint32_t ledger;
    uint16_t code;
    uint16_t flags;
    uint64_t timestamp;
} tbgpu_transfer_t;

/* {index, result}: sparse, only non-ok events, ascending index. */
typedef struct tbgpu_create_accounts_result_t { uint32_t index; uint32_t result; } tbgpu_create_accounts_result_t;
typedef struct tbgpu_create_transfers_result_t { uint32_t index; uint32_t result; } tbgpu_create_transfers_result_t;

/* AccountHistoryGrooveValue, src/state_machine.zig:275-294 (256 B). */
typedef struct tbgpu_account_history_t {
    tbgpu_uint128_t dr_account_id;
    tbgpu_uint128_t dr_debits_pending;
    tbgpu_uint128_t dr_debits_posted;
    tbgpu_uint128_t dr_credits_pending;
    tbgpu_uint128_t dr_credits_posted;
    tbgpu_uint128_t cr_account_id;
    tbgpu_uint128_t cr_debits_pending;
    tbgpu_uint128_t cr_debits_posted;
    tbgpu_uint128_t cr_credits_pending;
    tbgpu_uint128_t cr_credits_posted;
    uint64_t timestamp;
    uint8_t reserved[88];
} tbgpu_account_history_t;

/* AccountFilter, src/tigerbeetle.zig:268-302 (64 B): the input of
 * get_account_transfers / get_account_history. */
typedef struct tbgpu_account_filter_t {
    tbgpu_uint128_t account_id;
    uint64_t timestamp_min;  /* inclusive; 0 = no lower bound */
    uint64_t timestamp_max;  /* inclusive; 0 = no upper bound */
    uint32_t limit;
    uint32_t flags;          /* TBGPU_ACCOUNT_FILTER_* */
    uint8_t reserved[24];
} tbgpu_account_filter_t;
/* AccountFilterFlags, src/tigerbeetle.zig:289-302 */
enum {
    TBGPU_ACCOUNT_FILTER_DEBITS = 1 << 0,
    TBGPU_ACCOUNT_FILTER_CREDITS = 1 << 1,
    TBGPU_ACCOUNT_FILTER_REVERSED = 1 << 2,
};

/* AccountBalance, src/tigerbeetle.zig:65-78 (128 B): one get_account_history row. */
typedef struct tbgpu_account_balance_t {
    tbgpu_uint128_t debits_pending;
    tbgpu_uint128_t debits_posted;
    tbgpu_uint128_t credits_pending;
    tbgpu_uint128_t credits_posted;
    uint64_t timestamp;
    uint8_t reserved[56];
} tbgpu_account_balance_t;

/* AccountFlags, src/tigerbeetle.zig:42-63 */
enum {
    TBGPU_ACCOUNT_LINKED = 1 << 0,
    TBGPU_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS = 1 << 1,
    TBGPU_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS = 1 << 2,
    TBGPU_ACCOUNT_HISTORY = 1 << 3,
};
/* TransferFlags, src/tigerbeetle.zig:107-120 */
enum {
    TBGPU_TRANSFER_LINKED = 1 << 0,
    TBGPU_TRANSFER_PENDING = 1 << 1,
    TBGPU_TRANSFER_POST_PENDING_TRANSFER = 1 << 2,
    TBGPU_TRANSFER_VOID_PENDING_TRANSFER = 1 << 3,
    TBGPU_TRANSFER_BALANCING_DEBIT = 1 << 4,
    TBGPU_TRANSFER_BALANCING_CREDIT = 1 << 5,
};

/* CreateAccountResult, src/tigerbeetle.zig:125-160 */
enum {
    TBGPU_CREATE_ACCOUNT_OK = 0,
    TBGPU_CREATE_ACCOUNT_LINKED_EVENT_FAILED = 1,
    TBGPU_CREATE_ACCOUNT_LINKED_EVENT_CHAIN_OPEN = 2,
    TBGPU_CREATE_ACCOUNT_TIMESTAMP_MUST_BE_ZERO = 3,
    TBGPU_CREATE_ACCOUNT_RESERVED_FIELD = 4,
    TBGPU_CREATE_ACCOUNT_RESERVED_FLAG = 5,
    TBGPU_CREATE_ACCOUNT_ID_MUST_NOT_BE_ZERO = 6,
    TBGPU_CREATE_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 7,
    TBGPU_CREATE_ACCOUNT_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 8,
    TBGPU_CREATE_ACCOUNT_DEBITS_PENDING_MUST_BE_ZERO = 9,
    TBGPU_CREATE_ACCOUNT_DEBITS_POSTED_MUST_BE_ZERO = 10,
    TBGPU_CREATE_ACCOUNT_CREDITS_PENDING_MUST_BE_ZERO = 11,
    TBGPU_CREATE_ACCOUNT_CREDITS_POSTED_MUST_BE_ZERO = 12,
    TBGPU_CREATE_ACCOUNT_LEDGER_MUST_NOT_BE_ZERO = 13,
    TBGPU_CREATE_ACCOUNT_CODE_MUST_NOT_BE_ZERO = 14,
    TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_FLAGS = 15,
    TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 16,
    TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 17,
    TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 18,
    TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_LEDGER = 19,
    TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_CODE = 20,
    TBGPU_CREATE_ACCOUNT_EXISTS = 21,
};

/* CreateTransferResult, src/tigerbeetle.zig:165-245 */
enum {
    TBGPU_CREATE_TRANSFER_OK = 0,
    TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED = 1,
    TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN = 2,
    TBGPU_CREATE_TRANSFER_TIMESTAMP_MUST_BE_ZERO = 3,
    TBGPU_CREATE_TRANSFER_RESERVED_FLAG = 4,
    TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_ZERO = 5,
    TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_INT_MAX = 6,
    TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 7,
    TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 8,
    TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 9,
    TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 10,
    TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 11,
    TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_BE_DIFFERENT = 12,
    TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_ZERO = 13,
    TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_ZERO = 14,
    TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_INT_MAX = 15,
    TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_DIFFERENT = 16,
    TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER = 17,
    TBGPU_CREATE_TRANSFER_AMOUNT_MUST_NOT_BE_ZERO = 18,
    TBGPU_CREATE_TRANSFER_LEDGER_MUST_NOT_BE_ZERO = 19,
    TBGPU_CREATE_TRANSFER_CODE_MUST_NOT_BE_ZERO = 20,
    TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_NOT_FOUND = 21,
    TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_NOT_FOUND = 22,
    TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER = 23,
    TBGPU_CREATE_TRANSFER_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS = 24,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_FOUND = 25,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_PENDING = 26,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID = 27,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID = 28,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER = 29,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_CODE = 30,
    TBGPU_CREATE_TRANSFER_EXCEEDS_PENDING_TRANSFER_AMOUNT = 31,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT = 32,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_ALREADY_POSTED = 33,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_ALREADY_VOIDED = 34,
    TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_EXPIRED = 35,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_FLAGS = 36,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID = 37,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID = 38,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_AMOUNT = 39,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_PENDING_ID = 40,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 41,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 42,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 43,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_TIMEOUT = 44,
    TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_CODE = 45,
    TBGPU_CREATE_TRANSFER_EXISTS = 46,
    TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS_PENDING = 47,
    TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS_PENDING = 48,
    TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS_POSTED = 49,
    TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS_POSTED = 50,
    TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS = 51,
    TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS = 52,
    TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT = 53,
    TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS = 54,
    TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS = 55,
};

/* constants.batch_max.create_transfers with production constants:
 * (message_size_max 1 MiB - 256 B header) / 128 B (src/state_machine.zig:53-76). */
#define TBGPU_BATCH_MAX 8190u

/* ------------------------------------------------------------------------ */
/* Engine                                                                    */
/* ------------------------------------------------------------------------ */

typedef struct tbgpu_ctx tbgpu_ctx;

/* Options replace StateMachine.Options (src/state_machine.zig:328-334): the
 * cache sizes become HBM table capacities. Zero means "default". */
typedef struct tbgpu_options {
    int32_t  device;              /* HIP device ordinal */
    uint32_t reserved0;
    uint64_t accounts_max;        /* accounts the ctx must hold                     */
    uint64_t transfers_max;       /* stored transfers (rows) the ctx must hold      */
    uint64_t history_max;         /* account-history rows                            */
    uint64_t events_per_call_max; /* events one (multi-batch) call may carry        */
    uint32_t flags;               /* TBGPU_OPT_*                                    */
    uint32_t dense_block_span;    /* 0, or S: ids (b << 32) | k, b < directory_max / S + 2,
                                     1 <= k <= S, sit in the direct-mapped directory  */
    uint64_t directory_max;       /* accounts the directory must know (0: accounts_max); more
                                     than accounts_max only for a ledger shard (below)  */
    uint64_t hashed_max;          /* accounts whose ids fall outside the direct-mapped
                                     directory (0: directory_max): sizes the hash index */
    uint32_t shard_world;         /* 0 or 1: one state machine.  N >= 2: this ctx is the
                                     ledger shard shard_rank of N (ledger % N == rank owns
                                     the ledger): it stores 128-byte rows only for accounts
                                     of its ledgers, and a directory entry (id, ledger) for
                                     every other account                */
    uint32_t shard_rank;
} tbgpu_options;

enum {
    TBGPU_OPT_FORCE_GENERAL = 1u << 0, /* disable the balance-insensitive fast path (tests) */
    TBGPU_OPT_WALK_EARLY = 1u << 1,    /* the fixed point hands its chunk to the sequential walk
                                          after two passes instead of its pass budget (tests:
                                          the walk's results are the passes' results) */
    TBGPU_OPT_PINNED_INPUT = 1u << 2,  /* the host event buffers the caller passes are its own
                                          page-locked allocations (hipHostMalloc,
                                          hipHostRegister): a small one-chunk call's events
                                          are read in place and uploads skip the staging
                                          ring.  Without it every host buffer is copied
                                          through the ctx's page-locked ring. */
    TBGPU_OPT_DENSE_INDEXES = 1u << 3, /* size the account and transfer-id hash indexes at
                                          load <= 1/2 (2 slots per id of capacity) instead of
                                          the default <= 1/8 (8 slots, while an index stays
                                          within 1 GiB / 8 GiB): a quarter of the memory, a
                                          second probe more often (random u128 ids) */
};

/* Replaces StateMachine.init/deinit (src/state_machine.zig:418-451).
 * Returns 0 on success; on failure *out is NULL and the return is a negative errno-like code.
 *
 * Concurrency: a ctx serves one caller at a time, as the reference's StateMachine serves
 * its replica's one thread.  The one exception is the router's send side
 * (tbgpu_route_stats, _prepare, _scatter, _scatter_packed, _unpack, _unpack_packed: they
 * run on the ctx's route stream with buffers of their own), which may run on one thread
 * while another thread commits on the same ctx (tbgpu_create_transfers_routed[_device]:
 * tigerbeetle_amd/shard.py's pipelined stream).  Any other overlap aborts the process
 * with "concurrent calls on one ctx" (a nested call on the same thread is allowed). */
int  tbgpu_init(tbgpu_ctx** out, const tbgpu_options* options);
void tbgpu_deinit(tbgpu_ctx* ctx);
/* StateMachine.reset (src/state_machine.zig:453): forget all state. */
void tbgpu_reset(tbgpu_ctx* ctx);

/* execute(.create_accounts) — src/state_machine.zig:1002-1088, :1198-1237.
 * `timestamp` is the prepare timestamp handed to commit (the events get
 * timestamp - n + index + 1). Returns the number of sparse results written
 * (reply bytes = 8 * count). Host buffers, 16-byte aligned, caller-owned. */
uint32_t tbgpu_create_accounts(tbgpu_ctx* ctx, uint64_t timestamp,
                               const tbgpu_account_t* events, uint32_t count,
                               tbgpu_create_accounts_result_t* results);

/* execute(.create_transfers) — src/state_machine.zig:1002-1088, :1239-1573. */
uint32_t tbgpu_create_transfers(tbgpu_ctx* ctx, uint64_t timestamp,
                                const tbgpu_transfer_t* events, uint32_t count,
                                tbgpu_create_transfers_result_t* results);

/* StateMachine.prefetch for create_transfers (src/state_machine.zig:514-655,
 * prefetch_create_transfers :598-655; the replica awaits its callback before commit,
 * src/vsr/replica.zig:3384-3415).  The tables are HBM-resident, so what prefetch has
 * left to do is the batch's host-to-device copy: this enqueues it into the ctx's
 * staging slot and returns; tbgpu_prefetch_wait returns once the copy has landed (the
 * callback's point).  The next tbgpu_create_transfers with the same `events` pointer
 * and `count` commits from the staged copy (no copy inside the commit); any other
 * create call (accounts, transfers, batches, device and routed forms), an import,
 * tbgpu_reset and tbgpu_open discard it.
 * When that commit will be a one-batch fast call, the prefetch also prepares it: its
 * launches are enqueued behind a gate kernel that waits (at most 10 ms) for the
 * commit's timestamp in pinned memory, so the commit itself launches nothing.  Any
 * call on the ctx other than tbgpu_prefetch_wait and that commit releases the gate
 * (the prepared launches then do nothing); a commit after the gate's wait ran out is an
 * ordinary prefetched call.  Results never depend on which of these happened.
 * As in the reference, the prepare's body must not change between prefetch and commit.
 * Returns 0, or -22 when count exceeds a batch. */
int tbgpu_prefetch_transfers(tbgpu_ctx* ctx, const tbgpu_transfer_t* events, uint32_t count);
int tbgpu_prefetch_wait(tbgpu_ctx* ctx);

/* StateMachine.prepare for create_transfers (src/state_machine.zig:503-512, called by
 * the primary from primary_pipeline_prepare, src/vsr/replica.zig:5159-5167, before the
 * prepare is journaled and replicated; the op is prefetched and committed once a quorum
 * has it, src/vsr/replica.zig:3137-3152).  Starts the body's host-to-device copy into
 * one of TBGPU_STAGE_SLOTS slots in HBM, keyed by `key`, and returns: the copy runs on a
 * stream of its own while the prepare is replicated.  `key` identifies the body's
 * content: the shim passes the message header's checksum_body, which the prepare keeps
 * from its request (the body is not changed between the two, :5193-5211).  Staging the
 * same key again does nothing.  It never releases a pending prepared commit.  A slot is
 * reused oldest-first (slots a prefetch took before the others); the body must not
 * change while its copy runs (until tbgpu_prefetch_transfers_staged of it returns, or
 * the next stage call).  Backups never call prepare: their prefetch copies as
 * tbgpu_prefetch_transfers does.  Returns 0, or -22 when count exceeds a batch. */
#define TBGPU_STAGE_SLOTS 8u /* constants.pipeline_prepare_queue_max */
int tbgpu_stage_transfers(tbgpu_ctx* ctx, tbgpu_uint128_t key, const tbgpu_transfer_t* events, uint32_t count);
/* tbgpu_prefetch_transfers for a body that may have been staged: when a slot holds
 * `key` with `count` events, the prefetch copies nothing and only prepares the commit
 * from that slot (tbgpu_prefetch_wait then waits for the staged copy, normally long
 * done); otherwise it is tbgpu_prefetch_transfers.  Results are the same either way. */
int tbgpu_prefetch_transfers_staged(tbgpu_ctx* ctx, tbgpu_uint128_t key, const tbgpu_transfer_t* events,
                                    uint32_t count);

/* Streaming form: `batch_count` consecutive commits of create_transfers, with
 * identical results to calling tbgpu_create_transfers once per batch in order.
 * Batch b has `counts[b]` events starting after the previous batch's events and
 * prepare timestamp `timestamps[b]`.  Results of batch b are written at
 * `results + (sum of counts before b)`; `result_counts[b]` receives its count.
 * Returns the total number of results. */
uint64_t tbgpu_create_transfers_batches(tbgpu_ctx* ctx, uint32_t batch_count,
                                        const uint64_t* timestamps, const uint32_t* counts,
                                        const tbgpu_transfer_t* events,
                                        tbgpu_create_transfers_result_t* results,
                                        uint32_t* result_counts);

/* Same with the events already resident in device memory (HBM) and the replies
 * left in device memory.  On the device the replies are concatenated: batch b's
 * `result_counts[b]` results follow batch b-1's (the streaming reply format);
 * each result's `index` is relative to its own batch.  `timestamps`, `counts`
 * and `result_counts` are host arrays. */
uint64_t tbgpu_create_transfers_batches_device(tbgpu_ctx* ctx, uint32_t batch_count,
                                               const uint64_t* timestamps, const uint32_t* counts,
                                               const void* events_device,
                                               void* results_device,
                                               uint32_t* result_counts);

uint64_t tbgpu_create_accounts_batches(tbgpu_ctx* ctx, uint32_t batch_count,
                                       const uint64_t* timestamps, const uint32_t* counts,
                                       const tbgpu_account_t* events,
                                       tbgpu_create_accounts_result_t* results,
                                       uint32_t* result_counts);

/* Same with the events and the replies in device memory (replies concatenated, as
 * for tbgpu_create_transfers_batches_device). */
uint64_t tbgpu_create_accounts_batches_device(tbgpu_ctx* ctx, uint32_t batch_count,
                                              const uint64_t* timestamps, const uint32_t* counts,
                                              const void* events_device, void* results_device,
                                              uint32_t* result_counts);

/* ------------------------------------------------------------------------ */
/* Sharded commit (the ledger router is tigerbeetle_amd/shard.py) */
/* ------------------------------------------------------------------------ */
/* The reference has one state machine; sharded by ledger, each GPU's ctx commits
 * the owner's sub-sequence of a routed step.  These entry points have no single
 * reference counterpart: they carry what `execute` (src/state_machine.zig:1018-1083)
 * derives from a batch's position -- the event timestamps and the linked-chain
 * bounds -- for sub-batches whose events are not contiguous in their batch. */
enum {
    /* A ledger shard's create_accounts reply for an event whose id names an account of
     * another shard's ledger (create_account_exists, src/state_machine.zig:1227-1237,
     * compares the existing row, which only its owner stores): a failure like every
     * `exists*` code, whose exact code the owner's reply for the same event carries
     * (tigerbeetle_amd/shard.py merges them).  Never returned by an unsharded ctx. */
    TBGPU_SHARD_ACCOUNT_EXISTS_ELSEWHERE = 255,
};

enum {
    /* The chain this event belongs to continues on another shard after it: the
     * event closes the local part of the chain (no linked_event_chain_open). */
    TBGPU_CTL_CHAIN_END = 1u << 0,
    /* The chain broke on another shard before this event: not evaluated, result
     * linked_event_failed (execute's chain_broken arm, :1037-1040). */
    TBGPU_CTL_SKIP = 1u << 1,
    /* The chain breaks on another shard after this event, the last local member:
     * the local part is evaluated, then rolled back (scope_close(.discard),
     * :1049-1058) and its members get linked_event_failed. */
    TBGPU_CTL_DOOM = 1u << 2,
};

/* create_transfers over `batch_count` owner sub-batches.  `event_timestamps[i]`
 * is event i's timestamp (T - n + index + 1 of its source batch).  `ctl` (may be
 * NULL) holds TBGPU_CTL_* bits per event.  With `dry_run` nonzero the replies and
 * the would-be commit timestamp are computed and nothing is stored (one call must
 * then fit events_per_call_max).  `*commit_timestamp` receives the ctx's commit
 * timestamp after the call (or, dry, what it would be).  Replies as in
 * tbgpu_create_transfers_batches (host buffers). */
uint64_t tbgpu_create_transfers_routed(tbgpu_ctx* ctx, uint32_t batch_count, const uint32_t* counts,
                                       const tbgpu_transfer_t* events, const uint64_t* event_timestamps,
                                       const uint8_t* ctl, int dry_run,
                                       tbgpu_create_transfers_result_t* results, uint32_t* result_counts,
                                       uint64_t* commit_timestamp);

/* Same with events, event timestamps, chain control (may be NULL) and the
 * replies in device memory (HBM); replies concatenated per sub-batch as in
 * tbgpu_create_transfers_batches_device.  `counts` / `result_counts` are host arrays. */
uint64_t tbgpu_create_transfers_routed_device(tbgpu_ctx* ctx, uint32_t batch_count, const uint32_t* counts,
                                              const void* events_device, const void* event_timestamps_device,
                                              const void* ctl_device, int dry_run, void* results_device,
                                              uint32_t* result_counts, uint64_t* commit_timestamp);

/* The 8-byte record that travels with each routed event (tbgpu_route_scatter): */
#define TBGPU_ROUTE_REC_POS 0x1FFFull        /* bits 0-12: the event's index in its batch */
#define TBGPU_ROUTE_REC_SPAN (1ull << 13)    /* its linked chain has members on several owners */
#define TBGPU_ROUTE_REC_LAST (1ull << 14)    /* it ends its chain (not linked, or last of its batch) */
#define TBGPU_ROUTE_REC_CS_SHIFT 15          /* bits 15-27: index of its chain's first member */
#define TBGPU_ROUTE_REC_CS_MASK 0x1FFFull
#define TBGPU_ROUTE_REC_BATCH_SHIFT 32       /* bits 32-63: global batch number */

/* The send side of a routed step (tigerbeetle_amd/shard.py): this rank's client
 * batches (`counts`, each <= 8192 events, prepare timestamps `batch_timestamps`,
 * global number of the first one `first_global_batch`), events in device memory,
 * are written to `send_events_device` (n * 128 B) owner-major -- owner = ledger %
 * world -- in event order within an owner, each with an 8-byte record
 * (TBGPU_ROUTE_REC_*) in `send_records_device` (n * 8 B).  `send_counts[world]`
 * (host) receives the events per owner; when not NULL, `send_batch_counts[world *
 * batch_count]` the events per (owner, batch) and `send_span_counts[world]` the
 * events per owner whose chain spans owners.  world <= 256.  Returns 0, or -22 for
 * a bad argument.  Synchronous. */
/* One pass over a routed step's local events (device memory) deciding whether the
 * device path applies: out[0] min id (low word), out[1] max id (low word), out[2]
 * bit 0: an id not above its predecessor, bit 1: an id with a high word or zero,
 * bit 2: a post/void, bit 3: an amount of 2^64 or more, bits 16-47: bit 16 + w set
 * when 4-byte word w (0-31) of some event is nonzero (the packed wire format's
 * mask, tbgpu_route_scatter_packed); out[3], out[4]: the sum of the amounts (low,
 * high word).  Returns 0.  Synchronous. */
int tbgpu_route_stats(tbgpu_ctx* ctx, const void* events_device, uint64_t count, uint64_t* out);
/* tbgpu_route_stats and the first pass of tbgpu_route_scatter (each event's owner
 * and rank) in one pass over the events; a tbgpu_route_scatter of the same events
 * and world that follows skips that pass.  Returns 0, or -22.  Synchronous. */
int tbgpu_route_prepare(tbgpu_ctx* ctx, uint32_t world, const void* events_device, uint64_t count, uint64_t* out);
int tbgpu_route_scatter(tbgpu_ctx* ctx, uint32_t world, uint32_t batch_count, const uint32_t* counts,
                        const uint64_t* batch_timestamps, uint64_t first_global_batch, const void* events_device,
                        void* send_events_device, void* send_records_device, uint64_t* send_counts,
                        uint32_t* send_batch_counts, uint32_t* send_span_counts);
/* tbgpu_route_scatter in the packed wire format: per event, the 4-byte words w of
 * the event with bit w of `word_mask` set (in word order), then the low word of its
 * record (TBGPU_ROUTE_REC_*; the owner knows each row's batch from the per-(owner,
 * batch) counts): popcount(word_mask) + 1 words of 4 bytes, owner-major in
 * `send_device`.  The mask is normally the union over the ranks of
 * tbgpu_route_stats' nonzero-word bits (config 4's events: 15 of 32 words, so 64
 * bytes on the wire instead of 136); an event with a nonzero word outside it
 * returns -22 (nothing is lost silently).  Synchronous. */
int tbgpu_route_scatter_packed(tbgpu_ctx* ctx, uint32_t world, uint32_t batch_count, const uint32_t* counts,
                               uint64_t first_global_batch, const void* events_device, uint32_t word_mask,
                               void* send_device, uint64_t* send_counts, uint32_t* send_batch_counts,
                               uint32_t* send_span_counts);
/* The owner side of the packed format: `count` received rows of
 * popcount(word_mask) + 1 words back to whole 128-byte events (words outside the
 * mask zero) in `events_device`, their whole records in `records_device` (count * 8
 * B) and their timestamps as tbgpu_route_unpack computes them.  The rows are the
 * owner's sub-batches in global order: sub-batch k starts at row
 * `sub_offsets_device[k]` (uint32, sub_batch_count + 1 entries, the last = count)
 * and belongs to global batch `sub_batches_device[k]` (uint32).  Returns 0, or -22
 * when a batch is >= batches.  Synchronous. */
int tbgpu_route_unpack_packed(tbgpu_ctx* ctx, const void* packed_device, uint64_t count, uint32_t word_mask,
                              uint32_t sub_batch_count, const void* sub_offsets_device,
                              const void* sub_batches_device, const void* ts_base_device, uint64_t batches,
                              void* events_device, void* records_device, void* timestamps_device);
/* The owner side: event timestamps from received records, timestamps[i] =
 * ts_base[batch of record i] + index + 1 with ts_base[g] = T_g - n_g of global batch
 * g (src/vsr/replica.zig:5148-5157; `batches` entries, device memory).  Returns 0,
 * or -22 when a record names a batch >= batches.  Synchronous. */
int tbgpu_route_unpack(tbgpu_ctx* ctx, const void* records_device, uint64_t count, const void* ts_base_device,
                       uint64_t batches, void* timestamps_device);

/* The general step's id directory (tigerbeetle_amd/shard_vec.py round_vec), on the
 * device.  `records_device`: `count` rows of five int64 (position in the step's global
 * order, kind 0 id / 1 pending id, key lo, key hi, route hint), all ranks' records
 * all-gathered.  _owners writes, per record, the owner (ledger % world) of this shard's
 * committed transfer with that key, or -1; the caller all-reduces them (MAX) over the
 * ranks.  tbgpu_route_directory then writes three int64 per record: its type (0 new,
 * 1 exists, 2 repeat, 3 pending found, 4 pending none, 5 pending created earlier by an
 * event that may land anywhere), its hint (the owner, or the first record's hint), and
 * the earliest position among the key's records of ids not committed (INT64_MAX: none).
 * The types follow src/state_machine.zig:1284 (exists) and :1409-1428 (the pending's
 * lookup); the key grouping is a hash table, not a sort.  Synchronous; 0, or -22. */
int tbgpu_route_directory_owners(tbgpu_ctx* ctx, uint32_t world, const void* records_device, uint64_t count,
                                 void* owners_device);
int tbgpu_route_directory(tbgpu_ctx* ctx, const void* records_device, const void* owners_device, uint64_t count,
                          void* out_device);

/* Copy committed transfers of another shard into this ctx's transfer table and id
 * index, without balance or posted effects: the `exists` comparisons of
 * :1370-1389 / :1500-1561 then see a colliding id committed elsewhere.  Returns 0. */
int tbgpu_import_transfers(tbgpu_ctx* ctx, const tbgpu_transfer_t* rows, uint32_t count);

/* commit_timestamp = max(commit_timestamp, timestamp): the node-wide commit
 * timestamp is the max over shards (:1366 advances it per created transfer). */
void tbgpu_advance_commit_timestamp(tbgpu_ctx* ctx, uint64_t timestamp);

/* execute_lookup_accounts / execute_lookup_transfers (src/state_machine.zig:1091-1126):
 * found objects are written densely in request order; returns the count. */
uint32_t tbgpu_lookup_accounts(tbgpu_ctx* ctx, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_account_t* out);
uint32_t tbgpu_lookup_transfers(tbgpu_ctx* ctx, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_transfer_t* out);

/* ------------------------------------------------------------------------ */
/* Account queries                                     */
/* ------------------------------------------------------------------------ */
/* constants.batch_max.get_account_transfers / _history: message_body_size_max /
 * 128 B (src/state_machine.zig:53-76). */
#define TBGPU_QUERY_MAX 8190u

/* The grooves' field index trees (src/state_machine.zig:1575-1641 tree_options_index):
 * Groove.insert puts (field, timestamp) into a field's tree for every stored object whose
 * field is nonzero (src/lsm/groove.zig:911-936); a scan of a tree with a field value as
 * its prefix yields the objects with that value in timestamp order.  The transfers groove
 * indexes every field below, the accounts groove user_data_128/64/32, ledger and code.
 * No operation of this snapshot's state machine reads them except through
 * debit/credit_account_id (get_account_transfers); the scans below expose them. */
enum tbgpu_index_field {
    TBGPU_INDEX_DEBIT_ACCOUNT_ID = 0,   /* transfers */
    TBGPU_INDEX_CREDIT_ACCOUNT_ID = 1,  /* transfers */
    TBGPU_INDEX_USER_DATA_128 = 2,
    TBGPU_INDEX_USER_DATA_64 = 3,
    TBGPU_INDEX_USER_DATA_32 = 4,
    TBGPU_INDEX_PENDING_ID = 5,         /* transfers */
    TBGPU_INDEX_TIMEOUT = 6,            /* transfers */
    TBGPU_INDEX_LEDGER = 7,
    TBGPU_INDEX_CODE = 8,
    TBGPU_INDEX_AMOUNT = 9,             /* transfers */
};
enum { TBGPU_INDEX_REVERSED = 1 << 0 };

typedef struct tbgpu_index_filter_t {
    tbgpu_uint128_t value;     /* the field's value (0: not indexed, so nothing matches) */
    uint64_t timestamp_min;    /* 0 = unbounded (src/lsm/timestamp_range.zig) */
    uint64_t timestamp_max;
    uint32_t limit;            /* at most min(limit, TBGPU_QUERY_MAX) objects */
    uint32_t field;            /* tbgpu_index_field */
    uint32_t flags;            /* TBGPU_INDEX_REVERSED: descending timestamps */
    uint32_t reserved;         /* 0 */
} tbgpu_index_filter_t;

/* The stored transfers (accounts) whose `field` equals `value`, timestamps within
 * [timestamp_min, timestamp_max], ascending (or descending), at most
 * min(limit, TBGPU_QUERY_MAX) whole objects into `out`.  Returns the count.  A filter
 * that is invalid (a field the groove does not index, a zero limit, timestamp_min >
 * timestamp_max != 0, a bound of UINT64_MAX, reserved flags or bytes) yields 0, as an
 * invalid account filter does.  The trees are built on demand: a scan first indexes
 * the objects stored since that tree's last scan. */
uint32_t tbgpu_scan_transfers(tbgpu_ctx* ctx, const tbgpu_index_filter_t* filter, tbgpu_transfer_t* out);
uint32_t tbgpu_scan_accounts(tbgpu_ctx* ctx, const tbgpu_index_filter_t* filter, tbgpu_account_t* out);

/* StateMachine.compact (src/state_machine.zig:930-955): fold the transfers stored
 * since the previous compaction into the account-transfers index (the
 * debit_account_id / credit_account_id index trees of the transfers groove,
 * :198-220).  Queries compact first, so calling it is optional; a replica calls it
 * once per op, off the commit's critical path.  Returns the rows indexed. */
uint64_t tbgpu_compact(tbgpu_ctx* ctx);

/* execute_get_account_transfers with its prefetch scan (src/state_machine.zig:693-734,
 * :822-885, :1128-1147): the stored transfers whose debit (flags.debits) or credit
 * (flags.credits) account is filter->account_id, with timestamp_min <= timestamp <=
 * timestamp_max (0 = unbounded), in timestamp order (descending with
 * flags.reversed), at most min(limit, TBGPU_QUERY_MAX).  An invalid filter
 * (:822-833) yields nothing.  Returns the count written to `out`. */
uint32_t tbgpu_get_account_transfers(tbgpu_ctx* ctx, const tbgpu_account_filter_t* filter, tbgpu_transfer_t* out);

/* execute_get_account_history (:736-808, :1149-1196): the same scan, each
 * transfer's account-history row (the filter account's balances after it), for
 * an account with flags.history.  A post/void transfer stores no history row
 * (:1342-1364 is create_transfer only); the reference's lookup then asserts
 * (src/lsm/scan_lookup.zig:179, :215) -- here the transfer is skipped. */
uint32_t tbgpu_get_account_history(tbgpu_ctx* ctx, const tbgpu_account_filter_t* filter, tbgpu_account_balance_t* out);

/* Many queries in one launch, everything in device memory: filter q's results
 * are written at out_device + q * stride (128-B rows), at most
 * min(limit, TBGPU_QUERY_MAX, stride); result_counts (host) receives the counts.
 * Returns the total. */
uint64_t tbgpu_get_account_transfers_device(tbgpu_ctx* ctx, uint32_t count, const void* filters_device,
                                            uint32_t stride, void* out_device, uint32_t* result_counts);
uint64_t tbgpu_get_account_history_device(tbgpu_ctx* ctx, uint32_t count, const void* filters_device,
                                          uint32_t stride, void* out_device, uint32_t* result_counts);

/* ------------------------------------------------------------------------ */
/* Benchmark load (src/tigerbeetle/benchmark_load.zig:209-330), in HBM        */
/* ------------------------------------------------------------------------ */
/* The `tigerbeetle benchmark` load at BASELINE config 5's scale, written straight
 * into device memory by a counter-based generator (record i depends only on
 * (seed, first_id + i)).  Accounts: ids first_id.., ledger (id - 1) /
 * accounts_per_ledger + 1, code 1.  Transfers: ids first_id.., a ledger among
 * ledger0 + ledger_stride * [0, ledgers) (stride N: the ledgers of one shard of N,
 * ledger % N), uniform distinct debit/credit accounts of that
 * ledger, amount floor(Exp(1) * 10000) + 1, random user data and code, flags 0.
 * Synchronous; 0 or a negative errno. */
int tbgpu_bench_generate_accounts(int device, uint64_t first_id, uint64_t count,
                                  uint32_t accounts_per_ledger, void* out_device);
int tbgpu_bench_generate_transfers(int device, uint64_t first_id, uint64_t count, uint64_t seed,
                                   uint32_t ledger0, uint32_t ledgers, uint32_t ledger_stride,
                                   uint32_t accounts_per_ledger, void* out_device);

/* The drop-in call timed from C, as the Zig shim issues it (bench.py host_path):
 * `calls` consecutive batches (batch k: counts[k] events at the running offset of
 * `events`, committed at timestamps[k]); mode 0 one tbgpu_create_transfers per batch,
 * mode 1 tbgpu_prefetch_transfers + tbgpu_prefetch_wait and then the commit of the same
 * batch.  Wall time per commit (and per prefetch, when prefetch_us is not NULL) in
 * microseconds.  Replies go to `results` (room for the largest batch).  0, or -22. */
int tbgpu_bench_host_calls(tbgpu_ctx* ctx, int mode, uint32_t calls, const tbgpu_transfer_t* events,
                           const uint32_t* counts, const uint64_t* timestamps,
                           tbgpu_create_transfers_result_t* results, double* commit_us, double* prefetch_us);
/* The primary's sequence for one op (bench): tbgpu_stage_transfers, a busy-wait of
 * gap_us standing for the replication round trip, then tbgpu_prefetch_transfers_staged
 * + tbgpu_prefetch_wait and tbgpu_create_transfers, timed per call from C. */
int tbgpu_bench_host_staged(tbgpu_ctx* ctx, uint32_t calls, const tbgpu_transfer_t* events,
                            const uint32_t* counts, const uint64_t* timestamps,
                            tbgpu_create_transfers_result_t* results, double gap_us, double* stage_us,
                            double* prefetch_us, double* commit_us);

/* Test harness `setup` action (src/state_machine.zig:1892-1908): overwrite an
 * existing account's four balances.  Returns 0, or -1 if the account is missing. */
int tbgpu_test_set_balances(tbgpu_ctx* ctx, tbgpu_uint128_t id,
                            tbgpu_uint128_t debits_pending, tbgpu_uint128_t debits_posted,
                            tbgpu_uint128_t credits_pending, tbgpu_uint128_t credits_posted);

/* Host memory into device memory by the engine's own copy kernel (the ctx's
 * page-locked staging ring, read by a kernel on the ctx's stream), for device
 * buffers the engine's kernels will read (the *_device entry points' inputs): such
 * buffers are then written by a kernel, never by a copy engine.  Synchronous;
 * returns 0. */
int tbgpu_copy_to_device(tbgpu_ctx* ctx, void* dst_device, const void* src_host, uint64_t bytes);

/* State export for parity checks (not on the reference's hot path). */
uint64_t tbgpu_account_count(tbgpu_ctx* ctx);
uint64_t tbgpu_transfer_count(tbgpu_ctx* ctx);
uint64_t tbgpu_history_count(tbgpu_ctx* ctx);
/* Stored transfers in commit order (rows [first, first+count)). */
uint64_t tbgpu_export_transfers(tbgpu_ctx* ctx, uint64_t first, uint64_t count, tbgpu_transfer_t* out);
/* All accounts, in unspecified order. `capacity` bounds `out`. */
uint64_t tbgpu_export_accounts(tbgpu_ctx* ctx, tbgpu_account_t* out, uint64_t capacity);
uint64_t tbgpu_export_history(tbgpu_ctx* ctx, uint64_t first, uint64_t count, tbgpu_account_history_t* out);
/* Posted groove (src/state_machine.zig:235-248): fulfillment of the pending transfer
 * with this id: -1 none/not found, 0 posted, 1 voided. */
int tbgpu_get_posted(tbgpu_ctx* ctx, tbgpu_uint128_t pending_id);
/* ------------------------------------------------------------------------ */
/* Persistence                                         */
/* ------------------------------------------------------------------------ */
/* StateMachine.checkpoint (src/state_machine.zig:957-970) / open (:486-500): the
 * state the ctx owns -- accounts, stored transfers, the posted groove, account
 * history, commit_timestamp -- as one self-describing image in a caller buffer
 * (the replica hands it to its grid / superblock).  Layout: a 64-B header
 * {magic "TBGPUCK1", version, shard, counts, commit_timestamp, checksum of the
 * rest}, then Account[n_accounts], Transfer[n_rows], posted u8[n_rows], imported
 * u8[n_rows], AccountHistoryGrooveValue[n_history], and for a ledger shard the
 * other shards' directory entries.  Version 1: an unsharded ctx; version 3: a
 * ledger shard (shard_world << 16 | shard_rank in `shard`); version 2: a legacy
 * shard image without its shard, still accepted by any shard ctx.  The indexes are
 * derived state, rebuilt on open. */
uint64_t tbgpu_checkpoint_size(tbgpu_ctx* ctx);
/* Returns the bytes written, or 0 when `capacity` is too small. */
uint64_t tbgpu_checkpoint(tbgpu_ctx* ctx, void* out, uint64_t capacity);
/* Replaces the ctx's state by the image's.  Returns 0, -22 (EINVAL) for a bad
 * magic/version/size/checksum or an image of another shard or kind, -95
 * (EOPNOTSUPP) for a version-1 image offered to a ledger-shard ctx, -28 (ENOSPC)
 * when the image exceeds the ctx's capacities. */
int tbgpu_open(tbgpu_ctx* ctx, const void* image, uint64_t size);

/* StateMachine.commit_timestamp (src/state_machine.zig:375). */
uint64_t tbgpu_commit_timestamp(tbgpu_ctx* ctx);

/* Diagnostics: statistics of the last call and the last error message. */
typedef struct tbgpu_stats {
    uint64_t events;          /* events in the last call                        */
    uint32_t iterations;      /* fixed-point passes of the last call            */
    uint32_t path;            /* 0 general (scan + rescan), 1 fast (no rescan),
                                 2 general, walked past the pass budget         */
    uint64_t sorts;           /* side sorts performed                           */
    double   device_ms;       /* HIP-event time of the last call's device work  */
    /* With profiling on: HIP-event time per phase of the last call, on the ctx
     * stream: [0] upload [1] classify+group [2] sort [3] balance scan
     * [4] evaluate [5] apply [6] reserved [7] reserved. */
    double   phase_ms[8];
    uint64_t walks;           /* chunks, since init, whose fixed point reached its
                                 pass budget and was walked in execute's order    */
    uint64_t index_rebuilds;  /* transfer-id index rebuilds since init: withdrawn
                                 claims of non-rising ids left tombstones          */
    uint64_t h64_redos;       /* general-path chunks, since init, redone in the
                                 u128 form after a 64-bit headroom left +-2^63    */
} tbgpu_stats;
void tbgpu_last_stats(tbgpu_ctx* ctx, tbgpu_stats* out);
/* Enable per-phase HIP-event timing (adds a few event records per call). */
void tbgpu_set_profiling(tbgpu_ctx* ctx, int enable);
int  tbgpu_last_error(tbgpu_ctx* ctx, char* buf, uint32_t len);

#ifdef __cplusplus
}
#endif
#endif /* TBGPU_H */
