/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Single-threaded CPU restatement of TigerBeetle's StateMachine commit path for
 * create_accounts / create_transfers (reference: src/state_machine.zig).  It is
 * the parity checker for the HIP engine and the "port" CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it; the product path (tigerbeetle_amd, libtbgpu.so) never links or calls it.
 *
 * Parity pinning: the reference is Zig 0.11 and cannot be built here (no zig
 * toolchain, no network), so the oracle is pinned by the
 * reference's own known-answer tables (src/state_machine.zig:2032-2575),
 * transcribed as data under tests/golden/ (*.tbl files), plus the sum_overflows edge
 * cases (:1657-1672).  See DESIGN.md "Oracle".
 */
#ifndef TB_ORACLE_H
#define TB_ORACLE_H
#include "../include/tbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc orc_t;

orc_t* orc_new(uint64_t accounts_hint, uint64_t transfers_hint);
void orc_free(orc_t* o);

uint32_t orc_create_accounts(orc_t* o, uint64_t timestamp, const tbgpu_account_t* events, uint32_t count,
                             tbgpu_create_accounts_result_t* results);
uint32_t orc_create_transfers(orc_t* o, uint64_t timestamp, const tbgpu_transfer_t* events, uint32_t count,
                              tbgpu_create_transfers_result_t* results);
/* Streaming: one create_transfers commit per batch, in order (same layout as
 * tbgpu_create_transfers_batches).  Returns the total result count; *elapsed_s
 * (if non-NULL) receives the wall time of the commit loop alone. */
uint64_t orc_create_transfers_batches(orc_t* o, uint32_t batch_count, const uint64_t* timestamps,
                                      const uint32_t* counts, const tbgpu_transfer_t* events,
                                      tbgpu_create_transfers_result_t* results, uint32_t* result_counts,
                                      double* elapsed_s);
uint64_t orc_create_accounts_batches(orc_t* o, uint32_t batch_count, const uint64_t* timestamps,
                                     const uint32_t* counts, const tbgpu_account_t* events,
                                     tbgpu_create_accounts_result_t* results, uint32_t* result_counts);

/* Sharded commit: the routed form of create_transfers and its helpers, with the
 * semantics of tbgpu_create_transfers_routed / tbgpu_import_transfers /
 * tbgpu_advance_commit_timestamp (include/tbgpu.h). */
uint64_t orc_create_transfers_routed(orc_t* o, uint32_t batch_count, const uint32_t* counts,
                                     const tbgpu_transfer_t* events, const uint64_t* event_ts, const uint8_t* ctl,
                                     int dry_run, tbgpu_create_transfers_result_t* results, uint32_t* result_counts,
                                     uint64_t* commit_timestamp);
int orc_import_transfers(orc_t* o, const tbgpu_transfer_t* rows, uint32_t count);
void orc_advance_commit_timestamp(orc_t* o, uint64_t timestamp);

uint32_t orc_lookup_accounts(orc_t* o, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_account_t* out);
uint32_t orc_lookup_transfers(orc_t* o, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_transfer_t* out);
int orc_set_balances(orc_t* o, tbgpu_uint128_t id, tbgpu_uint128_t dp, tbgpu_uint128_t dpo, tbgpu_uint128_t cp,
                     tbgpu_uint128_t cpo);

uint32_t orc_get_account_transfers(orc_t* o, const tbgpu_account_filter_t* f, tbgpu_transfer_t* out);
uint32_t orc_get_account_history(orc_t* o, const tbgpu_account_filter_t* f, tbgpu_account_balance_t* out);

uint64_t orc_account_count(orc_t* o);
uint64_t orc_transfer_count(orc_t* o);
uint64_t orc_history_count(orc_t* o);
uint64_t orc_export_accounts(orc_t* o, tbgpu_account_t* out, uint64_t capacity); /* insertion order */
uint64_t orc_export_transfers(orc_t* o, uint64_t first, uint64_t count, tbgpu_transfer_t* out);
uint64_t orc_export_history(orc_t* o, uint64_t first, uint64_t count, tbgpu_account_history_t* out);
int orc_get_posted(orc_t* o, tbgpu_uint128_t pending_id);
uint64_t orc_commit_timestamp(orc_t* o);

/* sum_overflows (src/state_machine.zig:1645-1650), exported for its own test. */
int orc_sum_overflows_u64(uint64_t a, uint64_t b);
int orc_sum_overflows_u128(tbgpu_uint128_t a, tbgpu_uint128_t b);

#ifdef __cplusplus
}
#endif
#endif
