// fast.hip — single-pass create_transfers for balance-insensitive calls.
//
// When no event of a call can observe another event of the same call, the
// sequential loop of `execute` (src/state_machine.zig:1018-1083) degenerates to
// independent events: every result is decided by the pre-call state alone and
// every account's final balance is its initial balance plus the sum of its
// accepted deltas.  That holds when the call has
//   - no linked chains (no scope rollback),
//   - no post/void (no pending resolution) and no balancing transfers (no
//     amount clamped from a running balance),
//   - no account with debits/credits_must_not_exceed_* (no limit check) or
//     history (no per-event balance snapshot),
//   - no id committed twice (no intra-call `exists`),
//   - no possible u128 overflow: amounts < 2^64 and the high words of every
//     touched balance < 2^62, so no prefix sum of < 2^32 events can reach the
//     overflow checks of :1308-1318.
// Every event checks its own eligibility; one ineligible event flags the call
// (FL_SLOW), its balance deltas are subtracted again (fp_undo, exact modular
// inverse) and the call is redone by the general fixed-point path.
//
// fp_commit: classify + balance deltas (LDS-aggregated, u64 atomics with carry)
//            + optimistic stored rows at row_base + event.
// fp_chains: linked-chain members (deferred by fp_commit): chain bounds, first
//            failure, final results, deltas of the chains that hold.
// fp_index:  publish the accepted ids in the transfer-id index.
// With failures (results other than ok, the rare case for this path) fp_mask +
// scan3 + fp_fix place the rows at their ranks and write the sparse replies, then
// fp_index runs on the final rows.
#include "common.h"
#include "engine.h"
#include "fast.h"

namespace {

#ifndef FP_TILE
#define FP_TILE 512
#endif
constexpr int FP_THREADS = FP_TILE;        // one event per thread, one tile per workgroup
constexpr int AGG_SLOTS = 4 * FP_THREADS;  // LDS aggregation table (2x the sides of a tile)
constexpr u32 AGG_EMPTY = 0xFFFFFFFFu;
constexpr u8 FRES_SLOW = 0xFE;
constexpr u8 FRES_CHAIN = 0x80;  // | own result: a chain member awaiting fp_chains

__device__ __forceinline__ u32 fp_batch_of(const u32* __restrict__ b_start, u32 nb, u32 i) {
    u32 lo = 0, hi = nb;
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (b_start[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void atomic_sub_u128_small(u128* p, u64 a) {
    u64* w = (u64*)p;
    const u64 old = atomicSub((unsigned long long*)&w[0], (unsigned long long)a);
    if (old < a) atomicSub((unsigned long long*)&w[1], 1ull);
}

// Call-local duplicate detection among accepted ids (only run when the call's ids
// are not strictly increasing).  Linear probing with claims (event + 1) placed in
// the first empty slot: a later claimant of the same id meets the earlier claim
// before any empty slot.  Every claimed slot is cleared again by fp_index, so the
// table is all-zero at the start of each call.
// The id of accepted event i for the duplicate check and the hash insert: fp_commit's
// key copy, or the event itself when fp_commit skipped the copies (CNT_NOKEYS).
__device__ __forceinline__ u128 fp_key(const FastArgs& F, u32 i) {
    return F.counters[CNT_NOKEYS] ? F.ev[i].id : F.keys[i];
}

__device__ __forceinline__ bool gtab_claim_is_dup(const FastArgs& F, u128 id, u32 i) {
    u64 h = hash128(id) & F.gmask;
    for (;;) {
        const u32 prev = atomicCAS(&F.gtab[h], 0u, i + 1);
        if (prev == 0) {
            F.gpos[i] = (u32)h;
            return false;
        }
        if (fp_key(F, prev - 1) == id) {
            F.gpos[i] = NONE32;
            return true;
        }
        h = (h + 1) & F.gmask;
    }
}

// create_transfer_exists (src/state_machine.zig:1370-1389)
__device__ __forceinline__ u8 fp_exists(const Transfer& t, const Transfer& e) {
    if (t.flags != e.flags) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_FLAGS;
    if (t.debit_account_id != e.debit_account_id) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (t.credit_account_id != e.credit_account_id) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t.amount != e.amount) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_AMOUNT;
    if (t.user_data_128 != e.user_data_128) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (t.user_data_64 != e.user_data_64) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (t.user_data_32 != e.user_data_32) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (t.timeout != e.timeout) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_TIMEOUT;
    if (t.code != e.code) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_CODE;
    return TBGPU_CREATE_TRANSFER_EXISTS;
}

// Continue an account index probe after a first-slot miss; returns the slot.
__device__ __forceinline__ u64 aidx_probe_from(const Tables& T, u64 h, u128 id) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    for (;;) {
        h = (h + 1) & T.aidx_mask;
        const AccIdx& e = T.aidx[h];
        if (e.row1 == 0 || (e.id_lo == lo && e.id_hi == hi)) return h;
    }
}

// The rows a probe may compare: committed before this call (row < row_base).  A slot
// that names a row of this call is an eager claim (FastArgs::eager), whose row may or
// may not be stored yet: the claim itself decides a repeat (fp_claim_is_dup), so a probe
// of the pre-call state walks past it like a tombstone.
__device__ __forceinline__ bool xidx_committed(const Tables& T, u64 e, u64 row_base, u128 id) {
    const u32 r1 = xidx_r1(e);
    return r1 != XIDX_TOMB && r1 - 1 < row_base && (u32)(e >> 32) == xidx_fp(id) && T.xrows[r1 - 1].id == id;
}

// A slot this call claimed was empty before the call, so no committed row with the id
// lies past it (linear probing): the probe ends there, as at an empty slot.  `*end` is
// where it ended: the slot an eager claim of the id starts at (the occupied slots before
// it hold other ids, and stay occupied through the call).
__device__ __forceinline__ bool xidx_ends_probe(u64 e, u64 row_base) {
    const u32 r1 = xidx_r1(e);
    return r1 == 0 || (r1 != XIDX_TOMB && r1 - 1 >= row_base);
}

__device__ __forceinline__ u32 xidx_probe_from(const Tables& T, u64 h, u128 id, u64 row_base, u64* end = nullptr) {
    for (;;) {
        h = (h + XIDX_STEP) & T.xidx_mask;
        const u64 e = T.xidx[h];
        if (xidx_ends_probe(e, row_base)) {
            if (end) *end = h;
            return NONE32;
        }
        if (xidx_committed(T, e, row_base, id)) return xidx_r1(e) - 1;
    }
}

// xidx_probe (engine.h) over the pre-call state only (see xidx_committed).
__device__ __forceinline__ u32 xidx_probe_pre(const Tables& T, u128 id, u64 row_base) {
    if (xidx_maybe_present(T, id)) {
        const u64 h = xidx_hash(id) & T.xidx_mask;
        const u64 e = T.xidx[h];
        if (xidx_r1(e) != 0) {
            const u32 r = xidx_committed(T, e, row_base, id) ? xidx_r1(e) - 1 : xidx_probe_from(T, h, id, row_base);
            if (r != NONE32) return r;
        }
    }
    return xrun_maybe(T, id) ? xrun_find(T, id) : NONE32;
}

// Eager claim of accepted event i's id (FastArgs::eager) at its optimistic row: the
// first empty slot of its probe sequence, by CAS.  The pre-call index was probed by
// classify (no committed row has this id), so any slot met on the way that names this
// call's rows (>= row_base: event row - row_base, whose id is read from the events)
// with the same id is a repeat within the call: returns true (nothing claimed).
__device__ __forceinline__ bool fp_claim_is_dup(const Tables& T, const FastArgs& F, u128 id, u64 row_base, u32 i,
                                                u64 h, u32* slot) {
    const u64 mine = xidx_slot(id, (u32)(row_base + i));
    const u32 fp = (u32)(mine >> 32);
    for (;;) {
        const u64 pe = atomicCAS((unsigned long long*)&T.xidx[h], 0ull, (unsigned long long)mine);
        const u32 prev = xidx_r1(pe);
        if (pe == 0) {
            *slot = (u32)h;
            return false;
        }
        if (prev != XIDX_TOMB && prev - 1 >= row_base && (u32)(pe >> 32) == fp && F.ev[prev - 1 - row_base].id == id) {
            *slot = NONE32;
            return true;
        }
        h = (h + XIDX_STEP) & T.xidx_mask;
    }
}

__device__ __forceinline__ u8 fp_classify_guarded(const Tables& T, const FastArgs& F, const Transfer& t, u32 i,
                                                  u64 ts, u64 row_base, u32* dslot_out, u32* cslot_out);

// Result of one event against the pre-call state, or FRES_SLOW.  The debit and
// credit account rows, the transfer-id slot and the duplicate claim are all
// issued before any of them is consumed (they are independent; only the
// precedence of the resulting checks is ordered), so one event costs about one
// memory round trip instead of four.
__device__ __forceinline__ u8 fp_classify(const Tables& T, const FastArgs& F, const Transfer& t, u32 i, u64 ts,
                                          u64 row_base, u32* dslot_out, u32* cslot_out, u64* xend) {
    const u16 f = t.flags;
    *xend = xidx_hash(t.id) & T.xidx_mask;  // (the guarded form's claims start at the id's slot)
    if (f & (TF_BDR | TF_BCR | TF_POST | TF_VOID) || (*T.big & 1))
        return fp_classify_guarded(T, F, t, i, ts, row_base, dslot_out, cslot_out);
    // speculative first-slot reads (hash tables at load <= 0.5: usually the hit).
    // The 32-byte account index entries carry ledger and flags, so the rows
    // themselves are only touched by the balance atomics.
    u64 hd = hash128(t.debit_account_id) & T.aidx_mask;
    u64 hc = hash128(t.credit_account_id) & T.aidx_mask;
    // Ids in the direct-mapped directory read its 8-byte entry, others the 32-byte index slot.
    AccIdx A, B;
    const bool dd = dense_has(T, t.debit_account_id), dc = dense_has(T, t.credit_account_id);
    u64 EA = 0, EB = 0;
    if (FP_ABLATE & ABL_PROBE) {  // timing only: no index reads (slots and fields made up)
        A = {(u64)t.debit_account_id, (u64)(t.debit_account_id >> 64), (u32)(hd % 1000) + 1, t.ledger, 0, 1, 0};
        B = {(u64)t.credit_account_id, (u64)(t.credit_account_id >> 64), (u32)(hc % 1000) + 1, t.ledger, 0, 1, 0};
    } else {
        if (dd) EA = T.dense[dense_slot(T, t.debit_account_id)]; else A = T.aidx[hd];
        if (dc) EB = T.dense[dense_slot(T, t.credit_account_id)]; else B = T.aidx[hc];
    }
    const bool maybe = !(FP_ABLATE & (ABL_IDS | ABL_XREAD)) && xidx_maybe_present(T, t.id);  // (ABL_*: timing only)
    const u64 hx = xidx_hash(t.id) & T.xidx_mask;
    const u64 x_r1 = maybe ? T.xidx[hx] : 0ull;
    if (t.timestamp != 0) return TBGPU_CREATE_TRANSFER_TIMESTAMP_MUST_BE_ZERO;
    if (f & 0xFFC0u) return TBGPU_CREATE_TRANSFER_RESERVED_FLAG;
    if (t.id == 0) return TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_ZERO;
    if (t.id == U128_MAX) return TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_INT_MAX;
    if (t.debit_account_id == 0) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t.debit_account_id == U128_MAX) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t.credit_account_id == 0) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t.credit_account_id == U128_MAX) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t.credit_account_id == t.debit_account_id) return TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_BE_DIFFERENT;
    if (t.pending_id != 0) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_ZERO;
    if (!(f & TF_PENDING) && t.timeout != 0) return TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    if (t.amount == 0) return TBGPU_CREATE_TRANSFER_AMOUNT_MUST_NOT_BE_ZERO;
    if (t.ledger == 0) return TBGPU_CREATE_TRANSFER_LEDGER_MUST_NOT_BE_ZERO;
    if (t.code == 0) return TBGPU_CREATE_TRANSFER_CODE_MUST_NOT_BE_ZERO;
    if (!(FP_ABLATE & ABL_PROBE)) {
        if (dd) A = {(u64)t.debit_account_id, 0, (u32)(EA & 0x1FFFFFFFu), (u32)(EA >> 32), (u16)((EA >> 28) & 0xE), 0, 0};
        if (dc) B = {(u64)t.credit_account_id, 0, (u32)(EB & 0x1FFFFFFFu), (u32)(EB >> 32), (u16)((EB >> 28) & 0xE), 0, 0};
    }
    const u64 dlo = (u64)t.debit_account_id, dhi = (u64)(t.debit_account_id >> 64);
    if (A.row1 != 0 && (A.id_lo != dlo || A.id_hi != dhi)) A = T.aidx[aidx_probe_from(T, hd, t.debit_account_id)];
    if (A.row1 == 0) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_NOT_FOUND;
    const u64 clo = (u64)t.credit_account_id, chi = (u64)(t.credit_account_id >> 64);
    if (B.row1 != 0 && (B.id_lo != clo || B.id_hi != chi)) B = T.aidx[aidx_probe_from(T, hc, t.credit_account_id)];
    if (B.row1 == 0) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_NOT_FOUND;
    if (A.ledger != B.ledger) return TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t.ledger != A.ledger) return TBGPU_CREATE_TRANSFER_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
    if (!ledger_owned(T, t.ledger)) return FRES_SLOW;  // another shard's ledger (the general path refuses it)
    if ((A.flags | B.flags) & (AF_DNEC | AF_CNED | AF_HISTORY)) return FRES_SLOW;  // limits / history
    if (maybe && !xidx_ends_probe(x_r1, row_base)) {
        const u32 pre = xidx_committed(T, x_r1, row_base, t.id) ? xidx_r1(x_r1) - 1
                                                                 : xidx_probe_from(T, hx, t.id, row_base, xend);
        if (pre != NONE32) return fp_exists(t, T.xrows[pre]);
    }
    if (xrun_maybe(T, t.id)) {  // the sorted run (an id replayed from an earlier call)
        const u32 pre = xrun_find(T, t.id);
        if (pre != NONE32) return fp_exists(t, T.xrows[pre]);
    }
    const u32 ds = A.row1 - 1, cs = B.row1 - 1;
    // an id repeated within the call is caught by fp_dupcheck (only when ids are not increasing)
    // u128 overflow is impossible: amount < 2^64, balances < 2^126 (T.big clear), < 2^32 events
    if ((u64)(t.amount >> 64) != 0) return FRES_SLOW;
    if (sum_overflows64(ts, (u64)t.timeout * NS_PER_S)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT;
    *dslot_out = ds;
    *cslot_out = cs;
    return TBGPU_CREATE_TRANSFER_OK;
}

// The static checks that precede what makes an event ineligible (their results
// are exact); otherwise FRES_SLOW.
__device__ __forceinline__ u8 fp_classify_guarded(const Tables& T, const FastArgs& F, const Transfer& t, u32 i,
                                                       u64 ts, u64 row_base, u32* dslot_out, u32* cslot_out) {
    const u16 f = t.flags;
    if (t.timestamp != 0) return TBGPU_CREATE_TRANSFER_TIMESTAMP_MUST_BE_ZERO;
    if (f & 0xFFC0u) return TBGPU_CREATE_TRANSFER_RESERVED_FLAG;
    if (t.id == 0) return TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_ZERO;
    if (t.id == U128_MAX) return TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_INT_MAX;
    if (f & (TF_POST | TF_VOID)) {
        if ((f & TF_POST) && (f & TF_VOID)) return TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
        if (f & (TF_PENDING | TF_BDR | TF_BCR)) return TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
        if (t.pending_id == 0) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_ZERO;
        if (t.pending_id == U128_MAX) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_INT_MAX;
        if (t.pending_id == t.id) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_DIFFERENT;
        if (t.timeout != 0) return TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
        return FRES_SLOW;  // resolves a pending transfer
    }
    if (t.debit_account_id == 0) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t.debit_account_id == U128_MAX) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t.credit_account_id == 0) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t.credit_account_id == U128_MAX) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t.credit_account_id == t.debit_account_id) return TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_BE_DIFFERENT;
    if (t.pending_id != 0) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_ZERO;
    if (!(f & TF_PENDING) && t.timeout != 0) return TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    if (!(f & (TF_BDR | TF_BCR)) && t.amount == 0) return TBGPU_CREATE_TRANSFER_AMOUNT_MUST_NOT_BE_ZERO;
    if (t.ledger == 0) return TBGPU_CREATE_TRANSFER_LEDGER_MUST_NOT_BE_ZERO;
    if (t.code == 0) return TBGPU_CREATE_TRANSFER_CODE_MUST_NOT_BE_ZERO;
    u32 dled, cled;
    u16 dfl, cfl;
    const u32 ds = acc_find(T, t.debit_account_id, &dled, &dfl);
    if (ds == NONE32) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_NOT_FOUND;
    const u32 cs = acc_find(T, t.credit_account_id, &cled, &cfl);
    if (cs == NONE32) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_NOT_FOUND;
    if (dled != cled) return TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t.ledger != dled) return TBGPU_CREATE_TRANSFER_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
    if (!ledger_owned(T, t.ledger)) return FRES_SLOW;  // another shard's ledger (the general path refuses it)
    if (f & (TF_BDR | TF_BCR)) return FRES_SLOW;                     // balancing
    if ((dfl | cfl) & (AF_DNEC | AF_CNED | AF_HISTORY)) return FRES_SLOW;  // limits / history
    const Account& dr = T.acc[ds];
    const Account& cr = T.acc[cs];
    const u32 pre = xidx_probe_pre(T, t.id, row_base);
    if (pre != NONE32) return fp_exists(t, T.xrows[pre]);
    // an id repeated within the call is caught by fp_dupcheck, as on the unguarded path
    // overflow impossible: amount < 2^64 and the touched balances' high words < 2^62
    const u64 lim = 1ull << 62;
    if ((u64)(t.amount >> 64) != 0) return FRES_SLOW;
    if ((u64)(dr.debits_pending >> 64) >= lim || (u64)(dr.debits_posted >> 64) >= lim) return FRES_SLOW;
    if ((u64)(cr.credits_pending >> 64) >= lim || (u64)(cr.credits_posted >> 64) >= lim) return FRES_SLOW;
    if (sum_overflows64(ts, (u64)t.timeout * NS_PER_S)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT;
    *dslot_out = ds;
    *cslot_out = cs;
    return TBGPU_CREATE_TRANSFER_OK;
}

// Balance field of an account row: 0 debits_pending, 1 debits_posted,
// 2 credits_pending, 3 credits_posted (offsets 16, 32, 48, 64).
__device__ __forceinline__ u128* acc_field(const Tables& T, u32 key) {
    return &(&T.acc[key >> 2].debits_pending)[key & 3];
}

// Add `a` to the tile's LDS partial sum for `key` (= slot * 4 + field).  Sums
// are 64-bit with a carry counter, so no precision is lost.
template <int SLOTS>
__device__ __forceinline__ void agg_add(u32* keys, u64* sums, u32* carries, u32 key, u64 a) {
    u32 h = (u32)(mix64(key) & (SLOTS - 1));
    for (;;) {
        u32 k = keys[h];
        if (k == AGG_EMPTY) {
            k = atomicCAS(&keys[h], AGG_EMPTY, key);
            if (k == AGG_EMPTY) k = key;
        }
        if (k == key) break;
        h = (h + 1) & (SLOTS - 1);
    }
    const u64 old = atomicAdd((unsigned long long*)&sums[h], (unsigned long long)a);
    if (old + a < old) atomicAdd(&carries[h], 1u);
}

// Events are loaded with coalesced 16-byte loads and handed to their lanes through
// LDS (0.95 vs 1.03 ms per 8.19M transfers for one 128-byte load per lane;
// FP_LANE_EVENTS builds the latter).  Stored rows staged the same way, or stored
// coalesced for every event right after the load, measured slower than the
// lane-per-row stores (profiles/micro/README.md).
#if !defined(FP_LANE_EVENTS)
#define FP_LDS_EVENTS 1
#endif
// Per-wave LDS staging of 128-byte records: STAGE_RECS records of 8 16-byte chunks,
// chunk c of record e at e*8 + (c ^ (e & 7)) so the lane-per-record writes and reads
// spread over the banks.  16 records (four rounds per wave) keep the workgroup's LDS
// at 49 KB, so three workgroups (24 waves) fit a CU; 32 records (two rounds, 66 KB)
// left room for two.
#ifndef FP_STAGE_RECS
#define FP_STAGE_RECS 16
#endif
constexpr int STAGE_RECS = FP_STAGE_RECS;
static_assert(STAGE_RECS == 16 || STAGE_RECS == 32, "staging rounds");
__device__ __forceinline__ u32 stage_slot(u32 e, u32 c) { return e * 8 + (c ^ (e & 7)); }
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef FP_WAVES_PER_EU
#define FP_WAVES_PER_EU 6  // 6: 24 waves per CU, the LDS limit (+5-7 % over 5, profiles/r06/ab_waves.txt); 7..8 slower
#endif
// One tile of TILE events per workgroup.  Rows are stored optimistically at
// row_base + event (every event accepted, the benchmark's case); failures are
// counted and, if there are any, fp_fix moves the rows to their ranks afterwards.
// SMALL (a drop-in call of at most FP_TAIL_MAX events, fp_commit_small): 64-event
// tiles, so one 8190-event prepare spans 128 CUs instead of 16; no fp_prep before it
// (its batch block comes in the kernel arguments, and the tile's flags and failure
// count go to its tile record instead of the call's counters, which fp_tail sets
// from the records: nothing here needs them reset first).
__device__ void fp_small_tail(const Tables& T, const FastArgs& F, const BlockInline& bi, const TailReport& rp);

// A prepared commit's gate, in each tile (one wave; lane 0 polls): the commit call's
// timestamp once the tiles agree on GO, or ~0 when they agree on OFF (cancelled, or no
// commit within the budget).  Tile 0 alone polls the host's word (128 tiles reading
// pinned memory in a loop slowed the whole call down), and publishes the timestamp in
// device memory, then the verdict, tagged with the call's sequence number, by CAS; the
// other tiles poll that device word.  Any tile whose budget runs out first sets OFF by
// the same CAS, so either every tile runs or none does.
__device__ __forceinline__ u64 fp_gate_wait(const FastArgs& F, const GateArgs& G) {
    u64 ts = ~0ull;
    if ((threadIdx.x & 63) == 0) {
        const u32 seq = F.gate_seq, tag_go = gate_tag(seq, GATE_GO), tag_off = gate_tag(seq, GATE_OFF);
        const bool poller = blockIdx.x == 0;
        u64* ts_dev = (u64*)(F.gate + 2);  // (8-byte aligned: the gate words are u32[4])
        const u64 t0 = wall_clock64();
        u32 v = 0;
        for (;;) {
            u32 d = __hip_atomic_load(F.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d == tag_go || d == tag_off) {
                v = d;
                break;
            }
            u32 want = 0;
            u64 t_go = 0;
            if (poller) {
                // (relaxed: the host wrote the timestamp before GO, and the timestamp is read
                // only after GO was seen, from the same coherent host memory)
                const u32 go = __hip_atomic_load(G.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (go == seq) {
                    want = tag_go;
                    t_go = __hip_atomic_load(G.ts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(ts_dev, t_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if ((go & GATE_CANCEL_BIT) && ((go - seq) & ~GATE_CANCEL_BIT) < (GATE_CANCEL_BIT >> 1)) {
                    want = tag_off;  // a cancel of every prepared commit up to a sequence >= ours
                }
            }
            if (!want && wall_clock64() - t0 > G.budget) want = tag_off;
            if (want) {
                // The timestamp's sc1 store has completed before the verdict's CAS, and the
                // other tiles read it with an sc1 load after seeing the verdict: the
                // hand-off of MI355X_MICROARCH.md's sc1 forms, without the release's L2
                // write-back or the acquire's L1 invalidate (≈1.7 µs each)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (__hip_atomic_compare_exchange_strong(F.gate, &d, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)) {
                    v = want;
                    if (want == tag_off) __hip_atomic_store(G.ack, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                continue;  // another tile decided first: follow it
            }
            if (poller) __builtin_amdgcn_s_sleep(2);
            else __builtin_amdgcn_s_sleep(8);
        }
        if (v == tag_go) ts = __hip_atomic_load(ts_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return __shfl((unsigned long long)ts, 0);
}

template <int TILE, bool SMALL>
__device__ __forceinline__ void fp_commit_body(const Tables& T, FastArgs F, const BlockInline& bi,
                                               const TailReport& rp = TailReport{}, const GateArgs& G = GateArgs{}) {
    constexpr int AGG = 4 * TILE;  // LDS aggregation table (2x the sides of a tile)
    __shared__ u64 s_maxts[TILE / 64];
    __shared__ u32 s_cnt[TILE / 64][2];
    __shared__ u64 s_idr[TILE / 64][4];
    __shared__ u32 s_keys[AGG];
    __shared__ u64 s_sums[AGG];
    __shared__ u32 s_carry[AGG];
    __shared__ u32 s_flags;
    __shared__ u32 s_blk[BLOCK_INLINE_WORDS];
#if defined(FP_LDS_EVENTS)
    __shared__ uint4 s_stage[TILE / 64][STAGE_RECS * 8];
#endif
    // a prepared commit (SMALL only): classify now, change state once the commit has come
    const bool gated = SMALL && F.gate != nullptr;
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32 tile = blockIdx.x;
    const u32 i = tile * TILE + tid;
    const bool valid = i < F.n;
    const u32 wbase = tile * TILE + wave * 64;
    if (SMALL) {
        // the call's batch block from the arguments (nothing has written it to memory yet)
        if (bi.words) {
            if (tid < bi.words) s_blk[tid] = bi.w[tid];
            F.b_start = s_blk;
            F.b_ts = (const u64*)(s_blk + ((F.nb + 2) & ~1u));  // batch_ts_offset
        }
    }
    // the tile's FL_* flags gather in LDS (a per-wave atomic on the call's flag word
    // serialized at the memory side: 128k waves of random ids each raising
    // FL_NONMONO, half of config 4's waves raising FL_FCHAIN), then one atomic per tile
    if (tid == 0) s_flags = 0;
    const u64 row_base = T.base[BASE_ROWS];  // device cursor: no host round trip between calls
    // When this call's rows will extend the id index's sorted run if every event is
    // accepted with rising ids (the benchmark's case: fp_run), nothing needs the id
    // copies: skip the 16 bytes per event (fp_key reads the events otherwise).
    bool keys = true;
    if (F.n && !F.dry) {
        const u64* xr = T.xrun;
        keys = !(xr[0] == xr[1] || (xr[1] == row_base && F.ev[0].id > (((u128)xr[5] << 64) | xr[4])));
#if defined(FP_KEYS_ALWAYS)  // timing variant: the copies as before
        keys = true;
#endif
        if (tile == 0 && tid == 0)  // (fp_tail keeps it; an sc1 store: the last small tile reads it)
            __hip_atomic_store(&F.counters[CNT_NOKEYS], keys ? 0u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#if defined(FP_LDS_EVENTS)
    // The wave's 64 events as coalesced 16-byte loads (lane k of load j holds chunk
    // (j*64 + k) of the wave's span), issued before the table init and the scalar
    // batch lookup, which do not depend on them.  (Measured alike to issuing them
    // after the lookup: 0.93-0.94 ms either way per 8.19M transfers.  Loading lane
    // 0's predecessor event up here in every lane, so that no branch waits on it,
    // was slower: 0.98 ms.)
    // Chunks past the last event re-read the last chunk (unconditional loads: no
    // branch between them); they only reach lanes without an event.
    // (eight named registers: an array live across the loops below went to scratch)
    uint4 c0{}, c1{}, c2{}, c3{}, c4{}, c5{}, c6{}, c7{};
    if (!(FP_ABLATE & ABL_EVENT) && F.n) {
        const uint4* src = (const uint4*)F.ev;
        const u64 last = (u64)F.n * 8 - 1, q0 = (u64)wbase * 8 + lane;
        c0 = src[min(q0, last)];
        c1 = src[min(q0 + 64, last)];
        c2 = src[min(q0 + 128, last)];
        c3 = src[min(q0 + 192, last)];
        c4 = src[min(q0 + 256, last)];
        c5 = src[min(q0 + 320, last)];
        c6 = src[min(q0 + 384, last)];
        c7 = src[min(q0 + 448, last)];
    }
#endif
    for (u32 h = tid; h < AGG; h += TILE) {
        s_keys[h] = AGG_EMPTY;
        s_sums[h] = 0;
        s_carry[h] = 0;
    }
    __syncthreads();

    u8 r = FRES_SLOW;
    u32 b = 0;
    u64 ts = 0;
    u128 id = 0;
    // batch of the event: one uniform (scalar) binary search per wave; a wave spans
    // 64 events, so usually one batch, and the lanes past a boundary walk on
    const u32 i0 = __builtin_amdgcn_readfirstlane(wbase);
    Transfer t{};
    u32 bs = 0, nbatch = 0;
    if (gated) {  // one batch; its timestamp comes with the commit (fp_gate_wait)
        if (valid) {
            b = 0;
            bs = 0;
            nbatch = F.n;
        }
    } else if (i0 < F.n) {
        const u32 b0 = fp_batch_of(F.b_start, F.nb, i0);
        const u32 s0 = F.b_start[b0], e0 = F.b_start[b0 + 1];
        const u64 t0 = F.ev_ts ? 0 : F.b_ts[b0];
        if (valid) {
            if (i < e0) {
                b = b0;
                bs = s0;
                nbatch = e0 - s0;
            } else {
                b = b0 + 1;
                while (F.b_start[b + 1] <= i) b++;
                bs = F.b_start[b];
                nbatch = F.b_start[b + 1] - bs;
            }
            ts = F.ev_ts ? F.ev_ts[i] : (b == b0 ? t0 : F.b_ts[b]) - nbatch + (i - bs) + 1;
        }
    }
    if (valid) {
        if (FP_ABLATE & ABL_EVENT) {  // timing only: a made-up plain event instead of the load
            t.id = (u128)i + 1 + F.row_base;
            t.debit_account_id = (i * 7919u) % 1000000u + 1;
            t.credit_account_id = (i * 104729u + 1) % 1000000u + 1;
            if (t.credit_account_id == t.debit_account_id) t.credit_account_id = t.debit_account_id % 1000000u + 1;
            t.amount = 5;
            t.ledger = 1;
            t.code = 1;
        } else {
#if !defined(FP_LDS_EVENTS)
            t = F.ev[i];
#endif
        }
    }
#if defined(FP_LDS_EVENTS)
    // the wave's events through LDS in rounds of STAGE_RECS, one record per lane
    if (!(FP_ABLATE & ABL_EVENT)) {
        uint4* st = s_stage[wave];
        constexpr int ROUNDS = 64 / STAGE_RECS;
#pragma unroll
        for (int h = 0; h < ROUNDS; h++) {
            // chunk j*64 + lane of the wave's span: event (j*64 + lane) / 8 - STAGE_RECS*h
#define STAGE(j, c) st[stage_slot(((j) * 64 + lane) / 8 - STAGE_RECS * h, lane & 7)] = (c)
            if (ROUNDS == 2) {
                if (h == 0) { STAGE(0, c0); STAGE(1, c1); STAGE(2, c2); STAGE(3, c3); }
                else { STAGE(4, c4); STAGE(5, c5); STAGE(6, c6); STAGE(7, c7); }
            } else {
                if (h == 0) { STAGE(0, c0); STAGE(1, c1); }
                else if (h == 1) { STAGE(2, c2); STAGE(3, c3); }
                else if (h == 2) { STAGE(4, c4); STAGE(5, c5); }
                else { STAGE(6, c6); STAGE(7, c7); }
            }
#undef STAGE
            wave_lds_sync();
            if (lane / STAGE_RECS == (u32)h && valid) {
                uint4* tv = (uint4*)&t;
#pragma unroll
                for (int c = 0; c < 8; c++) tv[c] = st[stage_slot(lane % STAGE_RECS, c)];
            }
            wave_lds_sync();
        }
    }
#endif
    if (F.ev_copy && valid) F.ev_copy[i] = t;  // events read in place from host memory: an HBM
                                               // copy for the launches after this one
    // Linked-chain membership (execute, src/state_machine.zig:1018-1035): linked
    // here, or the batch's previous event is (the router may close a chain that
    // continues on another shard: TBGPU_CTL_CHAIN_END).
    const u8 myctl = (valid && F.ctl) ? F.ctl[i] : 0;
    const bool lk = valid && (t.flags & TF_LINKED) && !(myctl & TBGPU_CTL_CHAIN_END);
    bool plk = __shfl_up(lk ? 1 : 0, 1) != 0;
    if (lane == 0 && valid && i > 0)
        plk = (F.ev[i - 1].flags & TF_LINKED) && !(F.ctl && (F.ctl[i - 1] & TBGPU_CTL_CHAIN_END));
    plk = plk && valid && i > bs;
    const bool member = lk || plk || (myctl & TBGPU_CTL_DOOM);
    if (__ballot(member) && lane == 0) atomicOr(&s_flags, (u32)FL_FCHAIN);
    bool own_ok = false;
#if defined(FP_NT_ROWS)  // timing variant: rows written with non-temporal stores
#define STORE_ROW() do { if (!(FP_ABLATE & ABL_ROWS)) { \
    typedef unsigned int v4u_ __attribute__((ext_vector_type(4))); \
    v4u_* d_ = (v4u_*)&T.xrows[row_base + i]; const v4u_* s_ = (const v4u_*)&t; \
    for (int c_ = 0; c_ < 8; c_++) __builtin_nontemporal_store(s_[c_], &d_[c_]); } } while (0)
#else
#define STORE_ROW() do { if (!(FP_ABLATE & ABL_ROWS)) T.xrows[row_base + i] = t; } while (0)
#endif
    u32 ds = NONE32, cs = NONE32;
    u64 xend = 0;  // where an eager claim starts (fp_classify)
#define FP_CLASSIFY()                                                                                                \
    do {                                                                                                             \
        id = t.id;                                                                                                   \
        xend = xidx_hash(t.id) & T.xidx_mask;                                                                        \
        if (lk && i - bs == nbatch - 1) r = TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN; /* checked first (:1024) */ \
        else if (myctl & TBGPU_CTL_SKIP) r = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED; /* broken on another shard */  \
        else r = fp_classify(T, F, t, i, ts, row_base, &ds, &cs, &xend);                                             \
    } while (0)
    if (SMALL && valid) FP_CLASSIFY();  // (gated: ts 0 until the commit)
    if (gated) {
        // everything above only read the pre-call state (the previous commit's launches
        // are done: they precede these on the stream); state changes only after GO
        const u64 T0 = fp_gate_wait(F, G);
        if (T0 == ~0ull) return;  // the commit did not come: nothing was changed
        if (tile == 0 && tid == 0) {
            // the batch block and the reply cursor for the launches after this one
            ((u32*)F.b_start)[0] = 0;
            ((u32*)F.b_start)[1] = F.n;
            *(u64*)F.b_ts = T0;
            T.base[BASE_REPLIES] = 0;
        }
        if (valid) {
            ts = T0 - F.n + i + 1;
            // overflows_timeout, the last check of create_transfer (:1323-1325) and the only
            // one that reads the timestamp: classify ran with 0, where it never fires
            if (r == TBGPU_CREATE_TRANSFER_OK && t.timeout != 0 && sum_overflows64(ts, (u64)t.timeout * NS_PER_S))
                r = TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT;
        }
    }
    if (valid) {
        if (!SMALL) FP_CLASSIFY();
#undef FP_CLASSIFY
        own_ok = r == TBGPU_CREATE_TRANSFER_OK;
        if (F.eager) {
            u32 slot = NONE32;
            if (FP_ABLATE & ABL_CLAIM_STORE) {  // timing only: the claim as a plain store, no repeat check
                if (own_ok) {
                    T.xidx[xend] = xidx_slot(t.id, (u32)(row_base + i));
                    slot = (u32)xend;
                }
            } else if (own_ok && !(FP_ABLATE & ABL_IDS) && fp_claim_is_dup(T, F, t.id, row_base, i, xend, &slot)) {
                r = FRES_SLOW;  // an id repeated within the call: the fixed point decides it
                own_ok = false;
            }
            F.gpos[i] = slot;
        }
        if (member && r != FRES_SLOW) {
            // deferred to fp_chains: no balance delta, no count; the optimistic row
            // and the id claim as for any accepted event
            F.fres[i] = FRES_CHAIN | r;
            if (own_ok) {
                if (keys) F.keys[i] = t.id;
                t.timestamp = ts;
                STORE_ROW();
            }
            r = FRES_CHAIN;
        } else {
            F.fres[i] = r;
        }
        if (r == TBGPU_CREATE_TRANSFER_OK) {
            if (keys) F.keys[i] = t.id;
            // tile-local aggregation first: a hot account costs one global atomic per tile
            const u64 a = (u64)t.amount;
            const u32 pend = (t.flags & TF_PENDING) ? 0u : 1u;
            if (!(FP_ABLATE & ABL_BALANCES)) {
                agg_add<AGG>(s_keys, s_sums, s_carry, ds * 4 + pend, a);
                agg_add<AGG>(s_keys, s_sums, s_carry, cs * 4 + 2 + pend, a);
            }
            // optimistic stored row (every predecessor accepted); fp_fix re-places it otherwise
            t.timestamp = ts;
            STORE_ROW();
        } else if (r == FRES_SLOW) {
            atomicOr(&s_flags, (u32)FL_SLOW);
        } else if (r != FRES_CHAIN && !SMALL) {
            atomicAdd(&F.batch_counts[b], 1u);  // (SMALL: fp_tail counts each batch's replies)
        }
    }
#undef STORE_ROW
    const bool ok = valid && r == TBGPU_CREATE_TRANSFER_OK;
    const bool bad = valid && r != TBGPU_CREATE_TRANSFER_OK && r != FRES_CHAIN;

    // Strictly increasing ids across the whole call cannot repeat: then fp_dupcheck
    // has nothing to do (sequential ids, the benchmark's default id order).
    {
        const u64 lo = valid ? (u64)id : ~0ull, hi = valid ? (u64)(id >> 64) : ~0ull;
        u64 plo = __shfl_up((unsigned long long)lo, 1), phi = __shfl_up((unsigned long long)hi, 1);
        if (lane == 0) {
            if (i > 0 && valid) {
                const u128 p = F.ev[i - 1].id;
                plo = (u64)p;
                phi = (u64)(p >> 64);
            } else {
                plo = phi = 0;
            }
        }
        const bool up = !valid || i == 0 || hi > phi || (hi == phi && lo > plo);
        if (__ballot(!up) && lane == 0) atomicOr(&s_flags, (u32)FL_NONMONO);
    }
    const u64 okm = __ballot(ok), badm = __ballot(bad);
    u64 mts = ok ? ts : 0;
    for (int off = 32; off > 0; off >>= 1) mts = max(mts, (u64)__shfl_xor((unsigned long long)mts, off));
    // componentwise id range of the tile's accepted ids (for the index key-range filter)
    const bool rng = ok || own_ok;  // a chain member's id may still be stored
    u64 mxl = rng ? (u64)id : 0, mxh = rng ? (u64)(id >> 64) : 0;
    u64 mnl = rng ? (u64)id : ~0ull, mnh = rng ? (u64)(id >> 64) : ~0ull;
    for (int off = 32; off > 0; off >>= 1) {
        mxl = max(mxl, (u64)__shfl_xor((unsigned long long)mxl, off));
        mxh = max(mxh, (u64)__shfl_xor((unsigned long long)mxh, off));
        mnl = min(mnl, (u64)__shfl_xor((unsigned long long)mnl, off));
        mnh = min(mnh, (u64)__shfl_xor((unsigned long long)mnh, off));
    }
    if (lane == 0) {
        s_maxts[wave] = mts;
        s_cnt[wave][0] = __popcll(okm);
        s_cnt[wave][1] = __popcll(badm);
        s_idr[wave][0] = mxl;
        s_idr[wave][1] = mxh;
        s_idr[wave][2] = mnl;
        s_idr[wave][3] = mnh;
    }
    __syncthreads();  // LDS sums and per-wave figures complete
    if (wave == 0) {
        if (lane < 4) {
            u64 v = s_idr[0][lane];
            for (int w = 1; w < TILE / 64; w++) v = lane < 2 ? max(v, s_idr[w][lane]) : min(v, s_idr[w][lane]);
            __hip_atomic_store(&F.tile_idr[TILE_WORDS * tile + lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            u32 nok = 0, nbad = 0;
            u64 maxts = 0;
            for (int w = 0; w < TILE / 64; w++) {
                nok += s_cnt[w][0];
                nbad += s_cnt[w][1];
                maxts = max(maxts, s_maxts[w]);
            }
            // accepted count and commit timestamp: folded by fp_index (one atomic per
            // tile on one address would serialize 16k tiles at the memory side)
            // (sc1 stores: the last small tile reads the records with sc1 loads, fp_small_tail)
            __hip_atomic_store(&F.tile_idr[TILE_WORDS * tile + 4], maxts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&F.tile_idr[TILE_WORDS * tile + 5], (u64)nok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (SMALL) {
                __hip_atomic_store(&F.tile_idr[TILE_WORDS * tile + 6], (u64)nbad, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&F.tile_idr[TILE_WORDS * tile + 7], (u64)s_flags, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (nbad) atomicAdd(&F.counters[CNT_BAD], nbad);
                const u32 fl = s_flags;  // (skipped when an earlier tile raised them already)
                if (fl && (__hip_atomic_load(&F.counters[CNT_FLAGS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & fl) != fl)
                    atomicOr(&F.counters[CNT_FLAGS], fl);
            }
        }
    }
    // flush the tile's partial sums: u128 += (carry:sum) with u64 atomics.  All of a
    // thread's low-word atomics are issued before any returns (memory-level
    // parallelism); the rare carries follow.
    if (F.dry) return;  // a dry run moves no balance
    constexpr int PER = AGG / TILE;
    u64* wp[PER];
    u64 av[PER], old[PER];
    u32 cv[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const u32 h = tid + k * TILE;
        const u32 key = s_keys[h];
        wp[k] = key == AGG_EMPTY ? nullptr : (u64*)acc_field(T, key);
        av[k] = s_sums[h];
        cv[k] = s_carry[h];
    }
#if defined(FP_NOFLUSH)  // timing-only variants (profiles/variants.py); results wrong
    return;
#elif defined(FP_NORET)
#pragma unroll
    for (int k = 0; k < PER; k++)
        if (wp[k]) __hip_atomic_fetch_add((unsigned long long*)&wp[k][0], (unsigned long long)av[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
#endif
#if defined(FP_SKIP_HOT)  // timing-only variant (profiles/variants.py): no flush for the hottest rows; results wrong
#pragma unroll
    for (int k = 0; k < PER; k++)
        if (wp[k] && (s_keys[tid + k * TILE] >> 2) < FP_SKIP_HOT) wp[k] = nullptr;
#endif
#pragma unroll
    for (int k = 0; k < PER; k++)
        old[k] = wp[k] ? atomicAdd((unsigned long long*)&wp[k][0], (unsigned long long)av[k]) : 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        if (!wp[k]) continue;
        const u64 c = (u64)cv[k] + (old[k] + av[k] < old[k] ? 1 : 0);
        if (!(old[k] >> 61) && ((old[k] + av[k]) >> 61 || c)) atomicOr(T.big, 2u);  // crossed 2^61
        if (c) {
            const u64 hi = atomicAdd((unsigned long long*)&wp[k][1], (unsigned long long)c);
            if (hi + c >= (1ull << 62)) atomicOr(T.big, 1u);  // later calls must prove no overflow
        }
    }
    if constexpr (SMALL) {
        if (F.fuse) {
            // the last tile to finish (one wave per tile: its fence covers its record)
            static_assert(!SMALL || TILE == 64, "one wave per small tile");
            // Every tile's record (and tile 0's CNT_NOKEYS) went out as sc1 stores; the
            // wave waits for them, then takes its ticket (an agent-scope atomic), and the
            // tile whose ticket is last reads the records with sc1 loads: the counter
            // hand-off of MI355X_MICROARCH.md's sc1 forms (no release or acquire fence:
            // ≈3.5 µs each way as __threadfence)
            const u32 ntiles = (F.n + TILE - 1) / TILE;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            u32 t = 0;
            if (lane == 0) t = __hip_atomic_fetch_add(&F.counters[CNT_TICKET], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            t = __shfl(t, 0);
            if (t != ntiles - 1) return;
            fp_small_tail(T, F, bi, rp);
        }
    }
}

__global__ __launch_bounds__(FP_THREADS) __attribute__((amdgpu_waves_per_eu(FP_WAVES_PER_EU)))
void fp_commit(Tables T, FastArgs F) {
    fp_commit_body<FP_THREADS, false>(T, F, BlockInline{});
}

__global__ __launch_bounds__(FP_SMALL_TILE) void fp_commit_small(Tables T, FastArgs F, BlockInline bi, TailReport rp,
                                                                 GateArgs G) {
    fp_commit_body<FP_SMALL_TILE, true>(T, F, bi, rp, G);
}

// Only when the call's ids were not increasing: claim every accepted id once.
__device__ __forceinline__ void fp_dupcheck_one(const FastArgs& F, u32 i) {
    F.gpos[i] = NONE32;
    const u8 r = F.fres[i];
    if (r != TBGPU_CREATE_TRANSFER_OK && r != (FRES_CHAIN | TBGPU_CREATE_TRANSFER_OK)) return;
    if (gtab_claim_is_dup(F, fp_key(F, i), i)) atomicOr(&F.counters[CNT_FLAGS], (u32)FL_SLOW);
}

// The launches that usually stand down (no repeated-id check, no chains) run a
// small grid-stride grid: a full grid of 32k workgroups that all return at once
// still costs its dispatch.
#define FOR_EACH_EVENT(i) \
    for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < F.n; i += gridDim.x * blockDim.x)

__global__ void fp_dupcheck(Tables T, FastArgs F) {
    // Every event records its claim (or NONE) so fp_index can clear the table.
    if (F.eager || !(F.counters[CNT_FLAGS] & FL_NONMONO)) return;  // (eager: fp_commit's claims found repeats)
    FOR_EACH_EVENT(i) fp_dupcheck_one(F, i);
}

// Whether this call's rows extend the sorted run of the id index (engine.h xrun):
// every event accepted, ids strictly increasing, the first above the run's last id
// and the rows right after the run's.  Then the run takes them (CNT_RUN) and
// fp_index inserts nothing; otherwise fp_index hashes them as before.  One thread.
__device__ void fp_run_one(const Tables& T, const FastArgs& F, u32 flags, u32 bad) {
    u32 take = 0;
    if (!F.dry && !F.eager && F.n && !(flags & (FL_SLOW | FL_ERROR | FL_NONMONO)) && bad == 0) {
        u64* r = T.xrun;
        const u64 row0 = T.base[BASE_ROWS];
        const u128 first = F.ev[0].id, last = F.ev[F.n - 1].id;
        const bool empty = r[0] == r[1];
        if (empty || (r[1] == row0 && first > (((u128)r[5] << 64) | r[4]))) {
            if (empty) {
                r[0] = row0;
                r[2] = (u64)first;
                r[3] = (u64)(first >> 64);
            }
            r[1] = row0 + F.n;
            r[4] = (u64)last;
            r[5] = (u64)(last >> 64);
            take = 1;
        }
    }
    F.counters[CNT_RUN] = take;
    // whether the call stands with failures (the fix launches run; all of them are
    // enqueued without waiting for this answer)
    F.counters[CNT_FIX] = (bad != 0 && !(flags & (FL_SLOW | FL_ERROR))) ? 1u : 0u;
}

__global__ void fp_run(Tables T, FastArgs F) {
    if (threadIdx.x == 0) fp_run_one(T, F, F.counters[CNT_FLAGS], F.counters[CNT_BAD]);
}

// Publish the accepted ids.  fixed = false: the launch right after fp_commit, which
// stands down when the call had failures (rows not final yet) and always clears the
// duplicate claims; fixed = true: after fp_fix, rows from F.rows.
// One wave: tiles k0 .. k0 + 63's componentwise id ranges into T.idr.
__device__ __forceinline__ void fp_fold_idr(const Tables& T, const FastArgs& F, u32 k0, u32 ntiles) {
    if (k0 >= ntiles) return;
    const u32 k = k0 + (threadIdx.x & 63);
    u64 r[4] = {0, 0, ~0ull, ~0ull};
    if (k < ntiles)
        for (int w = 0; w < 4; w++)  // (sc1 loads: fp_small_tail reads records of this launch's tiles)
            r[w] = __hip_atomic_load(&F.tile_idr[TILE_WORDS * k + w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int off = 32; off > 0; off >>= 1) {
        r[0] = max(r[0], (u64)__shfl_xor((unsigned long long)r[0], off));
        r[1] = max(r[1], (u64)__shfl_xor((unsigned long long)r[1], off));
        r[2] = min(r[2], (u64)__shfl_xor((unsigned long long)r[2], off));
        r[3] = min(r[3], (u64)__shfl_xor((unsigned long long)r[3], off));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax((unsigned long long*)&T.idr[0], (unsigned long long)r[0]);
        atomicMax((unsigned long long*)&T.idr[1], (unsigned long long)r[1]);
        atomicMin((unsigned long long*)&T.idr[2], (unsigned long long)r[2]);
        atomicMin((unsigned long long*)&T.idr[3], (unsigned long long)r[3]);
    }
}

__global__ void fp_index(Tables T, FastArgs F, bool fixed) {
    if (fixed) {  // after fp_fix: the accepted ids at their final rows (grid-stride; gated like the fix)
        if (!F.counters[CNT_FIX] || F.dry) return;
        const u32 ntiles = (F.n + F.tile - 1) / F.tile;
        if (threadIdx.x < 64)
            for (u32 k0 = blockIdx.x * 64; k0 < ntiles; k0 += gridDim.x * 64) fp_fold_idr(T, F, k0, ntiles);
        if (!F.eager) FOR_EACH_EVENT(j) if (F.fres[j] == TBGPU_CREATE_TRANSFER_OK) xidx_insert(T, fp_key(F, j), F.rows[j]);
        return;
    }
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    const u32 flags = F.counters[CNT_FLAGS];
    if (!fixed && !F.eager && (flags & FL_NONMONO) && i < F.n) {
        // leave the claim table all-zero for the next call (also when falling back)
        const u32 g = F.gpos[i];
        if (g != NONE32) F.gtab[g] = 0;
    }
    const u32 ntiles = (F.n + F.tile - 1) / F.tile;
    if (!fixed && threadIdx.x < 64 && blockIdx.x * 64 < ntiles) {
        // the call's accepted count and commit timestamp from fp_commit's tiles
        // (also for dry runs and calls with failures; fp_undo restores the timestamp
        // when the call falls back)
        const u32 k = blockIdx.x * 64 + threadIdx.x;
        u64 mts = 0, nok = 0;
        if (k < ntiles) {
            mts = F.tile_idr[TILE_WORDS * k + 4];
            nok = F.tile_idr[TILE_WORDS * k + 5];
        }
        for (int off = 32; off > 0; off >>= 1) {
            mts = max(mts, (u64)__shfl_xor((unsigned long long)mts, off));
            nok += (u64)__shfl_xor((unsigned long long)nok, off);
        }
        if (threadIdx.x == 0) {
            if (nok) atomicAdd(&F.counters[CNT_OK], (u32)nok);
            if (mts) atomicMax((unsigned long long*)F.commit_ts, (unsigned long long)mts);
        }
    }
    if (flags & (FL_SLOW | FL_ERROR)) return;
    if (F.dry) return;
    if (!fixed && F.counters[CNT_BAD] != 0) return;
    if (!fixed && F.counters[CNT_RUN]) return;  // the rows extend the sorted run
    // fold the tiles' id ranges into the index's key range: one wave per 64 tiles (a
    // single wave over 16k tiles was a serial tail of this launch)
    if (threadIdx.x < 64) fp_fold_idr(T, F, blockIdx.x * 64, ntiles);
    if (i >= F.n || F.eager) return;  // (eager: claimed by fp_commit at these rows)
    if (F.fres[i] != TBGPU_CREATE_TRANSFER_OK) return;
    xidx_insert(T, fp_key(F, i), (u32)(T.base[BASE_ROWS] + i));
}

__device__ __forceinline__ bool fp_linked(const FastArgs& F, u32 j) {
    return (F.ev[j].flags & TF_LINKED) && !(F.ctl && (F.ctl[j] & TBGPU_CTL_CHAIN_END));
}

__device__ __forceinline__ void add_u128_small(const Tables& T, u128* p, u64 a) {
    u64* w = (u64*)p;
    const u64 old = atomicAdd((unsigned long long*)&w[0], (unsigned long long)a);
    if (!(old >> 61) && ((old + a) >> 61 || old + a < old)) atomicOr(T.big, 2u);  // crossed 2^61
    if (old + a < old) {
        const u64 hi = atomicAdd((unsigned long long*)&w[1], 1ull);
        if (hi + 1 >= (1ull << 62)) atomicOr(T.big, 1u);
    }
}

// Linked chains of eligible events (execute, src/state_machine.zig:1018-1083): a
// chain holds iff no member fails; otherwise the first failing member keeps its
// own result, every other member gets linked_event_failed (members after the
// break are not evaluated; linked_event_chain_open is checked before the break),
// and commit_timestamp advanced only by the accepted members before the break
// (:1366, not undone by scope_close).  Each member walks its own (short) chain;
// results go to fres2 so that no thread reads a finalized code.
// Counts and the timestamp go to the caller's per-thread sums (one atomic per
// workgroup after the loop: per-member atomics on one address serialize).
__device__ void fp_chains_one(const Tables& T, const FastArgs& F, u32 i, u32& n_ok, u32& n_bad, u64& mts) {
    const u8 fr = F.fres[i];
    if (!(fr & FRES_CHAIN) || fr == FRES_SLOW) return;
    const u8 own = fr & 0x7F;
    const u32 b = fp_batch_of(F.b_start, F.nb, i);
    const u32 bs = F.b_start[b], be = F.b_start[b + 1];
    u32 s = i;
    while (s > bs && fp_linked(F, s - 1)) s--;
    u32 e = i;
    while (e + 1 < be && fp_linked(F, e)) e++;
    u32 j = NONE32;
    for (u32 k = s; k <= e; k++)
        if ((F.fres[k] & 0x7F) != TBGPU_CREATE_TRANSFER_OK) { j = k; break; }
    if (j == NONE32 && F.ctl && (F.ctl[e] & TBGPU_CTL_DOOM)) j = e + 1;  // breaks on another shard
    u8 fin;
    if (j == NONE32) fin = TBGPU_CREATE_TRANSFER_OK;
    else if (own == TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN) fin = own;
    else if (i == j) fin = own;
    else fin = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
    F.fres2[i] = fin;
    const u64 nbatch = be - bs;
    const u64 ts = F.ev_ts ? F.ev_ts[i] : F.b_ts[b] - nbatch + (i - bs) + 1;
    if (own == TBGPU_CREATE_TRANSFER_OK && (j == NONE32 || i < j)) mts = max(mts, ts);
    if (fin == TBGPU_CREATE_TRANSFER_OK) {
        n_ok++;
        if (!F.dry) {
            const Transfer& t = F.ev[i];
            u32 led;
            u16 afl;
            const u32 ds = acc_find(T, t.debit_account_id, &led, &afl);
            const u32 cs = acc_find(T, t.credit_account_id, &led, &afl);
            const u64 a = (u64)t.amount;
            if (t.flags & TF_PENDING) {
                add_u128_small(T, &T.acc[ds].debits_pending, a);
                add_u128_small(T, &T.acc[cs].credits_pending, a);
            } else {
                add_u128_small(T, &T.acc[ds].debits_posted, a);
                add_u128_small(T, &T.acc[cs].credits_posted, a);
            }
        }
    } else {
        n_bad++;
        if (!F.small) atomicAdd(&F.batch_counts[b], 1u);  // (small: fp_tail counts each batch's replies)
        if (F.eager && F.gpos[i] != NONE32) {  // its claim withdrawn
            T.xidx[F.gpos[i]] = XIDX_TOMB;  // (the fingerprint goes too: a tombstone matches nothing)
            atomicAdd(&T.hcount[2], 1u);  // (xidx_tombs_check)
        }
    }
}

// Chain members are few (config 4: 1 %) and each costs a chain of dependent loads,
// so a wave first gathers the members among its grid-stride events into LDS (16
// result bytes per lane in one load), then its lanes take one member each: the
// members of ~1k events wait on memory together instead of one grid-stride step
// after the other (177 -> ~30 us per 8.19M events on config 4).
constexpr u32 CH_LIST = 1024;  // a wave's 64 lanes x 16 events: every member of one step
__global__ __launch_bounds__(256) void fp_chains(Tables T, FastArgs F) {
    const u32 flags = F.counters[CNT_FLAGS];
    if (!(flags & FL_FCHAIN) || (flags & (FL_SLOW | FL_ERROR))) return;
    u32 n_ok = 0, n_bad = 0;
    u64 mts = 0;
    __shared__ u32 s_list[4][CH_LIST];
    __shared__ u32 s_cnt[4];
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u32 nq = (F.n + 15) / 16, stride = gridDim.x * blockDim.x;
    for (u32 qb = blockIdx.x * blockDim.x + w * 64; qb < nq; qb += stride) {
        if (lane == 0) s_cnt[w] = 0;
        wave_lds_sync();
        const u32 q = qb + lane;
        if (q < nq) {
            const uint4 v = ((const uint4*)F.fres)[q];
            const u8* fb = (const u8*)&v;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const u32 i = q * 16 + k;
                if (i < F.n && (fb[k] & FRES_CHAIN) && fb[k] != FRES_SLOW) s_list[w][atomicAdd(&s_cnt[w], 1u)] = i;
            }
        }
        wave_lds_sync();
        const u32 cnt = s_cnt[w];
        for (u32 k = lane; k < cnt; k += 64) fp_chains_one(T, F, s_list[w][k], n_ok, n_bad, mts);
        wave_lds_sync();
    }
    __shared__ u32 s_ok, s_bad;
    __shared__ u64 s_mts;
    if (threadIdx.x == 0) { s_ok = 0; s_bad = 0; s_mts = 0; }
    __syncthreads();
    for (int off = 32; off > 0; off >>= 1) {
        n_ok += __shfl_xor(n_ok, off);
        n_bad += __shfl_xor(n_bad, off);
        mts = max(mts, (u64)__shfl_xor((unsigned long long)mts, off));
    }
    if ((threadIdx.x & 63) == 0) {
        if (n_ok) atomicAdd(&s_ok, n_ok);
        if (n_bad) atomicAdd(&s_bad, n_bad);
        if (mts) atomicMax((unsigned long long*)&s_mts, (unsigned long long)mts);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_ok) atomicAdd(&F.counters[CNT_OK], s_ok);
        if (s_bad) atomicAdd(&F.counters[CNT_BAD], s_bad);
        if (s_mts) atomicMax((unsigned long long*)F.commit_ts, (unsigned long long)s_mts);
    }
}

__global__ void fp_chains_fin(FastArgs F) {
    const u32 flags = F.counters[CNT_FLAGS];
    if (!(flags & FL_FCHAIN) || (flags & (FL_SLOW | FL_ERROR))) return;
    const u32 nq = (F.n + 15) / 16;  // 16 result bytes per lane per load
    for (u32 q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
        const uint4 v = ((const uint4*)F.fres)[q];
        const u8* fb = (const u8*)&v;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const u32 i = q * 16 + k;
            if (i < F.n && (fb[k] & FRES_CHAIN) && fb[k] != FRES_SLOW) F.fres[i] = F.fres2[i];
        }
    }
}

// With failures: mask for the rank scan (bit0 accepted, bit1 failed).
// The fix launches are enqueued whether or not the call has failures (CNT_FIX decides
// on the device), so they run small grid-stride grids: a full grid that stands down
// still costs its dispatch.
__global__ void fp_mask(FastArgs F, u8* mask) {
    if (!F.counters[CNT_FIX]) return;
    FOR_EACH_EVENT(i) mask[i] = F.fres[i] == TBGPU_CREATE_TRANSFER_OK ? 1 : 2;
}

// With failures: stored rows at their ranks (re-copied from the events, so the
// order of the writes does not matter) and the sparse replies.
__device__ __forceinline__ void fp_fix_one(const FastArgs& F, const Tables& T, u32 i, u32 rank_ok, u32 rank_bad) {
    const u32 b = fp_batch_of(F.b_start, F.nb, i);
    const u32 bs = F.b_start[b];
    const u8 r = F.fres[i];
    if (r != TBGPU_CREATE_TRANSFER_OK) {
        F.results[T.base[BASE_REPLIES] + rank_bad] = {i - bs, (u32)r};  // concatenated replies
        return;
    }
    const u32 row = (u32)(T.base[BASE_ROWS] + rank_ok);
    Transfer t = F.ev[i];
    t.timestamp = F.ev_ts ? F.ev_ts[i] : F.b_ts[b] - (F.b_start[b + 1] - bs) + (i - bs) + 1;
    T.xrows[row] = t;
    F.rows[i] = row;
    if (F.eager) T.xidx[F.gpos[i]] = xidx_slot(t.id, row);  // the claim follows its row
}

__global__ void fp_fix(FastArgs F, Tables T, const uint4* rk) {
    if (!F.counters[CNT_FIX]) return;
    FOR_EACH_EVENT(i) fp_fix_one(F, T, i, rk[i].x, rk[i].y);
}

// After an accepted attempt: advance the device cursors by its stored rows and replies.
__global__ void fp_advance(Tables T, FastArgs F) {
    if (threadIdx.x != 0) return;
    if (F.counters[CNT_FLAGS] & (FL_SLOW | FL_ERROR)) return;  // the call falls back (fp_undo)
    T.base[BASE_REPLIES] += F.counters[CNT_BAD];
    if (!F.dry) T.base[BASE_ROWS] += F.counters[CNT_OK];
}

// Per-call reset of the fast path's counters and reply counts, and a copy of
// commit_timestamp for the fallback: fp_commit raises it for every event it
// classifies ok against the pre-call state, which the sequential result may not
// (an id repeated later in the call answers `exists`).
__global__ void fp_prep(FastArgs F, BlockInline bi) {
    const u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < bi.words) bi.block[k] = bi.w[k];
    if (k == 0 && bi.words && bi.reset_replies) bi.base[BASE_REPLIES] = 0;
    if (k < CNT_TS_SAVE) F.counters[k] = 0;
    if (k == 0) *(u64*)&F.counters[CNT_TS_SAVE] = *F.commit_ts;
    if (k < F.nb) F.batch_counts[k] = 0;
}

// The simple small call's end, by fp_commit_small's last tile (one wave, F.fuse): the
// tiles' records say no event failed, none is a chain member and no repeat check is
// left (ids rising, or claimed eagerly), and either the rows extend the sorted run or
// their ids are claimed already: then fp_tail's phases reduce to counters, the run's
// bounds or the key range, the cursors and the report, done here in one round of loads
// and one of stores, and the host's wait ends without the kernel boundary and fp_tail's
// launch.  Otherwise nothing is written (fp_tail does the whole tail, as without F.fuse).
__device__ void fp_small_tail(const Tables& T, const FastArgs& F, const BlockInline& bi, const TailReport& rp) {
    const u32 lane = threadIdx.x & 63, n = F.n;
    const u32 ntiles = (n + F.tile - 1) / F.tile;
    auto ld64 = [](const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    // one round of loads: the tiles' records (every lane), and in lane 0 what the run
    // decision and the cursors need
    u32 fl = 0, nbad = 0, nok = 0;
    u64 mts = 0;
    for (u32 k = lane; k < ntiles; k += 64) {
        const u64* r = F.tile_idr + TILE_WORDS * k;
        mts = max(mts, ld64(r + 4));
        nok += (u32)ld64(r + 5);
        nbad += (u32)ld64(r + 6);
        fl |= (u32)ld64(r + 7);
    }
    u64 xr[6] = {0, 0, 0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, cts = 0;
    u128 first = 0, last = 0;
    if (lane == 0) {
        for (int k = 0; k < 6; k++) xr[k] = ld64(T.xrun + k);
        for (int k = 0; k < 4; k++) b[k] = ld64(T.base + k);
        cts = ld64(F.commit_ts);
        first = F.ev[0].id;
        last = F.ev[n - 1].id;
    }
    for (int off = 32; off > 0; off >>= 1) {
        nbad += __shfl_xor(nbad, off);
        nok += __shfl_xor(nok, off);
        fl |= __shfl_xor(fl, off);
        mts = max(mts, (u64)__shfl_xor((unsigned long long)mts, off));
    }
    // what fp_tail would decide (fp_run_one), without writing anything yet
    u32 take = 0, ok = 0;
    if (lane == 0) {
        const bool simple = !(fl & (FL_SLOW | FL_ERROR | FL_FCHAIN)) && nbad == 0 && (!(fl & FL_NONMONO) || F.eager);
        if (simple && !F.eager && n && !(fl & FL_NONMONO)) {
            const bool empty = xr[0] == xr[1];
            take = (empty || (xr[1] == b[BASE_ROWS] && first > (((u128)xr[5] << 64) | xr[4]))) ? 1u : 0u;
        }
        ok = simple && (take || F.eager) && rp.out && rp.seq_out && !F.dry ? 1u : 0u;
    }
    ok = __shfl(ok, 0);
    take = __shfl(take, 0);
    if (!ok) {
        if (lane == 0) __hip_atomic_store(&F.counters[CNT_TICKET], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;  // fp_tail ends the call
    }
    // the stores: fp_prep's (the batch block, the reply counts), the counters, the run or
    // the key range, the cursors
    if (lane < bi.words) bi.block[lane] = bi.w[lane];
    for (u32 k = lane; k < F.nb; k += 64) F.batch_counts[k] = 0;
    if (!take) {  // (eager: the claims are the index inserts) the tiles' id ranges into T.idr
        for (u32 k0 = 0; k0 < ntiles; k0 += 64) fp_fold_idr(T, F, k0, ntiles);
    }
    if (lane == 0) {
        const u32 nokeys = __hip_atomic_load(&F.counters[CNT_NOKEYS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int k = 0; k < CNT_TS_SAVE; k++) F.counters[k] = 0;
        F.counters[CNT_NOKEYS] = nokeys;
        F.counters[CNT_FLAGS] = fl;
        F.counters[CNT_OK] = nok;
        F.counters[CNT_RUN] = take;
        *(u64*)&F.counters[CNT_TS_SAVE] = cts;
        if (mts > cts) *F.commit_ts = mts;
        if (take) {
            u64* r = T.xrun;
            if (xr[0] == xr[1]) {
                r[0] = b[BASE_ROWS];
                r[2] = (u64)first;
                r[3] = (u64)(first >> 64);
            }
            r[1] = b[BASE_ROWS] + n;
            r[4] = (u64)last;
            r[5] = (u64)(last >> 64);
        }
        if ((bi.words && bi.reset_replies) || F.gate) b[BASE_REPLIES] = 0;  // (a prepared commit's starts at 0)
        b[BASE_ROWS] += nok;
        T.base[BASE_REPLIES] = b[BASE_REPLIES];
        T.base[BASE_ROWS] = b[BASE_ROWS];
    }
    for (int k = 0; k < 4; k++) b[k] = __shfl(b[k], 0);  // (lane 0's cursors, for the report)
    // the report (k_report's words: flags, accepted, run; the cursors; no replies), then
    // the sequence word once the report is visible to the host
    for (u32 k = lane; k < RPT_COUNTS + rp.nb; k += 64) {
        u32 v = 0;
        if (k == CNT_FLAGS) v = fl;
        else if (k == CNT_OK) v = nok;
        else if (k == CNT_RUN) v = take;
        else if (k >= RPT_BASE && k < RPT_COUNTS) {
            const u32 w = k - RPT_BASE;
            const u64 bw = (w >> 1) == 0 ? b[0] : (w >> 1) == 1 ? b[1] : (w >> 1) == 2 ? b[2] : b[3];
            v = (w & 1) ? (u32)(bw >> 32) : (u32)bw;
        }
        __hip_atomic_store(&rp.out[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // the report's system-scope stores (past every cache, into coherent host memory) are
    // complete before the sequence word goes out: no L2 write-back of the rows the tiles
    // stored on this XCD (a system-scope release fence would make one)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
        __hip_atomic_store(&F.counters[CNT_TAILSEQ], rp.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&F.counters[CNT_TICKET], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(rp.seq_out, rp.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Small calls (n <= FP_TAIL_MAX, e.g. one drop-in batch of 8190): everything after
// fp_commit in ONE workgroup, the launches of fp_launch_index, fp_launch_fix and
// fp_launch_advance run as phases separated by barriers.  A batch of 8190 events
// is ~2 us of work per phase, but each of those ~12 launches cost its dispatch and
// host enqueue (the single-call timeline in profiles/README.md); this keeps the
// small call at 3 launches.  Same results as the launch sequence, phase by phase.
// Counters written by atomics in this launch are read with agent-scope loads (not
// through the CU's L1) and broadcast through LDS so that every branch is uniform.
__device__ __forceinline__ u32 fp_cnt(const FastArgs& F, int k) {
    return __hip_atomic_load(&F.counters[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(FP_TAIL_THREADS) void fp_tail(Tables T, FastArgs F, BlockInline bi, TailReport rp) {
    if (F.gate && __hip_atomic_load(F.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gate_tag(F.gate_seq, GATE_GO))
        return;  // a prepared commit that did not come
    if (F.fuse && fp_cnt(F, CNT_TAILSEQ) == rp.seq) return;  // fp_commit_small's last tile ended the call
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n = F.n;
    const u32 ntiles = (n + F.tile - 1) / F.tile;
    __shared__ u32 s_flags, s_bad, s_run, s_ok, s_fix;
    __shared__ u32 s_wsum[FP_TAIL_THREADS / 64];
    if (F.small) {
        // fp_prep's work (no launch of its own before fp_commit_small): the batch block
        // into memory for the launches after this one, the reply cursor, the timestamp
        // the fallback restores; then the call's counters from the tiles' records
        if (tid < bi.words) bi.block[tid] = bi.w[tid];
        if (tid == 0 && bi.words && bi.reset_replies) bi.base[BASE_REPLIES] = 0;
        for (u32 b = tid; b < F.nb; b += FP_TAIL_THREADS) F.batch_counts[b] = 0;
        if (w == 0) {
            // the tiles' records in one round: flags, failures, accepted, latest timestamp
            u32 fl = 0, nbad = 0, nok = 0;
            u64 mts = 0;
            for (u32 k = lane; k < ntiles; k += 64) {
                mts = max(mts, F.tile_idr[TILE_WORDS * k + 4]);
                nok += (u32)F.tile_idr[TILE_WORDS * k + 5];
                nbad += (u32)F.tile_idr[TILE_WORDS * k + 6];
                fl |= (u32)F.tile_idr[TILE_WORDS * k + 7];
            }
            for (int off = 32; off > 0; off >>= 1) {
                nbad += __shfl_xor(nbad, off);
                nok += __shfl_xor(nok, off);
                fl |= __shfl_xor(fl, off);
                mts = max(mts, (u64)__shfl_xor((unsigned long long)mts, off));
            }
            if (lane == 0) {
                const u32 nokeys = F.counters[CNT_NOKEYS];
                for (int k = 0; k < CNT_TS_SAVE; k++)
                    __hip_atomic_store(&F.counters[k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&F.counters[CNT_NOKEYS], nokeys, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&F.counters[CNT_FLAGS], fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&F.counters[CNT_BAD], nbad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&F.counters[CNT_OK], nok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // the timestamp the fallback restores, then this call's (same thread: in order)
                *(u64*)&F.counters[CNT_TS_SAVE] = *F.commit_ts;
                if (mts) atomicMax((unsigned long long*)F.commit_ts, (unsigned long long)mts);
                s_flags = fl;  // the call's figures in LDS: no global re-read below
                s_bad = nbad;
                s_ok = nok;
            }
        }
        __syncthreads();
    } else {
        if (tid == 0) s_flags = fp_cnt(F, CNT_FLAGS);
        __syncthreads();
    }
    // fp_dupcheck (eager claims: fp_commit found the repeats)
    const bool dupcheck = (s_flags & FL_NONMONO) && !F.eager;
    if (dupcheck) {
        for (u32 i = tid; i < n; i += FP_TAIL_THREADS) fp_dupcheck_one(F, i);
        __syncthreads();
        if (tid == 0) s_flags = fp_cnt(F, CNT_FLAGS);
    }
    __syncthreads();
    const u32 flags = s_flags;
    // fp_chains, fp_chains_fin
    const bool chains = (flags & FL_FCHAIN) && !(flags & (FL_SLOW | FL_ERROR));
    if (chains) {
        u32 n_ok = 0, n_bad = 0;
        u64 mts = 0;
        for (u32 i = tid; i < n; i += FP_TAIL_THREADS) fp_chains_one(T, F, i, n_ok, n_bad, mts);
        for (int off = 32; off > 0; off >>= 1) {
            n_ok += __shfl_xor(n_ok, off);
            n_bad += __shfl_xor(n_bad, off);
            mts = max(mts, (u64)__shfl_xor((unsigned long long)mts, off));
        }
        if (lane == 0) {
            if (n_ok) atomicAdd(&F.counters[CNT_OK], n_ok);
            if (n_bad) atomicAdd(&F.counters[CNT_BAD], n_bad);
            if (mts) atomicMax((unsigned long long*)F.commit_ts, (unsigned long long)mts);
            if (F.small) {
                if (n_ok) atomicAdd(&s_ok, n_ok);
                if (n_bad) atomicAdd(&s_bad, n_bad);
            }
        }
        __syncthreads();
        for (u32 i = tid; i < n; i += FP_TAIL_THREADS) {
            const u8 r = F.fres[i];
            if ((r & FRES_CHAIN) && r != FRES_SLOW) F.fres[i] = F.fres2[i];
        }
    }
    __syncthreads();
    // fp_run
    if (tid == 0) {
        if (!F.small) s_bad = fp_cnt(F, CNT_BAD);  // (small: kept in LDS)
        fp_run_one(T, F, flags, s_bad);
        s_run = F.counters[CNT_RUN];
    }
    __syncthreads();
    const u32 bad = s_bad;
    // fp_index (first launch): clear the claims, the tiles' accepted count and
    // timestamp, then the ids when the call stands without failures
    if ((flags & FL_NONMONO) && !F.eager)
        for (u32 i = tid; i < n; i += FP_TAIL_THREADS) {
            const u32 g = F.gpos[i];
            if (g != NONE32) F.gtab[g] = 0;
        }
    if (w == 0 && !F.small) {  // (small: folded with the flags above)
        u64 mts = 0, nok = 0;
        for (u32 k = lane; k < ntiles; k += 64) {
            mts = max(mts, F.tile_idr[TILE_WORDS * k + 4]);
            nok += F.tile_idr[TILE_WORDS * k + 5];
        }
        for (int off = 32; off > 0; off >>= 1) {
            mts = max(mts, (u64)__shfl_xor((unsigned long long)mts, off));
            nok += (u64)__shfl_xor((unsigned long long)nok, off);
        }
        if (lane == 0) {
            if (nok) atomicAdd(&F.counters[CNT_OK], (u32)nok);
            if (mts) atomicMax((unsigned long long*)F.commit_ts, (unsigned long long)mts);
        }
    }
    const bool stands = !(flags & (FL_SLOW | FL_ERROR));
    if (stands && !F.dry && bad == 0 && !s_run) {
        if (w == 0)
            for (u32 k0 = 0; k0 < ntiles; k0 += 64) fp_fold_idr(T, F, k0, ntiles);
        const u64 row0 = T.base[BASE_ROWS];
        if (!F.eager)
            for (u32 i = tid; i < n; i += FP_TAIL_THREADS)
                if (F.fres[i] == TBGPU_CREATE_TRANSFER_OK) xidx_insert(T, fp_key(F, i), (u32)(row0 + i));
    }
    // fp_mask, scan3, fp_fix, fp_index (fixed): each thread takes a contiguous range,
    // so its ranks are the workgroup's exclusive prefix plus a running count
    if (stands && bad != 0) {
        const u32 per = (n + FP_TAIL_THREADS - 1) / FP_TAIL_THREADS;
        const u32 i0 = min(n, tid * per), i1 = min(n, i0 + per);
        u32 v = 0;  // accepted | failed << 16 (n <= FP_TAIL_MAX < 65536)
        for (u32 i = i0; i < i1; i++) v += F.fres[i] == TBGPU_CREATE_TRANSFER_OK ? 1u : 1u << 16;
        u32 inc = v;
        for (int off = 1; off < 64; off <<= 1) {
            const u32 t = __shfl_up(inc, off);
            if (lane >= (u32)off) inc += t;
        }
        if (lane == 63) s_wsum[w] = inc;
        __syncthreads();
        u32 ex = inc - v;
        for (u32 k = 0; k < w; k++) ex += s_wsum[k];
        u32 ra = ex & 0xFFFF, rf = ex >> 16;
        for (u32 i = i0; i < i1; i++) {
            if (F.fres[i] == TBGPU_CREATE_TRANSFER_OK) fp_fix_one(F, T, i, ra++, rf);
            else fp_fix_one(F, T, i, ra, rf++);
        }
        if (!F.dry) {
            if (w == 0)
                for (u32 k0 = 0; k0 < ntiles; k0 += 64) fp_fold_idr(T, F, k0, ntiles);
            if (!F.eager)
                for (u32 i = i0; i < i1; i++)
                    if (F.fres[i] == TBGPU_CREATE_TRANSFER_OK) xidx_insert(T, fp_key(F, i), F.rows[i]);
        }
    }
    __syncthreads();
    // fp_advance
    __shared__ u64 s_base[4];  // (small) the device cursors after the call, for the report
    if (tid == 0) {
        if (F.small) {
            // the cursors once, updated in registers (the report reads them from LDS)
            u64 b[4];
            for (int k = 0; k < 4; k++) b[k] = T.base[k];
            if (stands) {
                b[BASE_REPLIES] += s_bad;
                if (!F.dry) b[BASE_ROWS] += s_ok;
                T.base[BASE_REPLIES] = b[BASE_REPLIES];
                T.base[BASE_ROWS] = b[BASE_ROWS];
            }
            for (int k = 0; k < 4; k++) s_base[k] = b[k];
            s_fix = F.counters[CNT_FIX];  // (this thread's own store in fp_run_one)
        } else if (stands) {
            T.base[BASE_REPLIES] += fp_cnt(F, CNT_BAD);
            if (!F.dry) T.base[BASE_ROWS] += fp_cnt(F, CNT_OK);
        }
    }
    if (!F.small) return;
    // each batch's reply count (its failures, final after the chains; none without them)
    if (stands && bad != 0)
        for (u32 i = tid; i < n; i += FP_TAIL_THREADS)
            if (F.fres[i] != TBGPU_CREATE_TRANSFER_OK) atomicAdd(&F.batch_counts[fp_batch_of(F.b_start, F.nb, i)], 1u);
    __syncthreads();
    if (!rp.out) return;
    // k_report: the call's end stored into pinned host memory.  The counter words the host
    // reads come from LDS (flags, accepted, failed, run, fix; the rest 0), the cursors
    // too; reply counts are all 0 without failures.  Without replies to copy, wave 0 alone
    // stores the report, fences its own stores and then the sequence word: no barrier.
    const u64 total = rp.out_replies ? s_base[BASE_REPLIES] : 0;
    const bool all = total != 0 || bad != 0;
    auto word = [&](u32 k) -> u32 {
        if (k < RPT_BASE) {
            return k == CNT_FLAGS ? s_flags : k == CNT_OK ? s_ok : k == CNT_BAD ? s_bad : k == CNT_RUN ? s_run
                 : k == CNT_FIX ? s_fix : 0u;
        }
        if (k < RPT_COUNTS) return ((const u32*)s_base)[k - RPT_BASE];
        return bad ? __hip_atomic_load(&F.batch_counts[k - RPT_COUNTS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : 0u;
    };
    if (all || w == 0) {
        const u32 stride = all ? FP_TAIL_THREADS : 64;
        for (u32 k = tid; k < RPT_COUNTS + rp.nb; k += stride) rp.out[k] = word(k);
        for (u64 j = tid; j < total; j += stride) rp.out_replies[j] = rp.replies[j];
        // the call's sequence number last, once every store above is visible to the
        // host: the host polls it instead of waiting for the launch's completion signal
        __threadfence_system();
    }
    if (all) __syncthreads();
    if (tid == 0 && rp.seq_out) __hip_atomic_store(rp.seq_out, rp.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Exact inverse of fp_commit's effects, before the general path redoes the call:
// commit_timestamp back to its pre-call value, and the balance deltas (none in a
// dry run).
__global__ void fp_undo(Tables T, FastArgs F) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *F.commit_ts = *(const u64*)&F.counters[CNT_TS_SAVE];
    if (F.dry || i >= F.n) return;
    // every eager claim of the call (each took a slot that was empty before it; all go
    // together, so no other id's probe sequence runs through them): the index as before
    if (F.eager && F.gpos[i] != NONE32) {
        // a claim fp_chains withdrew is a tombstone it counted: uncount it with the slot
        if ((u32)T.xidx[F.gpos[i]] == XIDX_TOMB) atomicSub(&T.hcount[2], 1u);
        T.xidx[F.gpos[i]] = 0;
    }
    if (F.fres[i] != TBGPU_CREATE_TRANSFER_OK) return;
    const Transfer& t = F.ev[i];
    const u32 ds = acc_row(T, t.debit_account_id);
    const u32 cs = acc_row(T, t.credit_account_id);
    const u64 a = (u64)t.amount;
    if (t.flags & TF_PENDING) {
        atomic_sub_u128_small(&T.acc[ds].debits_pending, a);
        atomic_sub_u128_small(&T.acc[cs].credits_pending, a);
    } else {
        atomic_sub_u128_small(&T.acc[ds].debits_posted, a);
        atomic_sub_u128_small(&T.acc[cs].credits_posted, a);
    }
}

}  // namespace

#define GRID(n) (u32)(((n) + 255) / 256), 256, 0, stream

void fp_launch_prep(const FastArgs& F, hipStream_t stream, const BlockInline& bi) {
    fp_prep<<<GRID(std::max<u32>(std::max<u32>(F.nb, CNT_COUNT), BLOCK_INLINE_WORDS))>>>(F, bi);
    HIP_CHECK(hipGetLastError());
}

void fp_launch_commit(const Tables& T, const FastArgs& F, hipStream_t stream, const BlockInline& bi,
                      const TailReport& rp, const GateArgs& ga) {
    if (F.small) {
        fp_commit_small<<<(F.n + FP_SMALL_TILE - 1) / FP_SMALL_TILE, FP_SMALL_TILE, 0, stream>>>(T, F, bi, rp, ga);
    } else {
        fp_commit<<<(F.n + FP_THREADS - 1) / FP_THREADS, FP_THREADS, 0, stream>>>(T, F);
    }
    HIP_CHECK(hipGetLastError());
}

void fp_launch_index(const Tables& T, const FastArgs& F, hipStream_t stream) {
    const u32 sg = std::min<u32>((F.n + 255) / 256, 2048);  // grid-stride: usually stands down
    fp_dupcheck<<<std::max(sg, 1u), 256, 0, stream>>>(T, F);
    fp_chains<<<std::max(sg, 1u), 256, 0, stream>>>(T, F);   // both stand down without FL_FCHAIN
    fp_chains_fin<<<std::max(sg, 1u), 256, 0, stream>>>(F);
    fp_run<<<1, 64, 0, stream>>>(T, F);
    fp_index<<<GRID(F.n)>>>(T, F, false);
    HIP_CHECK(hipGetLastError());
}

void fp_launch_fix(const Tables& T, const FastArgs& F, u8* mask, uint4* ranks, Scan3Scratch& sc, hipStream_t stream) {
    const u32 sg = std::max<u32>(std::min<u32>((F.n + 255) / 256, 2048), 1);
    fp_mask<<<sg, 256, 0, stream>>>(F, mask);
    scan3_exclusive(mask, ranks, F.n, sc, stream, F.counters + CNT_FIX);
    fp_fix<<<sg, 256, 0, stream>>>(F, T, ranks);
    if (!F.dry) fp_index<<<sg, 256, 0, stream>>>(T, F, true);
    HIP_CHECK(hipGetLastError());
}

void fp_launch_tail(const Tables& T, const FastArgs& F, hipStream_t stream, const BlockInline& bi,
                    const TailReport& rp) {
    fp_tail<<<1, FP_TAIL_THREADS, 0, stream>>>(T, F, bi, rp);
    HIP_CHECK(hipGetLastError());
}

void fp_launch_advance(const Tables& T, const FastArgs& F, hipStream_t stream) {
    fp_advance<<<1, 64, 0, stream>>>(T, F);
    HIP_CHECK(hipGetLastError());
}

void fp_launch_undo(const Tables& T, const FastArgs& F, hipStream_t stream) {
    fp_undo<<<GRID(F.n)>>>(T, F);
    HIP_CHECK(hipGetLastError());
}

u64 fp_tiles(u64 n) { return (n + FP_THREADS - 1) / FP_THREADS; }
u32 fp_tile_events() { return FP_THREADS; }
