// engine.h — host/device interfaces between the engine's translation units.
#pragma once
#include "common.h"

// HBM-resident state owned by a ctx (replaces the grooves' object caches and
// LSM trees for the hot path: src/lsm/groove.zig:623-1006).
struct Tables {
    Account* acc;      // open-addressed by id; empty slot <=> timestamp == 0
    u64 acc_mask;      // capacity - 1 (power of two)
    Transfer* xrows;   // stored transfers, append-only, commit order
    u8* xful;          // posted groove by pending row: 0 none, 1 posted, 2 voided
    IdSlot* xidx;      // transfer id -> row index
    u64 xidx_mask;
    History* hrows;    // account-history groove rows, append-only
    u64* commit_ts;    // device copy of StateMachine.commit_timestamp (atomicMax)
    // Componentwise range of the ids in xidx: [0] max lo, [1] max hi, [2] min lo,
    // [3] min hi.  An id outside it is absent without a probe (the LSM key-range
    // short-circuit of src/lsm/tree.zig:289-300, why sequential ids are cheap).
    u64* idr;
    // Set once any balance high word reaches 2^62: until then a call of < 2^32
    // events with amounts < 2^64 cannot overflow a u128 sum (fast.hip).
    u32* big;
};

__device__ __forceinline__ bool xidx_maybe_present(const Tables& T, u128 id) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    return lo <= T.idr[0] && hi <= T.idr[1] && lo >= T.idr[2] && hi >= T.idr[3];
}

__device__ __forceinline__ void xidx_range_add(const Tables& T, u128 id) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    atomicMax((unsigned long long*)&T.idr[0], (unsigned long long)lo);
    atomicMax((unsigned long long*)&T.idr[1], (unsigned long long)hi);
    atomicMin((unsigned long long*)&T.idr[2], (unsigned long long)lo);
    atomicMin((unsigned long long*)&T.idr[3], (unsigned long long)hi);
}

// One double-buffered fixed-point state (see transfers.hip).
struct EvalState {
    u8* res;     // own evaluation result (0 = ok)
    u8* ok;      // bit0 eval-ok, bit1 final-ok (chain persisted)
    u32* pref;   // resolved pending transfer reference
    u32* cfail;  // per chain start: first failing member (NONE32 = none)
    u128* amt;   // effective amount (balancing clamp / post amount)
    u128* pamt;  // pending transfer amount (post/void)
    u128* dpend; // side delta on the *_pending balance (two's complement for void/post)
    u128* dpost; // side delta on the *_posted balance
};

struct SideScanArgs {
    const u32* skey;  // sorted side keys (account slot; >= invalid for inert)
    const u32* sval;  // sorted side ids (2*event + 0 debit / 1 credit)
    const u32* cs;    // chain start per event
    const u8* ok;
    const u128* dpend;
    const u128* dpost;
};

u64 side_scan_tile_bytes(u64 capacity);
void side_scan(const SideScanArgs& A, u64 m, u32 invalid, bool has_chains, void* tile_scratch, const Account* acc,
               Bal4* bb, hipStream_t stream);
void side_final_balances(const SideScanArgs& A, u64 m, u32 invalid, const Bal4* bb, Account* acc, u32* big,
                         hipStream_t stream);

// Device probes shared by the kernels.
__device__ __forceinline__ u32 acc_probe(const Account* __restrict__ acc, u64 mask, u128 id) {
    u64 h = hash128(id) & mask;
    for (;;) {
        const Account& a = acc[h];
        if (a.timestamp == 0) return NONE32;
        if (a.id == id) return (u32)h;
        h = (h + 1) & mask;
    }
}

__device__ __forceinline__ u32 xidx_probe(const IdSlot* __restrict__ x, u64 mask, u128 id) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    u64 h = hash128(lo, hi) & mask;
    for (;;) {
        const IdSlot& s = x[h];
        if (s.ref == 0) return NONE32;
        if (s.key_lo == lo && s.key_hi == hi) return (u32)(s.ref - 1);
        h = (h + 1) & mask;
    }
}

__device__ __forceinline__ void xidx_insert(IdSlot* __restrict__ x, u64 mask, u128 id, u32 row) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    u64 h = hash128(lo, hi) & mask;
    for (;;) {
        unsigned long long prev = atomicCAS((unsigned long long*)&x[h].ref, 0ull, (unsigned long long)row + 1);
        if (prev == 0) {
            x[h].key_lo = lo;
            x[h].key_hi = hi;
            return;
        }
        h = (h + 1) & mask;
    }
}

// Counter words (device u32[16]) used for host decisions.
enum {
    CNT_FLAGS = 0,      // FL_* bits
    CNT_CHANGES = 1,    // fixed-point: events whose state changed this pass
    CNT_KEYS = 2,       // side keys changed since the last sort
    CNT_OK = 3,         // fast path: accepted events
    CNT_COUNT = 16,
};
enum {
    FL_CHAINS = 1u << 0,      // some event is in a linked chain
    FL_POSTVOID = 1u << 1,    // some post/void passed static validation
    FL_BALANCING = 1u << 2,   // balancing_debit / balancing_credit present
    FL_LIMITS = 1u << 3,      // an account with *_must_not_exceed_* is touched
    FL_MULTI_ID = 1u << 4,    // an id repeats among dynamically-evaluated events
    FL_MULTI_PEND = 1u << 5,  // two post/voids name the same pending id
    FL_PENDING = 1u << 6,     // pending transfers present
    FL_HISTORY = 1u << 7,     // an account with flags.history is touched
    FL_SLOW = 1u << 8,        // fast path: some event needs the fixed point
    FL_ERROR = 1u << 9,       // device-side protocol error (bounded spin expired)
    FL_NONMONO = 1u << 10,    // fast path: ids of the call are not strictly increasing
};
