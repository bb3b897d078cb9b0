// engine.h — host/device interfaces between the engine's translation units.
#pragma once
#include "common.h"

// Account id index entry: 32 bytes, so the index of 1M accounts (at load 0.5)
// is 64 MB and stays resident in the 256 MB Infinity Cache while the 128-byte
// rows live densely elsewhere.  ledger and flags are immutable after
// create_account, so the state-independent checks of create_transfer
// (src/state_machine.zig:1273-1281) never touch the row.
struct alignas(32) AccIdx {
    u64 id_lo, id_hi;
    u32 row1;    // dense row + 1; 0 = empty slot
    u32 ledger;
    u16 flags;
    u16 code;
    u32 pad;
};
static_assert(sizeof(AccIdx) == 32, "AccIdx layout");

// HBM-resident state owned by a ctx (replaces the grooves' object caches and
// LSM trees for the hot path: src/lsm/groove.zig:623-1006).
struct Tables {
    Account* acc;      // dense account rows, index = account row (creation order)
    AccIdx* aidx;      // open-addressed account id -> row
    u64 aidx_mask;     // capacity - 1 (power of two)
    Transfer* xrows;   // stored transfers, append-only, commit order
    u8* xful;          // posted groove by pending row: 0 none, 1 posted, 2 voided
    u64* xidx;         // transfer id -> slot: row + 1 (low word; 0 empty) | key fingerprint << 32
    u64 xidx_mask;
    History* hrows;    // account-history groove rows, append-only
    u64* commit_ts;    // device copy of StateMachine.commit_timestamp (atomicMax)
    // Componentwise range of the ids in xidx: [0] max lo, [1] max hi, [2] min lo,
    // [3] min hi.  An id outside it is absent without a probe (the LSM key-range
    // short-circuit of src/lsm/tree.zig:289-300, why sequential ids are cheap).
    u64* idr;
    // Bit 0 set once any balance high word reaches 2^62: until then a call of < 2^32
    // events with amounts < 2^64 cannot overflow a u128 sum (fast.hip).  Bit 1 once any
    // balance reaches 2^61 (the general path's 64-bit headroom passes, FL_WIDE64).
    u32* big;
    // Account index occupancy: [0] hash-index entries reserved so far, [1] nonzero once
    // an insert was refused because `hash_limit` (half the slots: load <= 0.5, so every
    // probe ends at an empty slot) was reached.  Ledger shards insert other shards'
    // accounts here too, which the owned-row capacity check does not cover.
    u32* hcount;
    u64 hash_limit;
    // Direct-mapped account directory.  Ids (b << 32) | k with b < dense_blocks and
    // 1 <= k <= dense_span have entry b * dense_span + k - 1, describing the account
    // as (row + 1) | (flags & 0xE) << 28 | ledger << 32, 0 = no such account.  Every
    // account with such an id has its entry, so the directory is exact for them;
    // other ids use `aidx`.  By default one block: ids 1..accounts_max, the reference
    // benchmark's numbering (src/tigerbeetle/benchmark_load.zig:134-138, :223); with
    // tbgpu_options.dense_block_span, ledger-major ids (ledger << 32 | k).  One
    // 8-byte read instead of a 32-byte probe of a twice-as-large hash index.
    u64* dense;
    u64 dense_n;       // entries (dense_blocks * dense_span)
    u64 dense_span, dense_blocks;
    // Device-side append cursors, so that consecutive chunks and calls need no host
    // round trip: [0] stored transfer rows, [1] account-history rows, [2] replies
    // written so far in the current call (the streaming reply offset).
    u64* base;
    u64 xrow_cap, hist_cap;
    // The sorted run of the transfer-id index: rows [xrun[0], xrun[1]) of xrows were
    // committed by calls whose ids rose strictly, each above the last id of the run,
    // and are not in `xidx`: their ids are sorted by row, so a lookup is a binary
    // search over the rows (an LSM table, src/lsm/tree.zig; the benchmark's
    // sequential ids never touch the hash index).  xrun[2..3] the first id (lo, hi),
    // xrun[4..5] the last; empty when xrun[0] == xrun[1].
    u64* xrun;
    // Ledger shard (tbgpu_options.shard_world >= 2): rows are stored only for accounts
    // of the ledgers this ctx owns (ledger % shard_world == shard_rank); every other
    // account has a directory entry whose row is ROW_FOREIGN (its id and ledger: what
    // create_transfer's checks of :1273-1281 read of an account on another ledger).
    u32 shard_world, shard_rank;
};
enum { BASE_ROWS = 0, BASE_HIST = 1, BASE_REPLIES = 2 };

// A ledger shard's record of another shard's account (checkpoint image, tbgpu_open).
struct ForeignAccount {
    u64 id_lo, id_hi;
    u32 ledger, pad;
};
static_assert(sizeof(ForeignAccount) == 24, "ForeignAccount layout");

// The row of an account another shard stores (directory entry only).
constexpr u32 ROW_FOREIGN = 0xFFFFFFFEu;
constexpr u32 DENSE_ROW1_MASK = 0x1FFFFFFFu;   // row + 1 in the directory entry's low 29 bits
constexpr u32 DENSE_FOREIGN1 = DENSE_ROW1_MASK;  // ... all ones: ROW_FOREIGN
__device__ __forceinline__ bool ledger_owned(const Tables& T, u32 ledger) {
    return T.shard_world < 2 || ledger % T.shard_world == T.shard_rank;
}

__device__ __forceinline__ bool dense_has(const Tables& T, u128 id) {
    const u64 lo = (u64)id;
    return (u64)(id >> 64) == 0 && (lo >> 32) < T.dense_blocks && (u64)(u32)lo - 1 < T.dense_span;
}
// the entry of an id for which dense_has holds
__device__ __forceinline__ u64 dense_slot(const Tables& T, u128 id) {
    const u64 lo = (u64)id;
    return (lo >> 32) * T.dense_span + (u32)lo - 1;
}
__device__ __forceinline__ u64 dense_entry(u32 row, u32 ledger, u16 flags) {
    const u64 r1 = row == ROW_FOREIGN ? DENSE_FOREIGN1 : row + 1;
    return r1 | ((u64)(flags & 0xEu) << 28) | ((u64)ledger << 32);
}
__device__ __forceinline__ u32 dense_row(u64 e) {  // of a nonzero entry
    const u32 r1 = (u32)e & DENSE_ROW1_MASK;
    return r1 == DENSE_FOREIGN1 ? ROW_FOREIGN : r1 - 1;
}

// Account lookup: the direct-mapped directory for ids 1..dense_n (8 bytes), the
// hash index otherwise (it holds only ids outside the directory).  Returns the row
// (NONE32 when absent, ROW_FOREIGN for an account another ledger shard stores) with
// its ledger and flags (limit / history bits), which are immutable after
// create_account.
__device__ __forceinline__ u32 acc_find(const Tables& T, u128 id, u32* ledger, u16* flags);

__device__ __forceinline__ bool xidx_maybe_present(const Tables& T, u128 id) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    return lo <= T.idr[0] && hi <= T.idr[1] && lo >= T.idr[2] && hi >= T.idr[3];
}

// One double-buffered fixed-point state (see transfers.hip).
struct EvalState {
    u8* res;     // own evaluation result (0 = ok)
    u8* ok;      // 1 = eval-ok (final-ok, chain persisted, is derived: final_ok below)
    u32* pref;   // resolved pending transfer reference
    u32* cfail;  // per chain start: first failing member (NONE32 = none)
    u128* amt;   // effective amount (balancing clamp / post amount)
    u128* pamt;  // pending transfer amount (post/void)
};

// Pass gate of the fixed point: the kernels of pass p run while the previous
// pass changed something (its change count != 0; forced to 1 for the first pass) and no
// side key has moved (a post/void resolved to another pending: the host re-sorts).
// Passes are enqueued in groups without host round trips; the kernels of the
// passes after convergence return at once.
struct PassGate {
    const u32* chg;     // the previous pass's change count (a ring word)
    const u32* halt;    // [0] a post/void resolved outside its sides (rebuild them), [1] the fused
                        // balance scan met an account segment longer than its window: nonzero halts
    u32 p;              // this pass's number
    u32 full;           // evaluate and rescan everything (no dirty tracking: the three-launch scan)
};

// Dirty tracking of the fixed point's passes (transfers.hip, balances.hip bs_fused).
// A pass re-evaluates only the events whose inputs moved in the previous pass, and the
// fused scan redoes only the windows whose side records moved.  Stamps hold the pass
// number for which something is due (no clearing between passes); the event, chain and
// slot stamps are kept per pass parity, so that marks for pass q + 1 never overwrite
// the marks pass q is reading.  An event evaluated at pass q reads state q - 1 and
// writes the other state buffer; a skipped event must hold the same outcome in both,
// so an event that changed at pass q is evaluated again at q + 1.
struct Dirty {
    u32* ev;          // [2][n] the pass at which the event is evaluated
    u32* chain;       // [2][n] by chain start: the pass at which every member is (a chain's first
                      // failure is recomputed from all its members)
    u32* slot;        // [2][g] by group-table slot: the pass at which the complex events of that id
                      // (its repeats, the post/voids naming it as pending) are
    u32* win;         // [windows] the pass at which the fused scan redoes the window
    const u32* all;   // the pass at which everything is (0: a chunk's first; after a side rebuild)
    u32 n, g;         // strides of ev / chain and of slot
};
__device__ __forceinline__ bool gate_open(const PassGate& g) { return *g.chg != 0 && g.halt[0] == 0 && g.halt[1] == 0; }

// final-ok: eval-ok and the event's chain persisted (execute's scope_close(.persist),
// src/state_machine.zig:1074-1082), and not doomed by a break on another shard.
__device__ __forceinline__ bool chain_persisted(const u32* cs, const u32* ce, const u32* cfail, const u8* ctl, u32 j) {
    const u32 s = cs[j], e = ce[j];
    if (ctl && (ctl[e] & TBGPU_CTL_DOOM)) return false;
    return s == e || cfail[s] == NONE32;
}
__device__ __forceinline__ bool final_ok(const u32* cs, const u32* ce, const u32* cfail, const u8* ctl, const u8* ok,
                                         u32 j) {
    return (ok[j] & 1) && chain_persisted(cs, ce, cfail, ctl, j);
}

// The account sides of a chunk's events, sorted by account row and, within an
// account, by event (a stable sort of the event-ordered sides).  A transfer has a
// debit and a credit side; a post/void has one pair per candidate pending (the
// pending it resolved to last pass, a committed transfer with that id, the first
// earlier events with that id: at most SIDE_CANDS), of which only the pair of the
// pending it resolves to carries its effect, so a post/void whose resolution moves
// needs no re-sort.  `sq_*` are in sorted order: the scan reads them contiguously.
constexpr u32 SIDE_CANDS = 3;
struct Sides {
    u32 m;            // sides of the chunk
    u32* soff;        // [n + 1] first side (unsorted id) of each event
    u32* sev;         // [m] unsorted: event | side << 31 (0 debit, 1 credit) | SQ_SENS | SQ_FIRST
    u32* scs;         // [m] unsorted: the side's sq_cs word (written by tr_side_build)
    u32* scand;       // [m] unsorted: the candidate pending of a post/void pair (pref encoding), else NONE32
    u32* spos;        // [m] sorted position of unsorted side s
    const u32* skey_s;  // [m] sorted keys (account row; >= invalid: no account)
    u32* sq_ev;       // [m] sorted: event | side << 31 | SQ_SENS
    u32* sq_cs;       // [m] sorted: chain start | standalone << 31 | doomed << 30
    u8* sq_ok;        // [m] sorted, per pass: the side's effect is evaluated-ok
    u128* sq_dpend;   // [m] sorted, per pass: its delta on the *_pending balance
    u128* sq_dpost;   // [m] sorted, per pass: its delta on the *_posted balance
    // The compact form of the deltas (a chunk in 64-bit headroom form, FL_WIDE64 clear):
    // [2m] (pending, posted) per side as 64-bit two's complement, in sq_dpend's memory;
    // null when the chunk keeps the u128 form.  One form per chunk (the host decides it
    // before tr_side_rec writes the first records).
    u64* sq_d64;
    u32* over;        // the flag word FL_H64_OVER goes to (a compact delta that does not fit)
    u32* tstart;      // [m / tile + 1] first account start in each fused-scan window (NONE32: none)
    uint2* epos;      // [n] sorted positions of each event's first side pair (debit, credit)
    u32 tile;         // the fused scan's window (sides)
    u32 inert;        // the key of sides that touch no account (each stands alone)
};
constexpr u32 SQ_STANDALONE = 1u << 31, SQ_DOOM = 1u << 30, SQ_CS = (1u << 30) - 1;
// sq_ev / sev: bit 30 set when the side's balance can decide its event's outcome in a
// headroom pass -- a debit side of an account with debits_must_not_exceed_credits or of
// a balancing_debit transfer, a credit side likewise (eval_balances_narrow reads nothing
// else of a balance; post/void and static failures read none).  The headroom scan marks
// an event due only through such a side.  Bit 29: the side belongs to its event's first
// pair (its sorted position goes to epos).  Events fit 29 bits (events_per_call_max).
constexpr u32 SQ_SENS = 1u << 30, SQ_FIRST = 1u << 29, SQ_EV = (1u << 29) - 1;

struct SideScanArgs {
    const u32* skey;  // sorted side keys (account row; >= invalid for inert)
    const u32* sq_ev;
    const u32* sq_cs;
    const u8* sq_ok;
    const u128* sq_dpend;
    const u128* sq_dpost;
    const u64* sq_d64;  // the compact form (Sides::sq_d64), or null
    const u32* cfail; // per-chain first failure of the state scanned
    u32* cfail_clear; // the next state's cfail, reset by the scan (NONE32), or null
    u32 n;            // events (cfail_clear length)
    PassGate gate;
    u32 probe;        // timing probes only (TBGPU_EVAL_PROBE): 1 no chain words, 2 no account rows, 4 no block scan
    const u32* epi;   // bs_final's gate (TrArgs::epi), or null; 2: use cfail_alt
    const u32* cfail_alt;
    // dirty tracking (bs_fused): windows to redo, balances that moved mark their events;
    // the complex list's events whose id / pending groups moved are marked here too
    Dirty dt;
    const u32* lst_complex;
    u32 n_complex;
    const u32 *gslot, *pslot, *cs, *ce;
    // headroom passes (side_scan_fused_narrow): the side's one balance figure its
    // evaluation reads, or null (the Bal4 passes)
    u128* bh;
    u64* bh64;        // the 64-bit headroom passes' figure (side_scan_fused_h64), or null
    u32* over;        // the flag word FL_H64_OVER goes to (a figure outside +-2^63)
    u32 all_sides;    // headroom passes: a moved balance marks its event whatever SQ_SENS says
                      // (TBGPU_NO_SENS=1, A/B timing)
};

// A 64-bit two's complement value as the u128 it stands for.
__device__ __forceinline__ u128 sext64(u64 v) { return (u128)(__int128)(long long)v; }
__device__ __forceinline__ bool fits64(u128 v) { return sext64((u64)v) == v; }

// Sorted side q's deltas (pending, posted), from whichever form the chunk keeps.
__device__ __forceinline__ void side_deltas(const SideScanArgs& A, u64 q, u128& dpe, u128& dpo) {
    if (A.sq_d64) {
        const ulonglong2 v = ((const ulonglong2*)A.sq_d64)[q];
        dpe = sext64(v.x);
        dpo = sext64(v.y);
    } else {
        dpe = A.sq_dpend[q];
        dpo = A.sq_dpost[q];
    }
}

// final-ok of a sorted side: evaluated-ok and its chain persisted
__device__ __forceinline__ bool side_final(const SideScanArgs& A, u64 q) {
    if (!(A.sq_ok[q] & 1)) return false;
    const u32 c = A.sq_cs[q];
    if (c & SQ_DOOM) return false;
    return (c & SQ_STANDALONE) || A.cfail[c & SQ_CS] == NONE32;
}

u64 side_scan_tile_bytes(u64 capacity);
void side_scan(const SideScanArgs& A, u64 m, u32 invalid, bool has_chains, void* tile_scratch, const Account* acc,
               Bal4* bb, hipStream_t stream);
// One-launch form (balances.hip bs_fused): raises *long_flag (= pass + 1) and leaves
// the pass incomplete when an account segment is longer than its window.
void side_scan_fused(const SideScanArgs& A, u64 m, u32 invalid, const u32* tstart, u32* long_flag,
                     const Account* acc, Bal4* bb, hipStream_t stream);
u32 side_scan_fused_tile();
// The passes' scan in headroom form (balances.hip): per side, the debit account's
// credits_posted - debits_pending - debits_posted (a debit side) or the credit account's
// debits_posted - credits_pending - credits_posted (a credit side), modulo 2^128, in A.bh.
void side_scan_fused_narrow(const SideScanArgs& A, u64 m, u32 invalid, const u32* tstart, u32* long_flag,
                            const Account* acc, hipStream_t stream);
// The same in 64-bit form (FL_WIDE64 clear: every headroom of the chunk lies within
// +-2^63, so it and every delta are exact as 64-bit two's complement): A.bh64 per side,
// the deltas from A.sq_d64 -- 8 + 16 bytes per side where the u128 form moves 16 + 32.
void side_scan_fused_h64(const SideScanArgs& A, u64 m, u32 invalid, const u32* tstart, u32* long_flag,
                         const Account* acc, hipStream_t stream);
void side_final_balances(const SideScanArgs& A, u64 m, u32 invalid, const Bal4* bb, Account* acc, u32* big,
                         hipStream_t stream);

// FL_* bits raised on a flags word the whole grid shares: the atomic only when a bit
// is missing.  Same-address atomics serialise at L2; one per workgroup of a large grid
// whose workgroups all raise the same bits cost ~9 ns each (a 10k-account check: 11 us).
__device__ __forceinline__ void raise_flags(u32* w, u32 fl) {
#ifdef TBGPU_PLAIN_RAISE  // (timing variant: one atomic per caller)
    if (fl) atomicOr(w, fl);
#else
    if (fl && (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & fl) != fl) atomicOr(w, fl);
#endif
}

// Device probes shared by the kernels.  acc_probe returns the account ROW.
__device__ __forceinline__ u32 acc_probe(const AccIdx* __restrict__ aidx, u64 mask, u128 id) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    u64 h = hash128(lo, hi) & mask;
    for (;;) {
        const AccIdx& e = aidx[h];
        if (e.row1 == 0) return NONE32;
        if (e.id_lo == lo && e.id_hi == hi) return e.row1 - 1;
        h = (h + 1) & mask;
    }
}

// A directory entry decoded (acc_find's direct-mapped case).
__device__ __forceinline__ u32 acc_from_dense(u64 e, u32* ledger, u16* flags) {
    if (e == 0) return NONE32;
    *ledger = (u32)(e >> 32);
    *flags = (u16)((e >> 28) & 0xE);
    return dense_row(e);
}

__device__ __forceinline__ u32 acc_find(const Tables& T, u128 id, u32* ledger, u16* flags) {
    if (dense_has(T, id)) return acc_from_dense(T.dense[dense_slot(T, id)], ledger, flags);
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    u64 h = hash128(lo, hi) & T.aidx_mask;
    for (;;) {
        const AccIdx& e = T.aidx[h];
        if (e.row1 == 0) return NONE32;
        if (e.id_lo == lo && e.id_hi == hi) {
            *ledger = e.ledger;
            *flags = e.flags;
            return e.row1 - 1;
        }
        h = (h + 1) & T.aidx_mask;
    }
}

// The row of an account (NONE32 absent, ROW_FOREIGN on another shard).
__device__ __forceinline__ u32 acc_row(const Tables& T, u128 id) {
    u32 led;
    u16 fl;
    return acc_find(T, id, &led, &fl);
}

// Insert of a new account's directory entry: the direct-mapped entry for ids it
// covers, a hash-index slot (claimed by CAS on its row word) for the others.  `row`
// may be ROW_FOREIGN (a ledger shard's entry for another shard's account).
// Returns false (inserting nothing, T.hcount[1] raised) when the hash index is at
// its load limit: the caller reports FL_CAPACITY and the host aborts the call.
__device__ __forceinline__ bool acc_insert(const Tables& T, u128 id, u32 row, u32 ledger, u16 flags, u16 code) {
    if (dense_has(T, id)) {
        T.dense[dense_slot(T, id)] = dense_entry(row, ledger, flags);
        return true;
    }
    {  // reserve an entry: one atomic per wave for the lanes inserting here
        const u64 act = __ballot(1);
        const u32 lane = threadIdx.x & 63, lead = (u32)__ffsll((unsigned long long)act) - 1;
        u32 base = 0;
        if (lane == lead) base = atomicAdd(&T.hcount[0], (u32)__popcll(act));
        base = __shfl(base, lead);
        if ((u64)base + __popcll(act & ((1ull << lane) - 1)) >= T.hash_limit) {
            atomicOr(&T.hcount[1], 1u);
            return false;
        }
    }
    u64 h = hash128(id) & T.aidx_mask;
    while (atomicCAS(&T.aidx[h].row1, 0u, row + 1) != 0) h = (h + 1) & T.aidx_mask;
    AccIdx& e = T.aidx[h];
    e.id_lo = (u64)id;
    e.id_hi = (u64)(id >> 64);
    e.ledger = ledger;
    e.flags = flags;
    e.code = code;
    return true;
}

// Transfer-id index hash: runs of 16 consecutive ids share one 64-byte line of
// slots in id order (the benchmark's sequential ids insert with whole-line
// writes); the run itself is placed by a full 128-bit mix, so random ids spread
// as with any hash.  Probing steps a whole line (XIDX_STEP), keeping each id's
// offset, so a run that meets an occupied line moves on together instead of
// walking through the other run slot by slot.  The mask is >= 16 (pow2_at_least).
constexpr u64 XIDX_STEP = 16;
__device__ __forceinline__ u64 xidx_hash(u128 id) {
    const u64 lo = (u64)id, hi = (u64)(id >> 64);
    return (hash128(lo >> 4, hi) << 4) | (lo & 15);
}

__device__ __forceinline__ bool xrun_maybe(const Tables& T, u128 id) {
    const u64* r = T.xrun;
    if (r[0] == r[1]) return false;
    return id >= (((u128)r[3] << 64) | r[2]) && id <= (((u128)r[5] << 64) | r[4]);
}

__device__ __forceinline__ double u128_to_double(u128 x) {
    return (double)(u64)(x >> 64) * 18446744073709551616.0 + (double)(u64)x;
}

// the row of `id` in the sorted run, or NONE32.  Interpolation search between rows of
// known ids (the run's ids rise, and in practice nearly evenly: the benchmark's are
// consecutive with the failed ones missing), then bisection after a few steps, so an
// uneven run costs at most a few probes more than a binary search.  A binary search
// over 2M rows read ~20 random rows per lookup (tr_classify: 520 B per event).
__device__ __forceinline__ u32 xrun_find(const Tables& T, u128 id) {
    const u64* r = T.xrun;
    if (r[0] == r[1]) return NONE32;
    u64 a = r[0], b = r[1] - 1;  // rows with known ids ka, kb; ka <= id <= kb holds
    u128 ka = ((u128)r[3] << 64) | r[2], kb = ((u128)r[5] << 64) | r[4];
    if (id < ka || id > kb) return NONE32;
    for (int it = 0;; it++) {
        if (id == ka) return (u32)a;
        if (id == kb) return (u32)b;
        if (b - a <= 1) return NONE32;
        u64 mid;
        if (it < 4) {
            const double f = u128_to_double(id - ka) / u128_to_double(kb - ka);
            mid = a + (u64)(f * (double)(b - a) + 0.5);
            mid = mid <= a ? a + 1 : (mid >= b ? b - 1 : mid);
        } else {
            mid = a + (b - a) / 2;
        }
        const u128 k = T.xrows[mid].id;
        if (k == id) return (u32)mid;
        if (k < id) { a = mid; ka = k; } else { b = mid; kb = k; }
    }
}

// A slot whose claim was withdrawn (fast.hip's eager claims: a chain of the call broke,
// or its event failed a later check): probes walk past it, inserts never reuse it.
constexpr u32 XIDX_TOMB = 0xFFFFFFFFu;
// A slot is 8 bytes: row + 1 in the low word (0: empty), in the high word 32 bits of the
// id's hash independent of the slot's own: a probe reads a row (its 128 bytes, for the
// key) only when the fingerprint matches, so colliding ids of random order cost one slot
// read each instead of a slot and a row.
__device__ __forceinline__ u32 xidx_fp(u128 id) {
    return (u32)(mix64((u64)(id >> 64) * 0x9E3779B97F4A7C15ull ^ (u64)id) >> 32);
}
__device__ __forceinline__ u64 xidx_slot(u128 id, u32 row) { return ((u64)xidx_fp(id) << 32) | (row + 1); }
__device__ __forceinline__ u32 xidx_r1(u64 e) { return (u32)e; }

__device__ __forceinline__ u32 xidx_probe(const Tables& T, u128 id) {
    if (xidx_maybe_present(T, id)) {  // else outside the hashed ids' key range
        const u32 fp = xidx_fp(id);
        u64 h = xidx_hash(id) & T.xidx_mask;
        for (;;) {
            const u64 e = T.xidx[h];
            const u32 r1 = xidx_r1(e);
            if (r1 == 0) break;
            if (r1 != XIDX_TOMB && (u32)(e >> 32) == fp && T.xrows[r1 - 1].id == id) return r1 - 1;
            h = (h + XIDX_STEP) & T.xidx_mask;
        }
    }
    return xrun_maybe(T, id) ? xrun_find(T, id) : NONE32;
}

// Inserts never compare keys: a call inserts ids that are absent and distinct.
__device__ __forceinline__ void xidx_insert(const Tables& T, u128 id, u32 row) {
    u64 h = xidx_hash(id) & T.xidx_mask;
    const u64 v = xidx_slot(id, row);
    while (atomicCAS((unsigned long long*)&T.xidx[h], 0ull, (unsigned long long)v) != 0)
        h = (h + XIDX_STEP) & T.xidx_mask;
}

// Counter words (device u32[16]) used for host decisions.
enum {
    CNT_FLAGS = 0,      // FL_* bits
    CNT_CHANGES = 1,    // fixed-point: events whose state changed this pass
    CNT_KEYS = 2,       // side keys changed since the last sort
    CNT_OK = 3,         // fast path: accepted events
    CNT_BAD = 4,        // fast path: events with a result other than ok
    CNT_RESORT = 5,     // general path: pass + 1 whose evaluation resolved a post/void outside its sides
    CNT_LONG = 6,       // general path: pass + 1 whose fused scan met a segment longer than its window
    CNT_RUN = 7,        // fast path: this call's rows extend the sorted run (fp_run), not the hash index
    CNT_NOKEYS = 10,    // fast path: fp_commit wrote no id keys (the run will likely take the rows)
    CNT_FIX = 11,       // fast path: the call stands with failures: fp_fix re-places rows, writes replies (fp_run)
    CNT_GCUR = 8,       // general path: id-group ranges reserved so far
    CNT_PCUR = 9,       // general path: pending-group ranges reserved so far
    CNT_TS_SAVE = 12,   // fast path: commit_timestamp before the call (u64 in words 12-13)
    CNT_TICKET = 14,    // fast path (small call): fp_commit_small's finished tiles (the last one resets it)
    CNT_TAILSEQ = 15,   // fast path (small call): the sequence number whose end fp_commit_small's last
                        // tile stored itself (fp_tail then has nothing to do)
    CNT_DBG = 16,       // diagnostics (words 16-21): changed events by kind, summed over a call's passes
    CNT_NSIMPLE = 22,   // general path: events on the per-pass simple list (tr_lists)
    CNT_NCOMPLEX = 23,  // general path: events on the per-pass complex list
    CNT_ALL = 24,       // general path: the pass at which every event is evaluated (Dirty::all)
    CNT_STICKY = 25,    // FL_ERROR / FL_FOREIGN raised by a chunk's apply kernels: no chunk's reset
                        // clears it (the host reads a pass group's counters before its apply
                        // kernels run, and this word with the call's end)
    CNT_COUNT = 26,
};
// A call's report in host memory (k_report, or fp_tail's last phase): counters, then the
// device cursors, then the reply count of each batch (words).
constexpr u32 RPT_BASE = CNT_COUNT, RPT_COUNTS = CNT_COUNT + 8;

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
    FL_FCHAIN = 1u << 11,     // fast path: linked chains, resolved by fp_chains
    FL_CAPACITY = 1u << 12,   // create_accounts: accounts_max reached (ac_apply wrote nothing past it)
    FL_WIDE = 1u << 14,       // general path: an amount >= 2^64 or a balance near 2^128 (no headroom passes)
    FL_FOREIGN = 1u << 13,    // ledger shard: a transfer on a ledger another shard owns reached its balances
    FL_AC_HASHED = 1u << 15,  // create_accounts' clean call: some id is outside the direct-mapped directory
    FL_WIDE64 = 1u << 16,     // general path: an amount >= 2^40 or a balance >= 2^61 (no 64-bit headroom passes)
    FL_H64_OVER = 1u << 17,   // general path: a headroom or delta of a 64-bit-form chunk left +-2^63 (redo it in u128)
};

// Sorted side q's deltas written in the chunk's form (SideScanArgs side_deltas reads them).
// `check`: whether a delta that does not fit raises FL_H64_OVER -- every evaluation's
// record (the headroom passes' amounts fit while their figures do; the walk reads full
// balances).  The initial state's records are not checked: a balancing transfer of
// amount 0 starts at maxInt(u64), which every 64-bit-form pass 0 replaces (its amount is
// clamped to a headroom within +-2^63) and rewrites.
__device__ __forceinline__ void side_deltas_put(const Sides& sd, u64 q, u128 dpe, u128 dpo, bool check = true) {
    if (sd.sq_d64) {
        if (check && (!fits64(dpe) || !fits64(dpo))) atomicOr(sd.over, (u32)FL_H64_OVER);
        ((ulonglong2*)sd.sq_d64)[q] = ulonglong2{(unsigned long long)(u64)dpe, (unsigned long long)(u64)dpo};
    } else {
        sd.sq_dpend[q] = dpe;
        sd.sq_dpost[q] = dpo;
    }
}
