// transfers.hip — create_transfers as a batch-parallel fixed point.
//
// Reference semantics: `execute` (src/state_machine.zig:1002-1088) runs the
// events of a batch one at a time; `create_transfer` (:1239-1368) and
// `post_or_void_pending_transfer` (:1391-1498) read balances, ids and pending
// transfers written by earlier events.  Here every event is evaluated at once,
// against the state its predecessors *would* have produced under the previous
// pass's outcomes (a Jacobi sweep over the event sequence):
//
//   pass k:  sides sorted by (account, index) -> segmented balance scan ->
//            evaluate every event against its predecessors' pass-(k-1) outcome
//
// An event whose predecessors are all correct is itself correct after one more
// pass, so event j is final after at most j+1 passes and the sweep stops at the
// first pass that changes nothing: that state is the unique sequential result.
// Batches without failures converge in one pass; a failure only re-evaluates
// what depends on it (its accounts' later sides, same-id / same-pending events,
// its linked chain).  Several batches of one call are one concatenated event
// stream (chains never cross a batch, :1029), each with its own timestamps.
#include "common.h"
#include "engine.h"
#include "transfers.h"

namespace {

__device__ __forceinline__ u32 batch_of(const u32* __restrict__ b_start, u32 nb, u32 i) {
    // largest b with b_start[b] <= i (empty batches resolve to the non-empty one)
    u32 lo = 0, hi = nb;  // invariant: b_start[lo] <= i < b_start[hi]
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (b_start[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// Find-or-insert of a transfer id into the per-call group table.  A slot is
// claimed by CAS of ((event << 1 | is_pending_key) + 1); the key itself is read
// back from the claimer's event, so no u128 CAS is needed.
__device__ __forceinline__ u32 gtab_find_or_insert(const TrArgs& C, u128 key, u32 i, u32 kindbit) {
    const u32 claim = ((i << 1) | kindbit) + 1;
    u64 h = hash128(key) & C.gmask;
    for (;;) {
        u32 cur = C.gclaim[h];
        if (cur == 0) {
            const u32 prev = atomicCAS(&C.gclaim[h], 0u, claim);
            if (prev == 0) return (u32)h;
            cur = prev;
        }
        const u32 ci = (cur - 1) >> 1;
        const u128 ck = ((cur - 1) & 1) ? C.ev[ci].pending_id : C.ev[ci].id;
        if (ck == key) return (u32)h;
        h = (h + 1) & C.gmask;
    }
}

__device__ __forceinline__ u32 gtab_find(const TrArgs& C, u128 key) {
    u64 h = hash128(key) & C.gmask;
    for (;;) {
        const u32 cur = C.gclaim[h];
        if (cur == 0) return NONE32;
        const u32 ci = (cur - 1) >> 1;
        const u128 ck = ((cur - 1) & 1) ? C.ev[ci].pending_id : C.ev[ci].id;
        if (ck == key) return (u32)h;
        h = (h + 1) & C.gmask;
    }
}

// ------------------------------------------------------------ classify ----
// State-independent part of create_transfer / post_or_void (precedence order of
// src/state_machine.zig:1239-1281 and :1398-1412), the timestamp and chain
// bookkeeping of execute (:1018-1035), and the probes that replace prefetch
// (:598-655): debit/credit account slots, pre-existing id, pending transfer.
__global__ void tr_classify(Tables T, TrArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u32 b = batch_of(C.b_start, C.nb, i);
    const u32 bs = C.b_start[b], be = C.b_start[b + 1];
    const u32 nbatch = be - bs, k = i - bs;
    const Transfer t = C.ev[i];
    const u64 ts = C.ev_ts ? C.ev_ts[i] : C.b_ts[b] - nbatch + k + 1;
    C.ts[i] = ts;

    // chain bounds: `linked` unless the router closed the local part of a chain
    // that continues on another shard (TBGPU_CTL_CHAIN_END)
    auto linked = [&](u32 j) {
        return (C.ev[j].flags & TF_LINKED) && !(C.ctl && (C.ctl[j] & TBGPU_CTL_CHAIN_END));
    };
    u32 s = i;
    while (s > bs && linked(s - 1)) s--;
    u32 e = i;
    while (e + 1 < be && linked(e)) e++;
    C.cs[i] = s;
    C.ce[i] = e;
    u32 fl = (s != e) ? FL_CHAINS : 0u;

    u32 dslot = NONE32, cslot = NONE32, pre_e = NONE32, pre_p = NONE32, ppd = NONE32, ppc = NONE32;
    u32 gslot = NONE32, pslot = NONE32;
    u8 sres;
    const u16 f = t.flags;
    if (linked(i) && k == nbatch - 1) {
        sres = TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN;
    } else if (C.ctl && (C.ctl[i] & TBGPU_CTL_SKIP)) {
        sres = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;  // chain broken on another shard
    } else if (t.timestamp != 0) {
        sres = TBGPU_CREATE_TRANSFER_TIMESTAMP_MUST_BE_ZERO;
    } else if (f & 0xFFC0u) {
        sres = TBGPU_CREATE_TRANSFER_RESERVED_FLAG;
    } else if (t.id == 0) {
        sres = TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_ZERO;
    } else if (t.id == U128_MAX) {
        sres = TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_INT_MAX;
    } else if (f & (TF_POST | TF_VOID)) {
        if ((f & TF_POST) && (f & TF_VOID)) sres = TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
        else if (f & TF_PENDING) sres = TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
        else if (f & TF_BDR) sres = TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
        else if (f & TF_BCR) sres = TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
        else if (t.pending_id == 0) sres = TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_ZERO;
        else if (t.pending_id == U128_MAX) sres = TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_INT_MAX;
        else if (t.pending_id == t.id) sres = TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_DIFFERENT;
        else if (t.timeout != 0) sres = TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
        else {
            sres = SRES_DYN;
            fl |= FL_POSTVOID;
            pre_e = xidx_probe(T, t.id);
            pre_p = xidx_probe(T, t.pending_id);
            if (pre_p != NONE32) {
                const Transfer& p = T.xrows[pre_p];
                ppd = acc_probe(T.aidx, T.aidx_mask, p.debit_account_id);
                ppc = acc_probe(T.aidx, T.aidx_mask, p.credit_account_id);
            }
            gslot = gtab_find_or_insert(C, t.id, i, 0);
            pslot = gtab_find_or_insert(C, t.pending_id, i, 1);
        }
    } else if (t.debit_account_id == 0) {
        sres = TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    } else if (t.debit_account_id == U128_MAX) {
        sres = TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    } else if (t.credit_account_id == 0) {
        sres = TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    } else if (t.credit_account_id == U128_MAX) {
        sres = TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    } else if (t.credit_account_id == t.debit_account_id) {
        sres = TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_BE_DIFFERENT;
    } else if (t.pending_id != 0) {
        sres = TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_ZERO;
    } else if (!(f & TF_PENDING) && t.timeout != 0) {
        sres = TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    } else if (!(f & (TF_BDR | TF_BCR)) && t.amount == 0) {
        sres = TBGPU_CREATE_TRANSFER_AMOUNT_MUST_NOT_BE_ZERO;
    } else if (t.ledger == 0) {
        sres = TBGPU_CREATE_TRANSFER_LEDGER_MUST_NOT_BE_ZERO;
    } else if (t.code == 0) {
        sres = TBGPU_CREATE_TRANSFER_CODE_MUST_NOT_BE_ZERO;
    } else if ((dslot = acc_probe(T.aidx, T.aidx_mask, t.debit_account_id)) == NONE32) {
        sres = TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_NOT_FOUND;
    } else if ((cslot = acc_probe(T.aidx, T.aidx_mask, t.credit_account_id)) == NONE32) {
        sres = TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_NOT_FOUND;
    } else {
        const Account& dr = T.acc[dslot];
        const Account& cr = T.acc[cslot];
        if (dr.ledger != cr.ledger) sres = TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
        else if (t.ledger != dr.ledger) sres = TBGPU_CREATE_TRANSFER_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
        else {
            sres = SRES_DYN;
            pre_e = xidx_probe(T, t.id);
            gslot = gtab_find_or_insert(C, t.id, i, 0);
            if (f & (TF_BDR | TF_BCR)) fl |= FL_BALANCING;
            if (f & TF_PENDING) fl |= FL_PENDING;
            if ((dr.flags | cr.flags) & (AF_DNEC | AF_CNED)) fl |= FL_LIMITS;
            if ((dr.flags | cr.flags) & AF_HISTORY) fl |= FL_HISTORY;
        }
    }
    if (sres != SRES_DYN) { dslot = NONE32; cslot = NONE32; }
    C.sres[i] = sres;
    C.dslot[i] = dslot;
    C.cslot[i] = cslot;
    C.pre_e[i] = pre_e;
    C.pre_p[i] = pre_p;
    C.pp_dslot[i] = ppd;
    C.pp_cslot[i] = ppc;
    C.gslot[i] = gslot;
    C.pslot[i] = pslot;
    C.prev_id[i] = NONE32;
    C.pend_last[i] = NONE32;
    C.prev_pend[i] = NONE32;
    if (gslot != NONE32) atomicAdd(&C.gcnt_id[gslot], 1u);
    if (pslot != NONE32) atomicAdd(&C.gcnt_pd[pslot], 1u);
    if (fl) atomicOr(&C.counters[CNT_FLAGS], fl);
}

// Single-member id groups record their member; multi-member groups need a sort.
__global__ void tr_group1(TrArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u32 g = C.gslot[i];
    if (g == NONE32) return;
    u32 fl = 0;
    if (C.gcnt_id[g] == 1) C.gmem[g] = i; else fl |= FL_MULTI_ID;
    const u32 p = C.pslot[i];
    if (p != NONE32 && C.gcnt_pd[p] >= 2) fl |= FL_MULTI_PEND;
    if (fl) atomicOr(&C.counters[CNT_FLAGS], fl);
}

// Sort keys for grouping: events by id slot (kind 0) or post/voids by pending slot (kind 1).
__global__ void tr_group_keys(TrArgs C, u32 kind, u32 invalid, u32* keys, u32* vals) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u32 g = kind == 0 ? C.gslot[i] : C.pslot[i];
    keys[i] = g == NONE32 ? invalid : g;
    vals[i] = i;
}

// Walk the id-sorted members: previous same-id event, and the group's range.
__global__ void tr_group_ranges(TrArgs C, u32 invalid, const u32* ks, const u32* vs) {
    const u32 q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= C.n) return;
    const u32 key = ks[q];
    if (key >= invalid) return;
    const u32 i = vs[q];
    const bool first = q == 0 || ks[q - 1] != key;
    const bool last = q + 1 == C.n || ks[q + 1] != key;
    C.prev_id[i] = first ? NONE32 : vs[q - 1];
    if (first) C.gbeg[key] = q;
    if (last) C.gend[key] = q + 1;
}

__global__ void tr_pend_ranges(TrArgs C, u32 invalid, const u32* ks, const u32* vs) {
    const u32 q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= C.n) return;
    const u32 key = ks[q];
    if (key >= invalid) return;
    C.prev_pend[vs[q]] = (q == 0 || ks[q - 1] != key) ? NONE32 : vs[q - 1];
}

// Last in-call event j < i whose id is i's pending_id.
__global__ void tr_group2(TrArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u32 p = C.pslot[i];
    if (p == NONE32) return;
    const u32 c = C.gcnt_id[p];
    u32 last = NONE32;
    if (c == 1) {
        const u32 j = C.gmem[p];
        if (j < i) last = j;
    } else if (c > 1) {
        u32 lo = C.gbeg[p], hi = C.gend[p];  // members sorted by index
        while (lo < hi) {
            const u32 mid = (lo + hi) >> 1;
            if (C.gmembers[mid] < i) lo = mid + 1; else hi = mid;
        }
        if (lo > C.gbeg[p]) last = C.gmembers[lo - 1];
    }
    C.pend_last[i] = last;
}

// ---------------------------------------------------------- evaluation ----

struct Ctx {
    const Tables& T;
    const TrArgs& C;
    const EvalState& S;  // the pass being read
};

__device__ __forceinline__ Transfer stored_regular(const TrArgs& C, const EvalState& S, u32 j) {
    Transfer t = C.ev[j];
    t.amount = S.amt[j];
    t.timestamp = C.ts[j];
    return t;
}

// The transfer a reference names, as stored (src/state_machine.zig:1326-1328 for
// create_transfer, :1446-1460 for post/void).
__device__ Transfer load_ref(const Tables& T, const TrArgs& C, const EvalState& S, u32 ref) {
    if (ref & PREF_ROW) return T.xrows[ref & ~PREF_ROW];
    const u32 j = ref;
    const Transfer t = C.ev[j];
    if (!(t.flags & (TF_POST | TF_VOID))) return stored_regular(C, S, j);
    const u32 pr = S.pref[j];
    Transfer p;
    if (pr == NONE32) {
        p = t;  // unreachable for a visible (ok) post/void
    } else if (pr & PREF_ROW) {
        p = T.xrows[pr & ~PREF_ROW];
    } else {
        p = stored_regular(C, S, pr);
    }
    Transfer s;
    s.id = t.id;
    s.debit_account_id = p.debit_account_id;
    s.credit_account_id = p.credit_account_id;
    s.user_data_128 = t.user_data_128 > 0 ? t.user_data_128 : p.user_data_128;
    s.user_data_64 = t.user_data_64 > 0 ? t.user_data_64 : p.user_data_64;
    s.user_data_32 = t.user_data_32 > 0 ? t.user_data_32 : p.user_data_32;
    s.ledger = p.ledger;
    s.code = p.code;
    s.pending_id = t.pending_id;
    s.timeout = 0;
    s.timestamp = C.ts[j];
    s.flags = t.flags;
    s.amount = S.amt[j];
    return s;
}

// create_transfer_exists (src/state_machine.zig:1370-1389)
__device__ __forceinline__ u8 create_transfer_exists(const Transfer& t, const Transfer& e) {
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

// post_or_void_pending_transfer_exists (src/state_machine.zig:1500-1561)
__device__ __forceinline__ u8 post_or_void_exists(const Transfer& t, const Transfer& e, const Transfer& p) {
    if (t.flags != e.flags) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_FLAGS;
    if (t.amount == 0) {
        if (e.amount != p.amount) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_AMOUNT;
    } else {
        if (t.amount != e.amount) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_AMOUNT;
    }
    if (t.pending_id != e.pending_id) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_PENDING_ID;
    if (t.user_data_128 == 0) {
        if (e.user_data_128 != p.user_data_128) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    } else {
        if (t.user_data_128 != e.user_data_128) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    }
    if (t.user_data_64 == 0) {
        if (e.user_data_64 != p.user_data_64) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    } else {
        if (t.user_data_64 != e.user_data_64) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    }
    if (t.user_data_32 == 0) {
        if (e.user_data_32 != p.user_data_32) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    } else {
        if (t.user_data_32 != e.user_data_32) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    }
    return TBGPU_CREATE_TRANSFER_EXISTS;
}

// Balance-dependent tail of create_transfer (src/state_machine.zig:1286-1322).
__device__ __forceinline__ u8 eval_balances(const Transfer& t, const Bal4& dr, const Bal4& cr, u16 dr_flags,
                                            u16 cr_flags, u128* amount_out) {
    const u16 f = t.flags;
    u128 amount = t.amount;
    if ((f & (TF_BDR | TF_BCR)) && amount == 0) amount = (u128)0xFFFFFFFFFFFFFFFFull;  // maxInt(u64)
    if (f & TF_BDR) {
        const u128 dr_balance = dr.dpo + dr.dp;
        const u128 avail = dr.cpo > dr_balance ? dr.cpo - dr_balance : 0;  // -| saturating
        if (avail < amount) amount = avail;
        if (amount == 0) return TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS;
    }
    if (f & TF_BCR) {
        const u128 cr_balance = cr.cpo + cr.cp;
        const u128 avail = cr.dpo > cr_balance ? cr.dpo - cr_balance : 0;
        if (avail < amount) amount = avail;
        if (amount == 0) return TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS;
    }
    if (f & TF_PENDING) {
        if (sum_overflows128(amount, dr.dp)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS_PENDING;
        if (sum_overflows128(amount, cr.cp)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS_PENDING;
    }
    if (sum_overflows128(amount, dr.dpo)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS_POSTED;
    if (sum_overflows128(amount, cr.cpo)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS_POSTED;
    if (sum_overflows128(amount, dr.dp + dr.dpo)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS;
    if (sum_overflows128(amount, cr.cp + cr.cpo)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS;
    if (sum_overflows64(t.timestamp, (u64)t.timeout * NS_PER_S)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT;
    if ((dr_flags & AF_DNEC) && dr.dp + dr.dpo + amount > dr.cpo) return TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS;
    if ((cr_flags & AF_CNED) && cr.cp + cr.cpo + amount > cr.dpo) return TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS;
    *amount_out = amount;
    return TBGPU_CREATE_TRANSFER_OK;
}

__device__ __forceinline__ bool visible(const TrArgs& C, const EvalState& S, u32 j, u32 csi) {
    const u8 o = S.ok[j];
    return C.cs[j] == csi ? (o & 1) : (o & 2);
}

// One Jacobi pass: read state S (pass k-1), write state D (pass k).
__global__ void tr_evaluate(Tables T, TrArgs C, EvalState S, EvalState D, const u32* __restrict__ spos,
                            const Bal4* __restrict__ bb) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 sr = C.sres[i];
    u8 res;
    u128 amt = 0, pamt = 0, dpe = 0, dpo = 0;
    u32 pref = NONE32;
    const u32 csi = C.cs[i];
    if (sr != SRES_DYN) {
        res = sr;
    } else {
        Transfer t = C.ev[i];
        t.timestamp = C.ts[i];
        u32 e = NONE32;
        for (u32 j = C.prev_id[i]; j != NONE32; j = C.prev_id[j])
            if (visible(C, S, j, csi)) { e = j; break; }
        if (e == NONE32 && C.pre_e[i] != NONE32) e = PREF_ROW | C.pre_e[i];
        if (!(t.flags & (TF_POST | TF_VOID))) {
            if (e != NONE32) {
                res = create_transfer_exists(t, load_ref(T, C, S, e));
            } else {
                const Bal4 bd = bb[spos[2 * i]];
                const Bal4 bc = bb[spos[2 * i + 1]];
                const u16 dfl = T.acc[C.dslot[i]].flags, cfl = T.acc[C.cslot[i]].flags;
                u128 amount = 0;
                res = eval_balances(t, bd, bc, dfl, cfl, &amount);
                if (res == TBGPU_CREATE_TRANSFER_OK) {
                    amt = amount;
                    if (t.flags & TF_PENDING) dpe = amount; else dpo = amount;
                }
            }
        } else {
            // post_or_void_pending_transfer (src/state_machine.zig:1391-1498)
            u32 p = NONE32;
            for (u32 j = C.pend_last[i]; j != NONE32; j = C.prev_id[j])
                if (visible(C, S, j, csi)) { p = j; break; }
            if (p == NONE32 && C.pre_p[i] != NONE32) p = PREF_ROW | C.pre_p[i];
            pref = p;
            const bool post = t.flags & TF_POST;
            if (p == NONE32) {
                res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_FOUND;
            } else {
                const Transfer P = load_ref(T, C, S, p);
                const u128 amount = t.amount > 0 ? t.amount : P.amount;
                if (!(P.flags & TF_PENDING)) res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_PENDING;
                else if (t.debit_account_id > 0 && t.debit_account_id != P.debit_account_id)
                    res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
                else if (t.credit_account_id > 0 && t.credit_account_id != P.credit_account_id)
                    res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
                else if (t.ledger > 0 && t.ledger != P.ledger) res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
                else if (t.code > 0 && t.code != P.code) res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_CODE;
                else if (amount > P.amount) res = TBGPU_CREATE_TRANSFER_EXCEEDS_PENDING_TRANSFER_AMOUNT;
                else if ((t.flags & TF_VOID) && amount < P.amount)
                    res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;
                else if (e != NONE32) res = post_or_void_exists(t, load_ref(T, C, S, e), P);
                else {
                    // posted groove (src/state_machine.zig:1431-1436)
                    u32 ful = 0;
                    for (u32 j = C.prev_pend[i]; j != NONE32; j = C.prev_pend[j])
                        if (visible(C, S, j, csi)) { ful = (C.ev[j].flags & TF_POST) ? 1 : 2; break; }
                    if (ful == 0 && (p & PREF_ROW)) ful = T.xful[p & ~PREF_ROW];
                    if (ful == 1) res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_ALREADY_POSTED;
                    else if (ful == 2) res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_ALREADY_VOIDED;
                    else if (P.timeout > 0 && t.timestamp >= P.timestamp + (u64)P.timeout * NS_PER_S)
                        res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_EXPIRED;
                    else {
                        res = TBGPU_CREATE_TRANSFER_OK;
                        amt = amount;
                        pamt = P.amount;
                        dpe = (u128)0 - P.amount;
                        dpo = post ? amount : 0;
                    }
                }
            }
        }
    }
    D.res[i] = res;
    D.ok[i] = res == TBGPU_CREATE_TRANSFER_OK ? 1 : 0;
    D.amt[i] = amt;
    D.pamt[i] = pamt;
    D.pref[i] = pref;
    D.dpend[i] = dpe;
    D.dpost[i] = dpo;
    if (res != TBGPU_CREATE_TRANSFER_OK && csi != C.ce[i]) atomicMin(&D.cfail[csi], i);
    const bool changed = res != S.res[i] || amt != S.amt[i] || pamt != S.pamt[i] || pref != S.pref[i];
    if (changed) atomicAdd(&C.counters[CNT_CHANGES], 1u);
}

// Optimistic starting point: every statically valid event succeeds.
__global__ void tr_init(Tables T, TrArgs C, EvalState D) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 sr = C.sres[i];
    u8 res = sr;
    u128 amt = 0, pamt = 0, dpe = 0, dpo = 0;
    u32 pref = NONE32;
    if (sr == SRES_DYN) {
        const Transfer& t = C.ev[i];
        if (!(t.flags & (TF_POST | TF_VOID))) {
            res = 0;
            amt = t.amount;
            if ((t.flags & (TF_BDR | TF_BCR)) && amt == 0) amt = (u128)0xFFFFFFFFFFFFFFFFull;
            if (t.flags & TF_PENDING) dpe = amt; else dpo = amt;
        } else {
            const u32 j = C.pend_last[i];
            pref = j != NONE32 ? j : (C.pre_p[i] != NONE32 ? (PREF_ROW | C.pre_p[i]) : NONE32);
            if (pref == NONE32) {
                res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_FOUND;
            } else {
                res = 0;
                pamt = (pref & PREF_ROW) ? T.xrows[pref & ~PREF_ROW].amount : C.ev[pref].amount;
                amt = t.amount > 0 ? t.amount : pamt;
                dpe = (u128)0 - pamt;
                dpo = (t.flags & TF_POST) ? amt : 0;
            }
        }
    }
    D.res[i] = res;
    D.ok[i] = res == 0 ? 1 : 0;
    D.amt[i] = amt;
    D.pamt[i] = pamt;
    D.pref[i] = pref;
    D.dpend[i] = dpe;
    D.dpost[i] = dpo;
    if (res != 0 && C.cs[i] != C.ce[i]) atomicMin(&D.cfail[C.cs[i]], i);
}

// final-ok = eval-ok and the event's chain was persisted (scope_close(.persist)).
__global__ void tr_finalize(TrArgs C, EvalState D) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 o = D.ok[i] & 1;
    const u32 cs = C.cs[i];
    const bool doom = C.ctl && (C.ctl[C.ce[i]] & TBGPU_CTL_DOOM);  // broken on another shard
    const bool persisted = (cs == C.ce[i] || D.cfail[cs] == NONE32) && !doom;
    D.ok[i] = o | ((o && persisted) ? 2 : 0);
}

// Side keys: the debit and credit account slots each event may touch.
__global__ void tr_sides(TrArgs C, EvalState S, u32 invalid, u32* skey, u32* sval) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    u32 d = NONE32, c = NONE32;
    if (C.sres[i] == SRES_DYN) {
        if (!(C.ev[i].flags & (TF_POST | TF_VOID))) {
            d = C.dslot[i];
            c = C.cslot[i];
        } else {
            // An unresolved post/void fails and moves no balance, so any key serves:
            // keep its candidate pending's accounts and the keys stay put from pass to
            // pass (a moved key costs a full re-sort).
            u32 p = S.pref[i];
            if (p == NONE32) p = C.pend_last[i] != NONE32 ? C.pend_last[i]
                                 : (C.pre_p[i] != NONE32 ? (PREF_ROW | C.pre_p[i]) : NONE32);
            if (p != NONE32) {
                if (p & PREF_ROW) { d = C.pp_dslot[i]; c = C.pp_cslot[i]; }
                else { d = C.dslot[p]; c = C.cslot[p]; }
            }
        }
    }
    if (d == NONE32 || c == NONE32) d = c = invalid;
    if (skey[2 * i] != d || skey[2 * i + 1] != c) atomicAdd(&C.counters[CNT_KEYS], 1u);
    skey[2 * i] = d;
    skey[2 * i + 1] = c;
    sval[2 * i] = 2 * i;
    sval[2 * i + 1] = 2 * i + 1;
}

__global__ void tr_side_pos(const u32* sval_s, u64 m, u32* spos) {
    const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < m) spos[sval_s[q]] = (u32)q;
}

// ---------------------------------------------------------------- apply ----

// Final result per event, as execute emits it (src/state_machine.zig:1051-1072).
__global__ void tr_mask(Tables T, TrArgs C, EvalState S, u8* fres, u8* mask) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u32 cs = C.cs[i];
    const bool doom = C.ctl && (C.ctl[C.ce[i]] & TBGPU_CTL_DOOM);
    const bool inch = cs != C.ce[i] || doom;
    u32 cf = inch ? S.cfail[cs] : NONE32;
    if (cf == NONE32 && doom) cf = C.ce[i] + 1;  // the chain breaks after its last local member
    u8 r;
    if (C.sres[i] == TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN) r = TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN;
    else if (cf < i) r = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
    else if (S.res[i] != 0) r = S.res[i];
    else if (cf != NONE32) r = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
    else r = TBGPU_CREATE_TRANSFER_OK;
    const bool ok = S.ok[i] & 2;
    bool hist = false;
    if (ok && !(C.ev[i].flags & (TF_POST | TF_VOID)))
        hist = (T.acc[C.dslot[i]].flags | T.acc[C.cslot[i]].flags) & AF_HISTORY;
    fres[i] = r;
    mask[i] = (ok ? 1 : 0) | (r != 0 ? 2 : 0) | (hist ? 4 : 0);
    // commit_timestamp is a plain field, not undone by scope_close(.discard): every
    // create_transfer that returned ok before its chain broke advanced it (:1366).
    if ((S.ok[i] & 1) && (cf == NONE32 || i < cf))
        atomicMax((unsigned long long*)C.commit_ts, (unsigned long long)C.ts[i]);
}

__global__ void tr_apply(Tables T, TrArgs C, EvalState S, const u8* __restrict__ fres, const uint4* __restrict__ rk,
                         const u32* __restrict__ spos, const Bal4* __restrict__ bb, u64 row_base, u64 hist_base,
                         tbgpu_create_transfers_result_t* __restrict__ results) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 r = fres[i];
    const uint4 q = rk[i];
    if (r != 0) {
        // replies of consecutive batches are concatenated: global non-ok rank
        const u32 b = batch_of(C.b_start, C.nb, i);
        results[q.y] = {i - C.b_start[b], (u32)r};
        return;
    }
    if (C.dry || !(S.ok[i] & 2)) return;
    const Transfer t = C.ev[i];
    const u64 row = row_base + q.x;
    const Transfer s = load_ref(T, C, S, i);
    T.xrows[row] = s;
    xidx_insert(T, t.id, (u32)row);
    if (t.flags & (TF_POST | TF_VOID)) {
        const u32 p = S.pref[i];
        const u64 prow = (p & PREF_ROW) ? (u64)(p & ~PREF_ROW) : row_base + rk[p].x;
        T.xful[prow] = (t.flags & TF_POST) ? 1 : 2;
    } else {
        const Account& dra = T.acc[C.dslot[i]];
        const Account& cra = T.acc[C.cslot[i]];
        if ((dra.flags | cra.flags) & AF_HISTORY) {
            // balances after this transfer (src/state_machine.zig:1342-1364)
            Bal4 d = bb[spos[2 * i]], c = bb[spos[2 * i + 1]];
            d.dp += S.dpend[i]; d.dpo += S.dpost[i];
            c.cp += S.dpend[i]; c.cpo += S.dpost[i];
            History h;
            memset(&h, 0, sizeof h);
            h.timestamp = s.timestamp;
            if (dra.flags & AF_HISTORY) {
                h.dr_account_id = dra.id;
                h.dr_debits_pending = d.dp; h.dr_debits_posted = d.dpo;
                h.dr_credits_pending = d.cp; h.dr_credits_posted = d.cpo;
            }
            if (cra.flags & AF_HISTORY) {
                h.cr_account_id = cra.id;
                h.cr_debits_pending = c.dp; h.cr_debits_posted = c.dpo;
                h.cr_credits_pending = c.cp; h.cr_credits_posted = c.cpo;
            }
            T.hrows[hist_base + q.z] = h;
        }
    }
}

// Widen the index's componentwise key range by the stored ids (one atomic per
// wave and word; every lane of every wave takes part).
__global__ void tr_range(Tables T, TrArgs C, EvalState S) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = i < C.n && (S.ok[i] & 2);
    const u128 id = ok ? C.ev[i].id : 0;
    u64 r[4] = {ok ? (u64)id : 0, ok ? (u64)(id >> 64) : 0, ok ? (u64)id : ~0ull, ok ? (u64)(id >> 64) : ~0ull};
    for (int off = 32; off > 0; off >>= 1) {
        r[0] = max(r[0], (u64)__shfl_xor((unsigned long long)r[0], off));
        r[1] = max(r[1], (u64)__shfl_xor((unsigned long long)r[1], off));
        r[2] = min(r[2], (u64)__shfl_xor((unsigned long long)r[2], off));
        r[3] = min(r[3], (u64)__shfl_xor((unsigned long long)r[3], off));
    }
    if ((threadIdx.x & 63) == 0 && r[0] | r[1] | ~r[2] | ~r[3]) {
        atomicMax((unsigned long long*)&T.idr[0], (unsigned long long)r[0]);
        atomicMax((unsigned long long*)&T.idr[1], (unsigned long long)r[1]);
        atomicMin((unsigned long long*)&T.idr[2], (unsigned long long)r[2]);
        atomicMin((unsigned long long*)&T.idr[3], (unsigned long long)r[3]);
    }
}

__global__ void batch_counts(const u32* b_start, u32 nb, const uint4* rk, u32* counts) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) counts[b] = rk[b_start[b + 1]].y - rk[b_start[b]].y;
}

}  // namespace

// ------------------------------------------------------------ launchers ----
#define GRID(n) (u32)(((n) + 255) / 256), 256, 0, stream

void tr_launch_classify(const Tables& T, const TrArgs& C, hipStream_t stream) {
    tr_classify<<<GRID(C.n)>>>(T, C);
    tr_group1<<<GRID(C.n)>>>(C);
}
void tr_launch_group_sort(const TrArgs& C, u32 kind, u32 invalid, int bits, u32* k_in, u32* v_in, u32* k_out,
                          u32* v_out, SortScratch& ss, hipStream_t stream) {
    tr_group_keys<<<GRID(C.n)>>>(C, kind, invalid, k_in, v_in);
    radix_sort_pairs(k_in, v_in, k_out, v_out, C.n, bits, ss, stream);
    if (kind == 0) tr_group_ranges<<<GRID(C.n)>>>(C, invalid, k_out, v_out);
    else tr_pend_ranges<<<GRID(C.n)>>>(C, invalid, k_out, v_out);
}
void tr_launch_group2(const TrArgs& C, hipStream_t stream) { tr_group2<<<GRID(C.n)>>>(C); }
void tr_launch_init(const Tables& T, const TrArgs& C, const EvalState& D, hipStream_t stream) {
    tr_init<<<GRID(C.n)>>>(T, C, D);
    tr_finalize<<<GRID(C.n)>>>(C, D);
}
void tr_launch_sides(const TrArgs& C, const EvalState& S, u32 invalid, u32* skey, u32* sval, hipStream_t stream) {
    tr_sides<<<GRID(C.n)>>>(C, S, invalid, skey, sval);
}
void tr_launch_side_pos(const u32* sval_s, u64 m, u32* spos, hipStream_t stream) {
    tr_side_pos<<<GRID(m)>>>(sval_s, m, spos);
}
void tr_launch_evaluate(const Tables& T, const TrArgs& C, const EvalState& S, const EvalState& D, const u32* spos,
                        const Bal4* bb, hipStream_t stream) {
    tr_evaluate<<<GRID(C.n)>>>(T, C, S, D, spos, bb);
    tr_finalize<<<GRID(C.n)>>>(C, D);
}
void tr_launch_mask(const Tables& T, const TrArgs& C, const EvalState& S, u8* fres, u8* mask, hipStream_t stream) {
    tr_mask<<<GRID(C.n)>>>(T, C, S, fres, mask);
}
void tr_launch_apply(const Tables& T, const TrArgs& C, const EvalState& S, const u8* fres, const uint4* rk,
                     const u32* spos, const Bal4* bb, u64 row_base, u64 hist_base,
                     tbgpu_create_transfers_result_t* results, u32* counts, hipStream_t stream) {
    tr_apply<<<GRID(C.n)>>>(T, C, S, fres, rk, spos, bb, row_base, hist_base, results);
    if (!C.dry) tr_range<<<GRID(C.n)>>>(T, C, S);
    batch_counts<<<GRID(C.nb)>>>(C.b_start, C.nb, rk, counts);
}
