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
#include <algorithm>

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

// Wave-level reductions: one global atomic per wave instead of one per event (a
// flag word or counter hit by every event serializes at the memory side).
__device__ __forceinline__ u32 wave_or(u32 v) {
    for (int off = 32; off > 0; off >>= 1) v |= __shfl_xor(v, off);
    return v;
}
// Workgroup reductions for flag words and counters: one atomic per workgroup, not
// per wave (same-address atomics serialize at the memory side, ≈5-10 ns each: one per
// wave of a 131k-event launch is 2k of them, longer than the launch's own work).
// Every thread of the workgroup must call; the result is valid in thread 0.
__device__ __forceinline__ u32 block_or(u32 v) {
    __shared__ u32 s_red[16];
    for (int off = 32; off > 0; off >>= 1) v |= __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    u32 r = 0;
    if (threadIdx.x == 0)
        for (u32 k = 0; k < (blockDim.x + 63) / 64; k++) r |= s_red[k];
    return r;
}
__device__ __forceinline__ u32 block_sum(u32 v) {
    __shared__ u32 s_sum[16];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = v;
    __syncthreads();
    u32 r = 0;
    if (threadIdx.x == 0)
        for (u32 k = 0; k < (blockDim.x + 63) / 64; k++) r += s_sum[k];
    return r;
}
__device__ __forceinline__ u32 block_min(u32 v) {
    __shared__ u32 s_min[16];
    for (int off = 32; off > 0; off >>= 1) v = min(v, (u32)__shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) s_min[threadIdx.x >> 6] = v;
    __syncthreads();
    u32 r = NONE32;
    if (threadIdx.x == 0)
        for (u32 k = 0; k < (blockDim.x + 63) / 64; k++) r = min(r, s_min[k]);
    return r;
}
__device__ __forceinline__ u32 wave_min(u32 v) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, (u32)__shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ u64 wave_max64(u64 v) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, (u64)__shfl_xor((unsigned long long)v, off));
    return v;
}

// Find-or-insert of a transfer id into the per-call group table.  A slot is
// claimed by CAS of ((event << 1 | is_pending_key) + 1); the key itself is read
// back from the claimer's event, so no u128 CAS is needed.
__device__ __forceinline__ u32 gtab_find_or_insert(const TrArgs& C, u128 key, u32 i, u32 kindbit) {
    const u32 claim = ((i << 1) | kindbit) + 1;
    u64 h = hash128(key) & C.gmask;
    for (;;) {
        // the CAS itself reads the slot (a load first cost a round trip more for the
        // usual empty slot)
        const u32 cur = atomicCAS(&C.gclaim[h], 0u, claim);
        if (cur == 0) return (u32)h;
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
__device__ __forceinline__ u32 classify_one(const Tables& T, const TrArgs& C, u32 i) {
    // the batch: one uniform (scalar) search per wave for its first event; a wave
    // spans 64 events, so lanes past a batch boundary walk on a step or two
    const u32 w0 = __builtin_amdgcn_readfirstlane(i - (threadIdx.x & 63));
    const Transfer t = C.ev[i];
    const u32 wb = batch_of(C.b_start, C.nb, w0);
    u32 b = wb;
    while (C.b_start[b + 1] <= i) b++;
    const u32 bs = C.b_start[b], be = C.b_start[b + 1];
    const u32 nbatch = be - bs, k = i - bs;
    // the accounts' directory entries, issued before the checks that order their use
    const bool dd = dense_has(T, t.debit_account_id), dc = dense_has(T, t.credit_account_id);
    const u64 ed = dd ? T.dense[dense_slot(T, t.debit_account_id)] : 0;
    const u64 ec = dc ? T.dense[dense_slot(T, t.credit_account_id)] : 0;
    const u64 ts = C.ev_ts ? C.ev_ts[i] : C.b_ts[b] - nbatch + k + 1;
    C.ts[i] = ts;

    // chain bounds: `linked` unless the router closed the local part of a chain
    // that continues on another shard (TBGPU_CTL_CHAIN_END)
    auto linked = [&](u32 j) {
        return (C.ev[j].flags & TF_LINKED) && !(C.ctl && (C.ctl[j] & TBGPU_CTL_CHAIN_END));
    };
    // within the wave from one ballot of the lanes' own flags; only a chain that
    // crosses the wave's edge walks on (lanes below an active lane are active)
    const u32 lane = threadIdx.x & 63;
    const u64 lm = __ballot((t.flags & TF_LINKED) && !(C.ctl && (C.ctl[i] & TBGPU_CTL_CHAIN_END)));
    const u64 below = ~lm & ((1ull << lane) - 1), above = ~lm & (~0ull << lane);
    u32 s, e;
    if (below) {
        s = w0 + 64 - __clzll((long long)below);  // one past the last unlinked lane below
    } else {
        s = w0;
        while (s > bs && linked(s - 1)) s--;
    }
    if (s < bs) s = bs;
    if (above) {
        e = w0 + __ffsll((unsigned long long)above) - 1;
    } else {
        e = w0 + 63;
        while (e + 1 < be && linked(e)) e++;
    }
    if (e > be - 1) e = be - 1;
    C.cs[i] = s;
    C.ce[i] = e;
    u32 fl = (s != e) ? FL_CHAINS : 0u;

    u32 dslot = NONE32, cslot = NONE32, pre_e = NONE32, pre_p = NONE32, ppd = NONE32, ppc = NONE32;
    u32 gslot = NONE32, pslot = NONE32;
    u32 dled = 0, cled = 0;
    u16 dfl = 0, cfl = 0;
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
            if ((u64)(t.amount >> 64) != 0) fl |= FL_WIDE;
            if (t.amount >> 40) fl |= FL_WIDE64;
            if (pre_p != NONE32) {
                const Transfer& p = T.xrows[pre_p];
                if ((u64)(p.amount >> 64) != 0) fl |= FL_WIDE;
                if (p.amount >> 40) fl |= FL_WIDE64;
                u32 lg;
                u16 af;
                ppd = acc_find(T, p.debit_account_id, &lg, &af);
                ppc = acc_find(T, p.credit_account_id, &lg, &af);
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
    } else if ((dslot = dd ? acc_from_dense(ed, &dled, &dfl) : acc_find(T, t.debit_account_id, &dled, &dfl)) ==
               NONE32) {
        sres = TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_NOT_FOUND;
    } else if ((cslot = dc ? acc_from_dense(ec, &cled, &cfl) : acc_find(T, t.credit_account_id, &cled, &cfl)) ==
               NONE32) {
        sres = TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_NOT_FOUND;
    } else {
        if (dled != cled) sres = TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
        else if (t.ledger != dled) sres = TBGPU_CREATE_TRANSFER_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
        else {
            // (a ledger shard: the accounts may be another shard's, ROW_FOREIGN, when the
            // router sent the event here because its id is committed or first seen here:
            // it can only answer `exists*`, which evaluate_one checks before any balance)
            sres = SRES_DYN;
            pre_e = xidx_probe(T, t.id);
            gslot = gtab_find_or_insert(C, t.id, i, 0);
            if (f & (TF_BDR | TF_BCR)) fl |= FL_BALANCING;
            if (f & TF_PENDING) fl |= FL_PENDING;
            if ((u64)(t.amount >> 64) != 0) fl |= FL_WIDE;
            if (t.amount >> 40) fl |= FL_WIDE64;
            if ((dfl | cfl) & (AF_DNEC | AF_CNED)) fl |= FL_LIMITS;
            if ((dfl | cfl) & AF_HISTORY) fl |= FL_HISTORY;
        }
    }
    if (sres != SRES_DYN) { dslot = NONE32; cslot = NONE32; }
    EvCore core;
    core.amount = t.amount;
    core.ts = ts;
    core.timeout = t.timeout;
    core.flags = f;
    core.aflags = (u8)((dfl & 0xF) | (cfl & 0xF) << 4);
    core.pad = 0;
    C.core[i] = core;
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
    C.pend_first[i] = NONE32;
    C.prev_pend[i] = NONE32;
    if (gslot != NONE32) atomicAdd(&C.gcnt_id[gslot], 1u);
    if (pslot != NONE32) atomicAdd(&C.gcnt_pd[pslot], 1u);
    return fl;
}

__global__ void tr_classify(Tables T, TrArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    u32 fl = block_or(i < C.n ? classify_one(T, C, i) : 0u);
    if (i == 0 && (*T.big & 1)) fl |= FL_WIDE;    // a committed balance near 2^128
    if (i == 0 && (*T.big & 2)) fl |= FL_WIDE64;  // a committed balance >= 2^61
    if (threadIdx.x == 0) raise_flags(&C.counters[CNT_FLAGS], fl);
}

// Single-member id groups record their member; multi-member groups need a sort.
__global__ void tr_group1(TrArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    u32 fl = 0;
    const u32 g = i < C.n ? C.gslot[i] : NONE32;
    if (g != NONE32) {
        if (C.gcnt_id[g] == 1) C.gmem[g] = i; else fl |= FL_MULTI_ID;
        const u32 p = C.pslot[i];
        if (p != NONE32 && C.gcnt_pd[p] >= 2) fl |= FL_MULTI_PEND;
    }
    fl = block_or(fl);
    if (threadIdx.x == 0) raise_flags(&C.counters[CNT_FLAGS], fl);
}

// Sort keys for grouping: events by id slot (kind 0) or post/voids by pending slot (kind 1).
// The group kernels run only when classify found what they are for (the flag
// word is on the device: no host round trip decides it).
__device__ __forceinline__ bool need(const TrArgs& C, u32 kind) {
    return C.counters[CNT_FLAGS] & (kind == 0 ? FL_MULTI_ID : FL_MULTI_PEND);
}

// Groups of 2+ members, without sorting the call: (1) one member of each group
// reserves the group's range (a per-wave prefix of the counts, one cursor atomic per
// wave), (2) every member takes a place in its range, (3) every member counts the
// members before it (its rank: the range ends up in event order) and finds its
// predecessor.  Groups are small; a group of k members costs k^2 / 2 reads in (3).
__device__ __forceinline__ void grp_fields(const TrArgs& C, u32 kind, u32 i, u32* slot, u32* cnt) {
    *slot = kind == 0 ? C.gslot[i] : C.pslot[i];
    *cnt = *slot == NONE32 ? 0u : (kind == 0 ? C.gcnt_id[*slot] : C.gcnt_pd[*slot]);
}

constexpr u32 GR_THREADS = 1024;  // one cursor atomic per 1024 events (per wave: ~10 us per chunk)
// The id groups (kind 0) and the pending groups (kind 1) do not read each other: each
// launch takes both, `nb` workgroups per kind (kind0 + blockIdx.x / nb).
__global__ __launch_bounds__(GR_THREADS) void tr_grp_reserve(TrArgs C, u32 kind0, u32 nb) {
    __shared__ u32 s_tot[GR_THREADS / 64];
    __shared__ u32 s_base;
    const u32 kind = kind0 + blockIdx.x / nb;
    const u32 i = (blockIdx.x % nb) * blockDim.x + threadIdx.x;
    if (!need(C, kind)) return;
    u32 slot = NONE32, cnt = 0;
    if (i < C.n) grp_fields(C, kind, i, &slot, &cnt);
    u32* beg = kind == 0 ? C.gbeg : C.pbeg;
    const bool win = cnt >= 2 && atomicCAS(&beg[slot], NONE32, NONE32 - 1) == NONE32;
    u32 mine = win ? cnt : 0u, pre = mine;
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int off = 1; off < 64; off <<= 1) {  // inclusive prefix over the wave
        const u32 o = __shfl_up(pre, off);
        if (lane >= (u32)off) pre += o;
    }
    if (lane == 63) s_tot[w] = pre;
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 tot = 0;
        for (u32 k = 0; k < GR_THREADS / 64; k++) tot += s_tot[k];
        s_base = tot ? atomicAdd(&C.counters[kind == 0 ? CNT_GCUR : CNT_PCUR], tot) : 0u;
    }
    __syncthreads();
    if (win) {
        u32 base = s_base;
        for (u32 k = 0; k < w; k++) base += s_tot[k];
        beg[slot] = base + pre - mine;
    }
}

__global__ void tr_grp_place(TrArgs C, u32 kind0, u32 nb) {
    const u32 kind = kind0 + blockIdx.x / nb;
    const u32 i = (blockIdx.x % nb) * blockDim.x + threadIdx.x;
    if (i >= C.n || !need(C, kind)) return;
    u32 slot, cnt;
    grp_fields(C, kind, i, &slot, &cnt);
    if (cnt < 2) return;
    const u32 b = kind == 0 ? C.gbeg[slot] : C.pbeg[slot];
    const u32 k = atomicAdd(kind == 0 ? &C.gfill[slot] : &C.pfill[slot], 1u);
    (kind == 0 ? C.glist : C.plist)[b + k] = i;
}

__global__ void tr_grp_rank(TrArgs C, u32 kind0, u32 nb) {
    const u32 kind = kind0 + blockIdx.x / nb;
    const u32 i = (blockIdx.x % nb) * blockDim.x + threadIdx.x;
    if (i >= C.n || !need(C, kind)) return;
    u32 slot, cnt;
    grp_fields(C, kind, i, &slot, &cnt);
    if (cnt < 2) return;
    const u32 b = kind == 0 ? C.gbeg[slot] : C.pbeg[slot];
    const u32* list = kind == 0 ? C.glist : C.plist;
    u32 r = 0, prev = NONE32;
    for (u32 j = b; j < b + cnt; j++) {
        const u32 v = list[j];
        if (v < i) {
            r++;
            prev = prev == NONE32 ? v : max(prev, v);
        }
    }
    if (kind == 0) {
        C.gmembers[b + r] = i;
        C.prev_id[i] = prev;
        if (r == 0) C.gend[slot] = b + cnt;
    } else {
        C.prev_pend[i] = prev;
    }
}

// Last in-call event j < i whose id is i's pending_id.
__global__ void tr_group2(TrArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n || !(C.counters[CNT_FLAGS] & FL_POSTVOID)) return;
    const u32 p = C.pslot[i];
    if (p == NONE32) return;
    const u32 c = C.gcnt_id[p];
    u32 last = NONE32, first = NONE32;
    if (c == 1) {
        const u32 j = C.gmem[p];
        if (j < i) last = first = j;
    } else if (c > 1) {
        u32 lo = C.gbeg[p], hi = C.gend[p];  // members sorted by index
        while (lo < hi) {
            const u32 mid = (lo + hi) >> 1;
            if (C.gmembers[mid] < i) lo = mid + 1; else hi = mid;
        }
        if (lo > C.gbeg[p]) {
            last = C.gmembers[lo - 1];
            first = C.gmembers[C.gbeg[p]];
        }
    }
    C.pend_last[i] = last;
    C.pend_first[i] = first;
}

// ---------------------------------------------------------- evaluation ----

__device__ __forceinline__ bool is_post_void_ev(const TrArgs& C, u32 i) {
    return C.sres[i] == SRES_DYN && (C.core[i].flags & (TF_POST | TF_VOID));
}

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
__device__ __forceinline__ u8 eval_balances(const EvCore& t, const Bal4& dr, const Bal4& cr, u128* amount_out) {
    const u16 f = t.flags;
    const u16 dr_flags = t.aflags & 0xF, cr_flags = t.aflags >> 4;
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
    if (sum_overflows64(t.ts, (u64)t.timeout * NS_PER_S)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT;
    if ((dr_flags & AF_DNEC) && dr.dp + dr.dpo + amount > dr.cpo) return TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS;
    if ((cr_flags & AF_CNED) && cr.cp + cr.cpo + amount > cr.dpo) return TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS;
    *amount_out = amount;
    return TBGPU_CREATE_TRANSFER_OK;
}

// The same tail in headroom form (balances.hip side_scan_fused_narrow), for passes of a
// chunk whose amounts are < 2^64 and whose committed balances are < 2^126 (FL_WIDE
// clear): then no overflow check can fire (a balance moves by < 2^84 inside a chunk),
// and the limit and balancing checks read hd = dr.credits_posted - dr.debits_pending -
// dr.debits_posted and hc = cr.debits_posted - cr.credits_pending - cr.credits_posted.
__device__ __forceinline__ u8 eval_balances_narrow(const EvCore& t, u128 hd, u128 hc, u128* amount_out) {
    typedef __int128 i128;
    const u16 f = t.flags;
    const u16 dr_flags = t.aflags & 0xF, cr_flags = t.aflags >> 4;
    const i128 sd = (i128)hd, sc = (i128)hc;
    u128 amount = t.amount;
    if ((f & (TF_BDR | TF_BCR)) && amount == 0) amount = (u128)0xFFFFFFFFFFFFFFFFull;  // maxInt(u64)
    if (f & TF_BDR) {
        const u128 avail = sd > 0 ? (u128)sd : 0;  // cpo -| (dp + dpo)
        if (avail < amount) amount = avail;
        if (amount == 0) return TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS;
    }
    if (f & TF_BCR) {
        const u128 avail = sc > 0 ? (u128)sc : 0;
        if (avail < amount) amount = avail;
        if (amount == 0) return TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS;
    }
    if (sum_overflows64(t.ts, (u64)t.timeout * NS_PER_S)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT;
    if ((dr_flags & AF_DNEC) && (i128)amount > sd) return TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS;
    if ((cr_flags & AF_CNED) && (i128)amount > sc) return TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS;
    *amount_out = amount;
    return TBGPU_CREATE_TRANSFER_OK;
}

// What event j's effects look like to a later event of chain csi (execute's scopes,
// src/state_machine.zig:1018-1083): evaluated inside the same open chain, final
// (chain persisted) outside it.
__device__ __forceinline__ bool visible(const TrArgs& C, const EvalState& S, u32 j, u32 csi) {
    if (C.cs[j] == csi) return S.ok[j] & 1;
    return final_ok(C.cs, C.ce, S.cfail, C.ctl, S.ok, j);
}
__device__ __forceinline__ bool fin_ok(const TrArgs& C, const EvalState& S, u32 j) {
    return final_ok(C.cs, C.ce, S.cfail, C.ctl, S.ok, j);
}

// One Jacobi pass: read state S (pass k-1), write state D (pass k).  `chg` counts the
// events whose outcome changed (the next pass's gate), `front` is the first of them
// (everything before it is final: each event depends only on earlier ones).  An
// accepted post/void whose balance effect sits under the wrong side keys (its
// pending resolved to an event with other accounts) asks the host to re-sort.
__device__ __forceinline__ bool write_sides(const TrArgs& C, u32 i, bool pv, bool ok, u32 pref, u128 dpe, u128 dpo,
                                            bool check = true);

// A sparse pass (tr_eval_lists: few events changed in the previous one) checks the
// event's due stamps before anything else, so that an event that is not due costs one
// round of loads, not the event's whole record.
__device__ __forceinline__ bool due_first(const TrArgs& C, const EvalState& S, const EvalState& D, const PassGate& g,
                                          u32 i) {
    const u32 q = g.p, par = q & 1;
    const u32 csi = C.cs[i], cei = C.ce[i];
    bool is_due = C.dt.ev[par * C.dt.n + i] == q;  // (a sparse pass is neither full nor after a rebuild)
    if (!is_due && csi != cei) is_due = C.dt.chain[par * C.dt.n + csi] == q;
    if (!is_due && i == csi && csi != cei) D.cfail[csi] = S.cfail[csi];
    return is_due;
}

// DUE: the pass's dirty check (Dirty) is made here, after the event's own words are
// issued, so that a due event's loads are already in flight when the check resolves
// (SPARSE: the check was made before, by due_first).
template <bool DUE = false, bool SPARSE = false>
__device__ __forceinline__ bool evaluate_one(const Tables& T, const TrArgs& C, const EvalState& S,
                                             const EvalState& D, const Bal4* __restrict__ bb, const PassGate& g,
                                             u32 i) {
    if (SPARSE && !due_first(C, S, D, g, i)) return false;
    // Everything a regular transfer reads is issued up front, unconditionally (the
    // indices are valid for every event; unused values are dropped): one memory
    // round trip for the event's records, one for its two balances.  A post/void's
    // pending references are issued in the same round.
    const u8 sr = C.sres[i];
    const u32 csi = C.cs[i];
    const EvCore k = C.core[i];
    const u32 pid = C.prev_id[i], pre_e = C.pre_e[i];
    const uint2 ep = C.sd.epos[i];
    const u8 s_res = S.res[i];
    const u128 s_amt = S.amt[i], s_pamt = S.pamt[i];
    const u32 s_pref = S.pref[i];
    const u32 pl = C.pend_last[i], pp = C.pre_p[i], pvp = C.prev_pend[i];
    if (DUE && !SPARSE) {
        const u32 cei = C.ce[i], q = g.p, par = q & 1;
        bool is_due = g.full || C.dt.ev[par * C.dt.n + i] == q || *C.dt.all == q;
        if (!is_due && csi != cei) is_due = C.dt.chain[par * C.dt.n + csi] == q;
        if (!is_due) {
            if (i == csi && csi != cei) D.cfail[csi] = S.cfail[csi];
            return false;
        }
    }
    if ((C.probe & 1) && (k.flags & (TF_POST | TF_VOID))) return false;
    Bal4 bd, bc;
    u128 hd = 0, hc = 0;
    if (C.bh64) {
        hd = sext64(C.bh64[ep.x]);
        hc = sext64(C.bh64[ep.y]);
    } else if (C.bh) {
        hd = C.bh[ep.x];
        hc = C.bh[ep.y];
    } else {
        bd = bb[ep.x];
        bc = bb[ep.y];
    }
    u8 res;
    u128 amt = 0, pamt = 0, dpe = 0, dpo = 0;
    u32 pref = NONE32;
    if (sr != SRES_DYN) {
        res = sr;
    } else {
        u32 e = NONE32;
        for (u32 j = pid; j != NONE32; j = C.prev_id[j])
            if (visible(C, S, j, csi)) { e = j; break; }
        if (e == NONE32 && pre_e != NONE32) e = PREF_ROW | pre_e;
        if (!(k.flags & (TF_POST | TF_VOID))) {
            if (e != NONE32) {
                Transfer t = C.ev[i];
                t.timestamp = k.ts;
                res = create_transfer_exists(t, load_ref(T, C, S, e));
            } else if (C.dslot[i] == ROW_FOREIGN || C.cslot[i] == ROW_FOREIGN) {
                // a ledger shard's event with another shard's accounts that is not a
                // repeat: the router never sends one (its rows are not here)
                atomicOr(&C.counters[CNT_FLAGS], (u32)FL_FOREIGN);
                res = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
            } else {
                u128 amount = 0;
                res = (C.bh || C.bh64) ? eval_balances_narrow(k, hd, hc, &amount) : eval_balances(k, bd, bc, &amount);
                if (res == TBGPU_CREATE_TRANSFER_OK) {
                    amt = amount;
                    if (k.flags & TF_PENDING) dpe = amount; else dpo = amount;
                }
            }
        } else {
            // post_or_void_pending_transfer (src/state_machine.zig:1391-1498).  What the
            // likely answers read is issued together: the last earlier event with the
            // pending id (its visibility inputs and its row), the committed pending row,
            // the previous post/void of the same pending -- then the chain words -- instead
            // of a walk of dependent loads.  The walks below stay for the other cases.
            Transfer t = C.ev[i];
            t.timestamp = k.ts;
            const bool pl_v = pl != NONE32, pp_v = pp != NONE32, pvp_v = pvp != NONE32;
            const u32 pl_cs = pl_v ? C.cs[pl] : 0u, pl_ce = pl_v ? C.ce[pl] : 0u;
            const u8 pl_ok = pl_v ? S.ok[pl] : 0;
            const Transfer pl_row = pl_v ? C.ev[pl] : t;
            const u128 pl_amt = pl_v ? S.amt[pl] : 0;
            const u64 pl_ts = pl_v ? C.ts[pl] : 0;
            const Transfer pp_row = pp_v ? T.xrows[pp] : t;
            const u8 pp_ful = pp_v ? T.xful[pp] : 0;
            const u32 pvp_cs = pvp_v ? C.cs[pvp] : 0u, pvp_ce = pvp_v ? C.ce[pvp] : 0u;
            const u8 pvp_ok = pvp_v ? S.ok[pvp] : 0;
            const u16 pvp_fl = pvp_v ? C.core[pvp].flags : 0;
            auto vis = [&](u32 j, u32 js, u32 je, u8 ok) {  // visible() from loaded words
                if (js == csi) return (ok & 1) != 0;
                if (!(ok & 1)) return false;
                if (C.ctl && (C.ctl[je] & TBGPU_CTL_DOOM)) return false;
                return js == je || S.cfail[js] == NONE32;
            };
            u32 p = NONE32;
            if (pl_v && vis(pl, pl_cs, pl_ce, pl_ok)) {
                p = pl;
            } else if (pl_v) {
                for (u32 j = C.prev_id[pl]; j != NONE32; j = C.prev_id[j])
                    if (visible(C, S, j, csi)) { p = j; break; }
            }
            if (p == NONE32 && pp_v) p = PREF_ROW | pp;
            pref = p;
            const bool post = t.flags & TF_POST;
            if (p == NONE32) {
                res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_FOUND;
            } else {
                Transfer P;
                if (p == pl && !(pl_row.flags & (TF_POST | TF_VOID))) {
                    P = pl_row;  // stored_regular
                    P.amount = pl_amt;
                    P.timestamp = pl_ts;
                } else if (p == (PREF_ROW | pp)) {
                    P = pp_row;
                } else {
                    P = load_ref(T, C, S, p);
                }
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
                    if (pvp_v && vis(pvp, pvp_cs, pvp_ce, pvp_ok)) {
                        ful = (pvp_fl & TF_POST) ? 1 : 2;
                    } else if (pvp_v) {
                        for (u32 j = C.prev_pend[pvp]; j != NONE32; j = C.prev_pend[j])
                            if (visible(C, S, j, csi)) { ful = (C.core[j].flags & TF_POST) ? 1 : 2; break; }
                    }
                    if (ful == 0 && (p & PREF_ROW)) ful = (p == (PREF_ROW | pp)) ? pp_ful : T.xful[p & ~PREF_ROW];
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
    if (res != TBGPU_CREATE_TRANSFER_OK && csi != C.ce[i]) {
        if (g.chg) {
            atomicMin(&D.cfail[csi], i);
        } else if (D.cfail[csi] == NONE32 || i < D.cfail[csi]) {
            // the walk (tr_walk, one lane, D == S): a plain store.  An atomic here ran in
            // L2 while the lane's later plain loads of the word (visible(), final_ok)
            // could still hit the CU's L1 copy from before it: a broken chain looked
            // persisted to the events after it.
            D.cfail[csi] = i;
        }
    }
    const bool changed = res != s_res || amt != s_amt || pamt != s_pamt || pref != s_pref;
    if (C.debug && changed) {
        const u16 f = k.flags;
        const u32 kind = (f & (TF_POST | TF_VOID)) ? 2 : (f & (TF_BDR | TF_BCR)) ? 1 : 0;
        atomicAdd(&C.counters[CNT_DBG + kind], 1u);
        if (res != s_res) atomicAdd(&C.counters[CNT_DBG + 3], 1u);
        if (csi != C.ce[i]) atomicAdd(&C.counters[CNT_DBG + 4], 1u);
        if (sr == SRES_DYN && !(f & (TF_POST | TF_VOID)) && (C.core[i].aflags & 0x66))
            atomicAdd(&C.counters[CNT_DBG + 5], 1u);
    }
    // the side records the next pass's balance scan reads: they hold the previous
    // state's (written by the previous pass, or tr_side_rec after a sort), so only an
    // event whose outcome changed rewrites them; static failures keep tr_side_rec's
    if (sr == SRES_DYN && changed && !(C.probe & 2) && !write_sides(C, i, k.flags & (TF_POST | TF_VOID), res == TBGPU_CREATE_TRANSFER_OK,
                                       pref, dpe, dpo))
        atomicMax(&C.counters[CNT_RESORT], g.p + 1);  // its pending is not among its sides: rebuild them
    return changed;
}

// `chg` is a ring word: this pass's count of changed events; the pass clears the
// word the pass after it writes (the host clears nothing per pass).
// `front` (a ring word beside chg): the first event this pass changed.  Every event
// before it is final (each depends only on earlier ones): the walk starts there.
__global__ void tr_evaluate(Tables T, TrArgs C, EvalState S, EvalState D, const Bal4* __restrict__ bb, PassGate g,
                            u32* chg, u32* chg_next, u32* front, u32* front_next) {
    if (!gate_open(g)) return;
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        *chg_next = 0;
        *front_next = NONE32;
    }
    const bool changed = i < C.n && evaluate_one(T, C, S, D, bb, g, i);
    const u32 c = block_sum(changed ? 1u : 0u);
    const u32 f = block_min(changed ? i : NONE32);
    if (threadIdx.x == 0 && c) {
        atomicAdd(chg, c);
        atomicMin(front, f);
    }
}

// The per-pass work lists (TrArgs::lst_simple / lst_complex), in event order within a
// 1024-event block; one cursor atomic per block and list (one per wave was 2.5k
// same-address atomics per 164k-event chunk, serialized at the memory side: 60 us).
__device__ __forceinline__ void init_one(const Tables& T, const TrArgs& C, const EvalState& D, const EvalState& D2,
                                         u32 i);
constexpr u32 LS_THREADS = 1024;
__global__ __launch_bounds__(LS_THREADS) void tr_lists(Tables T, TrArgs C, EvalState D, EvalState D2) {
    __shared__ u32 s_cnt[2][LS_THREADS / 64];
    __shared__ u32 s_base[2];
    const u32 i = blockIdx.x * LS_THREADS + threadIdx.x;
    if (i < C.n) init_one(T, C, D, D2, i);  // the initial state (one launch with the lists)
    u32 cls = 0;  // 0 final after the initial state, 1 simple, 2 complex
    if (i < C.n) {
        const u8 sr = C.sres[i];
        if (sr != SRES_DYN) cls = C.cs[i] != C.ce[i] ? 1 : 0;
        else if (C.core[i].flags & (TF_POST | TF_VOID)) cls = 2;
        else if (C.dslot[i] == ROW_FOREIGN || C.cslot[i] == ROW_FOREIGN) cls = 2;  // can only answer exists*
        else cls = (C.prev_id[i] == NONE32 && C.pre_e[i] == NONE32) ? 1 : 2;
    }
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u64 m[2] = {__ballot(cls == 1), __ballot(cls == 2)};
    if (lane == 0) {
        s_cnt[0][w] = (u32)__popcll(m[0]);
        s_cnt[1][w] = (u32)__popcll(m[1]);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        u32 tot = 0;
        for (u32 k = 0; k < LS_THREADS / 64; k++) tot += s_cnt[threadIdx.x][k];
        s_base[threadIdx.x] = tot ? atomicAdd(&C.counters[threadIdx.x == 0 ? CNT_NSIMPLE : CNT_NCOMPLEX], tot) : 0u;
    }
    __syncthreads();
    if (cls) {
        const u32 k = cls - 1;
        u32 at = s_base[k] + (u32)__popcll(m[k] & ((1ull << lane) - 1));
        for (u32 v = 0; v < w; v++) at += s_cnt[k][v];
        (k == 0 ? C.lst_simple : C.lst_complex)[at] = i;
    }
}

// ------------------------------------------------------- dirty tracking ----
// (engine.h Dirty.)  Whether event i is due at pass q: everything is at a chunk's
// first pass and after a side rebuild; otherwise an event whose balances moved (the
// scan marked it), that changed last pass, whose chain has a member that is, or (the
// scan's resolve step) whose id / pending group moved.
// (evaluated inline by eval_simple_one and evaluate_one<true>, with the event's loads in flight)

// What reads event j's outcome: the scan windows of its sides (every candidate pair of
// a post/void), and the complex events keyed by its id or its pending id (later
// repeats of the id, post/voids naming it, later post/voids of the same pending).
__device__ __forceinline__ void mark_readers(const TrArgs& C, u32 j, u32 par, u32 nq) {
    const u32 tile = C.sd.tile;
    if (is_post_void_ev(C, j)) {
        for (u32 s = C.sd.soff[j]; s < C.sd.soff[j + 1]; s++) C.dt.win[C.sd.spos[s] / tile] = nq;
    } else {
        const uint2 ep = C.sd.epos[j];
        C.dt.win[ep.x / tile] = nq;
        C.dt.win[ep.y / tile] = nq;
    }
    const u32 gs = C.gslot[j], ps = C.pslot[j];
    if (gs != NONE32) C.dt.slot[par * C.dt.g + gs] = nq;
    if (ps != NONE32) C.dt.slot[par * C.dt.g + ps] = nq;
}

// Event i changed at pass q: it is due again at q + 1 (the other state buffer still
// holds its old outcome), and so is everything that reads it.  A chain member's
// change can move the chain's first failure, which every member's visibility and
// sides depend on: the whole chain is due, with its members' readers (marked once per
// chain and pass).
__device__ __forceinline__ void mark_changed(const TrArgs& C, u32 i, u32 q) {
    const u32 nq = q + 1, par = nq & 1;
    C.dt.ev[par * C.dt.n + i] = nq;
    mark_readers(C, i, par, nq);
    const u32 cs = C.cs[i], ce = C.ce[i];
    if (cs != ce && atomicExch(&C.dt.chain[par * C.dt.n + cs], nq) != nq)
        for (u32 j = cs; j <= ce; j++)
            if (j != i) mark_readers(C, j, par, nq);
}

// A pass over the simple list: create_transfer's balance tail (src/state_machine.zig:
// 1286-1322) for transfers whose id nothing before them holds, and the static failures
// inside chains (they break their chain every pass).  What evaluate_one does for them,
// without its post/void and `exists` work (most of a pass's events are here).
template <bool SPARSE>
__device__ __forceinline__ bool eval_simple_one(const TrArgs& C, const EvalState& S, const EvalState& D,
                                                const Bal4* __restrict__ bb, const PassGate& g, u32 i) {
    // The event's own words and its due stamp in one round of loads (most events are
    // due in the early passes, which dominate), the chain stamp and the balances in a
    // second: two memory round trips before the evaluation instead of four.  A sparse
    // pass checks the stamps first (due_first).
    if (SPARSE && !due_first(C, S, D, g, i)) return false;
    const u32 q = g.p, par = q & 1;
    const u8 sr = C.sres[i];
    const u32 csi = C.cs[i], cei = C.ce[i];
    const u32 dte = (g.full || SPARSE) ? q : C.dt.ev[par * C.dt.n + i];
    const EvCore e = C.core[i];
    const uint2 ep = C.sd.epos[i];
    const u8 s_res = S.res[i];
    const u128 s_amt = S.amt[i];
    if (!SPARSE) {
        bool is_due = g.full || dte == q || *C.dt.all == q;
        if (!is_due && csi != cei) is_due = C.dt.chain[par * C.dt.n + csi] == q;
        if (!is_due) {
            // outcome unchanged in both buffers; a chain nobody re-evaluates keeps its
            // first failure (the scan reset the next state's)
            if (i == csi && csi != cei) D.cfail[csi] = S.cfail[csi];
            return false;
        }
    }
    // (pamt and pref of a simple event are zero / none in both buffers after tr_init and
    // pass 0: later passes leave them)
    if (sr != SRES_DYN) {  // a static failure inside a chain
        D.res[i] = sr;
        D.ok[i] = 0;
        D.amt[i] = 0;
        if (q == 0) {
            D.pamt[i] = 0;
            D.pref[i] = NONE32;
        }
        atomicMin(&D.cfail[csi], i);
        return false;
    }
    u128 amount = 0;
    u8 res;
    if (C.bh64) {
        res = eval_balances_narrow(e, sext64(C.bh64[ep.x]), sext64(C.bh64[ep.y]), &amount);
    } else if (C.bh) {
        res = eval_balances_narrow(e, C.bh[ep.x], C.bh[ep.y], &amount);
    } else {
        const Bal4 bd = bb[ep.x], bc = bb[ep.y];
        res = eval_balances(e, bd, bc, &amount);
    }
    const bool ok = res == TBGPU_CREATE_TRANSFER_OK;
    const u128 amt = ok ? amount : 0;
    D.res[i] = res;
    D.ok[i] = ok ? 1 : 0;
    D.amt[i] = amt;
    if (q == 0) {
        D.pamt[i] = 0;
        D.pref[i] = NONE32;
    }
    if (!ok && csi != cei) atomicMin(&D.cfail[csi], i);
    const bool changed = res != s_res || amt != s_amt;
    if (changed) {
        const u128 dpe = ok && (e.flags & TF_PENDING) ? amt : 0, dpo = ok && !(e.flags & TF_PENDING) ? amt : 0;
        C.sd.sq_ok[ep.x] = C.sd.sq_ok[ep.y] = ok ? 1 : 0;
        side_deltas_put(C.sd, ep.x, dpe, dpo);
        side_deltas_put(C.sd, ep.y, dpe, dpo);
        mark_changed(C, i, q);
    }
    return changed;
}

// evaluate_one over the complex list
template <bool SPARSE>
__device__ __forceinline__ bool eval_complex_one(const Tables& T, const TrArgs& C, const EvalState& S,
                                                 const EvalState& D, const Bal4* __restrict__ bb, const PassGate& g,
                                                 u32 k, u32& i) {
    i = C.lst_complex[k];
    const bool changed = evaluate_one<true, SPARSE>(T, C, S, D, bb, g, i);
    if (changed) mark_changed(C, i, g.p);
    return changed;
}

// One pass's evaluation of both work lists in one launch: the first `nbc` workgroups
// take the complex list (dispatched first: their events are the longer dependent-load
// chains), the rest the simple list.  Two launches ran the lists one after the other;
// here the complex list's latency hides under the simple list's work.
#ifndef TR_EV_THREADS
#define TR_EV_THREADS 256
#endif
constexpr u32 EV_THREADS = TR_EV_THREADS;
__global__ __launch_bounds__(EV_THREADS) void tr_eval_lists(Tables T, TrArgs C, EvalState S, EvalState D,
                                                            const Bal4* __restrict__ bb, PassGate g, u32 n_simple,
                                                            u32 n_complex, u32 nbc, u32* chg, u32* chg_next,
                                                            u32* front, u32* front_next) {
    if (!gate_open(g)) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *chg_next = 0;
        *front_next = NONE32;
    }
    // sparse: the previous pass changed few events, so few are due (uniform)
    const bool sparse = C.sparse && !g.full && *C.dt.all != g.p && *g.chg < ((n_simple + n_complex) >> C.sparse);
    bool changed = false;
    u32 i = NONE32;
    if (blockIdx.x < nbc) {
        const u32 k = blockIdx.x * EV_THREADS + threadIdx.x;
        if (k < n_complex)
            changed = sparse ? eval_complex_one<true>(T, C, S, D, bb, g, k, i)
                             : eval_complex_one<false>(T, C, S, D, bb, g, k, i);
    } else {
        const u32 k = (blockIdx.x - nbc) * EV_THREADS + threadIdx.x;
        if (k < n_simple) {
            i = C.lst_simple[k];
            changed = sparse ? eval_simple_one<true>(C, S, D, bb, g, i) : eval_simple_one<false>(C, S, D, bb, g, i);
        }
    }
    const u32 c = block_sum(changed ? 1u : 0u);
    const u32 f = block_min(changed ? i : NONE32);
    if (threadIdx.x == 0 && c) {
        // (one of ~960 workgroups' two same-address atomics at the end of an early pass:
        // measured free, profiles/r06/ab_pass_atomics_config3.txt)
        atomicAdd(chg, c);
        atomicMin(front, f);
    }
}

// The pending an unresolved post/void most likely resolves to: a committed transfer
// with that id, else the first earlier event with that id (a later one repeats
// its id and fails with `exists` unless the first one fails).
__device__ __forceinline__ u32 pending_guess(const TrArgs& C, u32 i) {
    if (C.pre_p[i] != NONE32) return PREF_ROW | C.pre_p[i];
    return C.pend_first[i];
}

// Starting point: every statically valid event succeeds, except that an id already
// committed, or seen earlier in the call, answers `exists` (the first event with an
// id is the one that succeeds), and a post/void resolves to its likeliest pending.
__device__ __forceinline__ void init_one(const Tables& T, const TrArgs& C, const EvalState& D, const EvalState& D2,
                                         u32 i) {
    if (C.sres[i] != SRES_DYN && C.cs[i] == C.ce[i]) {
        // a static failure outside any chain: final, on no work list; both state
        // buffers hold it for every pass
        for (const EvalState* E : {&D, &D2}) {
            E->res[i] = C.sres[i];
            E->ok[i] = 0;
            E->amt[i] = 0;
            E->pamt[i] = 0;
            E->pref[i] = NONE32;
        }
        return;
    }
    u8 sr = C.sres[i];
    if (sr == SRES_DYN && (C.prev_id[i] != NONE32 || C.pre_e[i] != NONE32)) sr = TBGPU_CREATE_TRANSFER_EXISTS;
    u8 res = sr;
    u128 amt = 0, pamt = 0;
    u32 pref = NONE32;
    if (sr == SRES_DYN) {
        const Transfer& t = C.ev[i];
        if (!(t.flags & (TF_POST | TF_VOID))) {
            res = 0;
            amt = t.amount;
            if ((t.flags & (TF_BDR | TF_BCR)) && amt == 0) amt = (u128)0xFFFFFFFFFFFFFFFFull;
        } else {
            pref = pending_guess(C, i);
            if (pref == NONE32) {
                res = TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_FOUND;
            } else {
                res = 0;
                pamt = (pref & PREF_ROW) ? T.xrows[pref & ~PREF_ROW].amount : C.ev[pref].amount;
                amt = t.amount > 0 ? t.amount : pamt;
            }
        }
    }
    D.res[i] = res;
    D.ok[i] = res == 0 ? 1 : 0;
    D.amt[i] = amt;
    D.pamt[i] = pamt;
    D.pref[i] = pref;
    if (res != 0 && C.cs[i] != C.ce[i]) atomicMin(&D.cfail[C.cs[i]], i);
}

// An accepted event's balance deltas (pending, posted) from its state: a transfer
// adds its amount to the pending or posted balances (src/state_machine.zig:1330-1340);
// a post/void releases the pending amount and a post adds the posted amount
// (:1470-1486).  Two's complement: a void or post is a subtraction.
__device__ __forceinline__ void state_deltas(const TrArgs& C, const EvalState& S, u32 i, u128* dpe, u128* dpo) {
    *dpe = *dpo = 0;
    if (!(S.ok[i] & 1)) return;
    const u16 f = C.core[i].flags;
    if (f & (TF_POST | TF_VOID)) {
        *dpe = (u128)0 - S.pamt[i];
        *dpo = (f & TF_POST) ? S.amt[i] : 0;
    } else if (f & TF_PENDING) {
        *dpe = S.amt[i];
    } else {
        *dpo = S.amt[i];
    }
}

// ------------------------------------------------------------------ sides ----
// The candidate pendings of post/void i (pref encoding), at most kmax, distinct:
// the one it resolved to in state S, a committed transfer with that id, then the
// earlier events of the call with that id from the first (the first is the one
// that succeeds unless it fails; a later one repeats its id).  The evaluation
// resolves to the last visible such event, else the committed one
// (src/state_machine.zig:1409-1428): when that is not among these, the host
// rebuilds the sides with it (PassGate.resort).
__device__ __forceinline__ u32 post_candidates(const TrArgs& C, const EvalState& S, u32 i, u32 kmax, u32* out) {
    u32 k = 0;
    auto add = [&](u32 v) {
        if (v == NONE32 || k >= kmax) return;
        for (u32 j = 0; j < k; j++)
            if (out[j] == v) return;
        out[k++] = v;
    };
    add(S.pref[i]);
    if (C.pre_p[i] != NONE32) add(PREF_ROW | C.pre_p[i]);
    const u32 p = C.pslot[i];
    if (p != NONE32) {
        const u32 cnt = C.gcnt_id[p];
        if (cnt == 1) {
            const u32 j = C.gmem[p];
            if (j < i) add(j);
        } else if (cnt > 1) {
            for (u32 q = C.gbeg[p]; q < C.gend[p] && k < kmax; q++) {
                const u32 j = C.gmembers[q];
                if (j >= i) break;
                add(j);
            }
        }
    }
    return k;
}

__device__ __forceinline__ bool is_post_void(const TrArgs& C, u32 i) {
    return C.sres[i] == SRES_DYN && (C.core[i].flags & (TF_POST | TF_VOID));
}

// Side pairs per event, as a popcount mask for scan3: 1 -> 0b001, 2 -> 0b011, 3 -> 0b111.
// An upper bound of post_candidates' count that classify's results alone decide (every
// candidate is the committed pending or an earlier event with the pending id, whatever
// the state), so the count and its round trip run before the grouping and the initial
// state, and overlap them; tr_side_build pads a post/void's unused pairs with inert keys.
// (In practice the bound is the count: a pending id is rarely repeated.)
__global__ void tr_side_count(TrArgs C, u32 kmax, u8* mask) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    u32 pairs = 1;
    if (is_post_void(C, i)) {
        const u32 p = C.pslot[i];
        const u32 k = (C.pre_p[i] != NONE32 ? 1u : 0u) + (p != NONE32 ? C.gcnt_id[p] : 0u);
        pairs = max(1u, min(kmax, k));
    }
    mask[i] = (u8)((1u << pairs) - 1);
}

// The account slots of a candidate pending (a committed row's were probed by classify).
__device__ __forceinline__ void cand_slots(const TrArgs& C, u32 i, u32 cand, u32* d, u32* c) {
    if (cand == NONE32) { *d = *c = NONE32; return; }
    if (cand & PREF_ROW) { *d = C.pp_dslot[i]; *c = C.pp_cslot[i]; return; }
    *d = C.dslot[cand];
    *c = C.cslot[cand];
}

// Every input is loaded into registers before the first store: the stores go through
// TrArgs pointers the compiler must assume alias the inputs, so a load issued after a
// store waited for its own round trip (three dependent trips per candidate pair: 33 us
// per 164k-event chunk).
__global__ void tr_side_build(TrArgs C, EvalState S, u32 kmax, const uint4* pairs, u32 invalid, u32* skey, u32* sval) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 tot = pairs[C.n];
    const bool ev = i < C.n;
    const uint4 pr = i <= C.n ? pairs[i] : make_uint4(0, 0, 0, 0);
    const uint4 pr1 = ev ? pairs[i + 1] : make_uint4(0, 0, 0, 0);
    const u8 sr = ev ? C.sres[i] : 0;
    const u16 fl = ev ? C.core[i].flags : 0;
    const u8 af = ev ? C.core[i].aflags : 0;
    const u32 ds = ev ? C.dslot[i] : NONE32, cs = ev ? C.cslot[i] : NONE32;
    const u32 pd = ev ? C.pp_dslot[i] : NONE32, pc = ev ? C.pp_cslot[i] : NONE32;
    const u32 ecs = ev ? C.cs[i] : 0u, ece = ev ? C.ce[i] : 0u;
    const bool pv = sr == SRES_DYN && (fl & (TF_POST | TF_VOID));
    u32 cand[SIDE_CANDS], cd[SIDE_CANDS], cc[SIDE_CANDS];
    u32 k = 1;
    cand[0] = NONE32;  // (a post/void without candidates keeps one inert pair)
    if (pv) k = max(1u, post_candidates(C, S, i, kmax, cand));
#pragma unroll
    for (u32 j = 0; j < SIDE_CANDS; j++) {  // the candidates' account slots, issued together
        cd[j] = cc[j] = NONE32;
        if (pv && j < k && cand[j] != NONE32) {
            if (cand[j] & PREF_ROW) { cd[j] = pd; cc[j] = pc; }
            else { cd[j] = C.dslot[cand[j]]; cc[j] = C.cslot[cand[j]]; }
        }
    }
    {
        // the fused scan's window words start empty (tr_side_pos lowers tstart, the
        // passes stamp win): cleared here rather than by two fills of their own
        const u64 m = 2ull * (tot.x + tot.y + tot.z), nwin = (m + C.sd.tile - 1) / C.sd.tile + 1;
        for (u64 q = i; q < nwin; q += (u64)gridDim.x * blockDim.x) {
            C.sd.tstart[q] = NONE32;
            C.dt.win[q] = NONE32;
        }
    }
    if (i > C.n) return;
    const u32 s0 = 2 * (pr.x + pr.y + pr.z);
    C.sd.soff[i] = s0;
    if (i == C.n) return;
    // the sorted chain word of every side of the event (tr_side_pos copies it in order)
    const bool doom = C.ctl && (C.ctl[ece] & TBGPU_CTL_DOOM);
    const u32 cw = ecs | (ecs == ece ? SQ_STANDALONE : 0u) | (doom ? SQ_DOOM : 0u);
    const u32 slots = (2 * (pr1.x + pr1.y + pr1.z) - s0) / 2;  // tr_side_count's bound
    if (k > slots) {  // (the bound holds by construction: a broken one is a device error)
        atomicOr(&C.counters[CNT_FLAGS], (u32)FL_ERROR);
        k = slots;
    }
#pragma unroll
    for (u32 j = 0; j < SIDE_CANDS; j++) {
        if (j >= slots) break;
        u32 d = NONE32, c = NONE32;
        if (j < k) {
            if (pv) { d = cd[j]; c = cc[j]; }
            else if (sr == SRES_DYN) { d = ds; c = cs; }
        }  // else padding: an inert pair that no resolution names
        if (d == NONE32 || c == NONE32 || d == ROW_FOREIGN || c == ROW_FOREIGN) d = c = invalid;
        const u32 s = s0 + 2 * j;
        skey[s] = d;
        skey[s + 1] = c;
        sval[s] = s;
        sval[s + 1] = s + 1;
        // (a regular transfer's own sides: whether their balance decides its outcome)
        const bool reg = !pv && sr == SRES_DYN && d != invalid;
        const bool sd = reg && ((af & AF_DNEC) || (fl & TF_BDR));
        const bool sc = reg && (((af >> 4) & AF_CNED) || (fl & TF_BCR));
        const u32 first = j == 0 ? SQ_FIRST : 0u;
        C.sd.sev[s] = i | first | (sd ? SQ_SENS : 0u);
        C.sd.sev[s + 1] = i | first | (1u << 31) | (sc ? SQ_SENS : 0u);
        C.sd.scs[s] = C.sd.scs[s + 1] = cw;
        C.sd.scand[s] = C.sd.scand[s + 1] = (pv && j < k) ? cand[j] : NONE32;
    }
}

// Sorted positions and the static per-side information in sorted order.
__global__ void tr_side_pos(TrArgs C, const u32* sval_s, u64 m) {
    const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    // account starts, for the fused scan's windows (inert sides each stand alone):
    // the wave's first start, one atomic per wave (a tile spans whole waves)
    u32 start = NONE32;
    if (q < m) {
        const u32 key = C.sd.skey_s[q];
        if (q == 0 || key != C.sd.skey_s[q - 1] || key == C.sd.inert) start = (u32)q;
    }
    start = wave_min(start);
    if (start != NONE32 && q == start) atomicMin(&C.sd.tstart[q / C.sd.tile], start);
    if (q >= m) return;
    // loads before stores (they may alias for the compiler: see tr_side_build); the
    // side's words were written by tr_side_build in unsorted order (two gathers here
    // instead of the event's offset, chain bounds and control byte)
    const u32 s = sval_s[q];
    const u32 ev = C.sd.sev[s], cw = C.sd.scs[s];
    C.sd.spos[s] = (u32)q;
    C.sd.sq_ev[q] = ev;
    if (ev & SQ_FIRST) ((u32*)&C.sd.epos[ev & SQ_EV])[ev >> 31] = (u32)q;
    C.sd.sq_cs[q] = cw;
}

// Write event i's side records (sorted order) for its outcome: the debit and credit
// sides of a transfer, or of the candidate pair of a post/void that it resolved to.
// Returns false when an accepted post/void's pending is not among its candidates.
__device__ __forceinline__ bool write_sides(const TrArgs& C, u32 i, bool pv, bool ok, u32 pref, u128 dpe, u128 dpo,
                                            bool check) {
    if (!pv) {  // one side pair
        const uint2 ep = C.sd.epos[i];
        C.sd.sq_ok[ep.x] = C.sd.sq_ok[ep.y] = ok ? 1 : 0;
        side_deltas_put(C.sd, ep.x, ok ? dpe : 0, ok ? dpo : 0, check);
        side_deltas_put(C.sd, ep.y, ok ? dpe : 0, ok ? dpo : 0, check);
        return true;
    }
    const u32 s0 = C.sd.soff[i], s1 = C.sd.soff[i + 1];
    bool found = !pv || !ok;
    for (u32 s = s0; s < s1; s += 2) {
        const bool act = ok && (!pv || C.sd.scand[s] == pref);
        found |= pv && act;
        const u32 q0 = C.sd.spos[s], q1 = C.sd.spos[s + 1];
        C.sd.sq_ok[q0] = C.sd.sq_ok[q1] = act ? 1 : 0;
        side_deltas_put(C.sd, q0, act ? dpe : 0, act ? dpo : 0, check);
        side_deltas_put(C.sd, q1, act ? dpe : 0, act ? dpo : 0, check);
    }
    return found;
}

__global__ void tr_side_rec(TrArgs C, EvalState S) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    u128 dpe, dpo;
    state_deltas(C, S, i, &dpe, &dpo);
    write_sides(C, i, is_post_void(C, i), S.ok[i] & 1, S.pref[i], dpe, dpo, /*check=*/false);
}

// ---------------------------------------------------------------- apply ----

// Final result per event, as execute emits it (src/state_machine.zig:1051-1072).
__device__ __forceinline__ bool epi_closed(const TrArgs& C) { return C.epi && *C.epi == 0; }
// the gated kernels' converged state: the argument, or epi_alt
__device__ __forceinline__ bool epi_state(const TrArgs& C, EvalState& S) {
    if (!C.epi) return true;
    const u32 e = *C.epi;
    if (e == 2) S = C.epi_alt;
    return e != 0;
}

__global__ void tr_mask(Tables T, TrArgs C, EvalState S, u8* fres, u8* mask) {
    if (!epi_state(C, S)) return;
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
    const bool ok = fin_ok(C, S, i);
    bool hist = false;
    if (ok && !(C.core[i].flags & (TF_POST | TF_VOID)))
        hist = C.core[i].aflags & (AF_HISTORY | AF_HISTORY << 4);
    fres[i] = r;
    mask[i] = (ok ? 1 : 0) | (r != 0 ? 2 : 0) | (hist ? 4 : 0);
}

// Rows, replies and history rows go after the device-side cursors T.base (the
// previous chunks' and calls' output), so chunks follow each other without a host
// round trip.  A call that would overflow a table writes nothing and raises
// FL_ERROR (the host aborts, as the reference asserts).
__global__ void tr_apply(Tables T, TrArgs C, EvalState S, const u8* __restrict__ fres, const uint4* __restrict__ rk,
                         const Bal4* __restrict__ bb, tbgpu_create_transfers_result_t* __restrict__ results) {
    if (!epi_state(C, S)) return;
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u64 row_base = T.base[BASE_ROWS], hist_base = T.base[BASE_HIST];
    const uint4 tot = rk[C.n];
    if (!C.dry && (row_base + tot.x > T.xrow_cap || hist_base + tot.z > T.hist_cap)) {
        if (i == 0) {
            atomicOr(&C.counters[CNT_FLAGS], (u32)FL_ERROR);
            atomicOr(&C.counters[CNT_STICKY], (u32)FL_ERROR);
        }
        return;
    }
    const u8 r = fres[i];
    const uint4 q = rk[i];
    if (r != 0) {
        // replies of consecutive batches are concatenated: global non-ok rank
        const u32 b = batch_of(C.b_start, C.nb, i);
        results[T.base[BASE_REPLIES] + q.y] = {i - C.b_start[b], (u32)r};
        return;
    }
    if (C.dry || !fin_ok(C, S, i)) return;
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
        if (C.dslot[i] == ROW_FOREIGN || C.cslot[i] == ROW_FOREIGN) {  // (never: evaluate_one flagged it)
            atomicOr(&C.counters[CNT_FLAGS], (u32)FL_FOREIGN);
            atomicOr(&C.counters[CNT_STICKY], (u32)FL_FOREIGN);
            return;
        }
        // the accounts' history flags are in the event's core (classify): the rows are
        // read only for a history row
        const u8 af = C.core[i].aflags;
        if ((af | (af >> 4)) & AF_HISTORY) {
            const Account& dra = T.acc[C.dslot[i]];
            const Account& cra = T.acc[C.cslot[i]];
            // balances after this transfer (src/state_machine.zig:1342-1364)
            const u32 s0 = C.sd.soff[i];
            Bal4 d = bb[C.sd.spos[s0]], c = bb[C.sd.spos[s0 + 1]];
            u128 dpe, dpo;
            state_deltas(C, S, i, &dpe, &dpo);
            d.dp += dpe; d.dpo += dpo;
            c.cp += dpe; c.cpo += dpo;
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

// Per 1024-event block: the componentwise key range of the stored ids (for the
// index's range filter) and the largest timestamp that advances commit_timestamp.
// commit_timestamp is a plain field, not undone by scope_close(.discard): every
// create_transfer that returned ok before its chain broke advanced it (:1366).
// tr_advance folds the blocks' records (no global atomics here: every block on
// the same five words would serialize).
constexpr int RG_THREADS = 1024;
__global__ __launch_bounds__(RG_THREADS) void tr_range(Tables T, TrArgs C, EvalState S, u64* part) {
    if (!epi_state(C, S)) return;
    __shared__ u64 sh[RG_THREADS / 64][5];
    const u32 i = blockIdx.x * RG_THREADS + threadIdx.x;
    const bool valid = i < C.n;
    const bool ok = valid && fin_ok(C, S, i);
    u64 mts = 0;
    if (valid && (S.ok[i] & 1)) {
        const u32 cs = C.cs[i];
        const bool doom = C.ctl && (C.ctl[C.ce[i]] & TBGPU_CTL_DOOM);
        u32 cf = (cs != C.ce[i] || doom) ? S.cfail[cs] : NONE32;
        if (cf == NONE32 && doom) cf = C.ce[i] + 1;
        if (cf == NONE32 || i < cf) mts = C.ts[i];
    }
    const u128 id = ok ? C.ev[i].id : 0;
    u64 r[5] = {ok ? (u64)id : 0, ok ? (u64)(id >> 64) : 0, ok ? (u64)id : ~0ull, ok ? (u64)(id >> 64) : ~0ull, mts};
    for (int off = 32; off > 0; off >>= 1) {
        r[0] = max(r[0], (u64)__shfl_xor((unsigned long long)r[0], off));
        r[1] = max(r[1], (u64)__shfl_xor((unsigned long long)r[1], off));
        r[2] = min(r[2], (u64)__shfl_xor((unsigned long long)r[2], off));
        r[3] = min(r[3], (u64)__shfl_xor((unsigned long long)r[3], off));
        r[4] = max(r[4], (u64)__shfl_xor((unsigned long long)r[4], off));
    }
    const u32 w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 5; k++) sh[w][k] = r[k];
    __syncthreads();
    if (threadIdx.x < 5) {
        const int k = threadIdx.x;
        u64 v = sh[0][k];
        for (int q = 1; q < RG_THREADS / 64; q++) v = (k == 2 || k == 3) ? min(v, sh[q][k]) : max(v, sh[q][k]);
        part[(u64)blockIdx.x * 8 + k] = v;
    }
}

__global__ void batch_counts(const u32* b_start, u32 nb, const uint4* rk, u32* counts, const u32* epi) {
    if (epi && *epi == 0) return;
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) counts[b] = rk[b_start[b + 1]].y - rk[b_start[b]].y;
}

// Fold tr_range's block records into the index key range and commit_timestamp, and
// advance the device cursors by the chunk's stored rows, replies and history rows.
__global__ __launch_bounds__(256) void tr_advance(Tables T, TrArgs C, const uint4* rk, const u64* part, u32 nparts) {
    if (epi_closed(C)) return;
    if (C.counters[CNT_FLAGS] & FL_ERROR) return;
    u64 r[5] = {0, 0, ~0ull, ~0ull, 0};
    for (u32 b = threadIdx.x; b < nparts; b += 256) {
        r[0] = max(r[0], part[b * 8 + 0]);
        r[1] = max(r[1], part[b * 8 + 1]);
        r[2] = min(r[2], part[b * 8 + 2]);
        r[3] = min(r[3], part[b * 8 + 3]);
        r[4] = max(r[4], part[b * 8 + 4]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        r[0] = max(r[0], (u64)__shfl_xor((unsigned long long)r[0], off));
        r[1] = max(r[1], (u64)__shfl_xor((unsigned long long)r[1], off));
        r[2] = min(r[2], (u64)__shfl_xor((unsigned long long)r[2], off));
        r[3] = min(r[3], (u64)__shfl_xor((unsigned long long)r[3], off));
        r[4] = max(r[4], (u64)__shfl_xor((unsigned long long)r[4], off));
    }
    if ((threadIdx.x & 63) == 0) {
        if (r[4]) atomicMax((unsigned long long*)C.commit_ts, (unsigned long long)r[4]);
        if (!C.dry && (r[0] | r[1] | ~r[2] | ~r[3])) {
            atomicMax((unsigned long long*)&T.idr[0], (unsigned long long)r[0]);
            atomicMax((unsigned long long*)&T.idr[1], (unsigned long long)r[1]);
            atomicMin((unsigned long long*)&T.idr[2], (unsigned long long)r[2]);
            atomicMin((unsigned long long*)&T.idr[3], (unsigned long long)r[3]);
        }
    }
    if (threadIdx.x != 0) return;
    const uint4 tot = rk[C.n];
    T.base[BASE_REPLIES] += tot.y;
    if (C.dry) return;
    T.base[BASE_ROWS] += tot.x;
    T.base[BASE_HIST] += tot.z;
}

// ------------------------------------------------------------- walker ----
// The fixed point's bounded worst case.  Its passes grow with a chunk's dependency
// depth, at most n + 1: an 8190-event batch in which every event's outcome decides
// the next one's takes 8190 passes, O(n^2) work where the reference's execute is
// O(n) (src/state_machine.zig:1018-1083).  Past a pass budget the engine walks the
// events from the front on -- the chain start of the first event the last pass
// changed; every event before it is final -- in execute's own order, in one thread:
// each account's balance as the walk has moved it, linked chains opened and closed
// as scopes (src/state_machine.zig:972-1000: a broken chain's balance moves are
// undone), every event evaluated by evaluate_one against a state whose predecessors
// are all final.  The walk leaves exactly the state the passes converge to, side
// records included, and the same apply kernels commit it.

// Before the walk: the side records of the walked events zeroed (the scan that
// follows then gives every side the balance of the events before the front alone),
// each side's account segment start (a binary search over the sorted keys), and the
// walked chains' first failures reset.
__global__ void tr_walk_prep(TrArgs C, u64 m, u32 start, u32* sstart, u32* cfail) {
    const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < m) {
        const u32 ev = C.sd.sq_ev[q] & SQ_EV;
        if (ev >= start) {
            C.sd.sq_ok[q] = 0;
            side_deltas_put(C.sd, q, 0, 0);
        }
        const u32 key = C.sd.skey_s[q];
        u64 lo = 0, hi = q;  // first position with this key
        if (key >= C.sd.inert) lo = q;
        while (lo < hi) {
            const u64 mid = (lo + hi) / 2;
            if (C.sd.skey_s[mid] < key) lo = mid + 1; else hi = mid;
        }
        sstart[q] = (u32)lo;
    }
    if (q >= start && q < C.n) cfail[q] = NONE32;
}

// After the scan: each account's balance before the walked events, at its segment
// start -- the scanned balance of its first side that belongs to a walked event
// (every earlier side is final; the walked sides' records are zero).
__global__ void tr_walk_init(TrArgs C, u64 m, u32 start, const u32* sstart, const Bal4* bb, Bal4* wbal) {
    const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= m) return;
    if ((C.sd.sq_ev[q] & SQ_EV) < start) return;
    const u32 s0 = sstart[q];
    if (q == s0 || (C.sd.sq_ev[q - 1] & SQ_EV) < start) wbal[s0] = bb[q];
}

struct WalkArgs {
    const u32* sstart;  // [m] first side of each side's account segment
    Bal4* wbal;         // [m] per segment start: the account's balance as the walk has moved it
    u32* undo_slot;     // the open chain's balance moves, for its rollback
    Bal4* undo_val;
    u32 undo_cap;
    u32 start;          // the first walked event (a chain start)
    u32* out;           // [0] resume point when the walk stopped early (NONE32: walked to the end), [1] error
};

// What the walk reads of an event, staged 64 events at a time by the whole wave so
// that the walking lane meets no memory latency but the balances'.
struct WalkRec {
    EvCore core;
    uint2 ep;
    u32 cs, ce, pid, pre_e, s0d, s0c;
    u8 sr, pad[7];
};
constexpr int WK_CACHE = 64;  // recently moved balances, direct-mapped by segment start

// The walk's balances: written by the walking lane, read back by it and (staged) by
// the wave's other lanes after the workgroup barrier -- plain accesses, which the
// barrier orders within the workgroup (one CU, one L1).  (L1-bypassing loads read L2
// before the walking lane's write-through stores had reached it.)
__device__ __forceinline__ Bal4 wk_load(const Bal4* p) { return *p; }

__global__ __launch_bounds__(64) void tr_walk(Tables T, TrArgs C, EvalState D, Bal4* bb, WalkArgs W) {
    __shared__ WalkRec rec[64];
    __shared__ Bal4 pre[64][2];          // the staged balances of each event's two sides
    __shared__ u32 ctag[WK_CACHE];
    __shared__ Bal4 cval[WK_CACHE];
    __shared__ u32 s_stop;
    const u32 lane = threadIdx.x;
    const PassGate G{nullptr, nullptr, 0, 1};
    u32 undo_n = 0;
    bool broken = false;
    if (lane == 0) {
        W.out[0] = NONE32;
        W.out[1] = 0;  // the error word: the buffer is not cleared anywhere else (recycled memory)
        s_stop = 0;
    }
    // a per-block bitmap of the segments moved in this block: their staged balances are stale
    u64 moved[16];
    for (u32 b0 = W.start; b0 < C.n; b0 += 64) {
        {  // stage the block's events
            const u32 i = b0 + lane;
            if (i < C.n) {
                WalkRec r;
                r.core = C.core[i];
                r.ep = C.sd.epos[i];
                r.cs = C.cs[i];
                r.ce = C.ce[i];
                r.pid = C.prev_id[i];
                r.pre_e = C.pre_e[i];
                r.sr = C.sres[i];
                r.s0d = W.sstart[r.ep.x];
                r.s0c = W.sstart[r.ep.y];
                rec[lane] = r;
                if (r.sr == SRES_DYN && !(r.core.flags & (TF_POST | TF_VOID))) {
                    pre[lane][0] = wk_load(&W.wbal[r.s0d]);
                    pre[lane][1] = wk_load(&W.wbal[r.s0c]);
                }
            }
            if (b0 == W.start) ctag[lane] = NONE32;
        }
        __syncthreads();
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 16; k++) moved[k] = 0;
            auto read_bal = [&](u32 s0, u32 k, int side) -> Bal4 {
                const u32 c = s0 % WK_CACHE;
                if (ctag[c] == s0) return cval[c];
                if (moved[(s0 >> 6) & 15] >> (s0 & 63) & 1) return wk_load(&W.wbal[s0]);
                return pre[k][side];
            };
            auto write_bal = [&](u32 s0, const Bal4& v) {
                const u32 c = s0 % WK_CACHE;
                ctag[c] = s0;
                cval[c] = v;
                moved[(s0 >> 6) & 15] |= 1ull << (s0 & 63);
                W.wbal[s0] = v;  // write-through: an evicted segment is read back from memory
            };
            auto move = [&](u32 s0, const Bal4& old, bool chain, const Bal4& nv) -> bool {
                if (chain) {  // the scope's undo log
                    if (undo_n + 1 > W.undo_cap) return false;
                    W.undo_slot[undo_n] = s0;
                    W.undo_val[undo_n++] = old;
                }
                write_bal(s0, nv);
                return true;
            };
            const u32 kn = min(64u, C.n - b0);
            for (u32 k = 0; k < kn; k++) {
                const u32 i = b0 + k;
                const WalkRec& R = rec[k];
                const bool chain = R.cs != R.ce;
                if (chain && i == R.cs) {  // scope_open (:1022-1026)
                    undo_n = 0;
                    broken = false;
                }
                const bool pv = R.sr == SRES_DYN && (R.core.flags & (TF_POST | TF_VOID));
                if (chain && broken) {
                    // execute evaluates nothing after the break: linked_event_failed (tr_mask)
                    D.res[i] = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
                    D.ok[i] = 0;
                    D.amt[i] = 0;
                    D.pamt[i] = 0;
                    D.pref[i] = NONE32;
                } else if (R.sr == SRES_DYN && !pv && R.pid == NONE32 && R.pre_e == NONE32 &&
                           C.dslot[i] != ROW_FOREIGN && C.cslot[i] != ROW_FOREIGN) {
                    // a transfer whose id nothing before it holds: create_transfer's balance tail
                    const Bal4 bd = read_bal(R.s0d, k, 0), bc = read_bal(R.s0c, k, 1);
                    bb[R.ep.x] = bd;  // the balances it saw (history rows, tr_apply)
                    bb[R.ep.y] = bc;
                    u128 amount = 0;
                    const u8 res = eval_balances(R.core, bd, bc, &amount);
                    const bool ok = res == TBGPU_CREATE_TRANSFER_OK;
                    D.res[i] = res;
                    D.ok[i] = ok ? 1 : 0;
                    D.amt[i] = ok ? amount : 0;
                    D.pamt[i] = 0;
                    D.pref[i] = NONE32;
                    const u128 dpe = ok && (R.core.flags & TF_PENDING) ? amount : 0;
                    const u128 dpo = ok && !(R.core.flags & TF_PENDING) ? amount : 0;
                    write_sides(C, i, false, ok, NONE32, dpe, dpo);
                    if (ok) {
                        Bal4 nd = bd, nc = bc;
                        nd.dp += dpe; nd.dpo += dpo;
                        nc.cp += dpe; nc.cpo += dpo;
                        if (!move(R.s0d, bd, chain, nd) || !move(R.s0c, bc, chain, nc)) {
                            W.out[1] = 1;
                            s_stop = 1;
                            break;
                        }
                    } else if (chain) {
                        if (D.cfail[R.cs] == NONE32) D.cfail[R.cs] = i;
                        broken = true;
                    }
                } else {
                    // everything else (repeated ids, post/void, static failures): evaluate_one
                    // against the walked state (every predecessor final in D)
                    u32 s0d = NONE32, s0c = NONE32;
                    Bal4 bd{}, bc{};
                    if (R.sr == SRES_DYN && !pv) {
                        s0d = R.s0d;
                        s0c = R.s0c;
                        bd = read_bal(s0d, k, 0);
                        bc = read_bal(s0c, k, 1);
                        bb[R.ep.x] = bd;
                        bb[R.ep.y] = bc;
                    }
                    evaluate_one(T, C, D, D, bb, G, i);
                    const bool ok = D.ok[i] & 1;
                    u128 dpe, dpo;
                    state_deltas(C, D, i, &dpe, &dpo);
                    if (R.sr == SRES_DYN && !write_sides(C, i, pv, ok, D.pref[i], dpe, dpo)) {
                        W.out[0] = R.cs;  // its pending lies outside its sides: rebuild them, walk on from its chain
                        s_stop = 1;
                        break;
                    }
                    if (ok && R.sr == SRES_DYN) {
                        if (pv) {
                            for (u32 s = C.sd.soff[i]; s < C.sd.soff[i + 1]; s += 2)
                                if (C.sd.scand[s] == D.pref[i]) {
                                    s0d = W.sstart[C.sd.spos[s]];
                                    s0c = W.sstart[C.sd.spos[s + 1]];
                                    break;
                                }
                            if (s0d != NONE32) {
                                const u32 cd = s0d % WK_CACHE, cc = s0c % WK_CACHE;
                                bd = ctag[cd] == s0d ? cval[cd] : wk_load(&W.wbal[s0d]);
                                bc = ctag[cc] == s0c ? cval[cc] : wk_load(&W.wbal[s0c]);
                            }
                        }
                        if (s0d != NONE32) {
                            Bal4 nd = bd, nc = bc;
                            nd.dp += dpe; nd.dpo += dpo;
                            if (s0c == s0d) nc = nd;
                            nc.cp += dpe; nc.cpo += dpo;
                            if (!move(s0d, bd, chain, nd) || !move(s0c, s0c == s0d ? nd : bc, chain, nc)) {
                                W.out[1] = 1;
                                s_stop = 1;
                                break;
                            }
                        }
                    } else if (!ok && chain) {
                        broken = true;
                    }
                }
                if (chain && i == R.ce && (broken || (C.ctl && (C.ctl[R.ce] & TBGPU_CTL_DOOM)))) {
                    while (undo_n) {  // scope_close(.discard): the chain's balance moves, newest first
                        undo_n--;
                        const u32 s0 = W.undo_slot[undo_n];
                        write_bal(s0, W.undo_val[undo_n]);
                    }
                }
            }
        }
        __syncthreads();  // the block's stores before the next block's staged loads
        if (s_stop) return;
    }
}

}  // namespace

// ------------------------------------------------------------ launchers ----
#define GRID(n) (u32)(((n) + 255) / 256), 256, 0, stream

// Per-chunk reset in one launch: counters, the group table, the initial state's
// chain failures, the pass-counter ring (the first pass's gate open).
__global__ void tr_prep(TrArgs C, u32* cfail0, u32* pc, u32 ring) {
    const u64 g = C.gmask + 1;
    const u64 tot = max(max(g, (u64)C.n), (u64)ring);
    for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < tot; k += (u64)gridDim.x * blockDim.x) {
        if (k < g) {
            C.gclaim[k] = 0;
            C.gcnt_id[k] = 0;
            C.gcnt_pd[k] = 0;
            C.gbeg[k] = NONE32;
            C.pbeg[k] = NONE32;
            C.gfill[k] = 0;
            C.pfill[k] = 0;
        }
        if (k < C.n) {
            cfail0[k] = NONE32;
            C.dt.ev[k] = C.dt.ev[C.n + k] = NONE32;  // no stamp: pass 0 evaluates everything (Dirty::all)
            C.dt.chain[k] = C.dt.chain[C.n + k] = NONE32;
        }
        if (k < g) C.dt.slot[k] = C.dt.slot[g + k] = NONE32;
        if (k < ring) {
            pc[k] = k == 0 ? 1u : 0u;
            pc[ring + k] = NONE32;
        }
        if (k == 0) pc[2 * ring] = 1;  // an open gate (the full scans after a headroom fixed point, the walk)
        if (k < CNT_COUNT && k != CNT_STICKY) C.counters[k] = 0;
    }
}

void tr_launch_prep(const TrArgs& C, u32* cfail0, u32* pc, u32 ring, hipStream_t stream) {
    const u64 tot = std::max<u64>(std::max<u64>(C.gmask + 1, C.n), ring);
    tr_prep<<<(u32)std::min<u64>((tot + 255) / 256, 2048), 256, 0, stream>>>(C, cfail0, pc, ring);
}

void tr_launch_classify(const Tables& T, const TrArgs& C, hipStream_t stream) {
    tr_classify<<<GRID(C.n)>>>(T, C);
    tr_group1<<<GRID(C.n)>>>(C);
}
// kinds: 0 the id groups, 1 the pending groups, 2 both
void tr_launch_group(const TrArgs& C, u32 kinds, hipStream_t stream) {
    const u32 k0 = kinds == 2 ? 0u : kinds, nk = kinds == 2 ? 2u : 1u;
    const u32 nr = (C.n + GR_THREADS - 1) / GR_THREADS, nt = (C.n + 255) / 256;
    if (!nr) return;
    tr_grp_reserve<<<nk * nr, GR_THREADS, 0, stream>>>(C, k0, nr);
    tr_grp_place<<<nk * nt, 256, 0, stream>>>(C, k0, nt);
    tr_grp_rank<<<nk * nt, 256, 0, stream>>>(C, k0, nt);
}
void tr_launch_group2(const TrArgs& C, hipStream_t stream) { tr_group2<<<GRID(C.n)>>>(C); }
// the initial state and the per-pass work lists, in one launch
void tr_launch_init_lists(const Tables& T, const TrArgs& C, const EvalState& D, const EvalState& D2,
                          hipStream_t stream) {
    tr_lists<<<(C.n + LS_THREADS - 1) / LS_THREADS, LS_THREADS, 0, stream>>>(T, C, D, D2);
}
void tr_launch_side_count(const TrArgs& C, u32 kmax, u8* mask, hipStream_t stream) {
    tr_side_count<<<GRID(C.n)>>>(C, kmax, mask);
}
void tr_launch_side_build(const TrArgs& C, const EvalState& S, u32 kmax, const uint4* pairs, u32 invalid, u32* skey,
                          u32* sval, hipStream_t stream) {
    tr_side_build<<<GRID(C.n + 1)>>>(C, S, kmax, pairs, invalid, skey, sval);
}
void tr_launch_side_pos(const TrArgs& C, const u32* sval_s, u64 m, hipStream_t stream) {
    tr_side_pos<<<GRID(m)>>>(C, sval_s, m);  // (tstart and win cleared by tr_side_build)
}
void tr_launch_side_rec(const TrArgs& C, const EvalState& S, hipStream_t stream) {
    tr_side_rec<<<GRID(C.n)>>>(C, S);
}
void tr_launch_evaluate(const Tables& T, const TrArgs& C, const EvalState& S, const EvalState& D, const Bal4* bb,
                        const PassGate& g, u32* chg, u32* chg_next, u32* front, u32* front_next, hipStream_t stream) {
    tr_evaluate<<<GRID(C.n)>>>(T, C, S, D, bb, g, chg, chg_next, front, front_next);
}
void tr_launch_evaluate_lists(const Tables& T, const TrArgs& C, const EvalState& S, const EvalState& D, const Bal4* bb,
                              const PassGate& g, u32* chg, u32* chg_next, u32* front, u32* front_next, u32 n_simple,
                              u32 n_complex, hipStream_t stream) {
    // always launched (its first thread clears the next pass's words)
    const u32 nbc = (n_complex + EV_THREADS - 1) / EV_THREADS, nbs = (n_simple + EV_THREADS - 1) / EV_THREADS;
    tr_eval_lists<<<std::max<u32>(nbc + nbs, 1), EV_THREADS, 0, stream>>>(T, C, S, D, bb, g, n_simple, n_complex, nbc,
                                                                          chg, chg_next, front, front_next);
}
void tr_launch_mask(const Tables& T, const TrArgs& C, const EvalState& S, u8* fres, u8* mask, hipStream_t stream) {
    tr_mask<<<GRID(C.n)>>>(T, C, S, fres, mask);
}
void tr_launch_walk_prep(const TrArgs& C, u64 m, u32 start, u32* sstart, u32* cfail, hipStream_t stream) {
    tr_walk_prep<<<GRID(std::max<u64>(m, C.n))>>>(C, m, start, sstart, cfail);
}
void tr_launch_walk(const Tables& T, const TrArgs& C, const EvalState& D, Bal4* bb, u64 m, const u32* sstart,
                    Bal4* wbal, u32* undo_slot, Bal4* undo_val, u32 undo_cap, u32 start, u32* out, hipStream_t stream) {
    if (m) tr_walk_init<<<GRID(m)>>>(C, m, start, sstart, bb, wbal);
    WalkArgs W{sstart, wbal, undo_slot, undo_val, undo_cap, start, out};
    tr_walk<<<1, 64, 0, stream>>>(T, C, D, bb, W);
}
void tr_launch_apply(const Tables& T, const TrArgs& C, const EvalState& S, const u8* fres, const uint4* rk,
                     const Bal4* bb, tbgpu_create_transfers_result_t* results, u32* counts, u64* part,
                     hipStream_t stream) {
    tr_apply<<<GRID(C.n)>>>(T, C, S, fres, rk, bb, results);
    tr_range<<<(C.n + RG_THREADS - 1) / RG_THREADS, RG_THREADS, 0, stream>>>(T, C, S, part);
    batch_counts<<<GRID(C.nb)>>>(C.b_start, C.nb, rk, counts, C.epi);
}
void tr_launch_advance(const Tables& T, const TrArgs& C, const uint4* rk, const u64* part, hipStream_t stream) {
    tr_advance<<<1, 256, 0, stream>>>(T, C, rk, part, (C.n + RG_THREADS - 1) / RG_THREADS);
}
u64 tr_range_part_words(u64 n) { return 8 * ((n + RG_THREADS - 1) / RG_THREADS + 1); }

namespace {
__global__ void tr_converged(const u32* ring, u32 ring_len, u32 p0, u32 p1, const u32* counters, u32* epi) {
    if (threadIdx.x != 0) return;
    u32 e = 0;
    // (a 64-bit-form chunk whose figures left +-2^63 applies nothing: the host redoes it)
    if (counters[CNT_RESORT] == 0 && counters[CNT_LONG] == 0 && !(counters[CNT_FLAGS] & FL_H64_OVER))
        for (u32 q = p0; q < p1; q++)
            if (ring[(q + 1) % ring_len] == 0) {
                e = 1 + ((q + 1) & 1);
                break;
            }
    *epi = e;
}
}  // namespace

void tr_launch_converged(const u32* ring, u32 ring_len, u32 p0, u32 p1, const u32* counters, u32* epi,
                         hipStream_t stream) {
    tr_converged<<<1, 64, 0, stream>>>(ring, ring_len, p0, p1, counters, epi);
    HIP_CHECK(hipGetLastError());
}
