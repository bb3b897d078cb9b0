// accounts.hip — create_accounts as a batch-parallel fixed point, plus the
// lookup / maintenance kernels.
//
// create_account (src/state_machine.zig:1198-1225) depends on earlier events
// only through the id (a second create of the same id in the batch sees the
// first) and through linked chains, so the same Jacobi sweep as transfers.hip
// applies without the balance scan.
#include "common.h"
#include "engine.h"
#include "transfers.h"
#include "fast.h"

namespace {

template <class Start>
__device__ __forceinline__ u32 ac_batch_of_f(Start start, u32 nb, u32 i) {
    u32 lo = 0, hi = nb;
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (start(mid) <= i) lo = mid; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ u32 ac_batch_of(const u32* __restrict__ b_start, u32 nb, u32 i) {
    return ac_batch_of_f([&](u32 k) { return b_start[k]; }, nb, i);
}

__device__ __forceinline__ u32 ac_gtab_insert(const AcArgs& C, u128 key, u32 i) {
    const u32 claim = i + 1;
    u64 h = hash128(key) & C.gmask;
    for (;;) {
        u32 cur = C.gclaim[h];
        if (cur == 0) {
            const u32 prev = atomicCAS(&C.gclaim[h], 0u, claim);
            if (prev == 0) return (u32)h;
            cur = prev;
        }
        if (C.ev[cur - 1].id == key) return (u32)h;
        h = (h + 1) & C.gmask;
    }
}

__device__ __forceinline__ u32 ac_classify_one(const Tables& T, const AcArgs& C, u32 i, bool dup_check) {
    const u32 b = ac_batch_of(C.b_start, C.nb, i);
    const u32 bs = C.b_start[b], be = C.b_start[b + 1];
    const u32 nbatch = be - bs, k = i - bs;
    const Account a = C.ev[i];
    C.ts[i] = C.b_ts[b] - nbatch + k + 1;
    u32 s = i;
    while (s > bs && (C.ev[s - 1].flags & AF_LINKED)) s--;
    u32 e = i;
    while (e + 1 < be && (C.ev[e].flags & AF_LINKED)) e++;
    C.cs[i] = s;
    C.ce[i] = e;
    u32 fl = (s != e) ? FL_CHAINS : 0u;
    u8 sres;
    u32 pre = NONE32, gslot = NONE32;
    // execute (:1018-1035) then create_account's static checks (:1201-1216)
    if ((a.flags & AF_LINKED) && k == nbatch - 1) sres = TBGPU_CREATE_ACCOUNT_LINKED_EVENT_CHAIN_OPEN;
    else if (a.timestamp != 0) sres = TBGPU_CREATE_ACCOUNT_TIMESTAMP_MUST_BE_ZERO;
    else if (a.reserved != 0) sres = TBGPU_CREATE_ACCOUNT_RESERVED_FIELD;
    else if (a.flags & 0xFFF0u) sres = TBGPU_CREATE_ACCOUNT_RESERVED_FLAG;
    else if (a.id == 0) sres = TBGPU_CREATE_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    else if (a.id == U128_MAX) sres = TBGPU_CREATE_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    else if ((a.flags & AF_DNEC) && (a.flags & AF_CNED)) sres = TBGPU_CREATE_ACCOUNT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    else if (a.debits_pending != 0) sres = TBGPU_CREATE_ACCOUNT_DEBITS_PENDING_MUST_BE_ZERO;
    else if (a.debits_posted != 0) sres = TBGPU_CREATE_ACCOUNT_DEBITS_POSTED_MUST_BE_ZERO;
    else if (a.credits_pending != 0) sres = TBGPU_CREATE_ACCOUNT_CREDITS_PENDING_MUST_BE_ZERO;
    else if (a.credits_posted != 0) sres = TBGPU_CREATE_ACCOUNT_CREDITS_POSTED_MUST_BE_ZERO;
    else if (a.ledger == 0) sres = TBGPU_CREATE_ACCOUNT_LEDGER_MUST_NOT_BE_ZERO;
    else if (a.code == 0) sres = TBGPU_CREATE_ACCOUNT_CODE_MUST_NOT_BE_ZERO;
    else {
        sres = SRES_DYN;
        pre = acc_row(T, a.id);  // ROW_FOREIGN: an account another ledger shard stores
        if (dup_check) {  // ids that rise strictly through the call cannot repeat (ac_mono)
            gslot = ac_gtab_insert(C, a.id, i);
            atomicAdd(&C.gcnt_id[gslot], 1u);
        }
    }
    C.sres[i] = sres;
    C.pre[i] = pre;
    C.gslot[i] = gslot;
    C.prev_id[i] = NONE32;
    return fl;
}

// Whether the call's ids rise strictly from event to event (the benchmark's sequential
// ids): then no id repeats and classify skips the call-local group table (a CAS and a
// count atomic per account).  One flag atomic per workgroup that sees a descent.
__global__ void ac_mono(AcArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    bool down = false;
    if (i > 0 && i < C.n) down = !(C.ev[i].id > C.ev[i - 1].id);
    if (__syncthreads_or(down) && threadIdx.x == 0) raise_flags(&C.counters[CNT_FLAGS], (u32)FL_NONMONO);
}

__global__ void ac_classify(Tables T, AcArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool dup_check = C.counters[CNT_FLAGS] & FL_NONMONO;
    u32 fl = 0;
    if (i < C.n) fl = ac_classify_one(T, C, i, dup_check);
    fl = wave_or_u32(fl);  // one flag atomic per wave, not per chain member
    if (wave_leader()) raise_flags(&C.counters[CNT_FLAGS], fl);
}

__global__ void ac_group1(AcArgs C) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u32 g = C.gslot[i];
    if (g != NONE32 && C.gcnt_id[g] > 1) atomicOr(&C.counters[CNT_FLAGS], (u32)FL_MULTI_ID);
}

__global__ void ac_group_keys(AcArgs C, u32 invalid, u32* keys, u32* vals) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u32 g = C.gslot[i];
    keys[i] = g == NONE32 ? invalid : g;
    vals[i] = i;
}

__global__ void ac_group_prev(AcArgs C, u32 invalid, const u32* ks, const u32* vs) {
    const u32 q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= C.n) return;
    const u32 key = ks[q];
    if (key >= invalid) return;
    C.prev_id[vs[q]] = (q == 0 || ks[q - 1] != key) ? NONE32 : vs[q - 1];
}

__global__ void ac_init(AcArgs C, u8* res, u8* ok, u32* cfail) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 sr = C.sres[i];
    u8 r = sr;
    if (sr == SRES_DYN) r = C.pre[i] != NONE32 ? TBGPU_CREATE_ACCOUNT_EXISTS : TBGPU_CREATE_ACCOUNT_OK;
    res[i] = r;
    ok[i] = r == 0 ? 1 : 0;
    if (r != 0 && C.cs[i] != C.ce[i]) atomicMin(&cfail[C.cs[i]], i);
}

__global__ void ac_finalize(AcArgs C, u8* ok, const u32* cfail) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 o = ok[i] & 1;
    const u32 cs = C.cs[i];
    const bool persisted = cs == C.ce[i] || cfail[cs] == NONE32;
    ok[i] = o | ((o && persisted) ? 2 : 0);
}

// create_account_exists (src/state_machine.zig:1227-1237)
__device__ __forceinline__ u8 account_exists(const Account& a, const Account& e) {
    if (a.flags != e.flags) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (a.user_data_128 != e.user_data_128) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (a.user_data_64 != e.user_data_64) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (a.user_data_32 != e.user_data_32) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (a.ledger != e.ledger) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_LEDGER;
    if (a.code != e.code) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_CODE;
    return TBGPU_CREATE_ACCOUNT_EXISTS;
}

__global__ void ac_evaluate(Tables T, AcArgs C, const u8* res_s, const u8* ok_s, u8* res_d, u8* ok_d, u32* cfail_d) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 sr = C.sres[i];
    u8 r = sr;
    const u32 csi = C.cs[i];
    if (sr == SRES_DYN) {
        const Account a = C.ev[i];
        u32 e = NONE32;
        for (u32 j = C.prev_id[i]; j != NONE32; j = C.prev_id[j]) {
            const u8 o = ok_s[j];
            if (C.cs[j] == csi ? (o & 1) : (o & 2)) { e = j; break; }
        }
        if (e != NONE32) r = account_exists(a, C.ev[e]);
        else if (C.pre[i] == ROW_FOREIGN) r = TBGPU_SHARD_ACCOUNT_EXISTS_ELSEWHERE;  // its owner compares
        else if (C.pre[i] != NONE32) r = account_exists(a, T.acc[C.pre[i]]);
        else r = TBGPU_CREATE_ACCOUNT_OK;
    }
    res_d[i] = r;
    ok_d[i] = r == 0 ? 1 : 0;
    if (r != 0 && csi != C.ce[i]) atomicMin(&cfail_d[csi], i);
    if (r != res_s[i]) atomicAdd(&C.counters[CNT_CHANGES], 1u);  // few: only events whose result moved
}

__device__ __forceinline__ u64 ac_mask_one(const Tables& T, const AcArgs& C, const u8* res, const u8* ok,
                                           const u32* cfail, u8* fres, u8* mask, u32 i) {
    const u32 cs = C.cs[i];
    const u32 cf = cs != C.ce[i] ? cfail[cs] : NONE32;
    u8 r;
    if (C.sres[i] == TBGPU_CREATE_ACCOUNT_LINKED_EVENT_CHAIN_OPEN) r = TBGPU_CREATE_ACCOUNT_LINKED_EVENT_CHAIN_OPEN;
    else if (cf < i) r = TBGPU_CREATE_ACCOUNT_LINKED_EVENT_FAILED;
    else if (res[i] != 0) r = res[i];
    else if (cf != NONE32) r = TBGPU_CREATE_ACCOUNT_LINKED_EVENT_FAILED;
    else r = TBGPU_CREATE_ACCOUNT_OK;
    fres[i] = r;
    // bit 0: a row here (persisted, this shard's ledger); bit 2: persisted on another
    // shard's ledger (a directory entry only)
    const bool kept = ok[i] & 2, own = ledger_owned(T, C.ev[i].ledger);
    mask[i] = (kept && own ? 1 : 0) | (r != 0 ? 2 : 0) | (kept && !own ? 4 : 0);
    // commit_timestamp survives rollback (:1223)
    return ((ok[i] & 1) && (cf == NONE32 || i < cf)) ? C.ts[i] : 0;
}

// The accepted events' max timestamp goes to a per-workgroup word, folded by one
// workgroup (ac_ts_fold) into the single commit_timestamp word: same-address atomics
// serialize at the memory side (one per accepted event took 897 us for 10M accounts,
// one per wave still 890 us).
__global__ void ac_mask(Tables T, AcArgs C, const u8* res, const u8* ok, const u32* cfail, u8* fres, u8* mask,
                        const u32* gate) {
    if (gate && *gate == 0) return;
    __shared__ u64 s_w[4];
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    u64 ts = i < C.n ? ac_mask_one(T, C, res, ok, cfail, fres, mask, i) : 0;
    ts = wave_max_u64(ts);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = ts;
    __syncthreads();
    if (threadIdx.x == 0) C.ts_part[blockIdx.x] = max(max(s_w[0], s_w[1]), max(s_w[2], s_w[3]));
}

__global__ void ac_ts_fold(const u64* part, u32 nparts, u64* commit_ts, const u32* gate) {
    if (gate && *gate == 0) return;
    __shared__ u64 s_w[16];
    u64 m = 0;
    for (u32 k = threadIdx.x; k < nparts; k += blockDim.x) m = max(m, part[k]);
    m = wave_max_u64(m);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (u32 w = 1; w < blockDim.x / 64; w++) m = max(m, s_w[w]);
        if (m) atomicMax((unsigned long long*)commit_ts, (unsigned long long)m);
    }
}

__global__ void ac_apply(Tables T, AcArgs C, const u8* ok, const u8* fres, const uint4* rk, u64 row_base, u64 cap,
                         tbgpu_create_accounts_result_t* results, const u32* gate) {
    if (gate && *gate == 0) return;
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const u8 r = fres[i];
    if (r != 0) {
        const u32 b = ac_batch_of(C.b_start, C.nb, i);
        const u32 bs = C.b_start[b];
        results[rk[i].y] = {i - bs, (u32)r};  // concatenated replies
        return;
    }
    if (!(ok[i] & 2)) return;
    Account a = C.ev[i];
    if (!ledger_owned(T, a.ledger)) {  // another ledger shard stores the row: the directory entry only
        if (!acc_insert(T, a.id, ROW_FOREIGN, a.ledger, a.flags, a.code))
            atomicOr(&C.counters[CNT_FLAGS], (u32)FL_CAPACITY);  // the account index is full
        return;
    }
    a.timestamp = C.ts[i];
    // accounts.insert: the row is the event's rank among the persisted accounts
    // (creation order); the directory entry (or index slot) names it.
    if (row_base + rk[i].x >= cap) {  // accounts_max exceeded: nothing past it is written (the host aborts)
        atomicOr(&C.counters[CNT_FLAGS], (u32)FL_CAPACITY);
        return;
    }
    const u32 row = (u32)(row_base + rk[i].x);
    T.acc[row] = a;
    if (!acc_insert(T, a.id, row, a.ledger, a.flags, a.code)) atomicOr(&C.counters[CNT_FLAGS], (u32)FL_CAPACITY);
}

// ---------------------------------------------- the clean call in two passes --
// The benchmark's create_accounts call (src/tigerbeetle/benchmark_load.zig:209-247):
// no repeated id, no chain, no existing id, every field valid.  Then every event is
// ok, its row is n_accounts + i and its timestamp T_b - n_b + k + 1 (execute,
// :1033-1035; create_account, :1198-1225), so the call is two passes (three when its
// ids do not rise):
//   ac_fast_check  8 lanes per account, 16 bytes each: the lane's fields checked,
//                  the chunk stored to the optimistic row (the timestamp patched in);
//                  one lane probes the directory / index and compares the id with
//                  the previous event's (ids that do not rise raise FL_NONMONO).
//                  Anything else raises FL_SLOW (one atomic per wave), and the host
//                  redoes the call on the general path (rows past n_accounts are free
//                  space; the directory entries the check wrote are cleared by
//                  ac_fast_index first).
//                  An id of the direct-mapped directory whose entry is empty gets
//                  its entry right there (two events writing one entry have one id:
//                  rising ids never do, and ac_fast_dup finds them otherwise).
//   ac_fast_dup    only with FL_NONMONO (--id-order=random / reversed, the benchmark's
//                  IdPermutation, src/testing/id.zig:28-48; otherwise it returns at
//                  once): every id claims a slot of a call-local table by CAS (event +
//                  1); a claim that meets an earlier claim of the same id (read from the
//                  events, which nothing writes) is a repeat: FL_SLOW.
//   ac_fast_index  on a clean check: the index slot of every hashed id (CAS on its row
//                  word; none when every id is in the directory, FL_AC_HASHED clear),
//                  zero reply counts, commit_timestamp.  On a failed check: the
//                  directory entries the check wrote are cleared again.  Either way
//                  the call-local claims are cleared.
constexpr int AF_THREADS = 256;

// INL: a small call, whose batch block comes in the arguments (no upload launch) and is
// copied to LDS, and whose flags are gathered per workgroup.  The other form is the
// plain kernel: its batch block in memory, no LDS, no barrier (one kernel for both took
// 96 us for 1M accounts against 66).
template <bool INL>
__global__ __launch_bounds__(AF_THREADS) void ac_fast_check(Tables T, AcArgs C, u64 row_base, BlockInline bi) {
    const u64 t = (u64)blockIdx.x * AF_THREADS + threadIdx.x;
    __shared__ u32 s_blk[INL ? BLOCK_INLINE_WORDS : 1];
    constexpr bool inl = INL;
    if constexpr (INL) {
        if (threadIdx.x < bi.words) s_blk[threadIdx.x] = bi.w[threadIdx.x];
        __syncthreads();
    }
    const u32 ts_off = (C.nb + 2) & ~1u;  // batch_ts_offset
    auto bstart = [&](u32 k) -> u32 { return inl ? s_blk[k] : C.b_start[k]; };
    auto bts = [&](u32 b) -> u64 {
        return inl ? ((u64)s_blk[ts_off + 2 * b + 1] << 32 | s_blk[ts_off + 2 * b]) : C.b_ts[b];
    };
    const u32 e = (u32)(t >> 3), ch = (u32)(t & 7), lane = threadIdx.x & 63;
    // The wave's 8 events are nearly always in one batch: one uniform binary search for
    // its first event, issued before the event loads, and lanes past a batch boundary
    // walk on (a search per event made every wave wait for seven dependent loads)
    const u32 e0 = __builtin_amdgcn_readfirstlane(e);
    u32 b = e0 < C.n ? ac_batch_of_f(bstart, C.nb, e0) : 0u;
    bool bad = false;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (e < C.n) v = ((const uint4*)&C.ev[e])[ch];
    // the previous event's id: from the lanes 8 below (chunk 0 of event e - 1), or, for
    // the wave's first event, from memory
    const u32 px = __shfl(v.x, lane - 8), py = __shfl(v.y, lane - 8), pz = __shfl(v.z, lane - 8),
              pw = __shfl(v.w, lane - 8);
    // the event's ledger and flags (chunk 7, seven lanes up), for its directory entry
    const u32 q7x = __shfl(v.x, lane + 7), q7y = __shfl(v.y, lane + 7);
    bool hashed = false, nonmono = false;
    if (e < C.n) {
        switch (ch) {
        case 0: {  // id: not 0 / maxInt (:1204-1205), absent, above the previous event's
            const u128 id = ((u128)(((u64)v.w << 32) | v.z) << 64) | (((u64)v.y << 32) | v.x);
            bad = id == 0 || id == U128_MAX;
            if (!bad && e > 0) {
                const u128 prev = lane >= 8 ? ((u128)(((u64)pw << 32) | pz) << 64) | (((u64)py << 32) | px)
                                            : C.ev[e - 1].id;
                nonmono = !(id > prev);  // (a repeat is possible: ac_fast_dup looks)
            }
            if (!bad) {
                if (dense_has(T, id)) {
                    // plain accesses: a CAS per account executes at the memory side (1M
                    // accounts took 0.164 ms with one, 0.091 ms without); two events of
                    // one id are a repeat, which ac_fast_dup finds
                    u64& d = T.dense[dense_slot(T, id)];
                    bad = d != 0;
                    if (!bad) d = dense_entry((u32)(row_base + e), q7x, (u16)(q7y >> 16));
                } else {
                    hashed = true;
                    bad = acc_probe(T.aidx, T.aidx_mask, id) != NONE32;
                }
            }
            break;
        }
        case 1: case 2: case 3: case 4:  // balances must be zero (:1208-1211)
            bad = (v.x | v.y | v.z | v.w) != 0;
            break;
        case 6:  // reserved (:1202)
            bad = v.w != 0;
            break;
        case 7: {  // ledger, code, flags, timestamp (:1201-1213, execute :1033)
            const u32 code = v.y & 0xFFFFu, flags = v.y >> 16;
            bad = v.x == 0 || code == 0 || (v.z | v.w) != 0 || (flags & (0xFFF0u | AF_LINKED)) != 0 ||
                  ((flags & AF_DNEC) && (flags & AF_CNED));
            while (b + 1 < C.nb && bstart(b + 1) <= e) b++;
            const u32 bs = bstart(b), nbatch = bstart(b + 1) - bs;
            const u64 ts = bts(b) - nbatch + (e - bs) + 1;
            v.z = (u32)ts;
            v.w = (u32)(ts >> 32);
            break;
        }
        default:
            break;
        }
        ((uint4*)&T.acc[row_base + e])[ch] = v;
    }
    // Only the bits not raised yet (raise_flags): with random ids every wave raises
    // FL_AC_HASHED | FL_NONMONO, and one atomic per wave on the one flags word
    // serialised at L2 (10k random ids: 1252 atomics; the kernel took 22.6 us with them,
    // 11.3 us without).  A small call gathers them per workgroup first (raise_flags per
    // wave, its load's round trip at every wave's end: 0.059 ms for the call against
    // 0.042); a large one per wave (no barrier).
    const u32 fl = (__ballot(bad) ? (u32)FL_SLOW : 0u) | (__ballot(hashed) ? (u32)FL_AC_HASHED : 0u) |
                   (__ballot(nonmono) ? (u32)FL_NONMONO : 0u);
    if constexpr (INL) {
        __shared__ u32 s_fl;
        if (threadIdx.x == 0) s_fl = 0;
        __syncthreads();
        if (fl && wave_leader()) atomicOr(&s_fl, fl);
        __syncthreads();
        if (threadIdx.x == 0) raise_flags(&C.fast_words[0], s_fl);
    } else {
        if (wave_leader()) raise_flags(&C.fast_words[0], fl);
    }
}

__global__ __launch_bounds__(AF_THREADS) void ac_fast_dup(AcArgs C) {
    if (!(C.fast_words[0] & FL_NONMONO)) return;  // ids rise through the call: none repeats
    const u32 i = blockIdx.x * AF_THREADS + threadIdx.x;
    bool dup = false;
    if (i < C.n) {
        const u128 id = C.ev[i].id;
        u64 h = hash128(id) & C.fmask;
        for (;;) {
            const u32 prev = atomicCAS(&C.ftab[h], 0u, i + 1);
            if (prev == 0) {
                C.fpos[i] = (u32)h;
                break;
            }
            if (C.ev[prev - 1].id == id) {
                C.fpos[i] = NONE32;
                dup = true;
                break;
            }
            h = (h + 1) & C.fmask;
        }
    }
    // (one flag atomic per workgroup at most, and none once the bit is up)
    if (__syncthreads_or(dup) && threadIdx.x == 0) raise_flags(&C.fast_words[0], (u32)FL_SLOW);
}

__global__ __launch_bounds__(AF_THREADS) void ac_fast_index(Tables T, AcArgs C, u64 row_base, BlockInline bi) {
    const u32 flags = C.fast_words[0];
    const u32 i = blockIdx.x * AF_THREADS + threadIdx.x;
    __shared__ u32 s_blk[BLOCK_INLINE_WORDS];
    const bool inl = bi.words != 0;
    if (inl) {  // a small call's batch block: to memory (the general path reads it there)
        if (threadIdx.x < bi.words) {
            s_blk[threadIdx.x] = bi.w[threadIdx.x];
            if (blockIdx.x == 0) bi.block[threadIdx.x] = bi.w[threadIdx.x];
        }
        __syncthreads();
    }
    const u32 ts_off = (C.nb + 2) & ~1u;  // batch_ts_offset
    auto bstart = [&](u32 k) -> u32 { return inl ? s_blk[k] : C.b_start[k]; };
    auto bts = [&](u32 b) -> u64 {
        return inl ? ((u64)s_blk[ts_off + 2 * b + 1] << 32 | s_blk[ts_off + 2 * b]) : C.b_ts[b];
    };
    if ((flags & FL_NONMONO) && i < C.n && C.fpos[i] != NONE32) C.ftab[C.fpos[i]] = 0;  // (all-zero again)
    if (flags & FL_SLOW) {
        // the call goes to the general path: the directory entries the check wrote go
        if (i < C.n) {
            const u128 id = C.ev[i].id;
            if (dense_has(T, id)) {
                u64& d = T.dense[dense_slot(T, id)];
                if (d != 0 && dense_row(d) == (u32)(row_base + i)) d = 0;
            }
        }
    } else {
        if (i < C.n && (flags & FL_AC_HASHED)) {
            const u32 row = (u32)(row_base + i);
            const uint4 k = ((const uint4*)&T.acc[row])[0];
            const uint4 m = ((const uint4*)&T.acc[row])[7];
            const u128 id = ((u128)(((u64)k.w << 32) | k.z) << 64) | (((u64)k.y << 32) | k.x);
            const u16 code = (u16)(m.y & 0xFFFFu), af = (u16)(m.y >> 16);
            if (!acc_insert(T, id, row, m.x, af, code)) atomicOr(&C.fast_words[0], (u32)FL_CAPACITY);
        }
        if (blockIdx.x == 0) {
            // replies: none; commit_timestamp: the latest event's (every event is accepted)
            u64 mts = 0;
            for (u32 b = threadIdx.x; b < C.nb; b += AF_THREADS) {
                C.counts_out[b] = 0;
                if (bstart(b + 1) > bstart(b)) mts = max(mts, bts(b));
            }
            mts = wave_max_u64(mts);
            if (wave_leader() && mts) atomicMax((unsigned long long*)T.commit_ts, (unsigned long long)mts);
        }
    }
    // The call's flags to the host from the last workgroup to finish (instead of a copy
    // after the kernel: a blit launch of 4.2 us and its gap).  Each
    // wave waits for its own memory operations (FL_CAPACITY's atomic among them), the
    // workgroup then takes a ticket, and the last one reads the final word: the counter
    // hand-off of MI355X_MICROARCH.md's sc1 forms.  The kernel's end makes the host
    // store visible to the host's wait on the stream.
    // Only for small grids (flags_out set): the tickets are returning atomics on one
    // word, ~12 ns each at the memory side, so 3907 workgroups (1M accounts) paid 47 us;
    // a large call's host copies the flags after the kernel instead.
    if (!C.flags_out) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const u32 t = __hip_atomic_fetch_add(&C.fast_words[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {
            const u32 f = __hip_atomic_load(&C.fast_words[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(C.flags_out, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // all-zero again for the next call (every workgroup has read the flags)
            __hip_atomic_store(&C.fast_words[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&C.fast_words[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void ac_batch_counts(const u32* b_start, u32 nb, const uint4* rk, u32* counts, const u32* gate) {
    if (gate && *gate == 0) return;
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) counts[b] = rk[b_start[b + 1]].y - rk[b_start[b]].y;
}

// ------------------------------------------------------------- lookups ----
__global__ void k_lookup_accounts(Tables T, const u128* ids, u32 n, Account* out, u8* found) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 s = acc_row(T, ids[i]);
    found[i] = s != NONE32 && s != ROW_FOREIGN;  // another shard's account: its owner answers
    if (found[i]) out[i] = T.acc[s];
}
__global__ void k_lookup_transfers(Tables T, const u128* ids, u32 n, Transfer* out, u8* found) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 r = xidx_probe(T, ids[i]);
    found[i] = r != NONE32;
    if (r != NONE32) out[i] = T.xrows[r];
}
__global__ void k_set_balances(Tables T, u128 id, Bal4 b, int* status) {
    const u32 s = acc_row(T, id);
    if (s == NONE32 || s == ROW_FOREIGN) { *status = -1; return; }
    Account& a = T.acc[s];
    a.debits_pending = b.dp;
    a.debits_posted = b.dpo;
    a.credits_pending = b.cp;
    a.credits_posted = b.cpo;
    const u64 lim = 1ull << 62;
    if ((u64)(b.dp >> 64) >= lim || (u64)(b.dpo >> 64) >= lim || (u64)(b.cp >> 64) >= lim || (u64)(b.cpo >> 64) >= lim)
        atomicOr(T.big, 1u);
    if ((b.dp | b.dpo | b.cp | b.cpo) >> 61) atomicOr(T.big, 2u);
    *status = 0;
}
__global__ void k_get_posted(Tables T, u128 id, int* status) {
    const u32 r = xidx_probe(T, id);
    if (r == NONE32) { *status = -1; return; }
    const u8 f = T.xful[r];
    *status = f == 0 ? -1 : (f == 1 ? 0 : 1);
}

// Foreign rows (tbgpu_import_transfers): stored rows + id index + key range, no
// balance or posted effects.
// The key range is folded per wave: four same-address atomics per row serialized at
// the memory side (125M rows per GPU at config 5's tbgpu_open).
__global__ void import_transfers(Tables T, const Transfer* rows, u32 n, u64 row_base, u32 in_place) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    u64 mxl = 0, mxh = 0, mnl = ~0ull, mnh = ~0ull;
    if (i < n) {
        if (!in_place) {  // the row, 16 bytes at a time
            const uint4* src = (const uint4*)&rows[i];
            uint4* dst = (uint4*)&T.xrows[row_base + i];
#pragma unroll
            for (int k = 0; k < 8; k++) dst[k] = src[k];
        }
        const u128 id = rows[i].id;
        xidx_insert(T, id, (u32)(row_base + i));
        mxl = mnl = (u64)id;
        mxh = mnh = (u64)(id >> 64);
    }
    mxl = wave_max_u64(mxl);
    mxh = wave_max_u64(mxh);
    mnl = wave_min_u64(mnl);
    mnh = wave_min_u64(mnh);
    if (wave_leader() && mnl <= mxl) {
        atomicMax((unsigned long long*)&T.idr[0], (unsigned long long)mxl);
        atomicMax((unsigned long long*)&T.idr[1], (unsigned long long)mxh);
        atomicMin((unsigned long long*)&T.idr[2], (unsigned long long)mnl);
        atomicMin((unsigned long long*)&T.idr[3], (unsigned long long)mnh);
    }
}

// The transfer-id index rebuilt from the stored rows (xidx_tombs_check, engine.hip):
// every row outside the sorted run, whose rows are found by search, not by the index.
__global__ void k_rehash_xidx(Tables T, u64 n) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n || (r >= T.xrun[0] && r < T.xrun[1])) return;
    xidx_insert(T, T.xrows[r].id, (u32)r);
}

// tbgpu_open: the account index from the dense rows (ac_apply's insert).
__global__ void k_rebuild_aidx(Tables T, u64 n) {
    const u64 row = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n) return;
    const Account& a = T.acc[row];
    acc_insert(T, a.id, (u32)row, a.ledger, a.flags, a.code);
}

// tbgpu_open of a ledger shard: the other shards' accounts' directory entries.
__global__ void k_insert_foreign(Tables T, const ForeignAccount* f, u64 n) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    acc_insert(T, ((u128)f[k].id_hi << 64) | f[k].id_lo, ROW_FOREIGN, f[k].ledger, 0, 0);
}

// tbgpu_checkpoint of a ledger shard: the directory entries of other shards'
// accounts, gathered (in no particular order; the host sorts them) from the
// direct-mapped directory and the hash index.
__global__ void k_collect_foreign(Tables T, ForeignAccount* out, u32* cursor, u64 cap) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    ForeignAccount f{};
    bool hit = false;
    if (k < T.dense_n) {
        const u64 e = T.dense[k];
        if (e != 0 && ((u32)e & DENSE_ROW1_MASK) == DENSE_FOREIGN1) {
            const u64 b = k / T.dense_span, j = k % T.dense_span + 1;
            f.id_lo = (b << 32) | j;
            f.ledger = (u32)(e >> 32);
            hit = true;
        }
    } else if (k - T.dense_n <= T.aidx_mask) {
        const AccIdx& e = T.aidx[k - T.dense_n];
        if (e.row1 == ROW_FOREIGN + 1) {
            f.id_lo = e.id_lo;
            f.id_hi = e.id_hi;
            f.ledger = e.ledger;
            hit = true;
        }
    }
    if (hit) {
        const u32 at = atomicAdd(cursor, 1u);
        if (at < cap) out[at] = f;
    }
}

// tbgpu_open: the fast path's overflow guard (fast.hip) from the restored balances.
__global__ void k_scan_big(Tables T, u64 n) {
    const u64 row = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n) return;
    const Account& a = T.acc[row];
    const u64 lim = 1ull << 62;
    if ((u64)(a.debits_pending >> 64) >= lim || (u64)(a.debits_posted >> 64) >= lim ||
        (u64)(a.credits_pending >> 64) >= lim || (u64)(a.credits_posted >> 64) >= lim)
        atomicOr(T.big, 1u);
    if ((a.debits_pending | a.debits_posted | a.credits_pending | a.credits_posted) >> 61) atomicOr(T.big, 2u);
}

}  // namespace

#define GRID(n) (u32)(((n) + 255) / 256), 256, 0, stream

void launch_insert_foreign(const Tables& T, const ForeignAccount* f, u64 n, hipStream_t stream) {
    if (!n) return;
    k_insert_foreign<<<GRID(n)>>>(T, f, n);
    HIP_CHECK(hipGetLastError());
}
void launch_collect_foreign(const Tables& T, ForeignAccount* out, u32* cursor, u64 cap, hipStream_t stream) {
    const u64 n = T.dense_n + T.aidx_mask + 1;
    k_collect_foreign<<<GRID(n)>>>(T, out, cursor, cap);
    HIP_CHECK(hipGetLastError());
}
void launch_rebuild_accounts(const Tables& T, u64 n, hipStream_t stream) {
    if (!n) return;
    k_rebuild_aidx<<<GRID(n)>>>(T, n);
    k_scan_big<<<GRID(n)>>>(T, n);
    HIP_CHECK(hipGetLastError());
}

void ac_launch_classify(const Tables& T, const AcArgs& C, hipStream_t stream) {
    ac_mono<<<GRID(C.n)>>>(C);
    ac_classify<<<GRID(C.n)>>>(T, C);
    ac_group1<<<GRID(C.n)>>>(C);
}
void ac_launch_group_sort(const AcArgs& C, u32 invalid, int bits, u32* k_in, u32* v_in, u32* k_out, u32* v_out,
                          SortScratch& ss, hipStream_t stream) {
    ac_group_keys<<<GRID(C.n)>>>(C, invalid, k_in, v_in);
    radix_sort_pairs(k_in, v_in, k_out, v_out, C.n, bits, ss, stream);
    ac_group_prev<<<GRID(C.n)>>>(C, invalid, k_out, v_out);
}
void ac_launch_init(const AcArgs& C, u8* res, u8* ok, u32* cfail, hipStream_t stream) {
    ac_init<<<GRID(C.n)>>>(C, res, ok, cfail);
    ac_finalize<<<GRID(C.n)>>>(C, ok, cfail);
}
void ac_launch_evaluate(const Tables& T, const AcArgs& C, const u8* res_s, const u8* ok_s, u8* res_d, u8* ok_d,
                        u32* cfail_d, hipStream_t stream) {
    ac_evaluate<<<GRID(C.n)>>>(T, C, res_s, ok_s, res_d, ok_d, cfail_d);
    ac_finalize<<<GRID(C.n)>>>(C, ok_d, cfail_d);
}
void ac_launch_mask(const Tables& T, const AcArgs& C, const u8* res, const u8* ok, const u32* cfail, u8* fres,
                    u8* mask, hipStream_t stream, const u32* gate) {
    static_assert(256 == 4 * 64, "ac_mask folds four waves per workgroup");
    ac_mask<<<GRID(C.n)>>>(T, C, res, ok, cfail, fres, mask, gate);
    ac_ts_fold<<<1, 1024, 0, stream>>>(C.ts_part, (C.n + 255) / 256, T.commit_ts, gate);
}
u32 ac_fast_index_grid(const AcArgs& C) { return (u32)((std::max(C.n, C.nb) + AF_THREADS - 1) / AF_THREADS); }
void ac_launch_fast(const Tables& T, const AcArgs& C, u64 row_base, const BlockInline& bi, hipStream_t stream) {
    const u64 lanes = 8ull * C.n;
    if (bi.words)
        ac_fast_check<true><<<(u32)((lanes + AF_THREADS - 1) / AF_THREADS), AF_THREADS, 0, stream>>>(T, C, row_base, bi);
    else
        ac_fast_check<false><<<(u32)((lanes + AF_THREADS - 1) / AF_THREADS), AF_THREADS, 0, stream>>>(T, C, row_base, bi);
    ac_fast_dup<<<(u32)((C.n + AF_THREADS - 1) / AF_THREADS), AF_THREADS, 0, stream>>>(C);
    ac_fast_index<<<ac_fast_index_grid(C), AF_THREADS, 0, stream>>>(T, C, row_base, bi);
    HIP_CHECK(hipGetLastError());
}
void ac_launch_apply(const Tables& T, const AcArgs& C, const u8* ok, const u8* fres, const uint4* rk, u64 row_base,
                     u64 cap, tbgpu_create_accounts_result_t* results, u32* counts, hipStream_t stream, const u32* gate) {
    ac_apply<<<GRID(C.n)>>>(T, C, ok, fres, rk, row_base, cap, results, gate);
    ac_batch_counts<<<GRID(C.nb)>>>(C.b_start, C.nb, rk, counts, gate);
}
namespace {
// The speculative one-evaluation path of create_accounts runs iff classify found neither
// a linked chain nor a repeated id (one thread).
__global__ void ac_gate(AcArgs C, u32* gate) {
    if (threadIdx.x == 0) *gate = (C.counters[CNT_FLAGS] & (FL_CHAINS | FL_MULTI_ID)) ? 0u : 1u;
}
}  // namespace
void ac_launch_gate(const AcArgs& C, u32* gate, hipStream_t stream) { ac_gate<<<1, 64, 0, stream>>>(C, gate); }
void launch_lookup_accounts(const Tables& T, const u128* ids, u32 n, Account* out, u8* found, hipStream_t stream) {
    if (n) k_lookup_accounts<<<GRID(n)>>>(T, ids, n, out, found);
}
void launch_lookup_transfers(const Tables& T, const u128* ids, u32 n, Transfer* out, u8* found, hipStream_t stream) {
    if (n) k_lookup_transfers<<<GRID(n)>>>(T, ids, n, out, found);
}
void launch_set_balances(const Tables& T, u128 id, Bal4 b, int* status, hipStream_t stream) {
    k_set_balances<<<1, 1, 0, stream>>>(T, id, b, status);
}
void launch_get_posted(const Tables& T, u128 id, int* status, hipStream_t stream) {
    k_get_posted<<<1, 1, 0, stream>>>(T, id, status);
}

void launch_rehash_xidx(const Tables& T, u64 n, hipStream_t s) {
    if (n) k_rehash_xidx<<<(u32)((n + 255) / 256), 256, 0, s>>>(T, n);
}

void launch_import_transfers(const Tables& T, const Transfer* rows, u32 n, u64 row_base, hipStream_t stream) {
    import_transfers<<<(n + 255) / 256, 256, 0, stream>>>(T, rows, n, row_base, rows == T.xrows + row_base ? 1u : 0u);
    HIP_CHECK(hipGetLastError());
}
