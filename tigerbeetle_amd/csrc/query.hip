// query.hip — get_account_transfers / get_account_history over the HBM tables.
//
// The reference answers both queries with a scan of the transfers groove's
// debit_account_id / credit_account_id index trees (a prefix scan per side,
// merged by timestamp: src/state_machine.zig:822-885), then looks the objects up
// by timestamp (src/lsm/scan_lookup.zig:134-208): the transfers themselves, or
// the account-history rows stored under the same timestamps (:311-316, :756-808).
//
// Here the two index trees are one sorted array of (account row, transfer row)
// entries, two per stored transfer (bit 0 of the value: 0 debit side, 1 credit
// side).  Stored transfer rows are in commit order, which is timestamp order, so
// an account's entries sorted by row are its transfers sorted by timestamp, both
// sides already merged.  The array is built like an LSM level structure: each
// compaction (tbgpu_compact, the analogue of StateMachine.compact :930-955) sorts
// the rows committed since the previous one into a new run, and runs of similar
// size are merged (a stable re-sort of their union), so there are O(log n) runs
// of geometrically decreasing size.  Run k covers rows [runs[k], runs[k+1]) and
// sits at entries [2 runs[k], 2 runs[k+1]): a query visits the runs in row order
// and concatenates their segments.
//
// One workgroup per filter: binary searches bound the account's segment in each
// run and narrow it to the timestamp range; the segment is then walked in
// chunks of 256 entries (a block-wide ballot compaction keeps order) until the
// limit is met, and the selected rows are copied out 16 B per lane.
#include "common.h"
#include "engine.h"
#include "query.h"

namespace {

constexpr int Q_THREADS = 256;
constexpr int Q_WAVES = Q_THREADS / 64;

// Entries of the rows [row0, row0 + n): (debit account row, 2r), (credit account
// row, 2r + 1), in row order.  Imported rows (another shard's, sharded commit)
// are not this shard's transfers: their keys are `invalid` (sorted last, never
// matched).
__global__ void q_entries(Tables T, u64 row0, u64 n, const u8* imported, u32 invalid, u32* key, u32* val) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const u64 r = row0 + k;
    u32 kd = invalid, kc = invalid;
    if (!imported || !imported[r]) {
        const Transfer& t = T.xrows[r];
        kd = acc_row(T, t.debit_account_id);
        kc = acc_row(T, t.credit_account_id);
        if (kd == ROW_FOREIGN) kd = invalid;  // (a shard stores transfers of its own ledgers only)
        if (kc == ROW_FOREIGN) kc = invalid;
    }
    key[2 * k] = kd;
    key[2 * k + 1] = kc;
    val[2 * k] = (u32)(r << 1);
    val[2 * k + 1] = (u32)(r << 1) | 1u;
}

// First e in [lo, hi) with key[e] >= k.
__device__ __forceinline__ u64 lb_key(const u32* key, u64 lo, u64 hi, u32 k) {
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (key[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// First e in [lo, hi) whose transfer's timestamp is >= ts (the rows of one
// account's segment ascend in timestamp).
__device__ __forceinline__ u64 lb_ts(const Tables& T, const u32* val, u64 lo, u64 hi, u64 ts) {
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (T.xrows[val[mid] >> 1].timestamp < ts) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// History row stored under timestamp ts (history rows ascend in timestamp), or NONE32.
__device__ __forceinline__ u32 hist_at(const Tables& T, u64 n_hist, u64 ts) {
    u64 lo = 0, hi = n_hist;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (T.hrows[mid].timestamp < ts) lo = mid + 1; else hi = mid;
    }
    return lo < n_hist && T.hrows[lo].timestamp == ts ? (u32)lo : NONE32;
}

// get_scan_from_filter's validity test (src/state_machine.zig:822-833).
__device__ __forceinline__ bool filter_valid(const tbgpu_account_filter_t& f) {
    const u128 id = ((u128)f.account_id.hi << 64) | f.account_id.lo;
    bool reserved_zero = true;
    for (int k = 0; k < 24; k++) reserved_zero &= f.reserved[k] == 0;
    return id != 0 && id != U128_MAX && f.timestamp_min != ~0ull && f.timestamp_max != ~0ull &&
           (f.timestamp_max == 0 || f.timestamp_min <= f.timestamp_max) && f.limit != 0 &&
           (f.flags & (TBGPU_ACCOUNT_FILTER_DEBITS | TBGPU_ACCOUNT_FILTER_CREDITS)) != 0 && (f.flags >> 3) == 0 &&
           reserved_zero;
}

__global__ __launch_bounds__(Q_THREADS) void q_scan(Tables T, QIndex X, QArgs A) {
    __shared__ u32 s_sel[TBGPU_QUERY_MAX];  // selected transfer (or history) rows, in output order
    __shared__ u32 s_wcnt[Q_WAVES];
    __shared__ u32 s_acc, s_lim, s_n;
    __shared__ u64 s_lo, s_hi;
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32 q = blockIdx.x;
    const tbgpu_account_filter_t f = A.filters[q];
    const u128 fid = ((u128)f.account_id.hi << 64) | f.account_id.lo;
    if (tid == 0) {
        u32 acc = filter_valid(f) ? acc_row(T, fid) : NONE32;
        if (acc == ROW_FOREIGN) acc = NONE32;  // another ledger shard's account: its owner answers
        // get_account_history: the account must exist and keep history (:756-797)
        if (A.history && acc != NONE32 && !(T.acc[acc].flags & AF_HISTORY)) acc = NONE32;
        s_acc = acc;
        s_lim = min(min(f.limit, (u32)TBGPU_QUERY_MAX), A.stride);
        s_n = 0;
    }
    __syncthreads();
    const u32 acc = s_acc, lim = s_lim;
    if (acc != NONE32) {
        // TimestampRange with 0 = unbounded (src/lsm/timestamp_range.zig:4-5)
        const u64 tlo = f.timestamp_min == 0 ? 1ull : f.timestamp_min;
        const u64 thi = f.timestamp_max == 0 ? ~0ull - 1 : f.timestamp_max;
        const bool rev = f.flags & TBGPU_ACCOUNT_FILTER_REVERSED;
        const bool want_dr = f.flags & TBGPU_ACCOUNT_FILTER_DEBITS, want_cr = f.flags & TBGPU_ACCOUNT_FILTER_CREDITS;
        const u64 lt = __lanemask_lt();
        for (u32 kk = 0; kk < X.nruns; kk++) {
            if (s_n >= lim) break;  // uniform (written before a barrier)
            const u32 k = rev ? X.nruns - 1 - kk : kk;
            if (tid == 0) {
                const u64 e0 = 2 * X.runs[k], e1 = 2 * X.runs[k + 1];
                u64 lo = lb_key(X.key, e0, e1, acc);
                u64 hi = lb_key(X.key, lo, e1, acc + 1);
                lo = lb_ts(T, X.val, lo, hi, tlo);
                hi = lb_ts(T, X.val, lo, hi, thi + 1);
                s_lo = lo;
                s_hi = hi;
            }
            __syncthreads();
            const u64 lo = s_lo, len = s_hi - s_lo;
            for (u64 base = 0; base < len; base += Q_THREADS) {
                const u32 have = s_n;
                if (have >= lim) break;  // uniform
                const u64 j = base + tid;
                bool m = false;
                u32 sel = 0;
                if (j < len) {
                    const u32 v = X.val[rev ? lo + len - 1 - j : lo + j];
                    m = (v & 1u) ? want_cr : want_dr;
                    sel = v >> 1;
                    if (m && A.history) {
                        // the history row stored under the transfer's timestamp; post/void
                        // transfers store none (:1342-1364 only in create_transfer), where
                        // the reference's lookup asserts (scan_lookup.zig:179, :215): skipped
                        sel = hist_at(T, A.n_hist, T.xrows[sel].timestamp);
                        m = sel != NONE32;
                    }
                }
                const u64 bal = __ballot(m);
                if (lane == 0) s_wcnt[wave] = __popcll(bal);
                __syncthreads();
                u32 off = have, tot = 0;
                for (u32 w = 0; w < Q_WAVES; w++) {
                    if (w < wave) off += s_wcnt[w];
                    tot += s_wcnt[w];
                }
                off += __popcll(bal & lt);
                if (m && off < lim) s_sel[off] = sel;
                __syncthreads();
                if (tid == 0) s_n = min(have + tot, lim);
                __syncthreads();
            }
            __syncthreads();  // s_lo / s_hi are rewritten by the next run
        }
    }
    __syncthreads();
    const u32 n = acc == NONE32 ? 0 : s_n;
    if (!A.history) {
        // whole rows, 16 B per lane: 32 rows per pass of the workgroup
        uint4* out = (uint4*)((Transfer*)A.out + (u64)q * A.stride);
        for (u32 k = tid; k < n * 8; k += Q_THREADS)
            out[k] = ((const uint4*)&T.xrows[s_sel[k >> 3]])[k & 7];
    } else {
        // execute_get_account_history (:1171-1192): the filter account's side
        tbgpu_account_balance_t* out = (tbgpu_account_balance_t*)A.out + (u64)q * A.stride;
        for (u32 k = tid; k < n; k += Q_THREADS) {
            const History& h = T.hrows[s_sel[k]];
            const bool dr = h.dr_account_id == fid;
            const u128 v[4] = {dr ? h.dr_debits_pending : h.cr_debits_pending,
                               dr ? h.dr_debits_posted : h.cr_debits_posted,
                               dr ? h.dr_credits_pending : h.cr_credits_pending,
                               dr ? h.dr_credits_posted : h.cr_credits_posted};
            tbgpu_account_balance_t b{};
            tbgpu_uint128_t* w = &b.debits_pending;
            for (int x = 0; x < 4; x++) w[x] = {(u64)v[x], (u64)(v[x] >> 64)};
            b.timestamp = h.timestamp;
            out[k] = b;
        }
    }
    if (tid == 0) A.counts[q] = n;
}

}  // namespace

void q_launch_entries(const Tables& T, u64 row0, u64 n, const u8* imported, u32 invalid, u32* key, u32* val,
                      hipStream_t stream) {
    if (!n) return;
    q_entries<<<(u32)((n + 255) / 256), 256, 0, stream>>>(T, row0, n, imported, invalid, key, val);
    HIP_CHECK(hipGetLastError());
}

void q_launch_scan(const Tables& T, const QIndex& X, const QArgs& A, hipStream_t stream) {
    if (!A.nq) return;
    q_scan<<<A.nq, Q_THREADS, 0, stream>>>(T, X, A);
    HIP_CHECK(hipGetLastError());
}
