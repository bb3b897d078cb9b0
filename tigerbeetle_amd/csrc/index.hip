// index.hip — the grooves' field index trees (src/state_machine.zig:1575-1641
// tree_options_index): for the transfers groove debit_account_id, credit_account_id,
// user_data_128/64/32, pending_id, timeout, ledger, code and amount; for the accounts
// groove user_data_128/64/32, ledger and code.  Groove.insert puts (field, timestamp)
// into a field's tree for every stored object whose field is nonzero
// (src/lsm/groove.zig:911-936); a scan of one tree with a field value as its prefix
// gives the objects with that value in timestamp order.
//
// Here each tree is an LSM-shaped array of 8-byte entries (key, object row), like the
// account-transfers index (query.hip): a 32-bit key per object — the field itself for
// fields of at most 32 bits, a nonzero hash of it for the 64- and 128-bit ones (a scan
// compares the row's full field, so a hash collision costs a read, not a wrong row) —
// with 0 for "not indexed"; runs of rows sorted by (key, row), built on demand when a
// scan of that tree arrives (engine.hip ix_extend), merged while the newest run is at
// least half as large as its predecessor.  Object rows are in timestamp order
// (transfers in commit order, accounts in creation order), so a key's segment of a run
// is already in timestamp order.
#include "common.h"
#include "engine.h"
#include "index.h"

namespace {

constexpr int IX_THREADS = 256;
constexpr int IX_WAVES = IX_THREADS / 64;

__device__ __forceinline__ u32 key_of_u128(u128 v) {
    if (v == 0) return 0;
    const u64 h = hash128((u64)v, (u64)(v >> 64));
    const u32 k = (u32)(h >> 32) ^ (u32)h;
    return k ? k : 1u;
}

// The field of object row r as (full value, 32-bit key).
__device__ __forceinline__ u128 field_value(const Tables& T, u32 kind, u32 field, u64 r) {
    if (kind == TBGPU_INDEX_TRANSFERS) {
        const Transfer& t = T.xrows[r];
        switch (field) {
            case TBGPU_INDEX_DEBIT_ACCOUNT_ID: return t.debit_account_id;
            case TBGPU_INDEX_CREDIT_ACCOUNT_ID: return t.credit_account_id;
            case TBGPU_INDEX_USER_DATA_128: return t.user_data_128;
            case TBGPU_INDEX_USER_DATA_64: return t.user_data_64;
            case TBGPU_INDEX_USER_DATA_32: return t.user_data_32;
            case TBGPU_INDEX_PENDING_ID: return t.pending_id;
            case TBGPU_INDEX_TIMEOUT: return t.timeout;
            case TBGPU_INDEX_LEDGER: return t.ledger;
            case TBGPU_INDEX_CODE: return t.code;
            default: return t.amount;  // TBGPU_INDEX_AMOUNT
        }
    }
    const Account& a = T.acc[r];
    switch (field) {
        case TBGPU_INDEX_USER_DATA_128: return a.user_data_128;
        case TBGPU_INDEX_USER_DATA_64: return a.user_data_64;
        case TBGPU_INDEX_USER_DATA_32: return a.user_data_32;
        case TBGPU_INDEX_LEDGER: return a.ledger;
        default: return a.code;  // TBGPU_INDEX_CODE
    }
}

__device__ __forceinline__ u32 field_key(u32 field, u128 v) {
    return ix_field_bits(field) <= 32 ? (u32)v : key_of_u128(v);
}

__device__ __forceinline__ u64 object_ts(const Tables& T, u32 kind, u64 r) {
    return kind == TBGPU_INDEX_TRANSFERS ? T.xrows[r].timestamp : T.acc[r].timestamp;
}

// Entries of object rows [row0, row0 + n): (key, row).  Imported transfers (another
// shard's rows, sharded commit) are not this shard's objects: key 0.
__global__ void ix_entries(Tables T, u32 kind, u32 field, u64 row0, u64 n, const u8* imported, u32* key, u32* val) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const u64 r = row0 + k;
    u32 kk = 0;
    if (kind != TBGPU_INDEX_TRANSFERS || !imported || !imported[r]) kk = field_key(field, field_value(T, kind, field, r));
    key[k] = kk;
    val[k] = (u32)r;
}

__device__ __forceinline__ u64 lb_key(const u32* key, u64 lo, u64 hi, u32 k) {
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (key[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ u64 lb_ts(const Tables& T, u32 kind, const u32* val, u64 lo, u64 hi, u64 ts) {
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (object_ts(T, kind, val[mid]) < ts) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// One workgroup: the filter's segment in every run (in row order, or reversed),
// narrowed to its timestamp range, walked in chunks with a block-wide ballot
// compaction that keeps order; rows whose full field differs (a hash collision)
// are dropped.  Then the selected rows are copied out 16 B per lane.
__global__ __launch_bounds__(IX_THREADS) void ix_scan(Tables T, IxArgs A) {
    __shared__ u32 s_sel[TBGPU_QUERY_MAX];
    __shared__ u32 s_wcnt[IX_WAVES];
    __shared__ u32 s_n;
    __shared__ u64 s_lo, s_hi;
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const tbgpu_index_filter_t f = *A.filter;
    const u128 v = ((u128)f.value.hi << 64) | f.value.lo;
    const u32 key = field_key(f.field, v);
    const u32 lim = min(f.limit, (u32)TBGPU_QUERY_MAX);
    if (tid == 0) s_n = 0;
    __syncthreads();
    if (A.valid && key != 0) {
        const u64 tlo = f.timestamp_min == 0 ? 1ull : f.timestamp_min;  // 0 = unbounded
        const u64 thi = f.timestamp_max == 0 ? ~0ull - 1 : f.timestamp_max;
        const bool rev = f.flags & TBGPU_INDEX_REVERSED;
        const u64 lt = __lanemask_lt();
        for (u32 kk = 0; kk < A.nruns; kk++) {
            if (s_n >= lim) break;  // uniform (written before a barrier)
            const u32 k = rev ? A.nruns - 1 - kk : kk;
            if (tid == 0) {
                const u64 e0 = A.runs[k], e1 = A.runs[k + 1];
                u64 lo = lb_key(A.key, e0, e1, key);
                u64 hi = key == 0xFFFFFFFFu ? e1 : lb_key(A.key, lo, e1, key + 1);
                lo = lb_ts(T, A.kind, A.val, lo, hi, tlo);
                hi = lb_ts(T, A.kind, A.val, lo, hi, thi + 1);
                s_lo = lo;
                s_hi = hi;
            }
            __syncthreads();
            const u64 lo = s_lo, len = s_hi - s_lo;
            for (u64 base = 0; base < len; base += IX_THREADS) {
                const u32 have = s_n;
                if (have >= lim) break;  // uniform
                const u64 j = base + tid;
                bool m = false;
                u32 row = 0;
                if (j < len) {
                    row = A.val[rev ? lo + len - 1 - j : lo + j];
                    m = field_value(T, A.kind, f.field, row) == v;
                }
                const u64 bal = __ballot(m);
                if (lane == 0) s_wcnt[wave] = __popcll(bal);
                __syncthreads();
                u32 off = have, tot = 0;
                for (u32 w = 0; w < IX_WAVES; w++) {
                    if (w < wave) off += s_wcnt[w];
                    tot += s_wcnt[w];
                }
                off += __popcll(bal & lt);
                if (m && off < lim) s_sel[off] = row;
                __syncthreads();
                if (tid == 0) s_n = min(have + tot, lim);
                __syncthreads();
            }
            __syncthreads();  // s_lo / s_hi are rewritten by the next run
        }
    }
    __syncthreads();
    const u32 n = s_n;
    uint4* out = (uint4*)A.out;
    const uint4* src = A.kind == TBGPU_INDEX_TRANSFERS ? (const uint4*)T.xrows : (const uint4*)T.acc;
    for (u32 k = tid; k < n * 8; k += IX_THREADS) out[k] = src[(u64)s_sel[k >> 3] * 8 + (k & 7)];
    if (tid == 0) *A.count = n;
}

}  // namespace

void ix_launch_entries(const Tables& T, u32 kind, u32 field, u64 row0, u64 n, const u8* imported, u32* key, u32* val,
                       hipStream_t stream) {
    if (!n) return;
    ix_entries<<<(u32)((n + IX_THREADS - 1) / IX_THREADS), IX_THREADS, 0, stream>>>(T, kind, field, row0, n, imported,
                                                                                    key, val);
    HIP_CHECK(hipGetLastError());
}

void ix_launch_scan(const Tables& T, const IxArgs& A, hipStream_t stream) {
    ix_scan<<<1, IX_THREADS, 0, stream>>>(T, A);
    HIP_CHECK(hipGetLastError());
}
