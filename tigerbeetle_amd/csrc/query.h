// query.h — the account-transfers index and the two account queries (query.hip).
#pragma once
#include "engine.h"

// Runs of (account row, transfer row << 1 | side) entries, sorted by account row
// within each run; run k covers the stored rows [runs[k], runs[k+1]) and sits at
// entries [2 runs[k], 2 runs[k+1]).
struct QIndex {
    const u32* key;
    const u32* val;
    const u64* runs;  // [nruns + 1], device
    u32 nruns;
};

struct QArgs {
    const tbgpu_account_filter_t* filters;  // [nq], device
    u32 nq;
    u32 stride;    // output rows reserved per filter
    void* out;     // Transfer[nq * stride] or tbgpu_account_balance_t[nq * stride]
    u32* counts;   // [nq] rows written per filter
    u32 history;   // 0 get_account_transfers, 1 get_account_history
    u64 n_hist;
};

constexpr u32 Q_RUNS_MAX = 64;

void q_launch_entries(const Tables& T, u64 row0, u64 n, const u8* imported, u32 invalid, u32* key, u32* val,
                      hipStream_t stream);
void q_launch_scan(const Tables& T, const QIndex& X, const QArgs& A, hipStream_t stream);
