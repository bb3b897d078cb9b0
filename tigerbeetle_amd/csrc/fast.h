// fast.h — arguments of the single-pass create_transfers kernels (fast.hip).
#pragma once
#include "engine.h"

struct FastArgs {
    const Transfer* ev;
    u32 n;
    u32 nb;
    const u32* b_start;
    const u64* b_ts;
    u64* gtab;          // epoch-tagged duplicate-id claims
    u64 gmask;
    u64 epoch;          // (call epoch) << 32, never 0
    u8* fres;           // per-event result (0 = accepted, deltas applied)
    u32* counters;
    u64* tile_status;   // decoupled look-back: [flag:2 | failures:31 | accepted:31]
    u32* tile_counter;
    u32* batch_counts;  // failures per batch
    tb_create_transfers_result_t* results;  // replies, concatenated across batches
    u64 row_base;
    u128* keys;         // accepted ids, for fp_index
    u32* rows;          // stored row per event or NONE32
    u64* tile_idr;      // per tile: componentwise max lo, max hi, min lo, min hi of accepted ids
};

void fp_launch_commit(const Tables& T, const FastArgs& F, hipStream_t stream);
void fp_launch_index(const Tables& T, const FastArgs& F, hipStream_t stream);
void fp_launch_undo(const Tables& T, const FastArgs& F, hipStream_t stream);
u64 fp_tiles(u64 n);
