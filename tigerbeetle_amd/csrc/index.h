// index.h — the grooves' field index trees (index.hip).
#pragma once
#include "engine.h"

enum : u32 { TBGPU_INDEX_TRANSFERS = 0, TBGPU_INDEX_ACCOUNTS = 1 };  // which groove

// Width of an indexed field (bits): the key is the field itself up to 32 bits, a hash above.
__host__ __device__ inline u32 ix_field_bits(u32 field) {
    switch (field) {
        case TBGPU_INDEX_USER_DATA_64: return 64;
        case TBGPU_INDEX_USER_DATA_32: case TBGPU_INDEX_TIMEOUT: case TBGPU_INDEX_LEDGER: return 32;
        case TBGPU_INDEX_CODE: return 16;
        default: return 128;
    }
}

// One scan: the filter (device), the tree's runs (run k covers entries [runs[k], runs[k+1])).
struct IxArgs {
    const tbgpu_index_filter_t* filter;
    u32 kind;
    u32 valid;       // the host's validity check of the filter (invalid: no rows)
    const u32* key;
    const u32* val;
    const u64* runs;  // device
    u32 nruns;
    void* out;        // TBGPU_QUERY_MAX objects
    u32* count;
};

void ix_launch_entries(const Tables& T, u32 kind, u32 field, u64 row0, u64 n, const u8* imported, u32* key, u32* val,
                       hipStream_t stream);
void ix_launch_scan(const Tables& T, const IxArgs& A, hipStream_t stream);
