// common.h — device-side types and helpers shared by the engine's HIP sources.
//
// The 128-byte Account / Transfer rows are the reference's extern structs
// (src/tigerbeetle.zig:7-40, :80-105); they are kept byte-identical so that rows
// move between the C-ABI (include/tbgpu.h) and HBM without repacking.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tbgpu.h"

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;

#define U128_MAX (~(u128)0)
#define NONE32 0xFFFFFFFFu
#define NS_PER_S 1000000000ull

struct alignas(16) Account {
    u128 id, debits_pending, debits_posted, credits_pending, credits_posted, user_data_128;
    u64 user_data_64;
    u32 user_data_32, reserved, ledger;
    u16 code, flags;
    u64 timestamp;
};
struct alignas(16) Transfer {
    u128 id, debit_account_id, credit_account_id, amount, pending_id, user_data_128;
    u64 user_data_64;
    u32 user_data_32, timeout, ledger;
    u16 code, flags;
    u64 timestamp;
};
struct alignas(16) History {
    u128 dr_account_id, dr_debits_pending, dr_debits_posted, dr_credits_pending, dr_credits_posted;
    u128 cr_account_id, cr_debits_pending, cr_debits_posted, cr_credits_pending, cr_credits_posted;
    u64 timestamp;
    u8 reserved[88];
};
static_assert(sizeof(Account) == 128, "Account layout");
static_assert(sizeof(Transfer) == 128, "Transfer layout");
static_assert(sizeof(History) == 256, "History layout");
static_assert(sizeof(Account) == sizeof(tbgpu_account_t), "ABI");
static_assert(sizeof(Transfer) == sizeof(tbgpu_transfer_t), "ABI");

// Four balances of an account (the scan state).
struct Bal4 {
    u128 dp, dpo, cp, cpo;
};

// Account flags (src/tigerbeetle.zig:42-63)
#define AF_LINKED 1u
#define AF_DNEC 2u   // debits_must_not_exceed_credits
#define AF_CNED 4u   // credits_must_not_exceed_debits
#define AF_HISTORY 8u
// Transfer flags (src/tigerbeetle.zig:107-120)
#define TF_LINKED 1u
#define TF_PENDING 2u
#define TF_POST 4u
#define TF_VOID 8u
#define TF_BDR 16u
#define TF_BCR 32u

// Static-result sentinel: the event passed every state-independent check.
#define SRES_DYN 0xFFu

// Resolved pending-transfer reference (u32): in-batch event index, or
// PREF_ROW | committed row, or NONE32.
#define PREF_ROW 0x80000000u

// splitmix64 finalizer; hash of a u128 key.
__host__ __device__ __forceinline__ u64 mix64(u64 z) {
    z ^= z >> 30;
    z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 27;
    z *= 0x94d049bb133111ebull;
    z ^= z >> 31;
    return z;
}
__host__ __device__ __forceinline__ u64 hash128(u128 k) {
    return mix64((u64)k ^ mix64((u64)(k >> 64)));
}
__host__ __device__ __forceinline__ u64 hash128(u64 lo, u64 hi) { return mix64(lo ^ mix64(hi)); }

// sum_overflows (src/state_machine.zig:1645-1650)
__device__ __forceinline__ bool sum_overflows128(u128 a, u128 b) { return a + b < a; }
__device__ __forceinline__ bool sum_overflows64(u64 a, u64 b) { return (u64)(a + b) < a; }

// Wave-level reductions (64 lanes, every lane active in the call): same-address
// device atomics serialize at the memory side (~5-10 ns each), so a kernel reduces
// over its wave first and lane 0 issues the one atomic.
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, (u64)__shfl_xor((unsigned long long)v, off));
    return v;
}
__device__ __forceinline__ u64 wave_min_u64(u64 v) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, (u64)__shfl_xor((unsigned long long)v, off));
    return v;
}
__device__ __forceinline__ u32 wave_or_u32(u32 v) {
    for (int off = 32; off > 0; off >>= 1) v |= (u32)__shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ u32 wave_sum_u32(u32 v) {
    for (int off = 32; off > 0; off >>= 1) v += (u32)__shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ bool wave_leader() { return (threadIdx.x & 63) == 0; }

#define HIP_CHECK(expr)                                                                   \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess) tbgpu_fatal(#expr, hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)

[[noreturn]] void tbgpu_fatal(const char* what, const char* why, const char* file, int line);

// ---------------------------------------------------------------- launchers --
// Radix sort of (u32 key, u32 value) pairs, stable, keys < 2^bits.
struct SortScratch {
    u32* keys_tmp;
    u32* vals_tmp;
    u32* hist;      // 256 * max_blocks
    u64 capacity;   // max items
};
// With `pred`, every kernel of the sort returns at once unless *pred & pred_mask.
void radix_sort_pairs(const u32* keys_in, const u32* vals_in, u32* keys_out, u32* vals_out, u64 n, int bits,
                      SortScratch& s, hipStream_t stream, const u32* pred = nullptr, u32 pred_mask = 0);
u64 radix_sort_hist_words(u64 capacity);

// Exclusive scan of three u32 counters packed per element from a u8 bitmask.
struct Scan3Scratch {
    uint4* tile_sums;
    u64 capacity;
};
// gate (optional): the kernels return at once while *gate == 0 (enqueued before the
// host knows whether the scan is needed)
void scan3_exclusive(const u8* mask, uint4* out, u64 n, Scan3Scratch& s, hipStream_t stream,
                     const u32* gate = nullptr);
u64 scan3_tile_words(u64 capacity);
