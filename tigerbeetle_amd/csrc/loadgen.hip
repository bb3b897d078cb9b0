// loadgen.hip — the benchmark's synthetic load, generated in HBM.
//
// `tigerbeetle benchmark` creates accounts with ids 1..N on one ledger and streams
// transfers between uniformly random distinct accounts with exponentially
// distributed amounts (src/tigerbeetle/benchmark_load.zig:209-247, :266-330).
// BASELINE config 5 is that load at scale: 100M accounts over 1000 ledgers and 1B
// transfers, each transfer inside one ledger.  Generating 10^8..10^9 128-byte
// records on the host would dominate any run, so these kernels write them
// straight into device memory from a counter-based generator: record i depends
// only on (seed, first + i), so any slice can be regenerated independently and
// identically (the parity tests copy leading batches back to the host oracle).
#include "common.h"

namespace {

__device__ __forceinline__ u64 lg_mix(u64 z) {  // splitmix64 finalizer
    z ^= z >> 30;
    z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 27;
    z *= 0x94d049bb133111ebull;
    z ^= z >> 31;
    return z;
}

__global__ void lg_accounts(Account* out, u64 first_id, u64 count, u32 accounts_per_ledger) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const u64 id = first_id + i;
    Account a;
    memset(&a, 0, sizeof a);
    a.id = id;
    a.ledger = (u32)((id - 1) / accounts_per_ledger) + 1;
    a.code = 1;
    out[i] = a;
}

// Transfer `first_id + i`: a ledger among ledger0 + stride * [0, ledgers), then a
// uniform debit account and a different uniform credit account of that ledger
// (ids (ledger - 1) * accounts_per_ledger + 1 ...), amount floor(Exp(1) * 10000) + 1
// (benchmark_load.zig:304-313; src/testing/fuzz.zig:16-24), code rand_u16 +| 1,
// random user data, flags 0.
__global__ void lg_transfers(Transfer* out, u64 first_id, u64 count, u64 seed, u32 ledger0, u32 ledgers,
                             u32 ledger_stride, u32 accounts_per_ledger) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const u64 id = first_id + i;
    const u64 base = lg_mix(seed * 0x9E3779B97F4A7C15ull + id);
    const u64 r1 = lg_mix(base ^ 0x1), r2 = lg_mix(base ^ 0x2), r3 = lg_mix(base ^ 0x3), r4 = lg_mix(base ^ 0x4);
    const u64 r5 = lg_mix(base ^ 0x5), r6 = lg_mix(base ^ 0x6);
    const u32 ledger = ledger0 + ledger_stride * (u32)(base % ledgers);
    const u64 apl = accounts_per_ledger;
    const u64 dr = r1 % apl;
    u64 cr = r2 % (apl - 1);
    if (cr >= dr) cr++;
    const u64 acc0 = (u64)(ledger - 1) * apl + 1;
    // (0, 1]: 53 random bits
    const double u = ((double)(r3 >> 11) + 1.0) * (1.0 / 9007199254740992.0);
    const double ex = -log(u) * 10000.0;
    Transfer t;
    memset(&t, 0, sizeof t);
    t.id = id;
    t.debit_account_id = acc0 + dr;
    t.credit_account_id = acc0 + cr;
    t.amount = (u128)(u64)ex + 1;
    t.user_data_128 = ((u128)r4 << 64) | r5;
    t.user_data_64 = r6;
    t.user_data_32 = (u32)(r4 >> 32);
    t.ledger = ledger;
    const u32 code = (u32)(r5 & 0xFFFF) + 1;
    t.code = (u16)(code > 0xFFFF ? 0xFFFF : code);
    out[i] = t;
}

}  // namespace

extern "C" int tbgpu_bench_generate_accounts(int device, uint64_t first_id, uint64_t count,
                                             uint32_t accounts_per_ledger, void* out_device) {
    if (hipSetDevice(device) != hipSuccess || accounts_per_ledger == 0 || first_id == 0) return -22;
    if (count) lg_accounts<<<(u32)((count + 255) / 256), 256>>>((Account*)out_device, first_id, count,
                                                               accounts_per_ledger);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -5;
}

extern "C" int tbgpu_bench_generate_transfers(int device, uint64_t first_id, uint64_t count, uint64_t seed,
                                              uint32_t ledger0, uint32_t ledgers, uint32_t ledger_stride,
                                              uint32_t accounts_per_ledger, void* out_device) {
    if (hipSetDevice(device) != hipSuccess || ledgers == 0 || ledger0 == 0 || ledger_stride == 0 ||
        accounts_per_ledger < 2)
        return -22;
    if (count) lg_transfers<<<(u32)((count + 255) / 256), 256>>>((Transfer*)out_device, first_id, count, seed,
                                                                ledger0, ledgers, ledger_stride, accounts_per_ledger);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -5;
}
