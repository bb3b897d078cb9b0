// directory.hip — the id directory of the router's general step, on the device.
//
// The general step (tigerbeetle_amd/shard_vec.py round_vec) decides,
// for every id and pending-id record of the step (all ranks' records, all-gathered),
// what the id already is: committed on some shard (its row's ledger owner, from each
// shard's own index: the shards are the directory of committed ids), first seen in the
// step (the earliest position among the records of ids not committed), a repeat of
// that first event, or -- for a pending id -- a pending committed elsewhere, one the
// step creates earlier, or none (src/state_machine.zig:1284 `exists`, :1409-1428 the
// pending's lookup).  On the host this was a stable sort of every record by u128 key;
// here the records are grouped by key in a hash table (no sort: only the per-key
// minimum position and the hint of that record are needed), in five launches:
//   rd_owners  : this shard's committed row for each record's key -> its owner, or -1
//                (the caller all-reduces MAX over the ranks, in place)
//   rd_init, rd_insert : the key table (claims are record indices; keys read back
//                from the records, as the call-local group table does)
//   rd_first   : per key, the earliest position among the id records of uncommitted ids
//   rd_out     : each record's (type, hint, first position), as shard_vec computes them
#include <algorithm>

#include "common.h"
#include "engine.h"

typedef int64_t i64;

namespace {

constexpr u32 RD_THREADS = 256;
constexpr i64 RD_INF = 0x7FFFFFFFFFFFFFFFll;
constexpr i64 RD_ANY = -1, RD_PV = -2;  // route hints (shard.py)
enum : i64 { RD_NEW = 0, RD_EXISTS, RD_DUP, RD_PEND, RD_PEND_NONE, RD_PEND_HAZARD };

// record r: pos, kind (0 id, 1 pending id), key lo, key hi, hint
struct Rec {
    i64 pos, kind, lo, hi, hint;
};

__global__ void rd_owners(Tables T, const Rec* __restrict__ rec, u64 n, u32 world, i64* __restrict__ owner) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u128 id = ((u128)(u64)rec[r].hi << 64) | (u64)rec[r].lo;
    const u32 row = xidx_probe(T, id);
    owner[r] = row == NONE32 ? -1 : (i64)(T.xrows[row].ledger % world);
}

__global__ void rd_init(u32* claim, i64* first_p, i64* first_h, u64 g) {
    for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < g; k += (u64)gridDim.x * blockDim.x) {
        claim[k] = 0;
        first_p[k] = RD_INF;
        first_h[k] = RD_ANY;
    }
}

__global__ void rd_insert(const Rec* __restrict__ rec, u64 n, u32* claim, u64 mask, u32* __restrict__ slot) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u64 lo = (u64)rec[r].lo, hi = (u64)rec[r].hi;
    u64 h = hash128(lo, hi) & mask;
    for (;;) {
        u32 cur = claim[h];
        if (cur == 0) {
            const u32 prev = atomicCAS(&claim[h], 0u, (u32)r + 1);
            if (prev == 0) break;
            cur = prev;
        }
        if ((u64)rec[cur - 1].lo == lo && (u64)rec[cur - 1].hi == hi) break;
        h = (h + 1) & mask;
    }
    slot[r] = (u32)h;
}

__global__ void rd_first(const Rec* __restrict__ rec, const i64* __restrict__ owner, u64 n,
                         const u32* __restrict__ slot, i64* first_p) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    if (rec[r].kind == 0 && owner[r] < 0)
        atomicMin((unsigned long long*)&first_p[slot[r]], (unsigned long long)rec[r].pos);
}

// the hint of each key's first record (positions are unique among id records)
__global__ void rd_hint(const Rec* __restrict__ rec, const i64* __restrict__ owner, u64 n,
                        const u32* __restrict__ slot, const i64* __restrict__ first_p, i64* first_h) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u32 s = slot[r];
    if (rec[r].kind == 0 && owner[r] < 0 && rec[r].pos == first_p[s]) first_h[s] = rec[r].hint;
}

__global__ void rd_out(const Rec* __restrict__ rec, const i64* __restrict__ owner, u64 n,
                       const u32* __restrict__ slot, const i64* __restrict__ first_p,
                       const i64* __restrict__ first_h, i64* __restrict__ out) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u32 s = slot[r];
    const i64 pos = rec[r].pos, own = owner[r], fp = first_p[s], fh = first_h[s];
    const bool k0 = rec[r].kind == 0;
    i64 typ;
    if (k0) typ = own >= 0 ? RD_EXISTS : (pos == fp ? RD_NEW : RD_DUP);
    else if (own >= 0) typ = RD_PEND;
    else if (fp < pos) typ = (fh == RD_ANY || fh == RD_PV) ? RD_PEND_HAZARD : RD_PEND;
    else typ = RD_PEND_NONE;
    out[3 * r + 0] = typ;
    out[3 * r + 1] = own >= 0 ? own : fh;
    out[3 * r + 2] = fp;
}

}  // namespace

#define RD_GRID(n) (u32)(((n) + RD_THREADS - 1) / RD_THREADS), RD_THREADS, 0, stream

void route_dir_owners(const Tables& T, const void* records, u64 n, u32 world, i64* owner, hipStream_t stream) {
    if (n) rd_owners<<<RD_GRID(n)>>>(T, (const Rec*)records, n, world, owner);
    HIP_CHECK(hipGetLastError());
}

// table: claims [g], then first positions [g], first hints [g]; slot [n]; g a power of two >= 2n
void route_dir_finish(const void* records, const i64* owner, u64 n, u32* claim, i64* first_p, i64* first_h, u64 g,
                      u32* slot, i64* out, hipStream_t stream) {
    if (!n) return;
    const Rec* rec = (const Rec*)records;
    rd_init<<<(u32)std::min<u64>((g + RD_THREADS - 1) / RD_THREADS, 4096), RD_THREADS, 0, stream>>>(claim, first_p,
                                                                                                    first_h, g);
    rd_insert<<<RD_GRID(n)>>>(rec, n, claim, g - 1, slot);
    rd_first<<<RD_GRID(n)>>>(rec, owner, n, slot, first_p);
    rd_hint<<<RD_GRID(n)>>>(rec, owner, n, slot, first_p, first_h);
    rd_out<<<RD_GRID(n)>>>(rec, owner, n, slot, first_p, first_h, out);
    HIP_CHECK(hipGetLastError());
}
