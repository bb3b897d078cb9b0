// route.hip — the send side of a routed step (tigerbeetle_amd/shard.py).
//
// A rank's client batches go to the owners of their ledgers (owner = ledger %
// world: a valid transfer has dr.ledger == cr.ledger == t.ledger,
// src/state_machine.zig:1280-1281).  Before the all-to-all every event is placed in
// an owner-major send buffer, in event order within an owner (each owner commits
// its sub-batches in global order), beside an 8-byte side record carrying what
// `execute` derives from the event's place in its batch (:1018-1035), packed as
// include/tbgpu.h TBGPU_ROUTE_REC_* describes:
//   global batch << 32 | chain start (index of the chain's first member) << 15 |
//   ends its chain << 14 | chain spans owners << 13 | index in its batch.
// The owner derives the timestamp T - n + index + 1 from the batch's (T, n), which
// every rank knows (tbgpu_route_unpack).  On several ranks the all-to-all moves the
// packed wire format: only the 4-byte words that are nonzero in some event of the
// step (the union mask the first pass finds), then the record's low word (the owner
// knows each row's batch from the per-(owner, batch) counts): 64 bytes per config-4
// event instead of 128 + 8 (rt_scatter's packed mode, rt_unpack_rows).
// Launches: classify + stable rank within the workgroup (with the step's
// eligibility figures and nonzero-word mask in the same pass over the events), an
// exclusive scan of the (owner, workgroup) counts, scatter.  Pure data movement:
// HBM-bound.
#include "common.h"

namespace {

constexpr int RT_THREADS = 256;
constexpr int RT_WAVES = RT_THREADS / 64;

struct RouteArgs {
    const Transfer* ev;
    u64 n;
    u32 world;
    u32 nb;
    const u32* b_start;   // [nb + 1] first event of each local batch
    u64 g0;               // global number of the first local batch
    uint2* orank;         // [n] owner, rank within (workgroup, owner)
    u32* blk;             // [world * nblk] per-owner counts, then their exclusive scan
    u32 nblk;
    u64* counts;          // [world] events per owner
    Transfer* out_ev;
    u64* out_side;        // [n * 4]
    u32* bcount;          // [world * nb] events per (owner, local batch)
    u32* scount;          // [world] events per owner whose chain spans owners
    u64* stats;           // rt_rank: the eligibility figures of rt_stats (out[0..4]), or null
    // packed wire format (pack_mask != 0): per event the 4-byte words of `pack_mask`
    // in word order, then the record's low word (the owner knows the batch), in
    // out_packed; a nonzero word outside the mask sets *error (nothing is lost silently)
    u32 pack_mask;
    u32* out_packed;
    u32* error;
};

constexpr u64 REC_POS = TBGPU_ROUTE_REC_POS, REC_SPAN = TBGPU_ROUTE_REC_SPAN, REC_LAST = TBGPU_ROUTE_REC_LAST;
constexpr int REC_CS_SHIFT = TBGPU_ROUTE_REC_CS_SHIFT;
static_assert(TBGPU_ROUTE_REC_BATCH_SHIFT == 32, "record layout");

__device__ __forceinline__ u32 rt_batch(const RouteArgs& A, u32 i) {
    u32 lo = 0, hi = A.nb;  // last b with b_start[b] <= i
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) / 2;
        if (A.b_start[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ u32 rt_owner(const RouteArgs& A, u64 i) { return A.ev[i].ledger % A.world; }

__device__ void rt_stats_block(u64 mn, u64 mx, u64 fl, u64 slo, u64 shi, u64* out, u64* part);

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(RT_THREADS) void rt_rank(RouteArgs A) {
    __shared__ u32 s_cnt[RT_WAVES][256];
    // the wave's 64 events' id, amount and ledger|code|flags words, loaded eight lanes
    // per row (coalesced: lane-per-row loads of 128-byte-strided rows ran 5x slower)
    __shared__ uint4 s_pc[RT_WAVES][64][3];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 i = (u64)blockIdx.x * RT_THREADS + tid;
    const u64 wbase = i - lane;
    const bool v = i < A.n;
    // with the figures, every piece is read: the step's nonzero 4-byte words (the
    // packed wire format's mask) come from the same pass
    u32 nzw = 0;
    {
        const uint4* rows = (const uint4*)A.ev;
        const u32 piece = lane & 7;
        const int slot = piece == 0 ? 0 : piece == 3 ? 1 : piece == 7 ? 2 : -1;
        const int sl = A.stats ? slot : (piece == 7 ? 2 : -1);  // without the figures: the ledger word
        uint4 x[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u32 k = (u32)r * 8 + (lane >> 3);
            x[r] = make_uint4(0, 0, 0, 0);
            if ((A.stats || sl >= 0) && wbase + k < A.n) x[r] = rows[(wbase + k) * 8 + piece];
        }
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u32 k = (u32)r * 8 + (lane >> 3);
            if (sl >= 0 && wbase + k < A.n) s_pc[w][k][sl] = x[r];
            nzw |= (x[r].x ? 1u : 0u) | (x[r].y ? 2u : 0u) | (x[r].z ? 4u : 0u) | (x[r].w ? 8u : 0u);
        }
        nzw <<= 4 * piece;
    }
    uint4 pidv = make_uint4(0, 0, 0, 0);
    if (A.stats && lane == 0 && v && i > 0) pidv = *(const uint4*)&A.ev[i - 1].id;
    for (u32 o = tid; o < A.world; o += RT_THREADS)
        for (int k = 0; k < RT_WAVES; k++) s_cnt[k][o] = 0;
    wave_lds_sync();
    const uint4 lw = s_pc[w][lane][2];
    const u64 lcf = v ? ((u64)lw.y << 32 | lw.x) : 0;  // bytes 112..119: ledger, code, flags
    uint4 idv = make_uint4(0, 0, 0, 0), amv = idv;
    if (A.stats && v) {
        idv = s_pc[w][lane][0];
        amv = s_pc[w][lane][1];
    }
    __syncthreads();
    const u32 own = v ? (u32)lcf % A.world : NONE32;
    if (A.stats) {
        const u64 lo = ((u64)idv.y << 32) | idv.x, hi = ((u64)idv.w << 32) | idv.z;
        u64 plo = (u64)__shfl_up((unsigned long long)lo, 1), phi = (u64)__shfl_up((unsigned long long)hi, 1);
        if (lane == 0) {
            plo = ((u64)pidv.y << 32) | pidv.x;
            phi = ((u64)pidv.w << 32) | pidv.z;
        }
        u64 mn = ~0ull, mx = 0, fl = (u64)nzw << 16, slo = 0, shi = 0;
        if (v) {
            mn = mx = lo;
            if (hi != 0 || lo == 0) fl |= 2;
            if (i > 0 && !(phi < hi || (phi == hi && plo < lo))) fl |= 1;
            const u64 alo = ((u64)amv.y << 32) | amv.x, ahi = ((u64)amv.w << 32) | amv.z;
            if (ahi) fl |= 8;
            slo = alo;
            shi = ahi;
            if ((lcf >> 48) & (TF_POST | TF_VOID)) fl |= 4;
        }
        rt_stats_block(mn, mx, fl, slo, shi, nullptr, A.stats);  // per-workgroup records: rt_stats_fold
    }
    // stable rank within the wave: one ballot per distinct owner present in the wave
    u32 rank = 0;
    u64 todo = __ballot(v);
    while (todo) {
        const u32 o = __shfl(own, __ffsll((unsigned long long)todo) - 1);
        const u64 m = __ballot(own == o);
        if (own == o) rank = __popcll(m & ((1ull << lane) - 1));
        if (lane == 0) s_cnt[w][o] = __popcll(m);
        todo &= ~m;
    }
    __syncthreads();
    if (v) {
        for (u32 k = 0; k < w; k++) rank += s_cnt[k][own];
        A.orank[i] = make_uint2(own, rank);
    }
    for (u32 o = tid; o < A.world; o += RT_THREADS) {
        u32 t = 0;
        for (int k = 0; k < RT_WAVES; k++) t += s_cnt[k][o];
        A.blk[(u64)o * A.nblk + blockIdx.x] = t;
    }
}

// Exclusive scan of blk (owner-major), one workgroup per owner row: row o's
// exclusive prefix in place and its total in counts[o] (the owner offsets, an
// exclusive scan of the totals, are summed by the scatter itself).  Tiles of 4096
// words, four consecutive words per thread (coalesced), wave scans by shuffles, the
// sixteen wave sums through LDS, a running carry.  (One workgroup over every row was a
// serial tail of the step at eight ranks: 256k words.)
__global__ __launch_bounds__(1024) void rt_scan(RouteArgs A) {
    __shared__ u32 wsum[16];
    const u32 o = blockIdx.x;
    u32* row = A.blk + (u64)o * A.nblk;
    const u64 total_n = A.nblk;
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u64 carry = 0;
    for (u64 base = 0; base < total_n; base += 4096) {
        const u64 k = base + (u64)tid * 4;
        u32 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = k + j < total_n ? row[k + j] : 0u;
        const u32 s = v[0] + v[1] + v[2] + v[3];
        u32 x = s;  // inclusive over the wave
        for (int off = 1; off < 64; off <<= 1) {
            const u32 y = __shfl_up(x, off);
            if (lane >= (u32)off) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        if (wave == 0) {
            u32 t = lane < 16 ? wsum[lane] : 0;
            for (int off = 1; off < 16; off <<= 1) {
                const u32 y = __shfl_up(t, off);
                if (lane >= (u32)off) t += y;
            }
            if (lane < 16) wsum[lane] = t;
        }
        __syncthreads();
        u32 run = (u32)carry + (wave ? wsum[wave - 1] : 0) + x - s;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (k + j < total_n) row[k + j] = run;
            run += v[j];
        }
        carry += wsum[15];
        __syncthreads();
    }
    if (tid == 0) A.counts[o] = carry;
}

// The scatter.  The workgroup's 256 rows are staged in LDS by coalesced 16-byte loads
// (eight lanes per row); every event then reads its own and its chain's flags and
// owners from there (a chain reaching past the workgroup reads the rows it needs
// from memory: lane-per-row loads of 128-byte-strided rows ran 5x slower than the
// staged ones), and the rows leave LDS for their owners' runs: whole rows, 16 bytes
// per lane, or packed (the 8-byte words of pack_mask, then the record), 8 bytes per
// lane over consecutive words.
__global__ __launch_bounds__(RT_THREADS) void rt_scatter(RouteArgs A) {
    __shared__ uint4 s_rows[RT_THREADS][8];  // 32 KiB
    __shared__ u32 s_om[RT_THREADS];         // owner << 1 | linked
    __shared__ u32 s_dst[RT_THREADS];
    __shared__ u64 s_rec[RT_THREADS];
    __shared__ u32 s_b0;
    __shared__ u8 s_sel[32];                 // the packed row's word k is row word s_sel[k]
    __shared__ u32 s_obase[256];             // each owner's first row: exclusive scan of the owner totals
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 blk0 = blockIdx.x * RT_THREADS;
    if (tid == 0) {
        u32 acc = 0;
        for (u32 o = 0; o < A.world; o++) {
            s_obase[o] = acc;
            acc += (u32)A.counts[o];
        }
    }
    const u64 i = (u64)blk0 + tid;
    const u64 wbase = i - lane;
    if (tid == 0) {
        // the workgroup's first batch by one binary search; each event steps on from it
        s_b0 = rt_batch(A, blk0);
        u32 k = 0;
        for (u32 wd = 0; wd < 32; wd++)
            if (A.pack_mask >> wd & 1) s_sel[k++] = (u8)wd;
    }
    {
        const uint4* src = (const uint4*)A.ev;
        const u32 piece = lane & 7;
        uint4 x[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u32 k = (u32)r * 8 + (lane >> 3);
            x[r] = wbase + k < A.n ? src[(wbase + k) * 8 + piece] : make_uint4(0, 0, 0, 0);
        }
        u32 lost = 0;  // nonzero words the packed format would drop
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u32 k = (u32)r * 8 + (lane >> 3);
            s_rows[w * 64 + k][piece] = x[r];
            lost |= (x[r].x ? 1u : 0u) | (x[r].y ? 2u : 0u) | (x[r].z ? 4u : 0u) | (x[r].w ? 8u : 0u);
        }
        if (A.pack_mask && ((lost << 4 * piece) & ~A.pack_mask)) atomicOr(A.error, 1u);
    }
    uint2 orr = make_uint2(0, 0);
    const bool v = i < A.n;
    if (v) orr = A.orank[i];
    __syncthreads();
    {
        const uint4 p7 = s_rows[tid][7];  // bytes 112..127: ledger, code, flags, timestamp
        s_om[tid] = (p7.x % A.world) << 1 | ((p7.y >> 16) & TF_LINKED);
    }
    __syncthreads();
    if (v) {
        const u32 dst = s_obase[orr.x] + A.blk[(u64)orr.x * A.nblk + blockIdx.x] + orr.y;
        s_dst[tid] = dst;
        // the record: position, chain start, span / end bits, global batch
        u32 b = s_b0;
        while (A.b_start[b + 1] <= (u32)i) b++;
        const u32 bs = A.b_start[b], be = A.b_start[b + 1];
        const u32 pos = (u32)i - bs, nbatch = be - bs;
        const u64 g = A.g0 + b;
        auto om = [&](u32 j) -> u32 {
            const u32 t = j - blk0;
            return t < RT_THREADS ? s_om[t] : (rt_owner(A, j) << 1 | (A.ev[j].flags & TF_LINKED));
        };
        u32 s = (u32)i, e = (u32)i;
        while (s > bs && (om(s - 1) & 1)) s--;
        while (e + 1 < be && (om(e) & 1)) e++;
        u32 omin = orr.x, omax = orr.x;
        for (u32 j = s; j <= e; j++) {
            const u32 o = om(j) >> 1;
            omin = min(omin, o);
            omax = max(omax, o);
        }
        const bool last = !(s_om[tid] & 1) || pos == nbatch - 1;
        const bool sp = omin != omax;
        s_rec[tid] = (g << 32) | ((u64)(s - bs) << REC_CS_SHIFT) | (last ? REC_LAST : 0) | (sp ? REC_SPAN : 0) | pos;
        // per (owner, batch) and per-owner spanning counts: one atomic per distinct key per wave
        const u32 key = orr.x * A.nb + b;
        const u64 live = __ballot(true);
        u64 todo = live;
        while (todo) {
            const u32 k = __shfl(key, __ffsll((unsigned long long)todo) - 1);
            const u64 mk = __ballot(key == k);
            if (key == k && lane == (u32)__ffsll((unsigned long long)mk) - 1) atomicAdd(&A.bcount[k], (u32)__popcll(mk));
            todo &= ~mk;
        }
        todo = __ballot(sp);
        while (todo) {
            const u32 o = __shfl(orr.x, __ffsll((unsigned long long)todo) - 1);
            const u64 mo = __ballot(sp && orr.x == o);
            if (sp && orr.x == o && lane == (u32)__ffsll((unsigned long long)mo) - 1)
                atomicAdd(&A.scount[o], (u32)__popcll(mo));
            todo &= ~mo;
        }
    }
    __syncthreads();
    const u32 nv = (u32)min<u64>(64, A.n > wbase ? A.n - wbase : 0);  // the wave's rows
    if (!A.pack_mask) {
        uint4* out = (uint4*)A.out_ev;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u32 k = (u32)r * 8 + (lane >> 3);
            if (k < nv) out[(u64)s_dst[w * 64 + k] * 8 + (lane & 7)] = s_rows[w * 64 + k][lane & 7];
        }
        if (v) A.out_side[s_dst[tid]] = s_rec[tid];
        return;
    }
    const u32 K = (u32)__popc(A.pack_mask) + 1;  // words per packed row
    for (u32 f = lane; f < nv * K; f += 64) {
        const u32 rr = f / K, wd = f - rr * K, row = w * 64 + rr;
        const u32 val = wd + 1 < K ? ((const u32*)&s_rows[row][0])[s_sel[wd]] : (u32)s_rec[row];
        A.out_packed[(u64)s_dst[row] * K + wd] = val;
    }
}

// The owner side of the packed format: rows of K = popcount(mask) + 1 words back to
// whole 128-byte rows (the words outside the mask are zero), the records (global
// batch from the sub-batch the row falls in: the owner's sub-batches are in global
// order, `sub_off[k]` the first row of sub-batch k, `sub_g[k]` its global batch), and
// each event's timestamp ts_base[g] + index + 1 (src/vsr/replica.zig:5148-5157).
__global__ __launch_bounds__(RT_THREADS) void rt_unpack_rows(const u32* __restrict__ packed, u64 m, u32 mask,
                                                             const u32* __restrict__ sub_off,
                                                             const u32* __restrict__ sub_g, u32 nsub,
                                                             const u64* __restrict__ ts_base, u64 batches,
                                                             Transfer* __restrict__ rows, u64* __restrict__ rec,
                                                             u64* __restrict__ ts, u32* error) {
    __shared__ uint4 s_rows[RT_THREADS][8];
    __shared__ u8 s_sel[32];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 i = (u64)blockIdx.x * RT_THREADS + tid;
    const u64 wbase = i - lane;
    const u32 K = (u32)__popc(mask) + 1;
    if (tid == 0) {
        u32 k = 0;
        for (u32 wd = 0; wd < 32; wd++)
            if (mask >> wd & 1) s_sel[k++] = (u8)wd;
    }
#pragma unroll
    for (int p = 0; p < 8; p++) s_rows[tid][p] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const u32 nv = (u32)min<u64>(64, m > wbase ? m - wbase : 0);
    for (u32 f = lane; f < nv * K; f += 64) {
        const u32 rr = f / K, wd = f - rr * K;
        const u32 val = packed[wbase * K + f];
        if (wd + 1 < K) {
            ((u32*)&s_rows[w * 64 + rr][0])[s_sel[wd]] = val;
        } else {
            const u32 j = (u32)(wbase + rr);
            u32 lo = 0, hi = nsub;  // the last sub-batch starting at or before row j
            while (hi - lo > 1) {
                const u32 mid = (lo + hi) / 2;
                if (sub_off[mid] <= j) lo = mid; else hi = mid;
            }
            const u64 g = sub_g[lo];
            rec[j] = (g << 32) | val;
            if (g >= batches || nsub == 0 || j >= sub_off[nsub]) {
                atomicOr(error, 1u);
                ts[j] = 0;
            } else {
                ts[j] = ts_base[g] + (val & REC_POS) + 1;
            }
        }
    }
    __syncthreads();
    uint4* out = (uint4*)rows;
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const u32 k = (u32)r * 8 + (lane >> 3);
        if (k < nv) out[(wbase + k) * 8 + (lane & 7)] = s_rows[w * 64 + k][lane & 7];
    }
}

// Timestamps of received events from their side records: batch g's events get
// ts_base[g] + index + 1, where ts_base[g] = T_g - n_g (src/vsr/replica.zig:5148-5157).
__global__ __launch_bounds__(RT_THREADS) void rt_unpack(const u64* __restrict__ rec, u64 n,
                                                        const u64* __restrict__ ts_base, u64 batches,
                                                        u64* __restrict__ ts, u32* error) {
    const u64 i = (u64)blockIdx.x * RT_THREADS + threadIdx.x;
    if (i >= n) return;
    const u64 r = rec[i], g = r >> 32;
    if (g >= batches) {
        atomicOr(error, 1u);
        return;
    }
    ts[i] = ts_base[g] + (r & REC_POS) + 1;
}

// Eligibility of a step for the device path, in one pass over its events:
// out[0] min id (low word), out[1] max id, out[2] bit 0: some id not above its
// predecessor, bit 1: some id with a high word or zero, bit 2: a post/void,
// bit 3: an amount with a high word; out[3..4] the sum of the amounts (u128).
__global__ __launch_bounds__(RT_THREADS) void rt_stats(const Transfer* ev, u64 n, u64* out) {
    // eight lanes per row, one 16-byte piece each (coalesced): piece 0 is the id,
    // piece 3 the amount, piece 7 holds the flags
    u64 mn = ~0ull, mx = 0, fl = 0, slo = 0, shi = 0;
    const u32 lane = threadIdx.x & 63, piece = lane & 7;
    const uint4* rows = (const uint4*)ev;
    const u64 waves = (u64)gridDim.x * (RT_THREADS / 64);
    constexpr int U = 4;  // rounds in flight per wave
    for (u64 r0 = (u64)blockIdx.x * (RT_THREADS / 64) + (threadIdx.x >> 6); r0 * 8 < n; r0 += U * waves) {
        uint4 v[U], pv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const u64 i = (r0 + u * waves) * 8 + (lane >> 3);
            v[u] = i < n ? rows[i * 8 + piece] : make_uint4(0, 0, 0, 0);
            pv[u] = piece == 0 && i < n && i > 0 ? rows[(i - 1) * 8] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const u64 i = (r0 + u * waves) * 8 + (lane >> 3);
            if (i >= n) continue;
            const u64 lo = ((u64)v[u].y << 32) | v[u].x, hi = ((u64)v[u].w << 32) | v[u].z;
            if (piece == 0) {
                mn = min(mn, lo);
                mx = max(mx, lo);
                if (hi != 0 || lo == 0) fl |= 2;
                const u64 plo = ((u64)pv[u].y << 32) | pv[u].x, phi = ((u64)pv[u].w << 32) | pv[u].z;
                if (i > 0 && !(phi < hi || (phi == hi && plo < lo))) fl |= 1;
            } else if (piece == 3) {
                if (hi) fl |= 8;
                slo += lo;
                shi += hi + (slo < lo ? 1 : 0);
            } else if (piece == 7) {
                if ((v[u].y >> 16) & (TF_POST | TF_VOID)) fl |= 4;
            }
            fl |= (u64)((v[u].x ? 1u : 0u) | (v[u].y ? 2u : 0u) | (v[u].z ? 4u : 0u) | (v[u].w ? 8u : 0u))
                  << (16 + 4 * piece);
        }
    }
    rt_stats_block(mn, mx, fl, slo, shi, out, nullptr);
}

// The workgroup's eligibility figures, then one set of atomics per workgroup
// (same-address atomics serialize: one set per wave cost more than the pass over
// the rows), or, with `part`, the workgroup's record part[5 * block] for
// rt_stats_fold (a grid of one workgroup per 256 events: 32k sets of atomics on five
// words took 1.5 ms).  Every thread of the workgroup calls.
__device__ void rt_stats_block(u64 mn, u64 mx, u64 fl, u64 slo, u64 shi, u64* out, u64* part) {
    const u32 lane = threadIdx.x & 63;
    for (int off = 32; off > 0; off >>= 1) {
        mn = min(mn, (u64)__shfl_xor((unsigned long long)mn, off));
        mx = max(mx, (u64)__shfl_xor((unsigned long long)mx, off));
        fl |= (u64)__shfl_xor((unsigned long long)fl, off);
        const u64 olo = (u64)__shfl_xor((unsigned long long)slo, off);
        const u64 ohi = (u64)__shfl_xor((unsigned long long)shi, off);
        const u64 t = slo + olo;
        shi += ohi + (t < slo ? 1 : 0);
        slo = t;
    }
    __shared__ u64 s_r[RT_THREADS / 64][5];
    const u32 w = threadIdx.x >> 6;
    if (lane == 0) {
        s_r[w][0] = mn; s_r[w][1] = mx; s_r[w][2] = fl; s_r[w][3] = slo; s_r[w][4] = shi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < RT_THREADS / 64; k++) {
            mn = min(mn, s_r[k][0]);
            mx = max(mx, s_r[k][1]);
            fl |= s_r[k][2];
            const u64 t = slo + s_r[k][3];
            shi += s_r[k][4] + (t < slo ? 1 : 0);
            slo = t;
        }
        if (part) {
            u64* r = part + 5ull * blockIdx.x;
            r[0] = mn; r[1] = mx; r[2] = fl; r[3] = slo; r[4] = shi;
            return;
        }
        atomicMin((unsigned long long*)&out[0], (unsigned long long)mn);
        atomicMax((unsigned long long*)&out[1], (unsigned long long)mx);
        if (fl) atomicOr((unsigned long long*)&out[2], (unsigned long long)fl);
        if (slo || shi) {
            const u64 old = atomicAdd((unsigned long long*)&out[3], (unsigned long long)slo);
            atomicAdd((unsigned long long*)&out[4], (unsigned long long)(shi + (old + slo < old ? 1 : 0)));
        }
    }
}

// The workgroup records of rt_rank into out[0..4]: one workgroup per 64 records,
// each folding its records and adding them to out with one set of atomics.
__global__ __launch_bounds__(RT_THREADS) void rt_stats_fold(const u64* __restrict__ part, u32 nblk, u64* out) {
    u64 mn = ~0ull, mx = 0, fl = 0, slo = 0, shi = 0;
    for (u32 b = blockIdx.x * 64 + threadIdx.x; threadIdx.x < 64 && b < nblk; b += (u32)gridDim.x * 64) {
        const u64* r = part + 5ull * b;
        mn = min(mn, r[0]);
        mx = max(mx, r[1]);
        fl |= r[2];
        const u64 t = slo + r[3];
        shi += r[4] + (t < slo ? 1 : 0);
        slo = t;
    }
    rt_stats_block(mn, mx, fl, slo, shi, out, nullptr);
}

}  // namespace

void route_stats(const Transfer* ev, u64 n, u64* out, hipStream_t stream) {
    // {~0, 0, 0, 0, 0}, set on the device (no host source)
    HIP_CHECK(hipMemsetAsync(out, 0xFF, sizeof(u64), stream));
    HIP_CHECK(hipMemsetAsync(out + 1, 0, 4 * sizeof(u64), stream));
    if (n) rt_stats<<<(u32)std::min<u64>((n + RT_THREADS / 8 - 1) / (RT_THREADS / 8), 1024), RT_THREADS, 0, stream>>>(ev, n, out);
    HIP_CHECK(hipGetLastError());
}

u64 route_block_count(u64 n) { return (n + RT_THREADS - 1) / RT_THREADS; }

// rt_rank alone, with the eligibility figures (stats: 5 words, initialized here):
// the first half of a routed step's send side; route_scatter(..., ranked = true)
// completes it.
// part: 5 words per workgroup (route_block_count(n) of them)
void route_rank(const Transfer* ev, u64 n, u32 world, uint2* orank, u32* blk, u64* part, u64* stats,
                hipStream_t stream) {
    HIP_CHECK(hipMemsetAsync(stats, 0xFF, sizeof(u64), stream));
    HIP_CHECK(hipMemsetAsync(stats + 1, 0, 4 * sizeof(u64), stream));
    RouteArgs A{};
    A.ev = ev; A.n = n; A.world = world; A.orank = orank; A.blk = blk; A.nblk = (u32)route_block_count(n);
    A.stats = part;
    if (n) {
        rt_rank<<<A.nblk, RT_THREADS, 0, stream>>>(A);
        rt_stats_fold<<<std::min<u32>((A.nblk + 63) / 64, 256), RT_THREADS, 0, stream>>>(part, A.nblk, stats);
    }
    HIP_CHECK(hipGetLastError());
}

void route_unpack(const u64* rec, u64 n, const u64* ts_base, u64 batches, u64* ts, u32* error, hipStream_t stream) {
    if (n) rt_unpack<<<(u32)((n + RT_THREADS - 1) / RT_THREADS), RT_THREADS, 0, stream>>>(rec, n, ts_base, batches,
                                                                                          ts, error);
    HIP_CHECK(hipGetLastError());
}

void route_scatter(const Transfer* ev, u64 n, u32 world, u32 nb, const u32* b_start, u64 g0,
                   uint2* orank, u32* blk, u64* counts, Transfer* out_ev, u64* out_side, u32* bcount, u32* scount,
                   u32 pack_mask, u32* out_packed, u32* error, bool ranked, hipStream_t stream) {
    RouteArgs A{};
    A.pack_mask = pack_mask;
    A.out_packed = out_packed;
    A.error = error;
    A.bcount = bcount;
    A.scount = scount;
    HIP_CHECK(hipMemsetAsync(bcount, 0, (u64)world * nb * sizeof(u32), stream));
    HIP_CHECK(hipMemsetAsync(scount, 0, world * sizeof(u32), stream));
    A.ev = ev; A.n = n; A.world = world; A.nb = nb; A.b_start = b_start; A.g0 = g0;
    A.orank = orank; A.blk = blk; A.nblk = (u32)route_block_count(n); A.counts = counts;
    A.out_ev = out_ev; A.out_side = out_side;
    if (n && !ranked) rt_rank<<<A.nblk, RT_THREADS, 0, stream>>>(A);
    if (world > 256) tbgpu_fatal("route_scatter", "more than 256 owners", __FILE__, __LINE__);
    rt_scan<<<world, 1024, 0, stream>>>(A);
    if (n) rt_scatter<<<A.nblk, RT_THREADS, 0, stream>>>(A);
    HIP_CHECK(hipGetLastError());
}

void route_unpack_rows(const u32* packed, u64 m, u32 mask, const u32* sub_off, const u32* sub_g, u32 nsub,
                       const u64* ts_base, u64 batches, Transfer* rows, u64* rec, u64* ts, u32* error,
                       hipStream_t stream) {
    if (m) rt_unpack_rows<<<(u32)((m + RT_THREADS - 1) / RT_THREADS), RT_THREADS, 0, stream>>>(
        packed, m, mask, sub_off, sub_g, nsub, ts_base, batches, rows, rec, ts, error);
    HIP_CHECK(hipGetLastError());
}
