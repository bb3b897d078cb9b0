// sort.hip — stable LSD radix sort of (u32 key, u32 value) pairs, and a
// 3-counter exclusive scan.  Hand-written for gfx950 (64-wide waves, LDS tiles).
//
// Used to group event sides by account slot (the segmented balance scan walks
// each account's debits/credits in batch-index order) and, when a batch repeats
// a transfer id, to group events by id.  Input arrives in index order and the
// sort is stable, so every group comes out index-ordered.
#include "common.h"

namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_IPT = 8;
constexpr int RS_TILE = RS_THREADS * RS_IPT;  // 2048 items per workgroup
constexpr int RS_WAVES = RS_THREADS / 64;

// A sort may be predicated on a device word (pred & mask != 0), so that the host
// enqueues it without knowing whether it is needed.
__device__ __forceinline__ bool rs_off(const u32* pred, u32 mask) { return pred && !(*pred & mask); }

__global__ __launch_bounds__(RS_THREADS) void rs_hist(const u32* __restrict__ keys, u64 n, int shift,
                                                      u32* __restrict__ hist, u32 nblocks, const u32* pred, u32 pmask) {
    if (rs_off(pred, pmask)) return;
    __shared__ u32 cnt[256];
    const u32 tid = threadIdx.x;
    cnt[tid] = 0;
    __syncthreads();
    const u64 base = (u64)blockIdx.x * RS_TILE;
#pragma unroll
    for (int r = 0; r < RS_IPT; r++) {
        u64 i = base + (u64)r * RS_THREADS + tid;
        if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    hist[(u64)tid * nblocks + blockIdx.x] = cnt[tid];
}

// Exclusive scan of `total` u32 words in place (total is a multiple of 256), one
// workgroup of 1024 threads.  Up to 64k words: each thread loads a contiguous run of
// at most 16 uint4 into registers at once (independent loads, one memory latency),
// one workgroup scan of the 1024 run sums (wave shuffles, the 16 wave sums through
// LDS), and each thread writes its run from its prefix.  Larger: a sweep of 4096-word
// tiles with a running carry (ten barriered rounds per 41k words took 12 us; a run
// loop without the register staging, 18 us).
constexpr u32 RSS_THREADS = 1024, RSS_RUN = 16;
__device__ __forceinline__ u32 rss_block_excl(u32 s, u32* wsum, u32& all) {
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u32 x = s;  // inclusive scan over the wave
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(x, off);
        if (lane >= (u32)off) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (wave == 0) {
        u32 t = lane < RSS_THREADS / 64 ? wsum[lane] : 0;
        for (int off = 1; off < RSS_THREADS / 64; off <<= 1) {
            const u32 y = __shfl_up(t, off);
            if (lane >= (u32)off) t += y;
        }
        if (lane < RSS_THREADS / 64) wsum[lane] = t;  // inclusive prefix of the wave sums
    }
    __syncthreads();
    const u32 excl = (wave ? wsum[wave - 1] : 0) + x - s;
    all = wsum[RSS_THREADS / 64 - 1];
    __syncthreads();  // wsum is free again
    return excl;
}
__global__ __launch_bounds__(RSS_THREADS) void rs_scan(u32* __restrict__ data, u64 total, const u32* pred, u32 pmask) {
    if (rs_off(pred, pmask)) return;
    __shared__ u32 wsum[RSS_THREADS / 64];
    const u32 tid = threadIdx.x;
    const u64 q = total / 4;  // uint4 words
    if (q <= (u64)RSS_THREADS * RSS_RUN) {
        const u32 run = (u32)((q + RSS_THREADS - 1) / RSS_THREADS);
        const u64 lo = (u64)tid * run;
        uint4 v[RSS_RUN];
        u32 s = 0;
#pragma unroll
        for (u32 k = 0; k < RSS_RUN; k++) {
            v[k] = (k < run && lo + k < q) ? ((const uint4*)data)[lo + k] : make_uint4(0, 0, 0, 0);
            s += v[k].x + v[k].y + v[k].z + v[k].w;
        }
        u32 all;
        u32 excl = rss_block_excl(s, wsum, all);
#pragma unroll
        for (u32 k = 0; k < RSS_RUN; k++) {
            if (k < run && lo + k < q)
                ((uint4*)data)[lo + k] = make_uint4(excl, excl + v[k].x, excl + v[k].x + v[k].y,
                                                    excl + v[k].x + v[k].y + v[k].z);
            excl += v[k].x + v[k].y + v[k].z + v[k].w;
        }
        return;
    }
    u32 carry = 0;
    for (u64 base = 0; base < total; base += 4 * RSS_THREADS) {
        const u64 k = base + (u64)tid * 4;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < total) v = *(const uint4*)(data + k);
        const u32 s = v.x + v.y + v.z + v.w;
        u32 all;
        const u32 excl = carry + rss_block_excl(s, wsum, all);
        if (k < total) *(uint4*)(data + k) = make_uint4(excl, excl + v.x, excl + v.x + v.y, excl + v.x + v.y + v.z);
        carry += all;
    }
}

// The histogram's digit rows scanned in parallel, one wave per digit: row d (every
// tile's count of digit d) becomes its exclusive prefix, and tot[d] the row's total.
// rs_scatter adds the digits' exclusive prefix of tot (a 256-entry scan per tile), so
// no single workgroup walks the whole histogram (rs_scan, 13-14 us per pass for the
// 41k words of a 330k-side sort, its per-thread runs far from coalesced).
__global__ __launch_bounds__(256) void rs_rowscan(u32* __restrict__ hist, u32 nblocks, u32* __restrict__ tot,
                                                  const u32* pred, u32 pmask) {
    if (rs_off(pred, pmask)) return;
    const u32 lane = threadIdx.x & 63, d = blockIdx.x * 4 + (threadIdx.x >> 6);
    u32* row = hist + (u64)d * nblocks;
    u32 carry = 0;
    for (u32 base = 0; base < nblocks; base += 64) {
        const u32 k = base + lane;
        const u32 v = k < nblocks ? row[k] : 0;
        u32 x = v;
        for (int off = 1; off < 64; off <<= 1) {
            const u32 y = __shfl_up(x, off);
            if (lane >= (u32)off) x += y;
        }
        if (k < nblocks) row[k] = carry + x - v;
        carry += __shfl(x, 63);
    }
    if (lane == 0) tot[d] = carry;
}

// Exclusive scan of one value per thread over a 256-thread workgroup.
__device__ __forceinline__ u32 rs_block_excl256(u32 v, u32* wsum) {
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32 x = v;
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(x, off);
        if (lane >= (u32)off) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    u32 pre = 0;
    for (u32 w = 0; w < wave; w++) pre += wsum[w];
    return pre + x - v;
}

// Stable scatter: item order within a tile is r*256 + tid (round-major), i.e.
// index order.  Ranks within a wave come from 8 ballots (one per digit bit);
// ranks across the 4 waves and the rounds come from LDS counters.
__global__ __launch_bounds__(RS_THREADS) void rs_scatter(const u32* __restrict__ keys_in,
                                                         const u32* __restrict__ vals_in, u32* __restrict__ keys_out,
                                                         u32* __restrict__ vals_out, u64 n, int shift,
                                                         const u32* __restrict__ hist, u32 nblocks,
                                                         const u32* __restrict__ tot, const u32* pred, u32 pmask) {
    if (rs_off(pred, pmask)) return;
    __shared__ u32 run_base[256];
    __shared__ u32 wcnt[RS_WAVES][256];
    __shared__ u32 wsum[RS_WAVES];
    const u32 tid = threadIdx.x;
    const u32 wave = tid >> 6;
    const u32 row = hist[(u64)tid * nblocks + blockIdx.x];
    run_base[tid] = row + (tot ? rs_block_excl256(tot[tid], wsum) : 0u);
    for (int w = 0; w < RS_WAVES; w++) wcnt[w][tid] = 0;
    __syncthreads();
    const u64 base = (u64)blockIdx.x * RS_TILE;
    const u64 lt = __lanemask_lt();
    for (int r = 0; r < RS_IPT; r++) {
        const u64 i = base + (u64)r * RS_THREADS + tid;
        const bool valid = i < n;
        u32 key = 0, val = 0, d = 0;
        if (valid) {
            key = keys_in[i];
            val = vals_in[i];
            d = (key >> shift) & 0xFFu;
        }
        u64 peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const u64 m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const u32 rank = __popcll(peers & lt);
        const bool leader = valid && (peers & lt) == 0;
        if (leader) wcnt[wave][d] = __popcll(peers);
        __syncthreads();
        if (valid) {
            u32 off = run_base[d] + rank;
            for (u32 w = 0; w < wave; w++) off += wcnt[w][d];
            keys_out[off] = key;
            vals_out[off] = val;
        }
        __syncthreads();
        {
            u32 t = 0;
            for (int w = 0; w < RS_WAVES; w++) {
                t += wcnt[w][tid];
                wcnt[w][tid] = 0;
            }
            run_base[tid] += t;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------ scan3 -------
constexpr int SC_THREADS = 256;
constexpr int SC_IPT = 8;
constexpr int SC_TILE = SC_THREADS * SC_IPT;

__device__ __forceinline__ uint4 unpack3(u8 m) {
    return make_uint4(m & 1u, (m >> 1) & 1u, (m >> 2) & 1u, 0u);
}
__device__ __forceinline__ uint4 add4(uint4 a, uint4 b) {
    return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ uint4 block_excl_scan4(uint4 v, uint4* sh, uint4* total) {
    const u32 tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (u32 off = 1; off < SC_THREADS; off <<= 1) {
        uint4 o = tid >= off ? sh[tid - off] : make_uint4(0, 0, 0, 0);
        __syncthreads();
        sh[tid] = add4(sh[tid], o);
        __syncthreads();
    }
    uint4 incl = sh[tid];
    *total = sh[SC_THREADS - 1];
    __syncthreads();
    return make_uint4(incl.x - v.x, incl.y - v.y, incl.z - v.z, incl.w - v.w);
}

__global__ __launch_bounds__(SC_THREADS) void sc_reduce(const u8* __restrict__ mask, u64 n,
                                                        uint4* __restrict__ tile_sums, const u32* gate) {
    if (gate && *gate == 0) return;
    __shared__ uint4 sh[SC_THREADS];
    const u64 base = (u64)blockIdx.x * SC_TILE + (u64)threadIdx.x * SC_IPT;
    uint4 s = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < SC_IPT; k++)
        if (base + k < n) s = add4(s, unpack3(mask[base + k]));
    uint4 total;
    block_excl_scan4(s, sh, &total);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void sc_tiles(uint4* __restrict__ tile_sums, u64 ntiles, const u32* gate) {
    if (gate && *gate == 0) return;
    __shared__ uint4 sums[1024];
    const u32 tid = threadIdx.x;
    const u64 chunk = (ntiles + 1023) / 1024;
    const u64 lo = (u64)tid * chunk;
    const u64 hi = lo + chunk < ntiles ? lo + chunk : ntiles;
    uint4 s = make_uint4(0, 0, 0, 0);
    for (u64 i = lo; i < hi; i++) s = add4(s, tile_sums[i]);
    sums[tid] = s;
    __syncthreads();
    for (u32 off = 1; off < 1024; off <<= 1) {
        uint4 v = tid >= off ? sums[tid - off] : make_uint4(0, 0, 0, 0);
        __syncthreads();
        sums[tid] = add4(sums[tid], v);
        __syncthreads();
    }
    uint4 run = tid ? sums[tid - 1] : make_uint4(0, 0, 0, 0);
    for (u64 i = lo; i < hi; i++) {
        uint4 v = tile_sums[i];
        tile_sums[i] = run;
        run = add4(run, v);
    }
    if (tid == 1023) tile_sums[ntiles] = sums[1023];
}

__global__ __launch_bounds__(SC_THREADS) void sc_down(const u8* __restrict__ mask, u64 n,
                                                      const uint4* __restrict__ tile_sums, uint4* __restrict__ out,
                                                      const u32* gate) {
    if (gate && *gate == 0) return;
    __shared__ uint4 sh[SC_THREADS];
    const u64 base = (u64)blockIdx.x * SC_TILE + (u64)threadIdx.x * SC_IPT;
    uint4 v[SC_IPT];
    uint4 s = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < SC_IPT; k++) {
        v[k] = base + k < n ? unpack3(mask[base + k]) : make_uint4(0, 0, 0, 0);
        s = add4(s, v[k]);
    }
    uint4 total;
    uint4 run = add4(block_excl_scan4(s, sh, &total), tile_sums[blockIdx.x]);
    for (int k = 0; k < SC_IPT; k++) {
        if (base + k < n) out[base + k] = run;
        run = add4(run, v[k]);
    }
    // the element after the last one carries the grand total
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == SC_THREADS - 1) out[n] = tile_sums[gridDim.x];
}

}  // namespace

u64 radix_sort_hist_words(u64 capacity) { return 256ull * ((capacity + RS_TILE - 1) / RS_TILE + 1); }

void radix_sort_pairs(const u32* keys_in, const u32* vals_in, u32* keys_out, u32* vals_out, u64 n, int bits,
                      SortScratch& s, hipStream_t stream, const u32* pred, u32 pred_mask) {
    if (n == 0) return;
    if (n > s.capacity) tbgpu_fatal("radix_sort_pairs", "n exceeds scratch capacity", __FILE__, __LINE__);
    const u32 nblocks = (u32)((n + RS_TILE - 1) / RS_TILE);
    const int passes = bits <= 0 ? 1 : (bits + 7) / 8;
    // the digit totals after the histogram (radix_sort_hist_words leaves 256 words);
    // TBGPU_SORT_ONE_SCAN=1: the single-workgroup scan (A/B timing)
    static const bool row_scan = getenv("TBGPU_SORT_ONE_SCAN") == nullptr;
    u32* tot = s.hist + 256ull * nblocks;
    const u32* ks = keys_in;
    const u32* vs = vals_in;
    for (int p = 0; p < passes; p++) {
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        u32* kd = to_out ? keys_out : s.keys_tmp;
        u32* vd = to_out ? vals_out : s.vals_tmp;
        const int shift = 8 * p;
        rs_hist<<<nblocks, RS_THREADS, 0, stream>>>(ks, n, shift, s.hist, nblocks, pred, pred_mask);
        if (row_scan) {
            rs_rowscan<<<64, 256, 0, stream>>>(s.hist, nblocks, tot, pred, pred_mask);
        } else {
            rs_scan<<<1, RSS_THREADS, 0, stream>>>(s.hist, 256ull * nblocks, pred, pred_mask);
        }
        rs_scatter<<<nblocks, RS_THREADS, 0, stream>>>(ks, vs, kd, vd, n, shift, s.hist, nblocks,
                                                       row_scan ? tot : nullptr, pred, pred_mask);
        ks = kd;
        vs = vd;
    }
    HIP_CHECK(hipGetLastError());
}

u64 scan3_tile_words(u64 capacity) { return (capacity + SC_TILE - 1) / SC_TILE + 2; }

// out[i] = exclusive prefix of (bit0, bit1, bit2) of mask[0..i); out[n] = totals.
void scan3_exclusive(const u8* mask, uint4* out, u64 n, Scan3Scratch& s, hipStream_t stream, const u32* gate) {
    if (n == 0) {
        HIP_CHECK(hipMemsetAsync(out, 0, sizeof(uint4), stream));
        return;
    }
    const u64 ntiles = (n + SC_TILE - 1) / SC_TILE;
    sc_reduce<<<(u32)ntiles, SC_THREADS, 0, stream>>>(mask, n, s.tile_sums, gate);
    sc_tiles<<<1, 1024, 0, stream>>>(s.tile_sums, ntiles, gate);
    sc_down<<<(u32)ntiles, SC_THREADS, 0, stream>>>(mask, n, s.tile_sums, out, gate);
    HIP_CHECK(hipGetLastError());
}
