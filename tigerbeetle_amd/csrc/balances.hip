// balances.hip — segmented u128 balance scan over account-sorted event sides.
//
// Every transfer has a debit side and a credit side.  After sorting the sides by
// (account slot, batch index), the running balances an event sees are a prefix
// sum over its account's earlier sides (src/state_machine.zig:1286-1340 read
// dr/cr balances, :1330-1340 update them).  Visibility follows `execute`'s
// linked-chain scopes (:1018-1083): a side counts with its FINAL status (chain
// persisted) for readers outside its chain, and with its EVALUATED status for
// later members of the same chain (their scope still holds its effects).  So
//
//   before(q) = init(account) + F_excl(q) + H_excl(q)
//
// F sums final-ok deltas, segmented by account; H sums (eval-ok but not final)
// deltas, segmented by (account, chain).  Both are one scan with a two-level
// segmented operator; H is compiled out when the call has no chains.
//
// Traffic per side: the 4-B key, the side record (4-B event, 4-B chain, 1-B ok,
// 32-B deltas, contiguous), a 4-B chain-failure gather for chain members, the 64-B
// initial balances (L2-local: consecutive sides share the account row) and the
// 64-B output.
#include "common.h"
#include "engine.h"

namespace {

constexpr int BS_THREADS = 256;
constexpr int BS_IPT = 4;
constexpr int BS_TILE = BS_THREADS * BS_IPT;

struct SE {
    Bal4 F, H;
    u32 fl;  // bit0: account segment starts here, bit1: chain group starts here
};

__device__ __forceinline__ void zero(Bal4& b) { b.dp = b.dpo = b.cp = b.cpo = 0; }
__device__ __forceinline__ Bal4 add(const Bal4& a, const Bal4& b) {
    Bal4 r;
    r.dp = a.dp + b.dp;
    r.dpo = a.dpo + b.dpo;
    r.cp = a.cp + b.cp;
    r.cpo = a.cpo + b.cpo;
    return r;
}

template <bool HAS_H>
__device__ __forceinline__ SE combine(const SE& a, const SE& b) {
    SE c;
    c.F = (b.fl & 1) ? b.F : add(a.F, b.F);
    if (HAS_H) c.H = (b.fl & 2) ? b.H : add(a.H, b.H);
    c.fl = a.fl | b.fl;
    return c;
}

template <bool HAS_H>
__device__ __forceinline__ SE identity() {
    SE e;
    zero(e.F);
    if (HAS_H) zero(e.H);
    e.fl = 0;
    return e;
}

// Load sorted position q as a scan element.  Invalid (inert) sides sort last and
// contribute nothing; they are marked as segment starts so they never leak.  The
// side records are in sorted order (written there by the evaluation): the scan
// reads them contiguously, plus the chain's first failure for chain members.
template <bool HAS_H>
__device__ __forceinline__ SE load_elem(const SideScanArgs& A, u64 q, u32 invalid) {
    SE e;
    const u32 key = A.skey[q];
    if (key >= invalid) {
        e = identity<HAS_H>();
        e.fl = 3;
        return e;
    }
    const u32 cs = A.sq_cs[q] & SQ_CS;
    bool f_start = true, h_start = true;
    if (q > 0) {
        f_start = A.skey[q - 1] != key;
        h_start = f_start || (A.sq_cs[q - 1] & SQ_CS) != cs;
    }
    e.fl = (f_start ? 1u : 0u) | (h_start ? 2u : 0u);
    zero(e.F);
    if (HAS_H) zero(e.H);
    const bool eval_ok = A.sq_ok[q] & 1;
    if (!eval_ok) return e;
    const bool fin = side_final(A, q);
    const u128 dpe = A.sq_dpend[q], dpo = A.sq_dpost[q];
    const bool credit = A.sq_ev[q] >> 31;
    if (fin) {
        if (credit) { e.F.cp = dpe; e.F.cpo = dpo; } else { e.F.dp = dpe; e.F.dpo = dpo; }
    } else if (HAS_H) {
        if (credit) { e.H.cp = dpe; e.H.cpo = dpo; } else { e.H.dp = dpe; e.H.dpo = dpo; }
    }
    return e;
}

// Exclusive segmented scan of one value per thread across the workgroup.
template <bool HAS_H>
__device__ SE block_excl(SE v, SE* sh, SE* total) {
    const u32 tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (u32 off = 1; off < BS_THREADS; off <<= 1) {
        SE o;
        const bool take = tid >= off;
        if (take) o = sh[tid - off];
        __syncthreads();
        if (take) sh[tid] = combine<HAS_H>(o, sh[tid]);
        __syncthreads();
    }
    SE excl = tid ? sh[tid - 1] : identity<HAS_H>();
    *total = sh[BS_THREADS - 1];
    __syncthreads();
    return excl;
}

template <bool HAS_H>
__global__ __launch_bounds__(BS_THREADS) void bs_reduce(SideScanArgs A, u64 m, u32 invalid, SE* __restrict__ tagg) {
    if (!gate_open(A.gate)) return;
    __shared__ SE sh[BS_THREADS];
    const u64 base = (u64)blockIdx.x * BS_TILE + (u64)threadIdx.x * BS_IPT;
    SE acc = identity<HAS_H>();
    for (int k = 0; k < BS_IPT; k++)
        if (base + k < m) acc = combine<HAS_H>(acc, load_elem<HAS_H>(A, base + k, invalid));
    SE total;
    block_excl<HAS_H>(acc, sh, &total);
    if (threadIdx.x == 0) tagg[blockIdx.x] = total;
}

template <bool HAS_H>
__global__ __launch_bounds__(BS_THREADS) void bs_tiles(PassGate gate, SE* __restrict__ tagg, u64 ntiles) {
    if (!gate_open(gate)) return;
    __shared__ SE sh[BS_THREADS];
    const u32 tid = threadIdx.x;
    const u64 chunk = (ntiles + BS_THREADS - 1) / BS_THREADS;
    const u64 lo = (u64)tid * chunk;
    const u64 hi = lo + chunk < ntiles ? lo + chunk : ntiles;
    SE acc = identity<HAS_H>();
    for (u64 t = lo; t < hi; t++) acc = combine<HAS_H>(acc, tagg[t]);
    SE total;
    SE run = block_excl<HAS_H>(acc, sh, &total);
    for (u64 t = lo; t < hi; t++) {
        SE v = tagg[t];
        tagg[t] = run;
        run = combine<HAS_H>(run, v);
    }
}

template <bool HAS_H>
__global__ __launch_bounds__(BS_THREADS) void bs_down(SideScanArgs A, u64 m, u32 invalid, const SE* __restrict__ tagg,
                                                      const Account* __restrict__ acc, Bal4* __restrict__ bb) {
    if (!gate_open(A.gate)) return;
    // the next state's per-chain first failures start at "none" (its evaluation
    // follows this scan and lowers them with atomicMin)
    if (A.cfail_clear)
        for (u64 k = (u64)blockIdx.x * BS_THREADS + threadIdx.x; k < A.n; k += (u64)gridDim.x * BS_THREADS)
            A.cfail_clear[k] = NONE32;
    __shared__ SE sh[BS_THREADS];
    const u64 base = (u64)blockIdx.x * BS_TILE + (u64)threadIdx.x * BS_IPT;
    SE acc_t = identity<HAS_H>();
    for (int k = 0; k < BS_IPT; k++)
        if (base + k < m) acc_t = combine<HAS_H>(acc_t, load_elem<HAS_H>(A, base + k, invalid));
    SE total;
    SE run = combine<HAS_H>(tagg[blockIdx.x], block_excl<HAS_H>(acc_t, sh, &total));
    for (int k = 0; k < BS_IPT; k++) {
        const u64 q = base + k;
        if (q >= m) break;
        SE e = load_elem<HAS_H>(A, q, invalid);
        const u32 key = A.skey[q];
        if (key < invalid) {
            const Account& a = acc[key];
            Bal4 out;
            out.dp = a.debits_pending;
            out.dpo = a.debits_posted;
            out.cp = a.credits_pending;
            out.cpo = a.credits_posted;
            if (!(e.fl & 1)) out = add(out, run.F);
            if (HAS_H && !(e.fl & 2)) out = add(out, run.H);
            bb[q] = out;
        }
        run = combine<HAS_H>(run, e);
    }
}

// After convergence: the last side of each account segment writes the account's
// final balances: before(q) minus the in-chain H part, plus its own final delta.
__global__ void bs_final(SideScanArgs A, u64 m, u32 invalid, const Bal4* __restrict__ bb, Account* __restrict__ acc,
                         u32* big) {
    const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= m) return;
    const u32 key = A.skey[q];
    if (key >= invalid) return;
    if (q + 1 < m && A.skey[q + 1] == key) return;
    Bal4 tot = bb[q];
    const u32 cs = A.sq_cs[q] & SQ_CS;
    // remove the H contribution (same account, same chain, eval-ok & !final-ok)
    for (u64 p = q; p > 0;) {
        --p;
        if (A.skey[p] != key || (A.sq_cs[p] & SQ_CS) != cs) break;
        if ((A.sq_ok[p] & 1) && !side_final(A, p)) {
            if (A.sq_ev[p] >> 31) { tot.cp -= A.sq_dpend[p]; tot.cpo -= A.sq_dpost[p]; }
            else { tot.dp -= A.sq_dpend[p]; tot.dpo -= A.sq_dpost[p]; }
        }
    }
    if (side_final(A, q)) {
        if (A.sq_ev[q] >> 31) { tot.cp += A.sq_dpend[q]; tot.cpo += A.sq_dpost[q]; }
        else { tot.dp += A.sq_dpend[q]; tot.dpo += A.sq_dpost[q]; }
    }
    Account& a = acc[key];
    a.debits_pending = tot.dp;
    a.debits_posted = tot.dpo;
    a.credits_pending = tot.cp;
    a.credits_posted = tot.cpo;
    const u64 lim = 1ull << 62;
    if ((u64)(tot.dp >> 64) >= lim || (u64)(tot.dpo >> 64) >= lim || (u64)(tot.cp >> 64) >= lim ||
        (u64)(tot.cpo >> 64) >= lim)
        atomicOr(big, 1u);
}

// --------------------------------------------------------- fused scan ----
// One launch per pass: a workgroup of BF_THREADS sides (one per thread) finds the
// balance carried into its tile from the previous tile alone -- the tail of the
// account segment that crosses the boundary, which starts inside the previous tile
// unless a segment is longer than BF_THREADS sides -- then scans its own tile.  No
// tile aggregates, no second launch, no single-workgroup tile scan.  A segment
// longer than the window raises halt[1] (the host redoes the pass with the
// three-launch scan above).
constexpr int BF_THREADS = 256;

__device__ __forceinline__ u64 shup(u64 v, int off) { return (u64)__shfl_up((unsigned long long)v, off); }
__device__ __forceinline__ u128 shup128(u128 v, int off) {
    return ((u128)shup((u64)(v >> 64), off) << 64) | shup((u64)v, off);
}
__device__ __forceinline__ Bal4 shup_bal(const Bal4& b, int off) {
    Bal4 r;
    r.dp = shup128(b.dp, off);
    r.dpo = shup128(b.dpo, off);
    r.cp = shup128(b.cp, off);
    r.cpo = shup128(b.cpo, off);
    return r;
}

// Exclusive segmented scan of one element per thread over the workgroup: wave
// scans by shuffles, the four wave totals through LDS.
template <bool HAS_H>
__device__ SE block_excl_waves(SE v, SE* wtot) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int off = 1; off < 64; off <<= 1) {
        SE o;
        o.F = shup_bal(v.F, off);
        if (HAS_H) o.H = shup_bal(v.H, off);
        o.fl = __shfl_up(v.fl, off);
        if (lane >= (u32)off) v = combine<HAS_H>(o, v);
    }
    // v is inclusive; exclusive by one more shift
    SE ex;
    ex.F = shup_bal(v.F, 1);
    if (HAS_H) ex.H = shup_bal(v.H, 1);
    ex.fl = __shfl_up(v.fl, 1);
    if (lane == 0) ex = identity<HAS_H>();
    if (lane == 63) wtot[w] = v;
    __syncthreads();
    SE pre = identity<HAS_H>();
    for (u32 k = 0; k < w; k++) pre = combine<HAS_H>(pre, wtot[k]);
    __syncthreads();
    return combine<HAS_H>(pre, ex);
}

__device__ __forceinline__ u32 block_max(u32 v, u32* sh) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, (u32)__shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    v = sh[0];
    for (int k = 1; k < BF_THREADS / 64; k++) v = max(v, sh[k]);
    __syncthreads();
    return v;
}

__device__ __forceinline__ u128 wave_sum128(u128 v) {
    u64 lo = (u64)v, hi = (u64)(v >> 64);
    for (int off = 32; off > 0; off >>= 1) {
        const u64 l2 = (u64)__shfl_xor((unsigned long long)lo, off), h2 = (u64)__shfl_xor((unsigned long long)hi, off);
        const u64 s = lo + l2;
        hi = hi + h2 + (s < lo ? 1 : 0);
        lo = s;
    }
    return ((u128)hi << 64) | lo;
}
__device__ __forceinline__ Bal4 block_sum_bal(Bal4 b, Bal4* sh) {
    b.dp = wave_sum128(b.dp);
    b.dpo = wave_sum128(b.dpo);
    b.cp = wave_sum128(b.cp);
    b.cpo = wave_sum128(b.cpo);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = b;
    __syncthreads();
    Bal4 r = sh[0];
    for (int k = 1; k < BF_THREADS / 64; k++) r = add(r, sh[k]);
    __syncthreads();
    return r;
}

template <bool HAS_H>
__global__ __launch_bounds__(BF_THREADS) void bs_fused(SideScanArgs A, u64 m, u32 invalid, u32* long_flag,
                                                       const Account* __restrict__ acc, Bal4* __restrict__ bb) {
    if (!gate_open(A.gate)) return;
    __shared__ SE wtot[BF_THREADS / 64];
    __shared__ Bal4 bsum[BF_THREADS / 64];
    __shared__ u32 umax[BF_THREADS / 64];
    // the next state's per-chain first failures start at "none"
    if (A.cfail_clear)
        for (u64 k = (u64)blockIdx.x * BF_THREADS + threadIdx.x; k < A.n; k += (u64)gridDim.x * BF_THREADS)
            A.cfail_clear[k] = NONE32;
    const u64 q0 = (u64)blockIdx.x * BF_THREADS;
    const u64 q = q0 + threadIdx.x;
    // 1. the carry: the tail, in the previous tile, of the segment that crosses into this one
    SE carry = identity<HAS_H>();
    const u32 K = q0 > 0 ? A.skey[q0 - 1] : invalid;
    if (K < invalid) {
        const u64 p = q0 - BF_THREADS + threadIdx.x;  // q0 >= BF_THREADS here
        SE e = load_elem<HAS_H>(A, p, invalid);
        const bool mine = A.skey[p] == K;
        const u32 fs = block_max(mine && (e.fl & 1) ? (u32)threadIdx.x + 1 : 0u, umax);
        const u32 hs = block_max(mine && (e.fl & 2) ? (u32)threadIdx.x + 1 : 0u, umax);
        if (fs == 0) {  // the segment started before the previous tile
            if (threadIdx.x == 0) atomicMax(long_flag, A.gate.p + 1);
            return;
        }
        Bal4 z;
        zero(z);
        carry.F = block_sum_bal(mine && threadIdx.x + 1 >= fs ? e.F : z, bsum);
        if (HAS_H) carry.H = block_sum_bal(mine && threadIdx.x + 1 >= hs ? e.H : z, bsum);
    }
    // 2. this tile
    SE e = q < m ? load_elem<HAS_H>(A, q, invalid) : identity<HAS_H>();
    if (q >= m) e.fl = 3;
    SE run = combine<HAS_H>(carry, block_excl_waves<HAS_H>(e, wtot));
    if (q >= m) return;
    const u32 key = A.skey[q];
    if (key >= invalid) return;
    const Account& a = acc[key];
    Bal4 out;
    out.dp = a.debits_pending;
    out.dpo = a.debits_posted;
    out.cp = a.credits_pending;
    out.cpo = a.credits_posted;
    if (!(e.fl & 1)) out = add(out, run.F);
    if (HAS_H && !(e.fl & 2)) out = add(out, run.H);
    bb[q] = out;
}

}  // namespace

void side_scan_fused(const SideScanArgs& A, u64 m, u32 invalid, u32* long_flag, const Account* acc, Bal4* bb,
                     hipStream_t stream) {
    if (m == 0) return;
    bs_fused<true><<<(u32)((m + BF_THREADS - 1) / BF_THREADS), BF_THREADS, 0, stream>>>(A, m, invalid, long_flag,
                                                                                        acc, bb);
    HIP_CHECK(hipGetLastError());
}

u64 side_scan_tile_bytes(u64 capacity) { return ((capacity + BS_TILE - 1) / BS_TILE + 1) * sizeof(SE); }

void side_scan(const SideScanArgs& A, u64 m, u32 invalid, bool has_chains, void* tile_scratch, const Account* acc,
               Bal4* bb, hipStream_t stream) {
    if (m == 0) return;
    const u64 ntiles = (m + BS_TILE - 1) / BS_TILE;
    SE* tagg = (SE*)tile_scratch;
    if (has_chains) {
        bs_reduce<true><<<(u32)ntiles, BS_THREADS, 0, stream>>>(A, m, invalid, tagg);
        bs_tiles<true><<<1, BS_THREADS, 0, stream>>>(A.gate, tagg, ntiles);
        bs_down<true><<<(u32)ntiles, BS_THREADS, 0, stream>>>(A, m, invalid, tagg, acc, bb);
    } else {
        bs_reduce<false><<<(u32)ntiles, BS_THREADS, 0, stream>>>(A, m, invalid, tagg);
        bs_tiles<false><<<1, BS_THREADS, 0, stream>>>(A.gate, tagg, ntiles);
        bs_down<false><<<(u32)ntiles, BS_THREADS, 0, stream>>>(A, m, invalid, tagg, acc, bb);
    }
    HIP_CHECK(hipGetLastError());
}

void side_final_balances(const SideScanArgs& A, u64 m, u32 invalid, const Bal4* bb, Account* acc, u32* big,
                         hipStream_t stream) {
    if (m == 0) return;
    bs_final<<<(u32)((m + 255) / 256), 256, 0, stream>>>(A, m, invalid, bb, acc, big);
    HIP_CHECK(hipGetLastError());
}
