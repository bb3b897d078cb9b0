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
    u128 dpe, dpo;
    side_deltas(A, q, dpe, dpo);
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
__device__ __forceinline__ SE block_excl(SE v, SE* sh, SE& total) {
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
    total = sh[BS_THREADS - 1];
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
    block_excl<HAS_H>(acc, sh, total);
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
    SE run = block_excl<HAS_H>(acc, sh, total);
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
    SE run = combine<HAS_H>(tagg[blockIdx.x], block_excl<HAS_H>(acc_t, sh, total));
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
            // a 64-bit-form chunk's Bal4 passes (a long segment, the walk): a balance past
            // 2^62 could give a headroom, or a balancing amount, past what its 64-bit
            // records hold -- the chunk is redone in the u128 form
            if (A.over && ((out.dp | out.dpo | out.cp | out.cpo) >> 62)) atomicOr(A.over, (u32)FL_H64_OVER);
            bb[q] = out;
        }
        run = combine<HAS_H>(run, e);
    }
}

// After convergence: the last side of each account segment writes the account's
// final balances: before(q) minus the in-chain H part, plus its own final delta.
__global__ void bs_final(SideScanArgs A, u64 m, u32 invalid, const Bal4* __restrict__ bb, Account* __restrict__ acc,
                         u32* big) {
    if (A.epi) {
        const u32 e = *A.epi;
        if (e == 0) return;
        if (e == 2) A.cfail = A.cfail_alt;
    }
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
            u128 dpe, dpo;
            side_deltas(A, p, dpe, dpo);
            if (A.sq_ev[p] >> 31) { tot.cp -= dpe; tot.cpo -= dpo; }
            else { tot.dp -= dpe; tot.dpo -= dpo; }
        }
    }
    if (side_final(A, q)) {
        u128 dpe, dpo;
        side_deltas(A, q, dpe, dpo);
        if (A.sq_ev[q] >> 31) { tot.cp += dpe; tot.cpo += dpo; }
        else { tot.dp += dpe; tot.dpo += dpo; }
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
    if ((tot.dp | tot.dpo | tot.cp | tot.cpo) >> 61) atomicOr(big, 2u);  // (the 64-bit headroom passes' guard)
}

// --------------------------------------------------------- fused scan ----
// One launch per pass.  Tiles are cut at account boundaries: tile t holds the
// accounts whose first side lies in [t*BF_TILE, (t+1)*BF_TILE) (tstart[t], found
// once per chunk by tr_side_pos), so no balance carries from one tile to the next
// and a workgroup scans its tile alone: at most 2*BF_TILE sides while no account
// has more than BF_TILE sides in the chunk.  An account with more (no account
// starts in some window) raises halt[1]: the host redoes the pass with the
// three-launch scan above.
constexpr int BF_THREADS = 512;
constexpr int BF_IPT = 1;                     // sides per thread
constexpr int BF_TILE = 256;                  // nominal tile (sides): the 2x slack covers the last account
static_assert(BF_THREADS * BF_IPT == 2 * BF_TILE, "a workgroup scans two nominal tiles");

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

// Exclusive segmented scan (F only) of one element per thread over the workgroup:
// wave scans by shuffles, the four wave totals through LDS.
struct SF {
    Bal4 F;
    u32 fl;
};
__device__ __forceinline__ SF combine_f(const SF& a, const SF& b) {
    SF c;
    c.F = (b.fl & 1) ? b.F : add(a.F, b.F);
    c.fl = a.fl | b.fl;
    return c;
}
// One DPP step of the wave's inclusive segmented scan: every lane combines the value
// `ctrl` names (row_shr:n within a row of 16, or the row_bcast of a row's last lane
// into the rows `row_mask` selects); a lane without a source gets zero: the identity.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ u32 dpp32(u32 x) {
    return (u32)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xf, true);
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ u128 dpp128(u128 x) {
    const u64 lo = (u64)x, hi = (u64)(x >> 64);
    const u64 l = (u64)dpp32<CTRL, ROW_MASK>((u32)lo) | ((u64)dpp32<CTRL, ROW_MASK>((u32)(lo >> 32)) << 32);
    const u64 h = (u64)dpp32<CTRL, ROW_MASK>((u32)hi) | ((u64)dpp32<CTRL, ROW_MASK>((u32)(hi >> 32)) << 32);
    return ((u128)h << 64) | l;
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void dpp_step(SF& v) {
    SF o;
    o.F.dp = dpp128<CTRL, ROW_MASK>(v.F.dp);
    o.F.dpo = dpp128<CTRL, ROW_MASK>(v.F.dpo);
    o.F.cp = dpp128<CTRL, ROW_MASK>(v.F.cp);
    o.F.cpo = dpp128<CTRL, ROW_MASK>(v.F.cpo);
    o.fl = dpp32<CTRL, ROW_MASK>(v.fl);
    v = combine_f(o, v);
}

__device__ __forceinline__ SF block_excl_f(SF v, SF* wtot) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // inclusive over the wave by DPP (no LDS round trips): within rows of 16, then
    // row 0's last into row 1 and row 2's into row 3, then row 1's into rows 2 and 3
    dpp_step<0x111, 0xf>(v);  // row_shr:1
    dpp_step<0x112, 0xf>(v);  // row_shr:2
    dpp_step<0x114, 0xf>(v);  // row_shr:4
    dpp_step<0x118, 0xf>(v);  // row_shr:8
    dpp_step<0x142, 0xa>(v);  // row_bcast:15
    dpp_step<0x143, 0xc>(v);  // row_bcast:31
    SF ex;
    ex.F = shup_bal(v.F, 1);
    ex.fl = __shfl_up(v.fl, 1);
    if (lane == 0) { zero(ex.F); ex.fl = 0; }
    if (lane == 63) wtot[w] = v;
    __syncthreads();
    SF pre;
    zero(pre.F);
    pre.fl = 0;
    for (u32 k = 0; k < w; k++) pre = combine_f(pre, wtot[k]);
    return combine_f(pre, ex);
}

// A sorted side's contributions: to F (final-ok), or to H (evaluated-ok in a chain
// that does not persist: visible only to later members of its chain).
// (by value and selects, not a pointer to one of two locals: that put both in scratch)
__device__ __forceinline__ void side_contrib(const SideScanArgs& A, u64 q, Bal4& F, Bal4& H) {
    zero(F);
    zero(H);
    if (!(A.sq_ok[q] & 1)) return;
    u128 dpe, dpo;
    side_deltas(A, q, dpe, dpo);
    const bool fin = (A.probe & 1) ? true : side_final(A, q), credit = A.sq_ev[q] >> 31;
    const u128 pe = credit ? 0 : dpe, po = credit ? 0 : dpo, ce = credit ? dpe : 0, co = credit ? dpo : 0;
    if (fin) { F.dp = pe; F.dpo = po; F.cp = ce; F.cpo = co; }
    else { H.dp = pe; H.dpo = po; H.cp = ce; H.cpo = co; }
}

// F is scanned (segmented by account); H, non-zero only behind earlier members of
// the side's own chain on the same account -- the sides right before it in sorted
// order -- is summed by walking back over that run, staged in LDS.
// The fused scans' per-tile prologue: [a0, b0) is the tile's side range (a0 = NONE32:
// no account starts in it), the result whether a side record in it moved last pass
// (always when `all`).  (Reading these before the group resolution, to overlap the two,
// measured slower: 177-179 vs 180.5 M/s on config 3.)
__device__ __forceinline__ bool tile_due(const SideScanArgs& A, const u32* __restrict__ tstart, u32 t, u32 ntiles,
                                         u32 m, u32 window, bool all, u32& a0, u32& b0) {
    a0 = tstart[t];
    b0 = m;
    if (a0 == NONE32) return false;
    for (u32 k = t + 1; k < ntiles; k++)
        if (tstart[k] != NONE32) { b0 = tstart[k]; break; }
    if (all || b0 - a0 > window) return true;
    bool due = false;
    for (u32 w = a0 / BF_TILE; w <= (b0 - 1) / BF_TILE; w++) due |= A.dt.win[w] == A.gate.p;
    return due;
}

// The complex events whose id / pending groups moved last pass are due, with their
// chains (decided here, before any evaluation of this pass reads it).  The fused scans
// give this its own leading workgroups (resolve_blocks), one complex event per thread:
// its three dependent loads then run beside the tiles' scans instead of ahead of them.
__host__ __device__ __forceinline__ u32 resolve_blocks(u32 n_complex) { return (n_complex + BF_THREADS - 1) / BF_THREADS; }
__device__ __forceinline__ void resolve_groups(const SideScanArgs& A, u32 par, u32 pq, u32 threads = BF_THREADS) {
    const u64 k = (u64)blockIdx.x * threads + threadIdx.x;
    if (k < A.n_complex) {
        const u32 i = A.lst_complex[k];
        const u32 gs = A.gslot[i], ps = A.pslot[i];
        if ((gs != NONE32 && A.dt.slot[par * A.dt.g + gs] == pq) ||
            (ps != NONE32 && A.dt.slot[par * A.dt.g + ps] == pq)) {
            A.dt.ev[par * A.dt.n + i] = pq;
            const u32 cs = A.cs[i];
            if (cs != A.ce[i]) A.dt.chain[par * A.dt.n + cs] = pq;
        }
    }
}

__global__ __launch_bounds__(BF_THREADS) void bs_fused(SideScanArgs A, u64 m, u32 invalid, const u32* __restrict__ tstart,
                                                       u32 ntiles, u32* long_flag, const Account* __restrict__ acc,
                                                       Bal4* __restrict__ bb) {
    if (!gate_open(A.gate)) return;
    if (A.epi) {  // the Bal4 scan behind a converged headroom fixed point: its state by the gate word
        const u32 e = *A.epi;
        if (e == 0) return;
        if (e == 2) A.cfail = A.cfail_alt;
    }
    __shared__ SF wtot[BF_THREADS / 64];
    __shared__ u32 s_key[BF_THREADS * BF_IPT], s_cs[BF_THREADS * BF_IPT];
    __shared__ Bal4 s_h[BF_THREADS * BF_IPT];
    // the next state's per-chain first failures start at "none"
    if (A.cfail_clear)
        for (u64 k = (u64)blockIdx.x * BF_THREADS + threadIdx.x; k < A.n; k += (u64)gridDim.x * BF_THREADS)
            A.cfail_clear[k] = NONE32;
    const u32 nres = resolve_blocks(A.n_complex);
    const u32 t = blockIdx.x - nres, tid = threadIdx.x;
    // Dirty tracking (engine.h Dirty): everything at a chunk's first pass and after a
    // side rebuild; otherwise only the windows whose side records moved last pass.
    const u32 pq = A.gate.p, par = pq & 1;
    const bool all = A.gate.full || *A.dt.all == pq;
    if (blockIdx.x < nres) {
        if (!all) resolve_groups(A, par, pq);
        return;
    }
    u32 a0, b0;
    const bool due = tile_due(A, tstart, t, ntiles, (u32)m, BF_THREADS * BF_IPT, all, a0, b0);
    if (a0 == NONE32) return;  // no account starts in this window: the previous tile has its sides
    if (b0 - a0 > BF_THREADS * BF_IPT) {  // an account longer than a window
        if (tid == 0) atomicMax(long_flag, A.gate.p + 1);
        return;
    }
    if (!due) return;  // no side of the tile moved: its balances stand
    // the thread's two sides (contiguous), loaded before any barrier
    const u64 qa = (u64)a0 + BF_IPT * tid;
    u32 key[BF_IPT], cs[BF_IPT];
    Bal4 f[BF_IPT], h[BF_IPT], row[BF_IPT];
    SF e[BF_IPT];
#pragma unroll
    for (int k = 0; k < BF_IPT; k++) {
        const u64 q = qa + k;
        key[k] = q < b0 ? A.skey[q] : invalid;
    }
#pragma unroll
    for (int k = 0; k < BF_IPT; k++) {
        // the account row (pre-chunk balances) is issued before the scan's barrier
        zero(row[k]);
        if (key[k] < invalid && !(A.probe & 2)) {
            const Account& ac = acc[key[k]];
            row[k].dp = ac.debits_pending;
            row[k].dpo = ac.debits_posted;
            row[k].cp = ac.credits_pending;
            row[k].cpo = ac.credits_posted;
        }
    }
#pragma unroll
    for (int k = 0; k < BF_IPT; k++) {
        const u64 q = qa + k;
        const u32 c = q < b0 ? A.sq_cs[q] : SQ_STANDALONE;
        cs[k] = c & SQ_CS;
        zero(f[k]);
        zero(h[k]);
        e[k].fl = 1;
        if (key[k] < invalid) {
            side_contrib(A, q, f[k], h[k]);
            const u32 prev = k > 0 ? key[k - 1] : (q == a0 ? invalid : A.skey[q - 1]);
            e[k].fl = prev != key[k] ? 1u : 0u;
        }
        e[k].F = f[k];
        s_key[BF_IPT * tid + k] = key[k];
        // chain members only: the walk below reads s_h behind a side of its own chain
        s_cs[BF_IPT * tid + k] = (c & SQ_STANDALONE) ? NONE32 : cs[k];
        if (!(c & SQ_STANDALONE)) s_h[BF_IPT * tid + k] = h[k];
    }
    SF agg = e[0];
#pragma unroll
    for (int k = 1; k < BF_IPT; k++) agg = combine_f(agg, e[k]);
    SF run;
    if (A.probe & 4) {
        zero(run.F);
        run.fl = 0;
        __syncthreads();
    } else {
        run = block_excl_f(agg, wtot);  // (its barrier publishes s_key / s_cs / s_h)
    }
#pragma unroll
    for (int k = 0; k < BF_IPT; k++) {
        const u64 q = qa + k;
        if (key[k] < invalid) {
            Bal4 H;
            zero(H);
            u32 j = BF_IPT * tid + k;
            if (s_cs[j] != NONE32)
                while (j > 0 && s_key[j - 1] == key[k] && s_cs[j - 1] == cs[k]) H = add(H, s_h[--j]);
            Bal4 out = row[k];
            if (!(e[k].fl & 1)) out = add(out, run.F);
            out = add(out, H);
            if (all) {
                bb[q] = out;
            } else {
                const Bal4 old = bb[q];
                if (old.dp != out.dp || old.dpo != out.dpo || old.cp != out.cp || old.cpo != out.cpo) {
                    // a balance moved: its event is due this pass (with its chain)
                    bb[q] = out;
                    A.dt.ev[par * A.dt.n + (A.sq_ev[q] & SQ_EV)] = pq;
                    const u32 c = A.sq_cs[q];
                    if (!(c & SQ_STANDALONE)) A.dt.chain[par * A.dt.n + (c & SQ_CS)] = pq;
                }
            }
        }
        run = combine_f(run, e[k]);
    }
}

// ------------------------------------------------- headroom (narrow) scan ----
// What a pass's evaluation reads of a balance, when no overflow check can fire (the
// chunk's amounts < 2^64 and every committed balance < 2^126: FL_WIDE clear): a debit
// side's limit and balancing checks read only H_d = credits_posted - debits_pending -
// debits_posted of its account (src/state_machine.zig:1290-1322: dr.debits_* + amount
// > dr.credits_posted <=> amount > H_d), a credit side only H_c = debits_posted -
// credits_pending - credits_posted.  Both are linear in the sides' deltas, so the scan
// carries (H_d, H_c) -- two u128 instead of four -- and writes one u128 per side.  The
// fixed point is the same; the apply kernels get the Bal4 form from one full scan
// after convergence.
struct SN {
    u128 hd, hc;
    u32 fl;
};
__device__ __forceinline__ SN combine_n(const SN& a, const SN& b) {
    SN c;
    if (b.fl & 1) { c.hd = b.hd; c.hc = b.hc; }
    else { c.hd = a.hd + b.hd; c.hc = a.hc + b.hc; }
    c.fl = a.fl | b.fl;
    return c;
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void dpp_step_n(SN& v) {
    SN o;
    o.hd = dpp128<CTRL, ROW_MASK>(v.hd);
    o.hc = dpp128<CTRL, ROW_MASK>(v.hc);
    o.fl = dpp32<CTRL, ROW_MASK>(v.fl);
    v = combine_n(o, v);
}
__device__ __forceinline__ SN block_excl_n(SN v, SN* wtot) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    dpp_step_n<0x111, 0xf>(v);
    dpp_step_n<0x112, 0xf>(v);
    dpp_step_n<0x114, 0xf>(v);
    dpp_step_n<0x118, 0xf>(v);
    dpp_step_n<0x142, 0xa>(v);
    dpp_step_n<0x143, 0xc>(v);
    SN ex;
    ex.hd = shup128(v.hd, 1);
    ex.hc = shup128(v.hc, 1);
    ex.fl = __shfl_up(v.fl, 1);
    if (lane == 0) { ex.hd = ex.hc = 0; ex.fl = 0; }
    if (lane == 63) wtot[w] = v;
    __syncthreads();
    SN pre;
    pre.hd = pre.hc = 0;
    pre.fl = 0;
    for (u32 k = 0; k < w; k++) pre = combine_n(pre, wtot[k]);
    return combine_n(pre, ex);
}

// Two sides per thread in 256-thread workgroups (the same 512-side window): the
// launch's 4-wave workgroups then all fit the chip at once, where 8-wave ones took a
// second round for the last fifth of the tiles.
constexpr int NF_THREADS = 256, NF_IPT = 2;
static_assert(NF_THREADS * NF_IPT == 2 * BF_TILE, "a workgroup scans two nominal tiles");
__host__ __device__ __forceinline__ u32 resolve_blocks_n(u32 n_complex) {
    return (n_complex + NF_THREADS - 1) / NF_THREADS;
}

// H64: the 64-bit form (side_scan_fused_h64): the figures and deltas are stored as 64-bit
// two's complement (exact: FL_WIDE64 clear bounds every headroom of the chunk within
// +-2^63), read sign-extended and scanned as before.
template <bool H64>
__global__ __launch_bounds__(NF_THREADS) void bs_fused_narrow(SideScanArgs A, u64 m, u32 invalid,
                                                              const u32* __restrict__ tstart, u32 ntiles,
                                                              u32* long_flag, const Account* __restrict__ acc) {
    if (!gate_open(A.gate)) return;
    __shared__ SN wtot[NF_THREADS / 64];
    __shared__ u32 s_key[NF_THREADS * NF_IPT], s_cs[NF_THREADS * NF_IPT];
    __shared__ u128 s_hd[NF_THREADS * NF_IPT], s_hc[NF_THREADS * NF_IPT];
    if (A.cfail_clear)
        for (u64 k = (u64)blockIdx.x * NF_THREADS + threadIdx.x; k < A.n; k += (u64)gridDim.x * NF_THREADS)
            A.cfail_clear[k] = NONE32;
    const u32 nres = resolve_blocks_n(A.n_complex);
    const u32 t = blockIdx.x - nres, tid = threadIdx.x;
    const u32 pq = A.gate.p, par = pq & 1;
    const bool all = A.gate.full || *A.dt.all == pq;
    if (blockIdx.x < nres) {
        if (!all) resolve_groups(A, par, pq, NF_THREADS);
        return;
    }
    u32 a0, b0;
    const bool due = tile_due(A, tstart, t, ntiles, (u32)m, NF_THREADS * NF_IPT, all, a0, b0);
    if (a0 == NONE32) return;
    if (b0 - a0 > NF_THREADS * NF_IPT) {
        if (tid == 0) atomicMax(long_flag, A.gate.p + 1);
        return;
    }
    if (!due) return;
    // Every word of the thread's two sides in one round of loads (the deltas count only
    // on an ok side), then the account rows and the chains' first failures in a second.
    const u64 qa = (u64)a0 + NF_IPT * tid;
    u32 key[NF_IPT], c[NF_IPT], ev[NF_IPT];
    u8 okw[NF_IPT];
    u128 dpe[NF_IPT], dpo[NF_IPT], old[NF_IPT];
#pragma unroll
    for (int k = 0; k < NF_IPT; k++) {
        const u64 q = qa + k;
        const bool in = q < b0;
        key[k] = in ? A.skey[q] : invalid;
        c[k] = in ? A.sq_cs[q] : SQ_STANDALONE;
        ev[k] = in ? A.sq_ev[q] : 0;
        okw[k] = in ? A.sq_ok[q] : 0;
        if (H64) {
            const ulonglong2 d = in ? ((const ulonglong2*)A.sq_d64)[q] : ulonglong2{0, 0};
            dpe[k] = sext64(d.x);
            dpo[k] = sext64(d.y);
            old[k] = (!all && in) ? sext64(A.bh64[q]) : 0;
        } else {
            dpe[k] = in ? A.sq_dpend[q] : 0;
            dpo[k] = in ? A.sq_dpost[q] : 0;
            old[k] = (!all && in) ? A.bh[q] : 0;
        }
    }
    const u32 prev0 = (qa < b0 && qa > a0) ? A.skey[qa - 1] : invalid;
    u32 cf[NF_IPT];
    u128 r_hd[NF_IPT], r_hc[NF_IPT];  // the accounts' pre-chunk headroom (an account's first side)
    bool first[NF_IPT];
#pragma unroll
    for (int k = 0; k < NF_IPT; k++) {
        const bool live = key[k] < invalid && (okw[k] & 1);
        cf[k] = live && !(c[k] & (SQ_STANDALONE | SQ_DOOM)) ? A.cfail[c[k] & SQ_CS] : NONE32;
        r_hd[k] = r_hc[k] = 0;
        // Only an account's first side reads its row: the pre-chunk headroom enters the
        // scan there and reaches the account's later sides through it (instead of a row
        // read per side; measured alike on config 3, whose 10k rows stay in L2)
        first[k] = key[k] < invalid && (k == 0 ? prev0 : key[k - 1]) != key[k];
        if (first[k]) {
            const Account& ac = acc[key[k]];
            const u128 adp = ac.debits_pending, adpo = ac.debits_posted, acp = ac.credits_pending,
                       acpo = ac.credits_posted;
            r_hd[k] = acpo - adp - adpo;
            r_hc[k] = adpo - acp - acpo;
        }
    }
    // each side's delta on (H_d, H_c): final-ok -> F, evaluated-ok in a chain that does
    // not persist -> H (visible only behind it in its own chain)
    SN e[NF_IPT];
#pragma unroll
    for (int k = 0; k < NF_IPT; k++) {
        const bool credit = ev[k] >> 31;
        u128 f_hd = 0, f_hc = 0, h_hd = 0, h_hc = 0;
        e[k].fl = 1;
        if (key[k] < invalid) {
            if (okw[k] & 1) {
                const u128 dhd = credit ? dpo[k] : (u128)0 - dpe[k] - dpo[k];
                const u128 dhc = credit ? (u128)0 - dpe[k] - dpo[k] : dpo[k];
                const bool fin = !(c[k] & SQ_DOOM) && ((c[k] & SQ_STANDALONE) || cf[k] == NONE32);  // side_final
                if (fin) { f_hd = dhd; f_hc = dhc; } else { h_hd = dhd; h_hc = dhc; }
            }
            const u32 prev = k == 0 ? prev0 : key[k - 1];
            e[k].fl = prev != key[k] ? 1u : 0u;
        }
        e[k].hd = f_hd;
        e[k].hc = f_hc;
        const u32 j = NF_IPT * tid + k;
        s_key[j] = key[k];
        s_cs[j] = (c[k] & SQ_STANDALONE) ? NONE32 : (c[k] & SQ_CS);
        if (!(c[k] & SQ_STANDALONE)) { s_hd[j] = h_hd; s_hc[j] = h_hc; }
    }
#pragma unroll
    for (int k = 0; k < NF_IPT; k++) {  // (an account's first side carries its pre-chunk headroom)
        if (!first[k]) continue;
        e[k].hd += r_hd[k];
        e[k].hc += r_hc[k];
    }
    SN run = block_excl_n(combine_n(e[0], e[1]), wtot);  // (its barrier publishes s_key / s_cs / s_h*)
#pragma unroll
    for (int k = 0; k < NF_IPT; k++) {
        const u64 q = qa + k;
        if (key[k] < invalid) {
            const bool credit = ev[k] >> 31;
            u128 h = 0;
            u32 j = NF_IPT * tid + k;
            const u32 cs = c[k] & SQ_CS;
            if (s_cs[j] != NONE32)
                while (j > 0 && s_key[j - 1] == key[k] && s_cs[j - 1] == cs) { --j; h += credit ? s_hc[j] : s_hd[j]; }
            // the first side: the row's figure; a later one: the headroom and the deltas
            // before it in its account, through the scan
            u128 out = first[k] ? (credit ? r_hc[k] : r_hd[k]) : (credit ? run.hc : run.hd);
            out += h;
            if (H64 && !fits64(out)) atomicOr(A.over, (u32)FL_H64_OVER);  // the chunk is redone in u128
            if (all) {
                if (H64) A.bh64[q] = (u64)out; else A.bh[q] = out;
            } else if (H64 ? (u64)old[k] != (u64)out : old[k] != out) {
                // a balance moved: its event is due this pass (with its chain) when this
                // balance can decide its outcome (SQ_SENS); otherwise only the figure moves
                if (H64) A.bh64[q] = (u64)out; else A.bh[q] = out;
                if ((ev[k] & SQ_SENS) || A.all_sides) {
                    A.dt.ev[par * A.dt.n + (ev[k] & SQ_EV)] = pq;
                    if (!(c[k] & SQ_STANDALONE)) A.dt.chain[par * A.dt.n + (c[k] & SQ_CS)] = pq;
                }
            }
        }
        run = combine_n(run, e[k]);
    }
}

}  // namespace

void side_scan_fused(const SideScanArgs& A, u64 m, u32 invalid, const u32* tstart, u32* long_flag,
                     const Account* acc, Bal4* bb, hipStream_t stream) {
    if (m == 0) return;
    const u32 ntiles = (u32)((m + BF_TILE - 1) / BF_TILE);
    bs_fused<<<resolve_blocks(A.n_complex) + ntiles, BF_THREADS, 0, stream>>>(A, m, invalid, tstart, ntiles, long_flag,
                                                                              acc, bb);
    HIP_CHECK(hipGetLastError());
}

void side_scan_fused_narrow(const SideScanArgs& A, u64 m, u32 invalid, const u32* tstart, u32* long_flag,
                            const Account* acc, hipStream_t stream) {
    if (m == 0) return;
    const u32 ntiles = (u32)((m + BF_TILE - 1) / BF_TILE);
    bs_fused_narrow<false><<<resolve_blocks_n(A.n_complex) + ntiles, NF_THREADS, 0, stream>>>(A, m, invalid, tstart,
                                                                                            ntiles, long_flag, acc);
    HIP_CHECK(hipGetLastError());
}

void side_scan_fused_h64(const SideScanArgs& A, u64 m, u32 invalid, const u32* tstart, u32* long_flag,
                         const Account* acc, hipStream_t stream) {
    if (m == 0) return;
    const u32 ntiles = (u32)((m + BF_TILE - 1) / BF_TILE);
    bs_fused_narrow<true><<<resolve_blocks_n(A.n_complex) + ntiles, NF_THREADS, 0, stream>>>(A, m, invalid, tstart,
                                                                                           ntiles, long_flag, acc);
    HIP_CHECK(hipGetLastError());
}

u32 side_scan_fused_tile() { return BF_TILE; }

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
