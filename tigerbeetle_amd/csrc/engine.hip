// engine.hip — host runtime of the commit engine and the C-ABI (include/tbgpu.h).
//
// A ctx owns the HBM state that replaces the StateMachine's forest for the hot
// path (accounts, transfers + id index, posted groove, account history) and the
// per-call scratch.  Each create_* call (one batch, or several consecutive
// batches streamed together) runs:
//
//   classify (static checks + probes) -> group same-id / same-pending events ->
//   fixed point { sides -> sort -> balance scan -> evaluate } -> apply
//
// See transfers.hip for why the fixed point reproduces execute() exactly.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <vector>

#include "common.h"
#include "engine.h"
#include "transfers.h"
#include "index.h"
#include "fast.h"
#include "query.h"

[[noreturn]] void tbgpu_fatal(const char* what, const char* why, const char* file, int line) {
    fprintf(stderr, "tbgpu: fatal: %s: %s (%s:%d)\n", what, why, file, line);
    fflush(stderr);
    if (const char* log = getenv("TBGPU_FATAL_LOG")) {  // where a test runner that captures stderr can find it
        if (FILE* f = fopen(log, "a")) {
            fprintf(f, "tbgpu: fatal: %s: %s (%s:%d)\n", what, why, file, line);
            fclose(f);
        }
    }
    abort();
}

namespace {

u64 pow2_at_least(u64 x) {
    u64 p = 16;
    while (p < x) p <<= 1;
    return p;
}
int log2u(u64 x) {
    int b = 0;
    while ((1ull << b) < x) b++;
    return b;
}

// u32 words before the batch timestamps in a chunk's batch block: nb + 1 starts, 8-byte aligned
inline u64 batch_ts_offset(u64 bmax) { return (bmax + 2) & ~1ull; }

// Waits on the engine's streams: blocking, or with TBGPU_POLL_SYNC=1 by polling
// (hipStreamQuery / hipEventQuery in a loop).  Polling was measured alike on config
// 3 (152 M/s either way) and slower on the routed step (gpurun_out/r02c13), so the
// blocking wait is the default.
inline bool blocking_sync() {
    static const bool b = getenv("TBGPU_POLL_SYNC") == nullptr;
    return b;
}
inline void wait_stream(hipStream_t s) {
    if (blocking_sync()) {
        HIP_CHECK(hipStreamSynchronize(s));
        return;
    }
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) HIP_CHECK(e);
    }
}
inline void wait_event(hipEvent_t ev) {
    if (blocking_sync()) {
        HIP_CHECK(hipEventSynchronize(ev));
        return;
    }
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) HIP_CHECK(e);
    }
}

// TBGPU_POISON_ALLOC=<byte> (diagnostics; "1" means 0xA5): every device allocation
// and every page-locked host buffer the ctx owns starts filled with that byte instead
// of whatever an earlier ctx (or a fresh page's zeros) left there.  A kernel or host
// step that reads a word before this ctx wrote it then goes wrong deterministically,
// in the test that does it, instead of only after earlier tests recycled the memory.
// The fill runs on the stream of the ctx that allocates (ZeroOn names it for the
// allocating scope), and the scope ends only when the fill is complete.
thread_local hipStream_t t_zero_stream = nullptr;
inline int poison_byte() {
    static const int b = [] {
        const char* e = getenv("TBGPU_POISON_ALLOC");
        if (!e || !*e) return -1;
        const long v = strtol(e, nullptr, 0);
        return v == 1 ? 0xA5 : (int)(v & 0xFF);
    }();
    return b;
}
inline bool zero_alloc() { return poison_byte() >= 0; }
struct ZeroOn {
    hipStream_t prev, mine;
    explicit ZeroOn(hipStream_t s) : prev(t_zero_stream), mine(s) { t_zero_stream = s; }
    ~ZeroOn() {
        if (zero_alloc()) HIP_CHECK(hipStreamSynchronize(mine));
        t_zero_stream = prev;
    }
};

inline void zero_new(void* p, u64 bytes) {
    if (!zero_alloc()) return;
    if (!t_zero_stream) tbgpu_fatal("alloc", "device allocation outside a ZeroOn scope", __FILE__, __LINE__);
    HIP_CHECK(hipMemsetAsync(p, poison_byte(), bytes, t_zero_stream));
}
// page-locked host memory: filled by the host (no kernel has seen it yet)
inline void poison_host(void* p, u64 bytes) {
    if (zero_alloc()) memset(p, poison_byte(), bytes);
}

// TBGPU_GUARD=1 (diagnostics): every device allocation gets GUARD_BYTES of a known
// word pattern behind it, and every entry point first checks all live guards: a
// kernel that writes past the end of its buffer fails the next call, naming the
// buffer (its size and allocation number), instead of corrupting a neighbour.
constexpr u64 GUARD_BYTES = 64 << 10;
constexpr u32 GUARD_WORD = 0xA5C3A5C3u;
struct Guard {
    void* base;
    u64 offset;  // the guard's start: the buffer's bytes rounded up to 256
    u64 bytes, elem;
    u64 serial;
};
std::mutex g_guard_mu;
std::vector<Guard> g_guards;
u64 g_guard_serial = 0;
inline bool guard_on() {
    static const bool g = getenv("TBGPU_GUARD") != nullptr;
    return g;
}
__global__ void k_guard_check(const u32* g, u32 words, u32* bad) {
    for (u32 k = blockIdx.x * blockDim.x + threadIdx.x; k < words; k += gridDim.x * blockDim.x)
        if (g[k] != GUARD_WORD) atomicAdd(bad, 1u);
}
// every live guard intact, else fatal (naming the first broken one)
void guard_check_all(hipStream_t s) {
    if (!guard_on()) return;
    std::lock_guard<std::mutex> lk(g_guard_mu);
    static u32* bad = nullptr;
    if (!bad) HIP_CHECK(hipMalloc(&bad, 4 * 4096));
    const size_t n = std::min<size_t>(g_guards.size(), 4096);
    HIP_CHECK(hipMemsetAsync(bad, 0, 4 * n, s));
    for (size_t k = 0; k < n; k++)
        k_guard_check<<<16, 256, 0, s>>>((const u32*)((u8*)g_guards[k].base + g_guards[k].offset),
                                         (u32)(GUARD_BYTES / 4), bad + k);
    std::vector<u32> h(n);
    HIP_CHECK(hipMemcpyAsync(h.data(), bad, 4 * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    for (size_t k = 0; k < n; k++)
        if (h[k]) {
            char why[200];
            snprintf(why, sizeof why, "%u guard words past allocation #%llu (%llu bytes, element %llu B) overwritten",
                     h[k], (unsigned long long)g_guards[k].serial, (unsigned long long)g_guards[k].bytes,
                     (unsigned long long)g_guards[k].elem);
            tbgpu_fatal("guard", why, __FILE__, __LINE__);
        }
}
void guard_release(void* p) {
    if (!guard_on() || !p) return;
    std::lock_guard<std::mutex> lk(g_guard_mu);
    for (size_t k = 0; k < g_guards.size(); k++)
        if (g_guards[k].base == p) {
            g_guards[k] = g_guards.back();
            g_guards.pop_back();
            return;
        }
}
inline u64 guard_extra(u64 bytes) { return guard_on() ? ((bytes + 255) & ~255ull) - bytes + GUARD_BYTES : 0; }
inline void guard_arm(void* p, u64 bytes, u64 elem) {
    if (!guard_on()) return;
    const u64 off = (bytes + 255) & ~255ull;
    if (t_zero_stream) {
        HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)((u8*)p + off), GUARD_WORD, GUARD_BYTES / 4, t_zero_stream));
        HIP_CHECK(hipStreamSynchronize(t_zero_stream));
    } else {
        HIP_CHECK(hipMemsetD32((hipDeviceptr_t)((u8*)p + off), GUARD_WORD, GUARD_BYTES / 4));
    }
    std::lock_guard<std::mutex> lk(g_guard_mu);
    g_guards.push_back(Guard{p, off, bytes, elem, g_guard_serial++});
}

template <typename T>
T* dalloc(u64 count, u64* total) {
    void* p = nullptr;
    const u64 bytes = std::max<u64>(count * sizeof(T), 16);
    HIP_CHECK(hipMalloc(&p, bytes + guard_extra(bytes)));
    zero_new(p, bytes);
    guard_arm(p, bytes, sizeof(T));
    *total += bytes;
    return (T*)p;
}

// The tables every transfer probes at random (account rows and directory, the id
// index).  Rounds 2-3 allocated them physically contiguous
// (hipExtMallocWithFlags(hipDeviceMallocContiguous)) for fewer translations.  In a
// process whose earlier contexts had freed such allocations, later contexts then
// read and wrote data that was not theirs (wrong query rows, account rows of an
// earlier state, an illegal address): the whole GPU suite passes with plain
// allocations and fails without them (gpurun_out/r04e).  Plain
// allocations it is; TBGPU_CONTIG=1 restores the contiguous ones for experiments.
template <typename T>
T* dalloc_hot(u64 count, u64* total) {
#if !defined(TBGPU_NO_CONTIG)
    static const bool contig = getenv("TBGPU_CONTIG") != nullptr;
    void* p = nullptr;
    const u64 bytes = std::max<u64>(count * sizeof(T), 16);
    if (contig && hipExtMallocWithFlags(&p, bytes + guard_extra(bytes), hipDeviceMallocContiguous) == hipSuccess && p) {
        zero_new(p, bytes);
        guard_arm(p, bytes, sizeof(T));
        *total += bytes;
        return (T*)p;
    }
    (void)hipGetLastError();
#endif
    return dalloc<T>(count, total);
}

}  // namespace

// TBGPU_FLUSH_CALLS=1 (diagnostics): every entry point first writes back and
// invalidates every XCD's L2 (system-scope release + acquire in many workgroups), so
// no kernel of the call can hit a line an earlier kernel or ctx left in an L2.
__global__ void k_flush_caches() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
}
static void entry_flush(hipStream_t s) {
    guard_check_all(s);
    static const bool on = getenv("TBGPU_FLUSH_CALLS") != nullptr;
    if (!on) return;
    k_flush_caches<<<4096, 64, 0, s>>>();
    HIP_CHECK(hipGetLastError());
}

constexpr u32 PC_RING = 1024;        // pass-counter ring (passes in flight << ring)
constexpr u32 PASS_GROUP_MAX = 48;   // passes enqueued between two host round trips
// The fixed point's pass budget: past it the chunk's events from the front on are
// walked in execute's order (transfers.hip tr_walk).  BASELINE config 3 converges in
// 14-18 passes per 20-batch chunk; a chunk past 64 is a deep dependency chain, where
// passes cost O(n) each and the walk O(1) per event.
constexpr u32 WALK_PASSES = 64;
constexpr u32 WALK_UNDO = 4 * 8192;   // a linked chain's balance moves (<= 2 per member, members <= a batch)
constexpr u32 PC_OFF = 32;           // the pass-change ring's offset behind the counter words
static_assert(PC_OFF >= CNT_COUNT, "counter words overlap the pass-change ring");
constexpr u32 EPI_WORD = 28;         // the apply kernels' gate (TrArgs::epi), between the counters and the ring
static_assert(EPI_WORD >= CNT_COUNT && EPI_WORD < PC_OFF, "gate word placement");
constexpr u32 AC_GATE_WORD = 27;     // create_accounts: the one-evaluation path's gate (ac_launch_gate)
static_assert(AC_GATE_WORD >= CNT_COUNT && AC_GATE_WORD < PC_OFF && AC_GATE_WORD != EPI_WORD, "gate word placement");

struct tbgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    tbgpu_options opt{};
    Tables T{};
    u64 aidx_cap = 0, xrow_cap = 0, xidx_cap = 0, hist_cap = 0;
    u64 accounts_max = 0;
    u64 n_accounts = 0, n_rows = 0, n_hist = 0;
    u64 n_foreign = 0;  // ledger shard: other shards' accounts in the directory
    u64 bytes = 0;

    // per-call scratch (nmax events, bmax batches)
    u64 nmax = 0, bmax = 0, gcap = 0;
    u8* ev_buf = nullptr;  // nmax * 128
    u32* b_start = nullptr;
    u64* b_ts = nullptr;
    u64* ts = nullptr;
    u32 *cs = nullptr, *ce = nullptr;
    u8* sres = nullptr;
    u32 *dslot, *cslot, *pre_e, *pre_p, *pp_dslot, *pp_cslot, *gslot, *pslot, *prev_id, *pend_last, *pend_first,
        *prev_pend;
    u32 *gclaim, *gcnt_id, *gcnt_pd, *gmem, *gbeg, *gend, *gfill, *pfill, *pbeg;
    EvalState st[2];
    u64 scap = 0, side_m = 0;  // side capacity, sides of the last fixed point
    u32 *skey, *sval, *skey_s, *sval_s, *spos;
    u32 *soff, *sev, *scs, *scand, *sq_ev, *sq_cs;
    EvCore* core = nullptr;
    u32* tstart = nullptr;
    uint2* epos = nullptr;
    u8* sq_ok = nullptr;
    u128 *sq_dpend = nullptr, *sq_dpost = nullptr;
    u32 *gkey_s, *gsorted;  // the id-group sort's output (the members of each id group, by event)
    u32 *lst_simple, *lst_complex;  // the fixed point's per-pass work lists (tr_lists)
    u32 *d_ev, *d_chain, *d_slot, *d_win;  // the passes' dirty stamps (engine.h Dirty)
    Bal4* bb = nullptr;
    u128* bh = nullptr;  // headroom passes: one balance figure per side (balances.hip)
    u64* sd64 = nullptr; // the current chunk's compact side deltas (Sides::sq_d64), or null
    SortScratch ss{};
    void* side_tiles = nullptr;
    Scan3Scratch sc{};
    u8 *fres, *mask;
    uint4* ranks = nullptr;
    u8* res_buf = nullptr;  // nmax * 8 results
    u32* counts = nullptr;
    u32* counters = nullptr;
    int* status = nullptr;
    u32* h_counters = nullptr;  // pinned
    u32* h_counts = nullptr;    // pinned, bmax
    u8* h_res = nullptr;        // pinned, nmax * 8: a chunk's replies for host-buffer calls
    u64* h_stage_ts = nullptr;  // pinned, bmax
    u32* h_stage_start = nullptr;  // pinned, bmax + 1
    u32* h_stage_dev = nullptr;    // its device address (k_upload_block reads it)
    bool ev_in_host = false;       // this chunk's events are read in place from host memory
    // fast path (fast.hip)
    u32* f_gtab = nullptr;
    u32* f_gpos = nullptr;
    u64 f_gcap = 0;
    u128* f_keys = nullptr;
    u32* f_rows = nullptr;
    u64* f_tile_idr = nullptr;
    // routed (sharded) calls: per-event timestamps / chain control of the current
    // chunk in device memory (null for ordinary calls), dry-run flag and sink
    u64* rt_ts_buf = nullptr;
    u8* rt_ctl_buf = nullptr;
    u64* rt_dry_ts = nullptr;
    u64* rt_stats = nullptr;  // [5] tbgpu_route_stats
    // the router's kernels run on their own stream: a routed step's scatter may
    // overlap the previous step's commit (tigerbeetle_amd/shard.py pipelining)
    hipStream_t route_stream = nullptr;
    // the router's send-side scatter (route.hip), grown on demand
    u64 ro_cap = 0, ro_bcap = 0;
    uint2* ro_orank = nullptr;
    u32* ro_blk = nullptr;
    u32* ro_bstart = nullptr;
    u64* ro_counts = nullptr;
    u32* ro_bcount = nullptr;  // [256] spanning counts per owner, then [world * batches] per (owner, batch)
    u64 ro_bc_cap = 0;
    u64* ro_spart = nullptr;  // rt_rank's per-workgroup eligibility records
    // the general step's device directory (directory.hip), grown on demand
    u64 rd_cap = 0;
    u32* rd_claim = nullptr;
    int64_t* rd_first = nullptr;  // [2 * table]: first positions, then their hints
    u32* rd_slot = nullptr;
    struct {
        const void* events;
        u64 n;
        u32 world;
    } ro_ranked{};  // what tbgpu_route_prepare ranked last (tbgpu_route_scatter skips that pass)
    const u64* rt_ev_ts = nullptr;
    const u8* rt_ctl = nullptr;
    bool rt_dry = false;
    u32 slow_chunks = 0;  // consecutive chunks that needed the fixed point
    u32 fast_misses = 0;  // consecutive fast attempts that fell back (they back off: fast_due)
    // a small chunk's batch block held back for fp_prep (upload_batches with
    // allow_inline): flush_block launches k_upload_block if no fp_prep took it
    BlockInline blk{};
    u32 blk_words = 0;
    // a fast attempt enqueued without its round trip (try_fast spec): settled at the
    // call's next wait (spec_settle), undone there if it fell back
    // one caller at a time (tbgpu.h "Concurrency"): main entry points, and the router's
    // send side, which may overlap a commit (its own stream and buffers)
    std::recursive_mutex call_mu, route_mu;
    bool spec_pending = false;
    FastArgs spec_F{};
    // a small one-chunk call's end stored by fp_tail (fp_commit_small's mode) instead of
    // k_report: where to (set for the call's last chunk), and whether it did
    TailReport tail_rp{};
    bool tail_reported = false;
    u32 call_seq = 0;          // the last small call's sequence number (fp_tail stores it last)
    // TBGPU_HOST_TRACE=1 (diagnostics): host time of the drop-in call's steps, averaged
    // over its calls and printed at deinit
    std::chrono::steady_clock::time_point ht0{};
    double ht_sum[8] = {};
    u64 ht_calls = 0;
    bool ht_on = false;
    bool stats_lazy = false;   // stats.device_ms still to be read from ev0 / ev1 (tbgpu_last_stats)
    // whether the last fast attempt's ids did not rise (FL_NONMONO): the next attempt then
    // claims its ids eagerly in fp_commit (FastArgs::eager)
    bool ids_nonmono = false;
    // The prepared drop-in commit (tbgpu_prefetch_transfers with a small fast call ahead):
    // pinned words the gate kernel polls -- [GW_GO] the commit's sequence number (or
    // | GATE_CANCEL_BIT), [GW_TS..+1] its timestamp, [GW_ACK] the sequence number of a
    // gate that let nothing through -- and the device word the gated kernels read.
    u32* h_gate = nullptr;
    u32* h_gate_dev = nullptr;
    u32* gate_status = nullptr;
    u32* ac_fast_words = nullptr;  // the clean create_accounts call's flags and ticket (all-zero between calls)
    bool gate_pending = false;  // a prepared commit is enqueued and not yet released or cancelled
    bool gate_arm = false;      // try_fast: gate the kernels it launches on gate_status
    u32 gate_seq = 0, gate_n = 0;
    // Prepared commits of staged bodies (tbgpu_stage_transfers), enqueued at prepare
    // time behind the current one, in commit order: each classifies its batch once the
    // commits before it have run, then waits for its own commit call.
    struct Prepared {
        u32 seq, n;
        int slot;
        u64 key_lo, key_hi;
        FastArgs F;
        TailReport rp;
    };
    std::deque<Prepared> pq;
    u64 pq_events = 0;  // their events (rows they may take)
    u32 gate_last = 0;  // the newest prepared commit's sequence number (a cancel covers it and all before)
    u64 gate_budget = 0;        // wall-clock ticks a gate waits before letting nothing through
    u32 last_passes = 8;  // passes the last fixed point took (sizes the next pass group)
    bool long_segments = false;  // this call has an account segment too long for the fused scan
    // fixed-point pass counters, a ring of PC_RING words: changes per pass (the gate
    // of the next pass); a second ring: the first event each pass changed (the
    // walk's front); a third is spare (diagnostics)
    u32* pc = nullptr;
    // the walk (tr_walk), allocated on first use: per side, its account segment's
    // start, and per segment start the running balance; the open chain's undo log
    u32* w_sstart = nullptr;
    Bal4* w_bal = nullptr;
    u32* w_undo_slot = nullptr;
    Bal4* w_undo_val = nullptr;
    u32* w_out = nullptr;
    u64* rg_part = nullptr;    // tr_range's per-block records
    u64* ac_part = nullptr;    // ac_mask's per-workgroup max accepted timestamp
    u32* h_pc = nullptr;       // pinned mirror of the change ring
    u64* h_base = nullptr;     // pinned mirror of T.base
    u32* h_rc = nullptr;       // pinned per-batch reply counts of the current call
    // the end of a call in one copy (k_report): counter words, T.base, the last chunk's
    // reply counts
    u32* h_report = nullptr;  // pinned
    // page-locked staging for copies to and from caller memory (h2d / d2h): one ring
    // per stream (the routed pipeline's threads use the ctx's two streams at once), two
    // halves each, a half reusable once the copy recorded behind it has run
    struct UpRing {
        u8* h[2] = {nullptr, nullptr};
        const u8* d[2] = {nullptr, nullptr};  // their device addresses (k_copy_in reads them)
        hipEvent_t ev[2] = {nullptr, nullptr};
        int next = 0;
    } up[2];
    u32* h_report_dev = nullptr;  // its device address, and h_res's
    u64* h_res_dev = nullptr;
    u64 h_rc_cap = 0;
    u64 rows_hi = 0;           // upper bound of T.base[BASE_ROWS] (n_rows + events enqueued since)
    u64 eager_events = 0;      // events of eager-claim attempts since the last tombstone check
    // tbgpu_prefetch_transfers: one batch staged in HBM ahead of its commit
    u8* pf_buf = nullptr;          // TBGPU_BATCH_MAX * 128 bytes
    const void* pf_src = nullptr;  // the caller's buffer it was copied from
    u32 pf_n = 0;
    bool pf_valid = false;
    hipEvent_t pf_ev = nullptr;    // recorded behind the copy
    const u8* pf_dev = nullptr;    // where the prefetched body is in HBM: pf_buf, or a stage slot
    int pf_slot = -1;              // the stage slot it is (-1: pf_buf)
    // tbgpu_stage_transfers (StateMachine.prepare): bodies copied into HBM at prepare
    // time, one slot per prepare the pipeline may hold, keyed by the caller's content key;
    // the copies run on a stream of their own, so staging never waits behind (or releases)
    // a prepared commit's gate on the engine stream.  Allocated on first use.
    struct StageSlot {
        u8* d = nullptr;           // TBGPU_BATCH_MAX * 128 bytes in HBM
        u8* h = nullptr;           // page-locked shadow for a pageable source (first need)
        const u8* h_dev = nullptr;
        u64 key_lo = 0, key_hi = 0;
        u32 n = 0;
        bool valid = false;
        bool used = false;         // a prefetch has taken it (the first to reuse)
        u64 seq = 0;               // staging order
        hipEvent_t staged = nullptr;    // behind its copy (stage stream)
    } stg[TBGPU_STAGE_SLOTS];
    hipStream_t stage_stream = nullptr;
    u64 stage_seq = 0;
    // account-transfers index (query.hip), allocated by the first compaction
    u32 *q_key = nullptr, *q_val = nullptr, *q_tkey = nullptr, *q_tval = nullptr;
    SortScratch q_ss{};
    u64* q_runs_dev = nullptr;
    std::vector<u64> q_runs{0};  // row boundaries of the index runs; back() = rows indexed
    // the grooves' field index trees (index.hip), per (groove, field), built on demand
    struct FieldIx {
        u32* key = nullptr;
        u32* val = nullptr;
        std::vector<u64> runs{0};  // object row boundaries of the runs; back() = rows indexed
        u64* runs_dev = nullptr;
    } ix[2][10];
    u32* ix_tkey = nullptr;
    u32* ix_tval = nullptr;
    SortScratch ix_ss{};
    u8* ximp = nullptr;          // per stored row: 1 = imported from another shard
    hipEvent_t ev0, ev1;
    hipEvent_t ev_side, ev_lists;  // fixed_point's side count and work-list lengths landed
    hipEvent_t ev_group;           // a pass group's counters landed (before its apply kernels ran)
    // phase profiler: consecutive marks on the ctx stream; segment k belongs to
    // the phase opened by mark k.
    bool prof = false;
    std::vector<hipEvent_t> prof_pool;
    std::vector<int> prof_phase;
    tbgpu_stats stats{};
    char err[256] = {0};
};

enum { GW_GO = 0, GW_TS = 2, GW_ACK = 4, GW_WORDS = 8 };

// Release a prepared commit that will not be committed (any other call on the ctx): its
// gate then lets nothing through, and the work behind it on the stream goes on.
// The queued ones behind it go too (their batches were classified against a state the
// released commit would have left).  The word only ever grows: a release is the next
// sequence number, a cancel covers every sequence number up to the newest prepared.
static void gate_cancel(tbgpu_ctx* c) {
    if (!c->gate_pending && c->pq.empty()) return;
    if (c->gate_pending) {
        c->gate_pending = false;
        c->spec_pending = false;
        c->tail_reported = false;
    }
    c->pq.clear();
    c->pq_events = 0;
    __atomic_store_n(&c->h_gate[GW_GO], c->gate_last | GATE_CANCEL_BIT, __ATOMIC_RELEASE);
}

// The next call sequence number (31 bits, never 0: the gate word's top bit marks a cancel).
static u32 next_seq(tbgpu_ctx* c) {
    c->call_seq = (c->call_seq + 1) & ~GATE_CANCEL_BIT;
    if (c->call_seq == 0) c->call_seq = 1;
    return c->call_seq;
}

// Entry guard (tbgpu.h "Concurrency"): a ctx serves one caller at a time, except that
// the router's send side (tbgpu_route_stats / _prepare / _scatter / _scatter_packed /
// _unpack / _unpack_packed: the route stream and buffers of their own) may run on one
// thread while another commits on the same ctx (shard.py's pipelined stream).  Nested
// entry on the same thread is allowed; overlapping calls otherwise abort.
struct CallGuard {
    std::recursive_mutex& mu;
    // keep_gate: the entry points that complete a prepared commit (prefetch_wait, the
    // commit itself); every other call on the engine stream releases it first
    CallGuard(tbgpu_ctx* c, bool route, bool keep_gate = false) : mu(route ? c->route_mu : c->call_mu) {
        HIP_CHECK(hipSetDevice(c->device));
        if (!mu.try_lock())
            tbgpu_fatal("ctx", route ? "concurrent router calls on one ctx" : "concurrent calls on one ctx", __FILE__,
                        __LINE__);
        if (!route && !keep_gate) gate_cancel(c);
    }
    ~CallGuard() { mu.unlock(); }
};


static bool host_trace() {
    static const bool on = getenv("TBGPU_HOST_TRACE") != nullptr;
    return on;
}
// mark k of the drop-in call's host timeline (no-op unless the call is being traced)
static inline void ht_mark(tbgpu_ctx* c, int k) {
    if (!c->ht_on || c->ht_calls <= 16) return;  // (the first calls load code objects)
    c->ht_sum[k] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c->ht0).count();
}

static void alloc_scratch(tbgpu_ctx* c, u64 nmax) {
    u64& B = c->bytes;
    c->nmax = nmax;
    c->bmax = nmax + 2;
    c->gcap = pow2_at_least(4 * nmax);
    // sides: two per transfer; a post/void with several candidate pendings has more
    // (engine.h Sides); beyond this capacity a call falls back to one pair each
    const u64 n = nmax, m = 3 * nmax;
    c->ev_buf = dalloc<u8>(n * 128, &B);
    // batch starts then batch timestamps in one block, staged by one copy per chunk
    c->b_start = dalloc<u32>(batch_ts_offset(c->bmax) + 2 * c->bmax, &B);
    c->b_ts = (u64*)(c->b_start + batch_ts_offset(c->bmax));
    c->ts = dalloc<u64>(n, &B);
    c->cs = dalloc<u32>(n, &B);
    c->ce = dalloc<u32>(n, &B);
    c->sres = dalloc<u8>(n, &B);
    u32** u32s[] = {&c->dslot, &c->cslot, &c->pre_e, &c->pre_p, &c->pp_dslot, &c->pp_cslot,
                    &c->gslot, &c->pslot, &c->prev_id, &c->pend_last, &c->pend_first, &c->prev_pend};
    for (u32** p : u32s) *p = dalloc<u32>(n, &B);
    u32** g32s[] = {&c->gclaim, &c->gcnt_id, &c->gcnt_pd, &c->gmem, &c->gbeg, &c->gend, &c->gfill, &c->pfill,
                    &c->pbeg};
    for (u32** p : g32s) *p = dalloc<u32>(c->gcap, &B);
    for (EvalState& s : c->st) {
        s.res = dalloc<u8>(n, &B);
        s.ok = dalloc<u8>(n, &B);
        s.pref = dalloc<u32>(n, &B);
        s.cfail = dalloc<u32>(n, &B);
        s.amt = dalloc<u128>(n, &B);
        s.pamt = dalloc<u128>(n, &B);
    }
    c->scap = m;
    c->skey = dalloc<u32>(m, &B);
    c->sval = dalloc<u32>(m, &B);
    c->skey_s = dalloc<u32>(m, &B);
    c->sval_s = dalloc<u32>(m, &B);
    c->spos = dalloc<u32>(m, &B);
    c->soff = dalloc<u32>(n + 1, &B);
    c->core = dalloc<EvCore>(n, &B);
    c->tstart = dalloc<u32>(m / side_scan_fused_tile() + 2, &B);
    c->epos = dalloc<uint2>(nmax + 1, &B);
    c->sev = dalloc<u32>(m, &B);
    c->scs = dalloc<u32>(m, &B);
    c->scand = dalloc<u32>(m, &B);
    c->sq_ev = dalloc<u32>(m, &B);
    c->sq_cs = dalloc<u32>(m, &B);
    c->sq_ok = dalloc<u8>(m, &B);
    c->sq_dpend = dalloc<u128>(m, &B);
    c->sq_dpost = dalloc<u128>(m, &B);
    c->lst_simple = dalloc<u32>(n, &B);
    c->lst_complex = dalloc<u32>(n, &B);
    c->d_ev = dalloc<u32>(2 * n, &B);
    c->d_chain = dalloc<u32>(2 * n, &B);
    c->d_slot = dalloc<u32>(2 * c->gcap, &B);
    c->d_win = dalloc<u32>(m / side_scan_fused_tile() + 2, &B);
    c->gkey_s = dalloc<u32>(n, &B);
    c->gsorted = dalloc<u32>(n, &B);
    c->bb = dalloc<Bal4>(m, &B);
    c->bh = dalloc<u128>(m, &B);
    c->ss.keys_tmp = dalloc<u32>(m, &B);
    c->ss.vals_tmp = dalloc<u32>(m, &B);
    c->ss.hist = dalloc<u32>(radix_sort_hist_words(m), &B);
    c->ss.capacity = m;
    c->side_tiles = dalloc<u8>(side_scan_tile_bytes(m), &B);
    c->sc.tile_sums = dalloc<uint4>(scan3_tile_words(n), &B);
    c->sc.capacity = n;
    c->fres = dalloc<u8>(n + 16, &B);  // + a 16-byte load's tail (fp_chains reads 16 results per lane)
    c->mask = dalloc<u8>(n, &B);
    c->ranks = dalloc<uint4>(n + 1, &B);
    c->res_buf = dalloc<u8>(n * 8, &B);
    c->counts = dalloc<u32>(c->bmax, &B);
    // the counters, then the pass-change ring: one copy brings both back per pass group
    c->counters = dalloc<u32>(PC_OFF + 3 * PC_RING, &B);
    c->status = dalloc<int>(4, &B);
    c->f_gcap = pow2_at_least(2 * nmax);
    c->f_gtab = dalloc<u32>(c->f_gcap, &B);
    c->f_gpos = dalloc<u32>(n, &B);
    c->f_keys = dalloc<u128>(n, &B);
    c->f_rows = dalloc<u32>(n, &B);
    c->f_tile_idr = dalloc<u64>(TILE_WORDS * (std::max<u64>(fp_tiles(nmax), FP_TAIL_MAX / FP_SMALL_TILE) + 1), &B);
    c->rt_ts_buf = dalloc<u64>(n, &B);
    c->rt_ctl_buf = dalloc<u8>(n, &B);
    c->rt_dry_ts = dalloc<u64>(1, &B);
    c->rt_stats = dalloc<u64>(8, &B);
    c->pc = c->counters + PC_OFF;
    c->rg_part = dalloc<u64>(tr_range_part_words(n), &B);
    c->ac_part = dalloc<u64>(n / 256 + 2, &B);
    c->pf_buf = dalloc<u8>((u64)TBGPU_BATCH_MAX * 128, &B);
    HIP_CHECK(hipEventCreateWithFlags(&c->pf_ev, hipEventDisableTiming));

    HIP_CHECK(hipHostMalloc((void**)&c->h_base, 8 * sizeof(u64), hipHostMallocDefault));  // [4..5]: a uint4
    HIP_CHECK(hipHostMalloc((void**)&c->h_counters, (PC_OFF + 3 * PC_RING) * sizeof(u32), hipHostMallocDefault));
    c->h_pc = c->h_counters + PC_OFF;
    // Host buffers that kernels read or write in place (k_report's stores, k_upload_block's
    // loads) are coherent: the GPU does not keep their lines in its caches, so a kernel
    // never reads a previous call's staged block and the host never reads a report the
    // device has not written back.
    constexpr unsigned HOST_COHERENT = hipHostMallocMapped | hipHostMallocCoherent;
    // (+1: the small calls' sequence word, fp_tail's last store; +1: the clean
    // create_accounts call's flags, ac_fast_index's last store)
    HIP_CHECK(hipHostMalloc((void**)&c->h_report, (RPT_COUNTS + c->bmax + 2) * sizeof(u32), HOST_COHERENT));
    HIP_CHECK(hipHostMalloc((void**)&c->h_res, c->nmax * 8 + 8, HOST_COHERENT));
    HIP_CHECK(hipHostMalloc((void**)&c->h_gate, GW_WORDS * sizeof(u32), HOST_COHERENT));
    memset(c->h_gate, 0, GW_WORDS * sizeof(u32));
    HIP_CHECK(hipHostGetDevicePointer((void**)&c->h_gate_dev, c->h_gate, 0));
    {
        int khz = 0;  // the wall clock the gate times its wait with
        HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
        c->gate_budget = (u64)std::max(khz, 1) * 10;  // 10 ms
    }
    HIP_CHECK(hipHostGetDevicePointer((void**)&c->h_res_dev, c->h_res, 0));
    HIP_CHECK(hipHostGetDevicePointer((void**)&c->h_report_dev, c->h_report, 0));
    HIP_CHECK(hipHostMalloc((void**)&c->h_counts, c->bmax * sizeof(u32), hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc((void**)&c->h_stage_start, (batch_ts_offset(c->bmax) + 2 * c->bmax) * sizeof(u32),
                            HOST_COHERENT));
    c->h_stage_ts = (u64*)(c->h_stage_start + batch_ts_offset(c->bmax));
    HIP_CHECK(hipHostGetDevicePointer((void**)&c->h_stage_dev, c->h_stage_start, 0));
    poison_host(c->h_base, 8 * sizeof(u64));
    poison_host(c->h_counters, (PC_OFF + 3 * PC_RING) * sizeof(u32));
    poison_host(c->h_report, (RPT_COUNTS + c->bmax + 1) * sizeof(u32));
    poison_host(c->h_res, c->nmax * 8 + 8);
    poison_host(c->h_counts, c->bmax * sizeof(u32));
    poison_host(c->h_stage_start, (batch_ts_offset(c->bmax) + 2 * c->bmax) * sizeof(u32));
}

enum { PH_UPLOAD = 0, PH_CLASSIFY = 1, PH_SORT = 2, PH_SCAN = 3, PH_EVAL = 4, PH_APPLY = 5, PH_INDEX = 6, PH_PREP = 7, PH_END = -1 };

static void prof_mark(tbgpu_ctx* c, int phase) {
    if (!c->prof) return;
    const size_t k = c->prof_phase.size();
    if (k >= c->prof_pool.size()) return;  // pool exhausted: stop recording
    HIP_CHECK(hipEventRecord(c->prof_pool[k], c->stream));
    c->prof_phase.push_back(phase);
}

static void prof_collect(tbgpu_ctx* c) {
    for (double& v : c->stats.phase_ms) v = 0;
    if (!c->prof || c->prof_phase.size() < 2) { c->prof_phase.clear(); return; }
    HIP_CHECK(hipEventSynchronize(c->prof_pool[c->prof_phase.size() - 1]));
    for (size_t k = 0; k + 1 < c->prof_phase.size(); k++) {
        const int ph = c->prof_phase[k];
        if (ph < 0 || ph >= 8) continue;
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, c->prof_pool[k], c->prof_pool[k + 1]));
        c->stats.phase_ms[ph] += ms;
    }
    c->prof_phase.clear();
}

extern "C" void tbgpu_set_profiling(tbgpu_ctx* c, int enable) {
    HIP_CHECK(hipSetDevice(c->device));
    c->prof = enable != 0;
    if (c->prof && c->prof_pool.empty()) {
        c->prof_pool.resize(4096);
        for (hipEvent_t& e : c->prof_pool) HIP_CHECK(hipEventCreate(&e));
    }
    c->prof_phase.clear();
}

static void stage_init(tbgpu_ctx* c);

extern "C" int tbgpu_init(tbgpu_ctx** out, const tbgpu_options* options) {
    *out = nullptr;
    tbgpu_options o{};
    if (options) o = *options;
    if (!o.accounts_max) o.accounts_max = 1u << 20;
    if (!o.transfers_max) o.transfers_max = 1u << 24;
    if (!o.history_max) o.history_max = 1u << 16;
    if (!o.events_per_call_max) o.events_per_call_max = 1u << 20;
    if (o.events_per_call_max < TBGPU_BATCH_MAX) o.events_per_call_max = TBGPU_BATCH_MAX;
    if (o.transfers_max >= 0x7FFFFFFFull || o.events_per_call_max >= (1ull << 29)) return -22;
    if (!o.directory_max) o.directory_max = o.accounts_max;
    if (o.directory_max < o.accounts_max) return -22;
    if (!o.hashed_max) o.hashed_max = o.directory_max;
    if (o.shard_world >= 2 && o.shard_rank >= o.shard_world) return -22;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -19;  // ENODEV
    if (o.device < 0 || o.device >= ndev) return -19;
    tbgpu_ctx* c = new tbgpu_ctx();
    c->opt = o;
    c->device = o.device;
    HIP_CHECK(hipSetDevice(c->device));
    HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&c->route_stream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&c->ev0));
    HIP_CHECK(hipEventCreate(&c->ev1));
    HIP_CHECK(hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&c->ev_lists, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&c->ev_group, hipEventDisableTiming));
    c->accounts_max = o.accounts_max;
    // ids outside the direct-mapped directory, at load <= 1/8 while the index stays within
    // 1 GiB (a probe's first slot then nearly always decides it: one dependent load for a
    // random u128 id), else <= 1/2 (TBGPU_OPT_DENSE_INDEXES, or TBGPU_AIDX_LOAD2 for A/B
    // timing: <= 1/2 always)
    static const bool load2 = getenv("TBGPU_AIDX_LOAD2") != nullptr;
    c->aidx_cap = pow2_at_least(2 * o.hashed_max);
    if (!load2 && !(o.flags & TBGPU_OPT_DENSE_INDEXES) && c->aidx_cap * 4 * sizeof(AccIdx) <= (1ull << 30))
        c->aidx_cap *= 4;
    c->xrow_cap = o.transfers_max;
    // the transfer-id index at load <= 1/8 while it stays within 8 GiB (random u128 ids:
    // an eager claim's first CAS then nearly always takes its slot), else <= 1/2
    // (TBGPU_OPT_DENSE_INDEXES, or TBGPU_XIDX_LOAD2 for A/B timing: <= 1/2 always)
    static const bool xload2 = getenv("TBGPU_XIDX_LOAD2") != nullptr;
    const bool dense_ix = (o.flags & TBGPU_OPT_DENSE_INDEXES) != 0;
    c->xidx_cap = pow2_at_least(2 * o.transfers_max);
    if (!xload2 && !dense_ix && c->xidx_cap * 4 * sizeof(u64) <= (8ull << 30)) c->xidx_cap *= 4;
    c->hist_cap = o.history_max;
    u64& B = c->bytes;
    ZeroOn zero_on(c->stream);
    c->T.acc = dalloc_hot<Account>(o.accounts_max, &B);
    c->T.aidx = dalloc_hot<AccIdx>(c->aidx_cap, &B);
    c->T.aidx_mask = c->aidx_cap - 1;
    c->T.xrows = dalloc<Transfer>(c->xrow_cap, &B);
    c->T.xful = dalloc<u8>(c->xrow_cap, &B);
    c->T.xidx = dalloc_hot<u64>(c->xidx_cap, &B);
    c->T.xidx_mask = c->xidx_cap - 1;
    c->T.hrows = dalloc<History>(c->hist_cap, &B);
    c->T.commit_ts = dalloc<u64>(2, &B);
    c->T.idr = dalloc<u64>(4, &B);
    c->T.xrun = dalloc<u64>(8, &B);
    c->T.big = dalloc<u32>(4, &B);
    c->gate_status = dalloc<u32>(4, &B);  // the prepared commit's verdict, and its timestamp at [2..3]
    c->ac_fast_words = dalloc<u32>(2, &B);
    c->T.hcount = c->T.big + 1;        // [1] entries, [2] refused, [3] transfer-id tombstones
    c->T.hash_limit = pow2_at_least(2 * o.hashed_max) / 2;  // hashed_max (rounded up): load <= 0.5 at most
    c->T.base = dalloc<u64>(4, &B);
    c->T.shard_world = o.shard_world >= 2 ? o.shard_world : 0;
    c->T.shard_rank = o.shard_world >= 2 ? o.shard_rank : 0;
    c->T.xrow_cap = c->xrow_cap;
    c->T.hist_cap = c->hist_cap;
    // row + 1 in 29 bits (all ones: another shard's account); ids below 2^32 in block
    // 0, or dense_block_span-wide blocks for ledger-major ids, one spare block (ledgers
    // are numbered from 1)
    if (o.accounts_max > 0 && o.accounts_max < (1ull << 29) - 2) {
        const u64 dm = o.directory_max;
        const u64 span = o.dense_block_span ? o.dense_block_span : std::max<u64>(dm, 1);
        c->T.dense_span = span;
        c->T.dense_blocks = o.dense_block_span ? (dm + span - 1) / span + 2 : 1;
        c->T.dense_n = c->T.dense_span * c->T.dense_blocks;
        if (!o.dense_block_span) c->T.dense_n = dm;
    }
    c->T.dense = dalloc_hot<u64>(c->T.dense_n, &B);
    alloc_scratch(c, o.events_per_call_max);
    stage_init(c);
    tbgpu_reset(c);
    *out = c;
    return 0;
}

extern "C" void tbgpu_reset(tbgpu_ctx* c) {
    CallGuard guard_(c, false);
    c->pf_valid = false;
    HIP_CHECK(hipMemsetAsync(c->T.aidx, 0, c->aidx_cap * sizeof(AccIdx), c->stream));
    HIP_CHECK(hipMemsetAsync(c->T.xful, 0, c->xrow_cap, c->stream));
    HIP_CHECK(hipMemsetAsync(c->T.xidx, 0, c->xidx_cap * sizeof(u64), c->stream));
    HIP_CHECK(hipMemsetAsync(c->T.commit_ts, 0, 2 * sizeof(u64), c->stream));
    HIP_CHECK(hipMemsetAsync(c->T.idr, 0, 2 * sizeof(u64), c->stream));                  // max = 0
    HIP_CHECK(hipMemsetAsync(c->T.idr + 2, 0xFF, 2 * sizeof(u64), c->stream));           // min = ~0
    HIP_CHECK(hipMemsetAsync(c->T.xrun, 0, 8 * sizeof(u64), c->stream));                 // empty run
    HIP_CHECK(hipMemsetAsync(c->T.big, 0, 4 * sizeof(u32), c->stream));  // the guard and the index occupancy
    HIP_CHECK(hipMemsetAsync(c->T.base, 0, 4 * sizeof(u64), c->stream));
    HIP_CHECK(hipMemsetAsync(c->counters, 0, CNT_COUNT * sizeof(u32), c->stream));  // CNT_STICKY included
    if (c->T.dense_n) HIP_CHECK(hipMemsetAsync(c->T.dense, 0, c->T.dense_n * sizeof(u64), c->stream));
    if (c->ximp) HIP_CHECK(hipMemsetAsync(c->ximp, 0, c->xrow_cap, c->stream));
    HIP_CHECK(hipMemsetAsync(c->f_gtab, 0, c->f_gcap * sizeof(u32), c->stream));  // fast path's claim table
    // Words matched against values a new ctx repeats (sequence numbers restart at 1,
    // the clean accounts call's ticket at 0): a recycled allocation must not hold a
    // previous ctx's prepared-commit verdict or ticket
    HIP_CHECK(hipMemsetAsync(c->gate_status, 0, 4 * sizeof(u32), c->stream));
    HIP_CHECK(hipMemsetAsync(c->ac_fast_words, 0, 2 * sizeof(u32), c->stream));
    wait_stream(c->stream);
    c->h_report[RPT_COUNTS + c->bmax] = 0;  // (the small calls' sequence word: never 0)
    c->n_accounts = c->n_rows = c->n_hist = 0;
    c->n_foreign = 0;
    c->rows_hi = 0;
    c->q_runs.assign(1, 0);
    for (auto& g : c->ix)
        for (auto& x : g) x.runs.assign(1, 0);
}

extern "C" void tbgpu_deinit(tbgpu_ctx* c) {
    if (!c) return;
    gate_cancel(c);  // (a prepared commit's gate lets nothing through; the sync below then ends)
    if (c->ht_calls) {
        static const char* what[8] = {"guard", "ev0 recorded", "batch block", "fp_commit launched",
                                      "fp_tail launched", "ev1 recorded", "end seen", "returned"};
        const double nc = (double)(c->ht_calls > 16 ? c->ht_calls - 16 : 1);
        fprintf(stderr, "tbgpu host trace: %llu drop-in calls after 16, mean us since entry:",
                (unsigned long long)(c->ht_calls > 16 ? c->ht_calls - 16 : 0));
        for (int k = 0; k < 8; k++) fprintf(stderr, " %s %.2f;", what[k], c->ht_sum[k] / nc);
        fprintf(stderr, "\n");
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->route_stream);
    // Free every device allocation by walking the struct's pointers.
    guard_check_all(c->stream);
    for (void* p : {(void*)c->ro_orank, (void*)c->ro_blk, (void*)c->ro_bstart, (void*)c->ro_counts,
                    (void*)c->ro_bcount, (void*)c->ro_spart, (void*)c->rd_claim, (void*)c->rd_first,
                    (void*)c->rd_slot})
        if (p) { guard_release(p); (void)hipFree(p); }
    void* ptrs[] = {c->T.dense, c->T.acc, c->T.aidx, c->T.xrows, c->T.xful, c->T.xidx, c->T.hrows, c->T.commit_ts, c->T.idr, c->T.xrun, c->T.big, c->gate_status, c->ac_fast_words, c->ev_buf,
                    c->b_start, c->ts, c->cs, c->ce, c->sres, c->dslot, c->cslot, c->pre_e, c->pre_p,
                    c->pp_dslot, c->pp_cslot, c->gslot, c->pslot, c->prev_id, c->pend_last, c->pend_first, c->prev_pend,
                    c->gclaim, c->gcnt_id, c->gcnt_pd, c->gmem, c->gbeg, c->gend, c->gfill, c->pfill, c->pbeg, c->skey, c->sval, c->skey_s,
                    c->soff, c->core, c->tstart, c->epos, c->sev, c->scs, c->scand, c->sq_ev, c->sq_cs, c->sq_ok, c->sq_dpend, c->sq_dpost, c->gkey_s,
                    c->gsorted,
                    c->sval_s, c->spos, c->bb, c->bh, c->ss.keys_tmp, c->ss.vals_tmp, c->ss.hist, c->side_tiles,
                    c->sc.tile_sums, c->fres, c->mask, c->ranks, c->res_buf, c->counts, c->counters, c->status,
                    c->f_gtab, c->f_gpos, c->f_keys, c->f_rows,
                    c->f_tile_idr, c->rt_ts_buf, c->rt_ctl_buf, c->rt_dry_ts, c->rt_stats, c->rg_part, c->T.base, c->q_key, c->q_val, c->q_tkey,
                    c->q_tval, c->q_ss.keys_tmp, c->q_ss.vals_tmp, c->q_ss.hist, c->q_runs_dev, c->ximp,
                    c->lst_simple, c->lst_complex, c->d_ev, c->d_chain, c->d_slot, c->d_win, c->w_sstart, c->w_bal,
                    c->w_undo_slot, c->w_undo_val, c->w_out, c->ac_part, c->pf_buf};
    for (void* p : ptrs) if (p) { guard_release(p); (void)hipFree(p); }
    for (auto& g : c->ix)
        for (auto& x : g)
            for (void* p : {(void*)x.key, (void*)x.val, (void*)x.runs_dev})
                if (p) { guard_release(p); (void)hipFree(p); }
    for (void* p : {(void*)c->ix_tkey, (void*)c->ix_tval, (void*)c->ix_ss.keys_tmp, (void*)c->ix_ss.vals_tmp,
                    (void*)c->ix_ss.hist})
        if (p) { guard_release(p); (void)hipFree(p); }
    for (EvalState& s : c->st) {
        void* q[] = {s.res, s.ok, s.pref, s.cfail, s.amt, s.pamt};
        for (void* p : q) if (p) { guard_release(p); (void)hipFree(p); }
    }
    if (c->h_counters) (void)hipHostFree(c->h_counters);
    if (c->h_report) (void)hipHostFree(c->h_report);
    if (c->h_gate) (void)hipHostFree(c->h_gate);
    if (c->h_counts) (void)hipHostFree(c->h_counts);
    if (c->h_stage_start) (void)hipHostFree(c->h_stage_start);
    if (c->h_base) (void)hipHostFree(c->h_base);
    if (c->h_rc) (void)hipHostFree(c->h_rc);
    if (c->h_res) (void)hipHostFree(c->h_res);
    for (auto& R : c->up)
        for (int h = 0; h < 2; h++) {
            if (R.h[h]) (void)hipHostFree(R.h[h]);
            if (R.ev[h]) (void)hipEventDestroy(R.ev[h]);
        }
    for (hipEvent_t e : c->prof_pool) (void)hipEventDestroy(e);
    if (c->pf_ev) (void)hipEventDestroy(c->pf_ev);
    if (c->stage_stream) (void)hipStreamSynchronize(c->stage_stream);
    for (auto& S : c->stg) {
        if (S.d) { guard_release(S.d); (void)hipFree(S.d); }
        if (S.h) (void)hipHostFree(S.h);
        if (S.staged) (void)hipEventDestroy(S.staged);
    }
    if (c->stage_stream) (void)hipStreamDestroy(c->stage_stream);
    (void)hipEventDestroy(c->ev0);
    (void)hipEventDestroy(c->ev1);
    (void)hipEventDestroy(c->ev_side);
    (void)hipEventDestroy(c->ev_lists);
    (void)hipEventDestroy(c->ev_group);
    (void)hipStreamDestroy(c->stream);
    (void)hipStreamDestroy(c->route_stream);
    delete c;
}

// ------------------------------------------------------------ helpers -----

// The end of a call: counter words, the device cursors and the last chunk's reply
// counts (and, for host-buffer calls, its replies) stored straight into pinned host
// memory, so that no copy follows the call's last kernel (three small copies and the
// replies' copy were four dispatches, each an engine hand-off of ~10 us).  Vector
// stores over PCIe, made visible to the host before the launch completes.
__global__ void k_report(const u32* counters, const u64* base, const u32* counts, u32 nb, u32* out,
                         const u64* replies, u64* out_replies) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < RPT_BASE) out[i] = counters[i];
    else if (i < RPT_COUNTS) out[i] = ((const u32*)base)[i - RPT_BASE];
    else if (i < RPT_COUNTS + nb) out[i] = counts[i - RPT_COUNTS];
    if (out_replies) {
        const u64 total = base[BASE_REPLIES];
        for (u64 j = i; j < total; j += (u64)gridDim.x * blockDim.x) out_replies[j] = replies[j];
    }
    __threadfence_system();
}

static void read_counters(tbgpu_ctx* c) {
    HIP_CHECK(hipMemcpyAsync(c->h_counters, c->counters, CNT_COUNT * sizeof(u32), hipMemcpyDeviceToHost, c->stream));
    wait_stream(c->stream);
}

// Host copies of the device cursors (stored rows, history rows), exact for all work
// enqueued so far.  One round trip.
static void refresh_bases(tbgpu_ctx* c) {
    HIP_CHECK(hipMemcpyAsync(c->h_base, c->T.base, 4 * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
    wait_stream(c->stream);
    c->n_rows = c->h_base[BASE_ROWS];
    c->n_hist = c->h_base[BASE_HIST];
    c->rows_hi = c->n_rows;
}

// A device word written by a kernel (the value travels as its argument): device
// memory that kernels read is only ever written by kernels (see h2d).
__global__ void k_store_u64(u64* p, u64 v) {
    if (threadIdx.x == 0) *p = v;
}
static void set_base(tbgpu_ctx* c, int k, u64 v) {
    k_store_u64<<<1, 64, 0, c->stream>>>(c->T.base + k, v);
    HIP_CHECK(hipGetLastError());
}

static void ensure_h_rc(tbgpu_ctx* c, u64 nb) {
    if (nb <= c->h_rc_cap) return;
    if (c->h_rc) HIP_CHECK(hipHostFree(c->h_rc));
    c->h_rc_cap = std::max<u64>(nb, 1024);
    HIP_CHECK(hipHostMalloc((void**)&c->h_rc, c->h_rc_cap * sizeof(u32), hipHostMallocDefault));
    poison_host(c->h_rc, c->h_rc_cap * sizeof(u32));
}

// Splits batches [b0, b_end) into chunks of whole batches of <= nmax events.
// The fixed point's passes grow with the dependency depth of a call, which grows
// with its batch count; calls that need it are cut into chunks of at most this
// many batches (the streaming semantics are those of consecutive calls anyway).
static u32 general_chunk_batches() {
    static const u32 v = [] {  // TBGPU_CHUNK_BATCHES: experiments only
        const char* e = getenv("TBGPU_CHUNK_BATCHES");
        // config 3, 60-batch calls (r04, profiles/r04/chunk_sweep2.sh): 16: 167-170, 20: 184-188,
        // 24: 182-186, 32 (then 28): 189-196, 40 (then 20): 182-183 M/s; cut evenly since
        return e ? (u32)strtoul(e, nullptr, 0) : 32u;
    }();
    return v;
}

// A chunk limit cuts the remaining batches into equal chunks (60 batches at a limit of
// 32: two of 30, not 32 + 28), so no short chunk pays the fixed point's setup alone.
static u32 chunk_end(const tbgpu_ctx* c, const uint32_t* counts, u32 b0, u32 nb, u32 max_batches = ~0u) {
    if (max_batches != ~0u && max_batches > 0 && nb > b0) {
        const u32 rest = nb - b0, k = (rest + max_batches - 1) / max_batches;
        max_batches = (rest + k - 1) / k;
    }
    u64 ev = 0;
    u32 b = b0;
    while (b < nb && b - b0 < c->bmax - 2 && b - b0 < max_batches) {
        if (ev + counts[b] > c->nmax) break;
        ev += counts[b];
        b++;
    }
    if (b == b0) tbgpu_fatal("batches", "a single batch exceeds events_per_call_max", __FILE__, __LINE__);
    return b;
}

// A chunk's batch block (starts, then timestamps) read by one kernel straight from
// the pinned staging buffer, with the reply cursor's reset when asked: one dispatch
// where a small copy (itself a blit dispatch) and a fill were two.
__global__ void k_upload_block(const u32* host_block, u32 words, u32* block, u64* base, u32 reset_replies) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < words) block[i] = host_block[i];
    if (i == 0 && reset_replies) base[BASE_REPLIES] = 0;
}

static void flush_block(tbgpu_ctx* c) {
    if (!c->blk_words) return;
    k_upload_block<<<1, 256, 0, c->stream>>>(c->h_stage_dev, c->blk_words, c->b_start, c->T.base,
                                             c->blk.reset_replies);
    HIP_CHECK(hipGetLastError());
    c->blk_words = 0;
}

// The held-back block for fp_prep (consumed: the caller launches fp_prep with it).
static BlockInline take_block(tbgpu_ctx* c) {
    BlockInline b{};
    if (c->blk_words) {
        b = c->blk;
        b.words = c->blk_words;
        c->blk_words = 0;
    }
    return b;
}

static bool inline_disabled() {
    static const bool d = getenv("TBGPU_NO_INLINE_BLOCK") != nullptr;  // A/B timing
    return d;
}

static void upload_batches(tbgpu_ctx* c, const uint64_t* timestamps, const uint32_t* counts, u32 nb,
                           std::vector<u32>& starts, bool reset_replies = false, bool allow_inline = false) {
    starts.resize(nb + 1);
    starts[0] = 0;
    for (u32 b = 0; b < nb; b++) starts[b + 1] = starts[b] + counts[b];
    // staged through pinned memory so the copies are truly asynchronous (every
    // call synchronizes before the staging buffer is reused)
    // one copy of this chunk's block: its nb + 1 starts, then (8-byte aligned) its nb
    // timestamps; b_ts points into the block for this chunk
    const u64 off = batch_ts_offset(nb);
    c->h_stage_ts = (u64*)(c->h_stage_start + off);
    c->b_ts = (u64*)(c->b_start + off);
    memcpy(c->h_stage_ts, timestamps, nb * sizeof(u64));
    memcpy(c->h_stage_start, starts.data(), (nb + 1) * sizeof(u32));
    const u32 words = (u32)(off + 2 * nb);
    // a block still held back belongs to a chunk none of whose kernels ran (a fast
    // attempt refused before its launches, the chunk redone): this one supersedes it
    c->blk_words = 0;
    if (allow_inline && words <= BLOCK_INLINE_WORDS && !inline_disabled()) {
        // a small call: fp_prep writes the block from its arguments (one launch less);
        // any other first kernel is preceded by flush_block
        c->blk.block = c->b_start;
        c->blk.base = c->T.base;
        c->blk.reset_replies = reset_replies ? 1u : 0u;
        memcpy(c->blk.w, c->h_stage_start, words * sizeof(u32));
        c->blk_words = words;
        return;
    }
    k_upload_block<<<(words + 255) / 256, 256, 0, c->stream>>>(c->h_stage_dev, words, c->b_start, c->T.base,
                                                               reset_replies ? 1u : 0u);
    HIP_CHECK(hipGetLastError());
}

// Device replies are concatenated across the chunk's batches; the host C-ABI
// places batch b's reply at the batch's event offset.  The caller has copied them
// back into the pinned staging buffer h_res (the chunk is complete).
static void copy_results_to_batches(tbgpu_ctx* c, u32 nb, const std::vector<u32>& starts, const u32* counts,
                                    u8* dst_chunk) {
    u64 total = 0;
    for (u32 b = 0; b < nb; b++) total += counts[b];
    if (total == 0) return;
    const u8* tmp = c->h_res;  // copied back with the chunk's counts
    u64 off = 0;
    for (u32 b = 0; b < nb; b++) {
        memcpy(dst_chunk + (u64)starts[b] * 8, tmp + off * 8, (u64)counts[b] * 8);
        off += counts[b];
    }
}

static TrArgs make_tr_args(tbgpu_ctx* c, const Transfer* ev, u32 n, u32 nb) {
    TrArgs C{};
    C.ev = ev; C.n = n; C.nb = nb;
    C.b_start = c->b_start; C.b_ts = c->b_ts;
    C.ts = c->ts; C.core = c->core; C.cs = c->cs; C.ce = c->ce; C.sres = c->sres;
    C.dslot = c->dslot; C.cslot = c->cslot; C.pre_e = c->pre_e; C.pre_p = c->pre_p;
    C.pp_dslot = c->pp_dslot; C.pp_cslot = c->pp_cslot; C.gslot = c->gslot; C.pslot = c->pslot;
    C.prev_id = c->prev_id; C.pend_last = c->pend_last; C.pend_first = c->pend_first; C.prev_pend = c->prev_pend;
    C.gclaim = c->gclaim; C.gcnt_id = c->gcnt_id; C.gcnt_pd = c->gcnt_pd; C.gmem = c->gmem;
    C.gbeg = c->gbeg; C.gend = c->gend; C.gmembers = c->gsorted;
    C.gfill = c->gfill; C.pfill = c->pfill; C.pbeg = c->pbeg;
    C.glist = c->gkey_s;  // scratch (free before the sides are built)
    C.plist = c->skey;
    C.sd.soff = c->soff; C.sd.sev = c->sev; C.sd.scs = c->scs; C.sd.scand = c->scand; C.sd.spos = c->spos; C.sd.skey_s = c->skey_s;
    C.sd.sq_ev = c->sq_ev; C.sd.sq_cs = c->sq_cs; C.sd.sq_ok = c->sq_ok; C.sd.sq_dpend = c->sq_dpend;
    C.sd.sq_dpost = c->sq_dpost;
    C.sd.tstart = c->tstart;
    C.sd.epos = c->epos;
    C.sd.tile = side_scan_fused_tile();
    C.sd.inert = (u32)c->accounts_max;
    // group table sized for this call: >= 2x the keys (ids + pending ids <= 2n)
    const u64 g = std::min<u64>(c->gcap, pow2_at_least(4ull * std::max<u32>(n, 1)));
    C.gmask = g - 1;
    C.counters = c->counters;
    C.ev_ts = c->rt_ev_ts;
    C.ctl = c->rt_ctl;
    C.dry = c->rt_dry ? 1u : 0u;
    C.commit_ts = c->rt_dry ? c->rt_dry_ts : c->T.commit_ts;
    static const bool debug = getenv("TBGPU_TRACE_PASSES") != nullptr;  // diagnostics only
    C.debug = debug ? 1u : 0u;
    // sparse passes below n / 8 changes (TBGPU_SPARSE_SHIFT: A/B timing, 0 = never)
    static const u32 sparse = getenv("TBGPU_SPARSE_SHIFT") ? (u32)atoi(getenv("TBGPU_SPARSE_SHIFT")) : 3u;
    C.sparse = sparse;
    C.lst_simple = c->lst_simple;
    C.lst_complex = c->lst_complex;
    C.dt = Dirty{c->d_ev, c->d_chain, c->d_slot, c->d_win, c->counters + CNT_ALL, n, (u32)(C.gmask + 1)};
    return C;
}

// Single-pass attempt (fast.hip).  Returns false, with every balance delta
// undone, when some event needs the fixed point.  Replies go after the device
// reply cursor; `counts_dev` receives the per-batch reply counts.
static bool try_fast(tbgpu_ctx* c, const Transfer* ev, u32 n, u32 nb, tbgpu_create_transfers_result_t* results_dev,
                     bool spec) {
    hipStream_t s = c->stream;
    if (c->rows_hi + n > c->xrow_cap) {
        refresh_bases(c);  // the bound is loose: look at the exact count
        if (c->n_rows + n > c->xrow_cap) return false;  // let the general path report capacity exactly
    }
    FastArgs F{};
    F.ev = ev; F.n = n; F.nb = nb; F.b_start = c->b_start; F.b_ts = c->b_ts; F.ev_ts = c->rt_ev_ts;
    F.gtab = c->f_gtab;
    F.gpos = c->f_gpos;
    F.gmask = std::min<u64>(c->f_gcap, pow2_at_least(2ull * n)) - 1;
    F.fres = c->fres;
    F.counters = c->counters;
    F.batch_counts = c->counts;
    F.results = results_dev;
    F.row_base = c->rows_hi;
    F.keys = c->f_keys;
    F.rows = c->f_rows;
    F.tile_idr = c->f_tile_idr;
    F.ctl = c->rt_ctl;
    F.fres2 = c->mask;
    F.dry = c->rt_dry ? 1u : 0u;
    F.commit_ts = c->rt_dry ? c->rt_dry_ts : c->T.commit_ts;
    static const bool no_tail = getenv("TBGPU_NO_TAIL") != nullptr;  // A/B timing of the launch sequence
    static const bool no_small = getenv("TBGPU_NO_SMALL") != nullptr;  // A/B timing: 512-event tiles, fp_prep
    // A drop-in call (one chunk of at most FP_TAIL_MAX events, its verdict read with the
    // call's end): two launches, fp_commit_small (64-event tiles over 128 CUs for 8190
    // events, no fp_prep before it) and fp_tail, which also stores the call's end into
    // pinned host memory (no k_report after it).
    F.small = (spec && n <= FP_TAIL_MAX && !no_tail && !no_small) ? 1u : 0u;
    F.tile = F.small ? FP_SMALL_TILE : fp_tile_events();
    static const bool no_eager = getenv("TBGPU_NO_EAGER") != nullptr;  // A/B timing: fp_dupcheck + inserts
    F.eager = (c->ids_nonmono && !F.dry && !no_eager) ? 1u : 0u;
    if (F.eager) c->eager_events += n;
    GateArgs ga{};
    if (c->gate_arm) {  // a prepared commit (prepare_gated): the tiles wait for the commit call
        F.gate = c->gate_status;
        F.gate_seq = c->gate_seq;
        ga = GateArgs{c->h_gate_dev + GW_GO, (const u64*)(c->h_gate_dev + GW_TS), c->h_gate_dev + GW_ACK, c->gate_budget};
    }
    const BlockInline bi = take_block(c);
    prof_mark(c, PH_PREP);
    if (!F.small) fp_launch_prep(F, s, bi);
    prof_mark(c, PH_CLASSIFY);
    F.ev_copy = c->ev_in_host ? (Transfer*)c->ev_buf : nullptr;
    // the simple small call ends in fp_commit_small's last tile (TBGPU_NO_FUSE: A/B timing)
    static const bool no_fuse = getenv("TBGPU_NO_FUSE") != nullptr;
    F.fuse = (F.small && c->tail_rp.out && c->tail_rp.seq_out && !no_fuse) ? 1u : 0u;
    fp_launch_commit(c->T, F, s, F.small ? bi : BlockInline{}, F.small ? c->tail_rp : TailReport{}, ga);
    ht_mark(c, 3);
    if (F.ev_copy) {  // the later launches read fp_commit's HBM copy of the events
        F.ev = F.ev_copy;
        F.ev_copy = nullptr;
    }
    prof_mark(c, PH_INDEX);
    if (n <= FP_TAIL_MAX && !no_tail) {
        // a small call: index, fix and advance in one workgroup, gated on the device's
        // flags like the speculative launches below
        c->tail_reported = F.small && c->tail_rp.out;
        fp_launch_tail(c->T, F, s, F.small ? bi : BlockInline{}, F.small ? c->tail_rp : TailReport{});
        ht_mark(c, 4);
        prof_mark(c, PH_END);
        c->stats.path = 1;
        c->stats.iterations = 1;
        if (spec) {  // the flags come back with the call's k_report
            c->spec_F = F;
            c->spec_pending = true;
            return true;
        }
        HIP_CHECK(hipMemcpyAsync(c->h_counters, c->counters, CNT_COUNT * sizeof(u32), hipMemcpyDeviceToHost, s));
        wait_stream(s);
        const u32 flags = c->h_counters[CNT_FLAGS];
        if (!F.dry) c->ids_nonmono = (flags & FL_NONMONO) != 0;
        if (flags & FL_ERROR) tbgpu_fatal("create_transfers", "fast path look-back did not complete", __FILE__, __LINE__);
        if (flags & FL_SLOW) {
            fp_launch_undo(c->T, F, s);
            return false;
        }
        if (!F.dry) c->rows_hi += c->h_counters[CNT_OK];
        return true;
    }
    fp_launch_index(c->T, F, s);
    if (spec) {
        // the whole call is this one chunk: the fix (replies and rows at their ranks
        // when there are failures) and the cursor advance are enqueued at once, gated
        // on the device's flags, and the flags come back with the call's own final
        // copies; spec_settle undoes the attempt if it fell back
        prof_mark(c, PH_APPLY);
        fp_launch_fix(c->T, F, c->mask, c->ranks, c->sc, s);
        fp_launch_advance(c->T, F, s);
        prof_mark(c, PH_END);
        c->spec_F = F;  // the flags come back with the call's k_report
        c->spec_pending = true;
        c->stats.path = 1;
        c->stats.iterations = 1;
        return true;
    }
    prof_mark(c, PH_END);
    // one round trip: the flags decide whether the attempt stands
    HIP_CHECK(hipMemcpyAsync(c->h_counters, c->counters, CNT_COUNT * sizeof(u32), hipMemcpyDeviceToHost, s));
    wait_stream(s);
    const u32 flags = c->h_counters[CNT_FLAGS];
    if (!F.dry) c->ids_nonmono = (flags & FL_NONMONO) != 0;
    if (flags & FL_ERROR) tbgpu_fatal("create_transfers", "fast path look-back did not complete", __FILE__, __LINE__);
    if (flags & FL_SLOW) {
        fp_launch_undo(c->T, F, s);  // commit_timestamp back; the deltas (a dry run applied none)
        return false;
    }
    if (c->h_counters[CNT_BAD]) {
        // failures: rows to their ranks, replies, then the index on the final rows
        prof_mark(c, PH_APPLY);
        fp_launch_fix(c->T, F, c->mask, c->ranks, c->sc, s);
        prof_mark(c, PH_END);
    }
    fp_launch_advance(c->T, F, s);
    if (!F.dry) c->rows_hi += c->h_counters[CNT_OK];
    c->stats.path = 1;
    c->stats.iterations = 1;
    return true;
}

// The fixed point's bounded worst case (transfers.hip tr_walk): the chunk's events
// from the chain start of `front`'s event on, walked in execute's order in state D
// (every earlier event final there).  The sides are rebuilt when a post/void resolves
// to a pending outside them, and the walk resumes at its chain.
template <typename Rebuild>
static void walk(tbgpu_ctx* c, const TrArgs& C, u32 n, EvalState& D, const u32* front_dev, u64& m,
                 Rebuild&& build_sides) {
    hipStream_t s = c->stream;
    if (!c->w_sstart) {
        u64& B = c->bytes;
        ZeroOn zero_on(s);
        c->w_sstart = dalloc<u32>(c->scap, &B);
        c->w_bal = dalloc<Bal4>(c->scap, &B);
        c->w_undo_slot = dalloc<u32>(WALK_UNDO, &B);
        c->w_undo_val = dalloc<Bal4>(WALK_UNDO, &B);
        c->w_out = dalloc<u32>(4, &B);
    }
    // the front's chain start: every event before it is final
    u32 f = 0;
    HIP_CHECK(hipMemcpyAsync(c->h_base + 4, front_dev, sizeof(u32), hipMemcpyDeviceToHost, s));
    wait_stream(s);
    memcpy(&f, c->h_base + 4, sizeof f);
    if (f >= n) f = 0;
    HIP_CHECK(hipMemcpyAsync(c->h_base + 4, C.cs + f, sizeof(u32), hipMemcpyDeviceToHost, s));
    wait_stream(s);
    u32 start = 0;
    memcpy(&start, c->h_base + 4, sizeof start);
    u32* one = c->pc + 2 * PC_RING;  // the scan's open gate
    for (;;) {
        tr_launch_walk_prep(C, m, start, c->w_sstart, D.cfail, s);
        HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)one, 1, 1, s));
        SideScanArgs SA{};
        SA.skey = c->skey_s; SA.sq_ev = c->sq_ev; SA.sq_cs = c->sq_cs; SA.sq_ok = c->sq_ok;
        SA.sq_dpend = c->sq_dpend; SA.sq_dpost = c->sq_dpost; SA.sq_d64 = c->sd64; SA.n = n;
        SA.over = c->sd64 ? c->counters + CNT_FLAGS : nullptr;  // (the walk's Bal4 scans of a 64-bit-form chunk)
        SA.cfail = D.cfail;
        SA.cfail_clear = nullptr;
        SA.gate = PassGate{one, c->counters + CNT_RESORT, 0, 1};
        // the balance of every side before the front's events (the walked ones' records are zero)
        side_scan(SA, m, (u32)c->accounts_max, true, c->side_tiles, c->T.acc, c->bb, s);
        tr_launch_walk(c->T, C, D, c->bb, m, c->w_sstart, c->w_bal, c->w_undo_slot, c->w_undo_val, WALK_UNDO, start,
                       c->w_out, s);
        HIP_CHECK(hipMemcpyAsync(c->h_base + 4, c->w_out, 2 * sizeof(u32), hipMemcpyDeviceToHost, s));
        wait_stream(s);
        u32 out[2];
        memcpy(out, c->h_base + 4, sizeof out);
        if (out[1]) tbgpu_fatal("create_transfers", "walk: a linked chain's undo log overflowed", __FILE__, __LINE__);
        if (out[0] == NONE32) {
            // the balances every side sees in the walked state, as a converged pass leaves
            // them for the apply kernels (bs_final's account balances, history rows)
            side_scan(SA, m, (u32)c->accounts_max, true, c->side_tiles, c->T.acc, c->bb, s);
            break;
        }
        // a post/void resolved to a pending outside its sides: rebuild them from D
        // (its resolution is then a candidate) and walk on from its chain
        HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)(c->counters + CNT_RESORT), 0, 1, s));
        build_sides(D);
        start = out[0];
    }
}

// The general path's fixed point over one chunk (transfers.hip): classify, group,
// the optimistic initial state, then Jacobi passes enqueued in groups without a
// host round trip inside a group (the kernels of the passes after convergence
// return at once), until a pass changes nothing.  Behind every group the host also
// enqueues the gate word and `epilogue(m)` (the apply kernels, gated on it), so when
// the group converges they run right behind it instead of after the round trip.
// Returns the converged state.
template <typename Epi>
static EvalState* fixed_point(tbgpu_ctx* c, const TrArgs& C0, u32 n, Epi&& epilogue, bool allow_h64 = true) {
    hipStream_t s = c->stream;
    TrArgs C = C0;  // (its side deltas' form is decided below, once classify's flags are back)
    C.sd.sq_d64 = nullptr;
    c->sd64 = nullptr;
    const u64 g = C.gmask + 1;
    const u32 inv_acc = (u32)c->accounts_max;  // side keys are account rows
    const int bits_acc = log2u(c->accounts_max + 1);

    u32* chg = c->pc;
    prof_mark(c, PH_CLASSIFY);
    tr_launch_prep(C, c->st[0].cfail, c->pc, PC_RING, s);
    tr_launch_classify(c->T, C, s);

    // The sides of the events, sorted by account.  Their count (tr_side_count's bound,
    // which classify's results decide) is enqueued right behind classify, so its host
    // round trip overlaps the grouping and the initial state instead of idling the GPU.
    u64 m = 0;
    u32 n_list[2] = {0, 0};  // the per-pass work lists' lengths (simple, complex)
    auto count_sides = [&](u32 kmax) {
        tr_launch_side_count(C, kmax, c->mask, s);
        scan3_exclusive(c->mask, c->ranks, n, c->sc, s);
        HIP_CHECK(hipMemcpyAsync(c->h_base + 4, c->ranks + n, sizeof(uint4), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipEventRecord(c->ev_side, s));
    };
    count_sides(SIDE_CANDS);
    bool counted = true;  // a count is in flight for the first build

    // grouping by id / pending id: each step runs only when classify found the need
    tr_launch_group(C, 2, s);  // id and pending groups together
    tr_launch_group2(C, s);
    tr_launch_init_lists(c->T, C, c->st[0], c->st[1], s);
    HIP_CHECK(hipMemcpyAsync(c->h_base + 6, c->counters + CNT_NSIMPLE, 2 * sizeof(u32), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(c->h_base + 7, c->counters + CNT_FLAGS, sizeof(u32), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipEventRecord(c->ev_lists, s));

    auto build_sides = [&](const EvalState& S, bool records = true) {
        prof_mark(c, PH_SORT);
        for (u32 kmax : {SIDE_CANDS, 1u}) {
            if (!counted) count_sides(kmax);
            counted = false;
            wait_event(c->ev_side);
            uint4 tot;
            memcpy(&tot, c->h_base + 4, sizeof tot);
            m = 2ull * (tot.x + tot.y + tot.z);
            if (m <= c->scap) {
                tr_launch_side_build(C, S, kmax, c->ranks, inv_acc, c->skey, c->sval, s);
                break;
            }
        }
        if (m > c->scap) tbgpu_fatal("create_transfers", "side capacity", __FILE__, __LINE__);
        radix_sort_pairs(c->skey, c->sval, c->skey_s, c->sval_s, m, bits_acc, c->ss, s);
        tr_launch_side_pos(C, c->sval_s, m, s);
        if (records) tr_launch_side_rec(C, S, s);
        c->stats.sorts++;
    };
    build_sides(c->st[0], false);  // (its side records once the deltas' form is known)
    wait_event(c->ev_lists);  // (long landed: the sort is queued behind it)
    memcpy(n_list, c->h_base + 6, sizeof n_list);
    u32 cflags = 0;
    memcpy(&cflags, c->h_base + 7, sizeof cflags);
    // Headroom passes (balances.hip side_scan_fused_narrow) unless an amount or a
    // committed balance is too large for them (FL_WIDE); the Bal4 form then comes from
    // one full scan behind the converged group, for the apply kernels.
    static const bool no_narrow = getenv("TBGPU_NO_HEADROOM") != nullptr;  // A/B timing
    const bool narrow = !(cflags & FL_WIDE) && !no_narrow;
    // ... in 64-bit form when every amount is < 2^40, every committed balance < 2^61
    // (FL_WIDE64 clear) and the chunk has at most 2^20 events: every headroom of the
    // chunk then lies within +-2^63 (the committed ones within +-2^62, and the chunk moves
    // one by less than 2^20 * 2^40; a balancing amount never exceeds the headroom it
    // draws on), so the figures and the side deltas are exact as 64-bit two's
    // complement, and a pass moves half the bytes per side.
    static const bool no_h64 = getenv("TBGPU_NO_H64") != nullptr;  // A/B timing
    // A figure can still leave +-2^63 when balancing transfers pile several accounts'
    // headroom onto one: the scan (a Bal4 pass of a long segment or the walk: a balance
    // past 2^62, or a delta that does not fit) raises FL_H64_OVER, the group applies
    // nothing, and the chunk is redone from its start in the u128 form.
    const bool h64 = allow_h64 && narrow && !c->long_segments && !(cflags & FL_WIDE64) && n <= (1u << 20) && !no_h64;
    if (h64) {
        c->sd64 = (u64*)c->sq_dpend;  // [2m] u64 in the u128 array's memory
        C.sd.sq_d64 = c->sd64;
        C.sd.over = c->counters + CNT_FLAGS;
    }
    tr_launch_side_rec(C, c->st[0], s);

    SideScanArgs SA{};
    SA.skey = c->skey_s; SA.sq_ev = c->sq_ev; SA.sq_cs = c->sq_cs; SA.sq_ok = c->sq_ok;
    SA.sq_dpend = c->sq_dpend; SA.sq_dpost = c->sq_dpost; SA.sq_d64 = c->sd64; SA.n = n;
    SA.over = h64 ? c->counters + CNT_FLAGS : nullptr;
    SA.dt = C.dt;
    SA.lst_complex = c->lst_complex;
    SA.gslot = c->gslot; SA.pslot = c->pslot; SA.cs = c->cs; SA.ce = c->ce;
    const bool chains = true;  // whether the call has chains is on the device: scan with the chain part
    static const bool no_incr = getenv("TBGPU_NO_INCR") != nullptr;  // A/B timing: every event every pass
    u32 p = 0;                  // next pass to enqueue
    // the first group: the last fixed point's passes plus a margin.  A pass past
    // convergence returns at once (≈3 µs a launch); a second group costs the host round
    // trip, the first group's gated epilogue run as no-ops and a second one launched
    // just in time (≈250 µs of a config-3 chunk in profiles/r05/kernel_trace_config3.csv)
    static const u32 margin = getenv("TBGPU_PASS_MARGIN") ? (u32)atoi(getenv("TBGPU_PASS_MARGIN")) : 3u;
    u32 group = std::max<u32>(2, std::min<u32>(c->last_passes + margin, PASS_GROUP_MAX));
    if (c->opt.flags & TBGPU_OPT_WALK_EARLY) group = 2;  // (tests) the walk after the first two passes
    u32 done_at = NONE32;
    for (;;) {
        if (p > n + 2 + PC_RING) tbgpu_fatal("create_transfers", "fixed point did not converge", __FILE__, __LINE__);
        prof_mark(c, PH_EVAL);  // the passes: balance scan + evaluation
        SA.n_complex = n_list[1];
        const u32 full = (no_incr || c->long_segments) ? 1u : 0u;
        for (u32 q = p; q < p + group; q++) {
            EvalState& S = c->st[q & 1];
            EvalState& D = c->st[(q + 1) & 1];
            PassGate G{chg + q % PC_RING, c->counters + CNT_RESORT, q, full};
            SA.cfail = S.cfail;
            SA.cfail_clear = D.cfail;
            SA.gate = G;
            const bool hr = narrow && !c->long_segments;
            TrArgs CE = C;
            CE.bh = hr && !h64 ? c->bh : nullptr;
            CE.bh64 = hr && h64 ? (const u64*)c->bh : nullptr;
            if (c->long_segments) {
                side_scan(SA, m, inv_acc, chains, c->side_tiles, c->T.acc, c->bb, s);
            } else if (hr) {
                SideScanArgs SN = SA;
                SN.bh = c->bh;
                SN.bh64 = (u64*)c->bh;
                static const bool no_sens = getenv("TBGPU_NO_SENS") != nullptr;  // A/B timing
                SN.all_sides = no_sens ? 1u : 0u;
                if (h64)
                    side_scan_fused_h64(SN, m, inv_acc, c->tstart, c->counters + CNT_LONG, c->T.acc, s);
                else
                    side_scan_fused_narrow(SN, m, inv_acc, c->tstart, c->counters + CNT_LONG, c->T.acc, s);
            } else {
                side_scan_fused(SA, m, inv_acc, c->tstart, c->counters + CNT_LONG, c->T.acc, c->bb, s);
            }
            tr_launch_evaluate_lists(c->T, CE, S, D, c->bb, G, chg + (q + 1) % PC_RING, chg + (q + 2) % PC_RING,
                                     chg + PC_RING + (q + 1) % PC_RING, chg + PC_RING + (q + 2) % PC_RING,
                                     n_list[0], n_list[1], s);
        }
        const u32 p0 = p;
        p += group;
        tr_launch_converged(chg, PC_RING, p0, p, c->counters, c->counters + EPI_WORD, s);
        // the group's counters come back now, and the host decides on them while the
        // apply kernels run (gated on the convergence word): a converged chunk's next
        // chunk is enqueued behind them without the GPU idling through the host's wake-up.
        // The apply kernels' own errors land in CNT_STICKY, read with the call's end.
        HIP_CHECK(hipMemcpyAsync(c->h_counters, c->counters, (PC_OFF + PC_RING) * sizeof(u32), hipMemcpyDeviceToHost,
                                 s));
        HIP_CHECK(hipEventRecord(c->ev_group, s));
        if (narrow && !c->long_segments) {
            // the Bal4 balances of the converged state (tr_apply's history rows, bs_final)
            SideScanArgs SF = SA;
            SF.gate = PassGate{c->pc + 2 * PC_RING, c->counters + CNT_RESORT, 0, 1};  // open, full
            SF.cfail = c->st[0].cfail;
            SF.cfail_alt = c->st[1].cfail;
            SF.cfail_clear = nullptr;
            SF.epi = c->counters + EPI_WORD;
            // (its long-segment word is the sticky one: the passes' narrow scans, over the
            // same windows, would have met such a segment first, so this is an error)
            side_scan_fused(SF, m, inv_acc, c->tstart, c->counters + CNT_STICKY, c->T.acc, c->bb, s);
        }
        epilogue(m);
        prof_mark(c, PH_END);
        wait_event(c->ev_group);
        if (c->h_counters[CNT_FLAGS] & FL_H64_OVER) {
            c->stats.h64_redos++;
            return fixed_point(c, C0, n, epilogue, false);
        }
        if (c->h_counters[CNT_FLAGS] & FL_FOREIGN)
            tbgpu_fatal("create_transfers", "a transfer of a ledger another shard owns (ledger shard ctx)", __FILE__,
                        __LINE__);
        if (c->h_counters[CNT_FLAGS] & FL_ERROR) tbgpu_fatal("create_transfers", "device error", __FILE__, __LINE__);
        static const bool trace = getenv("TBGPU_TRACE_PASSES") != nullptr;  // diagnostics only
        if (trace) {
            for (u32 q = p0; q < p; q++)
                fprintf(stderr, "tbgpu: n=%u pass %u changes %u\n", n, q, c->h_pc[(q + 1) % PC_RING]);
            const u32* d = c->h_counters + CNT_DBG;
            fprintf(stderr, "tbgpu: changed so far: regular %u balancing %u post/void %u; result changed %u, "
                            "chain members %u, limit accounts %u; resort %u\n", d[0], d[1], d[2], d[3], d[4], d[5],
                    c->h_counters[CNT_RESORT]);
        }
        const u32 lng = c->h_counters[CNT_LONG];
        if (lng) {
            // pass r's fused scan met an account segment longer than its window: redo
            // it, and the rest of the call, with the three-launch scan
            const u32 r = lng - 1;
            c->long_segments = true;
            HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)(c->counters + CNT_LONG), 0, 1, s));
            p = r;
            continue;
        }
        const u32 resort = c->h_counters[CNT_RESORT];
        if (resort) {
            // eval r resolved a post/void to a pending outside its sides: rebuild the
            // sides from its state (its resolution is then a candidate), go on at r + 1
            const u32 r = resort - 1;
            build_sides(c->st[(r + 1) & 1]);
            HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)(c->counters + CNT_RESORT), 0, 1, s));
            // new side positions: pass r + 1 evaluates and rescans everything
            HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)(c->counters + CNT_ALL), r + 1, 1, s));
            HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)(chg + (r + 1) % PC_RING), 1, 1, s));
            p = r + 1;
            continue;
        }
        for (u32 q = p0; q < p; q++)
            if (c->h_pc[(q + 1) % PC_RING] == 0) { done_at = q; break; }
        if (done_at != NONE32) break;
        const u32 budget = (c->opt.flags & TBGPU_OPT_WALK_EARLY) ? 2u : WALK_PASSES;
        if (p >= budget) {
            // past the pass budget: the last pass (p - 1) wrote st[p & 1]; walk on from its front
            walk(c, C, n, c->st[p & 1], c->pc + PC_RING + p % PC_RING, m, build_sides);
            if (h64) {  // the walk's Bal4 deltas of a 64-bit-form chunk
                HIP_CHECK(hipMemcpyAsync(c->h_counters + CNT_FLAGS, c->counters + CNT_FLAGS, sizeof(u32),
                                         hipMemcpyDeviceToHost, s));
                wait_stream(s);
                if (c->h_counters[CNT_FLAGS] & FL_H64_OVER) {
                    c->stats.h64_redos++;
                    return fixed_point(c, C0, n, epilogue, false);
                }
            }
            HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)(c->counters + EPI_WORD), (p & 1) ? 2 : 1, 1, s));
            epilogue(m);
            c->stats.iterations = p;
            c->stats.path = 2;
            c->last_passes = 8;
            c->side_m = m;
            c->stats.walks++;
            return &c->st[p & 1];
        }
        // the changes decay about geometrically: enqueue the passes that decay predicts
        const double last = c->h_pc[p % PC_RING], prev = c->h_pc[(p - 1) % PC_RING];
        const double r = prev > 0 ? std::min(0.9, std::max(0.05, last / prev)) : 0.5;
        group = (u32)std::ceil(std::log(last + 1.0) / -std::log(r)) + 1;
        group = std::max<u32>(2, std::min<u32>(group, PASS_GROUP_MAX));
    }
    static const bool probe = getenv("TBGPU_EVAL_PROBE") != nullptr;  // timing diagnostics only
    if (probe) {
        // the converged state evaluated again into the other buffer (unused afterwards)
        // under each probe mode: where a pass's evaluation time goes
        EvalState& S = c->st[(done_at + 1) & 1];
        EvalState& D = c->st[done_at & 1];
        u32* one = c->pc + 2 * PC_RING;  // spare ring: an open gate
        HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)one, 1, 1, s));
        PassGate G{one, c->counters + CNT_RESORT, 0, 1};
        for (u32 mode : {0u, 1u, 2u, 3u}) {
            TrArgs P = C;
            P.probe = mode;
            hipEvent_t e0, e1;
            HIP_CHECK(hipEventCreate(&e0));
            HIP_CHECK(hipEventCreate(&e1));
            HIP_CHECK(hipEventRecord(e0, s));
            for (int r = 0; r < 5; r++) tr_launch_evaluate(c->T, P, S, D, c->bb, G, one + 2, one + 3, one + 4, one + 5, s);
            HIP_CHECK(hipEventRecord(e1, s));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            fprintf(stderr, "tbgpu: eval probe mode %u: %.2f us per launch (n=%u)\n", mode, ms * 1e3f / 5, n);
            HIP_CHECK(hipEventDestroy(e0));
            HIP_CHECK(hipEventDestroy(e1));
        }
        for (u32 mode : {0u, 1u, 2u, 4u, 7u}) {
            SideScanArgs P = SA;
            P.probe = mode;
            P.cfail = S.cfail;
            P.cfail_clear = nullptr;
            P.gate = G;
            hipEvent_t e0, e1;
            HIP_CHECK(hipEventCreate(&e0));
            HIP_CHECK(hipEventCreate(&e1));
            HIP_CHECK(hipEventRecord(e0, s));
            for (int r = 0; r < 5; r++)
                side_scan_fused(P, m, inv_acc, c->tstart, c->counters + CNT_LONG, c->T.acc, c->bb, s);
            HIP_CHECK(hipEventRecord(e1, s));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            fprintf(stderr, "tbgpu: scan probe mode %u: %.2f us per launch (m=%llu)\n", mode, ms * 1e3f / 5,
                    (unsigned long long)m);
            HIP_CHECK(hipEventDestroy(e0));
            HIP_CHECK(hipEventDestroy(e1));
        }
        HIP_CHECK(hipMemsetAsync(c->counters + CNT_RESORT, 0, sizeof(u32), s));
    }
    c->stats.iterations = done_at + 1;
    c->last_passes = done_at + 1;
    c->side_m = m;
    return &c->st[(done_at + 1) & 1];
}

// One chunk of create_transfers: events already at `ev` on the device.  Replies go
// to `results_dev` after the device reply cursor, per-batch reply counts to c->counts.
// Returns false (nothing committed, every effect undone) when the fast path does
// not apply and `split` asks the caller to redo these batches in smaller chunks.
// Whether a chunk of a slow run tries the fast path first: every 8th chunk while the
// attempts are new, backing off to every 64th while they keep falling back (a failed
// attempt costs its fp_commit and its undo, ~0.15 ms per config-3 chunk).
static bool fast_due(const tbgpu_ctx* c) {
    return c->slow_chunks % (8u << std::min<u32>(c->fast_misses, 3u)) == 0;
}

static bool run_transfers_chunk(tbgpu_ctx* c, const Transfer* ev, u32 n, u32 nb,
                                tbgpu_create_transfers_result_t* results_dev, bool try_fast_path, bool split,
                                bool spec = false) {
    hipStream_t s = c->stream;
    c->stats.iterations = 0;
    c->stats.path = 0;
    if (n == 0) {
        flush_block(c);
        HIP_CHECK(hipMemsetAsync(c->counts, 0, nb * sizeof(u32), s));
        return true;
    }
    const bool fast_ok = try_fast_path && !(c->opt.flags & TBGPU_OPT_FORCE_GENERAL);
    if (fast_ok) {
        if (try_fast(c, ev, n, nb, results_dev, spec)) {
            c->slow_chunks = 0;
            if (!spec) c->fast_misses = 0;
            return true;
        }
        c->fast_misses++;
        if (split) return false;
    }
    c->slow_chunks++;
    flush_block(c);  // (a fast attempt's fp_prep has written it already)
    TrArgs C = make_tr_args(c, ev, n, nb);
    C.epi = c->counters + EPI_WORD;  // the apply kernels run only behind a converged pass group
    C.epi_alt = c->st[1];
    // apply: ranks of stored rows / results / history rows, at the device cursors,
    // from the converged state (st[0], or st[1] by the gate word)
    auto epilogue = [&](u64 m) {
        prof_mark(c, PH_APPLY);
        tr_launch_mask(c->T, C, c->st[0], c->fres, c->mask, s);
        scan3_exclusive(c->mask, c->ranks, n, c->sc, s);
        tr_launch_apply(c->T, C, c->st[0], c->fres, c->ranks, c->bb, results_dev, c->counts, c->rg_part, s);
        if (!c->rt_dry) {
            SideScanArgs SA{};
            SA.skey = c->skey_s; SA.sq_ev = c->sq_ev; SA.sq_cs = c->sq_cs; SA.sq_ok = c->sq_ok;
            SA.sq_dpend = c->sq_dpend; SA.sq_dpost = c->sq_dpost; SA.sq_d64 = c->sd64; SA.n = n;
            SA.cfail = c->st[0].cfail;
            SA.cfail_alt = c->st[1].cfail;
            SA.epi = C.epi;
            side_final_balances(SA, m, (u32)c->accounts_max, c->bb, c->T.acc, c->T.big, s);
        }
        tr_launch_advance(c->T, C, c->ranks, c->rg_part, s);
    };
    fixed_point(c, C, n, epilogue);
    if (!c->rt_dry) c->rows_hi += n;
    return true;
}

// TBGPU_NO_SPEC=1: every fast attempt waits for its own verdict (A/B timing)
static bool zero_copy_disabled() {  // TBGPU_NO_ZERO_COPY=1: always copy (A/B timing)
    static const bool d = getenv("TBGPU_NO_ZERO_COPY") != nullptr;
    return d;
}

// The device address of `bytes` of page-locked host memory at `p` (hipHostMalloc,
// hipHostRegister, a pinned torch tensor), or null for pageable memory.  The last
// byte must map into the same allocation, at the same offset: a buffer that runs past
// one pinned allocation (a region registered only in part, two adjacent registered
// regions) takes the copy path.
static const void* pinned_device_ptr(const void* p, u64 bytes) {
    hipPointerAttribute_t a{}, z{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable: not an error of the call
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || bytes == 0) return nullptr;
    const u8* last = (const u8*)p + bytes - 1;
    if (hipPointerGetAttributes(&z, last) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (z.type != hipMemoryTypeHost || z.devicePointer != (const u8*)a.devicePointer + (bytes - 1)) return nullptr;
    void* base = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&base, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) == hipSuccess &&
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) == hipSuccess && base) {
        if (last >= (const u8*)base + size) return nullptr;  // past the allocation that holds p
    } else {
        (void)hipGetLastError();  // the range is not reported: the last byte's mapping decided
    }
    return a.devicePointer;
}

// Host-to-device copy on `s`.  Sources are staged through the ctx's page-locked ring
// (a host memcpy per UP_HALF bytes) so every copy is a plain DMA from page-locked
// memory; a caller that declares its buffers page-locked (TBGPU_OPT_PINNED_INPUT) is
// copied from directly.  The runtime's pointer attributes alone are not trusted to
// tell page-locked from pageable memory.  The runtime's own handling of pageable sources was measured to
// let kernels read stale data in a long process (the copies' destinations are reused
// buffers -- the event buffer, the query filter -- and a later kernel saw the previous
// contents: DESIGN.md §5), so the engine never hands it a pageable source.
constexpr u64 UP_HALF = 4ull << 20;
// Device-to-device copy as a kernel on `s` (whole 4-byte words): the runtime's copy
// engines are not used between device buffers that kernels just wrote (a merged query
// index copied that way came back with entries missing in a long process).
__global__ void k_copy_words(u32* __restrict__ dst, const u32* __restrict__ src, u64 n) {
    for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x) dst[k] = src[k];
}
static void dcopy(void* dst, const void* src, u64 bytes, hipStream_t s) {
    if (bytes % 4) tbgpu_fatal("dcopy", "not whole words", __FILE__, __LINE__);
    const u64 n = bytes / 4;
    if (n == 0) return;
    k_copy_words<<<(u32)std::min<u64>((n + 255) / 256, 4096), 256, 0, s>>>((u32*)dst, (const u32*)src, n);
    HIP_CHECK(hipGetLastError());
}

// Host memory (page-locked, mapped) into device memory by a kernel: the kernel's loads
// cross PCIe uncached and its stores go through the L2s like every other kernel's, so
// later kernels see them.  (A copy engine writes HBM behind the L2s: kernels that had
// read the buffer before could go on reading their L2's old lines -- DESIGN.md §5.)
__global__ void k_copy_in(u8* __restrict__ dst, const u8* __restrict__ src, u64 n) {
    const u64 stride = (u64)gridDim.x * blockDim.x;
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
        const u64 n16 = n / 16;
        for (u64 k = t; k < n16; k += stride) ((uint4*)dst)[k] = ((const uint4*)src)[k];
        for (u64 k = n16 * 16 + t; k < n; k += stride) dst[k] = src[k];
    } else {
        for (u64 k = t; k < n; k += stride) dst[k] = src[k];
    }
}
static void copy_in(void* dst, const void* src_dev, u64 bytes, hipStream_t s) {
    const u64 items = std::max<u64>(bytes / 16, 1);
    const u32 blocks = (u32)std::min<u64>((items + 255) / 256, 1024);
    k_copy_in<<<blocks, 256, 0, s>>>((u8*)dst, (const u8*)src_dev, bytes);
    HIP_CHECK(hipGetLastError());
}

static bool sdma_h2d() {  // TBGPU_SDMA_H2D=1: uploads by the copy engine (A/B diagnostics)
    static const bool b = getenv("TBGPU_SDMA_H2D") != nullptr;
    return b;
}

static tbgpu_ctx::UpRing& up_ring(tbgpu_ctx* c, hipStream_t s) {
    tbgpu_ctx::UpRing& R = c->up[s == c->route_stream ? 1 : 0];
    if (R.h[0]) return R;
    for (int h = 0; h < 2; h++) {
        HIP_CHECK(hipHostMalloc((void**)&R.h[h], UP_HALF, hipHostMallocMapped | hipHostMallocCoherent));
        void* d = nullptr;
        HIP_CHECK(hipHostGetDevicePointer(&d, R.h[h], 0));
        R.d[h] = (const u8*)d;
        poison_host(R.h[h], UP_HALF);
        HIP_CHECK(hipEventCreateWithFlags(&R.ev[h], hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(R.ev[h], s));
    }
    return R;
}

static void h2d(tbgpu_ctx* c, void* dst, const void* src, u64 bytes, hipStream_t s) {
    if (bytes == 0) return;
    if (c->opt.flags & TBGPU_OPT_PINNED_INPUT) {
        if (const void* dev = pinned_device_ptr(src, bytes)) {
            if (sdma_h2d()) HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
            else copy_in(dst, dev, bytes, s);
            return;
        }
    }
    tbgpu_ctx::UpRing& R = up_ring(c, s);
    for (u64 off = 0; off < bytes;) {
        const u64 k = std::min<u64>(bytes - off, UP_HALF);
        const int h = R.next;
        R.next ^= 1;
        HIP_CHECK(hipEventSynchronize(R.ev[h]));  // the half's previous copy has read it
        memcpy(R.h[h], (const u8*)src + off, k);
        if (sdma_h2d()) HIP_CHECK(hipMemcpyAsync((u8*)dst + off, R.h[h], k, hipMemcpyHostToDevice, s));
        else copy_in((u8*)dst + off, R.d[h], k, s);
        HIP_CHECK(hipEventRecord(R.ev[h], s));
        off += k;
    }
}

// Device-to-host copy into caller memory, in stream order on `s`, complete on return:
// a DMA into the ctx's page-locked ring, then a host memcpy per UP_HALF bytes.  Copies
// into pageable memory are never handed to the runtime.
static void d2h(tbgpu_ctx* c, void* dst, const void* src, u64 bytes, hipStream_t s) {
    if (bytes == 0) return;
    tbgpu_ctx::UpRing& R = up_ring(c, s);
    // the copy into one half runs while the host copies the other half out
    int pend = -1;
    u64 pend_off = 0, pend_k = 0;
    for (u64 off = 0; off < bytes || pend >= 0;) {
        int h = -1;
        u64 k = 0;
        if (off < bytes) {
            k = std::min<u64>(bytes - off, UP_HALF);
            h = R.next;
            R.next ^= 1;
            HIP_CHECK(hipEventSynchronize(R.ev[h]));  // (its previous contents were copied out)
            HIP_CHECK(hipMemcpyAsync(R.h[h], (const u8*)src + off, k, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipEventRecord(R.ev[h], s));
        }
        if (pend >= 0) {
            HIP_CHECK(hipEventSynchronize(R.ev[pend]));
            memcpy((u8*)dst + pend_off, R.h[pend], pend_k);
        }
        pend = h;
        pend_off = off;
        pend_k = k;
        off += k;
    }
}

static bool spec_disabled() {
    static const bool d = getenv("TBGPU_NO_SPEC") != nullptr;
    return d;
}

// After the wait that follows a speculative fast attempt: true when it stood; false
// when it fell back, with its effects undone (the caller redoes the call).
static bool spec_settle(tbgpu_ctx* c) {
    if (!c->spec_pending) return true;
    c->spec_pending = false;
    const u32 flags = c->h_counters[CNT_FLAGS];
    if (!c->spec_F.dry) c->ids_nonmono = (flags & FL_NONMONO) != 0;
    if (flags & FL_ERROR) tbgpu_fatal("create_transfers", "fast path look-back did not complete", __FILE__, __LINE__);
    if (!(flags & FL_SLOW)) {
        c->fast_misses = 0;
        return true;
    }
    fp_launch_undo(c->T, c->spec_F, c->stream);  // commit_timestamp back; the deltas
    c->slow_chunks = 1;                          // the redo goes to the fixed point
    c->fast_misses++;
    return false;
}

// Withdrawn eager claims leave tombstones in the transfer-id index (XIDX_TOMB), which no
// insert reuses.  Stored rows keep the load at or below 0.5; tombstones could fill the
// rest over a long life, and a probe needs an empty slot to end.  So every 1/8 of the
// slots' worth of eager-claim events the count is read (one round trip), and past 1/16
// of the slots the index is rebuilt from the stored rows outside the sorted run: the load
// stays below 0.5 + 1/16 + 1/8.  Never with a prepared commit queued (its gate would
// hold the stream): the entry points call it before they prepare one.
static void xidx_tombs_check(tbgpu_ctx* c) {
    const u64 slots = c->T.xidx_mask + 1;
    if (c->eager_events <= slots / 8) return;
    c->eager_events = 0;
    hipStream_t s = c->stream;
    u32 tombs = 0;
    d2h(c, &tombs, c->T.hcount + 2, sizeof(u32), s);
    if (tombs <= slots / 16) return;
    u64 rows = 0;
    d2h(c, &rows, c->T.base + BASE_ROWS, sizeof(u64), s);
    HIP_CHECK(hipMemsetAsync(c->T.xidx, 0, slots * sizeof(u64), s));
    HIP_CHECK(hipMemsetAsync(c->T.hcount + 2, 0, sizeof(u32), s));
    launch_rehash_xidx(c->T, rows, s);
    c->stats.index_rebuilds++;
}

static uint64_t transfers_batches(tbgpu_ctx* c, uint32_t nb_total, const uint64_t* timestamps, const uint32_t* counts,
                                  const Transfer* ev_src, bool src_device, tbgpu_create_transfers_result_t* results,
                                  bool dst_device, uint32_t* result_counts, const uint64_t* ev_ts_host = nullptr,
                                  const uint8_t* ctl_host = nullptr, bool routed_device = false) {
    HIP_CHECK(hipSetDevice(c->device));
    entry_flush(c->stream);
    xidx_tombs_check(c);
    c->stats_lazy = false;
    static const bool no_call_events = getenv("TBGPU_NO_CALL_EVENTS") != nullptr;  // experiment
    const bool call_events = !no_call_events || c->prof;
    if (call_events) HIP_CHECK(hipEventRecord(c->ev0, c->stream));
    ht_mark(c, 1);
    ensure_h_rc(c, nb_total);
    std::vector<u32> starts;
    u64 ev_off = 0, events = 0;
    u32 iters = 0;
    u64 sorts = 0;
    c->stats.sorts = 0;
    bool ended = false;   // the last chunk brought the call's end back (k_report)
    u32 small_until = 0;  // batches before this one go in general-path-sized chunks
    c->long_segments = false;
    for (u32 b0 = 0; b0 < nb_total;) {
        // After a call needed the fixed point, the next ones probably do too: small
        // chunks, and the fast attempt only every 8th (it undoes itself when it fails).
        // A dry run must stay one call (its chunks cannot see each other's effects).
        const bool small = !c->rt_dry && (b0 < small_until || c->slow_chunks > 0);
        const u32 b1 = chunk_end(c, counts, b0, nb_total, small ? general_chunk_batches() : ~0u);
        const u32 nb = b1 - b0;
        prof_mark(c, PH_UPLOAD);
        u32 n = 0;
        for (u32 b = b0; b < b1; b++) n += counts[b];
        const Transfer* ev;
        // A small one-chunk call from pinned (or registered) host memory, on its fast
        // attempt: the kernels read the events where they are, over PCIe (fp_commit
        // reads each once): no copy and no DMA / compute hand-off.  A fallback redoes the
        // call with a copy (slow_chunks).
        const bool zc = !src_device && (c->opt.flags & TBGPU_OPT_PINNED_INPUT) && b0 == 0 && b1 == nb_total &&
                        n <= FP_TAIL_MAX && fast_due(c) &&
                        !c->rt_dry && !ev_ts_host && !ctl_host && !(c->opt.flags & TBGPU_OPT_FORCE_GENERAL) &&
                        !spec_disabled() && !zero_copy_disabled();
        const Transfer* ev_zc = zc ? (const Transfer*)pinned_device_ptr(ev_src + ev_off, (u64)n * 128) : nullptr;
        if (src_device) {
            ev = ev_src + ev_off;
        } else if (ev_zc) {
            ev = ev_zc;
            c->ev_in_host = true;
        } else {
            // the events' copy (a DMA engine) first, then the small uploads and resets on
            // the compute queue: one engine hand-off before the chunk's kernels, not two.
            // A pageable source is staged through the ctx's page-locked ring (h2d); the
            // drain first: the previous chunk's kernels (and a fallen-back attempt's undo)
            // have read ev_buf before it is rewritten.
            wait_stream(c->stream);
            h2d(c, c->ev_buf, ev_src + ev_off, (u64)n * 128, c->stream);
            ev = (const Transfer*)c->ev_buf;
        }
        // the replies start at the front of `results` (device results: the call's first
        // chunk; host results: every chunk, staged in res_buf)
        upload_batches(c, timestamps + b0, counts + b0, nb, starts, ev_off == 0 || !dst_device, /*allow_inline=*/true);
        ht_mark(c, 2);
        c->rt_ev_ts = nullptr;
        c->rt_ctl = nullptr;
        if (routed_device) {  // already in HBM
            c->rt_ev_ts = ev_ts_host ? ev_ts_host + ev_off : nullptr;
            c->rt_ctl = ctl_host ? ctl_host + ev_off : nullptr;
        } else {
            if (ev_ts_host) {
                h2d(c, c->rt_ts_buf, ev_ts_host + ev_off, (u64)n * 8, c->stream);
                c->rt_ev_ts = c->rt_ts_buf;
            }
            if (ctl_host) {
                h2d(c, c->rt_ctl_buf, ctl_host + ev_off, n, c->stream);
                c->rt_ctl = c->rt_ctl_buf;
            }
        }
        // device results: the call's buffer (cursor-relative); host results: staged in
        // res_buf one chunk at a time
        tbgpu_create_transfers_result_t* rdev = dst_device ? results : (tbgpu_create_transfers_result_t*)c->res_buf;
        const bool try_fast_path = fast_due(c);
        // a call that is one chunk makes its fast attempt without the round trip that
        // decides whether it stands: that answer comes with the call's final wait
        const bool spec = try_fast_path && !c->rt_dry && b0 == 0 && b1 == nb_total &&
                          !(c->opt.flags & TBGPU_OPT_FORCE_GENERAL) && !spec_disabled();
        c->tail_rp = TailReport{};
        c->tail_reported = false;
        if (b1 == nb_total)
            c->tail_rp = TailReport{c->h_report_dev, nb, (const u64*)c->res_buf, dst_device ? nullptr : c->h_res_dev,
                                    c->h_report_dev + RPT_COUNTS + c->bmax, next_seq(c)};
        const bool stood = run_transfers_chunk(c, ev, n, nb, rdev, try_fast_path,
                                               /*split=*/!c->rt_dry && nb > general_chunk_batches(), spec);
        c->ev_in_host = false;
        if (!stood) {
            small_until = b1;  // redo these batches in small chunks, on the general path
            c->slow_chunks = 1;
            continue;
        }
        if (b1 == nb_total) {
            // the call's end: counters, cursors and reply counts in one copy, with the
            // replies, and one wait
            const bool tail_done = c->tail_reported;  // fp_tail stored the report already: a small call
            c->tail_reported = false;
            if (!tail_done) {
                const u32 rb = std::max<u32>((RPT_COUNTS + nb + 255) / 256,
                                             dst_device ? 1u : std::min<u32>(n / 256, 1024));
                k_report<<<rb, 256, 0, c->stream>>>(c->counters, c->T.base, c->counts, nb, c->h_report_dev,
                                                    (const u64*)c->res_buf, dst_device ? nullptr : c->h_res_dev);
                HIP_CHECK(hipGetLastError());
            }
            if (call_events || !tail_done) HIP_CHECK(hipEventRecord(c->ev1, c->stream));
            ht_mark(c, 5);
            if (tail_done && !c->prof) {
                // a small call: fp_tail's last store is its sequence word in pinned host
                // memory, after everything it reported; spin on it (no completion signal,
                // no wake-up), and only past a bound wait for the launch as any other call
                const volatile u32* seqw = c->h_report + RPT_COUNTS + c->bmax;
                const u32 want = c->tail_rp.seq;
                for (u32 k = 0;; k++) {
                    if (__atomic_load_n(seqw, __ATOMIC_ACQUIRE) == want) break;
                    // now and then: has the launch ended (or failed) without the word?
                    if ((k & 1023) == 1023 && (call_events ? hipEventQuery(c->ev1) : hipStreamQuery(c->stream)) !=
                                                  hipErrorNotReady) {
                        if (call_events) wait_event(c->ev1); else wait_stream(c->stream);  // (reports a failure)
                        break;
                    }
                }
                c->stats_lazy = call_events;
            } else {
                wait_event(c->ev1);
            }
            ht_mark(c, 6);
            memcpy(c->h_counters, c->h_report, CNT_COUNT * sizeof(u32));
            memcpy(c->h_base, c->h_report + RPT_BASE, 4 * sizeof(u64));
            memcpy(c->h_rc + b0, c->h_report + RPT_COUNTS, nb * sizeof(u32));
            if (c->h_counters[CNT_STICKY])  // an apply kernel's error in any chunk of the call
                tbgpu_fatal("create_transfers", (c->h_counters[CNT_STICKY] & FL_FOREIGN) ?
                            "a transfer of a ledger another shard owns (ledger shard ctx)" :
                            "device error in the apply kernels (table capacity)", __FILE__, __LINE__);
            if (!spec_settle(c))  // the speculative fast attempt fell back: redo the call
                return transfers_batches(c, nb_total, timestamps, counts, ev_src, src_device, results, dst_device,
                                         result_counts, ev_ts_host, ctl_host, routed_device);
            if (!dst_device) copy_results_to_batches(c, nb, starts, c->h_rc + b0, (u8*)(results + ev_off));
            ended = true;
        } else {
            HIP_CHECK(hipMemcpyAsync(c->h_rc + b0, c->counts, nb * sizeof(u32), hipMemcpyDeviceToHost, c->stream));
            if (!dst_device) {
                // the chunk's replies (at most one per event) come back with its counts: one
                // round trip (no speculative attempt here: that is a one-chunk call)
                HIP_CHECK(hipMemcpyAsync(c->h_res, c->res_buf, (u64)n * 8, hipMemcpyDeviceToHost, c->stream));
                wait_stream(c->stream);
                copy_results_to_batches(c, nb, starts, c->h_rc + b0, (u8*)(results + ev_off));
            }
        }
        iters = std::max(iters, c->stats.iterations);
        sorts += c->stats.sorts;
        c->stats.sorts = 0;
        ev_off += n;
        events += n;
        b0 = b1;
    }
    if (!ended) {  // no batches
        HIP_CHECK(hipMemcpyAsync(c->h_base, c->T.base, 4 * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(hipEventRecord(c->ev1, c->stream));
        wait_event(c->ev1);
    }
    if (!spec_settle(c))  // the speculative fast attempt fell back: redo the call
        return transfers_batches(c, nb_total, timestamps, counts, ev_src, src_device, results, dst_device,
                                 result_counts, ev_ts_host, ctl_host, routed_device);
    float ms = 0;
    if (!c->stats_lazy && call_events) HIP_CHECK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->n_rows = c->h_base[BASE_ROWS];
    c->n_hist = c->h_base[BASE_HIST];
    c->rows_hi = c->n_rows;
    u64 total = 0;
    for (u32 b = 0; b < nb_total; b++) total += c->h_rc[b];
    memcpy(result_counts, c->h_rc, nb_total * sizeof(u32));
    prof_collect(c);
    c->stats.events = events;
    c->stats.iterations = iters;
    c->stats.sorts = sorts;
    c->stats.device_ms = ms;
    return total;
}

static uint64_t routed(tbgpu_ctx* c, uint32_t batch_count, const uint32_t* counts, const void* events,
                       const uint64_t* event_timestamps, const uint8_t* ctl, int dry_run, void* results,
                       uint32_t* result_counts, uint64_t* commit_timestamp, bool device);

extern "C" uint64_t tbgpu_create_transfers_routed(tbgpu_ctx* c, uint32_t batch_count, const uint32_t* counts,
                                                  const tbgpu_transfer_t* events, const uint64_t* event_timestamps,
                                                  const uint8_t* ctl, int dry_run,
                                                  tbgpu_create_transfers_result_t* results, uint32_t* result_counts,
                                                  uint64_t* commit_timestamp) {
    return routed(c, batch_count, counts, events, event_timestamps, ctl, dry_run, results, result_counts,
                  commit_timestamp, false);
}

extern "C" uint64_t tbgpu_create_transfers_routed_device(tbgpu_ctx* c, uint32_t batch_count, const uint32_t* counts,
                                                         const void* events_device,
                                                         const void* event_timestamps_device, const void* ctl_device,
                                                         int dry_run, void* results_device, uint32_t* result_counts,
                                                         uint64_t* commit_timestamp) {
    return routed(c, batch_count, counts, events_device, (const uint64_t*)event_timestamps_device,
                  (const uint8_t*)ctl_device, dry_run, results_device, result_counts, commit_timestamp, true);
}

static uint64_t routed(tbgpu_ctx* c, uint32_t batch_count, const uint32_t* counts, const void* events,
                       const uint64_t* event_timestamps, const uint8_t* ctl, int dry_run, void* results,
                       uint32_t* result_counts, uint64_t* commit_timestamp, bool device) {
    CallGuard guard_(c, false);
    c->pf_valid = false;  // any other create call discards a prefetched batch
    u64 n = 0;
    for (u32 b = 0; b < batch_count; b++) n += counts[b];
    if (dry_run && (n > c->nmax || batch_count > c->bmax - 2))
        tbgpu_fatal("create_transfers_routed", "a dry run must fit one call (events_per_call_max)", __FILE__, __LINE__);
    // the batch timestamps are unused: every event carries its own
    std::vector<u64> bts(batch_count, 0);
    c->rt_dry = dry_run != 0;
    if (c->rt_dry) {
        dcopy(c->rt_dry_ts, c->T.commit_ts, sizeof(u64), c->stream);
    }
    const u64 total = transfers_batches(c, batch_count, bts.data(), counts, (const Transfer*)events, device,
                                        (tbgpu_create_transfers_result_t*)results, device, result_counts,
                                        event_timestamps, ctl, device);
    c->rt_ev_ts = nullptr;
    c->rt_ctl = nullptr;
    u64 ts = 0;
    d2h(c, &ts, c->rt_dry ? c->rt_dry_ts : c->T.commit_ts, sizeof(u64), c->stream);
    c->rt_dry = false;
    if (commit_timestamp) *commit_timestamp = ts;
    return total;
}

extern "C" int tbgpu_import_transfers(tbgpu_ctx* c, const tbgpu_transfer_t* rows, uint32_t count) {
    CallGuard guard_(c, false);
    c->pf_valid = false;
    if (count == 0) return 0;
    // rows already held (committed here or imported before) are skipped: rows are
    // immutable, and the id index must hold each id once
    std::vector<tbgpu_uint128_t> ids(count);
    for (u32 i = 0; i < count; i++) ids[i] = rows[i].id;
    std::vector<tbgpu_transfer_t> found(count);
    const u32 held = tbgpu_lookup_transfers(c, ids.data(), count, found.data());
    std::vector<tbgpu_transfer_t> keep;
    keep.reserve(count);
    for (u32 i = 0, f = 0; i < count; i++) {
        if (f < held && found[f].id.lo == rows[i].id.lo && found[f].id.hi == rows[i].id.hi) { f++; continue; }
        bool dup = false;  // a repeated id within this call
        for (const tbgpu_transfer_t& k : keep) dup |= k.id.lo == rows[i].id.lo && k.id.hi == rows[i].id.hi;
        if (!dup) keep.push_back(rows[i]);
    }
    const u64 n = keep.size();
    refresh_bases(c);
    if (c->n_rows + n > c->xrow_cap) tbgpu_fatal("import_transfers", "transfers_max exceeded", __FILE__, __LINE__);
    u64 off = 0;
    while (off < n) {
        const u32 k = (u32)std::min<u64>(n - off, c->nmax);
        h2d(c, c->ev_buf, keep.data() + off, (u64)k * 128, c->stream);
        launch_import_transfers(c->T, (const Transfer*)c->ev_buf, k, c->n_rows, c->stream);
        if (!c->ximp) {
            ZeroOn zero_on(c->stream);
            c->ximp = dalloc<u8>(c->xrow_cap, &c->bytes);
            HIP_CHECK(hipMemsetAsync(c->ximp, 0, c->xrow_cap, c->stream));
        }
        HIP_CHECK(hipMemsetAsync(c->ximp + c->n_rows, 1, k, c->stream));  // not this shard's: never queried
        wait_stream(c->stream);
        c->n_rows += k;
        off += k;
    }
    set_base(c, BASE_ROWS, c->n_rows);
    c->rows_hi = c->n_rows;
    return 0;
}

u64 route_block_count(u64 n);
void route_stats(const Transfer* ev, u64 n, u64* out, hipStream_t stream);

extern "C" int tbgpu_route_stats(tbgpu_ctx* c, const void* events_device, uint64_t count, uint64_t* out) {
    CallGuard guard_(c, true);
    route_stats((const Transfer*)events_device, count, c->rt_stats, c->route_stream);
    d2h(c, out, c->rt_stats, 5 * sizeof(u64), c->route_stream);
    wait_stream(c->route_stream);
    return 0;
}
void route_scatter(const Transfer* ev, u64 n, u32 world, u32 nb, const u32* b_start, u64 g0,
                   uint2* orank, u32* blk, u64* counts, Transfer* out_ev, u64* out_side, u32* bcount, u32* scount,
                   u32 pack_mask, u32* out_packed, u32* error, bool ranked, hipStream_t stream);
void route_unpack_rows(const u32* packed, u64 m, u32 mask, const u32* sub_off, const u32* sub_g, u32 nsub,
                       const u64* ts_base, u64 batches, Transfer* rows, u64* rec, u64* ts, u32* error,
                       hipStream_t stream);
void route_rank(const Transfer* ev, u64 n, u32 world, uint2* orank, u32* blk, u64* part, u64* stats,
                hipStream_t stream);
void route_unpack(const u64* rec, u64 n, const u64* ts_base, u64 batches, u64* ts, u32* error, hipStream_t stream);

void route_dir_owners(const Tables& T, const void* records, u64 n, u32 world, int64_t* owner, hipStream_t stream);
void route_dir_finish(const void* records, const int64_t* owner, u64 n, u32* claim, int64_t* first_p,
                      int64_t* first_h, u64 g, u32* slot, int64_t* out, hipStream_t stream);

static void route_capacity(tbgpu_ctx* c, u32 world, u32 batch_count, u64 n) {
    const u64 nblk = route_block_count(n);
    if (n > c->ro_cap || world * std::max<u64>(nblk, 1) > c->ro_bcap || batch_count + 1 > c->ro_cap + 2 ||
        (u64)world * batch_count > c->ro_bc_cap) {
        wait_stream(c->route_stream);
        for (void* p : {(void*)c->ro_orank, (void*)c->ro_blk, (void*)c->ro_bstart, (void*)c->ro_counts,
                        (void*)c->ro_bcount, (void*)c->ro_spart})
            if (p) { guard_release(p); HIP_CHECK(hipFree(p)); }
        c->ro_cap = std::max<u64>(std::max<u64>(n, batch_count + 1), c->ro_cap);
        u64 ro_bytes = 0;
        ZeroOn zero_on(c->route_stream);
        c->ro_spart = dalloc<u64>(5 * (route_block_count(c->ro_cap) + 1), &ro_bytes);
        c->ro_bcap = 256ull * std::max<u64>(route_block_count(c->ro_cap), 1);
        c->ro_orank = dalloc<uint2>(c->ro_cap, &ro_bytes);
        c->ro_blk = dalloc<u32>(c->ro_bcap, &ro_bytes);
        c->ro_bstart = dalloc<u32>(c->ro_cap + 3, &ro_bytes);
        c->ro_counts = dalloc<u64>(256, &ro_bytes);
        c->ro_bc_cap = std::max<u64>((u64)world * std::max<u32>(batch_count, 1), 256ull * 64);
        c->ro_bcount = dalloc<u32>(c->ro_bc_cap + 256, &ro_bytes);
        c->ro_ranked = {};
    }
}

extern "C" int tbgpu_route_prepare(tbgpu_ctx* c, uint32_t world, const void* events_device, uint64_t count,
                                   uint64_t* out) {
    CallGuard guard_(c, true);
    entry_flush(c->route_stream);
    if (world == 0 || world > 256) return -22;
    route_capacity(c, world, 0, count);
    route_rank((const Transfer*)events_device, count, world, c->ro_orank, c->ro_blk, c->ro_spart, c->rt_stats,
               c->route_stream);
    d2h(c, out, c->rt_stats, 5 * sizeof(u64), c->route_stream);
    wait_stream(c->route_stream);
    c->ro_ranked = {events_device, count, world};
    return 0;
}

static int route_scatter_any(tbgpu_ctx* c, uint32_t world, uint32_t batch_count, const uint32_t* counts,
                             uint64_t first_global_batch, const void* events_device, void* send_events_device,
                             void* send_records_device, uint32_t word_mask, void* send_packed_device,
                             uint64_t* send_counts, uint32_t* send_batch_counts, uint32_t* send_span_counts) {
    CallGuard guard_(c, true);  // the router's send side (may overlap a commit on another thread)
    entry_flush(c->route_stream);
    if (world == 0 || world > 256) return -22;
    std::vector<u32> starts(batch_count + 1, 0);
    for (u32 b = 0; b < batch_count; b++) {
        if (counts[b] > TBGPU_ROUTE_REC_POS + 1) return -22;  // an index must fit its record field
        starts[b + 1] = starts[b] + counts[b];
    }
    const u64 n = starts[batch_count];
    route_capacity(c, world, batch_count, n);
    // tbgpu_route_prepare ranked these very events for this world: skip that pass
    const bool ranked = c->ro_ranked.events == events_device && c->ro_ranked.n == n && c->ro_ranked.world == world;
    c->ro_ranked = {};
    if (n == 0) {
        for (u32 o = 0; o < world; o++) send_counts[o] = 0;
        if (send_batch_counts) memset(send_batch_counts, 0, (u64)world * batch_count * sizeof(u32));
        if (send_span_counts) memset(send_span_counts, 0, world * sizeof(u32));
        return 0;
    }
    u32* err = (u32*)(c->rt_stats + 7);
    HIP_CHECK(hipMemsetAsync(err, 0, sizeof(u32), c->route_stream));
    h2d(c, c->ro_bstart, starts.data(), (batch_count + 1) * sizeof(u32), c->route_stream);
    route_scatter((const Transfer*)events_device, n, world, batch_count, c->ro_bstart, first_global_batch,
                  c->ro_orank, c->ro_blk, c->ro_counts, (Transfer*)send_events_device, (u64*)send_records_device,
                  c->ro_bcount + 256, c->ro_bcount, word_mask, (u32*)send_packed_device, err, ranked, c->route_stream);
    d2h(c, send_counts, c->ro_counts, world * sizeof(u64), c->route_stream);
    if (send_batch_counts)
        d2h(c, send_batch_counts, c->ro_bcount + 256, (u64)world * batch_count * sizeof(u32), c->route_stream);
    if (send_span_counts)
        d2h(c, send_span_counts, c->ro_bcount, world * sizeof(u32), c->route_stream);
    u32 e = 0;
    d2h(c, &e, err, sizeof(u32), c->route_stream);
    wait_stream(c->route_stream);
    return e ? -22 : 0;
}

extern "C" int tbgpu_route_scatter(tbgpu_ctx* c, uint32_t world, uint32_t batch_count, const uint32_t* counts,
                                   const uint64_t* batch_timestamps, uint64_t first_global_batch,
                                   const void* events_device, void* send_events_device, void* send_records_device,
                                   uint64_t* send_counts, uint32_t* send_batch_counts, uint32_t* send_span_counts) {
    (void)batch_timestamps;  // the owner derives the timestamps (tbgpu_route_unpack)
    return route_scatter_any(c, world, batch_count, counts, first_global_batch, events_device, send_events_device,
                             send_records_device, 0, nullptr, send_counts, send_batch_counts, send_span_counts);
}

extern "C" int tbgpu_route_scatter_packed(tbgpu_ctx* c, uint32_t world, uint32_t batch_count, const uint32_t* counts,
                                          uint64_t first_global_batch, const void* events_device, uint32_t word_mask,
                                          void* send_device, uint64_t* send_counts, uint32_t* send_batch_counts,
                                          uint32_t* send_span_counts) {
    if (word_mask == 0) return -22;
    return route_scatter_any(c, world, batch_count, counts, first_global_batch, events_device, nullptr, nullptr,
                             word_mask, send_device, send_counts, send_batch_counts, send_span_counts);
}

extern "C" int tbgpu_route_unpack_packed(tbgpu_ctx* c, const void* packed_device, uint64_t count, uint32_t word_mask,
                                         uint32_t sub_batch_count, const void* sub_offsets_device,
                                         const void* sub_batches_device, const void* batch_ts_base_device,
                                         uint64_t batches, void* events_device, void* records_device,
                                         void* timestamps_device) {
    CallGuard guard_(c, true);
    if (word_mask == 0 || (count && sub_batch_count == 0)) return -22;
    u32* err = (u32*)(c->rt_stats + 6);
    HIP_CHECK(hipMemsetAsync(err, 0, sizeof(u32), c->route_stream));
    route_unpack_rows((const u32*)packed_device, count, word_mask, (const u32*)sub_offsets_device,
                      (const u32*)sub_batches_device, sub_batch_count, (const u64*)batch_ts_base_device, batches,
                      (Transfer*)events_device, (u64*)records_device, (u64*)timestamps_device, err, c->route_stream);
    u32 e = 0;
    d2h(c, &e, err, sizeof(u32), c->route_stream);
    wait_stream(c->route_stream);
    return e ? -22 : 0;
}

extern "C" int tbgpu_route_unpack(tbgpu_ctx* c, const void* records_device, uint64_t count,
                                  const void* batch_ts_base_device, uint64_t batches, void* timestamps_device) {
    CallGuard guard_(c, true);
    u32* err = (u32*)(c->rt_stats + 6);
    HIP_CHECK(hipMemsetAsync(err, 0, sizeof(u32), c->route_stream));
    route_unpack((const u64*)records_device, count, (const u64*)batch_ts_base_device, batches, (u64*)timestamps_device,
                 err, c->route_stream);
    u32 e = 0;
    d2h(c, &e, err, sizeof(u32), c->route_stream);
    wait_stream(c->route_stream);
    return e ? -22 : 0;
}

extern "C" int tbgpu_route_directory_owners(tbgpu_ctx* c, uint32_t world, const void* records_device, uint64_t count,
                                            void* owners_device) {
    CallGuard guard_(c, false);
    if (world == 0) return -22;
    route_dir_owners(c->T, records_device, count, world, (int64_t*)owners_device, c->stream);
    wait_stream(c->stream);
    return 0;
}

extern "C" int tbgpu_route_directory(tbgpu_ctx* c, const void* records_device, const void* owners_device,
                                     uint64_t count, void* out_device) {
    CallGuard guard_(c, false);
    if (count >= 0xFFFFFFFFull) return -22;
    const u64 g = pow2_at_least(2 * std::max<u64>(count, 8));
    if (g > c->rd_cap) {
        wait_stream(c->stream);
        for (void* p : {(void*)c->rd_claim, (void*)c->rd_first, (void*)c->rd_slot})
            if (p) { guard_release(p); HIP_CHECK(hipFree(p)); }
        u64 b = 0;
        ZeroOn zero_on(c->stream);
        c->rd_cap = g;
        c->rd_claim = dalloc<u32>(g, &b);
        c->rd_first = dalloc<int64_t>(2 * g, &b);
        c->rd_slot = dalloc<u32>(g / 2, &b);
    }
    route_dir_finish(records_device, (const int64_t*)owners_device, count, c->rd_claim, c->rd_first, c->rd_first + g,
                     g, c->rd_slot, (int64_t*)out_device, c->stream);
    wait_stream(c->stream);
    return 0;
}

// max into the device scalar, ordered on the engine's stream (no host round trip)
__global__ void k_advance_commit_ts(u64* ts, u64 v) {
    if (threadIdx.x == 0 && *ts < v) *ts = v;
}

extern "C" void tbgpu_advance_commit_timestamp(tbgpu_ctx* c, uint64_t timestamp) {
    CallGuard guard_(c, false);
    k_advance_commit_ts<<<1, 64, 0, c->stream>>>(c->T.commit_ts, timestamp);
    HIP_CHECK(hipGetLastError());
}

extern "C" int tbgpu_copy_to_device(tbgpu_ctx* c, void* dst_device, const void* src_host, uint64_t bytes) {
    CallGuard guard_(c, false);
    h2d(c, dst_device, src_host, bytes, c->stream);
    wait_stream(c->stream);
    return 0;
}

// tbgpu_prefetch_transfers, when the commit that follows will be a one-batch fast call
// (fp_commit_small + fp_tail): everything but the timestamp is known, so both launches
// are enqueued now, and fp_commit_small classifies the batch against the pre-call state
// at once; its tiles then wait (fp_gate_wait) for the commit call, which only writes its
// timestamp and sequence number into pinned memory: no launch, and only the state
// changes and the call's end, on its critical path.  Any other call releases the gate
// (gate_cancel), and tiles that wait past the budget change nothing; the commit then
// runs as an ordinary prefetched call.
static bool prepare_ok(const tbgpu_ctx* c, u32 n) {
    static const bool off = getenv("TBGPU_NO_GATE") != nullptr;  // A/B timing
    static const bool no_tail = getenv("TBGPU_NO_TAIL") != nullptr, no_small = getenv("TBGPU_NO_SMALL") != nullptr;
    return !(off || no_tail || no_small || n == 0 || n > FP_TAIL_MAX || c->prof || c->rt_dry ||
             (c->opt.flags & TBGPU_OPT_FORCE_GENERAL) || spec_disabled() || !fast_due(c));
}

// Enqueue a prepared commit of n events at `ev` (in HBM) with sequence number `seq`: the
// current commit's host state (spec_F, tail_rp, ...) is left describing it.
static void prepare_launch(tbgpu_ctx* c, const Transfer* ev, u32 n, u32 seq) {
    c->rt_ev_ts = nullptr;
    c->rt_ctl = nullptr;
    c->blk_words = 0;  // the gated tiles write the block
    c->b_ts = (u64*)(c->b_start + batch_ts_offset(1));
    c->gate_seq = seq;
    c->tail_rp = TailReport{c->h_report_dev, 1, (const u64*)c->res_buf, c->h_res_dev,
                            c->h_report_dev + RPT_COUNTS + c->bmax, seq};
    c->tail_reported = false;
    c->gate_arm = true;
    const bool launched = try_fast(c, ev, n, 1, (tbgpu_create_transfers_result_t*)c->res_buf, /*spec=*/true);
    c->gate_arm = false;
    if (!launched || !c->tail_reported)
        tbgpu_fatal("prefetch", "a prepared commit did not take the small fast launches", __FILE__, __LINE__);
    c->gate_last = seq;
}

static void prepare_gated(tbgpu_ctx* c, u32 n) {
    if (!prepare_ok(c, n) || c->rows_hi + n > c->xrow_cap) return;
    ensure_h_rc(c, 1);
    prepare_launch(c, (const Transfer*)c->pf_dev, n, next_seq(c));
    c->gate_pending = true;
    c->gate_n = n;
}

// tbgpu_stage_transfers: the staged body's commit prepared at once, behind the current
// and the queued ones (no host round trip: the engine stream may be held by a gate).
static void stage_prepare(tbgpu_ctx* c, int k, u32 n) {
    const u64 ahead = c->pq_events + (c->gate_pending ? c->gate_n : 0);
    if (!prepare_ok(c, n) || c->pq.size() + 2 > TBGPU_STAGE_SLOTS || c->h_rc_cap < 1 ||
        c->rows_hi + ahead + n > c->xrow_cap)
        return;
    auto& S = c->stg[k];
    // the current prepared commit's host state, kept
    const FastArgs sF = c->spec_F;
    const bool sP = c->spec_pending, sT = c->tail_reported;
    const TailReport sR = c->tail_rp;
    const u32 sG = c->gate_seq;
    const tbgpu_stats sS = c->stats;
    if (hipEventQuery(S.staged) != hipSuccess) HIP_CHECK(hipStreamWaitEvent(c->stream, S.staged, 0));
    const u32 seq = next_seq(c);
    prepare_launch(c, (const Transfer*)S.d, n, seq);
    c->pq.push_back(tbgpu_ctx::Prepared{seq, n, k, S.key_lo, S.key_hi, c->spec_F, c->tail_rp});
    c->pq_events += n;
    c->spec_F = sF;
    c->spec_pending = sP;
    c->tail_reported = sT;
    c->tail_rp = sR;
    c->gate_seq = sG;
    c->stats = sS;
}

// The commit of a prepared call: release the gate with the timestamp, then wait for
// fp_tail's sequence word (or the gate's note that it let nothing through).  Returns
// false when the call must run as an ordinary one (the gate let nothing through, or the
// fast attempt fell back: its effects are undone by spec_settle's fp_undo).
static bool commit_gated(tbgpu_ctx* c, u64 timestamp, tbgpu_create_transfers_result_t* results, u32* count_out) {
    c->gate_pending = false;
    const u32 seq = c->gate_seq, n = c->gate_n;
    memcpy(c->h_gate + GW_TS, &timestamp, sizeof timestamp);
    __atomic_store_n(&c->h_gate[GW_GO], seq, __ATOMIC_RELEASE);
    ht_mark(c, 4);
    const volatile u32* seqw = c->h_report + RPT_COUNTS + c->bmax;
    bool go = true;
    for (u32 k = 0;; k++) {
        if (__atomic_load_n(seqw, __ATOMIC_ACQUIRE) == seq) break;
        if (__atomic_load_n(&c->h_gate[GW_ACK], __ATOMIC_ACQUIRE) == seq) {
            go = false;
            break;
        }
        if ((k & 1023) == 1023 && hipStreamQuery(c->stream) != hipErrorNotReady) {
            wait_stream(c->stream);  // (reports a failure)
            go = __atomic_load_n(seqw, __ATOMIC_ACQUIRE) == seq;
            break;
        }
    }
    ht_mark(c, 6);
    c->tail_reported = false;
    if (!go) {
        c->spec_pending = false;
        gate_cancel(c);  // the queued commits classified against the state this one would have left
        return false;
    }
    memcpy(c->h_counters, c->h_report, CNT_COUNT * sizeof(u32));
    memcpy(c->h_base, c->h_report + RPT_BASE, 4 * sizeof(u64));
    memcpy(c->h_rc, c->h_report + RPT_COUNTS, sizeof(u32));
    if (c->h_counters[CNT_FLAGS] & (FL_SLOW | FL_ERROR)) gate_cancel(c);  // (before the undo waits behind them)
    if (!spec_settle(c)) return false;
    // the call's replies only (none when every event is ok): the count fp_tail reported
    const std::vector<u32> starts = {0u, n};
    copy_results_to_batches(c, 1, starts, c->h_rc, (u8*)results);
    c->n_rows = c->h_base[BASE_ROWS];
    c->n_hist = c->h_base[BASE_HIST];
    c->rows_hi = c->n_rows;
    c->slow_chunks = 0;
    c->stats.events = n;
    c->stats.iterations = 1;
    c->stats.sorts = 0;
    c->stats.path = 1;
    c->stats.device_ms = 0;  // (no call events around a prepared commit)
    c->stats_lazy = false;
    for (double& v : c->stats.phase_ms) v = 0;
    *count_out = c->h_rc[0];
    return true;
}

extern "C" int tbgpu_prefetch_transfers(tbgpu_ctx* c, const tbgpu_transfer_t* events, uint32_t count) {
    CallGuard guard_(c, false);  // (releases an earlier prepared commit)
    c->pf_valid = false;
    if (count > TBGPU_BATCH_MAX) return -22;
    xidx_tombs_check(c);
    // behind the previous commit on the ctx's stream (that commit has returned: its
    // kernels no longer read the slot); a DMA engine moves it while the caller goes on
    h2d(c, c->pf_buf, events, (u64)count * 128, c->stream);
    HIP_CHECK(hipEventRecord(c->pf_ev, c->stream));
    c->pf_src = events;
    c->pf_n = count;
    c->pf_dev = c->pf_buf;
    c->pf_slot = -1;
    c->pf_valid = true;
    prepare_gated(c, count);
    return 0;
}

// ---- staging at prepare (tbgpu_stage_transfers) --------------------------------------
//
// The replica hands every request body to StateMachine.prepare when it makes the prepare
// (src/vsr/replica.zig:5159-5167 -> src/state_machine.zig:503), before the journal write
// and the replication round trip; it prefetches and commits that op only once a quorum
// has it (src/vsr/replica.zig:3137-3152), back to back.  Staging the body's copy at
// prepare takes the copy out of that back-to-back sequence: prefetch then finds the
// body in HBM and only enqueues the prepared commit.

static void stage_init(tbgpu_ctx* c) {
    if (c->stage_stream) return;
    HIP_CHECK(hipSetDevice(c->device));
    HIP_CHECK(hipStreamCreateWithFlags(&c->stage_stream, hipStreamNonBlocking));
    for (auto& S : c->stg) {
        S.d = dalloc<u8>((u64)TBGPU_BATCH_MAX * 128, &c->bytes);
        HIP_CHECK(hipEventCreateWithFlags(&S.staged, hipEventDisableTiming));
    }
}

static int stage_find(tbgpu_ctx* c, tbgpu_uint128_t key, u32 n) {
    for (int k = 0; k < (int)TBGPU_STAGE_SLOTS; k++) {
        const auto& S = c->stg[k];
        if (S.valid && S.key_lo == key.lo && S.key_hi == key.hi && S.n == n) return k;
    }
    return -1;
}

extern "C" int tbgpu_stage_transfers(tbgpu_ctx* c, tbgpu_uint128_t key, const tbgpu_transfer_t* events,
                                     uint32_t count) {
    CallGuard guard_(c, false, /*keep_gate=*/true);  // (a prepared commit may be pending)
    if (count > TBGPU_BATCH_MAX) return -22;
    if (count == 0) return 0;
    stage_init(c);
    if (stage_find(c, key, count) >= 0) return 0;  // the same content is staged already
    // the slot: a free one, else the oldest a prefetch has taken, else the oldest; never
    // the one the pending prefetch reads or one a queued prepared commit will read
    int pick = -1;
    for (int round = 0; round < 2 && pick < 0; round++) {
        if (round == 1) gate_cancel(c);  // every slot is spoken for: the queued commits go
        for (int pass = 0; pass < 3 && pick < 0; pass++) {
            u64 best = ~0ull;
            for (int k = 0; k < (int)TBGPU_STAGE_SLOTS; k++) {
                const auto& S = c->stg[k];
                if (c->pf_valid && c->pf_slot == k) continue;
                bool queued = false;
                for (const auto& p : c->pq) queued |= p.slot == k;
                if (queued) continue;
                const bool fits = pass == 0 ? !S.valid : pass == 1 ? S.used : true;
                if (fits && S.seq < best) {
                    best = S.seq;
                    pick = k;
                }
            }
        }
    }
    if (pick < 0) tbgpu_fatal("stage", "no stage slot", __FILE__, __LINE__);
    auto& S = c->stg[pick];
    S.valid = false;
    // Nothing reads the slot any more: a slot is read only by the launches of a commit
    // of its body, which have read it when that commit returns (a prepared commit's
    // sequence word is the last store of its last launch that reads the events; an
    // ordinary call waits for its launches; a released gate lets them read nothing),
    // and the slot of the prefetch still pending was not picked.
    const u64 bytes = (u64)count * 128;
    const void* src = (c->opt.flags & TBGPU_OPT_PINNED_INPUT) ? pinned_device_ptr(events, bytes) : nullptr;
    if (!src) {
        // a pageable body: through the slot's page-locked shadow (its previous copy out of
        // the shadow has run: staged)
        if (!S.h) {
            HIP_CHECK(hipHostMalloc((void**)&S.h, (u64)TBGPU_BATCH_MAX * 128, hipHostMallocMapped | hipHostMallocCoherent));
            void* d = nullptr;
            HIP_CHECK(hipHostGetDevicePointer(&d, S.h, 0));
            S.h_dev = (const u8*)d;
        } else {
            HIP_CHECK(hipEventSynchronize(S.staged));
        }
        memcpy(S.h, events, bytes);
        src = S.h_dev;
    }
    if (sdma_h2d()) HIP_CHECK(hipMemcpyAsync(S.d, src == S.h_dev ? (const void*)S.h : (const void*)events, bytes,
                                             hipMemcpyHostToDevice, c->stage_stream));
    else copy_in(S.d, src, bytes, c->stage_stream);
    HIP_CHECK(hipEventRecord(S.staged, c->stage_stream));
    S.key_lo = key.lo;
    S.key_hi = key.hi;
    S.n = count;
    S.used = false;
    S.seq = ++c->stage_seq;
    S.valid = true;
    stage_prepare(c, pick, count);
    return 0;
}

extern "C" int tbgpu_prefetch_transfers_staged(tbgpu_ctx* c, tbgpu_uint128_t key, const tbgpu_transfer_t* events,
                                               uint32_t count) {
    CallGuard guard_(c, false, /*keep_gate=*/true);
    if (count > TBGPU_BATCH_MAX) return -22;
    if (!c->gate_pending && !c->pq.empty() && c->pq.front().key_lo == key.lo && c->pq.front().key_hi == key.hi &&
        c->pq.front().n == count) {
        // its commit was prepared when it was staged: it becomes the current one
        const tbgpu_ctx::Prepared p = c->pq.front();
        c->pq.pop_front();
        c->pq_events -= p.n;
        c->pf_src = events;
        c->pf_n = count;
        c->pf_dev = c->stg[p.slot].d;
        c->pf_slot = p.slot;
        c->pf_valid = true;
        c->stg[p.slot].used = true;
        c->gate_pending = true;
        c->gate_seq = p.seq;
        c->gate_n = p.n;
        c->spec_F = p.F;
        c->spec_pending = true;
        c->tail_rp = p.rp;
        c->tail_reported = true;
        return 0;
    }
    gate_cancel(c);  // (what is queued is not what commits next)
    const int k = c->stage_stream ? stage_find(c, key, count) : -1;
    if (k < 0) return tbgpu_prefetch_transfers(c, events, count);  // not staged: copy it now
    c->pf_valid = false;
    xidx_tombs_check(c);
    auto& S = c->stg[k];
    // the engine stream waits for the slot's copy only while it still runs (a finished
    // copy needs no cross-queue dependency)
    if (hipEventQuery(S.staged) != hipSuccess) HIP_CHECK(hipStreamWaitEvent(c->stream, S.staged, 0));
    c->pf_src = events;
    c->pf_n = count;
    c->pf_dev = S.d;
    c->pf_slot = k;
    c->pf_valid = true;
    S.used = true;
    prepare_gated(c, count);
    return 0;
}

extern "C" int tbgpu_prefetch_wait(tbgpu_ctx* c) {
    CallGuard guard_(c, false, /*keep_gate=*/true);
    if (c->pf_valid) {
        if (c->pf_slot >= 0) wait_event(c->stg[c->pf_slot].staged);
        else wait_event(c->pf_ev);
    }
    return 0;
}

extern "C" uint32_t tbgpu_create_transfers(tbgpu_ctx* c, uint64_t timestamp, const tbgpu_transfer_t* events,
                                           uint32_t count, tbgpu_create_transfers_result_t* results) {
    if (host_trace()) {
        c->ht_on = true;
        c->ht0 = std::chrono::steady_clock::now();
        c->ht_calls++;
    }
    CallGuard guard_(c, false, /*keep_gate=*/true);
    ht_mark(c, 0);
    uint32_t rc = 0;
    const uint64_t ts = timestamp;
    uint32_t out;
    const bool prepared = c->pf_valid && c->pf_src == (const void*)events && c->pf_n == count;
    if (prepared && c->gate_pending && c->gate_n == count) {
        c->pf_valid = false;
        if (commit_gated(c, timestamp, results, &out)) {
            ht_mark(c, 7);
            c->ht_on = false;
            return out;
        }
        // the gate let nothing through, or the attempt fell back: an ordinary call
        out = (uint32_t)transfers_batches(c, 1, &ts, &count, (const Transfer*)c->pf_dev, true, results, false, &rc);
        ht_mark(c, 7);
        c->ht_on = false;
        return out;
    }
    gate_cancel(c);
    if (prepared) {
        // prefetched: the events are in HBM already (the copy is ahead on the stream)
        c->pf_valid = false;
        out = (uint32_t)transfers_batches(c, 1, &ts, &count, (const Transfer*)c->pf_dev, true, results, false, &rc);
    } else {
        c->pf_valid = false;
        out = (uint32_t)transfers_batches(c, 1, &ts, &count, (const Transfer*)events, false, results, false, &rc);
    }
    ht_mark(c, 7);
    c->ht_on = false;
    return out;
}

extern "C" uint64_t tbgpu_create_transfers_batches(tbgpu_ctx* c, uint32_t batch_count, const uint64_t* timestamps,
                                                   const uint32_t* counts, const tbgpu_transfer_t* events,
                                                   tbgpu_create_transfers_result_t* results, uint32_t* result_counts) {
    CallGuard guard_(c, false);
    c->pf_valid = false;
    return transfers_batches(c, batch_count, timestamps, counts, (const Transfer*)events, false, results, false,
                             result_counts);
}

extern "C" uint64_t tbgpu_create_transfers_batches_device(tbgpu_ctx* c, uint32_t batch_count,
                                                          const uint64_t* timestamps, const uint32_t* counts,
                                                          const void* events_device, void* results_device,
                                                          uint32_t* result_counts) {
    CallGuard guard_(c, false);
    c->pf_valid = false;
    return transfers_batches(c, batch_count, timestamps, counts, (const Transfer*)events_device, true,
                             (tbgpu_create_transfers_result_t*)results_device, true, result_counts);
}

// ------------------------------------------------------- create_accounts --

static void run_accounts_chunk(tbgpu_ctx* c, const Account* ev, u32 n, u32 nb,
                               tbgpu_create_accounts_result_t* results_dev, u32* counts_host) {
    hipStream_t s = c->stream;
    if (n == 0) {
        c->blk_words = 0;  // (no kernel reads the batch block)
        std::fill(counts_host, counts_host + nb, 0u);
        return;
    }
    AcArgs C{};
    C.ev = ev; C.n = n; C.nb = nb; C.b_start = c->b_start; C.b_ts = c->b_ts;
    C.ts = c->ts; C.cs = c->cs; C.ce = c->ce; C.sres = c->sres; C.pre = c->pre_e;
    C.gslot = c->gslot; C.prev_id = c->prev_id; C.gclaim = c->gclaim; C.gcnt_id = c->gcnt_id;
    const u64 g = std::min<u64>(c->gcap, pow2_at_least(4ull * n));
    C.gmask = g - 1;
    C.counters = c->counters;
    C.ts_part = c->ac_part;
    C.counts_out = c->counts;
    C.ftab = c->f_gtab;  // (the fast path's claim table: all-zero between calls, >= 2n slots)
    C.fpos = c->f_gpos;
    C.fmask = std::min<u64>(c->f_gcap, pow2_at_least(2ull * n)) - 1;
    static const bool no_fast = getenv("TBGPU_NO_AC_FAST") != nullptr;  // A/B timing of the general path
    if (!no_fast && !(c->opt.flags & TBGPU_OPT_FORCE_GENERAL) && c->n_accounts + n <= c->accounts_max &&
        !c->T.shard_world) {
        // the clean call (accounts.hip ac_fast_*): one round trip decides whether it stood
        // (two launches: the batch block in their arguments when it is small, the flags
        // in words of their own that the last workgroup zeroes again, the outcome stored
        // to the host by that workgroup)
        volatile u32* flags_host = c->h_report + RPT_COUNTS + c->bmax + 1;
        *flags_host = FL_SLOW | FL_ERROR;  // (a kernel that never stored it reads as failed)
        C.fast_words = c->ac_fast_words;
        const bool ticket = ac_fast_index_grid(C) <= AC_TICKET_GRID_MAX;
        C.flags_out = ticket ? c->h_report_dev + RPT_COUNTS + c->bmax + 1 : nullptr;
        const BlockInline bi = take_block(c);
        ac_launch_fast(c->T, C, c->n_accounts, bi, s);
        if (!ticket) {  // (into ordinary page-locked memory: a copy into the coherent report took longer)
            HIP_CHECK(hipMemcpyAsync(c->h_counters, c->ac_fast_words, sizeof(u32), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipMemsetAsync(c->ac_fast_words, 0, 2 * sizeof(u32), s));
        }
        wait_stream(s);
        const u32 flags = ticket ? *flags_host : c->h_counters[0];
        if (flags & FL_ERROR) tbgpu_fatal("create_accounts", "the clean call reported no outcome", __FILE__, __LINE__);
        if (!(flags & FL_SLOW)) {
            if (flags & FL_CAPACITY)
                tbgpu_fatal("create_accounts", "account index full (hashed_max exceeded)", __FILE__, __LINE__);
            std::fill(counts_host, counts_host + nb, 0u);
            c->n_accounts += n;
            c->stats.iterations = 1;
            return;
        }
        // not clean: nothing visible changed (rows past n_accounts are free); the general path below
    }
    flush_block(c);  // (when the fast call did not take it)
    HIP_CHECK(hipMemsetAsync(c->counters, 0, CNT_COUNT * sizeof(u32), s));
    HIP_CHECK(hipMemsetAsync(c->gclaim, 0, g * sizeof(u32), s));
    HIP_CHECK(hipMemsetAsync(c->gcnt_id, 0, g * sizeof(u32), s));
    ac_launch_classify(c->T, C, s);
    EvalState* A = &c->st[0];
    EvalState* Bst = &c->st[1];
    HIP_CHECK(hipMemsetAsync(A->cfail, 0xFF, n * sizeof(u32), s));
    ac_launch_init(C, A->res, A->ok, A->cfail, s);
    // Without chains and repeated ids no event sees another (create_account depends on
    // earlier events only through the id and the chain, :1198-1237): one evaluation
    // against the committed accounts is the sequential result.  That case (the
    // benchmark's) is enqueued whole, its mask, ranks and apply gated on classify's
    // device flags, and the call's end comes back in one wait; otherwise the gated
    // launches were no-ops and the fixed point below runs from the initial state.
    u32* gate = c->counters + AC_GATE_WORD;
    HIP_CHECK(hipMemsetAsync(Bst->cfail, 0xFF, n * sizeof(u32), s));
    ac_launch_evaluate(c->T, C, A->res, A->ok, Bst->res, Bst->ok, Bst->cfail, s);
    ac_launch_gate(C, gate, s);
    ac_launch_mask(c->T, C, Bst->res, Bst->ok, Bst->cfail, c->fres, c->mask, s, gate);
    scan3_exclusive(c->mask, c->ranks, n, c->sc, s, gate);
    ac_launch_apply(c->T, C, Bst->ok, c->fres, c->ranks, c->n_accounts, c->accounts_max, results_dev, c->counts, s,
                    gate);
    uint4 tot;
    HIP_CHECK(hipMemcpyAsync(c->h_counters, c->counters, CNT_COUNT * sizeof(u32), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(c->h_base + 4, c->ranks + n, sizeof(uint4), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(c->h_counts, c->counts, nb * sizeof(u32), hipMemcpyDeviceToHost, s));
    wait_stream(s);
    memcpy(counts_host, c->h_counts, nb * sizeof(u32));
    memcpy(&tot, c->h_base + 4, sizeof tot);
    const u32 flags = c->h_counters[CNT_FLAGS];
    if (!(flags & (FL_CHAINS | FL_MULTI_ID))) {
        if (flags & FL_CAPACITY)
            tbgpu_fatal("create_accounts", "account capacity exceeded (accounts_max, or hashed_max for the account "
                        "index)", __FILE__, __LINE__);
        if (flags & FL_ERROR) tbgpu_fatal("create_accounts", "device error", __FILE__, __LINE__);
        c->stats.iterations = 1;
        c->n_accounts += tot.x;
        c->n_foreign += tot.z;
        return;
    }
    if (flags & FL_MULTI_ID)
        ac_launch_group_sort(C, (u32)g, log2u(g + 1), c->skey, c->sval, c->skey_s, c->sval_s, c->ss, s);
    u32 it = 0;
    for (;; it++) {
        if (it > n + 2) tbgpu_fatal("create_accounts", "fixed point did not converge", __FILE__, __LINE__);
        HIP_CHECK(hipMemsetAsync(c->counters + CNT_CHANGES, 0, sizeof(u32), s));
        HIP_CHECK(hipMemsetAsync(Bst->cfail, 0xFF, n * sizeof(u32), s));
        ac_launch_evaluate(c->T, C, A->res, A->ok, Bst->res, Bst->ok, Bst->cfail, s);
        read_counters(c);
        std::swap(A, Bst);
        if (c->h_counters[CNT_CHANGES] == 0) break;
    }
    c->stats.iterations = it + 1;
    ac_launch_mask(c->T, C, A->res, A->ok, A->cfail, c->fres, c->mask, s);
    scan3_exclusive(c->mask, c->ranks, n, c->sc, s);
    d2h(c, &tot, c->ranks + n, sizeof(uint4), s);
    wait_stream(s);
    if (c->n_accounts + tot.x > c->accounts_max) tbgpu_fatal("create_accounts", "accounts_max exceeded", __FILE__, __LINE__);
    ac_launch_apply(c->T, C, A->ok, c->fres, c->ranks, c->n_accounts, c->accounts_max, results_dev, c->counts, s);
    d2h(c, counts_host, c->counts, nb * sizeof(u32), s);
    read_counters(c);
    if (c->h_counters[CNT_FLAGS] & FL_CAPACITY)
        tbgpu_fatal("create_accounts", "account index full (hashed_max exceeded)", __FILE__, __LINE__);
    c->n_accounts += tot.x;
    c->n_foreign += tot.z;
}

static uint64_t accounts_batches(tbgpu_ctx* c, uint32_t nb_total, const uint64_t* timestamps, const uint32_t* counts,
                                 const Account* events, bool device, tbgpu_create_accounts_result_t* results,
                                 uint32_t* result_counts) {
    CallGuard guard_(c, false);
    c->pf_valid = false;  // any other create call discards a prefetched batch
    entry_flush(c->stream);
    c->stats_lazy = false;
    HIP_CHECK(hipEventRecord(c->ev0, c->stream));
    std::vector<u32> starts;
    u64 total = 0, ev_off = 0;
    for (u32 b0 = 0; b0 < nb_total;) {
        const u32 b1 = chunk_end(c, counts, b0, nb_total);
        const u32 nb = b1 - b0;
        upload_batches(c, timestamps + b0, counts + b0, nb, starts, false, /*allow_inline=*/true);
        const u32 n = starts[nb];
        const Account* ev = events + ev_off;
        if (!device) {
            h2d(c, c->ev_buf, ev, (u64)n * 128, c->stream);
            ev = (const Account*)c->ev_buf;
        }
        run_accounts_chunk(c, ev, n, nb, (tbgpu_create_accounts_result_t*)c->res_buf, result_counts + b0);
        u64 chunk_total = 0;
        for (u32 b = 0; b < nb; b++) chunk_total += result_counts[b0 + b];
        if (device) {  // replies concatenated in device memory, as for create_transfers
            if (chunk_total)
                dcopy(results + total, c->res_buf, chunk_total * 8, c->stream);
        } else {
            if (chunk_total) {
                HIP_CHECK(hipMemcpyAsync(c->h_res, c->res_buf, chunk_total * 8, hipMemcpyDeviceToHost, c->stream));
                wait_stream(c->stream);
            }
            copy_results_to_batches(c, nb, starts, result_counts + b0, (u8*)(results + ev_off));
        }
        total += chunk_total;
        ev_off += n;
        b0 = b1;
    }
    HIP_CHECK(hipEventRecord(c->ev1, c->stream));
    wait_event(c->ev1);
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->stats.events = ev_off;
    c->stats.device_ms = ms;  // the call's device time (host round trips between chunks included)
    return total;
}

extern "C" uint64_t tbgpu_create_accounts_batches(tbgpu_ctx* c, uint32_t nb_total, const uint64_t* timestamps,
                                                  const uint32_t* counts, const tbgpu_account_t* events,
                                                  tbgpu_create_accounts_result_t* results, uint32_t* result_counts) {
    return accounts_batches(c, nb_total, timestamps, counts, (const Account*)events, false, results, result_counts);
}

extern "C" uint64_t tbgpu_create_accounts_batches_device(tbgpu_ctx* c, uint32_t nb_total, const uint64_t* timestamps,
                                                         const uint32_t* counts, const void* events_device,
                                                         void* results_device, uint32_t* result_counts) {
    return accounts_batches(c, nb_total, timestamps, counts, (const Account*)events_device, true,
                            (tbgpu_create_accounts_result_t*)results_device, result_counts);
}

extern "C" uint32_t tbgpu_create_accounts(tbgpu_ctx* c, uint64_t timestamp, const tbgpu_account_t* events,
                                          uint32_t count, tbgpu_create_accounts_result_t* results) {
    uint32_t rc = 0;
    return (uint32_t)tbgpu_create_accounts_batches(c, 1, &timestamp, &count, events, results, &rc);
}

// ------------------------------------------------------------- lookups ----

template <typename Row, typename Launch>
static uint32_t lookup(tbgpu_ctx* c, const tbgpu_uint128_t* ids, uint32_t count, Row* out, Launch launch) {
    CallGuard guard_(c, false);
    entry_flush(c->stream);
    uint32_t found_total = 0;
    std::vector<Row> rows;
    std::vector<u8> found;
    const u32 step = (u32)std::min<u64>(c->nmax, 1u << 20);
    for (u32 off = 0; off < count; off += step) {
        const u32 k = std::min(step, count - off);
        u128* d_ids = (u128*)c->ev_buf;  // k * 16 <= nmax * 128
        Row* d_out = (Row*)c->bb;        // 2 * nmax * 64 bytes >= k * 128
        u8* d_found = c->fres;
        h2d(c, d_ids, ids + off, (u64)k * 16, c->stream);
        launch(d_ids, k, d_out, d_found);
        rows.resize(k);
        found.resize(k);
        // into pageable memory: blocking copies behind a drain of the ctx's stream (an
        // asynchronous copy into pageable memory returned stale rows)
        wait_stream(c->stream);
        d2h(c, rows.data(), d_out, (u64)k * sizeof(Row), c->stream);
        d2h(c, found.data(), d_found, k, c->stream);
        for (u32 i = 0; i < k; i++)
            if (found[i]) memcpy(&out[found_total++], &rows[i], sizeof(Row));
    }
    return found_total;
}

extern "C" uint32_t tbgpu_lookup_accounts(tbgpu_ctx* c, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_account_t* out) {
    return lookup(c, ids, count, (Account*)out, [&](const u128* d, u32 k, Account* o, u8* f) {
        launch_lookup_accounts(c->T, d, k, o, f, c->stream);
    });
}

extern "C" uint32_t tbgpu_lookup_transfers(tbgpu_ctx* c, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_transfer_t* out) {
    return lookup(c, ids, count, (Transfer*)out, [&](const u128* d, u32 k, Transfer* o, u8* f) {
        launch_lookup_transfers(c->T, d, k, o, f, c->stream);
    });
}

// ------------------------------------------- account-transfers index ------

// Stable re-sort of the index entries [e0, e1) by account row: rows already in
// order within an account stay in order (query.hip).
static void q_sort(tbgpu_ctx* c, u64 e0, u64 e1) {
    const u64 m = e1 - e0;
    radix_sort_pairs(c->q_key + e0, c->q_val + e0, c->q_tkey + e0, c->q_tval + e0, m, log2u(c->accounts_max + 1),
                     c->q_ss, c->stream);
    dcopy(c->q_key + e0, c->q_tkey + e0, m * 4, c->stream);
    dcopy(c->q_val + e0, c->q_tval + e0, m * 4, c->stream);
}

// TBGPU_CHECK_INDEX=1 (diagnostics): after every compaction, the whole index against
// its definition.  Entries are rebuilt from the stored rows into the sort's output
// buffers (free between compactions); then every run [2 runs[k], 2 runs[k+1]) must
// hold exactly the entries of its rows, ordered by (account row, transfer row << 1 |
// side), each with the key its row's account probe gives.
static void check_index(tbgpu_ctx* c) {
    const u64 rows = c->q_runs.back();
    if (rows == 0) return;
    q_launch_entries(c->T, 0, rows, c->ximp, (u32)c->accounts_max, c->q_tkey, c->q_tval, c->stream);
    std::vector<u32> want(2 * rows), key(2 * rows), val(2 * rows);
    d2h(c, want.data(), c->q_tkey, 2 * rows * 4, c->stream);
    d2h(c, key.data(), c->q_key, 2 * rows * 4, c->stream);
    d2h(c, val.data(), c->q_val, 2 * rows * 4, c->stream);
    wait_stream(c->stream);
    char why[200];
    for (size_t k = 0; k + 1 < c->q_runs.size(); k++) {
        const u64 e0 = 2 * c->q_runs[k], e1 = 2 * c->q_runs[k + 1];
        std::vector<u8> seen(e1 - e0, 0);
        for (u64 e = e0; e < e1; e++) {
            const u32 v = val[e];
            const bool order = e == e0 || key[e - 1] < key[e] || (key[e - 1] == key[e] && val[e - 1] < v);
            const bool inside = v >= e0 && v < e1;
            if (!order || !inside || seen[v - e0] || key[e] != want[v]) {
                snprintf(why, sizeof why, "index run %zu [%llu, %llu) entry %llu: key %u val %u (expected key %u, %s)",
                         k, (unsigned long long)e0, (unsigned long long)e1, (unsigned long long)e, key[e], v,
                         inside ? want[v] : ~0u, !order ? "out of order" : !inside ? "foreign" :
                         seen[v - e0] ? "repeated" : "wrong key");
                tbgpu_fatal("compact", why, __FILE__, __LINE__);
            }
            seen[v - e0] = 1;
        }
    }
}

extern "C" uint64_t tbgpu_compact(tbgpu_ctx* c) {
    CallGuard guard_(c, false);
    entry_flush(c->stream);
    const u64 r0 = c->q_runs.back(), r1 = c->n_rows;
    if (r1 == r0) return r1;
    if (!c->q_key) {
        u64& B = c->bytes;
        ZeroOn zero_on(c->stream);
        const u64 cap = 2 * c->xrow_cap;  // two entries per stored row
        c->q_key = dalloc<u32>(cap, &B);
        c->q_val = dalloc<u32>(cap, &B);
        c->q_tkey = dalloc<u32>(cap, &B);
        c->q_tval = dalloc<u32>(cap, &B);
        c->q_ss.keys_tmp = dalloc<u32>(cap, &B);
        c->q_ss.vals_tmp = dalloc<u32>(cap, &B);
        c->q_ss.hist = dalloc<u32>(radix_sort_hist_words(cap), &B);
        c->q_ss.capacity = cap;
        c->q_runs_dev = dalloc<u64>(Q_RUNS_MAX + 1, &B);
    }
    q_launch_entries(c->T, r0, r1 - r0, c->ximp, (u32)c->accounts_max, c->q_key + 2 * r0, c->q_val + 2 * r0,
                     c->stream);
    q_sort(c, 2 * r0, 2 * r1);
    c->q_runs.push_back(r1);
    // binary-counter merging: the newest run absorbs its predecessor while it is at
    // least half as large, so run sizes more than halve from one run to the next
    while (c->q_runs.size() >= 3) {
        const size_t k = c->q_runs.size() - 1;
        const u64 older = c->q_runs[k - 1] - c->q_runs[k - 2], newer = c->q_runs[k] - c->q_runs[k - 1];
        if (2 * newer < older) break;
        q_sort(c, 2 * c->q_runs[k - 2], 2 * c->q_runs[k]);
        c->q_runs.erase(c->q_runs.end() - 2);
    }
    if (c->q_runs.size() > Q_RUNS_MAX + 1) tbgpu_fatal("compact", "index runs exceed Q_RUNS_MAX", __FILE__, __LINE__);
    h2d(c, c->q_runs_dev, c->q_runs.data(), c->q_runs.size() * sizeof(u64), c->stream);
    wait_stream(c->stream);
    static const bool check = getenv("TBGPU_CHECK_INDEX") != nullptr;  // diagnostics (tests)
    if (check) check_index(c);
    return r1;
}

// `nq` filters in device memory; results at out + q * stride rows.
static u64 run_queries(tbgpu_ctx* c, const tbgpu_account_filter_t* filters, u32 nq, u32 stride, void* out, bool history,
                       uint32_t* counts_host) {
    tbgpu_compact(c);
    QIndex X{c->q_key, c->q_val, c->q_runs_dev, (u32)(c->q_runs.size() - 1)};
    u64 total = 0;
    const u32 step = (u32)c->bmax;  // c->counts holds bmax words
    for (u32 q0 = 0; q0 < nq; q0 += step) {
        const u32 k = std::min(step, nq - q0);
        QArgs A{filters + q0, k, stride, (u8*)out + (u64)q0 * stride * 128, c->counts, history ? 1u : 0u, c->n_hist};
        q_launch_scan(c->T, X, A, c->stream);
        d2h(c, counts_host + q0, c->counts, k * sizeof(u32), c->stream);
        wait_stream(c->stream);
        for (u32 j = 0; j < k; j++) total += counts_host[q0 + j];
    }
    return total;
}

static uint32_t query_host(tbgpu_ctx* c, const tbgpu_account_filter_t* filter, void* out, bool history) {
    HIP_CHECK(hipSetDevice(c->device));
    tbgpu_account_filter_t* fd = (tbgpu_account_filter_t*)c->res_buf;  // nmax * 8 B >= 64 B
    h2d(c, fd, filter, sizeof *filter, c->stream);
    uint32_t n = 0;
    run_queries(c, fd, 1, TBGPU_QUERY_MAX, c->ev_buf, history, &n);  // ev_buf: nmax * 128 B >= 8190 rows
    if (n) d2h(c, out, c->ev_buf, (u64)n * 128, c->stream);
    return n;
}

// ---------------------------------------------------------- index trees ----
// The grooves' field index trees (index.hip): a tree indexes the objects stored since
// its last scan into a new run, then merges runs as tbgpu_compact does.
static bool ix_field_ok(u32 kind, u32 field) {
    if (kind == TBGPU_INDEX_TRANSFERS) return field <= TBGPU_INDEX_AMOUNT;
    return field == TBGPU_INDEX_USER_DATA_128 || field == TBGPU_INDEX_USER_DATA_64 ||
           field == TBGPU_INDEX_USER_DATA_32 || field == TBGPU_INDEX_LEDGER || field == TBGPU_INDEX_CODE;
}

static bool ix_filter_ok(u32 kind, const tbgpu_index_filter_t& f) {
    return ix_field_ok(kind, f.field) && f.limit != 0 && (f.flags & ~(u32)TBGPU_INDEX_REVERSED) == 0 &&
           f.reserved == 0 && f.timestamp_min != ~0ull && f.timestamp_max != ~0ull &&
           (f.timestamp_max == 0 || f.timestamp_min <= f.timestamp_max);
}

static void ix_sort(tbgpu_ctx* c, tbgpu_ctx::FieldIx& x, u32 field, u64 e0, u64 e1) {
    const u64 m = e1 - e0;
    if (m < 2) return;
    radix_sort_pairs(x.key + e0, x.val + e0, c->ix_tkey, c->ix_tval, m, (int)std::min<u32>(ix_field_bits(field), 32),
                     c->ix_ss, c->stream);
    dcopy(x.key + e0, c->ix_tkey, m * 4, c->stream);
    dcopy(x.val + e0, c->ix_tval, m * 4, c->stream);
}

static tbgpu_ctx::FieldIx& ix_extend(tbgpu_ctx* c, u32 kind, u32 field) {
    tbgpu_ctx::FieldIx& x = c->ix[kind][field];
    if (kind == TBGPU_INDEX_TRANSFERS) refresh_bases(c);
    const u64 cap = kind == TBGPU_INDEX_TRANSFERS ? c->xrow_cap : c->accounts_max;
    const u64 r0 = x.runs.back(), r1 = kind == TBGPU_INDEX_TRANSFERS ? c->n_rows : c->n_accounts;
    if (!c->ix_tkey) {
        u64& B = c->bytes;
        ZeroOn zero_on(c->stream);
        const u64 sc = std::max<u64>(c->xrow_cap, c->accounts_max);
        c->ix_tkey = dalloc<u32>(sc, &B);
        c->ix_tval = dalloc<u32>(sc, &B);
        c->ix_ss.keys_tmp = dalloc<u32>(sc, &B);
        c->ix_ss.vals_tmp = dalloc<u32>(sc, &B);
        c->ix_ss.hist = dalloc<u32>(radix_sort_hist_words(sc), &B);
        c->ix_ss.capacity = sc;
    }
    if (!x.key) {
        u64& B = c->bytes;
        ZeroOn zero_on(c->stream);
        x.key = dalloc<u32>(cap, &B);
        x.val = dalloc<u32>(cap, &B);
        x.runs_dev = dalloc<u64>(Q_RUNS_MAX + 1, &B);
    }
    if (r1 == r0) return x;
    ix_launch_entries(c->T, kind, field, r0, r1 - r0, c->ximp, x.key + r0, x.val + r0, c->stream);
    ix_sort(c, x, field, r0, r1);
    x.runs.push_back(r1);
    while (x.runs.size() >= 3) {  // binary-counter merging (tbgpu_compact)
        const size_t k = x.runs.size() - 1;
        const u64 older = x.runs[k - 1] - x.runs[k - 2], newer = x.runs[k] - x.runs[k - 1];
        if (2 * newer < older) break;
        ix_sort(c, x, field, x.runs[k - 2], x.runs[k]);
        x.runs.erase(x.runs.end() - 2);
    }
    if (x.runs.size() > Q_RUNS_MAX + 1) tbgpu_fatal("scan", "index runs exceed Q_RUNS_MAX", __FILE__, __LINE__);
    h2d(c, x.runs_dev, x.runs.data(), x.runs.size() * sizeof(u64), c->stream);
    return x;
}

static uint32_t scan_objects(tbgpu_ctx* c, u32 kind, const tbgpu_index_filter_t* filter, void* out) {
    if (!ix_filter_ok(kind, *filter)) return 0;
    tbgpu_ctx::FieldIx& x = ix_extend(c, kind, filter->field);
    tbgpu_index_filter_t* fd = (tbgpu_index_filter_t*)c->res_buf;  // nmax * 8 B >= 48 B
    h2d(c, fd, filter, sizeof *filter, c->stream);
    IxArgs A{fd, kind, 1u, x.key, x.val, x.runs_dev, (u32)(x.runs.size() - 1), c->ev_buf, c->counts};
    ix_launch_scan(c->T, A, c->stream);
    uint32_t n = 0;
    d2h(c, &n, c->counts, sizeof n, c->stream);
    if (n) d2h(c, out, c->ev_buf, (u64)n * 128, c->stream);
    return n;
}

extern "C" uint32_t tbgpu_scan_transfers(tbgpu_ctx* c, const tbgpu_index_filter_t* filter, tbgpu_transfer_t* out) {
    CallGuard guard_(c, false);
    return scan_objects(c, TBGPU_INDEX_TRANSFERS, filter, out);
}

extern "C" uint32_t tbgpu_scan_accounts(tbgpu_ctx* c, const tbgpu_index_filter_t* filter, tbgpu_account_t* out) {
    CallGuard guard_(c, false);
    return scan_objects(c, TBGPU_INDEX_ACCOUNTS, filter, out);
}

extern "C" uint32_t tbgpu_get_account_transfers(tbgpu_ctx* c, const tbgpu_account_filter_t* filter, tbgpu_transfer_t* out) {
    return query_host(c, filter, out, false);
}

extern "C" uint32_t tbgpu_get_account_history(tbgpu_ctx* c, const tbgpu_account_filter_t* filter,
                                              tbgpu_account_balance_t* out) {
    return query_host(c, filter, out, true);
}

extern "C" uint64_t tbgpu_get_account_transfers_device(tbgpu_ctx* c, uint32_t count, const void* filters_device,
                                                       uint32_t stride, void* out_device, uint32_t* result_counts) {
    CallGuard guard_(c, false);
    return run_queries(c, (const tbgpu_account_filter_t*)filters_device, count, stride, out_device, false, result_counts);
}

extern "C" uint64_t tbgpu_get_account_history_device(tbgpu_ctx* c, uint32_t count, const void* filters_device,
                                                     uint32_t stride, void* out_device, uint32_t* result_counts) {
    CallGuard guard_(c, false);
    return run_queries(c, (const tbgpu_account_filter_t*)filters_device, count, stride, out_device, true, result_counts);
}

// ------------------------------------------------------- persistence ------

namespace {
constexpr u64 CK_MAGIC = 0x314B435550474254ull;  // "TBGPUCK1"
// version 1: one state machine; version 3: a ledger shard's image, which also lists
// the other shards' accounts its directory knows (n_foreign ForeignAccount records,
// sorted by id, after the history rows) and names its shard: `shard` = world << 16 |
// rank.  An image opens only into a ctx of the same kind and, for a shard, the same
// world and rank.  Version 2 is the shard image of round 5's first trees, which did not
// name its shard (`shard` 0): it still opens into any shard ctx.  A shard ctx refuses a
// version-1 image with -95 (those trees wrote a shard image without foreign accounts as
// version 1, which cannot be told apart from an unsharded image).
struct CkHeader {
    u64 magic;
    u32 version, shard;
    u64 n_accounts, n_rows, n_hist, commit_ts, checksum;
    u64 n_foreign;
};
static_assert(sizeof(CkHeader) == 64, "checkpoint header");

u64 ck_payload_bytes(u64 na, u64 nr, u64 nh, u64 nf) {
    return na * 128 + nr * 128 + 2 * nr + nh * 256 + nf * sizeof(ForeignAccount);
}

// Checksum of the payload: four interleaved multiply-xor lanes over u64 words
// (integrity against truncation and corruption, not an adversary).
u64 ck_checksum(const u8* p, u64 n) {
    u64 h[4] = {0x9E3779B97F4A7C15ull, 0xC2B2AE3D27D4EB4Full, 0x165667B19E3779F9ull, 0x27D4EB2F165667C5ull};
    const u64 words = n / 8;
    const u64* w = (const u64*)p;
    for (u64 k = 0; k < words; k++) h[k & 3] = (h[k & 3] ^ w[k]) * 0x100000001B3ull;
    u64 tail = 0;
    memcpy(&tail, p + words * 8, n - words * 8);
    return mix64(h[0] ^ mix64(h[1] ^ mix64(h[2] ^ mix64(h[3] ^ tail ^ n))));
}
}  // namespace

extern "C" uint64_t tbgpu_checkpoint_size(tbgpu_ctx* c) {
    return sizeof(CkHeader) + ck_payload_bytes(c->n_accounts, c->n_rows, c->n_hist, c->n_foreign);
}

extern "C" uint64_t tbgpu_checkpoint(tbgpu_ctx* c, void* out, uint64_t capacity) {
    CallGuard guard_(c, false);
    const u64 size = tbgpu_checkpoint_size(c);
    if (capacity < size) return 0;
    wait_stream(c->stream);
    u8* p = (u8*)out + sizeof(CkHeader);
    const u64 na = c->n_accounts, nr = c->n_rows, nh = c->n_hist;
    if (na) d2h(c, p, c->T.acc, na * 128, c->stream);
    if (nr) d2h(c, p + na * 128, c->T.xrows, nr * 128, c->stream);
    if (nr) d2h(c, p + na * 128 + nr * 128, c->T.xful, nr, c->stream);
    u8* imp = p + na * 128 + nr * 129;
    if (nr && c->ximp) d2h(c, imp, c->ximp, nr, c->stream);
    else memset(imp, 0, nr);
    if (nh) d2h(c, imp + nr, c->T.hrows, nh * 256, c->stream);
    const u64 nf = c->n_foreign;
    if (nf) {
        // the directory's entries for other shards' accounts, gathered, then sorted by id
        // (the gather's order is not deterministic; the image is)
        ForeignAccount* buf = nullptr;
        u32* cur = nullptr;
        HIP_CHECK(hipMalloc((void**)&buf, nf * sizeof(ForeignAccount)));
        HIP_CHECK(hipMalloc((void**)&cur, sizeof(u32)));
        HIP_CHECK(hipMemsetAsync(cur, 0, sizeof(u32), c->stream));
        launch_collect_foreign(c->T, buf, cur, nf, c->stream);
        u32 got = 0;
        d2h(c, &got, cur, sizeof(u32), c->stream);
        ForeignAccount* fa = (ForeignAccount*)(imp + nr + nh * 256);
        d2h(c, fa, buf, nf * sizeof(ForeignAccount), c->stream);
        wait_stream(c->stream);
        HIP_CHECK(hipFree(buf));
        HIP_CHECK(hipFree(cur));
        if (got != nf) tbgpu_fatal("checkpoint", "directory holds another count of foreign accounts", __FILE__, __LINE__);
        std::sort(fa, fa + nf, [](const ForeignAccount& a, const ForeignAccount& b) {
            return a.id_hi != b.id_hi ? a.id_hi < b.id_hi : a.id_lo < b.id_lo;
        });
    }
    CkHeader h{};
    h.magic = CK_MAGIC;
    h.version = c->T.shard_world ? 3 : 1;
    h.shard = c->T.shard_world ? (c->T.shard_world << 16 | c->T.shard_rank) : 0;
    h.n_foreign = nf;
    h.n_accounts = na;
    h.n_rows = nr;
    h.n_hist = nh;
    h.commit_ts = tbgpu_commit_timestamp(c);
    h.checksum = ck_checksum(p, size - sizeof(CkHeader));
    memcpy(out, &h, sizeof h);
    return size;
}

extern "C" int tbgpu_open(tbgpu_ctx* c, const void* image, uint64_t size) {
    CallGuard guard_(c, false);
    if (size < sizeof(CkHeader)) return -22;
    CkHeader h;
    memcpy(&h, image, sizeof h);
    if (h.magic != CK_MAGIC || h.version < 1 || h.version > 3) return -22;
    if (h.version == 1 && (h.n_foreign != 0 || h.shard != 0)) return -22;
    if (h.version == 2 && h.shard != 0) return -22;
    // a ledger shard's image only into the ctx of the same shard, and an unsharded one
    // only into an unsharded ctx
    if (h.version == 1 && c->T.shard_world) return -95;
    if (h.version != 1 && !c->T.shard_world) return -22;
    if (h.version == 3 && h.shard != (c->T.shard_world << 16 | c->T.shard_rank)) return -22;
    if (size != sizeof(CkHeader) + ck_payload_bytes(h.n_accounts, h.n_rows, h.n_hist, h.n_foreign)) return -22;
    const u8* p = (const u8*)image + sizeof(CkHeader);
    if (ck_checksum(p, size - sizeof(CkHeader)) != h.checksum) return -22;
    if (h.n_accounts > c->accounts_max || h.n_rows > c->xrow_cap || h.n_hist > c->hist_cap) return -28;
    {  // the account index: every id outside the directory takes a hash slot (load <= 0.5)
        auto hashed = [&](u64 lo, u64 hi) {
            return !(hi == 0 && (lo >> 32) < c->T.dense_blocks && (u64)(u32)lo - 1 < c->T.dense_span);
        };
        u64 nhash = 0;
        const Account* acc = (const Account*)p;
        for (u64 k = 0; k < h.n_accounts; k++) nhash += hashed((u64)acc[k].id, (u64)(acc[k].id >> 64));
        const ForeignAccount* fa =
            (const ForeignAccount*)(p + h.n_accounts * 128 + h.n_rows * 130 + h.n_hist * 256);
        for (u64 k = 0; k < h.n_foreign; k++) nhash += hashed(fa[k].id_lo, fa[k].id_hi);
        if (nhash > c->T.hash_limit) return -28;
    }
    tbgpu_reset(c);
    const u64 na = h.n_accounts, nr = h.n_rows, nh = h.n_hist;
    hipStream_t s = c->stream;
    // the reset's memsets run on the ctx's non-blocking stream, which the blocking
    // copies below do not wait for
    wait_stream(s);
    if (na) h2d(c, c->T.acc, p, na * 128, c->stream);
    if (nr) h2d(c, c->T.xrows, p + na * 128, nr * 128, c->stream);
    if (nr) h2d(c, c->T.xful, p + na * 128 + nr * 128, nr, c->stream);
    const u8* imp = p + na * 128 + nr * 129;
    bool any_imported = false;
    for (u64 k = 0; k < nr && !any_imported; k++) any_imported = imp[k] != 0;
    if (any_imported) {
        if (!c->ximp) {
            ZeroOn zero_on(s);
            c->ximp = dalloc<u8>(c->xrow_cap, &c->bytes);
        }
        HIP_CHECK(hipMemsetAsync(c->ximp, 0, c->xrow_cap, s));
        wait_stream(s);
        h2d(c, c->ximp, imp, nr, c->stream);
    }
    if (nh) h2d(c, c->T.hrows, imp + nr, nh * 256, c->stream);
    // derived state: the account index, the transfer-id index and its key range,
    // the overflow guard; the account-transfers index rebuilds on the next query
    launch_rebuild_accounts(c->T, na, s);
    const u64 nf = h.n_foreign;
    if (nf) {  // a ledger shard: the other shards' accounts back into the directory
        ForeignAccount* buf = nullptr;
        HIP_CHECK(hipMalloc((void**)&buf, nf * sizeof(ForeignAccount)));
        h2d(c, buf, imp + nr + nh * 256, nf * sizeof(ForeignAccount), s);
        launch_insert_foreign(c->T, buf, nf, s);
        wait_stream(s);
        HIP_CHECK(hipFree(buf));
    }
    for (u64 off = 0; off < nr; off += 1u << 30) {
        const u32 k = (u32)std::min<u64>(nr - off, 1u << 30);
        launch_import_transfers(c->T, c->T.xrows + off, k, off, s);  // rows in place: index + key range
    }
    h2d(c, c->T.commit_ts, &h.commit_ts, sizeof(u64), s);
    HIP_CHECK(hipMemsetAsync(c->T.hcount + 2, 0, sizeof(u32), s));  // a fresh index: no tombstones
    c->eager_events = 0;
    u32 refused = 0;
    d2h(c, &refused, c->T.hcount + 1, sizeof(u32), s);
    if (refused) tbgpu_fatal("open", "account index full after the capacity check", __FILE__, __LINE__);
    c->n_accounts = na;
    c->n_foreign = nf;
    c->n_rows = nr;
    c->n_hist = nh;
    c->rows_hi = nr;
    set_base(c, BASE_ROWS, nr);
    set_base(c, BASE_HIST, nh);
    return 0;
}

static u128 to128(tbgpu_uint128_t x) { return ((u128)x.hi << 64) | x.lo; }

extern "C" int tbgpu_test_set_balances(tbgpu_ctx* c, tbgpu_uint128_t id, tbgpu_uint128_t dp, tbgpu_uint128_t dpo,
                                       tbgpu_uint128_t cp, tbgpu_uint128_t cpo) {
    CallGuard guard_(c, false);
    Bal4 b{to128(dp), to128(dpo), to128(cp), to128(cpo)};
    launch_set_balances(c->T, to128(id), b, c->status, c->stream);
    int st = 0;
    d2h(c, &st, c->status, sizeof(int), c->stream);
    wait_stream(c->stream);
    return st;
}

extern "C" int tbgpu_get_posted(tbgpu_ctx* c, tbgpu_uint128_t pending_id) {
    CallGuard guard_(c, false);
    launch_get_posted(c->T, to128(pending_id), c->status, c->stream);
    int st = 0;
    d2h(c, &st, c->status, sizeof(int), c->stream);
    wait_stream(c->stream);
    return st;
}

extern "C" uint64_t tbgpu_account_count(tbgpu_ctx* c) { return c->n_accounts; }
extern "C" uint64_t tbgpu_transfer_count(tbgpu_ctx* c) { return c->n_rows; }
extern "C" uint64_t tbgpu_history_count(tbgpu_ctx* c) { return c->n_hist; }

extern "C" uint64_t tbgpu_export_transfers(tbgpu_ctx* c, uint64_t first, uint64_t count, tbgpu_transfer_t* out) {
    CallGuard guard_(c, false);
    if (first >= c->n_rows) return 0;
    count = std::min<u64>(count, c->n_rows - first);
    wait_stream(c->stream);  // the blocking copy (null stream) does not wait for the ctx's stream
    d2h(c, out, c->T.xrows + first, count * sizeof(Transfer), c->stream);
    return count;
}

extern "C" uint64_t tbgpu_export_history(tbgpu_ctx* c, uint64_t first, uint64_t count, tbgpu_account_history_t* out) {
    CallGuard guard_(c, false);
    if (first >= c->n_hist) return 0;
    count = std::min<u64>(count, c->n_hist - first);
    wait_stream(c->stream);  // the blocking copy (null stream) does not wait for the ctx's stream
    d2h(c, out, c->T.hrows + first, count * sizeof(History), c->stream);
    return count;
}

extern "C" uint64_t tbgpu_export_accounts(tbgpu_ctx* c, tbgpu_account_t* out, uint64_t capacity) {
    CallGuard guard_(c, false);
    const u64 n = std::min<u64>(capacity, c->n_accounts);  // dense rows, creation order
    wait_stream(c->stream);  // the blocking copy (null stream) does not wait for the ctx's stream
    if (n) d2h(c, out, c->T.acc, n * sizeof(Account), c->stream);
    return n;
}

extern "C" uint64_t tbgpu_commit_timestamp(tbgpu_ctx* c) {
    CallGuard guard_(c, false);
    u64 v = 0;  // behind whatever the engine's stream still has queued (tbgpu_advance_commit_timestamp)
    d2h(c, &v, c->T.commit_ts, sizeof(u64), c->stream);
    wait_stream(c->stream);
    return v;
}

extern "C" void tbgpu_last_stats(tbgpu_ctx* c, tbgpu_stats* out) {
    if (c->stats_lazy) {  // a polled small call: its device time once the launch has ended
        c->stats_lazy = false;
        wait_event(c->ev1);
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->stats.device_ms = ms;
    }
    *out = c->stats;
}

extern "C" int tbgpu_last_error(tbgpu_ctx* c, char* buf, uint32_t len) {
    if (!buf || !len) return 0;
    snprintf(buf, len, "%s", c ? c->err : "no ctx");
    return (int)strlen(buf);
}

// The drop-in call timed from C (bench.py host_path): what the Zig shim's call costs,
// without a host-language wrapper around it.  Batch k is counts[k] events at the running
// offset of `events`, committed at timestamps[k]; mode 0: tbgpu_create_transfers per
// batch; mode 1: tbgpu_prefetch_transfers + tbgpu_prefetch_wait, then
// tbgpu_create_transfers of the same batch, as the replica runs them.
extern "C" int tbgpu_bench_host_calls(tbgpu_ctx* c, int mode, uint32_t calls, const tbgpu_transfer_t* events,
                                      const uint32_t* counts, const uint64_t* timestamps,
                                      tbgpu_create_transfers_result_t* results, double* commit_us,
                                      double* prefetch_us) {
    using clk = std::chrono::steady_clock;
    u64 off = 0;
    for (uint32_t k = 0; k < calls; k++) {
        const tbgpu_transfer_t* ev = events + off;
        const auto t0 = clk::now();
        if (mode == 1) {
            if (tbgpu_prefetch_transfers(c, ev, counts[k]) != 0) return -22;
            tbgpu_prefetch_wait(c);
        }
        const auto t1 = clk::now();
        tbgpu_create_transfers(c, timestamps[k], ev, counts[k], results);
        const auto t2 = clk::now();
        commit_us[k] = std::chrono::duration<double, std::micro>(t2 - t1).count();
        if (prefetch_us) prefetch_us[k] = std::chrono::duration<double, std::micro>(t1 - t0).count();
        off += counts[k];
    }
    return 0;
}

// The replica's sequence for one op on the primary, timed from C (bench.py host_path
// `staged`): tbgpu_stage_transfers at prepare, a busy-wait of `gap_us` standing for the
// journal write and the replication round trip, then prefetch (staged) + its wait and
// the commit back to back (src/vsr/replica.zig:3137-3152).  The key is the call's index
// (a stand-in for the header's checksum_body).
extern "C" int tbgpu_bench_host_staged(tbgpu_ctx* c, uint32_t calls, const tbgpu_transfer_t* events,
                                       const uint32_t* counts, const uint64_t* timestamps,
                                       tbgpu_create_transfers_result_t* results, double gap_us, double* stage_us,
                                       double* prefetch_us, double* commit_us) {
    using clk = std::chrono::steady_clock;
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    u64 off = 0;
    for (uint32_t k = 0; k < calls; k++) {
        const tbgpu_transfer_t* ev = events + off;
        const tbgpu_uint128_t key{0x5354414745ull, (u64)k + 1};
        const auto t0 = clk::now();
        if (tbgpu_stage_transfers(c, key, ev, counts[k]) != 0) return -22;
        const auto t1 = clk::now();
        while (us(t1, clk::now()) < gap_us) {
        }
        const auto t2 = clk::now();
        if (tbgpu_prefetch_transfers_staged(c, key, ev, counts[k]) != 0) return -22;
        tbgpu_prefetch_wait(c);
        const auto t3 = clk::now();
        tbgpu_create_transfers(c, timestamps[k], ev, counts[k], results);
        const auto t4 = clk::now();
        stage_us[k] = us(t0, t1);
        prefetch_us[k] = us(t2, t3);
        commit_us[k] = us(t3, t4);
        off += counts[k];
    }
    return 0;
}
