"""One round of the exact sharded router over whole arrays (shard.py `_round`'s
algorithm, without per-event Python objects or pickled collectives).

The router's general step is what takes every step the device fast
step cannot: post/void whose pending may live on another shard
(src/state_machine.zig:1391-1498), repeated ids (`:1284`), ids that are not strictly
rising along the global order.  `ShardedStateMachine._round` states it event by event
(dicts, sorted tuples, `all_gather_object` of pickled lists): the reference form, kept
for the tests.  This module computes the same round with sorts, segment reductions
and tensor collectives (`all_gather` / `all_to_all_single` of int64 rows over the
step's communicator: RCCL on GPUs, gloo in the CPU tests), so that a general step
costs O(events log events) array work per rank:

1. directory: every rank's id and pending-id records (position, kind, key, route
   hint) are all-gathered; the unique keys are looked up in each shard's engine
   (the engines are the directory of committed ids) and the owners all-reduced;
   a sort by (key, position) gives each key's first occurrence in the step;
2. routing of this rank's events by the rules of `_round` (committed id -> its
   holder, duplicate on the same owner or in the same chain -> follow, post/void ->
   its pending's holder), chains filled to one owner where members can go anywhere,
   and the earliest hazard over all ranks splits the step;
3. imports of colliding committed rows, the exchange of the events to their owners,
   the spanning chains, the dry rounds and their serial fallback, the commit, and
   the replies back to their sources -- all as arrays.

Results are bit-identical to `_round` (tests/test_shard.py runs both against one
oracle fed the global order).
"""
from __future__ import annotations

import numpy as np

from .types import RESULT_DTYPE, TRANSFER_DTYPE, U128_DTYPE

POST_VOID = 4 | 8          # TransferFlags post_pending_transfer | void_pending_transfer
LINKED = 1
ANY, PV = -1, -2           # route hints (shard.py)
NEW, EXISTS, DUP, PEND, PEND_NONE, PEND_HAZARD = range(6)
CTL_CHAIN_END, CTL_SKIP, CTL_DOOM = 1, 2, 4
LINKED_EVENT_FAILED = 1
INF = np.iinfo(np.int64).max
U64_MAX = np.uint64(0xFFFFFFFFFFFFFFFF)
HL = np.dtype([("hi", "<u8"), ("lo", "<u8")])  # u128 in numeric order (structured compare)
LOOKUP_CHUNK = 4096


# ----------------------------------------------------------- collectives --
def gather_rows(comm, rows: np.ndarray) -> tuple[np.ndarray, list[int]]:
    """All-gather an int64 [k, w] array of every rank (k may differ): the rows of
    rank 0, then rank 1, ...; and each rank's row count."""
    torch, dist = comm.torch, comm.dist
    w = rows.shape[1]
    k = torch.tensor([rows.shape[0]], dtype=torch.int64, device=comm.device)
    ks = [torch.empty_like(k) for _ in range(comm.world)]
    dist.all_gather(ks, k, group=comm.group)
    counts = [int(x.item()) for x in ks]
    mx = max(max(counts), 1)
    pad = np.zeros((mx, w), dtype=np.int64)
    pad[:rows.shape[0]] = rows
    t = torch.from_numpy(pad).to(comm.device)
    outs = [torch.empty_like(t) for _ in range(comm.world)]
    dist.all_gather(outs, t, group=comm.group)
    return np.concatenate([o.cpu().numpy()[:c] for o, c in zip(outs, counts)]), counts


def allreduce_max(comm, a: np.ndarray) -> np.ndarray:
    torch, dist = comm.torch, comm.dist
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(comm.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=comm.group)
    return t.cpu().numpy()


def alltoall_rows(comm, parts: list[np.ndarray], width: int) -> list[np.ndarray]:
    """parts[d]: int64 [k_d, width] rows for rank d; returns the rows received, by source."""
    got = comm.alltoallv([np.ascontiguousarray(p, dtype=np.int64).reshape(-1).view(np.uint8) for p in parts])
    return [g.view(np.int64).reshape(-1, width) if len(g) else np.zeros((0, width), np.int64) for g in got]


def alltoall_events(comm, parts: list[np.ndarray]) -> list[np.ndarray]:
    got = comm.alltoallv([np.ascontiguousarray(p, dtype=TRANSFER_DTYPE).view(np.uint8).reshape(-1) for p in parts])
    return [g.view(TRANSFER_DTYPE) if len(g) else np.zeros(0, TRANSFER_DTYPE) for g in got]


def min_over_ranks(comm, v: int) -> int:
    return -int(allreduce_max(comm, np.array([-v], dtype=np.int64))[0])


# ------------------------------------------------------------------ keys --
def _hl(lo: np.ndarray, hi: np.ndarray) -> np.ndarray:
    k = np.zeros(len(lo), dtype=HL)
    k["lo"] = lo
    k["hi"] = hi
    return k


def lookup_owners(sm, keys: np.ndarray) -> np.ndarray:
    """Collective.  For sorted unique u128 keys (HL), the shard that holds each as a
    committed transfer (the owner of its row's ledger; imported copies answer the same),
    or -1: every rank looks the keys up in its engine, the owners are all-reduced."""
    own = np.full(len(keys), -1, dtype=np.int64)
    q = np.zeros(len(keys), dtype=U128_DTYPE)
    q["lo"], q["hi"] = keys["lo"], keys["hi"]
    for c0 in range(0, len(keys), LOOKUP_CHUNK):
        rows = sm.backend.lookup_transfers(q[c0:c0 + LOOKUP_CHUNK])
        if len(rows):
            at = np.searchsorted(keys, _hl(rows["id_lo"], rows["id_hi"]))
            own[at] = sm.owners_vec(rows["ledger"])
    return allreduce_max(sm.comm, own)


def directory_device(sm, R: np.ndarray) -> np.ndarray | None:
    """Collective.  The directory step of the round on the device (csrc/directory.hip),
    when this rank's backend is the HIP engine and the step's collectives run on a GPU
    (RCCL): every rank's records all-gathered into one device tensor, each shard's
    committed owners (tbgpu_route_directory_owners) all-reduced, then the key grouping
    (tbgpu_route_directory).  Returns this rank's rows (type, hint, first position), or
    None where the host form applies (CPU ranks: the oracle backend of the CPU tests;
    an owner map other than ledger % world)."""
    comm = sm.comm
    torch, dist = comm.torch, comm.dist
    if not (hasattr(sm.backend, "route_directory") and comm.device.type == "cuda" and sm._ledger_mod):
        return None
    k = torch.tensor([R.shape[0]], dtype=torch.int64, device=comm.device)
    ks = [torch.empty_like(k) for _ in range(comm.world)]
    dist.all_gather(ks, k, group=comm.group)
    counts = [int(x.item()) for x in ks]
    mx = max(max(counts), 1)
    pad = np.zeros((mx, 5), dtype=np.int64)
    pad[:R.shape[0]] = R
    t = torch.from_numpy(pad).to(comm.device)
    outs = [torch.empty_like(t) for _ in range(comm.world)]
    dist.all_gather(outs, t, group=comm.group)
    A = torch.cat([o[:c] for o, c in zip(outs, counts)]).contiguous()
    owners = torch.empty(A.shape[0], dtype=torch.int64, device=comm.device)
    sm.backend.route_directory_owners(sm.world, A, owners)
    dist.all_reduce(owners, op=dist.ReduceOp.MAX, group=comm.group)
    out = torch.empty((A.shape[0], 3), dtype=torch.int64, device=comm.device)
    sm.backend.route_directory(A, owners, out)
    off = sum(counts[:comm.rank])
    return out[off:off + R.shape[0]].cpu().numpy()


def segment_first(starts: np.ndarray, n: int) -> np.ndarray:
    """Index of each element's segment start (starts: bool[n], starts[0] True)."""
    return np.maximum.accumulate(np.where(starts, np.arange(n), 0)) if n else np.zeros(0, np.int64)


def _directory_host(sm, R: np.ndarray):
    """Collective.  The directory step on the host (numpy): the same types, hints and
    first positions as directory_device, by a stable sort of every record by key."""
    comm = sm.comm
    A, counts = gather_rows(comm, R)
    keys = _hl(A[:, 2].view(np.uint64), A[:, 3].view(np.uint64))
    order = np.argsort(keys, kind="stable")
    ks = keys[order]
    newk = np.ones(len(ks), dtype=bool)
    if len(ks) > 1:
        newk[1:] = ks[1:] != ks[:-1]
    uid = np.empty(len(A), dtype=np.int64)
    uid[order] = np.cumsum(newk) - 1
    U = ks[newk]
    cown = lookup_owners(sm, U)[uid] if len(U) else np.zeros(len(A), np.int64)
    # the first occurrence of each key among the id records of ids not committed
    k0 = A[:, 1] == 0
    cand = k0 & (cown < 0)
    firstP = np.full(len(U), INF, dtype=np.int64)
    np.minimum.at(firstP, uid[cand], A[cand, 0])
    firstH = np.full(len(U), ANY, dtype=np.int64)
    isfirst = cand & (A[:, 0] == firstP[uid])
    firstH[uid[isfirst]] = A[isfirst, 4]
    fP, fH = firstP[uid], firstH[uid]
    typ = np.where(k0, np.where(cown >= 0, EXISTS, np.where(isfirst, NEW, DUP)),
                   np.where(cown >= 0, PEND, np.where(fP < A[:, 0],
                                                       np.where((fH == ANY) | (fH == PV), PEND_HAZARD, PEND),
                                                       PEND_NONE)))
    ahint = np.where(cown >= 0, cown, fH)
    off = sum(counts[:comm.rank])
    mine_t, mine_h, mine_p = typ[off:off + len(R)], ahint[off:off + len(R)], fP[off:off + len(R)]
    return mine_t, mine_h, mine_p


# ----------------------------------------------------------------- round --
def window_cut(sm, glob, my_events, g0, i0) -> int:
    """Collective when the window ends inside a batch.  The global position where this
    round stops at the latest: about sm.round_window events after (g0, i0), moved back
    to the start of the chain it falls in (chains never cross a batch; the batch's
    owner knows its chains), or past that chain when it is the round's first.  A round
    only commits its prefix before the first hazard, so its routing needs no events
    beyond this point; the window bounds the host work of the rounds that hazards
    make many.  INF: the rest of the step fits the window."""
    left = sm.round_window
    if not left:
        return INF
    g, i = g0, i0
    while g < len(glob):
        if left <= 0:
            return g << 32
        c = glob[g][2]
        if c - i > left:
            break
        left -= c - i
        g, i = g + 1, 0
    else:
        return INF
    iw = i + left
    prop = INF
    if glob[g][0] == sm.rank:
        linked = (my_events[g]["flags"] & LINKED) != 0
        s = iw
        while s > 0 and linked[s - 1]:
            s -= 1
        if g == g0 and s <= i0:  # the window's first chain: cut after it
            e = iw
            while e < c - 1 and linked[e]:
                e += 1
            s = e + 1
        prop = (g << 32) | s if s < c else (g + 1) << 32
    return min_over_ranks(sm.comm, prop)


def round_vec(sm, glob, T, my_events, replies, start, done=None):
    """ShardedStateMachine._round over arrays: the same routing, splits, dry rounds
    and commit; returns None when the round committed every remaining event, else the
    (global batch, index) to resume from.  `done` (per global batch of this rank: which
    events committed in earlier rounds) enables per-shard stops (shard_stops): then a
    round commits, on each shard, its events before that shard's stop, and the resume
    point is the first event not done anywhere."""
    comm = sm.comm
    W, me = sm.world, sm.rank
    g0, i0 = start
    P0 = (g0 << 32) | i0
    mark = _phase_clock(sm)
    # ---- 1. my remaining events of the round's window, in global order
    wcut = window_cut(sm, glob, my_events, g0, i0)
    wg, wi = (wcut >> 32, wcut & 0xFFFFFFFF) if wcut != INF else (INF, 0)
    evs, Gs, Is = [], [], []
    for g in sorted(my_events):
        if g < g0 or g > wg:
            continue
        b = my_events[g]
        lo = i0 if g == g0 else 0
        hi = wi if g == wg else len(b)
        if lo < hi:
            idx = np.arange(lo, hi, dtype=np.int64)
            if done is not None:
                idx = idx[~done[g][lo:hi]]
            if len(idx):
                evs.append(b[idx])
                Gs.append(np.full(len(idx), g, np.int64))
                Is.append(idx)
    E = np.concatenate(evs) if evs else np.zeros(0, TRANSFER_DTYPE)
    G = np.concatenate(Gs) if Gs else np.zeros(0, np.int64)
    I = np.concatenate(Is) if Is else np.zeros(0, np.int64)
    n = len(E)
    P = (G << 32) | I
    flags = E["flags"].astype(np.int64)
    pv = (flags & POST_VOID) != 0
    linked = (flags & LINKED) != 0
    # chain key (position of its first member): a run of linked events and the event
    # that ends it, within one batch (execute, src/state_machine.zig:1018-1035)
    cstart = np.ones(n, dtype=bool)
    if n > 1:
        cstart[1:] = (G[1:] != G[:-1]) | (I[1:] != I[:-1] + 1) | ~linked[:-1]
    chain = P[segment_first(cstart, n)] if n else np.zeros(0, np.int64)

    mark("order")
    # ---- 2. directory
    xlo, xhi = E["id_lo"], E["id_hi"]
    plo, phi = E["pending_id_lo"], E["pending_id_hi"]
    zero = lambda lo, hi: (lo == 0) & (hi == 0)
    imax = lambda lo, hi: (lo == U64_MAX) & (hi == U64_MAX)
    xval = ~(zero(xlo, xhi) | imax(xlo, xhi))
    pval = pv & ~(zero(plo, phi) | imax(plo, phi) | ((plo == xlo) & (phi == xhi)))
    led = E["ledger"].astype(np.int64)
    own = np.where(led != 0, sm.owners_vec(led), ANY)
    hint = np.where(pv, PV, own)
    r0, r1 = np.nonzero(xval)[0], np.nonzero(pval)[0]
    R = np.zeros((len(r0) + len(r1), 5), dtype=np.int64)
    R[:len(r0), 0] = P[r0]
    R[:len(r0), 2] = xlo[r0].view(np.int64)
    R[:len(r0), 3] = xhi[r0].view(np.int64)
    R[:len(r0), 4] = hint[r0]
    R[len(r0):, 0] = P[r1]
    R[len(r0):, 1] = 1
    R[len(r0):, 2] = plo[r1].view(np.int64)
    R[len(r0):, 3] = phi[r1].view(np.int64)
    R[len(r0):, 4] = ANY
    dev = directory_device(sm, R)
    if dev is not None:
        mine_t, mine_h, mine_p = dev[:, 0], dev[:, 1], dev[:, 2]
    else:
        mine_t, mine_h, mine_p = _directory_host(sm, R)
    id_t = np.full(n, NEW, np.int64)
    id_h = np.full(n, ANY, np.int64)
    id_p = np.full(n, INF, np.int64)
    id_t[r0], id_h[r0], id_p[r0] = mine_t[:len(r0)], mine_h[:len(r0)], mine_p[:len(r0)]
    p_t = np.full(n, PEND_NONE, np.int64)
    p_h = np.full(n, ANY, np.int64)
    p_p = np.full(n, INF, np.int64)
    p_t[r1], p_h[r1], p_p[r1] = mine_t[len(r0):], mine_h[len(r0):], mine_p[len(r0):]
    mark("directory")

    # ---- 3. routing of my events (shard.py _round, rule for rule)
    def same_chain(pos):
        j = np.clip(np.searchsorted(P, pos), 0, max(n - 1, 0))
        ok = (pos != INF) & (n > 0)
        ok &= P[j] == pos if n else ok
        return ok & (chain[j] == chain), j

    route = np.full(n, ANY, dtype=np.int64)
    follow = np.full(n, -1, dtype=np.int64)
    hazard = np.zeros(n, dtype=bool)
    # post/void
    sc_p, jp = same_chain(p_p)
    r_pv = np.where(p_t == PEND, p_h, ANY)
    fol_pv = pv & (p_t == PEND_HAZARD) & sc_p
    hazard |= pv & (p_t == PEND_HAZARD) & ~sc_p
    follow = np.where(fol_pv, jp, follow)
    sc_i, ji = same_chain(id_p)
    dup_moves = pv & (id_t == DUP) & (fol_pv | (id_h != r_pv) | (id_h == ANY) | (id_h == PV))
    follow = np.where(dup_moves & sc_i, ji, follow)
    hazard |= dup_moves & ~sc_i
    route = np.where(pv, r_pv, route)
    # regular transfers
    reg = ~pv
    route = np.where(reg & (id_t == EXISTS), id_h, route)
    route = np.where(reg & (id_t == NEW), own, route)
    dup = reg & (id_t == DUP)
    follow = np.where(dup & sc_i, ji, follow)
    route = np.where(dup & ~sc_i, own, route)
    hazard |= dup & ~sc_i & (id_h != ANY) & (own != ANY) & (id_h != own)
    # follows (their targets are earlier members of the same chain)
    for k in np.nonzero(follow >= 0)[0]:
        route[k] = route[follow[k]]
    # members that can go anywhere follow their chain's first member that cannot
    if n:
        seg = np.nonzero(cstart)[0]
        firstfix = np.minimum.reduceat(np.where(route != ANY, np.arange(n), INF), seg)
        fill = np.where(firstfix == INF, me, route[np.minimum(firstfix, n - 1)])
        route = np.where(route == ANY, np.repeat(fill, np.diff(np.append(seg, n))), route)
    # post/voids whose id is committed on another shard: that row, imported
    imp = pv & (id_t == EXISTS) & (id_h != route)
    mark("routing")

    # ---- 4. the earliest hazard over all ranks splits the step (per-shard stops: each
    # shard stops at its own first event that must wait)
    stops = None
    if done is not None and sm.shard_stops:
        # the effect shard (ShardStops)
        ef = np.where(led != 0, own, np.where(~pv | (p_t == PEND_NONE), EF_NONE,
                                              np.where(p_t == PEND, p_h, EF_ALL)))
        stops = ShardStops(sm, P, chain, ef, hazard, _key_hash(xlo, xhi, xval), _key_hash(plo, phi, pval), wcut)
        stop = INF if stops.any_commits() else P0
    else:
        hz = int(chain[np.nonzero(hazard)[0]].min()) if hazard.any() else INF
        stop = min_over_ranks(comm, hz)
    if stop <= P0:
        stops = None
        sm.stats["serial_fallbacks"] += 1
        nxt = INF
        if n and P[0] == P0:
            c = chain[0]
            after = np.nonzero((chain != c) & (P > P0))[0]
            nxt = int(P[after[0]]) if len(after) else int(((P[chain == c][-1] >> 32) + 1) << 32)
        stop = min_over_ranks(comm, nxt)
    stop = min(stop, wcut)
    loc = P < stop if stops is None else stops.committed(P)
    _do_imports(sm, xlo[imp], xhi[imp], id_h[imp], route[imp])
    mark("split_imports")

    # ---- 5. events to their owners (global order kept per source)
    dest = route[loc]
    parts, meta = [], []
    for d in range(W):
        s = np.nonzero(loc)[0][dest == d]
        parts.append(E[s])
        meta.append(np.stack([P[s], chain[s]], axis=1))
    recv = alltoall_events(comm, parts)
    rmeta = alltoall_rows(comm, meta, 2)
    mE = np.concatenate(recv) if recv else np.zeros(0, TRANSFER_DTYPE)
    mM = np.concatenate(rmeta) if rmeta else np.zeros((0, 2), np.int64)
    o = np.argsort(mM[:, 0], kind="stable")
    mE, mP, mC = mE[o], mM[o, 0], mM[o, 1]

    # spanning chains (the source knows every member's owner) and their last members
    lp, lc, lr = P[loc], chain[loc], route[loc]
    span_rows = np.zeros((0, 2), np.int64)
    if len(lp):
        sstart = np.ones(len(lp), dtype=bool)
        sstart[1:] = lc[1:] != lc[:-1]
        seg = np.nonzero(sstart)[0]
        rmin = np.minimum.reduceat(lr, seg)
        rmax = np.maximum.reduceat(lr, seg)
        last = np.maximum.reduceat(lp, seg)
        sp = rmin != rmax
        span_rows = np.stack([lc[seg][sp], last[sp]], axis=1)
    allspan, _ = gather_rows(comm, span_rows)
    so = np.argsort(allspan[:, 0], kind="stable") if len(allspan) else np.zeros(0, np.int64)
    span_keys, span_last = allspan[so, 0], allspan[so, 1]
    if me == 0:
        sm.stats["cross_chains"] += len(span_keys)

    mark("exchange")
    # ---- 6. commit (dry rounds while chains span shards)
    in_span = np.isin(mC, span_keys)
    mG, mI = mP >> 32, mP & 0xFFFFFFFF
    lastloc = np.ones(len(mP), dtype=bool)  # the owner's last local member of its chain
    if len(mP):
        co = np.lexsort((mP, mC))
        islast = np.ones(len(co), dtype=bool)
        islast[:-1] = mC[co][1:] != mC[co][:-1]
        lastloc = np.zeros(len(mP), dtype=bool)
        lastloc[co[islast]] = True
    mlast = span_last[np.clip(np.searchsorted(span_keys, mC), 0, max(len(span_keys) - 1, 0))] \
        if len(span_keys) else np.full(len(mP), -1, np.int64)
    brk = {}        # chain key -> position of its first failure (global)
    rounds = 0
    mask = np.ones(len(mP), dtype=bool)   # the events of this round (a serial fallback cuts it)
    while True:
        res = _commit_vec(sm, T, glob, mE[mask], mP[mask], mG[mask], mI[mask], mC[mask], in_span[mask],
                          lastloc[mask], mlast[mask], brk, dry=bool(len(span_keys)))
        if not len(span_keys):
            break
        rounds += 1
        sm.stats["dry_rounds"] += 1
        nb = _breaks(sm, mP[mask], mC[mask], in_span[mask], res)
        if nb == brk:
            res2 = _commit_vec(sm, T, glob, mE[mask], mP[mask], mG[mask], mI[mask], mC[mask], in_span[mask],
                               lastloc[mask], mlast[mask], brk, dry=False)
            # the commit is exact as long as it breaks every spanning chain where its
            # control said.  Whether to check is decided collectively first: `_breaks`
            # runs collectives, so every rank must enter it or none
            if int(allreduce_max(comm, np.array([int(not np.array_equal(res2, res))], np.int64))[0]):
                sm.stats["dry_commit_mismatch"] = sm.stats.get("dry_commit_mismatch", 0) + 1
                if _breaks(sm, mP[mask], mC[mask], in_span[mask], res2) != brk:
                    raise AssertionError("sharded commit: a committed chain broke elsewhere than its dry run "
                                         "(engine invariant: the same events and state gave other results)")
            res = res2
            break
        if rounds >= sm.max_rounds:
            head = int(mP[mask].min()) if mask.any() else INF
            head = min_over_ranks(comm, head)
            ks_ = span_keys
            cut = int(ks_[0]) if ks_[0] > head else (int(ks_[1]) if len(ks_) > 1 else None)
            tail = -min_over_ranks(comm, -(int(mP[mask].max()) if mask.any() else -1))  # collective
            if cut is None and tail > int(span_last[0]):
                # the lone spanning chain heads the round: commit it alone (its members'
                # outcomes then depend on the committed state only), the rest after it
                cut = int(span_last[0]) + 1
            if cut is not None:
                mask &= mP < cut
                keep = span_keys < cut
                span_keys, span_last = span_keys[keep], span_last[keep]
                in_span = np.isin(mC, span_keys)
                stop = min(stop, cut)
                if stops is not None:
                    stops.cut(cut)
                sm.stats["serial_fallbacks"] += 1
                brk, rounds = {}, 0
                continue
            if rounds >= sm.max_rounds + 2:
                raise RuntimeError("sharded commit: a lone cross-shard chain did not settle "
                                   "(its break depends on no other chain: an engine invariant failed)")
        brk = nb

    mark("commit")
    # ---- 7. replies to their sources
    rp, rg, ri = mP[mask], mG[mask], mI[mask]
    bad = res != 0
    src = np.array([glob[int(g)][0] for g in rg[bad]], dtype=np.int64) if bad.any() else np.zeros(0, np.int64)
    rows = np.stack([rg[bad], ri[bad], res[bad]], axis=1) if bad.any() else np.zeros((0, 3), np.int64)
    for got in alltoall_rows(comm, [rows[src == d] for d in range(W)], 3):
        for g, i, code in got.tolist():
            replies[g].append((i, code))
    top = 0
    if mask.any():
        ids = _hl(mE["id_lo"][mask], mE["id_hi"][mask])
        m = np.sort(ids)[-1]
        top = (int(m["hi"]) << 64) | int(m["lo"])
    sm.max_id = max(sm.max_id, sm.comm.allreduce_max(top))
    mark("replies")
    if done is not None:
        ok = P < stop if stops is None else stops.committed(P)
        for g in np.unique(G[ok]).tolist():
            done[g][I[ok & (G == g)]] = True
    if stops is not None:
        stop = stops.resume()
    if stop == INF:
        return None
    return (int(stop) >> 32, int(stop) & 0xFFFFFFFF)


def _key_hash(lo, hi, valid) -> np.ndarray:
    """A nonzero 64-bit hash of each valid u128 key (0: none).  Used only to find events
    that share a key; a collision makes the stops more conservative, never wrong."""
    with np.errstate(over="ignore"):
        h = lo.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        h ^= hi.astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)
        h ^= h >> np.uint64(29)
    h = (h | np.uint64(1)).view(np.int64)
    return np.where(valid, h, 0)


EF_NONE, EF_ALL = -3, -4    # effect shard of an event that cannot change state / whose shard is open


class ShardStops:
    """Collective (one all-gather).  Per-shard stops of a round: which events of the
    round's window wait, chosen so that each shard still applies its state changes in
    global order.  Every rank gathers the round's events (position, chain, effect shard,
    hazard, id and pending-id key hashes) and computes the same answer: the smallest
    closed set of waiting events that holds

    - every hazard (its outcome needs an earlier uncommitted event of another shard);
    - whole chains (linked events commit together, src/state_machine.zig:1018-1035);
    - events that share a key (id or pending id, in either role) in global order: a later
      one waits while an earlier one does (an earlier post/void must not see a pending
      created after it; a later repeat of an id must see the first one);
    - every event at or after the stop of its *effect shard*: the only shard where it can
      change state.  That is its ledger's owner (a transfer routed anywhere else fails:
      `exists*`, or accounts / pending of another ledger), nothing for a transfer with
      ledger 0 (it fails), and for a post/void with ledger 0 its pending's holder
      (committed, or the first occurrence in the step: if that one fails, the occurrence
      that holds the pending next round is an earlier hazard, which stopped its own
      shard before this event), nothing when no pending precedes it (it fails; a later
      event with that id waits with it, by the keys), or every shard for a pending
      hazard (its pending may come from a later repeat of an id whose first occurrence
      had no shard).  A shard's stop is the earliest chain start among the waiting events
      it is the effect shard of.

    Everything else an event reads is on its own shard or committed (the routing sends a
    post/void to its pending's holder and a repeat of an id to the holder or into a
    hazard), so the results are those of the global order: each shard applies the
    state-changing events it commits in increasing position, round after round; a
    waiting event that lands on another shard later can only fail there.  Fixed point
    over the stops (each only falls, to a chain start); past 64 iterations every event
    from the earliest waiting one on waits (the single stop of a round without them)."""

    def __init__(self, sm, P, chain, ef, hazard, kx, kp, wcut):
        rows = np.stack([P, chain, ef, hazard.astype(np.int64), kx, kp], axis=1) if len(P) else \
            np.zeros((0, 6), np.int64)
        A, _ = gather_rows(sm.comm, rows)
        A = A[np.argsort(A[:, 0], kind="stable")]
        self.P = A[:, 0]
        self.wcut = wcut
        self.wait = self._solve(sm.world, A[:, 0], A[:, 1], A[:, 2], A[:, 3] != 0, A[:, 4], A[:, 5], wcut)

    @staticmethod
    def _solve(W, P, C, EF, H, kx, kp, wcut):
        n = len(P)
        if not n:
            return np.zeros(0, bool)
        wait = H | (P >= wcut)
        if not wait.any():
            return wait
        # chains are runs of consecutive positions: their starts rise along P
        cidx = np.zeros(n, np.int64)
        np.cumsum(C[1:] != C[:-1], out=cidx[1:])
        nch = int(cidx[-1]) + 1
        # keys held by two or more of the round's records (a single record orders nothing)
        ke = np.concatenate([np.nonzero(kx)[0], np.nonzero(kp)[0]])
        kk = np.concatenate([kx[kx != 0], kp[kp != 0]])
        _, kinv, kcnt = np.unique(kk, return_inverse=True, return_counts=True)
        multi = kcnt[kinv] > 1
        ke, kinv = ke[multi], kinv[multi]
        kP = P[ke]
        nk = len(kcnt)
        one = EF >= 0
        efi = np.where(one, EF, 0)
        allm = EF == EF_ALL
        S = np.full(W, wcut, np.int64)

        def close(w):
            w = np.bincount(cidx, weights=w, minlength=nch)[cidx] > 0
            if len(ke):
                wk = w[ke]
                if wk.any():
                    fd = np.full(nk, INF, np.int64)
                    np.minimum.at(fd, kinv[wk], kP[wk])
                    later = kP > fd[kinv]
                    if later.any():
                        w[ke[later]] = True
                        w = np.bincount(cidx, weights=w, minlength=nch)[cidx] > 0
            return w

        for _ in range(64):
            w = close(wait | (one & (P >= S[efi])) | (allm & (P >= S.min())))
            S2 = S.copy()
            m = w & one
            np.minimum.at(S2, EF[m], C[m])
            if (w & allm).any():
                np.minimum(S2, C[w & allm].min(), out=S2)
            if np.array_equal(S2, S) and np.array_equal(w, wait):
                return w
            S, wait = S2, w
        first = P[wait].min() if wait.any() else wcut
        return P >= first

    def any_commits(self) -> bool:
        return bool((~self.wait).any())

    def committed(self, P) -> np.ndarray:
        if not len(P):
            return np.zeros(0, bool)
        return ~self.wait[np.searchsorted(self.P, P)]

    def cut(self, pos: int) -> None:
        self.wait |= self.P >= pos
        self.wcut = min(self.wcut, pos)

    def resume(self) -> int:
        """The first position not committed (INF: the step is done)."""
        return min(int(self.P[self.wait].min()) if self.wait.any() else INF, self.wcut)


def _phase_clock(sm):
    """Wall time (and this thread's CPU time, "cpu_" keys) of the general step's phases
    into sm.gtiming (ms) when sm.timed.  The phases end in a host value (every device call of the step returns host arrays), so
    the marks need no device synchronisation."""
    if not sm.timed:
        return lambda name: None
    import time
    t = [time.perf_counter(), time.thread_time()]

    def mark(name):
        now, cpu = time.perf_counter(), time.thread_time()
        sm.gtiming[name] = sm.gtiming.get(name, 0.0) + (now - t[0]) * 1e3
        sm.gtiming["cpu_" + name] = sm.gtiming.get("cpu_" + name, 0.0) + (cpu - t[1]) * 1e3
        t[0], t[1] = now, cpu
    return mark


def _do_imports(sm, lo, hi, holder, dest):
    """Rows of committed ids requested by this rank for `dest` shards, shipped from their
    holders and imported there (rows are immutable: importing early is harmless)."""
    W = sm.world
    req = np.stack([lo.view(np.int64), hi.view(np.int64), dest], axis=1) if len(lo) else np.zeros((0, 3), np.int64)
    if len(req):
        req = np.unique(np.concatenate([req, holder[:, None]], axis=1), axis=0)
    got = alltoall_rows(sm.comm, [req[req[:, 3] == h, :3] for h in range(W)] if len(req) else
                        [np.zeros((0, 3), np.int64)] * W, 3)
    send = [[] for _ in range(W)]
    for rows in got:
        if not len(rows):
            continue
        q = np.zeros(len(rows), dtype=U128_DTYPE)
        q["lo"], q["hi"] = rows[:, 0].view(np.uint64), rows[:, 1].view(np.uint64)
        found = sm.backend.lookup_transfers(q)
        fk = _hl(found["id_lo"], found["id_hi"])
        # the same id may be requested for several destinations (one row per request)
        if not np.isin(_hl(q["lo"], q["hi"]), fk).all():
            raise RuntimeError("sharded commit: the directory names a shard that does not hold the transfer")
        fo = np.argsort(fk, kind="stable")
        rows_by_q = found[fo[np.searchsorted(fk[fo], _hl(q["lo"], q["hi"]))]]
        for d in range(W):
            sel = rows[:, 2] == d
            if sel.any():
                send[d].append(rows_by_q[sel])
    recv = alltoall_events(sm.comm, [np.concatenate(s) if s else np.zeros(0, TRANSFER_DTYPE) for s in send])
    rows = np.concatenate(recv) if recv else np.zeros(0, TRANSFER_DTYPE)
    if len(rows):
        _, first = np.unique(_hl(rows["id_lo"], rows["id_hi"]), return_index=True)
        rows = rows[np.sort(first)]
        sm.backend.import_transfers(rows)
        sm.stats["imports"] += len(rows)


def _commit_vec(sm, T, glob, E, P, G, I, C, in_span, lastloc, mlast, brk, dry):
    """The owner's sub-batches (one per source batch, global order) with the chain
    control of the round; returns each event's result code (0 = ok)."""
    m = len(P)
    if not m:
        return np.zeros(0, np.int64)
    q = np.full(m, INF, dtype=np.int64)
    if brk:
        bk = np.array(sorted(brk), dtype=np.int64)
        bv = np.array([brk[k] for k in bk.tolist()], dtype=np.int64)
        ix = np.clip(np.searchsorted(bk, C), 0, len(bk) - 1)
        q = np.where(bk[ix] == C, bv[ix], INF)
    ctl = np.zeros(m, dtype=np.uint8)
    ctl[in_span & (q != INF) & (P > q)] |= CTL_SKIP
    end = in_span & lastloc & (P != mlast)
    ctl[end] |= CTL_CHAIN_END
    ctl[end & (q != INF) & (P < q)] |= CTL_DOOM
    gstart = np.ones(m, dtype=bool)
    gstart[1:] = G[1:] != G[:-1]
    seg = np.nonzero(gstart)[0]
    counts = np.diff(np.append(seg, m))
    n_g = np.array([glob[int(g)][2] for g in G[seg]], dtype=np.int64)
    Tg = np.array([T[int(g)] for g in G[seg]], dtype=np.int64)
    ts = (np.repeat(Tg - n_g, counts) + I + 1).astype(np.uint64)
    out, rc, _ = sm.backend.create_transfers_routed(counts.astype(np.uint32), E, ts,
                                                    ctl if ctl.any() else None, dry)
    res = np.zeros(m, dtype=np.int64)
    rc = rc.astype(np.int64)
    if rc.sum():
        rows = np.concatenate([np.arange(s, s + k) for s, k in zip(seg, rc) if k])
        base = np.repeat(seg, rc)
        res[base + out["index"][rows].astype(np.int64)] = out["result"][rows]
    return res


def _breaks(sm, P, C, in_span, res):
    """The all-gathered first failing member of every cross-shard chain."""
    v = in_span & (res != 0) & (res != LINKED_EVENT_FAILED)
    rows = np.zeros((0, 2), np.int64)
    if v.any():
        c, p = C[v], P[v]
        o = np.lexsort((p, c))
        c, p = c[o], p[o]
        first = np.ones(len(c), dtype=bool)
        first[1:] = c[1:] != c[:-1]
        rows = np.stack([c[first], p[first]], axis=1)
    allr, _ = gather_rows(sm.comm, rows)
    nb = {}
    for c, p in allr.tolist():
        nb[c] = min(nb.get(c, INF), p)
    return nb
