"""Ledger-sharded commit across GPUs: one process per GPU.

The reference has a single state machine that commits batches one at a time
(`StateMachine.commit`, src/state_machine.zig:894-928).  Here the state is
partitioned by ledger -- a valid transfer has `dr.ledger == cr.ledger ==
t.ledger` (:1280-1281) -- and each rank's engine owns the balances, stored
transfers and posted entries of its ledgers.  Results are those of the single
sequential state machine committing the step's batches in global order
(rank 0's batches, then rank 1's, ...), bit for bit; the tests check this
against one CPU oracle fed the same global sequence.

Per step (`create_transfers`):

1. Timestamps.  The batch counts are all-gathered; batch g of the global order
   gets T_g = T_{g-1} + 1 + n_g (the harness rule, src/state_machine.zig:1973)
   and event i of it T_g - n_g + i + 1 (execute, :1031).
2. Id directory.  The engines are the directory: a committed transfer is stored
   on the owner of its ledger, so "is id X committed, and where" is a lookup in
   every shard's id index (tbgpu_lookup_transfers).  The step's ids are
   all-gathered and resolved in global order: committed on shard O (EXISTS),
   first seen earlier in this step (DUP, with that event's route) or new.
   Pending ids resolve the same way to the shard holding (or creating) the
   pending.  (The device fast step below needs no directory at all when the
   step's ids rise above every id seen before -- the benchmark's sequential ids,
   and the key-range short-circuit of src/lsm/tree.zig:289-300.)
3. Routing.  Regular transfers go to owner(t.ledger); a transfer whose id is
   committed on O goes to O (it can only fail there, with `exists*` or an
   earlier code, so no balance moves); post/void goes to the pending's shard,
   with a colliding committed id imported there (tbgpu_import_transfers) for the
   `exists` comparison.  Events that fail state-independently stay with their
   chain.  create_accounts runs on every rank over every rank's batches, so the
   account directory (id -> ledger, what the checks of :1273-1281 read) is
   complete everywhere; with ledger-shard engines (tbgpu_options.shard_world)
   each rank stores the 128-byte rows of its own ledgers' accounts only, and the
   `exists*` comparison against another ledger's account (:1227-1237) comes from
   the rank that stores it (create_accounts below merges it).
4. Exchange.  Events travel to their owners with one all-to-all (RCCL over
   xGMI on GPUs, gloo in the CPU tests); each owner commits its sub-batches in
   global order with tbgpu_create_transfers_routed (per-event timestamps).
5. Chains spanning shards.  Each shard commits its part of such a chain as a
   chain of its own (TBGPU_CTL_CHAIN_END).  While any exist, rounds of dry runs
   find every part's first failure; the all-gathered minimum is the chain's
   break, after which members are skipped (TBGPU_CTL_SKIP) and parts that lie
   wholly before it are rolled back (TBGPU_CTL_DOOM).  The rounds stop
   when no break moves (a Jacobi fixed point over the step, as in the engine's
   own general path), then the step commits for real.
6. Hazards.  A duplicate id whose first occurrence (in another chain) routes
   to a shard that does not own the later event's ledger, or a post/void of a
   transfer created by a post/void in the same step, depends on an outcome on
   another shard: the step is split before the hazard's chain, the prefix
   commits, and the rest is routed again.
7. Replies go back to the source ranks with a second all-to-all;
   commit_timestamp is the max over shards and is propagated to every engine.

The backend of a rank is anything with the engine's commit API: the HIP
engine (`tigerbeetle_amd.engine.Engine`) on GPUs; the CPU tests use the
oracle per rank (test infrastructure) as the shard backend and a separate
oracle as the checker.
"""
from __future__ import annotations

from dataclasses import dataclass
from types import SimpleNamespace

import numpy as np

from .types import ACCOUNT_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE, TransferFlags

CTL_CHAIN_END = 1  # include/tbgpu.h TBGPU_CTL_CHAIN_END
CTL_SKIP = 2       # include/tbgpu.h TBGPU_CTL_SKIP
CTL_DOOM = 4       # include/tbgpu.h TBGPU_CTL_DOOM
LINKED_EVENT_FAILED = 1
SHARD_EXISTS_ELSEWHERE = 255  # include/tbgpu.h TBGPU_SHARD_ACCOUNT_EXISTS_ELSEWHERE
ACCOUNT_EXISTS_CODES = range(15, 22)  # CreateAccountResult exists_with_different_flags .. exists
LINKED = int(TransferFlags.linked)
POST_VOID = int(TransferFlags.post_pending_transfer | TransferFlags.void_pending_transfer)
ANY = -1           # route: state-independent failure, any shard computes it
PV = -2            # directory hint of a post/void: its shard is that of its pending
MAX_ROUNDS = 8     # dry rounds before the serial fallback (one cross-shard chain per round)
NB_GATHER = 2048   # batch counts per rank carried by the device step's first all-gather
LIMITS = 2 | 4     # AccountFlags debits_must_not_exceed_credits | credits_must_not_exceed_debits
BALANCING = 8 | 16  # TransferFlags balancing_debit | balancing_credit
# The 8-byte record of a routed event (include/tbgpu.h TBGPU_ROUTE_REC_*):
# global batch << 32 | chain start << 15 | ends its chain << 14 | chain spans owners << 13 | index
REC_POS = 0x1FFF
REC_SPAN = 1 << 13
REC_LAST = 1 << 14
REC_CS_SHIFT = 15
REC_CS_MASK = 0x1FFF


def rec_position(rec):
    """global batch << 32 | index in the batch (the event's place in the global order)"""
    return ((rec >> 32) << 32) | (rec & REC_POS)


def rec_chain_key(rec):
    """global batch << 32 | index of the chain's first member"""
    return ((rec >> 32) << 32) | ((rec >> REC_CS_SHIFT) & REC_CS_MASK)

# directory replies
NEW, EXISTS, DUP, PEND, PEND_NONE, PEND_HAZARD = range(6)


def _id(lo, hi) -> int:
    return (int(hi) << 64) | int(lo)


_NO_REPLIES = np.zeros(0, dtype=RESULT_DTYPE)  # a batch without replies (shared, read-only)
_NO_REPLIES.setflags(write=False)


class Comm:
    """The collectives the router needs, over a torch.distributed group (gloo on
    CPU, nccl = RCCL on GPU: tensors then live on the rank's device)."""

    def __init__(self, rank: int, world: int, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.rank, self.world, self.group = rank, world, group
        self.device = device if device is not None else torch.device("cpu")

    def all_gather_object(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def alltoallv(self, parts: list[np.ndarray]) -> list[np.ndarray]:
        """parts[d]: bytes (uint8 array) for rank d.  Returns the parts received, by source."""
        torch = self.torch
        sizes = torch.tensor([len(p) for p in parts], dtype=torch.int64, device=self.device)
        rsizes = torch.empty_like(sizes)
        self.dist.all_to_all_single(rsizes, sizes, group=self.group)
        rs = rsizes.cpu().tolist()
        src = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        inp = torch.from_numpy(np.ascontiguousarray(src, dtype=np.uint8)).to(self.device)
        out = torch.empty(sum(rs), dtype=torch.uint8, device=self.device)
        self.dist.all_to_all_single(out, inp, rs, [len(p) for p in parts], group=self.group)
        o = out.cpu().numpy()
        res, off = [], 0
        for n in rs:
            res.append(o[off:off + n])
            off += n
        return res

    def allreduce_max(self, v: int) -> int:
        return max(self.all_gather_object(int(v)))


@dataclass
class _Event:
    """Routing view of one event of the step (global order = index in the step)."""
    src: int        # source rank
    batch: int      # source rank's batch index
    index: int      # index in that batch
    g: int          # global batch number within the step


class ShardedStateMachine:
    """create_accounts / create_transfers for one rank of a ledger-sharded node."""

    def __init__(self, backend, comm: Comm, owner_of_ledger=None):
        self.backend = backend
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world
        self._ledger_mod = owner_of_ledger is None
        self.owner_of_ledger = owner_of_ledger or (lambda ledger: int(ledger) % self.world)
        # the general step's rounds over whole arrays (shard_vec.round_vec); False: the
        # event-by-event reference form (_round), kept for the tests
        self.vectorized = True
        self.prepare_timestamp = 0
        self.commit_timestamp = 0
        self.max_id = 0         # every transfer id seen so far is <= this (the fast step's id filter)
        self.max_rounds = MAX_ROUNDS
        # events of the general step's round window (shard_vec.window_cut); 0: the whole step
        self.round_window = 4096
        # True: the general step's rounds stop each shard at its own first waiting event
        # (shard_vec.ShardStops); False: one stop for all, at the first hazard.  Off by
        # default: on the flag-heavy mix it saves 8-10 % of the rounds and costs more in
        # its gather and solve (profiles/r05/general_rehearsal.txt)
        self.shard_stops = False
        self.limit_ids: set[int] = set()  # ids of accounts created with a balance limit flag
        self.amount_bound = 0.0  # >= the sum of every transfer amount routed: bounds every balance
        self.timed = False       # accumulate per-phase wall times of the device step (with syncs)
        self.wire_bytes_per_event = 0  # the last device step's all-to-all bytes per event
        self._worker = None       # the pipelined stream's commit thread
        self.timing = {"eligibility_ms": 0.0, "order_ms": 0.0, "partition_ms": 0.0, "exchange_ms": 0.0,
                       "commit_ms": 0.0, "replies_ms": 0.0}
        self.gtiming = {}         # the general step's phases (shard_vec.round_vec), when timed
        self.stats = {"steps": 0, "splits": 0, "dry_rounds": 0, "cross_chains": 0, "imports": 0,
                      "preruns": 0, "serial_fallbacks": 0, "device_fallbacks": 0}

    def owners_vec(self, ledgers) -> np.ndarray:
        """owner_of_ledger over an array of ledgers."""
        led = np.asarray(ledgers).astype(np.int64)
        if self._ledger_mod:
            return led % self.world
        return np.array([self.owner_of_ledger(int(x)) for x in led.tolist()], dtype=np.int64)

    def note_accounts(self, accounts: np.ndarray) -> None:
        """Record the balance-limited accounts among `accounts` (every rank sees every
        account batch).  A plain transfer between accounts without limit flags has an
        outcome that no other transfer can change (src/state_machine.zig:1273-1346:
        only the limit and overflow checks read balances), which lets the device step
        settle cross-shard chains with one dry run of their members alone."""
        a = np.asarray(accounts)
        lim = (a["flags"] & LIMITS) != 0
        for lo, hi in zip(a["id_lo"][lim].tolist(), a["id_hi"][lim].tolist()):
            self.limit_ids.add((int(hi) << 64) | int(lo))

    def adopt_accounts(self, accounts: np.ndarray, prepare_timestamp: int) -> None:
        """Accounts every rank created itself (the same batches and timestamps on every
        engine, as create_accounts would have replicated them): bring the router up."""
        self.note_accounts(accounts)
        self.prepare_timestamp = int(prepare_timestamp)
        self._sync_commit_timestamp()

    # ------------------------------------------------------------ accounts --
    def create_accounts(self, batches: list[np.ndarray]) -> list[np.ndarray]:
        """Every rank commits every rank's account batches (replicated accounts):
        the account checks of create_transfer are then exact on any shard."""
        allb = self.comm.all_gather_object([np.ascontiguousarray(b, ACCOUNT_DTYPE).tobytes() for b in batches])
        flat, counts, ts, owner = [], [], [], []
        for r, bl in enumerate(allb):
            for j, raw in enumerate(bl):
                ev = np.frombuffer(raw, dtype=ACCOUNT_DTYPE)
                self.prepare_timestamp += 1 + len(ev)
                flat.append(ev)
                counts.append(len(ev))
                ts.append(self.prepare_timestamp)
                owner.append((r, j))
        if not counts:
            return []
        events = np.concatenate(flat) if flat else np.zeros(0, ACCOUNT_DTYPE)
        self.note_accounts(events)
        out, rc = self.backend.create_accounts_batches(np.array(ts, np.uint64), np.array(counts, np.uint32),
                                                       events)
        self._sync_commit_timestamp()
        per = []  # per global batch: its replies
        off = 0
        for c, k in zip(counts, rc):
            per.append(out[off:off + int(k)].copy())
            off += c
        if getattr(self.backend, "shard_world", 0) >= 2:
            self._merge_elsewhere(per)
        return [per[g] for g, (r, _) in enumerate(owner) if r == self.rank]

    def _merge_elsewhere(self, per: list[np.ndarray]) -> None:
        """Ledger-shard engines: an event whose id names an account created before the
        call on another shard's ledger gets TBGPU_SHARD_ACCOUNT_EXISTS_ELSEWHERE on every
        rank but that account's owner, whose engine compared the row
        (create_account_exists, src/state_machine.zig:1227-1237).  Every rank fails the
        same events (any `exists*` is a failure, so chains break alike); the owner's
        code replaces the placeholder (one all-gather of the `exists*` replies)."""
        mine = {}
        for g, r in enumerate(per):
            for ix, code in zip(r["index"].tolist(), r["result"].tolist()):
                if code in ACCOUNT_EXISTS_CODES:
                    mine[(g, ix)] = code
        exact = {}
        for d in self.comm.all_gather_object(mine):
            exact.update(d)
        for g, r in enumerate(per):
            hole = r["result"] == SHARD_EXISTS_ELSEWHERE
            if hole.any():
                for k in np.nonzero(hole)[0].tolist():
                    key = (g, int(r["index"][k]))
                    if key not in exact:
                        raise AssertionError(f"create_accounts: no shard compared the existing account of {key}")
                    r["result"][k] = exact[key]

    # ----------------------------------------------------------- transfers --
    def create_transfers(self, batches: list[np.ndarray]) -> list[np.ndarray]:
        """One routed step over this rank's batches; returns this rank's replies."""
        batches = [np.ascontiguousarray(b, TRANSFER_DTYPE) for b in batches]
        amt = sum(float(b["amount_lo"].astype(np.float64).sum()) + float(b["amount_hi"].astype(np.float64).sum()) * 2.0**64
                  for b in batches)
        gathered = self.comm.all_gather_object(([len(b) for b in batches], amt))
        counts_all = [c for c, _ in gathered]
        self.amount_bound += sum(a for _, a in gathered) * (1 + 1e-9) + 1
        # global order and timestamps (identical on every rank)
        glob = [(r, j, c) for r, cl in enumerate(counts_all) for j, c in enumerate(cl)]
        T = []
        for r, j, c in glob:
            self.prepare_timestamp += 1 + c
            T.append(self.prepare_timestamp)
        gidx = {(r, j): g for g, (r, j, c) in enumerate(glob)}
        # the step's events in global order, addressed by (g, index)
        my_events = {gidx[(self.rank, j)]: b for j, b in enumerate(batches)}
        replies = {g: [] for g in my_events}
        start = (0, 0)  # resume point (global batch, index) after a hazard split
        done = {g: np.zeros(len(b), dtype=bool) for g, b in my_events.items()}  # committed in a round
        while True:
            self.stats["steps"] += 1
            if self.vectorized:
                from .shard_vec import round_vec
                split = round_vec(self, glob, T, my_events, replies, start, done)
            else:
                split = self._round(glob, T, my_events, replies, start)
            if split is None:
                break
            self.stats["splits"] += 1
            start = split
        self._sync_commit_timestamp()
        out = []
        for j in range(len(batches)):
            r = replies[gidx[(self.rank, j)]]
            a = np.array(sorted(r), dtype=np.uint32).reshape(-1, 2)
            res = np.zeros(len(a), dtype=RESULT_DTYPE)
            if len(a):
                res["index"], res["result"] = a[:, 0], a[:, 1]
            out.append(res)
        return out

    # ------------------------------------------------------ device step --
    def create_transfers_device(self, events, counts):
        """One routed step with the events already in device memory: `events` is a
        uint8 tensor of n*128 bytes on this rank's device, `counts` its batch sizes.
        Returns this rank's replies (one RESULT_DTYPE array per batch).

        Fast when the step has no post/void and its ids rise strictly along the
        global order above every id seen before (no directory lookup can hit);
        routing, partition and exchange then stay on the device: owner = ledger
        % world, a stable partition by owner, RCCL all-to-all of the events and of
        8-byte records {(batch, index), chain start, span / end bits} (REC_*), and the
        owner's tbgpu_create_transfers_routed_device.  Chains that span shards are
        settled before the commit: when every member is a plain transfer between
        accounts without balance limits (its outcome then depends on no other
        transfer: src/state_machine.zig:1273-1346), one dry run of the members alone
        gives every part's first failure; otherwise dry rounds over the whole step
        run to their fixed point, and past `max_rounds` the step goes to the exact
        router (create_transfers), which settles one cross-shard chain at a time.
        Anything else goes through create_transfers too."""
        if self._single_rank(events):
            return self._single_rank_step(events, counts)
        st = self.route_device(events, counts)
        if st.fallback:
            return self._host_step(st.ev, st.counts, st.offs_h)
        self.exchange_device(st)
        self.commit_routed(st)
        return self.finish_routed(st)

    def create_transfers_device_stream(self, steps):
        """create_transfers_device over consecutive steps ((events, counts) pairs),
        pipelined: step k + 1 is routed (eligibility, scatter: HBM-bound) before step
        k's owner commit starts, and its all-to-all (xGMI-bound) runs while that commit
        runs on a worker thread.  Yields each step's replies, equal to
        create_transfers_device's (the results do not depend on the overlap)."""
        it = iter(steps)
        nxt = next(it, None)
        if nxt is not None and self._single_rank(nxt[0]):
            # one rank: nothing to exchange, so nothing to overlap
            while nxt is not None:
                yield self._single_rank_step(*nxt)
                nxt = next(it, None)
            return
        st = self.route_device(*nxt) if nxt is not None else None
        if st is not None and not st.fallback:
            self.exchange_device(st)
        while st is not None:
            if st.fallback:
                yield self._host_step(st.ev, st.counts, st.offs_h)
                nxt = next(it, None)
                st = self.route_device(*nxt) if nxt is not None else None
                if st is not None and not st.fallback:
                    self.exchange_device(st)
                continue
            # step k's cross-shard settle (dry rounds, or its fallback to the exact
            # router) decides before step k + 1 is routed: routing moves the router's
            # state (prepare_timestamp, max_id, amount_bound) that a fallback of step
            # k restores and then advances by step k alone
            self.commit_routed(st, background=True)
            nxt = next(it, None)
            st2 = self.route_device(*nxt) if nxt is not None else None
            if st2 is not None and not st2.fallback:
                self.exchange_device(st2)
            yield self.finish_routed(st)
            st = st2

    def _single_rank(self, events) -> bool:
        """One rank owns every ledger: the step is the engine's own streamed call."""
        return self.world == 1 and getattr(events, "is_cuda", False) and \
            hasattr(self.backend, "create_transfers_batches_device")

    def _single_rank_step(self, events, counts):
        """A one-rank group owns every ledger, so routing is the identity: the step is
        one tbgpu_create_transfers_batches_device call over the rank's batches in
        their order (the same global order, the same timestamps T_g - n_g + i + 1;
        the engine is the whole state machine, so repeated or non-monotone ids and
        post/void need no directory either).  Returns this rank's replies."""
        torch = self.comm.torch
        clock = self._clock()
        cnt = np.asarray(list(map(int, counts)), dtype=np.int64)
        n = int(cnt.sum())
        T = self.prepare_timestamp + np.cumsum(cnt + 1)
        if len(T):
            self.prepare_timestamp = int(T[-1])
        ev = events.view(torch.uint8).reshape(-1)[:n * 128]
        res = torch.empty(max(n, 1) * 8, dtype=torch.uint8, device=ev.device)
        torch.cuda.current_stream(ev.device).synchronize()  # the engine runs on its own stream
        clock("order_ms")
        total, rc = self.backend.create_transfers_batches_device(T.astype(np.uint64), cnt.astype(np.uint32),
                                                                 ev.data_ptr(), res.data_ptr())
        clock("commit_ms")
        out = res[:int(total) * 8].cpu().numpy().view(RESULT_DTYPE) if total else np.zeros(0, RESULT_DTYPE)
        replies, off = [], 0
        for k in rc.tolist():
            replies.append(out[off:off + k].copy() if k else _NO_REPLIES)
            off += k
        # (max_id, the multi-rank device step's id filter, is never read on one rank)
        self.commit_timestamp = self.backend.commit_timestamp()
        self.stats["steps"] += 1
        clock("replies_ms")
        return replies

    def _host_step(self, ev, counts, offs_h):
        host = ev.cpu().numpy().view(TRANSFER_DTYPE)
        return self.create_transfers([host[offs_h[j]:offs_h[j + 1]] for j in range(len(counts))])

    def route_device(self, events, counts):
        """Phase 1 of a device step: eligibility, global order, scatter to the owners,
        exchange, and what the owner side needs to settle cross-shard chains.  Returns
        a step record; `fallback` set (and nothing changed) when the step must go
        through the exact host router."""
        clock = self._clock()
        import math
        torch = self.comm.torch
        dev = self.comm.device
        W, me = self.world, self.rank
        clock = self._clock()
        n = int(sum(counts))
        ev = events.view(torch.uint8).reshape(-1)[:n * 128]
        w32 = ev.view(torch.int32).view(n, 32)
        w64 = ev.view(torch.int64).view(n, 16)
        id_lo, id_hi = w64[:, 0], w64[:, 1]
        # eligibility, one small all-gather: [n, min id, max id, monotone, plain, amount bound in 2^32 units]
        native = n and ev.is_cuda and hasattr(self.backend, "route_scatter")
        # this rank can send and receive the packed wire format (csrc/route.hip)
        can_pack = W > 1 and ev.is_cuda and hasattr(self.backend, "route_scatter_packed")
        wmask = 0xFFFFFFFF
        if n and ev.is_cuda and hasattr(self.backend, "route_stats"):
            # one pass of the engine's kernel (csrc/route.hip) instead of the torch reductions;
            # the same pass ranks the events for the scatter below and finds their nonzero words
            mn, mx, mono, ids_ok, pv, big, asum, wmask = self.backend.route_stats(ev, n, world=W if native else 0,
                                                                                 word_mask=True)
            ok_ids = ids_ok and mx < (1 << 63)  # the all-gather below carries int64
            units = (1 << 62) if big else (asum >> 32) + 2
            st = [n, mn if ok_ids else 0, mx if ok_ids else 0, int(mono), int(ok_ids and not pv), units]
        elif n:
            mono = bool((id_lo[1:] > id_lo[:-1]).all()) if n > 1 else True
            flags = (w32[:, 29] >> 16) & 0xFFFF
            plain = bool(((flags & POST_VOID) == 0).all() & (id_hi == 0).all() & (id_lo > 0).all())
            a = w64[:, 6].double()
            a = torch.where(a < 0, a + 2.0**64, a)
            big = bool((w64[:, 7] != 0).any())
            units = (1 << 62) if big else int(math.ceil(float(a.sum()) * (1 + 1e-9) / 2.0**32)) + 1
            st = [n, int(id_lo.min()), int(id_lo.max()), int(mono), int(plain), units]
        else:
            st = [0, 0, 0, 1, 1, 0]
        # the packed format's words and capability, then the batch counts of the step
        # (the global order), in the same all-gather
        st += [(wmask if n else 0) | (int(can_pack) << 32)]
        nb_here = len(counts)
        sta = np.zeros(8 + NB_GATHER, dtype=np.int64)
        sta[:7] = st
        sta[7] = nb_here
        if nb_here <= NB_GATHER:
            sta[8:8 + nb_here] = np.asarray(counts, dtype=np.int64)
        if W > 1:
            stats = torch.from_numpy(sta).to(dev)
            allst = [torch.empty_like(stats) for _ in range(W)]
            self.comm.dist.all_gather(allst, stats, group=self.comm.group)
            allst = torch.stack(allst).cpu().numpy()
        else:  # one rank: nothing to gather
            allst = sta[None, :]
        ok, prev = True, self.max_id
        for (cnt, lo, hi, mono, plain, _) in (x[:6].tolist() for x in allst):
            if cnt == 0:
                continue
            ok &= bool(mono and plain and lo > prev)
            prev = hi
        offs_h = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        if not ok:
            return SimpleNamespace(fallback=True, ev=ev, counts=counts, offs_h=offs_h)
        clock("eligibility_ms")
        saved = (self.prepare_timestamp, self.max_id, self.amount_bound)
        self.max_id = max(self.max_id, prev)
        self.amount_bound += sum(float(x[5]) for x in allst) * 2.0**32

        # global order and timestamps (host: one entry per batch)
        # every rank packs when every rank can: the union of the nonzero words travels
        packed = W > 1 and all(int(x[6]) >> 32 for x in allst)
        pmask = 0
        for x in allst:
            pmask |= int(x[6]) & 0xFFFFFFFF
        pmask = pmask or 1
        K = bin(pmask).count("1") + 1  # 4-byte words per packed row: the masked words, the record
        if all(int(x[7]) <= NB_GATHER for x in allst):
            counts_all = [x[8:8 + int(x[7])] for x in allst]
        else:
            counts_all = self.comm.all_gather_object(list(map(int, counts)))
        # the global order as arrays (one entry per batch of every rank: 8000 at N = 8,
        # so no per-batch Python): each batch's size, source rank and prepare timestamp
        nbs = [len(cl) for cl in counts_all]
        gcount = np.concatenate([np.asarray(cl, np.int64) for cl in counts_all]) if sum(nbs) else \
            np.zeros(0, np.int64)
        grank = np.repeat(np.arange(W, dtype=np.int64), nbs)
        T = self.prepare_timestamp + np.cumsum(gcount + 1)
        if len(T):
            self.prepare_timestamp = int(T[-1])
        g0 = sum(nbs[:me])
        clock("order_ms")
        nb_me = len(counts)
        send = None
        if packed:
            # the engine's scatter straight into the packed wire format (csrc/route.hip)
            send = torch.empty((n, K), dtype=torch.int32, device=dev)
            if n:
                sc, bc, spc = self.backend.route_scatter_packed(W, list(map(int, counts)), g0, ev, pmask, send)
            else:
                sc, bc, spc = np.zeros(W, np.int64), np.zeros((W, 0), np.int64), np.zeros(W, np.int64)
            ev_s = side_s = None
        elif native:
            # the engine's scatter kernels (csrc/route.hip): same layout as partition_torch
            ev_s = torch.empty((n, 128), dtype=torch.uint8, device=dev)
            side_s = torch.empty(n, dtype=torch.int64, device=dev)
            sc, bc, spc = self.backend.route_scatter(W, list(map(int, counts)), T[g0:g0 + nb_me], g0, ev, ev_s,
                                                     side_s, detail=True)
        elif n:
            ev_s, side_s, send_t, bc_t, spc_t = partition_torch(torch, ev, counts, T[g0:g0 + nb_me], g0, W, dev,
                                                                detail=True)
            sc, bc, spc = send_t.cpu().numpy(), bc_t.cpu().numpy(), spc_t.cpu().numpy()
        else:
            sc, bc, spc = np.zeros(W, np.int64), np.zeros((W, 0), np.int64), np.zeros(W, np.int64)
            ev_s = torch.zeros((0, 128), dtype=torch.uint8, device=dev)
            side_s = torch.zeros(0, dtype=torch.int64, device=dev)
        clock("partition_ms")
        # per owner: [events, spanning events, all spanning events sent, events per batch...]
        meta = np.concatenate([np.asarray(sc, np.int64)[:, None], np.asarray(spc, np.int64)[:, None],
                               np.full((W, 1), int(np.sum(spc)), np.int64), np.asarray(bc, np.int64)], axis=1)
        if W > 1:
            rmeta = torch.empty(sum(3 + k for k in nbs), dtype=torch.int64, device=dev)
            self.comm.dist.all_to_all_single(rmeta, torch.from_numpy(meta.reshape(-1)).to(dev), [3 + k for k in nbs],
                                             [3 + nb_me] * W, group=self.comm.group)
            rmeta = rmeta.cpu().numpy()
        else:
            rmeta = meta.reshape(-1)
        sl, rl, sub_counts, sub_g, n_span, span_sent = [int(x) for x in sc], [], [], [], 0, 0
        off = gb = 0
        for k in nbs:
            row = rmeta[off:off + 3 + k]
            rl.append(int(row[0]))
            n_span += int(row[1])
            span_sent += int(row[2])
            nz = np.nonzero(row[3:])[0]
            sub_counts += row[3:][nz].tolist()
            sub_g += (nz + gb).tolist()
            off += 3 + k
            gb += k
        m = int(sum(rl))
        clock("exchange_ms")
        # phase 1b (exchange_device) moves the events: the all-to-all over xGMI, which a
        # pipelined stream overlaps with the previous step's owner commit
        return SimpleNamespace(**{k: v for k, v in locals().items() if k not in ("self", "clock")},
                               fallback=False)

    def exchange_device(self, st):
        """Phase 1b of a device step: the all-to-all of the events (packed wire format
        when every rank runs the engine's kernels), the owner-side unpack (rows,
        records, timestamps), and what the owner needs to settle cross-shard chains."""
        torch = self.comm.torch
        clock = self._clock()
        g = st.__dict__
        dev, W, m, T, gcount, packed, K, pmask = (g[x] for x in ("dev", "W", "m", "T", "gcount", "packed", "K",
                                                                 "pmask"))
        rl, sl, sub_counts, sub_g, n_span, span_sent = (g[x] for x in ("rl", "sl", "sub_counts", "sub_g", "n_span",
                                                                       "span_sent"))
        send, ev_s, side_s = g.pop("send"), g.pop("ev_s"), g.pop("side_s")
        self.wire_bytes_per_event = 4 * K if packed else 128 + 8  # what the all-to-all moves per event
        # the received events' timestamps: T - n + index + 1 of their global batch
        tsb = torch.from_numpy(T - gcount).to(dev)
        ts_r = None
        if packed:
            recv = torch.empty((m, K), dtype=torch.int32, device=dev)
            self.comm.dist.all_to_all_single(recv, send, rl, sl, group=self.comm.group)
            send = None
            R = torch.empty((m, 128), dtype=torch.uint8, device=dev)
            S = torch.empty(m, dtype=torch.int64, device=dev)
            ts_r = torch.empty(m, dtype=torch.int64, device=dev)
            if m:
                # each row's global batch: the owner's sub-batches arrive in global order
                sub = torch.tensor(np.concatenate([[0], np.cumsum(sub_counts), sub_g]).astype(np.int32), device=dev)
                ns = len(sub_counts)
                self.backend.route_unpack_packed(recv, pmask, sub[:ns + 1], sub[ns + 1:], tsb, R, S, ts_r)
            del recv
        elif W > 1:
            R = torch.empty((m, 128), dtype=torch.uint8, device=dev)
            S = torch.empty(m, dtype=torch.int64, device=dev)
            self.comm.dist.all_to_all_single(R, ev_s, rl, sl, group=self.comm.group)
            self.comm.dist.all_to_all_single(S, side_s, rl, sl, group=self.comm.group)
        else:  # one owner: the send buffers are what it receives
            R, S = ev_s, side_s
        ev_s = side_s = None
        clock("exchange_ms")

        # owner side: sub-batches in global order (from the senders' counts), chain control
        si = torch.zeros(0, dtype=torch.int64, device=dev)
        if n_span:
            gk = S >> 32
            key = rec_chain_key(S)
            spanm = (S & REC_SPAN) != 0
            lastm = (S & REC_LAST) != 0
            nxt = torch.ones(m, dtype=torch.bool, device=dev)
            nxt[:-1] = key[1:] != key[:-1]                 # last local member of its chain
            base = (spanm & nxt & ~lastm).to(torch.uint8) * CTL_CHAIN_END
            si = torch.nonzero(spanm).flatten()
            assert int(si.numel()) == n_span, "spanning counts disagree with the received records"
        plain_local = True
        if n_span:
            Rs = R.index_select(0, si)
            f32 = Rs.view(torch.int32).view(n_span, 32)
            f64 = Rs.view(torch.int64).view(n_span, 16)
            sf = (f32[:, 29] >> 16) & 0xFFFF
            plain_local = bool((((sf & (BALANCING | POST_VOID)) == 0) & (f64[:, 7] == 0)).all())
            if plain_local and self.limit_ids:
                acc = f64[:, 2:6].cpu().numpy().astype(np.uint64)
                for lo, hi in ((acc[:, 0], acc[:, 1]), (acc[:, 2], acc[:, 3])):
                    if any(((int(h) << 64) | int(lo_)) in self.limit_ids for lo_, h in zip(lo.tolist(), hi.tolist())):
                        plain_local = False
                        break
        # every rank knows whether anything spans (the senders' totals came with the counts)
        any_span = span_sent > 0
        all_plain = True
        if any_span:
            all_plain = all(self.comm.all_gather_object(plain_local)) and self.amount_bound < 2.0**125
        g.update({k: v for k, v in locals().items() if k not in ("self", "clock", "g", "st", "torch")})
        return st

    def commit_routed(self, st, background: bool = False):
        """Phase 2: settle the step's cross-shard chains (collectives, on this thread),
        then the owner commit -- on a worker thread when `background`, so that the next
        step's routing (phase 1) overlaps it.  Sets st.out / st.at / st.cts (or, after a
        device fallback, st.replies)."""
        torch = self.comm.torch
        clock = self._clock()
        g = st.__dict__
        dev, m, R, S, si, n_span = g["dev"], g["m"], g["R"], g["S"], g["si"], g["n_span"]
        sub_counts, any_span, all_plain = g["sub_counts"], g["any_span"], g["all_plain"]
        key, nxt, lastm, base, gk = (g.get(x) for x in ("key", "nxt", "lastm", "base", "gk"))
        st.replies = None
        st.thread = None
        results = torch.empty(max(m, 1) * 8, dtype=torch.uint8, device=dev)
        if not m:
            ts_r = torch.zeros(1, dtype=torch.int64, device=dev)
        elif g.get("ts_r") is not None:  # unpacked with the events (packed wire format)
            ts_r = g["ts_r"]
        elif S.is_cuda and hasattr(self.backend, "route_unpack"):
            ts_r = torch.empty(m, dtype=torch.int64, device=dev)
            self.backend.route_unpack(S, g["tsb"], ts_r)
        else:
            ts_r = g["tsb"][S >> 32] + (S & REC_POS) + 1
        Rf = R.reshape(-1) if m else torch.zeros(128, dtype=torch.uint8, device=dev)
        offs = np.concatenate([[0], np.cumsum(sub_counts)]).astype(np.int64)
        si_np = si.cpu().numpy()

        def commit(ctl, dry, sel=None):
            if not m or (sel is not None and not len(si_np)):
                return np.zeros(0, dtype=RESULT_DTYPE), np.zeros(0, dtype=np.int64), 0
            if sel is None:
                cnts, rx, tx, cx, ox = sub_counts, Rf, ts_r, ctl, offs
            else:
                _, c = torch.unique_consecutive(gk.index_select(0, sel), return_counts=True)
                cnts = c.cpu().tolist()
                rx = R.index_select(0, sel).reshape(-1)
                tx = ts_r.index_select(0, sel)
                cx = None if ctl is None else ctl.index_select(0, sel)
                ox = np.concatenate([[0], np.cumsum(cnts)]).astype(np.int64)
            rc, cts = self.backend.create_transfers_routed_tensors(cnts, rx, tx, cx, dry, results)
            return decode(rc, cts, ox, sel)

        def decode(rc, cts, ox, sel=None):
            tot = int(np.sum(rc))
            out = results[:tot * 8].cpu().numpy().view(RESULT_DTYPE).copy() if tot else np.zeros(0, RESULT_DTYPE)
            at = np.repeat(ox[:-1], rc.astype(np.int64)) + out["index"].astype(np.int64) if tot else \
                np.zeros(0, np.int64)
            if sel is not None and tot:
                at = si_np[at]
            return out, at, cts

        if any_span:
            span_key = key.index_select(0, si).cpu().numpy() if n_span else np.zeros(0, np.int64)
            span_pos = rec_position(S[si]).cpu().numpy() if n_span else np.zeros(0, np.int64)
            span_base = base.index_select(0, si).cpu().numpy() if n_span else np.zeros(0, np.uint8)
            span_last = (nxt[si] & ~lastm[si]).cpu().numpy() if n_span else np.zeros(0, bool)
            where = np.full(max(m, 1), -1, dtype=np.int64)
            where[si_np] = np.arange(n_span)

            def control(brk):
                c = span_base.copy()
                if brk and n_span:
                    bk = np.array(sorted(brk), dtype=np.int64)
                    bv = np.array([brk[k] for k in bk.tolist()], dtype=np.int64)
                    ix = np.minimum(np.searchsorted(bk, span_key), len(bk) - 1)
                    has = bk[ix] == span_key
                    b = bv[ix]
                    c[has & (span_pos > b)] |= CTL_SKIP
                    c[has & span_last & (span_pos < b)] |= CTL_DOOM
                ctl = torch.zeros(max(m, 1), dtype=torch.uint8, device=dev)
                if n_span:
                    ctl[si] = torch.from_numpy(c).to(dev)
                return ctl

            def breaks(out, at):
                """The all-gathered first failing member of every cross-shard chain."""
                fails = {}
                if len(at):
                    q = where[at]
                    r = out["result"].astype(np.int64)
                    v = (q >= 0) & (r != 0) & (r != LINKED_EVENT_FAILED)
                    if v.any():
                        k, p = span_key[q[v]], span_pos[q[v]]
                        o = np.lexsort((p, k))
                        k, p = k[o], p[o]
                        first = np.concatenate([[True], k[1:] != k[:-1]])
                        fails = dict(zip(k[first].tolist(), p[first].tolist()))
                nb_ = {}
                for d in self.comm.all_gather_object(fails):
                    for k, p in d.items():
                        nb_[k] = min(nb_.get(k, 1 << 62), p)
                return nb_

            if all_plain:
                # every member's outcome is independent of the other transfers: one dry
                # run of the cross-shard members alone finds every chain's break
                self.stats["preruns"] += 1
                d_out, d_at, _ = commit(control({}), True, sel=si)
                final_ctl = control(breaks(d_out, d_at))
            else:
                brk = {}
                for _ in range(self.max_rounds):
                    self.stats["dry_rounds"] += 1
                    ctl = control(brk)
                    out, at, cts = commit(ctl, True)
                    nb_ = breaks(out, at)
                    if nb_ == brk:
                        out2, at2, cts = commit(ctl, False)
                        # the commit is exact as long as it breaks every spanning chain where
                        # its control said (decided collectively: every rank alike)
                        if self.comm.allreduce_max(int(out2.tobytes() != out.tobytes())):
                            self.stats["dry_commit_mismatch"] = self.stats.get("dry_commit_mismatch", 0) + 1
                            if breaks(out2, at2) != brk:
                                raise AssertionError("sharded commit: a committed chain broke elsewhere than its "
                                                     "dry run (engine invariant)")
                        st.out, st.at, st.cts = out2, at2, cts
                        clock("commit_ms")
                        return st
                    brk = nb_
                else:
                    # no fixed point within max_rounds: nothing was committed; the exact
                    # router settles the step one cross-shard chain at a time
                    self.stats["device_fallbacks"] += 1
                    self.prepare_timestamp, self.max_id, self.amount_bound = g["saved"]
                    st.replies = self._host_step(g["ev"], g["counts"], g["offs_h"])
                    return st
        else:
            final_ctl = None
        if background and m:
            # the real commit on a worker thread; its results are read by finish_routed
            if R.is_cuda:
                torch.cuda.current_stream(R.device).synchronize()
            box = {}

            def run():
                try:
                    box["rc"] = self.backend.create_transfers_routed_tensors(
                        sub_counts, Rf, ts_r, final_ctl, False, results, sync_inputs=False)
                except BaseException as e:  # noqa: BLE001 -- re-raised by finish_routed
                    box["error"] = e
            # one long-lived worker: a fresh OS thread per step paid the HIP runtime's
            # per-thread setup on every commit
            if self._worker is None:
                from concurrent.futures import ThreadPoolExecutor
                self._worker = ThreadPoolExecutor(max_workers=1, thread_name_prefix="tb-commit")
            st.thread = self._worker.submit(run)
            st.box, st.decode, st.offs = box, decode, offs
            return st
        out, at, cts = commit(final_ctl, False)
        st.out, st.at, st.cts = out, at, cts
        clock("commit_ms")
        return st

    def finish_routed(self, st):
        """Phase 3: the owner commit's results, the node's commit timestamp, replies back
        to their sources.  Returns this rank's replies."""
        torch = self.comm.torch
        clock = self._clock()
        if st.replies is not None:
            return st.replies
        if st.thread is not None:
            st.thread.result()
            if "error" in st.box:
                raise st.box["error"]
            rc, cts = st.box["rc"]
            st.out, st.at, st.cts = st.decode(rc, cts, st.offs)
            st.thread = None
        g = st.__dict__
        dev, W, m, S, grank, g0, counts = g["dev"], g["W"], g["m"], g["S"], g["grank"], g["g0"], g["counts"]
        out, at, cts = st.out, st.at, st.cts
        # the node's commit timestamp and whether any owner has replies, in one all-gather
        fin = [len(at), int(cts) if m else self.backend.commit_timestamp()]
        fin_own = fin[1]
        if W > 1:
            fin = torch.tensor(fin, dtype=torch.int64, device=dev)
            allfin = [torch.empty_like(fin) for _ in range(W)]
            self.comm.dist.all_gather(allfin, fin, group=self.comm.group)
            allfin = torch.stack(allfin).cpu().tolist()
        else:
            allfin = [fin]
        ts_all = max(x[1] for x in allfin)
        mine = {}
        if any(x[0] for x in allfin):
            # replies to their sources
            if len(at):
                pg = rec_position(S[torch.from_numpy(at).to(dev)]).cpu().numpy()
            else:
                pg = np.zeros(0, np.int64)
            rep = [[] for _ in range(W)]
            for pgv, r in zip(pg.tolist(), out["result"].tolist()):
                gg = pgv >> 32
                rep[int(grank[gg])].append((gg, pgv & 0xFFFFFFFF, r))
            for lst in self._exchange_objects(rep):
                for (gg, i, r) in lst:
                    mine.setdefault(gg - g0, []).append((i, r))
        if ts_all > fin_own:
            self.backend.advance_commit_timestamp(ts_all)
        self.commit_timestamp = ts_all
        replies = []
        for j in range(len(counts)):
            if j not in mine:
                replies.append(_NO_REPLIES)
                continue
            a = np.array(sorted(mine[j]), dtype=np.uint32).reshape(-1, 2)
            res = np.zeros(len(a), dtype=RESULT_DTYPE)
            res["index"], res["result"] = a[:, 0], a[:, 1]
            replies.append(res)
        self.stats["steps"] += 1
        clock("replies_ms")
        return replies

    def _clock(self):
        """Per-phase wall time of the device step into self.timing when self.timed
        (each mark waits for the device, so phases do not overlap)."""
        import time
        if not self.timed:
            return lambda name: None
        torch = self.comm.torch
        sync = (lambda: torch.cuda.synchronize(self.comm.device)) if self.comm.device.type == "cuda" else (lambda: None)
        sync()
        t = [time.perf_counter()]

        def mark(name):
            sync()
            now = time.perf_counter()
            self.timing[name] += (now - t[0]) * 1e3
            t[0] = now
        return mark

    def _sync_commit_timestamp(self):
        ts = self.comm.allreduce_max(self.backend.commit_timestamp())
        self.backend.advance_commit_timestamp(ts)
        self.commit_timestamp = ts

    # One routing + commit round over the step's events at or after `start`.
    # Returns None when they all committed, else the split point where the next
    # round resumes (the prefix before it committed).
    def _round(self, glob, T, my_events, replies, start):
        W, me = self.world, self.rank
        g0, i0 = start
        # ---- 1. local view of my events in the remaining range
        loc = []   # (g, i) of my remaining events, in global order
        for g in sorted(my_events):
            if g < g0:
                continue
            n = len(my_events[g])
            for i in range(i0 if g == g0 else 0, n):
                loc.append((g, i))
        ev = {k: my_events[k[0]][k[1]] for k in loc}

        # ---- 2. id directory round: every rank sees the step's ids in global order;
        # the engines themselves are the directory of committed ids (a committed
        # transfer lives on the owner of its ledger: routing below keeps that so)
        mine = []
        for (g, i) in loc:
            t = ev[(g, i)]
            x = _id(t["id_lo"], t["id_hi"])
            f = int(t["flags"])
            pv = bool(f & POST_VOID)
            if x == 0 or x == (1 << 128) - 1:
                continue  # fails statically (:1250-1251): no directory entry
            hint = PV if pv else (self.owner_of_ledger(t["ledger"]) if int(t["ledger"]) else ANY)
            mine.append((g, i, 0, x, hint))
            if pv:
                p = _id(t["pending_id_lo"], t["pending_id_hi"])
                if p != 0 and p != (1 << 128) - 1 and p != x:
                    mine.append((g, i, 1, p, ANY))
        recs = sorted((r for lst in self.comm.all_gather_object(mine) for r in lst), key=lambda r: (r[0], r[1], r[2]))
        committed = self._owners_of(sorted({r[3] for r in recs}))
        first = {}  # key -> (g, i, route hint) of its first occurrence this round
        dir_id, dir_p = {}, {}
        for (g, i, k, key, hint) in recs:
            if k == 0:
                if key in committed:
                    a = (EXISTS, committed[key], None)
                elif key in first:
                    fg, fi, fh = first[key]
                    a = (DUP, fh, (fg, fi))
                else:
                    first[key] = (g, i, hint)
                    a = (NEW, None, None)
                dir_id[(g, i)] = a
            else:
                if key in committed:
                    a = (PEND, committed[key], None)
                elif key in first and first[key][:2] < (g, i):
                    fg, fi, fh = first[key]
                    a = (PEND_HAZARD, None, (fg, fi)) if fh in (ANY, PV) else (PEND, fh, (fg, fi))
                else:
                    a = (PEND_NONE, None, None)
                dir_p[(g, i)] = a

        # ---- 3. routing of my events
        route, hazard = {}, None
        chain_of = self._chains(loc, ev)
        for (g, i) in loc:
            t = ev[(g, i)]
            f = int(t["flags"])
            a_id = dir_id.get((g, i), (NEW, None, None))
            if f & POST_VOID:
                a_p = dir_p.get((g, i), (PEND_NONE, None, None))
                if a_p[0] == PEND:
                    r = a_p[1]
                elif a_p[0] == PEND_HAZARD:
                    fg, fi = a_p[2]
                    if (fg, fi) in chain_of and chain_of[(fg, fi)] == chain_of[(g, i)]:
                        r = ("follow", (fg, fi))   # same chain: it can only fail; go where the creator goes
                    else:
                        hazard = self._min(hazard, (g, i))
                        r = ANY
                else:
                    r = ANY  # pending_transfer_not_found or an earlier static failure
                if a_id[0] == DUP and (a_id[1] != r or a_id[1] in (ANY, PV)):
                    fg, fi = a_id[2]
                    if (fg, fi) in chain_of and chain_of[(fg, fi)] == chain_of[(g, i)]:
                        r = ("follow", (fg, fi))   # same chain: it can only fail; go with the first
                    else:
                        hazard = self._min(hazard, (g, i))
                route[(g, i)] = r
            else:
                own = self.owner_of_ledger(t["ledger"]) if int(t["ledger"]) else ANY
                if a_id[0] == EXISTS:
                    r = a_id[1]
                elif a_id[0] == DUP:
                    fg, fi = a_id[2]
                    same_chain = (fg, fi) in chain_of and chain_of[(fg, fi)] == chain_of[(g, i)]
                    if same_chain:
                        r = ("follow", (fg, fi))   # it can only fail: go where the first goes
                    elif a_id[1] == ANY or own == ANY:
                        r = own                    # the first fails statically / so does this one
                    elif a_id[1] == own:
                        r = own
                    else:
                        hazard = self._min(hazard, (g, i))
                        r = own
                else:
                    r = own
                route[(g, i)] = r
        # resolve "follow" routes (same chain, so same source) and ANY inside chains
        for k in loc:
            seen = 0
            while isinstance(route[k], tuple) and seen < len(loc):
                route[k] = route[route[k][1]]
                seen += 1
            if isinstance(route[k], tuple):
                route[k] = ANY
        for members in self._chain_members(loc, chain_of).values():
            owners = [route[m] for m in members if route[m] != ANY]
            fill = owners[0] if owners else me
            for m in members:
                if route[m] == ANY:
                    route[m] = fill
        # post/void whose id is committed on another shard: import that row
        imports = []
        for (g, i) in loc:
            t = ev[(g, i)]
            if int(t["flags"]) & POST_VOID:
                a_id = dir_id.get((g, i), (NEW, None, None))
                if a_id[0] == EXISTS and a_id[1] != route[(g, i)]:
                    imports.append((_id(t["id_lo"], t["id_hi"]), a_id[1], route[(g, i)]))

        # ---- 4. hazards: the earliest one over all ranks splits the step
        hz = [h for h in self.comm.all_gather_object(
            None if hazard is None else self._chain_start(hazard, ev, my_events)) if h is not None]
        stop = min(hz) if hz else None
        if stop is not None and stop <= (g0, i0):
            # A hazard's dependency lies in an earlier chain, so the split lands after
            # the resume point; should one ever name the resume point itself, this
            # round commits the single chain there (its members' dependencies on each
            # other are resolved by "follow" routes) and the next round goes on after it.
            self.stats["serial_fallbacks"] += 1
            stop = self._next_chain_start(loc, chain_of, (g0, i0))
        if stop is not None:
            loc = [k for k in loc if k < stop]
        self._do_imports(imports)  # rows are immutable: importing one early is harmless

        # ---- 5. exchange events to owners (global order is preserved per source)
        parts = [[] for _ in range(W)]
        meta = [[] for _ in range(W)]
        for k in loc:
            d = route[k]
            parts[d].append(ev[k])
            meta[d].append((k[0], k[1], chain_of[k]))
        recv = self._exchange_events(parts)
        recv_meta = self._exchange_objects(meta)
        mine = []   # (g, i, chain key, event) received, in global order
        for src in range(W):
            for (g, i, c), e in zip(recv_meta[src], recv[src]):
                mine.append((g, i, c, e))
        mine.sort(key=lambda x: (x[0], x[1]))

        # cross-shard chains: chain key -> set of owners (all-gathered)
        my_chains = {}
        for k in loc:
            my_chains.setdefault(chain_of[k], set()).add(route[k])
        span = {}
        for d in self.comm.all_gather_object({c: sorted(o) for c, o in my_chains.items() if len(o) > 1}):
            span.update(d)
        self.stats["cross_chains"] += len(span) if self.rank == 0 else 0
        last_member = {}
        for d in self.comm.all_gather_object({c: max(k for k in loc if chain_of[k] == c) for c in span
                                              if any(chain_of[k] == c for k in loc)}):
            for c, m in d.items():
                last_member[c] = max(last_member.get(c, m), m)

        # ---- 6. commit (dry rounds while chains span shards)
        brk = {}   # chain key -> (g, i) of its first failure (global)
        rounds = 0
        while True:
            sub = self._build_sub(mine, T, glob, span, last_member, brk)
            dry = bool(span)
            res = self._commit(sub, dry)
            if not dry:
                break
            rounds += 1
            self.stats["dry_rounds"] += 1
            fails = {}
            for (g, i, c), code in res:
                if c in span and code not in (0, LINKED_EVENT_FAILED):
                    if c not in fails or (g, i) < fails[c]:
                        fails[c] = (g, i)
            nb = {}
            for d in self.comm.all_gather_object(fails):
                for c, p in d.items():
                    if c not in nb or p < nb[c]:
                        nb[c] = p
            if nb == brk:
                sub = self._build_sub(mine, T, glob, span, last_member, brk)
                res2 = self._commit(sub, False)
                # exact as long as every spanning chain broke where its control said
                if self.comm.allreduce_max(int(sorted(res2) != sorted(res))):
                    self.stats["dry_commit_mismatch"] = self.stats.get("dry_commit_mismatch", 0) + 1
                    fails2 = {}
                    for (g, i, c), code in res2:
                        if c in span and code not in (0, LINKED_EVENT_FAILED):
                            if c not in fails2 or (g, i) < fails2[c]:
                                fails2[c] = (g, i)
                    nb2 = {}
                    for d in self.comm.all_gather_object(fails2):
                        for c, p in d.items():
                            if c not in nb2 or p < nb2[c]:
                                nb2[c] = p
                    if nb2 != brk:
                        raise AssertionError("sharded commit: a committed chain broke elsewhere than its dry run "
                                             "(engine invariant)")
                res = res2
                break
            if rounds >= self.max_rounds:
                # Serial fallback: no fixed point yet and nothing committed.  Shrink the
                # round to a prefix that makes progress and settles: the events before
                # the first cross-shard chain (no chain spans there: no dry rounds), or,
                # when that chain starts the round, the chain and what follows it up to
                # the next spanning chain.  A chain with no spanning chain after it
                # settles in two dry rounds: its parts before the break see the same
                # shard states either way.  Every cut is a chain start after the resume
                # point, so the rounds of a step stay bounded by its chains.
                chains = sorted(span)
                head = min((x[0], x[1]) for x in mine) if mine else None
                head = min([h for h in self.comm.all_gather_object(head) if h is not None])
                cut = chains[0] if chains[0] > head else (chains[1] if len(chains) > 1 else None)
                if cut is None:
                    # the lone spanning chain heads the round: commit it alone (its members'
                    # outcomes then depend on the committed state only), the rest after it
                    tail = max((x[0], x[1]) for x in mine) if mine else None
                    tail = max([t for t in self.comm.all_gather_object(tail) if t is not None], default=None)
                    lm = last_member[chains[0]]
                    if tail is not None and tail > lm:
                        cut = (lm[0], lm[1] + 1)
                if cut is not None:
                    mine = [x for x in mine if (x[0], x[1]) < cut]
                    span = {c: o for c, o in span.items() if c < cut}
                    stop = cut if stop is None else min(stop, cut)
                    self.stats["serial_fallbacks"] += 1
                    brk, rounds = {}, 0
                    continue
                # a lone spanning chain at the head of the round settles within two rounds
                if rounds >= self.max_rounds + 2:
                    raise RuntimeError("sharded commit: a lone cross-shard chain did not settle "
                                       "(its break depends on no other chain: an engine invariant failed)")
            brk = nb

        # ---- 7. replies to sources
        rep = [[] for _ in range(W)]
        for (g, i, c), code in res:
            if code != 0:
                rep[glob[g][0]].append((g, i, code))
        for lst in self._exchange_objects(rep):
            for (g, i, code) in lst:
                replies[g].append((i, code))
        top = max([0] + [_id(e["id_lo"], e["id_hi"]) for (g, i, c, e) in mine])
        self.max_id = max(self.max_id, self.comm.allreduce_max(top))
        if stop is None:
            return None
        return stop

    # ----------------------------------------------------------- helpers --
    @staticmethod
    def _min(a, b):
        return b if a is None or b < a else a

    def _next_chain_start(self, loc, chain_of, at):
        """Collective.  The global position of the first event after the chain that
        starts at `at` (None when that chain ends the step)."""
        c = chain_of.get(at)
        nxt = None
        if c is not None:
            after = [k for k in loc if k > at and chain_of[k] != c]
            tail = [k for k in loc if chain_of[k] == c]
            nxt = after[0] if after else (tail[-1][0] + 1, 0)
        got = [x for x in self.comm.all_gather_object(nxt) if x is not None]
        return min(got) if got else None

    @staticmethod
    def _chains(loc, ev):
        """Chain key (g, first index) of each event: a run of `linked` events plus the
        event that ends it, within one batch (execute, :1018-1035)."""
        out = {}
        cur = None
        prev_g = None
        for (g, i) in loc:
            if g != prev_g:
                cur = None
                prev_g = g
            if cur is None:
                cur = (g, i)
            out[(g, i)] = cur
            if not (int(ev[(g, i)]["flags"]) & LINKED):
                cur = None
        return out

    @staticmethod
    def _chain_members(loc, chain_of):
        m = {}
        for k in loc:
            m.setdefault(chain_of[k], []).append(k)
        return m

    @staticmethod
    def _chain_start(k, ev, my_events):
        g, i = k
        b = my_events[g]
        while i > 0 and int(b[i - 1]["flags"]) & LINKED:
            i -= 1
        return (g, i)

    def _exchange_objects(self, parts):
        import pickle
        enc = [np.frombuffer(pickle.dumps(p), dtype=np.uint8) for p in parts]
        return [pickle.loads(x.tobytes()) for x in self.comm.alltoallv(enc)]

    def _owners_of(self, keys):
        """Collective.  {transfer id: owning shard} for the committed ids among `keys`
        (the same list on every rank), looked up in every shard's engine.  Imported
        copies answer like the original: the owner follows the row's ledger."""
        found = {}
        for k0 in range(0, len(keys), 4096):
            part = keys[k0:k0 + 4096]
            for r in self.backend.lookup_transfers(part):
                found[_id(r["id_lo"], r["id_hi"])] = int(r["ledger"])
        out = {}
        for d in self.comm.all_gather_object(found):
            for x, ledger in d.items():
                out[x] = self.owner_of_ledger(ledger)
        return out

    def _exchange_events(self, parts):
        enc = [np.ascontiguousarray(np.array(p, dtype=TRANSFER_DTYPE) if p else np.zeros(0, TRANSFER_DTYPE))
               .view(np.uint8).reshape(-1) for p in parts]
        return [x.view(TRANSFER_DTYPE) if len(x) else np.zeros(0, TRANSFER_DTYPE) for x in self.comm.alltoallv(enc)]

    def _do_imports(self, imports):
        """imports: (id, holder shard, destination shard) requested by this rank."""
        reqs = [[] for _ in range(self.world)]
        for (x, holder, dest) in sorted(set(imports)):
            reqs[holder].append((x, dest))
        got = self._exchange_objects(reqs)
        send = [[] for _ in range(self.world)]
        for lst in got:
            for (x, dest) in lst:
                row = self.backend.lookup_transfers([x])
                assert len(row) == 1, "directory names a shard that does not hold the transfer"
                send[dest].append(row[0])
        rows, seen = [], set()
        for lst in self._exchange_events(send):
            for r in lst:
                x = _id(r["id_lo"], r["id_hi"])
                if x not in seen:
                    seen.add(x)
                    rows.append(r)
        if rows:
            self.backend.import_transfers(np.array(rows, dtype=TRANSFER_DTYPE))
            self.stats["imports"] += len(rows)

    def _build_sub(self, mine, T, glob, span, last_member, brk):
        """Owner sub-batches (one per source batch, global order) with chain control."""
        evs, ts, ctl, keys, counts = [], [], [], [], []
        cur_g, cnt = None, 0
        last_local = {}
        for idx, (g, i, c, e) in enumerate(mine):
            last_local[c] = idx
        for idx, (g, i, c, e) in enumerate(mine):
            if g != cur_g:
                if cur_g is not None:
                    counts.append(cnt)
                cur_g, cnt = g, 0
            b = 0
            if c in span:
                q = brk.get(c)
                if q is not None and (g, i) > q:
                    b |= CTL_SKIP
                if idx == last_local[c] and (g, i) != last_member[c]:
                    b |= CTL_CHAIN_END
                    if q is not None and (g, i) < q:
                        b |= CTL_DOOM   # the chain breaks after this part: roll it back
            evs.append(e)
            ts.append(T[g] - glob[g][2] + i + 1)
            ctl.append(b)
            keys.append((g, i, c))
            cnt += 1
        if cur_g is not None:
            counts.append(cnt)
        return evs, ts, ctl, keys, counts

    def _commit(self, sub, dry):
        evs, ts, ctl, keys, counts = sub
        if not counts:
            return []
        events = np.array(evs, dtype=TRANSFER_DTYPE)
        c = np.array(ctl, dtype=np.uint8)
        out, rc, _ = self.backend.create_transfers_routed(np.array(counts, np.uint32), events,
                                                          np.array(ts, np.uint64), c if c.any() else None, dry)
        res, off = [], 0
        for n, k in zip(counts, rc):
            got = {int(r["index"]): int(r["result"]) for r in out[off:off + int(k)]}
            for j in range(n):
                key = keys[off + j]
                if key is not None:
                    res.append((key, got.get(j, 0)))
            off += n
        return res

    # -------------------------------------------------------------- export --
    def export_state(self):
        """(accounts of the ledgers this shard owns, transfers committed on this shard --
        imported copies excluded): for parity checks."""
        acc = self.backend.export_accounts()
        own = np.array([self.owner_of_ledger(l) == self.rank for l in acc["ledger"]], dtype=bool)
        xs = self.backend.export_transfers()
        keep = np.array([self.owner_of_ledger(l) == self.rank for l in xs["ledger"]], dtype=bool)
        return acc[own] if len(acc) else acc, xs[keep] if len(xs) else xs


def partition_torch(torch, ev, counts, batch_ts, g0: int, W: int, dev, detail: bool = False):
    """The send side of a routed step with torch tensor ops (the CPU-collective tests'
    path; on GPUs the engine's tbgpu_route_scatter computes the same thing): events
    owner-major (owner = ledger % W), in event order within an owner, with their
    8-byte records (REC_*: g << 32 | chain start << 15 | end << 14 | span << 13 |
    index).  `batch_ts` is no longer part of the record (the owner derives the
    timestamps).  Returns (events [n, 128], records [n], per-owner counts)."""
    if any(int(c) > REC_POS + 1 for c in counts):
        raise ValueError("a routed batch holds at most 8192 events")
    n = int(sum(counts))
    w32 = ev.view(torch.int32).view(n, 32)
    flags = (w32[:, 29] >> 16) & 0xFFFF
    cnt_t = torch.tensor(list(counts), dtype=torch.int64, device=dev)
    nb = len(counts)
    bidx = torch.repeat_interleave(torch.arange(nb, device=dev), cnt_t)
    bstart = torch.cumsum(cnt_t, 0) - cnt_t
    pos = torch.arange(n, device=dev) - bstart[bidx]
    g = bidx + g0
    linked = (flags & LINKED) != 0
    prev_l = torch.zeros_like(linked)
    prev_l[1:] = linked[:-1]
    prev_l &= pos > 0
    ar = torch.arange(n, device=dev)
    cstart = torch.cummax(torch.where(prev_l, torch.zeros_like(ar), ar), 0).values
    last = ~linked | (pos == cnt_t[bidx] - 1)      # the chain's own last member
    owner = ((w32[:, 28].to(torch.int64) & 0xFFFFFFFF) % W)
    omin = torch.full((n,), W, dtype=torch.int64, device=dev).scatter_reduce(0, cstart, owner, "amin")
    omax = torch.full((n,), -1, dtype=torch.int64, device=dev).scatter_reduce(0, cstart, owner, "amax")
    span = omin[cstart] != omax[cstart]
    side = (g << 32) | ((cstart - bstart[bidx]) << REC_CS_SHIFT) | (last.to(torch.int64) << 14) | \
        (span.to(torch.int64) << 13) | pos
    perm = torch.argsort(owner, stable=True)
    send = torch.bincount(owner, minlength=W)
    out = (ev.view(n, 128).index_select(0, perm), side.index_select(0, perm), send)
    if not detail:
        return out
    per_batch = torch.bincount(owner * nb + bidx, minlength=W * nb).view(W, nb)
    spanning = torch.bincount(owner[span], minlength=W)
    return out + (per_batch, spanning)
