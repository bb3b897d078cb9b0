"""Deterministic synthetic workloads for BASELINE.json's configs.

config 1  `tigerbeetle benchmark` defaults (src/tigerbeetle/benchmark_load.zig:209-330):
          10k accounts (ledger 2, code 1), uniform random debit/credit pairs,
          amount = floor(Exp(1) * 10000) +| 1, code = rand_u16 +| 1, flags 0,
          ids = transfer index + 1 (identity IdPermutation).
config 2  1M accounts on one ledger, debit/credit ranks drawn independently from
          Zipf(s = 0.99), rank -> id through a fixed random permutation.
config 3  flag-heavy mix: limit accounts, pending / post / void, balancing,
          linked chains, duplicate ids and invalid fields, periodic ticks.
config 4  1000 ledgers x 10k accounts, uniform pairs within a ledger, 1%
          cross-ledger linked pairs (ledger-sharded across GPUs).
config 5  100M accounts over 1000 ledgers, 1B transfers over 8 ledger shards,
          generated in HBM (DeviceLoad: the load is too large for the host).

The reference draws from Zig's std.rand; only the *distributions* are
reproduced (numpy PCG64 streams, seed 42 by default).  Timestamps follow the
reference test harness (src/state_machine.zig:1973-1978): before each commit
prepare_timestamp += 1 + len(batch) and the commit timestamp is that value.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from .types import ACCOUNT_DTYPE, BATCH_MAX, TRANSFER_DTYPE, U64_MAX, AccountFlags, TransferFlags

NS_PER_S = 1_000_000_000


@dataclass
class Workload:
    name: str
    accounts: np.ndarray
    account_counts: np.ndarray
    transfers: np.ndarray
    transfer_counts: np.ndarray
    # extra prepare_timestamp ticks applied before transfer batch b (harness `tick`)
    ticks: dict = field(default_factory=dict)

    def timestamps(self, start: int = 0):
        """Commit timestamps for the account batches then the transfer batches."""
        t = start
        acc_ts = np.zeros(len(self.account_counts), dtype=np.uint64)
        for b, n in enumerate(self.account_counts):
            t += 1 + int(n)
            acc_ts[b] = t
        tr_ts = np.zeros(len(self.transfer_counts), dtype=np.uint64)
        for b, n in enumerate(self.transfer_counts):
            t += self.ticks.get(b, 0)
            t += 1 + int(n)
            tr_ts[b] = t
        return acc_ts, tr_ts


def _batches(total: int, size: int = BATCH_MAX) -> np.ndarray:
    n_full, rem = divmod(total, size)
    c = [size] * n_full + ([rem] if rem else [])
    return np.array(c, dtype=np.uint32)


def _set128(arr, name, lo, hi=None):
    arr[name + "_lo"] = lo
    arr[name + "_hi"] = 0 if hi is None else hi


def _amounts(rng, n):
    # random_int_exponential(u64, 10_000) +| 1  (src/testing/fuzz.zig:16-24)
    a = np.floor(rng.exponential(1.0, n) * 10_000.0)
    return np.minimum(a, float(U64_MAX - 1)).astype(np.uint64) + np.uint64(1)


def _codes(rng, n):
    c = rng.integers(0, 1 << 16, n, dtype=np.uint32) + 1
    return np.minimum(c, 0xFFFF).astype(np.uint16)  # +| saturating


ID_ORDERS = ("sequential", "random", "reversed")


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64's finalizer over a u64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def encode_ids(data: np.ndarray, order: str = "sequential", seed: int = 0):
    """IdPermutation.encode (src/testing/id.zig:28-48) as the benchmark applies it
    (`--id-order`, src/tigerbeetle/cli.zig:205, benchmark_load.zig:134-138): returns
    the u128 ids of `data` (u64 indices, the benchmark's index + 1) as (lo, hi).
      sequential  identity;
      reversed    maxInt(u128) - data;
      random      data << 32 with bits 0..32 and 96..128 random (a pseudo-UUID whose
                  index is recoverable).  The reference seeds Zig's DefaultPrng with
                  seed + data; here a splitmix64 stream of seed + data gives the bits
                  (the layout, not Zig's stream, is reproduced)."""
    d = np.asarray(data, dtype=np.uint64)
    if order == "sequential":
        return d.copy(), np.zeros_like(d)
    if order == "reversed":
        return ~d, np.full_like(d, U64_MAX)
    if order != "random":
        raise ValueError(f"id order {order!r}")
    with np.errstate(over="ignore"):
        k = np.uint64(seed & U64_MAX) + d
        r0 = _mix64(k * np.uint64(2) + np.uint64(0x9E3779B97F4A7C15))
        r1 = _mix64(k * np.uint64(2) + np.uint64(1) + np.uint64(0x9E3779B97F4A7C15))
    lo = (d << np.uint64(32)) | (r0 & np.uint64(0xFFFFFFFF))
    hi = (d >> np.uint64(32)) | (r1 & np.uint64(0xFFFFFFFF00000000))
    return lo, hi


def make_accounts(ids: np.ndarray, ledger, code=1, flags=None, ids_hi=None) -> np.ndarray:
    a = np.zeros(len(ids), dtype=ACCOUNT_DTYPE)
    _set128(a, "id", ids.astype(np.uint64), None if ids_hi is None else ids_hi.astype(np.uint64))
    a["ledger"] = ledger
    a["code"] = code
    if flags is not None:
        a["flags"] = flags
    return a


def _transfers(rng, ids, dr, cr, ledger, order="sequential", id_seed=0):
    """Transfers with ids encode(ids), accounts encode(dr), encode(cr) under the id
    order (the benchmark uses one permutation for both, benchmark_load.zig:296-301)."""
    n = len(ids)
    t = np.zeros(n, dtype=TRANSFER_DTYPE)
    _set128(t, "id", *encode_ids(ids, order, id_seed))
    _set128(t, "debit_account_id", *encode_ids(dr, order, id_seed))
    _set128(t, "credit_account_id", *encode_ids(cr, order, id_seed))
    _set128(t, "user_data_128", rng.integers(0, U64_MAX, n, dtype=np.uint64, endpoint=True),
            rng.integers(0, U64_MAX, n, dtype=np.uint64, endpoint=True))
    t["user_data_64"] = rng.integers(0, U64_MAX, n, dtype=np.uint64, endpoint=True)
    t["user_data_32"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    t["ledger"] = ledger
    t["code"] = _codes(rng, n)
    _set128(t, "amount", _amounts(rng, n))
    return t


def _id_seed(seed: int) -> int:
    """The permutation's seed, drawn from the workload's seed as the benchmark draws it
    from its PRNG (`.random = random.int(u64)`, benchmark_load.zig:134-138)."""
    return int(np.random.default_rng(seed ^ 0x1D0D).integers(0, U64_MAX, dtype=np.uint64, endpoint=True))


def config1(transfer_count: int = 10_000_000, account_count: int = 10_000, seed: int = 42,
            batch: int = BATCH_MAX, id_order: str = "sequential") -> Workload:
    rng = np.random.default_rng(seed)
    ids_seed = _id_seed(seed)
    acc_ids = np.arange(1, account_count + 1, dtype=np.uint64)
    lo, hi = encode_ids(acc_ids, id_order, ids_seed)
    accounts = make_accounts(lo, ledger=2, ids_hi=hi)
    dr = rng.integers(0, account_count, transfer_count, dtype=np.uint64)
    cr = rng.integers(0, account_count, transfer_count, dtype=np.uint64)
    cr = np.where(dr == cr, (cr + 1) % account_count, cr)  # benchmark_load.zig:291-295
    ids = np.arange(1, transfer_count + 1, dtype=np.uint64)
    transfers = _transfers(rng, ids, dr + 1, cr + 1, ledger=2, order=id_order, id_seed=ids_seed)
    name = "config1" if id_order == "sequential" else f"config1-{id_order}"
    return Workload(name, accounts, _batches(account_count), transfers, _batches(transfer_count, batch))


def zipf_sampler(rng, n: int, s: float):
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]

    def draw(k):
        return np.minimum(np.searchsorted(cdf, rng.random(k), side="right"), n - 1).astype(np.uint64)
    return draw


def config2(transfer_count: int = 8_190_000, account_count: int = 1_000_000, seed: int = 42, s: float = 0.99,
            batch: int = BATCH_MAX, id_order: str = "sequential") -> Workload:
    rng = np.random.default_rng(seed)
    ids_seed = _id_seed(seed)
    perm = rng.permutation(account_count).astype(np.uint64)  # rank -> account index
    if os.environ.get("TB_ZIPF_IDENTITY") == "1":  # timing experiments only: rank r is row r (profiles/r04/var_c2.sh)
        perm = np.arange(account_count, dtype=np.uint64)
    acc_ids = np.arange(1, account_count + 1, dtype=np.uint64)
    lo, hi = encode_ids(acc_ids, id_order, ids_seed)
    accounts = make_accounts(lo, ledger=1, ids_hi=hi)
    draw = zipf_sampler(rng, account_count, s)
    dr = perm[draw(transfer_count)]
    cr = perm[draw(transfer_count)]
    cr = np.where(dr == cr, (cr + 1) % account_count, cr)
    ids = np.arange(1, transfer_count + 1, dtype=np.uint64)
    transfers = _transfers(rng, ids, dr + 1, cr + 1, ledger=1, order=id_order, id_seed=ids_seed)
    name = "config2" if id_order == "sequential" else f"config2-{id_order}"
    return Workload(name, accounts, _batches(account_count), transfers, _batches(transfer_count, batch))


def config4(transfer_count: int = 16_380_000, ledgers: int = 1000, accounts_per_ledger: int = 10_000,
            seed: int = 42, cross_ledger_pairs: float = 0.01, batch: int = BATCH_MAX) -> Workload:
    """Ledger-sharded workload.  Account id = ledger * 2^32 + k (k in 1..accounts_per_ledger)."""
    rng = np.random.default_rng(seed)
    led = np.repeat(np.arange(1, ledgers + 1, dtype=np.uint64), accounts_per_ledger)
    k = np.tile(np.arange(1, accounts_per_ledger + 1, dtype=np.uint64), ledgers)
    accounts = make_accounts((led << np.uint64(32)) | k, ledger=led.astype(np.uint32))
    tl = rng.integers(1, ledgers + 1, transfer_count, dtype=np.uint64)
    dr = rng.integers(0, accounts_per_ledger, transfer_count, dtype=np.uint64)
    cr = rng.integers(0, accounts_per_ledger, transfer_count, dtype=np.uint64)
    cr = np.where(dr == cr, (cr + 1) % accounts_per_ledger, cr)
    ids = np.arange(1, transfer_count + 1, dtype=np.uint64)
    transfers = _transfers(rng, ids, (tl << np.uint64(32)) | (dr + 1), (tl << np.uint64(32)) | (cr + 1),
                           ledger=tl.astype(np.uint32))
    # cross-ledger linked pairs (currency exchange, docs/reference/transfers.md:282): event i and
    # i+1 linked, the second moved to another ledger.
    n_pairs = int(transfer_count * cross_ledger_pairs / 2)
    if n_pairs:
        starts = rng.choice(np.arange(0, transfer_count - 1, 2), size=n_pairs, replace=False)
        starts = starts[(starts % batch) != batch - 1]
        t0 = transfers[starts]
        t0["flags"] |= np.uint16(int(TransferFlags.linked))
        transfers[starts] = t0
        other = (tl[starts] % ledgers) + 1
        t1 = transfers[starts + 1]
        t1["ledger"] = other.astype(np.uint32)
        _set128(t1, "debit_account_id", (other << np.uint64(32)) | (dr[starts + 1] + 1))
        _set128(t1, "credit_account_id", (other << np.uint64(32)) | (cr[starts + 1] + 1))
        transfers[starts + 1] = t1
    return Workload("config4", accounts, _batches(len(accounts)), transfers, _batches(transfer_count, batch))


def _weighted(rng, pool: np.ndarray, weights: np.ndarray, k: int) -> np.ndarray:
    c = np.cumsum(weights, dtype=np.float64)
    return pool[np.minimum(np.searchsorted(c, rng.random(k) * c[-1], side="right"), len(pool) - 1)]


def _chain_links(rng, n: int, share: float = 0.25, lo: int = 2, hi: int = 8) -> np.ndarray:
    """bool[n]: event j carries `linked` (chains of lo..hi events over ~`share` of events)."""
    mean = (lo + hi) / 2.0
    p_chain = share / (mean - share * (mean - 1.0))  # a unit starts a chain w.p. p_chain
    k = n // 2 + 16
    lens = np.where(rng.random(k) < p_chain, rng.integers(lo, hi + 1, k), 1)
    ends = np.cumsum(lens)
    lens = lens[:np.searchsorted(ends, n) + 1]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    linked = np.zeros(n + hi, dtype=bool)
    for s, ln in zip(starts[lens > 1], lens[lens > 1]):
        linked[s:s + ln - 1] = True
    linked = linked[:n]
    linked[n - 1] = False  # a chain never runs off the batch here (open chains: below)
    return linked


def config3(batches: int = 200, batch: int = BATCH_MAX, account_count: int = 10_000, seed: int = 42,
            tick_every: int = 50, tick_ns: int = 60 * NS_PER_S, plain_batches=()) -> Workload:
    """Flag-heavy mix at BASELINE config 3's shape, tuned to ~10 % non-ok.

    10k accounts on one ledger: 30 % debits_must_not_exceed_credits, 10 %
    credits_must_not_exceed_debits, 2 % history, the rest unflagged.  A funding
    phase credits every D<C account and debits every C<D account.  Main phase, per
    event: single-phase 45 %, pending 20 % (timeout 0 or Exp(5 s)+1), post 15 %
    (amount 0 = inherit, or partial 1..p.amount), void 10 %, balancing debit /
    credit 5 % each (amount 0 or random); ~25 % of events in linked chains of 2-8,
    ~1 % repeated ids, ~1 % invalid fields (the invalid kinds of
    src/state_machine/workload.zig:143-161), an occasional chain left open at the
    batch end, and a +60 s tick every 50 batches that expires timed pendings.

    What keeps the failure rate near 10 % (the stress mix `config3_stress` runs
    near 40 %): limit accounts drift away from their limits (D<C accounts are
    credited more often than debited, C<D accounts the reverse), balancing
    transfers mostly draw on accounts that hold a balance of the right sign, and
    posts / voids resolve pendings that are still open (most from earlier batches,
    some from earlier in the same batch), so `already_posted/voided` and `expired`
    stay the exceptions they are in practice.  The rate is printed by bench.py.

    `plain_batches`: indices of main-phase batches made of plain transfers between
    unflagged accounts only (the single-pass path takes them), to mix the engine's
    two paths inside one streamed call.
    """
    rng = np.random.default_rng(seed)
    acc_ids = np.arange(1, account_count + 1, dtype=np.uint64)
    roll = rng.random(account_count)
    aflags = np.where(roll < 0.30, int(AccountFlags.debits_must_not_exceed_credits),
                      np.where(roll < 0.40, int(AccountFlags.credits_must_not_exceed_debits), 0)).astype(np.uint16)
    hist = rng.random(account_count) < 0.02
    aflags = aflags | np.where(hist, int(AccountFlags.history), 0).astype(np.uint16)
    accounts = make_accounts(acc_ids, ledger=1, flags=aflags)
    idx = np.arange(account_count, dtype=np.int64)
    dnec = idx[(aflags & 2) != 0]
    cned = idx[(aflags & 4) != 0]
    free = idx[(aflags & 6) == 0]
    plain_pool = idx[aflags == 0]
    # debit-side / credit-side account weights: limit accounts drift away from their limits
    w_dr = np.where((aflags & 2) != 0, 0.5, np.where((aflags & 4) != 0, 1.5, 1.0))
    w_cr = np.where((aflags & 2) != 0, 1.5, np.where((aflags & 4) != 0, 0.5, 1.0))

    out, counts = [], []
    next_id = 1
    fund_d = np.concatenate([free[rng.integers(0, len(free), len(dnec))], cned])
    fund_c = np.concatenate([dnec, free[rng.integers(0, len(free), len(cned))]])
    for s in range(0, len(fund_d), batch):
        k = min(batch, len(fund_d) - s)
        t = np.zeros(k, dtype=TRANSFER_DTYPE)
        t["id_lo"] = np.arange(next_id, next_id + k, dtype=np.uint64)
        next_id += k
        t["debit_account_id_lo"] = fund_d[s:s + k].astype(np.uint64) + 1
        t["credit_account_id_lo"] = fund_c[s:s + k].astype(np.uint64) + 1
        t["amount_lo"] = rng.integers(20_000, 60_000, k, dtype=np.uint64)
        t["ledger"] = 1
        t["code"] = 1
        out.append(t)
        counts.append(k)

    ticks = {}
    open_pend: list[tuple[int, int, int, int]] = []  # (id, amount, debit row, credit row), oldest first
    recent_ids = np.zeros(0, dtype=np.uint64)
    plain = set(int(b) for b in plain_batches)
    for b in range(batches):
        if tick_every and b > 0 and b % tick_every == 0:
            ticks[len(counts)] = tick_ns
            # pendings with a timeout expire at the tick: a few stay in the pool (-> expired)
            open_pend = [p for p in open_pend if p[2] == 0 or rng.random() < 0.1]
        n = batch
        t = np.zeros(n, dtype=TRANSFER_DTYPE)
        ids = np.arange(next_id, next_id + n, dtype=np.uint64)
        next_id += n
        t["ledger"] = 1
        t["user_data_64"] = rng.integers(0, 3, n, dtype=np.uint64)
        t["user_data_32"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        if b in plain:
            d = plain_pool[rng.integers(0, len(plain_pool), n)]
            c = plain_pool[rng.integers(0, len(plain_pool) - 1, n)]
            c = np.where(c == d, plain_pool[(np.searchsorted(plain_pool, d) + 1) % len(plain_pool)], c)
            t["id_lo"] = ids
            t["debit_account_id_lo"] = d.astype(np.uint64) + 1
            t["credit_account_id_lo"] = c.astype(np.uint64) + 1
            t["amount_lo"] = _amounts(rng, n) % np.uint64(3000) + np.uint64(1)
            t["code"] = rng.integers(1, 100, n).astype(np.uint16)
            out.append(t)
            counts.append(n)
            continue
        kinds = rng.choice(6, size=n, p=[0.45, 0.20, 0.15, 0.10, 0.05, 0.05])
        d = _weighted(rng, idx, w_dr, n)
        c = _weighted(rng, idx, w_cr, n)
        # balancing debits draw on accounts holding credit, balancing credits on debit balances
        bd = kinds == 4
        pick = bd & (rng.random(n) < 0.8)
        d[pick] = dnec[rng.integers(0, len(dnec), int(pick.sum()))]
        bc = kinds == 5
        pick = bc & (rng.random(n) < 0.8)
        c[pick] = cned[rng.integers(0, len(cned), int(pick.sum()))]
        same = d == c
        c[same] = (c[same] + 1 + rng.integers(0, account_count - 1, int(same.sum()))) % account_count
        amt = np.floor(rng.exponential(1.0, n) * 2000).astype(np.uint64) + np.uint64(1)
        t["id_lo"] = ids
        t["code"] = rng.integers(1, 100, n).astype(np.uint16)
        t["debit_account_id_lo"] = d.astype(np.uint64) + 1
        t["credit_account_id_lo"] = c.astype(np.uint64) + 1
        t["amount_lo"] = amt
        fl = np.zeros(n, dtype=np.uint16)
        fl[kinds == 1] = int(TransferFlags.pending)
        fl[bd] = int(TransferFlags.balancing_debit)
        fl[bc] = int(TransferFlags.balancing_credit)
        zero_amt = (bd | bc) & (rng.random(n) < 0.15)
        t["amount_lo"][zero_amt] = 0
        timed = (kinds == 1) & (rng.random(n) < 0.5)
        t["timeout"][timed] = (np.floor(rng.exponential(5.0, int(timed.sum()))) + 1).astype(np.uint32)
        # posts and voids: resolve open pendings, oldest-first from earlier batches, or one
        # created earlier in this batch
        batch_pend: list[int] = []  # positions of this batch's pendings seen so far
        for j in range(n):
            k = kinds[j]
            if k == 1:
                batch_pend.append(j)
                continue
            if k not in (2, 3):
                continue
            src = None
            if batch_pend and rng.random() < 0.15:
                q = batch_pend.pop(int(rng.integers(0, len(batch_pend))))
                src = (int(ids[q]), int(amt[q]))
            elif open_pend:
                # mostly recent pendings; older ones (perhaps expired) now and then
                back = int(rng.integers(1, min(len(open_pend), 4096) + 1))
                if rng.random() < 0.03:
                    back = int(rng.integers(1, len(open_pend) + 1))
                p = open_pend.pop(len(open_pend) - back)
                src = (p[0], p[1])
            if src is None:
                kinds[j] = 0  # nothing open to resolve: a single-phase transfer instead
                continue
            pid, pamt = src
            fl[j] = int(TransferFlags.post_pending_transfer if k == 2 else TransferFlags.void_pending_transfer)
            t[j]["pending_id_lo"] = pid
            t[j]["debit_account_id_lo"] = 0
            t[j]["credit_account_id_lo"] = 0
            t[j]["timeout"] = 0
            if k == 2:
                t[j]["amount_lo"] = 0 if rng.random() < 0.3 else int(rng.integers(1, pamt + 1))
            else:
                t[j]["amount_lo"] = 0 if rng.random() < 0.5 else pamt
            t[j]["ledger"] = 0 if rng.random() < 0.5 else 1
            t[j]["code"] = 0
        for q in batch_pend:  # still open at the end of the batch
            open_pend.append((int(ids[q]), int(amt[q]), int(t[q]["timeout"]), 0))
        if len(open_pend) > 60_000:
            open_pend = open_pend[-60_000:]
        # repeated ids (~1 %): an id of an earlier event, in this batch or a recent one
        rep = np.nonzero(rng.random(n) < 0.01)[0]
        rep = rep[rep > 0]
        for j in rep:
            if len(recent_ids) and rng.random() < 0.5:
                t[j]["id_lo"] = recent_ids[int(rng.integers(0, len(recent_ids)))]
            else:
                t[j]["id_lo"] = t[int(rng.integers(0, j))]["id_lo"]
        # invalid fields (~1 %)
        bad = np.nonzero(rng.random(n) < 0.01)[0]
        for j in bad:
            which = int(rng.integers(0, 4))
            pv = int(fl[j]) & 12
            if which == 0:
                t[j]["ledger"] = 7 if pv else 0
            elif which == 1:
                t[j]["code"] = 7 if pv else 0
            elif which == 2 and not (int(fl[j]) & 2):
                t[j]["timeout"] = 5
            else:
                t[j]["debit_account_id_lo"] = account_count + 77
        links = _chain_links(rng, n)
        if rng.random() < 0.02:
            links[n - 1] = True  # linked_event_chain_open
        fl |= np.where(links, int(TransferFlags.linked), 0).astype(np.uint16)
        t["flags"] = fl
        out.append(t)
        counts.append(n)
        recent_ids = np.concatenate([recent_ids, t["id_lo"]])[-20_000:]
    transfers = np.concatenate(out)
    return Workload("config3", accounts, _batches(account_count), transfers, np.array(counts, dtype=np.uint32),
                    ticks)


def config3_stress(batches: int = 200, batch: int = BATCH_MAX, account_count: int = 10_000, seed: int = 42,
                   tick_every: int = 50, tick_ns: int = 60 * NS_PER_S) -> Workload:
    """Flag-heavy stress mix (round 1's config 3, ~40 % non-ok): posts and voids pick
    random earlier pendings (often resolved or expired already), limit accounts
    random-walk into their limits, balancing amounts are random.

    Per event: single-phase 45%, pending 20% (timeout 0 or Exp(5 s)+1), post 15%
    (partial 1..p.amount or 0 = inherit), void 10%, balancing debit/credit 5% each.
    ~25% of events in linked chains of length 2-8, ~1% duplicate ids, ~1%
    invalid fields.  The first batch funds the limit accounts.
    """
    rng = np.random.default_rng(seed)
    acc_ids = np.arange(1, account_count + 1, dtype=np.uint64)
    roll = rng.random(account_count)
    aflags = np.where(roll < 0.30, int(AccountFlags.debits_must_not_exceed_credits),
                      np.where(roll < 0.40, int(AccountFlags.credits_must_not_exceed_debits), 0)).astype(np.uint16)
    hist = rng.random(account_count) < 0.02
    aflags = aflags | np.where(hist, int(AccountFlags.history), 0).astype(np.uint16)
    accounts = make_accounts(acc_ids, ledger=1, flags=aflags)
    free = np.nonzero((aflags & 6) == 0)[0]
    dnec = np.nonzero(aflags & 2)[0]
    cned = np.nonzero(aflags & 4)[0]

    out = []
    counts = []
    next_id = 1
    pendings: list[tuple[int, int]] = []  # (id, amount)
    recent_ids: list[int] = []

    def rand_free():
        return int(free[rng.integers(0, len(free))])

    # funding batch(es): credit every D<C account, debit every C<D account
    fund = []
    for a in dnec:
        fund.append((rand_free(), int(a), int(rng.integers(5_000, 50_000))))
    for a in cned:
        fund.append((int(a), rand_free(), int(rng.integers(5_000, 50_000))))
    for s in range(0, len(fund), batch):
        part = fund[s:s + batch]
        t = np.zeros(len(part), dtype=TRANSFER_DTYPE)
        for j, (d, c, amt) in enumerate(part):
            t[j]["id_lo"] = next_id
            next_id += 1
            t[j]["debit_account_id_lo"] = d + 1
            t[j]["credit_account_id_lo"] = c + 1
            t[j]["amount_lo"] = amt
            t[j]["ledger"] = 1
            t[j]["code"] = 1
        out.append(t)
        counts.append(len(part))

    ticks = {}
    for b in range(batches):
        if tick_every and b > 0 and b % tick_every == 0:
            ticks[len(counts)] = tick_ns
        t = np.zeros(batch, dtype=TRANSFER_DTYPE)
        kinds = rng.choice(6, size=batch, p=[0.45, 0.20, 0.15, 0.10, 0.05, 0.05])
        new_pend = []
        for j in range(batch):
            r = t[j]
            k = kinds[j]
            tid = next_id
            next_id += 1
            if rng.random() < 0.01 and recent_ids:
                tid = recent_ids[int(rng.integers(0, len(recent_ids)))]  # duplicate id
            r["id_lo"] = tid
            r["ledger"] = 1
            r["code"] = int(rng.integers(1, 100))
            r["user_data_64"] = int(rng.integers(0, 3))
            d = int(rng.integers(0, account_count))
            c = int(rng.integers(0, account_count - 1))
            c = c + 1 if c >= d else c
            amt = int(np.floor(rng.exponential(1.0) * 3000)) + 1
            if k in (2, 3) and pendings:  # post / void an earlier pending
                pid, pamt = pendings[int(rng.integers(0, len(pendings)))]
                r["pending_id_lo"] = pid
                r["flags"] = int(TransferFlags.post_pending_transfer if k == 2 else TransferFlags.void_pending_transfer)
                if k == 2:
                    roll = rng.random()
                    r["amount_lo"] = 0 if roll < 0.3 else int(rng.integers(1, max(2, pamt + 1)))
                else:
                    r["amount_lo"] = 0 if rng.random() < 0.5 else pamt
                r["ledger"] = 0 if rng.random() < 0.5 else 1
                r["code"] = 0
            else:
                r["debit_account_id_lo"] = d + 1
                r["credit_account_id_lo"] = c + 1
                r["amount_lo"] = amt
                if k == 1:
                    r["flags"] = int(TransferFlags.pending)
                    r["timeout"] = 0 if rng.random() < 0.5 else int(np.floor(rng.exponential(5.0))) + 1
                    new_pend.append((tid, amt))
                elif k == 4:
                    r["flags"] = int(TransferFlags.balancing_debit)
                    if rng.random() < 0.5:
                        r["amount_lo"] = 0
                elif k == 5:
                    r["flags"] = int(TransferFlags.balancing_credit)
                    if rng.random() < 0.5:
                        r["amount_lo"] = 0
            if rng.random() < 0.01:  # invalid field
                which = int(rng.integers(0, 4))
                if which == 0:
                    r["ledger"] = 0 if not (int(r["flags"]) & 12) else 7
                elif which == 1:
                    r["code"] = 0 if not (int(r["flags"]) & 12) else 7
                elif which == 2:
                    r["timeout"] = 5 if not (int(r["flags"]) & 2) else r["timeout"]
                else:
                    r["debit_account_id_lo"] = account_count + 77
            recent_ids.append(tid)
        # linked chains covering ~25% of events
        j = 0
        while j < batch - 1:
            if rng.random() < 0.25 / 5.0:
                ln = int(rng.integers(2, 9))
                ln = min(ln, batch - j)
                for q in range(j, j + ln - 1):
                    t[q]["flags"] |= int(TransferFlags.linked)
                j += ln
            else:
                j += 1
        # an occasional open chain at the batch end
        if rng.random() < 0.02:
            t[batch - 1]["flags"] |= int(TransferFlags.linked)
        out.append(t)
        counts.append(batch)
        pendings.extend(new_pend)
        if len(pendings) > 50_000:
            pendings = pendings[-50_000:]
        if len(recent_ids) > 20_000:
            recent_ids = recent_ids[-20_000:]
    transfers = np.concatenate(out)
    return Workload("config3_stress", accounts, _batches(account_count), transfers,
                    np.array(counts, dtype=np.uint32), ticks)


@dataclass
class DeviceLoad:
    """BASELINE config 5's load for one ledger shard, generated in HBM by the engine's
    counter-based generator (engine.generate_accounts / generate_transfers,
    csrc/loadgen.hip): record i depends only on (seed, first id + i).

    100M accounts over 1000 ledgers (ids 1..100M, ledger (id - 1) / 100k + 1;
    every shard's directory knows them all, its rows are its own ledgers'), 1B
    transfers split evenly over `shards` ledger shards: shard s owns the ledgers
    with ledger % shards == s (the router's owner_of_ledger) and draws its
    transfers from them, ledger0 + ledger_stride * [0, ledgers), uniform distinct
    debit / credit accounts within a ledger, amount floor(Exp(1) * 10000) + 1 --
    the `tigerbeetle benchmark` distribution (src/tigerbeetle/benchmark_load.zig:
    266-330) within each ledger."""
    accounts: int
    accounts_per_ledger: int
    ledger0: int
    ledgers: int
    transfers: int
    seed: int
    first_transfer_id: int = 1
    ledger_stride: int = 1
    shard: int = 0
    shards: int = 1

    def owned_ledgers(self) -> np.ndarray:
        return self.ledger0 + self.ledger_stride * np.arange(self.ledgers, dtype=np.int64)

    def owned_accounts(self) -> int:
        return self.ledgers * self.accounts_per_ledger

    def account_batches(self, batch: int = BATCH_MAX) -> np.ndarray:
        return _batches(self.accounts, batch)

    def transfer_batches(self, batch: int = BATCH_MAX) -> np.ndarray:
        return _batches(self.transfers, batch)

    def timestamps(self, batch: int = BATCH_MAX):
        """Commit timestamps of the account batches then the transfer batches (the
        reference harness rule, as Workload.timestamps)."""
        ac, tc = self.account_batches(batch).astype(np.uint64), self.transfer_batches(batch).astype(np.uint64)
        acc_ts = np.cumsum(ac + np.uint64(1))
        tr_ts = acc_ts[-1] + np.cumsum(tc + np.uint64(1))
        return acc_ts, tr_ts


def config5(shard: int = 0, shards: int = 8, accounts: int = 100_000_000, ledgers: int = 1000,
            transfers_total: int = 1_000_000_000, seed: int = 42) -> DeviceLoad:
    per = ledgers // shards
    return DeviceLoad(accounts=accounts, accounts_per_ledger=accounts // ledgers, ledger0=shard if shard else shards,
                      ledgers=per, transfers=transfers_total // shards, seed=seed + shard,
                      first_transfer_id=shard * (transfers_total // shards) + 1, ledger_stride=shards,
                      shard=shard, shards=shards)


def make(config: int, **kw) -> Workload:
    return {1: config1, 2: config2, 3: config3, 4: config4}[config](**kw)
