"""Shard backends for the CPU router tests (test infrastructure).

`LedgerShardOracle` stands in for a ledger-shard engine (tbgpu_options.shard_world,
include/tbgpu.h): the oracle runs the replicated create_accounts as the engine does,
and its replies are the engine's: an `exists*` reply for an id created before the call
on another shard's ledger is TBGPU_SHARD_ACCOUNT_EXISTS_ELSEWHERE (the engine keeps no
row of such an account to compare, src/state_machine.zig:1227-1237); its exported
accounts are its own ledgers'.  Everything else is the oracle's."""
from __future__ import annotations

import numpy as np

from tigerbeetle_amd.shard import ACCOUNT_EXISTS_CODES, SHARD_EXISTS_ELSEWHERE
from tigerbeetle_amd.types import ACCOUNT_DTYPE


class LedgerShardOracle:
    def __init__(self, inner, world: int, rank: int):
        self.inner, self.shard_world, self.shard_rank = inner, world, rank

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def _owned(self, ledger) -> bool:
        return int(ledger) % self.shard_world == self.shard_rank

    def create_accounts_batches(self, timestamps, counts, events):
        events = np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE)
        ids = (events["id_hi"].astype(object) << 64) | events["id_lo"].astype(object)
        before = {}
        uniq = sorted({int(x) for x in ids if 0 < int(x) < (1 << 128) - 1})
        for row in (self.inner.lookup_accounts(uniq) if uniq else []):
            before[(int(row["id_hi"]) << 64) | int(row["id_lo"])] = int(row["ledger"])
        out, rc = self.inner.create_accounts_batches(timestamps, counts, events)
        off_ev, off_r = 0, 0
        for c, k in zip(counts, rc):
            for q in range(off_r, off_r + int(k)):
                code = int(out[q]["result"])
                x = int(ids[off_ev + int(out[q]["index"])])
                if code in ACCOUNT_EXISTS_CODES and x in before and not self._owned(before[x]):
                    out[q]["result"] = SHARD_EXISTS_ELSEWHERE
            off_ev += int(c)
            off_r += int(c)
        return out, rc

    def export_accounts(self):
        a = self.inner.export_accounts()
        return a[np.array([self._owned(x) for x in a["ledger"]], dtype=bool)] if len(a) else a


def with_account_recreates(sw, seed: int):
    """A second round of account batches that re-creates a third of the accounts with
    one field changed (flags, user data, ledger, code) or unchanged (`exists`), mixed
    with new accounts in linked chains that those failures break."""
    from tigerbeetle_amd.types import AccountFlags
    rng = np.random.default_rng(seed)
    acc = sw.accounts
    pick = np.nonzero(rng.random(len(acc)) < 0.35)[0]
    again = acc[pick].copy()
    field = rng.integers(0, 6, len(again))
    again["user_data_128_lo"] += (field == 1).astype(np.uint64)
    again["user_data_64"] += (field == 2).astype(np.uint64)
    again["user_data_32"] += (field == 3).astype(np.uint32)
    again["ledger"] += (field == 4).astype(np.uint32)
    again["code"] += (field == 5).astype(np.uint16)
    flip = field == 0
    again["flags"][flip] ^= np.uint16(int(AccountFlags.history))
    again["timestamp"] = 0
    fresh = acc[:len(again) // 2].copy()
    fresh["id_hi"] = np.uint64(9)  # new ids
    fresh["flags"] = 0
    mixed = np.empty(len(again) + len(fresh), dtype=ACCOUNT_DTYPE)
    order = rng.permutation(len(mixed))
    mixed[order[:len(again)]] = again
    mixed[order[len(again):]] = fresh
    linked = rng.random(len(mixed)) < 0.2
    mixed["flags"] |= np.where(linked, np.uint16(int(AccountFlags.linked)), np.uint16(0)).astype(np.uint16)
    mixed["flags"][-1] &= np.uint16(~int(AccountFlags.linked) & 0xFFFF)
    sw.account_batches = list(sw.account_batches) + [mixed[i:i + 40] for i in range(0, len(mixed), 40)]
    for b in sw.account_batches[-((len(mixed) + 39) // 40):]:
        b["flags"][-1] &= np.uint16(~int(AccountFlags.linked) & 0xFFFF)  # no chain left open
    return sw
