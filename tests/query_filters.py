"""Filters and a definitional checker for get_account_transfers / get_account_history.

`expected_*` restate the two queries directly from their definition in the
reference (src/state_machine.zig:822-885 scan conditions and validity, :1128-1196
outputs) over exported state, with numpy: an independent check of the oracle's C
restatement.  No reference fixture covers these queries (its table tests have
none, and its workload leaves them unimplemented: src/state_machine/workload.zig:
365-366), so their parity is pinned to that definition, not to reference outputs.
"""
from __future__ import annotations

import numpy as np

from tigerbeetle_amd.types import (BALANCE_DTYPE, QUERY_MAX, TRANSFER_DTYPE, U64_MAX, AccountFlags,
                                   account_filter)


def _id(rec, name):
    return (int(rec[name + "_hi"]) << 64) | int(rec[name + "_lo"])


def valid(f) -> bool:
    """get_scan_from_filter's validity test (src/state_machine.zig:822-833)."""
    f = f.reshape(-1)[0]
    aid = _id(f, "account_id")
    tmin, tmax = int(f["timestamp_min"]), int(f["timestamp_max"])
    return (aid != 0 and aid != (1 << 128) - 1 and tmin != U64_MAX and tmax != U64_MAX
            and (tmax == 0 or tmin <= tmax) and int(f["limit"]) != 0 and (int(f["flags"]) & 3) != 0
            and (int(f["flags"]) >> 3) == 0 and not f["reserved"].any())


def _scan(rows, f):
    f = f.reshape(-1)[0]
    aid = _id(f, "account_id")
    lo, hi = aid & U64_MAX, aid >> 64
    tmin = int(f["timestamp_min"]) or 1
    tmax = int(f["timestamp_max"]) or U64_MAX - 1
    fl = int(f["flags"])
    m = np.zeros(len(rows), dtype=bool)
    if fl & 1:
        m |= (rows["debit_account_id_lo"] == lo) & (rows["debit_account_id_hi"] == hi)
    if fl & 2:
        m |= (rows["credit_account_id_lo"] == lo) & (rows["credit_account_id_hi"] == hi)
    m &= (rows["timestamp"] >= tmin) & (rows["timestamp"] <= tmax)
    idx = np.nonzero(m)[0]
    idx = idx[np.argsort(rows["timestamp"][idx], kind="stable")]
    if fl & 4:
        idx = idx[::-1]
    return idx, min(int(f["limit"]), QUERY_MAX), aid


def expected_transfers(rows, f):
    if not valid(f):
        return np.zeros(0, dtype=TRANSFER_DTYPE)
    idx, limit, _ = _scan(rows, f)
    return rows[idx[:limit]]


def expected_history(rows, accounts, hist, f):
    if not valid(f):
        return np.zeros(0, dtype=BALANCE_DTYPE)
    idx, limit, aid = _scan(rows, f)
    acc = accounts[(accounts["id_lo"] == (aid & U64_MAX)) & (accounts["id_hi"] == (aid >> 64))]
    if len(acc) == 0 or not (int(acc[0]["flags"]) & int(AccountFlags.history)):
        return np.zeros(0, dtype=BALANCE_DTYPE)
    by_ts = {int(h["timestamp"]): h for h in hist}
    out = []
    for i in idx:
        h = by_ts.get(int(rows[i]["timestamp"]))
        if h is None:
            continue  # post/void: no history row (the reference's lookup would assert)
        b = np.zeros(1, dtype=BALANCE_DTYPE)
        side = "dr" if _id(h, "dr_account_id") == aid else "cr"
        for fld in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
            b[fld + "_lo"] = h[f"{side}_{fld}_lo"]
            b[fld + "_hi"] = h[f"{side}_{fld}_hi"]
        b["timestamp"] = h["timestamp"]
        out.append(b)
        if len(out) == limit:
            break
    return np.concatenate(out) if out else np.zeros(0, dtype=BALANCE_DTYPE)


def random_filters(rng, account_ids, rows, n: int) -> list:
    """Filters over real accounts with timestamp bounds drawn from stored rows, and
    every kind of invalid filter (:822-833)."""
    ts = rows["timestamp"] if len(rows) else np.array([1], dtype=np.uint64)
    out = []
    for _ in range(n):
        aid = int(account_ids[int(rng.integers(0, len(account_ids)))])
        roll = rng.random()
        if roll < 0.03:
            aid = 0
        elif roll < 0.05:
            aid = (1 << 128) - 1
        elif roll < 0.08:
            aid = 10**9 + int(rng.integers(0, 1000))  # no such account
        t0 = int(ts[int(rng.integers(0, len(ts)))])
        t1 = int(ts[int(rng.integers(0, len(ts)))])
        tmin, tmax = [(0, 0), (min(t0, t1), max(t0, t1)), (t0, 0), (0, t1)][int(rng.integers(0, 4))]
        limit = [1, 3, 100, 8190, 10_000, 1 << 31][int(rng.integers(0, 6))]
        flags = int(rng.integers(1, 4)) | (4 if rng.random() < 0.4 else 0)
        f = account_filter(aid, tmin, tmax, limit, flags)
        bad = rng.random()
        if bad < 0.02:
            f["limit"] = 0
        elif bad < 0.04:
            f["flags"] = 4  # neither debits nor credits
        elif bad < 0.06:
            f["flags"] |= 8  # padding
        elif bad < 0.08:
            f["reserved"][0][int(rng.integers(0, 24))] = 1
        elif bad < 0.10:
            f["timestamp_min"], f["timestamp_max"] = 5, 4
        elif bad < 0.11:
            f["timestamp_min"] = U64_MAX
        elif bad < 0.12:
            f["timestamp_max"] = U64_MAX
        out.append(f)
    return out
