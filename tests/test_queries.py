"""get_account_transfers / get_account_history in the oracle (CPU).

The oracle's C restatement (oracle.c, src/state_machine.zig:693-885, :1128-1196)
against the definitional numpy checker in query_filters.py, over the flag-heavy
config-3 mix (history accounts, two-phase transfers, chains, failures).
"""
import numpy as np
import pytest

import oracle
from parity import run_workload
from query_filters import expected_history, expected_transfers, random_filters
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import U64_MAX, account_filter


@pytest.fixture(scope="module")
def committed():
    w = workload.config3(batches=4, batch=1500, account_count=120, seed=17)
    o = oracle.Oracle(len(w.accounts), len(w.transfers))
    run_workload(o, w)
    return w, o


def test_oracle_account_transfers_match_definition(committed):
    w, o = committed
    rows = o.export_transfers()
    rng = np.random.default_rng(3)
    nonempty = 0
    for f in random_filters(rng, w.accounts["id_lo"], rows, 300):
        got, want = o.get_account_transfers(f), expected_transfers(rows, f)
        assert got.tobytes() == want.tobytes(), f
        nonempty += len(got) > 0
    assert nonempty > 100


def test_oracle_account_history_match_definition(committed):
    w, o = committed
    rows, acc, hist = o.export_transfers(), o.export_accounts(), o.export_history()
    hist_ids = w.accounts["id_lo"][(w.accounts["flags"] & 8) != 0]
    assert len(hist_ids) > 0 and len(hist) > 0
    rng = np.random.default_rng(4)
    nonempty = 0
    for f in random_filters(rng, hist_ids, rows, 150) + random_filters(rng, w.accounts["id_lo"], rows, 50):
        got, want = o.get_account_history(f), expected_history(rows, acc, hist, f)
        assert got.tobytes() == want.tobytes(), f
        nonempty += len(got) > 0
    assert nonempty > 30


def test_invalid_filters_return_nothing(committed):
    w, o = committed
    aid = int(w.accounts["id_lo"][0])
    assert len(o.get_account_transfers(account_filter(aid))) > 0
    bad = [account_filter(0), account_filter((1 << 128) - 1), account_filter(aid, limit=0),
           account_filter(aid, flags=4), account_filter(aid, flags=3 | 8), account_filter(aid, 9, 8),
           account_filter(aid, U64_MAX, 0), account_filter(aid, 0, U64_MAX)]
    r = account_filter(aid)
    r["reserved"][0][23] = 1
    bad.append(r)
    for f in bad:
        assert len(o.get_account_transfers(f)) == 0, f
        assert len(o.get_account_history(f)) == 0, f


def test_limit_and_order(committed):
    w, o = committed
    aid = int(w.accounts["id_lo"][5])
    allr = o.get_account_transfers(account_filter(aid))
    assert len(allr) > 20
    assert np.all(np.diff(allr["timestamp"].astype(np.int64)) > 0)
    rev = o.get_account_transfers(account_filter(aid, flags=7))
    assert rev.tobytes() == allr[::-1].tobytes()
    assert o.get_account_transfers(account_filter(aid, limit=7)).tobytes() == allr[:7].tobytes()
    t = allr["timestamp"]
    mid = o.get_account_transfers(account_filter(aid, int(t[3]), int(t[10])))
    assert mid.tobytes() == allr[3:11].tobytes()
    dr = o.get_account_transfers(account_filter(aid, flags=1))
    assert np.all(dr["debit_account_id_lo"] == aid)
