"""The grooves' field index trees (tbgpu_scan_transfers / tbgpu_scan_accounts;
src/state_machine.zig:1575-1641 tree_options_index, src/lsm/groove.zig:911-936: a stored
object's (field, timestamp) in the field's tree when the field is nonzero).  No operation
of the reference snapshot reads these trees, so no fixture pins them (parity unpinned):
each scan is checked against a numpy reading of the definition over the oracle's stored
objects — every object whose field equals the value, in the timestamp range, in
timestamp order (or reversed), at most the limit — with scans interleaved between
commits so that trees are extended and their runs merged."""
import numpy as np
import pytest

import oracle
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import (ACCOUNT_INDEX_FIELDS, INDEX_FILTER_DTYPE, QUERY_MAX, TRANSFER_INDEX_FIELDS,
                                   IndexField)

pytestmark = pytest.mark.gpu

U128 = {IndexField.debit_account_id: "debit_account_id", IndexField.credit_account_id: "credit_account_id",
        IndexField.user_data_128: "user_data_128", IndexField.pending_id: "pending_id", IndexField.amount: "amount"}
PLAIN = {IndexField.user_data_64: "user_data_64", IndexField.user_data_32: "user_data_32",
         IndexField.timeout: "timeout", IndexField.ledger: "ledger", IndexField.code: "code"}


def _values(rows, field):
    if field in U128:
        name = U128[field]
        return [(int(h) << 64) | int(l) for l, h in zip(rows[name + "_lo"], rows[name + "_hi"])]
    return [int(x) for x in rows[PLAIN[field]]]


def _filter(field, value, ts_min=0, ts_max=0, limit=QUERY_MAX, reversed_=False):
    f = np.zeros(1, dtype=INDEX_FILTER_DTYPE)
    f["value_lo"] = value & (2**64 - 1)
    f["value_hi"] = value >> 64
    f["timestamp_min"], f["timestamp_max"], f["limit"], f["field"] = ts_min, ts_max, limit, int(field)
    f["flags"] = 1 if reversed_ else 0
    return f


def _expected(rows, field, value, ts_min, ts_max, limit, reversed_):
    if value == 0:
        return rows[:0]
    vals = _values(rows, field)
    ts = rows["timestamp"].astype(np.uint64)
    lo = 1 if ts_min == 0 else ts_min
    hi = 2**64 - 2 if ts_max == 0 else ts_max
    sel = np.array([v == value for v in vals], dtype=bool) & (ts >= lo) & (ts <= hi)
    out = rows[sel]
    out = out[np.argsort(out["timestamp"], kind="stable")]
    if reversed_:
        out = out[::-1]
    return out[:min(limit, QUERY_MAX)]


def _check_scans(scan, rows, fields, rng, n):
    for _ in range(n):
        field = fields[rng.integers(0, len(fields))]
        vals = _values(rows, field)
        pick = rng.random()
        value = vals[rng.integers(0, len(vals))] if pick < 0.8 and len(vals) else (0 if pick < 0.9 else 2**100 + 3)
        ts = rows["timestamp"].astype(np.int64)
        ts_min = ts_max = 0
        if rng.random() < 0.5 and len(ts):
            a, b = sorted(rng.integers(int(ts.min()), int(ts.max()) + 1, 2).tolist())
            ts_min, ts_max = a, b
        limit = int(rng.choice([1, 3, 50, QUERY_MAX, 2**31]))
        rev = bool(rng.random() < 0.5)
        got = scan(_filter(field, value, ts_min, ts_max, limit, rev))
        want = _expected(rows, field, value, ts_min, ts_max, limit, rev)
        assert got.tobytes() == want.tobytes(), (field, value, ts_min, ts_max, limit, rev, len(got), len(want))


def test_transfer_and_account_index_scans_match_the_definition():
    from tigerbeetle_amd.engine import Engine
    w = workload.config3(batches=12, batch=2000, account_count=300, seed=21)
    rng = np.random.default_rng(5)
    # accounts with varied user data, ledgers and codes (their index trees)
    acc = w.accounts.copy()
    acc["user_data_64"] = rng.integers(0, 4, len(acc))
    acc["user_data_32"] = rng.integers(0, 3, len(acc))
    acc["user_data_128_lo"] = rng.integers(0, 5, len(acc))
    acc["code"] = rng.integers(1, 4, len(acc))
    orc = oracle.Oracle(len(acc), len(w.transfers))
    gpu = Engine(accounts_max=len(acc) + 16, transfers_max=len(w.transfers) + 1024, history_max=len(w.transfers) + 1024,
                 events_per_call_max=1 << 16)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, acc)
        accounts = orc.export_accounts()
        _check_scans(gpu.scan_accounts, accounts, ACCOUNT_INDEX_FIELDS, rng, 60)
        offs = np.concatenate([[0], np.cumsum(w.transfer_counts.astype(np.int64))])
        nb = len(w.transfer_counts)
        for b0, b1 in ((0, 3), (3, 4), (4, 9), (9, nb)):
            for be in (orc, gpu):
                be.create_transfers_batches(tts[b0:b1], w.transfer_counts[b0:b1], w.transfers[offs[b0]:offs[b1]])
            rows = orc.export_transfers()
            _check_scans(gpu.scan_transfers, rows, TRANSFER_INDEX_FIELDS, rng, 80)
        # invalid filters: a field the accounts groove does not index, a zero limit, reversed bounds,
        # reserved flags and bytes, an unbounded sentinel
        v = _values(rows, IndexField.code)[0]
        assert len(gpu.scan_accounts(_filter(IndexField.amount, 5))) == 0
        for f in (_filter(IndexField.code, v, limit=0), _filter(IndexField.code, v, ts_min=10, ts_max=5),
                  _filter(IndexField.code, v, ts_min=2**64 - 1), _filter(99, v)):
            assert len(gpu.scan_transfers(f)) == 0
        f = _filter(IndexField.code, v)
        f["flags"] = 2
        assert len(gpu.scan_transfers(f)) == 0
        f = _filter(IndexField.code, v)
        f["reserved"] = 1
        assert len(gpu.scan_transfers(f)) == 0
        assert len(gpu.scan_transfers(_filter(IndexField.code, v))) == min(QUERY_MAX, int((rows["code"] == v).sum()))
    finally:
        gpu.close()
