"""BASELINE config 2 at its full size on the GPU: 1M accounts, 1000 batches of 8190
Zipf(0.99) transfers (8,190,000), streamed as the bench streams them.  Checked
bit for bit against the oracle (every reply, every account row, every stored
transfer row, commit_timestamp) and through size-independent properties:
conservation (total debits == total credits == total amount committed) and
idempotence (re-submitting a committed batch changes nothing and answers
`exists` for every event)."""
import numpy as np
import pytest

import oracle
from parity import assert_results_equal, per_batch_results, sort_accounts
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import CreateTransferResult

pytestmark = pytest.mark.gpu


def _sum128(a, name):
    return int(a[name + "_lo"].astype(object).sum()) + (int(a[name + "_hi"].astype(object).sum()) << 64)


def test_config2_full_size():
    from tigerbeetle_amd.engine import Engine
    w = workload.config2(transfer_count=8_190_000, account_count=1_000_000, seed=42)
    ats, tts = w.timestamps()
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    gpu = Engine(accounts_max=len(w.accounts), transfers_max=len(w.transfers) + 8190, history_max=1024,
                 events_per_call_max=len(w.transfers))
    try:
        for be in (orc, gpu):
            _, rc = be.create_accounts_batches(ats, w.account_counts, w.accounts)
            assert int(rc.sum()) == 0
        o, orc_rc, _ = orc.create_transfers_batches(tts, w.transfer_counts, w.transfers)
        g, grc, _ = gpu.create_transfers_batches(tts, w.transfer_counts, w.transfers)  # one streamed call
        assert gpu.stats().path == 1
        assert int(grc.sum()) == 0 and int(orc_rc.sum()) == 0
        assert gpu.commit_timestamp() == orc.commit_timestamp()
        ga, oa = sort_accounts(gpu.export_accounts()), sort_accounts(orc.export_accounts())
        assert ga.tobytes() == oa.tobytes()
        assert gpu.transfer_count() == orc.transfer_count() == len(w.transfers)
        step = 1_000_000
        for k in range(0, len(w.transfers), step):
            assert gpu.export_transfers(k, step).tobytes() == orc.export_transfers(k, step).tobytes(), k
        # conservation: every committed amount is debited once and credited once
        total = _sum128(w.transfers, "amount")
        assert _sum128(ga, "debits_posted") == _sum128(ga, "credits_posted") == total
        assert _sum128(ga, "debits_pending") == _sum128(ga, "credits_pending") == 0
        # idempotence: the last batch again (next timestamp) answers `exists` everywhere
        last = w.transfers[-int(w.transfer_counts[-1]):]
        ts = int(tts[-1]) + 1 + len(last)
        r_gpu = gpu.create_transfers(ts, last)
        r_orc = orc.create_transfers(ts, last)
        assert r_gpu.tobytes() == r_orc.tobytes()
        assert len(r_gpu) == len(last) and np.all(r_gpu["result"] == int(CreateTransferResult.exists))
        assert sort_accounts(gpu.export_accounts()).tobytes() == ga.tobytes()
    finally:
        gpu.close()


@pytest.mark.parametrize("order", ["random", "reversed"])
def test_config1_full_size_id_orders(order):
    """BASELINE config 1 at its full size (10k accounts, 10M transfers: 1221 batches of
    8190 and one of 10) with the reference benchmark's --id-order (src/tigerbeetle/
    cli.zig:205, IdPermutation src/testing/id.zig:28-48): u128 pseudo-UUID or
    descending ids, so the hashed account index, the hashed id insert and the call's
    duplicate check, never the direct-mapped directory or the sorted id run.  Streamed
    in 1000-batch calls as the bench streams them, bit for bit against the oracle,
    then idempotence: a committed batch again answers `exists` everywhere."""
    from tigerbeetle_amd.engine import Engine
    w = workload.config1(transfer_count=10_000_000, account_count=10_000, seed=42, id_order=order)
    assert int(w.accounts["id_hi"].max()) != 0  # not the directory's ids
    ats, tts = w.timestamps()
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    gpu = Engine(accounts_max=len(w.accounts), transfers_max=len(w.transfers) + 8190, history_max=1024,
                 events_per_call_max=1000 * 8190)
    try:
        for be in (orc, gpu):
            _, rc = be.create_accounts_batches(ats, w.account_counts, w.accounts)
            assert int(rc.sum()) == 0
        counts = w.transfer_counts
        off = 0
        for b0 in range(0, len(counts), 1000):
            b1 = min(b0 + 1000, len(counts))
            m = int(counts[b0:b1].sum())
            g, grc, _ = gpu.create_transfers_batches(tts[b0:b1], counts[b0:b1], w.transfers[off:off + m])
            assert gpu.stats().path == 1, "the fast path did not take the call"
            o, orc_rc, _ = orc.create_transfers_batches(tts[b0:b1], counts[b0:b1], w.transfers[off:off + m])
            assert np.array_equal(grc, orc_rc) and int(grc.sum()) == 0
            off += m
        assert gpu.commit_timestamp() == orc.commit_timestamp()
        ga, oa = sort_accounts(gpu.export_accounts()), sort_accounts(orc.export_accounts())
        assert ga.tobytes() == oa.tobytes()
        step = 1_000_000
        for k in range(0, len(w.transfers), step):
            assert gpu.export_transfers(k, step).tobytes() == orc.export_transfers(k, step).tobytes(), k
        total = _sum128(w.transfers, "amount")
        assert _sum128(ga, "debits_posted") == _sum128(ga, "credits_posted") == total
        first = w.transfers[:int(counts[0])]
        ts = int(tts[-1]) + 1 + len(first)
        r_gpu = gpu.create_transfers(ts, first)
        assert r_gpu.tobytes() == orc.create_transfers(ts, first).tobytes()
        assert len(r_gpu) == len(first) and np.all(r_gpu["result"] == int(CreateTransferResult.exists))
        lk = w.transfers["id_lo"][::99_991].copy(), w.transfers["id_hi"][::99_991].copy()
        from tigerbeetle_amd.types import U128_DTYPE
        q = np.zeros(len(lk[0]), dtype=U128_DTYPE)
        q["lo"], q["hi"] = lk
        assert gpu.lookup_transfers(q).tobytes() == orc.lookup_transfers(q).tobytes()
    finally:
        gpu.close()
