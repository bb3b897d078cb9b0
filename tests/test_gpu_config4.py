"""BASELINE config 4 at its per-GPU size on one MI355X: 10M accounts over 1000
ledgers (ids ledger << 32 | k, the blocked account directory), 1000 full batches of
8190 transfers (8,190,000) with 1 % cross-ledger linked pairs, streamed as the bench
streams them.  Checked bit for bit against the oracle (every reply, every account row,
every stored transfer row, commit_timestamp), then by conservation per ledger and by
idempotence (src/state_machine.zig:1239-1368, the linked scopes of :1018-1083)."""
import numpy as np
import pytest

import oracle
from parity import sort_accounts
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import CreateTransferResult

pytestmark = pytest.mark.gpu


def _sum128(a, name):
    return int(a[name + "_lo"].astype(object).sum()) + (int(a[name + "_hi"].astype(object).sum()) << 64)


def test_config4_full_size():
    from tigerbeetle_amd.engine import Engine
    ledgers, per_ledger = 1000, 10_000
    w = workload.config4(transfer_count=8_190_000, ledgers=ledgers, accounts_per_ledger=per_ledger, seed=42)
    assert len(w.accounts) == 10_000_000
    ats, tts = w.timestamps()
    orc = oracle.Oracle(len(w.accounts), len(w.transfers) + 8190)
    gpu = Engine(accounts_max=len(w.accounts), transfers_max=len(w.transfers) + 8190, history_max=1024,
                 events_per_call_max=len(w.transfers), dense_block_span=per_ledger)
    try:
        for be in (orc, gpu):
            _, rc = be.create_accounts_batches(ats, w.account_counts, w.accounts)
            assert int(rc.sum()) == 0
        o, orc_rc, _ = orc.create_transfers_batches(tts, w.transfer_counts, w.transfers)
        g, grc, _ = gpu.create_transfers_batches(tts, w.transfer_counts, w.transfers)  # one streamed call
        assert gpu.stats().path == 1, "config 4 stays on the fast path (chains decided by fp_chains)"
        assert np.array_equal(grc, orc_rc)
        n_bad = int(grc.sum())
        assert g[:n_bad].tobytes() == o[:n_bad].tobytes()
        assert gpu.commit_timestamp() == orc.commit_timestamp()
        ga, oa = sort_accounts(gpu.export_accounts()), sort_accounts(orc.export_accounts())
        assert ga.tobytes() == oa.tobytes(), "account rows differ"
        assert gpu.transfer_count() == orc.transfer_count()
        step = 1_000_000
        for k in range(0, gpu.transfer_count(), step):
            assert gpu.export_transfers(k, step).tobytes() == orc.export_transfers(k, step).tobytes(), k
        # conservation per ledger: what a ledger's accounts were debited equals what they
        # were credited, and the total equals the committed amounts
        stored = gpu.export_transfers(0, gpu.transfer_count())
        led = ga["ledger"]
        for name in ("debits_posted", "credits_posted"):
            assert _sum128(ga, name) == _sum128(stored, "amount")
        for L in (1, 500, 1000):
            sel = ga[led == L]
            assert _sum128(sel, "debits_posted") == _sum128(sel, "credits_posted")
        # idempotence: the last batch again answers `exists` for every event (the later
        # members of a linked pair, whose first member now fails, `linked_event_failed`),
        # and nothing moves
        last = w.transfers[-int(w.transfer_counts[-1]):]
        ts = int(tts[-1]) + 1 + len(last)
        r_gpu = gpu.create_transfers(ts, last)
        r_orc = orc.create_transfers(ts, last)
        assert r_gpu.tobytes() == r_orc.tobytes()
        assert len(r_gpu) == len(last)
        assert set(np.unique(r_gpu["result"]).tolist()) <= {int(CreateTransferResult.exists),
                                                             int(CreateTransferResult.linked_event_failed)}
        assert sort_accounts(gpu.export_accounts()).tobytes() == ga.tobytes()
    finally:
        gpu.close()
        orc.close()
