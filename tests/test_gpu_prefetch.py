"""StateMachine.prefetch for create_transfers (tbgpu_prefetch_transfers): the batch is
staged in HBM before its commit (src/state_machine.zig:514-655; the replica commits
after the prefetch callback, src/vsr/replica.zig:3384-3415).  Replies and the final
state must equal the oracle's, whether a commit uses the staged copy or not."""
import numpy as np
import pytest

import oracle
from parity import assert_results_equal, assert_state_equal
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import Operation

pytestmark = pytest.mark.gpu


def _engine(w, **kw):
    from tigerbeetle_amd.engine import Engine
    args = dict(accounts_max=len(w.accounts) + 16, transfers_max=len(w.transfers) + 1024,
                history_max=len(w.transfers) + 1024, events_per_call_max=1 << 16)
    args.update(kw)
    return Engine(**args)


def _batches(w):
    offs = np.concatenate([[0], np.cumsum(w.transfer_counts.astype(np.int64))])
    return [np.ascontiguousarray(w.transfers[offs[b]:offs[b + 1]]) for b in range(len(w.transfer_counts))]


@pytest.mark.parametrize("mix", ["config1", "config3"])
def test_prefetched_commits_match_oracle(mix):
    w = workload.config1(transfer_count=40_000, account_count=700, seed=3) if mix == "config1" else \
        workload.config3(batches=5, batch=2000, account_count=300, seed=5)
    orc, gpu = oracle.Oracle(len(w.accounts), len(w.transfers)), _engine(w)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        got, want = [], []
        for b, ev in enumerate(_batches(w)):
            if b % 3 != 2:  # most batches prefetched; every third committed without it
                gpu.prefetch_transfers(ev)
                if b % 2:
                    gpu.prefetch_wait()
            got.append(gpu.create_transfers(int(tts[b]), ev))
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], ev)
            want.append(res[:int(rc[0])].copy())
        assert_results_equal(got, want, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_prefetch_of_another_body_is_not_used():
    """A commit whose body is not the prefetched one copies its own events; a prefetch
    discarded by a streamed call is not used later either."""
    w = workload.config1(transfer_count=30_000, account_count=500, seed=4)
    orc, gpu = oracle.Oracle(len(w.accounts), len(w.transfers)), _engine(w)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        bs = _batches(w)
        got, want = [], []
        for b in range(len(bs)):
            # stage the NEXT batch's body, then commit this one (a different buffer)
            if b + 1 < len(bs):
                gpu.prefetch_transfers(bs[b + 1])
            if b == 1:
                # a streamed call between prefetch and commit discards the staged copy
                res, rc, _ = gpu.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], bs[b])
                got.append(res[:int(rc[0])].copy())
            else:
                got.append(gpu.create_transfers(int(tts[b]), bs[b]))
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], bs[b])
            want.append(res[:int(rc[0])].copy())
        assert_results_equal(got, want, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_state_machine_prefetch_then_commit():
    """The host mirror: prefetch(create_transfers, body) then commit(body) as the
    replica drives it, against the oracle."""
    from tigerbeetle_amd.state_machine import StateMachine
    w = workload.config3(batches=3, batch=1500, account_count=200, seed=9)
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    sm = StateMachine(engine=_engine(w))
    try:
        ats, tts = w.timestamps()
        orc.create_accounts_batches(ats, w.account_counts, w.accounts)
        sm.engine.create_accounts_batches(ats, w.account_counts, w.accounts)
        sm.commit_timestamp = int(ats[-1])
        for b, ev in enumerate(_batches(w)):
            body = ev.tobytes()
            done = []
            sm.prefetch(lambda _: done.append(True), b + 1, Operation.create_transfers, body)
            assert done
            reply = sm.commit(0, b + 1, int(tts[b]), Operation.create_transfers, body)
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], ev)
            assert reply == res[:int(rc[0])].tobytes(), b
        assert_state_equal(sm.engine, orc)
    finally:
        sm.engine.close()


def test_prepared_commit_gate_released_expired_and_cancelled():
    """A prefetch prepares the commit (its launches wait behind a gate for the commit's
    timestamp).  Whatever happens between prefetch and commit the replies and the state
    equal the oracle's: the commit right away (the gate lets the prepared launches
    through), the commit after the gate's 10-ms budget (nothing went through: an
    ordinary call), another call in between (a lookup releases the gate), a second
    prefetch (releases the first), and a prefetch followed by a different call only."""
    import time
    w = workload.config1(transfer_count=8190 * 8, account_count=600, seed=6)
    orc, gpu = oracle.Oracle(len(w.accounts), len(w.transfers)), _engine(w)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        bs = _batches(w)
        q = [1, 2, 3]  # account ids
        got, want = [], []
        for b, ev in enumerate(bs):
            mode = b % 5
            if mode == 0:
                gpu.prefetch_transfers(ev)
                gpu.prefetch_wait()
            elif mode == 1:
                gpu.prefetch_transfers(ev)
                time.sleep(0.03)  # past the gate's budget
            elif mode == 2:
                gpu.prefetch_transfers(ev)
                assert len(gpu.lookup_accounts(q)) == 3  # releases the gate
            elif mode == 3:
                gpu.prefetch_transfers(bs[(b + 1) % len(bs)])
                gpu.prefetch_transfers(ev)  # releases the first preparation
            # mode 4: no prefetch at all
            got.append(gpu.create_transfers(int(tts[b]), ev))
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], ev)
            want.append(res[:int(rc[0])].copy())
        # a prefetch no commit follows, then a lookup and the end of the engine
        gpu.prefetch_transfers(bs[0])
        assert len(gpu.lookup_accounts(q)) == 3
        assert_results_equal(got, want, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()
