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


@pytest.mark.parametrize("role,mix", [("backup", "config3"), ("primary", "config3"), ("primary", "config1")])
def test_state_machine_prefetch_then_commit(role, mix):
    """The host mirror: prefetch(create_transfers, body) then commit(body) as the
    replica drives it, against the oracle.  A primary also prepares every body two ops
    ahead of its commit (StateMachine.prepare stages it, src/vsr/replica.zig:5159-5167);
    a backup never prepares."""
    from tigerbeetle_amd.state_machine import StateMachine
    w = workload.config3(batches=3, batch=1500, account_count=200, seed=9) if mix == "config3" else \
        workload.config1(transfer_count=8190 * 5, account_count=500, seed=19)
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    sm = StateMachine(engine=_engine(w))
    try:
        ats, tts = w.timestamps()
        orc.create_accounts_batches(ats, w.account_counts, w.accounts)
        sm.engine.create_accounts_batches(ats, w.account_counts, w.accounts)
        sm.commit_timestamp = int(ats[-1])
        bodies = [ev.tobytes() for ev in _batches(w)]
        if role == "primary":
            for body in bodies[:2]:
                sm.prepare(Operation.create_transfers, body)
        for b, ev in enumerate(_batches(w)):
            body = bodies[b]
            if role == "primary" and b + 2 < len(bodies):
                sm.prepare(Operation.create_transfers, bodies[b + 2])
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


@pytest.mark.parametrize("mix,pinned,depth", [("config1", False, 3), ("config1", True, 3), ("config1", True, 11),
                                               ("config3", False, 3), ("config3", False, 11)])
def test_staged_bodies_commit_in_order(mix, pinned, depth):
    """StateMachine.prepare stages each body (tbgpu_stage_transfers) a pipeline's depth
    ahead of its commit, as the primary does (src/vsr/replica.zig:5159-5167, then
    :3137-3152): op k is staged, then op k - depth is prefetched from its slot and
    committed.  Depth 3 stays inside the 8 slots; depth 11 overruns them, so the oldest
    bodies are evicted and their prefetch copies them again.  Both replies and state
    equal the oracle's, for page-locked and pageable bodies and on the general path."""
    import torch
    w = workload.config1(transfer_count=8190 * 14, account_count=700, seed=11) if mix == "config1" else \
        workload.config3(batches=14, batch=1200, account_count=300, seed=12)
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    gpu = _engine(w, pinned_input=pinned)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        bs = _batches(w)
        if pinned:
            from tigerbeetle_amd.types import TRANSFER_DTYPE
            keep = []
            for b, ev in enumerate(bs):
                t = torch.empty(max(len(ev), 1) * 128, dtype=torch.uint8, pin_memory=True)
                v = t.numpy().view(TRANSFER_DTYPE)[:len(ev)]
                v[:] = ev
                keep.append(t)
                bs[b] = v
        got, want = [], []
        key = lambda b: (0xB0D1 << 64) | (b * 7919 + 1)  # any content key, one per body
        for k in range(len(bs) + depth):
            if k < len(bs):
                gpu.stage_transfers(key(k), bs[k])
            b = k - depth
            if b < 0:
                continue
            gpu.prefetch_transfers_staged(key(b), bs[b])
            gpu.prefetch_wait()
            got.append(gpu.create_transfers(int(tts[b]), bs[b]))
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], bs[b])
            want.append(res[:int(rc[0])].copy())
        assert_results_equal(got, want, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_stage_key_mismatch_and_interleaved_calls():
    """A prefetch whose key no slot holds (or whose count differs) copies its body; a
    stage call between a prefetch and its commit does not release the prepared commit
    and does not disturb it (its own prepared commit queues behind, and is dropped when
    the next prefetch names another body); a lookup in between does release it; staged
    commits whose gates ran out (the commit came after the budget) take the ordinary
    path.  Replies equal the oracle's throughout."""
    import time
    w = workload.config1(transfer_count=8190 * 8, account_count=500, seed=13)
    orc, gpu = oracle.Oracle(len(w.accounts), len(w.transfers)), _engine(w)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        bs = _batches(w)
        got, want = [], []
        for b, ev in enumerate(bs):
            if b == 0:
                gpu.stage_transfers(100, ev[:-1])      # same key, another count: not this body
                gpu.prefetch_transfers_staged(100, ev)
            elif b == 1:
                gpu.prefetch_transfers_staged(555, ev)  # never staged
            elif b == 5:
                for k in range(3):  # three prepared commits queued ...
                    gpu.stage_transfers(500 + b + k, bs[b + k])
                time.sleep(0.05)    # ... whose gates all run out before the commits come
                gpu.prefetch_transfers_staged(500 + b, ev)
            elif b in (6, 7):
                gpu.prefetch_transfers_staged(500 + b, ev)
            else:
                gpu.stage_transfers(200 + b, ev)
                gpu.prefetch_transfers_staged(200 + b, ev)
                if b == 3:
                    gpu.stage_transfers(900, bs[0])     # staging between prefetch and commit
                if b == 4:
                    assert len(gpu.lookup_accounts([1, 2])) == 2  # releases the gate
            gpu.prefetch_wait()
            got.append(gpu.create_transfers(int(tts[b]), ev))
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], ev)
            want.append(res[:int(rc[0])].copy())
        assert_results_equal(got, want, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_prepared_commit_with_failures_writes_only_its_replies():
    """A prepared (gated) commit whose batch has fast-path failures -- ids committed by
    an earlier batch (`exists`, `exists_with_different_*`) and static failures -- writes
    exactly its sparse replies and leaves the caller's buffer past them untouched
    (the whole event count used to be copied)."""
    import ctypes
    from tigerbeetle_amd.types import RESULT_DTYPE
    w = workload.config1(transfer_count=8190 * 3, account_count=400, seed=14)
    orc, gpu = oracle.Oracle(len(w.accounts), len(w.transfers) * 2), _engine(w)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        bs = _batches(w)
        bad = bs[2].copy()
        rng = np.random.default_rng(3)
        pick = rng.choice(len(bad), 40, replace=False)
        bad["id_lo"][pick[:20]] = bs[0]["id_lo"][pick[:20]]      # committed by batch 0
        bad["amount_lo"][pick[10:20]] += 1                       # ... with another amount
        bad["credit_account_id_lo"][pick[20:30]] = bad["debit_account_id_lo"][pick[20:30]]
        bad["code"][pick[30:]] = 0
        bodies = [bs[0], bs[1], np.ascontiguousarray(bad)]
        for b, ev in enumerate(bodies):
            gpu.prefetch_transfers(ev)
            gpu.prefetch_wait()
            out = np.full(len(ev) + 8, 0xABABABABABABABAB, dtype=np.uint64).view(RESULT_DTYPE)
            n = gpu._L.tbgpu_create_transfers(gpu._h, int(tts[b]), ev.ctypes.data_as(ctypes.c_void_p), len(ev),
                                              out.ctypes.data_as(ctypes.c_void_p))
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], np.array([len(ev)], np.uint32), ev)
            assert n == int(rc[0]), (b, n, int(rc[0]))
            assert out[:n].tobytes() == res[:n].tobytes(), b
            assert (out[n:].view(np.uint64) == 0xABABABABABABABAB).all(), f"batch {b}: replies past the count written"
        assert n == 40
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_staged_random_schedules(seed):
    """Random schedules of the drop-in entry points, as a primary, a backup and other
    callers would interleave them: staging up to 6 bodies ahead (tbgpu_stage_transfers,
    each queuing its prepared commit), staged and plain prefetches, commits with and
    without a prefetch, lookups and streamed calls in between (each releases whatever
    is prepared), bodies staged twice or never committed, a gap past the gates' budget.
    Mixes with failures, chains, two-phase transfers and (seeds 3-4) random u128 ids.
    Every reply and the final state equal the oracle's."""
    import time
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    rng = np.random.default_rng(100 + seed)
    if seed % 2:
        w = workload.config3(batches=24, batch=int(rng.integers(300, 1500)), account_count=300, seed=seed)
    else:
        w = workload.config1(transfer_count=24 * 1200, account_count=400, seed=seed, batch=1200,
                             id_order="random" if seed >= 3 else "sequential")
    orc = oracle.Oracle(len(w.accounts), len(w.transfers) + 1024)
    gpu = _engine(w, pinned_input=seed >= 3)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        bs = _batches(w)
        if seed >= 3:  # page-locked bodies (the copy kernels read them in place)
            import torch
            keep = []
            for b, ev in enumerate(bs):
                t = torch.empty(max(len(ev), 1) * 128, dtype=torch.uint8, pin_memory=True)
                v = t.numpy().view(TRANSFER_DTYPE)[:len(ev)]
                v[:] = ev
                keep.append(t)
                bs[b] = v
        key = lambda b: (seed << 96) | (b * 2654435761 + 7)
        staged = 0  # bodies staged so far (in commit order)
        got, want = [], []
        for b, ev in enumerate(bs):
            # stage ahead, as prepares arrive
            ahead = int(rng.integers(0, 7))
            while staged < min(len(bs), b + 1 + ahead):
                gpu.stage_transfers(key(staged), bs[staged])
                if rng.random() < 0.1:
                    gpu.stage_transfers(key(staged), bs[staged])  # the same body again: nothing new
                staged += 1
            r = rng.random()
            if r < 0.03:
                time.sleep(0.03)  # past the gates' budget
            elif r < 0.08:
                q = [int(w.accounts["id_lo"][k]) | (int(w.accounts["id_hi"][k]) << 64) for k in range(3)]
                assert len(gpu.lookup_accounts(q)) == 3  # releases what is prepared
            elif r < 0.11 and b + 1 < len(bs):
                gpu.stage_transfers(key(10_000 + b), bs[b + 1][:-1])  # a body that never commits
            mode = rng.random()
            if mode < 0.7:
                gpu.prefetch_transfers_staged(key(b), ev)
                gpu.prefetch_wait()
            elif mode < 0.85:
                gpu.prefetch_transfers(ev)
                gpu.prefetch_wait()
            got.append(gpu.create_transfers(int(tts[b]), ev))
            res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], ev)
            want.append(res[:int(rc[0])].copy())
        assert_results_equal(got, want, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_new_ctx_after_another_on_recycled_memory():
    """Contexts one after another, each with the same sizes (so the allocator tends to
    hand a new ctx the memory of the last one): a ctx's prepared-commit verdict word,
    its clean create_accounts ticket and its small calls' sequence word are matched
    against values every ctx repeats (sequence numbers restart at 1), so a new ctx must
    not read the previous one's.  Each ctx's stream has other timestamps."""
    for k in range(4):
        w = workload.config1(transfer_count=12_000, account_count=600, seed=20 + k)
        orc, gpu = oracle.Oracle(len(w.accounts), len(w.transfers)), _engine(w)
        try:
            ats, tts = w.timestamps(start=1_000_000 * k)
            for be in (orc, gpu):
                be.create_accounts_batches(ats, w.account_counts, w.accounts)
            got, want = [], []
            for b, ev in enumerate(_batches(w)):
                gpu.prefetch_transfers(ev)
                got.append(gpu.create_transfers(int(tts[b]), ev))
                res, rc, _ = orc.create_transfers_batches(tts[b:b + 1], w.transfer_counts[b:b + 1], ev)
                want.append(res[:int(rc[0])].copy())
            assert_results_equal(got, want, "create_transfers")
            assert_state_equal(gpu, orc)
        finally:
            gpu.close()
