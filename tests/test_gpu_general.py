"""The general (fixed-point) create_transfers path at BASELINE config 3's shape.

Whole streamed calls of full 8190-event batches over 10k accounts are committed by
the GPU and by the oracle and compared bit for bit: every reply, every account row,
every stored transfer row, the account history, the posted groove and
commit_timestamp.  Calls of 60 and 200 batches exercise the engine's chunking of
long calls (a failed single-pass attempt, the split into general-path-sized
chunks, the periodic fast re-attempt: `transfers_batches` in csrc/engine.hip);
the mixed stream switches between the two paths inside one call; the stress mix
(~40 % non-ok) and the adversarial dependency chain push the fixed point's pass
count.  Reference: `execute` (src/state_machine.zig:1018-1083).
"""
import numpy as np
import pytest

import oracle
from parity import assert_results_equal, assert_state_equal, run_workload
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import BATCH_MAX, TRANSFER_DTYPE, AccountFlags

pytestmark = pytest.mark.gpu


def _engine(w, **kw):
    from tigerbeetle_amd.engine import Engine
    n = len(w.transfers)
    args = dict(accounts_max=max(len(w.accounts), 1024), transfers_max=n + 1024, history_max=n + 1024,
                events_per_call_max=max(int(w.transfer_counts.max()) * 2, min(n, 210 * BATCH_MAX)))
    args.update(kw)
    return Engine(**args)


def _parity(w, split=None, **kw):
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    gpu = _engine(w, **kw)
    try:
        oa, ot = run_workload(orc, w)
        ga, gt = run_workload(gpu, w, split=split)
        assert_results_equal(ga, oa, "create_accounts")
        assert_results_equal(gt, ot, "create_transfers")
        assert_state_equal(gpu, orc)
        non_ok = sum(len(r) for r in ot)
        return gpu.stats(), non_ok / len(w.transfers)
    finally:
        gpu.close()


@pytest.mark.parametrize("batches", [60, 200])
def test_config3_baseline_whole_call(batches):
    """10k accounts, full batches, the whole run (funding batch + `batches`) in one call."""
    w = workload.config3(batches=batches, account_count=10_000, seed=42)
    st, rate = _parity(w)
    assert 0.05 < rate < 0.15, rate  # BASELINE config 3: ~10 % non-ok


def test_config3_baseline_chunked_calls():
    """The same stream as 24-batch calls (each cut again into general-path chunks)."""
    w = workload.config3(batches=96, account_count=10_000, seed=5)
    _parity(w, split=24)


@pytest.mark.parametrize("split", [None, 24])
def test_config3_mixed_paths_in_one_call(split):
    """Plain batches (single-pass path), then flag-heavy ones, then plain again, in
    one streamed call: the fast attempt fails, the call is redone in small chunks,
    and the fast path is re-attempted on the plain tail."""
    plain = list(range(0, 20)) + list(range(36, 60))
    w = workload.config3(batches=60, account_count=10_000, seed=8, plain_batches=plain)
    _parity(w, split=split)


def test_config3_forced_general_whole_call():
    w = workload.config3(batches=40, account_count=10_000, seed=9)
    _parity(w, force_general=True)


@pytest.mark.parametrize("batches,split", [(40, None), (40, 7)])
def test_config3_stress_mix(batches, split):
    """Round 1's ~40 %-non-ok mix: resolved or expired pendings, drained limit accounts."""
    w = workload.config3_stress(batches=batches, account_count=10_000, seed=4)
    _parity(w, split=split)


def _relay_chain(n: int, accounts: int, relay: int, fund: int = 0):
    """One batch where event k moves 10 units from account k to account k+1 (all
    debits_must_not_exceed_credits): every event's outcome depends on its
    predecessor's, a dependency chain as long as the batch.  Account 1 receives `fund`
    credits first, so with fund=0 every relay fails -- as far from the fixed point's
    optimistic start (every statically valid event succeeds) as a batch can be: a
    plain Jacobi sweep needs one pass per event -- and with fund=10 every relay
    succeeds (the optimistic start is right)."""
    acc = workload.make_accounts(np.arange(1, accounts + 1, dtype=np.uint64), ledger=1,
                                 flags=int(AccountFlags.debits_must_not_exceed_credits))
    acc[-1]["flags"] = 0  # the funding source
    src = accounts
    t = np.zeros(n + 1, dtype=TRANSFER_DTYPE)
    t["id_lo"] = np.arange(1, n + 2)
    t["ledger"] = 1
    t["code"] = 1
    t[0]["debit_account_id_lo"] = src
    t[0]["credit_account_id_lo"] = 1
    t[0]["amount_lo"] = max(fund, 1)
    if fund == 0:
        t[0]["debit_account_id_lo"] = accounts + 99  # the funding transfer fails: not found
    for k in range(1, n + 1):
        a = (k - 1) % relay + 1
        t[k]["debit_account_id_lo"] = a
        t[k]["credit_account_id_lo"] = a % relay + 1
        t[k]["amount_lo"] = 10
    return workload.Workload("relay", acc, np.array([len(acc)], dtype=np.uint32), t,
                             np.array([n + 1], dtype=np.uint32))


@pytest.mark.parametrize("fund", [0, 10])
def test_adversarial_relay_chain(fund):
    """A whole batch is one dependency chain; exact results whatever the depth.  With
    fund=0 the passes would need one per event (O(n^2)); past the pass budget the
    engine walks the rest of the batch in execute's order (tr_walk), so the call is
    bounded by O(n) work."""
    w = _relay_chain(BATCH_MAX - 1, accounts=BATCH_MAX + 1, relay=BATCH_MAX, fund=fund)
    st, _ = _parity(w)
    print(f"relay chain fund={fund}: {st.iterations} passes, path {st.path}, {st.device_ms:.2f} ms device time "
          f"for the {BATCH_MAX}-event batch")
    if fund == 0:
        assert st.path == 2 and st.iterations <= 64 + 48, (st.path, st.iterations)
        assert st.device_ms < 100.0, st.device_ms
    else:
        assert st.iterations <= 2


@pytest.mark.parametrize("kind", ["config3", "stress"])
def test_walk_matches_the_passes(kind):
    """The walk from the front after two passes (TBGPU_OPT_WALK_EARLY) on the flag-heavy
    mixes: chains, two-phase, balancing, limits, duplicates, expiry -- the same results
    and state as the oracle (and so as the converged passes)."""
    mk = workload.config3 if kind == "config3" else workload.config3_stress
    w = mk(batches=6, account_count=2_000, seed=21)
    st, _ = _parity(w, split=2, force_general=True, walk_early=True)
    assert st.walks > 0, st.walks
