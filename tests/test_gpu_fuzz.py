"""Randomized differential tests: small plain workloads with random mutations at
random positions -- repeated ids (also as the last event of a call), unknown
accounts, zero amounts, reserved flags, linked chains (open at a batch end too),
pending transfers and posts/voids of earlier ones, timeouts, balancing -- committed
whole-call, batch by batch and on the forced general path, every reply and the
whole state bit-exact vs the oracle.  The fast path's eligibility boundaries are
where such mutations land."""
import os
import sys

import numpy as np
import pytest

import oracle
from parity import assert_results_equal, assert_state_equal, run_workload
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import TransferFlags as TF

pytestmark = pytest.mark.gpu


def _mutate(w, rng, rate):
    t = w.transfers.copy()
    n = len(t)
    ends = set((np.cumsum(w.transfer_counts) - 1).tolist())
    pend = []
    for i in range(n):
        if rng.random() >= rate:
            if int(t[i]["flags"]) & int(TF.pending):
                pend.append(i)
            continue
        k = int(rng.integers(0, 11))
        j = int(rng.integers(0, i)) if i else 0
        if k == 0:
            t[i]["id_lo"], t[i]["id_hi"] = t[j]["id_lo"], t[j]["id_hi"]  # repeated id
        elif k == 1:
            t[i]["debit_account_id_lo"] = 10_000 + i            # unknown account
        elif k == 2:
            t[i]["amount_lo"] = 0
        elif k == 3:
            t[i]["flags"] |= np.uint16(1 << 9)                  # reserved flag
        elif k == 4 and i not in ends:
            t[i]["flags"] |= np.uint16(int(TF.linked))          # chain with the next event
        elif k == 5:
            t[i]["flags"] |= np.uint16(int(TF.pending))
            t[i]["timeout"] = int(rng.integers(0, 3))
            pend.append(i)
        elif k in (6, 7) and pend:
            p = pend[int(rng.integers(0, len(pend)))]
            t[i]["flags"] = np.uint16(int(TF.post_pending_transfer if k == 6 else TF.void_pending_transfer))
            t[i]["pending_id_lo"], t[i]["pending_id_hi"] = t[p]["id_lo"], t[p]["id_hi"]
            t[i]["amount_lo"] = 0 if rng.random() < 0.5 else max(1, int(t[p]["amount_lo"]) // 2)
            t[i]["ledger"] = 0
            t[i]["code"] = 0
        elif k == 8:
            t[i]["flags"] |= np.uint16(int(TF.balancing_debit if rng.random() < 0.5 else TF.balancing_credit))
        elif k == 9:
            t[i]["timeout"] = 1                                 # timeout without pending
        elif i:
            t[i]["id_lo"], t[i]["id_hi"] = t[i - 1]["id_lo"], t[i - 1]["id_hi"]  # adjacent repeat
        else:
            t[i]["id_lo"], t[i]["id_hi"] = 0, 0                 # id zero
    if rng.random() < 0.5:
        j = int(rng.integers(0, n - 1))
        t[-1]["id_lo"], t[-1]["id_hi"] = t[j]["id_lo"], t[j]["id_hi"]  # the call's last event repeats an id
    w.transfers = t
    return w


def _check(w, **kw):
    from tigerbeetle_amd.engine import Engine
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    nt = len(w.transfers)
    gpu = Engine(accounts_max=1 << 10, transfers_max=max(1 << 15, 2 * nt), history_max=max(1 << 12, 2 * nt),
                 events_per_call_max=max(1 << 13, nt),
                 force_general=kw.pop("force_general", False), walk_early=kw.pop("walk_early", False))
    try:
        oa, ot = run_workload(orc, w)
        ga, gt = run_workload(gpu, w, **kw)
        assert_results_equal(ga, oa, "create_accounts")
        assert_results_equal(gt, ot, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


@pytest.mark.parametrize("seed", range(96))
def test_fuzz_mutations(seed):
    rng = np.random.default_rng(1000 + seed)
    nb = int(rng.integers(2, 6))
    batch = int(rng.integers(50, 700))
    w = workload.config1(transfer_count=nb * batch, account_count=int(rng.integers(3, 40)), seed=seed,
                         batch=batch)
    rate = [0.0005, 0.005, 0.03, 0.15][seed % 4]
    w = _mutate(w, rng, rate)
    _check(w)
    _check(w, split=1)
    if seed % 3 == 0:
        _check(w, force_general=True)
    if seed % 3 == 1:
        # the sequential walk from the front after two passes (the fixed point's bound)
        _check(w, force_general=True, walk_early=True)


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_random_ids(seed):
    """The same mutations on random u128 ids (benchmark --id-order=random), committed batch
    by batch: from the second call on the fast path claims ids eagerly in fp_commit
    (repeats inside a call, withdrawn claims of broken chains, fallbacks that clear them)."""
    rng = np.random.default_rng(5000 + seed)
    nb = int(rng.integers(3, 7))
    batch = int(rng.integers(50, 700))
    w = workload.config1(transfer_count=nb * batch, account_count=int(rng.integers(3, 40)), seed=seed,
                         batch=batch, id_order="random")
    w = _mutate(w, rng, [0.0005, 0.005, 0.03, 0.15][seed % 4])
    _check(w, split=1)
    if seed % 4 == 0:
        _check(w)


STRESS = os.environ.get("TB_FUZZ_STRESS")  # "first:count": a wider sweep on demand (profiles/r04/fuzz_stress.sh)


@pytest.mark.skipif(not STRESS, reason="the wider sweep runs only with TB_FUZZ_STRESS=first:count")
def test_fuzz_stress_sweep():
    """The same mutations over many more seeds, every one also on the forced general path
    (the passes, the side sort and the headroom scan this sweep is for)."""
    first, count = (int(x) for x in STRESS.split(":"))
    big = os.environ.get("TB_FUZZ_BIG") == "1"  # full-size batches, more accounts
    order = "random" if os.environ.get("TB_FUZZ_RANDOM") == "1" else "sequential"  # random u128 ids
    for seed in range(first, first + count):
        rng = np.random.default_rng(1000 + seed)
        nb = int(rng.integers(2, 6))
        batch = int(rng.integers(500, 8191)) if big else int(rng.integers(50, 700))
        w = workload.config1(transfer_count=nb * batch, account_count=int(rng.integers(3, 300 if big else 40)),
                             seed=seed, batch=batch, id_order=order)
        w = _mutate(w, rng, [0.0005, 0.005, 0.03, 0.15][seed % 4])
        _check(w)
        _check(w, force_general=True)
        if seed % 5 == 0 or order == "random":
            _check(w, split=1)
        if seed % 7 == 0:
            _check(w, force_general=True, walk_early=True)
        if seed % 50 == 0:
            print(f"fuzz stress: seed {seed} ok", flush=True, file=sys.stderr)
