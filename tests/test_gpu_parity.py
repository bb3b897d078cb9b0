"""Bit-exact parity of the HIP engine with the CPU oracle on seeded workloads.

Compares, per batch, the sparse results, then the whole state: every account row,
every stored transfer row in commit order, the account-history rows, the posted
groove and commit_timestamp.
"""
import numpy as np
import pytest

import oracle
from parity import assert_results_equal, assert_state_equal, run_workload
from tigerbeetle_amd import workload

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from tigerbeetle_amd.engine import Engine
    args = dict(accounts_max=1 << 17, transfers_max=1 << 21, history_max=1 << 18, events_per_call_max=1 << 17)
    args.update(kw)
    return Engine(**args)


def _parity(w, split=None, **kw):
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    gpu = _engine(**kw)
    try:
        oa, ot = run_workload(orc, w)
        ga, gt = run_workload(gpu, w, split=split)
        assert_results_equal(ga, oa, "create_accounts")
        assert_results_equal(gt, ot, "create_transfers")
        assert_state_equal(gpu, orc)
        return gpu.stats()
    finally:
        gpu.close()


def test_config1_small():
    _parity(workload.config1(transfer_count=50_000, account_count=1000))


def test_config1_batch_by_batch():
    _parity(workload.config1(transfer_count=20_000, account_count=500), split=1)


def test_config2_small_zipf():
    _parity(workload.config2(transfer_count=100_000, account_count=20_000))


def test_config3_flag_mix():
    _parity(workload.config3(batches=6, batch=2000, account_count=2000))


def test_config3_batch_by_batch():
    _parity(workload.config3(batches=4, batch=1000, account_count=500, seed=7), split=1)


def test_config3_full_batches():
    _parity(workload.config3(batches=4, account_count=10_000, seed=3))


def test_posted_groove():
    w = workload.config3(batches=3, batch=1500, account_count=800, seed=11)
    orc = oracle.Oracle()
    gpu = _engine()
    try:
        run_workload(orc, w)
        run_workload(gpu, w)
        pend = w.transfers[(w.transfers["flags"] & 2) != 0]["id_lo"][:500]
        for pid in pend:
            assert gpu.get_posted(int(pid)) == orc.get_posted(int(pid))
    finally:
        gpu.close()


def test_lookups_match():
    w = workload.config1(transfer_count=5000, account_count=300)
    orc, gpu = oracle.Oracle(), _engine()
    try:
        run_workload(orc, w)
        run_workload(gpu, w)
        ids = list(range(0, 400)) + [(1 << 128) - 1]
        assert gpu.lookup_accounts(ids).tobytes() == orc.lookup_accounts(ids).tobytes()
        tids = list(range(0, 6000, 7)) + [(1 << 128) - 1]
        assert gpu.lookup_transfers(tids).tobytes() == orc.lookup_transfers(tids).tobytes()
    finally:
        gpu.close()
