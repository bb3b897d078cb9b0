"""Checkpoint / open (tbgpu_checkpoint, tbgpu_open): the StateMachine.checkpoint /
open pair (src/state_machine.zig:486-500, :957-970).  A run is checkpointed half
way, restored into a fresh engine, and continued there: every later reply, the
final state and the queries must equal the uninterrupted oracle's, and the image
of the restored engine must equal the original's byte for byte."""
import numpy as np
import pytest

import oracle
from parity import assert_results_equal, assert_state_equal, per_batch_results
from query_filters import random_filters
from tigerbeetle_amd import workload

pytestmark = pytest.mark.gpu


def _engine(w):
    from tigerbeetle_amd.engine import Engine
    return Engine(accounts_max=len(w.accounts) + 16, transfers_max=len(w.transfers) + 1024,
                  history_max=len(w.transfers) + 1024, events_per_call_max=1 << 16)


def _run(be, w, tts, b0, b1, off):
    counts = list(w.transfer_counts)
    n = int(sum(counts[b0:b1]))
    res, rcs, _ = be.create_transfers_batches(tts[b0:b1], counts[b0:b1], w.transfers[off:off + n])
    return per_batch_results(res, counts[b0:b1], rcs), off + n


@pytest.mark.parametrize("config", [1, 3])
def test_checkpoint_restore_continue(config):
    if config == 3:
        w = workload.config3(batches=6, batch=1500, account_count=400, seed=12)
    else:
        w = workload.config1(transfer_count=60_000, account_count=500, seed=12)
    ats, tts = w.timestamps()
    nb = len(w.transfer_counts)
    half = nb // 2
    orc, a = oracle.Oracle(len(w.accounts), len(w.transfers)), _engine(w)
    b = _engine(w)
    try:
        for be in (orc, a):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        want1, off_o = _run(orc, w, tts, 0, half, 0)
        got1, off = _run(a, w, tts, 0, half, 0)
        assert_results_equal(got1, want1)
        image = a.checkpoint()
        assert b.open(image) == 0
        assert np.array_equal(b.checkpoint(), image), "restored image differs"
        assert_state_equal(b, a)
        want2, _ = _run(orc, w, tts, half, nb, off_o)
        got2, _ = _run(b, w, tts, half, nb, off)
        assert_results_equal(got2, want2)
        assert_state_equal(b, orc)
        rows = orc.export_transfers()
        for f in random_filters(np.random.default_rng(1), w.accounts["id_lo"], rows, 60):
            assert b.get_account_transfers(f).tobytes() == orc.get_account_transfers(f).tobytes()
        # the uninterrupted engine agrees too
        _run(a, w, tts, half, nb, off)
        assert np.array_equal(a.checkpoint(), b.checkpoint())
    finally:
        a.close()
        b.close()


def test_open_rejects_bad_images():
    w = workload.config1(transfer_count=5000, account_count=100, seed=2)
    ats, tts = w.timestamps()
    a = _engine(w)
    try:
        a.create_accounts_batches(ats, w.account_counts, w.accounts)
        a.create_transfers_batches(tts, w.transfer_counts, w.transfers)
        image = a.checkpoint()
        bad = image.copy()
        bad[200] ^= 1
        assert a.open(bad) == -22          # checksum
        assert a.open(image[:-8]) == -22   # truncated
        bad = image.copy()
        bad[0] ^= 1
        assert a.open(bad) == -22          # magic
        assert a.open(image) == 0
        assert a.transfer_count() == len(w.transfers)
    finally:
        a.close()
