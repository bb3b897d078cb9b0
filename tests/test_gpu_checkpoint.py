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


def _shard_engine(n_acc, world, rank, hashed_max=0):
    from tigerbeetle_amd.engine import Engine
    return Engine(accounts_max=n_acc + 16, directory_max=n_acc + 16, hashed_max=hashed_max or n_acc + 16,
                  transfers_max=1 << 16, history_max=1024, events_per_call_max=1 << 14,
                  shard_world=world, shard_rank=rank)


def test_ledger_shard_checkpoint_round_trip():
    """A ledger shard's image: it names its world and rank, opens only
    into the ctx of the same shard (not another rank's, not an unsharded ctx, and an
    unsharded image not into a shard ctx), and checkpoint -> open -> checkpoint gives
    the same bytes.  Accounts have random u128 ids (hash index) and sequential ones
    (directory), across 8 ledgers; each shard commits transfers of its own ledgers."""
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE
    rng = np.random.default_rng(5)
    n = 800
    acc = np.zeros(n, dtype=ACCOUNT_DTYPE)
    acc["id_lo"] = np.arange(1, n + 1, dtype=np.uint64)
    rnd = np.arange(n) % 2 == 1  # every other account: a random u128 id
    acc["id_lo"][rnd] = rng.integers(1, 1 << 62, rnd.sum(), dtype=np.uint64)
    acc["id_hi"][rnd] = rng.integers(1, 1 << 62, rnd.sum(), dtype=np.uint64)
    acc["ledger"] = (np.arange(n) % 8 + 1).astype(np.uint32)
    acc["code"] = 1
    world = 2
    engines = [_shard_engine(n, world, r) for r in range(world)]
    other = _shard_engine(n, world, 1)
    plain = _engine(workload.config1(transfer_count=10, account_count=n, seed=1))
    try:
        for r, e in enumerate(engines):
            _, rc = e.create_accounts_batches(np.array([n + 1], np.uint64), np.array([n], np.uint32), acc)
            assert int(rc.sum()) == 0
            own = np.nonzero(acc["ledger"] % world == r)[0]
            t = np.zeros(400, dtype=TRANSFER_DTYPE)
            t["id_lo"] = np.arange(1, 401) + 1000 * r
            pick = own[rng.integers(0, len(own), (400, 2))]
            same = acc["ledger"][pick[:, 0]] == acc["ledger"][pick[:, 1]]
            pick[~same, 1] = pick[~same, 0]  # (an account with itself: accounts_must_be_different)
            t["debit_account_id_lo"], t["debit_account_id_hi"] = acc["id_lo"][pick[:, 0]], acc["id_hi"][pick[:, 0]]
            t["credit_account_id_lo"], t["credit_account_id_hi"] = acc["id_lo"][pick[:, 1]], acc["id_hi"][pick[:, 1]]
            t["ledger"] = acc["ledger"][pick[:, 0]]
            t["code"] = 1
            t["amount_lo"] = 5
            e.create_transfers_batches(np.array([n + 403 + r], np.uint64), np.array([400], np.uint32), t)
        for r, e in enumerate(engines):
            image = e.checkpoint()
            assert image[8:12].view(np.uint32)[0] == 3  # version 3: a shard's image, naming its shard
            assert image[12:16].view(np.uint32)[0] == (world << 16 | r)
            wrong = other if r == 0 else _shard_engine(n, world, 0)
            try:
                assert wrong.open(image) == -22, "another rank's ctx accepted the image"
            finally:
                if wrong is not other:
                    wrong.close()
            assert plain.open(image) == -22, "an unsharded ctx accepted a shard image"
            fresh = _shard_engine(n, world, r)
            try:
                assert fresh.open(image) == 0
                assert np.array_equal(fresh.checkpoint(), image), "restored shard image differs"
                # a legacy version-2 image (round 5's first trees: no shard in the
                # header) still opens into a shard ctx and comes back as version 3
                legacy = image.copy()
                legacy[8:12].view(np.uint32)[0] = 2
                legacy[12:16].view(np.uint32)[0] = 0
                again = _shard_engine(n, world, r)
                try:
                    assert again.open(legacy) == 0
                    assert np.array_equal(again.checkpoint(), image), "legacy image restored differently"
                finally:
                    again.close()
                bad = legacy.copy()
                bad[12:16].view(np.uint32)[0] = world << 16 | r  # a version 2 never named a shard
                assert fresh.open(bad) == -22
                # an image whose hashed ids exceed the ctx's account index is refused
                small = _shard_engine(n, world, r, hashed_max=64)
                try:
                    assert small.open(image) == -28
                finally:
                    small.close()
            finally:
                fresh.close()
        plain_img = plain.checkpoint()
        # -95: a version-1 image cannot be told from an old shard image without foreign
        # accounts, so a shard ctx refuses it with its own code
        assert engines[0].open(plain_img) == -95, "a shard ctx accepted an unsharded image"
    finally:
        for e in engines + [other, plain]:
            e.close()
