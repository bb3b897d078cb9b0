"""Sharded commit (tigerbeetle_amd/shard.py) over gloo on CPU, world sizes 2 and 3.

Each rank runs the router with a CPU oracle as its shard backend (test
infrastructure standing in for the per-GPU engine); the checker is one more
oracle that commits the same batches in the router's global order.  Replies,
the accounts each shard owns, the transfers each shard stored and the commit
timestamp must equal the single state machine's, bit for bit.
"""
from __future__ import annotations

import os
import pickle
import socket
import tempfile

import numpy as np
import pytest

import oracle
from tigerbeetle_amd.types import TRANSFER_DTYPE
from tests.shard_workload import ShardWorkload, config4_failing, config4_small, random_u128_ids


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _backend(kind, w, rank=0, world=1):
    if kind == "ledgershard":  # the oracle standing in for a ledger-shard engine (tests/shard_backends.py)
        from tests.shard_backends import LedgerShardOracle
        return LedgerShardOracle(oracle.Oracle(len(w.accounts), 1 << 14), world, rank)
    if kind == "gpu":
        from tigerbeetle_amd.engine import Engine
        return Engine(device=0, accounts_max=len(w.accounts) + 16, transfers_max=1 << 15, history_max=1 << 14,
                      events_per_call_max=1 << 14)
    return oracle.Oracle(len(w.accounts), 1 << 14)


def _worker(rank, world, port, out_dir, spec, kind="oracle", device_step=False, max_rounds=None, vectorized=True,
            skew_dry_rank=None, window=None, shard_stops=False):
    import torch.distributed as dist
    from tigerbeetle_amd.shard import Comm, ShardedStateMachine
    if skew_dry_rank == rank:
        _skew_dry_runs()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = _make(spec)
        sm = ShardedStateMachine(_backend(kind, w, rank, world), Comm(rank, world))
        if max_rounds is not None:
            sm.max_rounds = max_rounds
        sm.vectorized = vectorized
        if window is not None:
            sm.round_window = window
        sm.shard_stops = shard_stops
        acc_replies = sm.create_accounts(w.account_batches if rank == 0 else [])
        replies = []
        if device_step == "stream":
            # the pipelined form: step k + 1 routed while step k commits
            import torch
            steps = []
            for s in range(w.steps):
                batches = w.step_batches(s, rank)
                flat = np.concatenate(batches) if batches else np.zeros(0, dtype=TRANSFER_DTYPE)
                steps.append((torch.from_numpy(flat.view(np.uint8).copy()), [len(b) for b in batches]))
            for got in sm.create_transfers_device_stream(steps):
                replies.append([r.tobytes() for r in got])
        for s in range(w.steps if device_step != "stream" else 0):
            batches = w.step_batches(s, rank)
            if device_step:
                import torch
                flat = np.concatenate(batches) if batches else np.zeros(0, dtype=TRANSFER_DTYPE)
                # the router's collectives are gloo here, so its tensors stay on the CPU
                # (a GPU backend stages them in HBM per call)
                t = torch.from_numpy(flat.view(np.uint8).copy())
                got = sm.create_transfers_device(t, [len(b) for b in batches])
            else:
                got = sm.create_transfers(batches)
            replies.append([r.tobytes() for r in got])
        acc, xs = sm.export_state()
        with open(os.path.join(out_dir, f"r{rank}.pkl"), "wb") as f:
            pickle.dump({"replies": replies, "acc_replies": [a.tobytes() for a in acc_replies],
                         "acc": acc.tobytes(), "xs": xs.tobytes(), "cts": sm.commit_timestamp,
                         "stats": sm.stats}, f)
    finally:
        dist.destroy_process_group()


def _skew_dry_runs():
    """This rank's dry runs answer a wrong code for every event outside a spanning
    chain (the dry run's breaks, which only read spanning members, stay right), so
    this rank alone sees its commit differ from its dry run."""
    from tigerbeetle_amd import shard_vec
    real = shard_vec._commit_vec

    def skewed(sm, T, glob, E, P, G, I, C, in_span, lastloc, mlast, brk, dry):
        res = real(sm, T, glob, E, P, G, I, C, in_span, lastloc, mlast, brk, dry)
        if dry:
            res = res.copy()
            res[~in_span] = 999
        return res

    shard_vec._commit_vec = skewed


def _make(spec):
    kind, seed, world, steps, B = spec
    if kind == "mix":
        return ShardWorkload(seed, world, steps, B)
    if kind == "mixr":
        return random_u128_ids(ShardWorkload(seed, world, steps, B), seed)
    if kind == "mixw":  # wider: 128-event batches over 8 ledgers of 1000 accounts
        return random_u128_ids(ShardWorkload(seed, world, steps, B, batch=128, ledgers=8, accounts_per_ledger=1000),
                               seed)
    if kind == "mixa":
        from tests.shard_backends import with_account_recreates
        return with_account_recreates(ShardWorkload(seed, world, steps, B), seed)
    if kind in ("c4f", "c4l"):
        return config4_failing(seed, world, steps, B, limits=kind == "c4l")
    return config4_small(seed, world, steps, B)


def _check(spec, world, kind="oracle", device_step=False, max_rounds=None, vectorized=True, skew_dry_rank=None,
           window=None, shard_stops=False):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, spec, kind, device_step, max_rounds, vectorized,
                                skew_dry_rank, window, shard_stops),
                 nprocs=world, join=True)
        outs = [pickle.load(open(os.path.join(d, f"r{r}.pkl"), "rb")) for r in range(world)]
    return verify(_make(spec), outs, world)


def verify(w, outs, world):
    """The single state machine (one oracle) over the router's global order: every
    reply of every rank, the accounts each shard owns, the transfers each stored and
    the commit timestamp, bit for bit.  Returns rank 0's router stats."""
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE
    # the single state machine over the global order
    o = oracle.Oracle(len(w.accounts), 1 << 14)
    ts = 0
    acc_rep = []
    for b in w.account_batches:
        ts += 1 + len(b)
        acc_rep.append(o.create_accounts(ts, b))
    assert outs[0]["acc_replies"] == [a.tobytes() for a in acc_rep]
    stats = outs[0]["stats"]
    for s in range(w.steps):
        for r in range(world):
            for j, b in enumerate(w.step_batches(s, r)):
                ts += 1 + len(b)
                want = o.create_transfers(ts, b)
                got = np.frombuffer(outs[r]["replies"][s][j], dtype=RESULT_DTYPE)
                assert got.tobytes() == want.tobytes(), (s, r, j, got, want)
    acc = np.concatenate([np.frombuffer(x["acc"], dtype=ACCOUNT_DTYPE) for x in outs])
    want_acc = o.export_accounts()
    key = lambda a: np.lexsort((a["id_lo"], a["id_hi"]))
    assert acc[key(acc)].tobytes() == want_acc[key(want_acc)].tobytes()
    xs = np.concatenate([np.frombuffer(x["xs"], dtype=TRANSFER_DTYPE) for x in outs])
    want_xs = o.export_transfers()
    assert len(xs) == len(want_xs)
    assert xs[key(xs)].tobytes() == want_xs[key(want_xs)].tobytes()
    for x in outs:
        assert x["cts"] == o.commit_timestamp()
    return stats


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_flag_mix_matches_single_state_machine(world):
    stats = _check(("mix", 7 + world, world, 3, 2), world)
    # the workload must exercise the cross-shard machinery
    assert stats["dry_rounds"] > 0


def test_sharded_config4_cross_ledger_pairs():
    stats = _check(("c4", 11, 2, 2, 2), 2)
    assert stats["dry_rounds"] > 0


@pytest.mark.parametrize("world", [2, 3])
def test_device_step_config4(world):
    """The device-resident step (monotone ids, no post/void: no directory, on-device
    partition + all-to-all, dry rounds for the cross-ledger pairs)."""
    stats = _check(("c4", 13 + world, world, 3, 2), world, device_step=True)
    assert stats["preruns"] > 0 and stats["dry_rounds"] == 0 and stats["splits"] == 0


def test_device_step_falls_back_exactly():
    """Non-monotone ids and post/void: the device step hands over to the exact router."""
    stats = _check(("mix", 31, 2, 2, 2), 2, device_step=True)
    assert stats["steps"] > 0


@pytest.mark.parametrize("world", [2, 3])
def test_device_step_settles_plain_cross_shard_chains_with_one_dry_run(world):
    """Cross-ledger pairs that break on static checks: one dry run of the spanning
    members alone, then the commit (no dry rounds over the step)."""
    stats = _check(("c4f", 41 + world, world, 3, 2), world, device_step=True)
    assert stats["preruns"] > 0 and stats["dry_rounds"] == 0 and stats["device_fallbacks"] == 0


def test_device_step_dry_rounds_with_limit_accounts():
    """Spanning members on balance-limited accounts: dry rounds to the fixed point."""
    stats = _check(("c4l", 51, 2, 3, 2), 2, device_step=True)
    assert stats["dry_rounds"] > 0 and stats["preruns"] == 0


def test_device_step_hands_over_after_max_rounds():
    """No fixed point within max_rounds (forced to 1): the device step hands the
    step, uncommitted, to the exact router and its serial fallback."""
    stats = _check(("c4l", 53, 2, 3, 2), 2, device_step=True, max_rounds=1)
    assert stats["device_fallbacks"] > 0 and stats["serial_fallbacks"] > 0


@pytest.mark.parametrize("world", [2, 3])
def test_serial_fallback_one_cross_shard_chain_per_round(world):
    """The exact router with max_rounds = 1: every step whose chains do not settle in
    one dry round is committed one cross-shard chain at a time, still bit-exact."""
    stats = _check(("mix", 61 + world, world, 2, 2), world, max_rounds=1)
    assert stats["serial_fallbacks"] > 0


@pytest.mark.parametrize("kind", ["c4", "c4f", "c4l"])
def test_device_step_pipelined(kind):
    """create_transfers_device_stream: the next step routed while this one commits on a
    worker thread; the same results as the single state machine."""
    _check((kind, 101, 2, 3, 2), 2, device_step="stream")


def test_device_step_pipelined_fallback_keeps_router_state():
    """The pipelined stream with max_rounds = 1: steps whose spanning chains do not
    settle fall back to the exact router; the next step is routed only after that
    decision, so its timestamps and id filter follow the fallen-back step."""
    stats = _check(("c4l", 57, 2, 4, 2), 2, device_step="stream", max_rounds=1)
    assert stats["device_fallbacks"] > 0


@pytest.mark.parametrize("world", [2, 3, 4])
def test_general_step_random_u128_ids(world):
    """The flag-heavy mix (two-phase across steps and ranks, balancing, limits, chains
    across ledgers, repeated ids) with random u128 ids through the device step: every
    step takes the general step (shard_vec.round_vec: array directory, routing and
    commit, tensor collectives), bit-exact against the single state machine."""
    stats = _check(("mixr", 71 + world, world, 3, 2), world, device_step=True)
    assert stats["steps"] > 0 and stats["dry_rounds"] > 0


def test_general_step_same_id_imported_to_two_shards():
    """A committed id requested by post/voids routed to two other shards in one round:
    its holder answers one row per request (4 ranks, 8 ledgers: the case the 2- and
    3-rank mixes did not reach; found by profiles/general_rehearsal.py)."""
    stats = _check(("mixw", 12, 4, 4, 2), 4)
    assert stats["imports"] > 0


@pytest.mark.parametrize("shard_stops", [True, False])
def test_general_step_per_shard_stops(shard_stops):
    """Rounds with a stop per shard (ShardStops: hazards, chains, shared keys and effect
    shards) and with one stop for all: both bit-exact, the first in fewer rounds."""
    stats = _check(("mixw", 14, 4, 3, 2), 4, window=200, shard_stops=shard_stops)
    assert stats["steps"] > 3


def test_shard_stops_rules():
    """ShardStops._solve on hand-made rounds (positions 0..; two shards)."""
    from tigerbeetle_amd.shard_vec import EF_ALL, EF_NONE, INF, ShardStops
    P = np.arange(8, dtype=np.int64)
    C = P.copy()
    z = np.zeros(8, np.int64)
    ef = np.array([0, 1, 0, 1, 0, 1, 0, 1])
    H = np.zeros(8, bool)
    H[2] = True  # a hazard on shard 0: shard 0 waits from 2 on, shard 1 goes on
    w = ShardStops._solve(2, P, C, ef, H, z, z, INF)
    assert w.tolist() == [False, False, True, False, True, False, True, False]
    # a chain over 3 and 4 (shard 1 and 0): it waits whole, and shard 1 from 3 on
    C2 = C.copy()
    C2[4] = 3
    w = ShardStops._solve(2, P, C2, ef, H, z, z, INF)
    assert w.tolist() == [False, False, True, True, True, True, True, True]
    # a later event sharing a key with a waiting one waits (5 on shard 1 names 2's id)
    kx = z.copy()
    kx[2] = 77
    kp = z.copy()
    kp[5] = 77
    w = ShardStops._solve(2, P, C, ef, H, kx, kp, INF)
    assert w.tolist() == [False, False, True, False, True, True, True, True]
    # an event that may change state anywhere stops every shard once it waits
    ef2 = ef.copy()
    ef2[2] = EF_ALL
    w = ShardStops._solve(2, P, C, ef2, H, z, z, INF)
    assert w.tolist() == [False, False, True, True, True, True, True, True]
    # one that cannot change state stops no shard
    ef2[2] = EF_NONE
    w = ShardStops._solve(2, P, C, ef2, H, z, z, INF)
    assert w.tolist() == [False, False, True, False, False, False, False, False]
    # the window
    w = ShardStops._solve(2, P, C, ef, np.zeros(8, bool), z, z, 6)
    assert w.tolist() == [False] * 6 + [True] * 2


@pytest.mark.parametrize("window", [1, 37])
def test_general_step_round_window(window):
    """Rounds bounded by a window of events (ShardedStateMachine.round_window, cut at
    the chain the window ends in, or after the round's first chain): the same replies
    and state as the single state machine, over more rounds."""
    stats = _check(("mixr", 75 + window, 3, 3, 2), 3, device_step=True, window=window, shard_stops=window == 37)
    assert stats["steps"] > 3 * 6


@pytest.mark.parametrize("spec", [("mix", 81, 2, 3, 2), ("mixr", 82, 3, 2, 2)])
def test_reference_router_still_exact(spec):
    """shard.py _round (the event-by-event statement of the general step) against the
    same oracle: it stays the reference that round_vec is checked against."""
    _check(spec, spec[2], vectorized=False)


@pytest.mark.parametrize("world", [2, 3])
def test_ledger_shard_rows_exists_codes_from_the_owner(world):
    """Ledger-shard backends (each rank keeps the rows of its own ledgers' accounts, a
    directory entry for the others): accounts re-created with a changed field answer
    the exact exists_with_different_* code, which only the row's owner can compare
    (src/state_machine.zig:1227-1237), through the router's merge; chains of new
    accounts that those failures break roll back alike on every rank."""
    stats = _check(("mixa", 41 + world, world, 2, 2), world, kind="ledgershard")
    assert stats["steps"] > 0


@pytest.mark.timeout(300)
def test_dry_commit_mismatch_on_one_rank_only():
    """when only one rank's commit differs from its dry run, the
    check of the breaks (a collective) must still be entered by every rank or none:
    the decision is all-reduced first.  Rank 1's dry runs are skewed outside the
    spanning chains; the step completes on both ranks, bit-exact, and rank 0 (whose
    own results agree) counts the mismatch too."""
    stats = _check(("mixr", 73, 2, 3, 2), 2, device_step=True, skew_dry_rank=1)
    assert stats.get("dry_commit_mismatch", 0) > 0
