"""The device-resident routed step with several ranks on one GPU and CUDA tensors:
the path `bench.py --gpus N` takes over RCCL (the engine's tbgpu_route_stats /
tbgpu_route_scatter, the all-to-all of events and side records, the owner commit,
the one-dry-run settlement of cross-shard chains), with the collectives stood in by
threads (tests/thread_dist.py) because one RCCL rank needs one GPU.  Checked against
the single CPU state machine over the router's global order (tests/test_shard.py)."""
import threading

import numpy as np
import pytest

from tests.shard_workload import ShardWorkload, config4_failing, config4_small, random_u128_ids
from tests.test_shard import verify
from tests.thread_dist import ThreadDist, ThreadGroup

pytestmark = pytest.mark.gpu


def _run(w, world, pipelined=False, expect_wire=True, shard_rows=False):
    import torch

    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.shard import Comm, ShardedStateMachine
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    group = ThreadGroup(world)
    outs, errors = [None] * world, []
    dev = torch.device("cuda", 0)

    def worker(rank):
        eng = None
        try:
            if shard_rows:  # a ledger shard: rows of its own ledgers' accounts, directory entries for all
                eng = Engine(device=0, accounts_max=len(w.accounts) + 16, directory_max=len(w.accounts) + 16,
                             transfers_max=1 << 16, history_max=1 << 12, events_per_call_max=1 << 14,
                             shard_world=world, shard_rank=rank)
            else:
                eng = Engine(device=0, accounts_max=len(w.accounts) + 16, transfers_max=1 << 16, history_max=1 << 12,
                             events_per_call_max=1 << 14)
            comm = Comm(rank, world, device=dev)
            comm.dist = ThreadDist(group, rank)
            sm = ShardedStateMachine(eng, comm)
            acc_replies = sm.create_accounts(w.account_batches if rank == 0 else [])
            replies = []
            steps = []
            for s in range(w.steps):
                batches = w.step_batches(s, rank)
                flat = np.concatenate(batches) if batches else np.zeros(0, dtype=TRANSFER_DTYPE)
                # uploaded by the engine's copy kernel (tbgpu_copy_to_device), as bench.py does
                steps.append((eng.to_device(flat, dev), [len(b) for b in batches]))
            if pipelined:
                for got in sm.create_transfers_device_stream(steps):
                    replies.append([r.tobytes() for r in got])
            else:
                for ev, cnt in steps:
                    got = sm.create_transfers_device(ev, cnt)
                    replies.append([r.tobytes() for r in got])
            acc, xs = sm.export_state()
            outs[rank] = {"replies": replies, "acc_replies": [a.tobytes() for a in acc_replies],
                          "acc": acc.tobytes(), "xs": xs.tobytes(), "cts": sm.commit_timestamp,
                          "stats": dict(sm.stats), "wire": sm.wire_bytes_per_event}
        except BaseException as e:  # noqa: BLE001 -- re-raised in the main thread
            errors.append(e)
            group.barrier.abort()
        finally:
            if eng is not None:
                eng.close()

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a rank did not finish"
    if errors:
        raise errors[0]
    # more than one rank: the device step ran and its events travelled in the packed wire
    # format (<= 33 words of 4 B); only the general step (round_vec) may send none
    if expect_wire and world > 1:
        assert all(0 < o["wire"] <= 4 * 33 for o in outs), [o["wire"] for o in outs]
    else:
        assert all(o["wire"] <= 4 * 33 for o in outs), [o["wire"] for o in outs]
    return verify(w, outs, world)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_routed_device_step_config4(world):
    stats = _run(config4_small(71 + world, world, 3, 2), world)
    assert stats["preruns"] > 0 and stats["dry_rounds"] == 0 and stats["device_fallbacks"] == 0


@pytest.mark.parametrize("world", [2, 4])
def test_routed_device_step_breaking_chains(world):
    stats = _run(config4_failing(81 + world, world, 3, 2), world)
    assert stats["preruns"] > 0 and stats["dry_rounds"] == 0


def test_routed_device_step_limit_accounts():
    stats = _run(config4_failing(91, 3, 3, 2, limits=True), 3)
    assert stats["dry_rounds"] > 0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_routed_device_stream_pipelined(world):
    """The pipelined form (bench.py's timed loop): step k + 1's stats, scatter and
    all-to-all while step k's owner commit runs on a worker thread."""
    stats = _run(config4_failing(111 + world, world, 4, 2), world, pipelined=True)
    assert stats["preruns"] > 0
    stats = _run(config4_failing(121 + world, world, 3, 2, limits=True), world, pipelined=True)
    assert stats["dry_rounds"] > 0


@pytest.mark.parametrize("world", [2, 4])
def test_general_step_random_u128_ids_on_gpu(world):
    """The flag-heavy mix with random u128 ids (two-phase across ranks, repeated ids,
    chains across ledgers): every step takes the general step (shard_vec.round_vec) with
    the HIP engines behind the ranks and CUDA tensors in the collectives."""
    w = random_u128_ids(ShardWorkload(131 + world, world, 3, 2), 131 + world)
    stats = _run(w, world, expect_wire=False)
    assert stats["steps"] > 0 and stats["dry_rounds"] > 0


@pytest.mark.parametrize("world", [2, 4])
def test_ledger_shard_engines(world):
    """Ledger-shard engines (tbgpu_options.shard_world): each keeps the 128-byte rows
    of its own ledgers' accounts only; re-created accounts answer the exact exists_*
    code through the router's merge; the flag-heavy mix and config 4's cross-ledger
    pairs commit as on replicated engines."""
    from tests.shard_backends import with_account_recreates
    stats = _run(with_account_recreates(ShardWorkload(141 + world, world, 3, 2), 141 + world), world,
                 expect_wire=False, shard_rows=True)
    assert stats["steps"] > 0
    stats = _run(config4_failing(151 + world, world, 3, 2), world, shard_rows=True)
    assert stats["preruns"] > 0
