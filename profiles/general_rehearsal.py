"""Rehearsal of the general sharded step (shard_vec.round_vec) at 2 and 4 ranks on one
GPU: the flag-heavy mix with random u128 ids (tests/shard_workload.py: chains across
ledgers, two-phase across ranks, repeated ids), every rank a HIP engine, the
collectives stood in by threads (tests/thread_dist.py) because one RCCL rank needs one
GPU.  Prints one JSON line per world size: the step's wall time (max over ranks), each
phase's wall and CPU time (mean over ranks, per step) and the owner commit beside
them.  The ranks are threads of one process, so the host phases share one interpreter
lock: their wall times are upper bounds of what separate processes would take; the
CPU times ("cpu_" keys) are each thread's own work.

    python profiles/general_rehearsal.py [--worlds 2 4] [--batch 8190] [--batches 2] [--steps 4] [--windows 0 4096] [--stops 1 0]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(world, batch, bpr, steps, seed, window=None, stops=True):
    import torch

    from tests.shard_workload import ShardWorkload, random_u128_ids
    from tests.thread_dist import ThreadDist, ThreadGroup
    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.shard import Comm, ShardedStateMachine
    t0 = time.perf_counter()
    w = random_u128_ids(ShardWorkload(seed, world, steps, bpr, batch=batch, ledgers=8, accounts_per_ledger=1000),
                        seed)
    gen_s = time.perf_counter() - t0
    group = ThreadGroup(world)
    dev = torch.device("cuda", 0)
    outs, errors = [None] * world, []
    per_step = batch * bpr * world

    def worker(rank):
        eng = None
        try:
            eng = Engine(device=0, accounts_max=len(w.accounts) + 16, transfers_max=per_step * steps + 1024,
                         history_max=per_step * steps + 1024, events_per_call_max=per_step)
            comm = Comm(rank, world, device=dev)
            comm.dist = ThreadDist(group, rank)
            sm = ShardedStateMachine(eng, comm)
            if window is not None:
                sm.round_window = window
            sm.shard_stops = stops
            sm.create_accounts(w.account_batches if rank == 0 else [])
            walls = []
            for s in range(steps):
                batches = w.step_batches(s, rank)
                if s == 1:  # step 0 warms up (code objects, allocations)
                    sm.timed, sm.gtiming = True, {}
                    for k in sm.stats:
                        sm.stats[k] = 0
                group.barrier.wait()
                t = time.perf_counter()
                sm.create_transfers(batches)
                walls.append((time.perf_counter() - t) * 1e3)
            outs[rank] = {"walls": walls[1:], "g": dict(sm.gtiming), "stats": dict(sm.stats)}
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
        t.join(timeout=600)
    if errors:
        raise errors[0]
    timed = steps - 1
    wall = float(np.mean([max(o["walls"][s] for o in outs) for s in range(timed)]))
    keys = sorted({k for o in outs for k in o["g"]})
    phases = {k: round(float(np.mean([o["g"].get(k, 0.0) for o in outs])) / timed, 3) for k in keys}
    host = sum(v for k, v in phases.items() if not k.startswith("cpu_") and k != "commit")
    host_cpu = sum(v for k, v in phases.items() if k.startswith("cpu_") and k != "cpu_commit")
    return {"world": world, "events_per_step": per_step, "round_window": window, "shard_stops": stops, "batch": batch, "batches_per_rank": bpr,
            "timed_steps": timed, "ms_per_step": round(wall, 3),
            "events_per_s": round(per_step / (wall * 1e-3), 1),
            "phases_ms_per_step": phases, "host_wall_ms_per_step": round(host, 3),
            "host_cpu_ms_per_step": round(host_cpu, 3), "commit_ms_per_step": phases.get("commit", 0.0),
            "stats": outs[0]["stats"], "workload_gen_s": round(gen_s, 1),
            "note": "ranks are threads of one process on one GPU (shared interpreter lock)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--batch", type=int, default=8190)
    ap.add_argument("--batches", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--stops", type=int, nargs="+", default=[1],
                    help="ShardedStateMachine.shard_stops values (1: per-shard stops, 0: one stop)")
    ap.add_argument("--windows", type=int, nargs="+", default=[None],
                    help="ShardedStateMachine.round_window values (0: the whole step per round)")
    a = ap.parse_args()
    for world in a.worlds:
        for win in a.windows:
            for st in a.stops:
                print(json.dumps(run(world, a.batch, a.batches, a.steps, a.seed + world, win, bool(st))), flush=True)


if __name__ == "__main__":
    main()
