#!/usr/bin/env python3
"""Committed transfers/s of the MI355X commit engine (BASELINE.json metric).

One *step* = one streamed create_transfers call over `--batches-per-step`
consecutive 8190-transfer batches, with the events already resident in HBM
(tbgpu_create_transfers_batches_device).  Results are bit-identical to one
StateMachine.commit per batch (tests/test_gpu_parity.py).

Default workload: BASELINE config 2 (configs[1]) — 1M accounts on one ledger,
Zipf(0.99) debit/credit accounts, 1000 batches of 8190 transfers: one step is
the whole config-2 run (8,190,000 transfers) in one streamed call.  With --gpus N > 1
(torchrun, one process per GPU) every rank owns its own ledger shard (weak
scaling, no data-path collective): the ledger partition of SURVEY.md §8e with
the routing already applied.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALGO_BYTES_PER_TRANSFER = 680  # 128 ev + 128 row + 2x128 acct + 2x64 bal + 16 probe + 24 insert
COMMIT_BYTES_PER_TRANSFER = 656  # the same minus the 24-B id insert (fp_index)
HBM_PEAK_GBPS = 8000.0         # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def pmc_traffic(kernel: str, events_per_launch: float):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/rNN/traffic.json, written by profiles/collect.sh on the same bench command:
    2 x FETCH_SIZE + WRITE_SIZE per dispatch, MI355X_MICROARCH.md's gfx950 correction),
    scaled to this run's events per launch.  None when no summary matches."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")), reverse=True):
        try:
            d = json.load(open(f))[kernel]
        except (OSError, KeyError, ValueError):
            continue
        per_ev = d["traffic_bytes"] / d["events_per_launch"]
        return round(per_ev * events_per_launch), (
            f"{os.path.relpath(f, ROOT)}: {per_ev:.1f} B/transfer (2xFETCH_SIZE+WRITE_SIZE, "
            f"rocprofv3 --pmc passes of this bench) x {events_per_launch:.0f} transfers per launch")
    return None, None


def query_phase(eng, w, acc_n, torch, dev, count=100, batch=1024):
    """The reference benchmark's second phase (src/tigerbeetle/benchmark_load.zig:401-446):
    `count` get_account_transfers queries, one at a time, for uniformly random accounts
    with limit = 8190 and both sides, over everything committed above; latency per
    query (host filter in, up to 1 MB of rows out).  Also: the compaction that indexes
    the committed rows (StateMachine.compact's work here, off the commit path) and the
    throughput of `batch` such queries in one device launch.  Reported beside the
    metric, never as `value`."""
    from tigerbeetle_amd.types import FILTER_DTYPE, QUERY_MAX, account_filter
    rows = eng.transfer_count()
    t0 = time.perf_counter()
    eng.compact()
    compact_s = time.perf_counter() - t0
    rng = np.random.default_rng(7)
    ids = w.accounts["id_lo"]
    lat, got = [], 0
    for _ in range(count):
        f = account_filter(int(ids[int(rng.integers(0, acc_n))]), limit=QUERY_MAX)
        t0 = time.perf_counter()
        got += len(eng.get_account_transfers(f))
        lat.append(time.perf_counter() - t0)
    lat = np.array(lat) * 1e6
    filters = np.concatenate([account_filter(int(ids[int(rng.integers(0, acc_n))]), limit=QUERY_MAX)
                              for _ in range(batch)]).astype(FILTER_DTYPE)
    fd = torch.from_numpy(filters.view(np.uint8).copy()).to(dev)
    out = torch.empty(batch * QUERY_MAX * 128, dtype=torch.uint8, device=dev)
    eng.query_device(fd.data_ptr(), batch, QUERY_MAX, out.data_ptr())  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total, _ = eng.query_device(fd.data_ptr(), batch, QUERY_MAX, out.data_ptr())
    batch_s = time.perf_counter() - t0
    del out
    return {"workload": f"benchmark_load.zig query phase: {count} get_account_transfers, random account of "
                        f"{acc_n}, limit {QUERY_MAX}, debits|credits, over {rows} stored transfers",
            "latency_us": {"p50": round(float(np.percentile(lat, 50)), 1),
                           "p99": round(float(np.percentile(lat, 99)), 1), "max": round(float(lat.max()), 1)},
            "rows_returned_per_query": round(got / count, 1),
            "batched": {"queries": batch, "seconds": round(batch_s, 6), "queries_per_s": round(batch / batch_s, 1),
                        "rows_per_s": round(total / batch_s, 1)},
            "compact": {"rows": rows, "seconds": round(compact_s, 4),
                        "ns_per_row": round(compact_s / max(rows, 1) * 1e9, 3)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 4),
                    help="4: 1000 ledgers x 10k accounts with 1%% cross-ledger linked pairs, on one GPU")
    ap.add_argument("--force-general", action="store_true", help="disable the fast path (measure the fixed point)")
    ap.add_argument("--batches-per-step", type=int, default=None,
                    help="default 1000 (config 1/2: a whole BASELINE config-2 run per call), 60 for config 3")
    ap.add_argument("--accounts", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-queries", action="store_true", help="skip the query phase (after the timed region)")
    ap.add_argument("--verify", action="store_true", help="check every result is ok (config 1/2 never fail)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch  # device memory + torch.distributed plumbing (loaded before libtbgpu: one HIP runtime)
    import torch.distributed as dist
    from tigerbeetle_amd import workload
    from tigerbeetle_amd.engine import PHASES, Engine
    from tigerbeetle_amd.types import BATCH_MAX

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    if args.batches_per_step is None:
        args.batches_per_step = 60 if args.config == 3 else 1000
    B, K, W = args.batches_per_step, args.steps, args.warmup
    n_batches = (K + W) * B
    n_transfers = n_batches * BATCH_MAX
    t_gen = time.time()
    if args.config == 2:
        acc_n = args.accounts or 1_000_000
        w = workload.config2(transfer_count=n_transfers, account_count=acc_n, seed=42 + rank)
    elif args.config == 4:
        acc_n = args.accounts or 10_000_000
        w = workload.config4(transfer_count=n_transfers, ledgers=1000, accounts_per_ledger=acc_n // 1000,
                             seed=42 + rank)
    elif args.config == 3:
        acc_n = args.accounts or 10_000
        w = workload.config3(batches=n_batches, account_count=acc_n, seed=42 + rank)
        n_batches = len(w.transfer_counts)  # + the funding batches
    else:
        acc_n = args.accounts or 10_000
        w = workload.config1(transfer_count=n_transfers, account_count=acc_n, seed=42 + rank)
    log(f"[rank {rank}] generated {n_transfers} transfers / {acc_n} accounts in {time.time() - t_gen:.1f}s")

    eng = Engine(device=local_rank, accounts_max=acc_n, transfers_max=int(w.transfer_counts.sum()) + 1024,
                 history_max=int(w.transfer_counts.sum()) + 1024 if args.config == 3 else 1024,
                 events_per_call_max=B * BATCH_MAX, force_general=args.force_general)
    ats, tts = w.timestamps()
    _, rc = eng.create_accounts_batches(ats, w.account_counts, w.accounts)
    assert int(rc.sum()) == 0, "account creation failed"

    dev = torch.device("cuda", local_rank)
    ev_dev = torch.from_numpy(w.transfers.view(np.uint8)).to(dev)
    res_dev = torch.empty(B * BATCH_MAX * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    counts = w.transfer_counts
    ev_base = ev_dev.data_ptr()
    res_ptr = res_dev.data_ptr()

    def step(k):
        b0 = k * B
        off = int(counts[:b0].sum()) * 128
        total, rcs = eng.create_transfers_batches_device(tts[b0:b0 + B], counts[b0:b0 + B], ev_base + off, res_ptr)
        return int(total)

    for k in range(W):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    eng.set_profiling(True)
    phase = np.zeros(8)
    dev_ms = 0.0
    iters = []
    sorts = []
    non_ok = 0
    t0 = time.perf_counter()
    for k in range(W, W + K):
        non_ok += step(k)
        st = eng.stats()
        phase += np.array(st.phase_ms[:8])
        dev_ms += st.device_ms
        iters.append(st.iterations)
        sorts.append(st.sorts)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nk = torch.tensor([non_ok], dtype=torch.int64, device=dev)
        dist.all_reduce(nk)
        non_ok = int(nk.item())
    per_rank = int(counts[W * B:(W + K) * B].sum())
    total = per_rank * world
    value = total / elapsed
    ms_per_step = elapsed / K * 1e3

    # Roofline of the dominant kernel, fp_commit (the single-pass create_transfers,
    # fast.hip): its algorithmic bytes per transfer are SURVEY.md §8d's 680 B minus the
    # 24-B id-index insert done by fp_index.  Its duration is the "classify" phase:
    # HIP events recorded on the engine's stream around each launch in the timed region.
    names = list(PHASES)
    dom = int(np.argmax(phase[:len(names)]))
    phase_ms_per_step = {names[i]: round(phase[i] / K, 4) for i in range(len(names))}
    commit_ms = phase[names.index("classify")] / K
    achieved = per_rank / K * COMMIT_BYTES_PER_TRANSFER / (commit_ms * 1e-3) / 1e9 if commit_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic("fp_commit", per_rank / K)
    e2e_gbps = value / world * ALGO_BYTES_PER_TRANSFER / 1e9
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 5),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "kernel": "fp_commit",
        "basis": f"{COMMIT_BYTES_PER_TRANSFER} B/transfer x {B * BATCH_MAX} transfers per launch "
                 f"/ fp_commit launch time ({commit_ms:.4f} ms, HIP events on the engine stream)",
        "end_to_end": {"achieved": round(e2e_gbps, 2), "frac": round(e2e_gbps / HBM_PEAK_GBPS, 5),
                       "basis": f"{ALGO_BYTES_PER_TRANSFER} B/transfer x per-GPU committed transfers/s"},
        "dominant_phase": names[dom],
        "phase_ms_per_step": phase_ms_per_step,
        "device_ms_per_step": round(dev_ms / K, 4),
    }

    queries = None
    if rank == 0 and not args.no_queries:
        queries = query_phase(eng, w, acc_n, torch, dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle  # the CPU baseline leg (test infrastructure, never the product path)
        orc = oracle.Oracle(acc_n, 4 << 20)
        orc.create_accounts_batches(ats, w.account_counts, w.accounts)
        done, spent, b = 0, 0.0, 0
        while spent < args.cpu_seconds and b < len(counts):
            k = min(16, len(counts) - b)
            off = int(counts[:b].sum())
            n = int(counts[b:b + k].sum())
            _, _, el = orc.create_transfers_batches(tts[b:b + k], counts[b:b + k], w.transfers[off:off + n])
            done += n
            spent += el
            b += k
        cpu = {"value": round(done / spent, 1), "unit": "transfers/s", "cores": 1, "kind": "port",
               "sample": f"oracle/oracle.c commit loop (single thread), first {b} batches ({done} transfers) "
                         f"of the same config-{args.config} stream after creating the {acc_n} accounts; "
                         f"{spent:.1f}s of CPU work on {cpu_model()}"}

    if rank == 0:
        line = {
            "metric": "committed transfers/sec (whole node), 8190-transfer batches; % HBM roofline",
            "value": round(value, 1),
            "unit": "transfers/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u128",
            "data": "synthetic",
            "config": {"workload": f"config{args.config}: {acc_n} accounts, "
                                   + {1: "uniform pairs", 2: "Zipf(0.99) pairs on 1 ledger",
                                      3: "flag-heavy mix (limits, two-phase, balancing, chains)",
                                      4: "1000 ledgers, uniform pairs within a ledger, 1% cross-ledger "
                                         "linked pairs (u128 account ids: the hash index)"}[args.config]
                                   + f", {B} x 8190-transfer batches per step (streamed, HBM-resident)",
                       "batches_per_step": B, "transfers_per_step_per_gpu": B * BATCH_MAX,
                       "parallelism": f"ledger-shard x{world}"},
            "non_ok_results": non_ok,
            "fixed_point_passes": max(iters) if iters else 0,
            "fixed_point_sorts": max(sorts) if sorts else 0,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "queries": queries,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
