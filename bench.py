#!/usr/bin/env python3
"""Committed transfers/s of the MI355X commit engine (BASELINE.json metric).

One *step* = one streamed create_transfers call over `--batches-per-step`
consecutive 8190-transfer batches, with the events already resident in HBM
(tbgpu_create_transfers_batches_device).  Results are bit-identical to one
StateMachine.commit per batch (tests/test_gpu_parity.py).

Default workload: BASELINE config 2 (configs[1]) — 1M accounts on one ledger,
Zipf(0.99) debit/credit accounts, 1000 batches of 8190 transfers: one step is
the whole config-2 run (8,190,000 transfers) in one streamed call.  With --gpus N > 1
(torchrun, one process per GPU) the step is BASELINE config 4 through the ledger
router (tigerbeetle_amd/shard.py): every rank's client batches are
scattered to the owners of their ledgers by RCCL all-to-all, committed there and
answered by a second all-to-all (weak scaling: 1000 x 8190 transfers per rank per
step); `--routed` runs the same on a one-rank group, `--unrouted` gives every rank
its own pre-routed ledger shard instead.

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
PV_BYTES = 824                 # post/void: + the pending row read and the posted insert (§8d)
HBM_PEAK_GBPS = 8000.0         # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# stdout carries exactly one line, the result: whatever the libraries print there
# (RCCL's version banner, gloo's connection notes) is sent to stderr instead
_RESULT_FD = None


def _claim_stdout():
    global _RESULT_FD
    if _RESULT_FD is None:
        sys.stdout.flush()
        _RESULT_FD = os.dup(1)
        os.dup2(2, 1)


def emit(line: dict):
    data = (json.dumps(line) + "\n").encode()
    if _RESULT_FD is None:
        sys.stdout.write(data.decode())
        sys.stdout.flush()
    else:
        os.write(_RESULT_FD, data)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def pmc_traffic(config: int, accounts: int, kernel=None, id_order: str = "sequential", routed: bool = False):
    """HBM bytes per launch from the newest committed rocprofv3 PMC summary of THIS
    workload (profiles/rNN/traffic*.json, written by profiles/collect.sh +
    summarize.py on the same bench command and tagged with its config and account
    count): 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md's gfx950 correction)
    per dispatch of `kernel`, or, with kernel=None, summed over every commit kernel
    of a profiled step (the general path's roofline unit).  (None, reason) when no
    summary of this workload exists."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic*.json")), reverse=True):
        try:
            d = json.load(open(f))
            meta = d["_meta"]
        except (OSError, KeyError, ValueError, TypeError):
            continue
        if meta.get("config") != config or meta.get("accounts") != accounts or \
                meta.get("id_order", "sequential") != id_order or bool(meta.get("routed", False)) != routed:
            continue
        rel = os.path.relpath(f, ROOT)
        ev = meta["events_per_step"]
        if kernel is None:
            per = meta["commit_traffic_bytes"] / meta["steps"]
            what = f"all commit kernels, {meta['steps']} profiled steps"
        elif kernel in d:
            per = d[kernel]["traffic_bytes"]
            what = f"{kernel} per dispatch"
        else:
            continue
        return round(per), f"{rel}: 2xFETCH_SIZE+WRITE_SIZE, {what} ({per / ev:.1f} B/transfer)"
    return None, (f"no rocprofv3 PMC summary of config {config}{' (routed)' if routed else ''} with {accounts} "
                  f"accounts{'' if id_order == 'sequential' else ', ' + id_order + ' ids'} under profiles/")


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
    fd = eng.to_device(filters, dev)
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


HOST_WARMUP = 8  # untimed drop-in calls before each timed set (first-call allocations, page faults)
HOST_PY = 40     # of each drop-in set, the calls made through the Python wrapper (the rest from C)
STAGE_GAP_US = 200.0  # host_path `staged`: the journal write + replication round trip between prepare and commit


def host_path(eng, w, tts, counts, b0, nbs, torch):
    """The drop-in's own call rate (INTEGRATION.md's Zig shim): events in pinned host
    memory, replies back in host memory, PCIe inside the timing.
    - `single`: one tbgpu_create_transfers call per 8190-event batch, as the shim
      issues it once per committed prepare (src/state_machine.zig:894-928,
      src/vsr/replica.zig:3755-3762): per-call latency and the rate it implies;
    - `prefetched`: the same with StateMachine.prefetch before each commit
      (tbgpu_prefetch_transfers, then its wait: the replica commits only after the
      prefetch callback, src/vsr/replica.zig:3384-3415): the commit's own latency, and
      prefetch + commit;
    - `staged`: the primary's whole sequence for one op: tbgpu_stage_transfers at
      StateMachine.prepare (src/vsr/replica.zig:5159-5167), a busy-wait standing for the
      journal write and the replication round trip (STAGE_GAP_US), then prefetch (the
      body found in HBM) + its wait and the commit back to back (:3137-3152);
    - `streamed`: tbgpu_create_transfers_batches over many batches from host memory.
    Reported beside the metric, never as `value` (which is HBM-resident)."""
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    single, prefetched, staged, streamed = nbs
    offs = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    o0, o1 = int(offs[b0]), int(offs[b0 + single + prefetched + staged + streamed])
    pinned = torch.empty((o1 - o0) * 128, dtype=torch.uint8, pin_memory=True)
    view = pinned.numpy().view(TRANSFER_DTYPE)
    view[:] = w.transfers[o0:o1]

    def batch(b):
        return view[int(offs[b]) - o0:int(offs[b + 1]) - o0]

    def pct(x):
        x = np.asarray(x)
        if not len(x):
            return None
        return {"p50": round(float(np.percentile(x, 50)), 1), "p99": round(float(np.percentile(x, 99)), 1),
                "max": round(float(x.max()), 1)}

    # Timed from C (tbgpu_bench_host_calls: the call as the Zig shim makes it, no Python
    # around it) on the first HOST_C of each set, then a sample through the Python
    # wrapper (engine.create_transfers) for comparison
    py_n = lambda k: HOST_PY if k >= HOST_PY + 2 * HOST_WARMUP + 8 else 0
    c_single, c_pre = single - py_n(single), prefetched - py_n(prefetched)

    def c_calls(mode, g0, k):
        ev = view[int(offs[g0]) - o0:int(offs[g0 + k]) - o0]
        com, pre = eng.bench_host_calls(mode, tts[g0:g0 + k], counts[g0:g0 + k], ev)
        return com[HOST_WARMUP:], pre[HOST_WARMUP:], int(offs[g0 + k] - offs[g0 + HOST_WARMUP])

    lat, _, ev_single = c_calls(0, b0, c_single)
    py_lat, dev_us = [], []
    for k in range(c_single, single):
        ev = batch(b0 + k)
        t0 = time.perf_counter()
        eng.create_transfers(int(tts[b0 + k]), ev)
        if k >= c_single + HOST_WARMUP:
            py_lat.append((time.perf_counter() - t0) * 1e6)
            dev_us.append(eng.stats().device_ms * 1e3)  # HIP events around the call on the engine stream
    p0 = b0 + single
    com_us, pre_us, ev_pre = c_calls(1, p0, c_pre)
    both_us = com_us + pre_us
    py_com = []
    for k in range(c_pre, prefetched):
        ev = batch(p0 + k)
        eng.prefetch_transfers(ev)
        eng.prefetch_wait()
        t1 = time.perf_counter()
        eng.create_transfers(int(tts[p0 + k]), ev)
        if k >= c_pre + HOST_WARMUP:
            py_com.append((time.perf_counter() - t1) * 1e6)
    g0 = p0 + prefetched
    st_out = None
    if staged:
        ev_g = view[int(offs[g0]) - o0:int(offs[g0 + staged]) - o0]
        st_us, spre_us, scom_us = eng.bench_host_staged(tts[g0:g0 + staged], counts[g0:g0 + staged], ev_g, STAGE_GAP_US)
        st_us, spre_us, scom_us = st_us[HOST_WARMUP:], spre_us[HOST_WARMUP:], scom_us[HOST_WARMUP:]
        ev_st = int(offs[g0 + staged] - offs[g0 + HOST_WARMUP])
        st_out = {"calls": len(scom_us), "warmup_calls": HOST_WARMUP, "gap_us": STAGE_GAP_US,
                  "stage_latency_us": pct(st_us), "prefetch_latency_us": pct(spre_us),
                  "commit_latency_us": pct(scom_us), "prefetch_plus_commit_us": pct(spre_us + scom_us),
                  "transfers_per_s_prefetch_plus_commit": round(ev_st / (np.sum(spre_us + scom_us) * 1e-6), 1),
                  "entry": "tbgpu_stage_transfers (at prepare), a busy-wait of gap_us, then "
                           "tbgpu_prefetch_transfers_staged + tbgpu_prefetch_wait and tbgpu_create_transfers, "
                           "timed from C (tbgpu_bench_host_staged)"}
    s0 = g0 + staged
    ev = view[int(offs[s0]) - o0:]
    t0 = time.perf_counter()
    eng.create_transfers_batches(tts[s0:s0 + streamed], counts[s0:s0 + streamed], ev)
    el = time.perf_counter() - t0
    out = {"single": {"calls": len(lat), "warmup_calls": HOST_WARMUP,
                      "events_per_call": int(ev_single // max(len(lat), 1)),
                      "latency_us": pct(lat),
                      "slowest_calls": [int(x) + HOST_WARMUP for x in np.argsort(lat)[::-1][:3]],
                      "device_us": pct(dev_us),
                      "python_wrapper_latency_us": pct(py_lat),
                      "transfers_per_s": round(ev_single / (lat.sum() * 1e-6), 1),
                      "entry": "tbgpu_create_transfers (one batch per call, pinned host buffers), timed from C "
                               "(tbgpu_bench_host_calls); python_wrapper_*: the same call through engine.py"},
           "streamed": {"batches": streamed, "transfers": len(ev), "seconds": round(el, 6),
                        "transfers_per_s": round(len(ev) / el, 1),
                        "entry": "tbgpu_create_transfers_batches (host buffers, H2D inside the call)"}}
    if len(com_us):
        out["prefetched"] = {"calls": len(com_us), "warmup_calls": HOST_WARMUP,
                             "commit_latency_us": pct(com_us), "prefetch_latency_us": pct(pre_us),
                             "prefetch_plus_commit_us": pct(both_us),
                             "python_wrapper_commit_latency_us": pct(py_com),
                             "commit_transfers_per_s": round(ev_pre / (np.sum(com_us) * 1e-6), 1),
                             "entry": "tbgpu_prefetch_transfers + tbgpu_prefetch_wait, then tbgpu_create_transfers "
                                      "(the batch staged in HBM before the commit)"}
    if st_out:
        out["staged"] = st_out
    return out


ACCOUNT_BYTES = 272  # create_account reads 128 B, writes the 128-B row, probes 16 B


def create_accounts_device(eng, torch, dev, ats, account_counts, accounts, rank=0):
    """create_accounts with the account events resident in HBM (the metric's own
    convention): every account batch in one streamed call, timed with HIP events
    around the call on the engine's stream (engine stats).  Returns the
    `create_accounts` object of the bench line (accounts/s and the roofline at §8d's
    272 B per account, the whole call as the unit: no kernel dominates it)."""
    n = int(np.sum(account_counts))
    evd = eng.to_device(np.ascontiguousarray(accounts), dev)  # written by the engine's copy kernel
    res = torch.empty(max(n, 1) * 8, dtype=torch.uint8, device=dev)
    # untimed: the same call on a small scratch ctx first, so that the timed call does
    # not pay the first launch of each kernel (code-object load) in this process
    from tigerbeetle_amd.engine import Engine
    warm = Engine(device=eng.device, accounts_max=8192, transfers_max=16, history_max=16, events_per_call_max=8190,
                  shard_world=eng.shard_world, shard_rank=eng.shard_rank)
    k = int(min(len(accounts), 4096))
    warm.create_accounts_batches_device(np.array([k + 1], np.uint64), np.array([k], np.uint32), evd.data_ptr(),
                                        res.data_ptr())
    warm.close()
    torch.cuda.synchronize()
    eng.set_profiling(True)
    t0 = time.perf_counter()
    tot, _ = eng.create_accounts_batches_device(ats, account_counts, evd.data_ptr(), res.data_ptr())
    wall = time.perf_counter() - t0
    st = eng.stats()
    eng.set_profiling(False)
    if int(tot) != 0:
        raise RuntimeError(f"[rank {rank}] account creation failed ({int(tot)} non-ok)")
    del evd, res
    return accounts_line(n, len(account_counts), st.device_ms, wall)


def accounts_line(n, nb, device_ms, wall_s):
    gbps = n * ACCOUNT_BYTES / (device_ms * 1e-3) / 1e9 if device_ms > 0 else 0.0
    return {"accounts": n, "batches": nb, "device_ms": round(device_ms, 4), "wall_ms": round(wall_s * 1e3, 3),
            "accounts_per_s": round(n / (device_ms * 1e-3), 1) if device_ms > 0 else None,
            "roofline": {"bound": "hbm", "achieved": round(gbps, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(gbps / HBM_PEAK_GBPS, 5),
                         "basis": f"{ACCOUNT_BYTES} B/account x {n} accounts / the call's device time (HIP events "
                                  "on the engine stream; events resident in HBM)"}}


def cpu_baseline_leg(args, acc_n, acc_cap, ats, account_counts, accounts, tts, counts, transfers):
    """The CPU baseline (`cpu_baseline`, kind "port"): the oracle's commit loop over the
    leading batches of the same stream, about `--cpu-seconds` of work, on one pinned
    host core -- TigerBeetle commits on one core (docs/deploy/hardware.md:98).  Test
    infrastructure as the measured baseline beside the GPU, never the product path."""
    import oracle
    allowed = sorted(os.sched_getaffinity(0))
    core = allowed[min(2, len(allowed) - 1)]  # the third core the process may use
    os.sched_setaffinity(0, {core})
    try:
        orc = oracle.Oracle(acc_cap, 4 << 20)
        orc.create_accounts_batches(ats, account_counts, accounts)
        done, spent, b = 0, 0.0, 0
        nb_host = len(counts)
        offs = np.concatenate([[0], np.cumsum(np.asarray(counts, np.int64))])
        while spent < args.cpu_seconds and b < nb_host:
            k = min(16, nb_host - b)
            o0, o1 = int(offs[b]), int(offs[b + k])
            _, _, el = orc.create_transfers_batches(tts[b:b + k], counts[b:b + k], transfers[o0:o1])
            done += o1 - o0
            spent += el
            b += k
        orc.close()
    finally:
        os.sched_setaffinity(0, set(allowed))
    return {"value": round(done / spent, 1), "unit": "transfers/s", "cores": 1, "kind": "port",
            "sample": f"oracle/oracle.c commit loop (single thread pinned to host core {core}), first {b} "
                      f"batches ({done} transfers) of the same config-{args.config} stream after creating "
                      f"the {acc_n} accounts; {spent:.1f}s of CPU work on {cpu_model()}"}


def routed_bench(args, rank, world, local_rank, torch, dist, backend="nccl"):
    """N > 1, BASELINE config 4 through the ledger-sharded router (SURVEY.md §8e,
    tigerbeetle_amd/shard.py): every rank receives its own client batches (1000
    ledgers, uniform pairs within a ledger, 1% cross-ledger linked pairs), the step
    scatters them to the owners of their ledgers (ledger % N) with RCCL all-to-all
    over xGMI, every owner commits its sub-batches in global order
    (tbgpu_create_transfers_routed_device), cross-shard pairs are settled by one
    dry run of their members, and replies go back to the sources.  Accounts are
    replicated (each rank creates all of them).  Transfer ids rise along the global
    order (step, rank, index), the benchmark's sequential ids."""
    from tigerbeetle_amd import workload
    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.shard import Comm, ShardedStateMachine
    from tigerbeetle_amd.types import BATCH_MAX
    B = args.batches_per_step
    K, W = args.steps, args.warmup
    per_step = B * BATCH_MAX
    acc_n = args.accounts or 10_000_000
    t_gen = time.time()
    P = 1  # a step after the timed region, run with per-phase synchronization for the breakdown
    w = workload.config4(transfer_count=(K + W + P) * per_step, ledgers=1000, accounts_per_ledger=acc_n // 1000,
                         seed=42 + rank)
    j = np.arange(len(w.transfers), dtype=np.uint64)
    w.transfers["id_lo"] = ((j // per_step) * world + rank) * per_step + (j % per_step) + 1
    w.transfers["id_hi"] = 0
    log(f"[rank {rank}] generated {len(w.transfers)} transfers / {acc_n} accounts in {time.time() - t_gen:.1f}s")
    dev = torch.device("cuda", local_rank)
    # N > 1: ledger shards (tbgpu_options.shard_world): rows only for this rank's
    # ledgers (ledger % N == rank), a directory entry for every account
    apl = acc_n // 1000
    owned = (len(range(rank, 1001, world)) - (1 if rank == 0 else 0)) * apl if world > 1 else acc_n
    eng = Engine(device=local_rank, accounts_max=owned, directory_max=acc_n, hashed_max=1024 if world > 1 else 0,
                 transfers_max=int((K + W + P) * per_step * 1.25) + 4096,
                 history_max=1024, events_per_call_max=int(per_step * 1.25) + BATCH_MAX,
                 dense_block_span=apl, shard_world=world if world > 1 else 0, shard_rank=rank if world > 1 else 0)
    ats, _ = w.timestamps()
    acc_line = create_accounts_device(eng, torch, torch.device("cuda", local_rank), ats, w.account_counts,
                                      w.accounts, rank)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where the router's tensors live
    ssm = ShardedStateMachine(eng, Comm(rank, world, device=cdev))
    ssm.adopt_accounts(w.accounts, int(ats[-1]))
    ev_dev = eng.to_device(w.transfers, cdev) if cdev.type == "cuda" else torch.from_numpy(w.transfers.view(np.uint8))
    counts = w.transfer_counts
    keep_host = rank == 0 and world == 1 and not args.no_cpu  # the CPU baseline leg reads the stream
    if not keep_host:
        del w
    torch.cuda.synchronize()

    def step_args(k):
        return ev_dev[k * per_step * 128:(k + 1) * per_step * 128], list(map(int, counts[k * B:(k + 1) * B]))

    for k in range(W):
        ssm.create_transfers_device(*step_args(k))
    torch.cuda.synchronize()
    dist.barrier()
    st0 = dict(ssm.stats)
    non_ok = 0
    # the timed steps; pipelined (the default on N > 1), step k + 1's all-to-all (xGMI)
    # runs while step k's owner commit (HBM) runs (shard.py create_transfers_device_stream)
    eng.set_profiling(True)
    commit_ms = []  # per step: the owner commit's fp_commit launch (HIP events on the engine stream)
    t0 = time.perf_counter()
    if args.pipelined:
        for reps in ssm.create_transfers_device_stream(step_args(k) for k in range(W, W + K)):
            non_ok += sum(len(r) for r in reps)
            commit_ms.append(eng.stats().phase_ms[1])
    else:
        for k in range(W, W + K):
            non_ok += sum(len(r) for r in ssm.create_transfers_device(*step_args(k)))
            commit_ms.append(eng.stats().phase_ms[1])
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_profiling(False)
    # one more step, unpipelined and synchronized per phase: where a step's time goes
    for key in ssm.timing:
        ssm.timing[key] = 0.0
    ssm.timed = True
    ssm.create_transfers_device(*step_args(W + K))
    ssm.timed = False
    t = torch.tensor([elapsed, non_ok] + [ssm.timing[x] for x in sorted(ssm.timing)] + [float(np.mean(commit_ms))],
                     dtype=torch.float64, device=cdev)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tsum = t.clone()
    dist.all_reduce(tsum)
    elapsed = float(tmax[0])
    non_ok = int(tsum[1])
    total = per_step * K * world
    value = total / elapsed
    phases = {x: round(float(tmax[2 + i]), 3) for i, x in enumerate(sorted(ssm.timing))}
    fp_ms = float(tmax[-1])  # the slowest rank's mean fp_commit launch
    cpu = None
    if keep_host:
        ats_c, tts_c = w.timestamps()
        cpu = cpu_baseline_leg(args, acc_n, acc_n, ats_c, w.account_counts, w.accounts, tts_c, counts, w.transfers)
    if rank == 0:
        fp_gbps = per_step * COMMIT_BYTES_PER_TRANSFER / (fp_ms * 1e-3) / 1e9 if fp_ms > 0 else 0.0
        # the owner commit's fp_commit from the PMC passes of this same routed command
        # (profiles/run.sh pmc:4:routed); per launch like `achieved`
        traffic, traffic_src = pmc_traffic(4, acc_n, kernel="fp_commit", routed=True) if world == 1 else \
            (None, "PMC passes are taken on one GPU (a one-rank routed group); the N-rank launch is not profiled")
        traffic_gbps = traffic / (fp_ms * 1e-3) / 1e9 if traffic and fp_ms > 0 else None
        e2e = value / world * ALGO_BYTES_PER_TRANSFER / 1e9
        a2a_bytes = per_step * ssm.wire_bytes_per_event * (world - 1) / world  # leaving each rank per step
        line = {
            "metric": "committed transfers/sec (whole node), 8190-transfer batches; % HBM roofline",
            "value": round(value, 1),
            "unit": "transfers/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u128",
            "data": "synthetic",
            "config": {"workload": f"config4 routed: {acc_n} accounts ({'rows on their ledger owner, a directory entry on every rank' if world > 1 else 'one rank'}), 1000 ledgers sharded by "
                                   f"ledger % {world}, uniform pairs within a ledger, 1% cross-ledger linked "
                                   f"pairs; per rank {B} x 8190-transfer client batches per step, scattered to "
                                   f"their ledger owners by RCCL all-to-all and replied to by all-to-all",
                       "batches_per_step": B, "transfers_per_step_per_gpu": per_step,
                       "parallelism": f"ledger-shard x{world}, routed (tigerbeetle_amd/shard.py device step, "
                                      f"{'RCCL' if backend == 'nccl' else backend} collectives)"},
            "non_ok_results": non_ok,
            "non_ok_rate": round(non_ok / total, 5),
            "routed": {"pipelined": bool(args.pipelined),
                       "wire_bytes_per_event": ssm.wire_bytes_per_event,
                       "phase_ms_one_unpipelined_step_max_over_ranks": phases,
                       "alltoall_bytes_per_rank_per_step": int(a2a_bytes),
                       "alltoall_GBps_per_rank": round(a2a_bytes / (phases["exchange_ms"] * 1e-3) / 1e9, 1)
                       if phases["exchange_ms"] > 0 else None,
                       "cross_shard_prerun_steps": ssm.stats["preruns"] - st0["preruns"],
                       "dry_rounds": ssm.stats["dry_rounds"] - st0["dry_rounds"],
                       "fallbacks": ssm.stats["device_fallbacks"] - st0["device_fallbacks"]},
            "roofline": {"bound": "hbm", "achieved": round(fp_gbps, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(fp_gbps / HBM_PEAK_GBPS, 5), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "traffic_achieved": round(traffic_gbps, 2) if traffic_gbps else None,
                         "traffic_frac": round(traffic_gbps / HBM_PEAK_GBPS, 5) if traffic_gbps else None,
                         "kernel": "fp_commit (the owner commit)",
                         "basis": f"{COMMIT_BYTES_PER_TRANSFER} B/transfer x {per_step} transfers per launch / "
                                  f"fp_commit launch time ({fp_ms:.4f} ms, HIP events on the engine stream, "
                                  f"mean over steps, max over ranks)",
                         "end_to_end": {"achieved": round(e2e, 2), "frac": round(e2e / HBM_PEAK_GBPS, 5),
                                        "basis": f"{ALGO_BYTES_PER_TRANSFER} B/transfer x per-GPU committed "
                                                 "transfers/s (partition, all-to-all, commit and replies inside "
                                                 "the time)"}},
            "cpu_baseline": cpu,
            "create_accounts": acc_line,
        }
        emit(line)
    eng.close()
    dist.destroy_process_group()


def verify_stream(eng, w, ats, tts, counts, B, steps, replies, acc_n):
    """The same stream through the CPU oracle (test infrastructure: the checker, never
    the thing measured): every batch's replies of every step, then every account row
    and every stored transfer row, bit for bit."""
    import oracle
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, RESULT_DTYPE
    nb = steps * B
    n = int(counts[:nb].sum())
    orc = oracle.Oracle(acc_n, n + 1024)
    try:
        orc.create_accounts_batches(ats, w.account_counts, w.accounts)
        off = 0
        mismatches = []
        for k in range(steps):
            b0 = k * B
            m = int(counts[b0:b0 + B].sum())
            o, orc_rc, _ = orc.create_transfers_batches(tts[b0:b0 + B], counts[b0:b0 + B], w.transfers[off:off + m])
            g_rc, g_res = replies[k]
            want = np.concatenate([o[int(s):int(s) + int(c)] for s, c in
                                   zip(np.concatenate([[0], np.cumsum(counts[b0:b0 + B])[:-1]]), orc_rc)]) \
                if int(orc_rc.sum()) else np.zeros(0, RESULT_DTYPE)
            if not np.array_equal(g_rc, orc_rc) or g_res.tobytes() != want.tobytes():
                mismatches.append(k)
            off += m
        key = lambda a: a[np.lexsort((a["id_lo"], a["id_hi"]))]
        ga, oa = key(eng.export_accounts()), key(orc.export_accounts())
        accounts_equal = ga.tobytes() == oa.tobytes()
        transfers_equal = eng.export_transfers().tobytes() == orc.export_transfers().tobytes()
        non_ok = sum(int(r[0].sum()) for r in replies)
        return {"steps": steps, "batches": nb, "transfers": n, "non_ok_results": non_ok,
                "replies_bit_exact": not mismatches, "mismatched_steps": mismatches[:8],
                "accounts_bit_exact": accounts_equal, "stored_transfers_bit_exact": transfers_equal,
                "checker": "oracle/oracle.c over the same batches in the same order"}
    finally:
        orc.close()


SUBCONFIGS = (
    # (key in the line, arguments): BASELINE configs 1 and 3 on one GPU, and the routed
    # config-4 step on a one-rank group (the same workload `--gpus N > 1` times), each
    # a bench.py child with a bounded CPU-baseline sample
    ("config1", ["--config", "1", "--steps", "3", "--warmup", "1"]),
    # the reference benchmark's --id-order=random (src/tigerbeetle/cli.zig:205): u128
    # pseudo-UUID ids, so the hashed account index, the hashed id insert and the call's
    # duplicate check instead of the direct-mapped directory and the sorted id run
    ("config1_random", ["--config", "1", "--id-order", "random", "--steps", "3", "--warmup", "1"]),
    ("config3", ["--config", "3", "--steps", "3", "--warmup", "1"]),
    # config 5's per-GPU ledger shard (100M accounts, 1/8 of 1B transfers), generated in HBM
    ("config5", ["--config", "5", "--steps", "3", "--warmup", "1"]),
    ("scaling_n1", ["--routed", "--steps", "3", "--warmup", "1"]),
)
SUB_DROP = ("metric", "higher_is_better", "vs_baseline", "dtype", "data", "scaling", "unit", "queries", "host_path",
            "verify", "configs", "scaling_n1")


def run_subconfigs(args) -> dict:
    """The driver's default command (`--gpus 1`, no --config) also measures BASELINE
    configs 1 and 3 and the scaling family's N = 1 point, each in a child process run
    before this process touches the GPU (children, never exec), so the line carries
    them with their own roofline and cpu_baseline.  Returns {key: compact line}."""
    import subprocess
    out = {}
    for key, argv in SUBCONFIGS:
        cmd = [sys.executable, os.path.abspath(__file__), *argv, "--no-queries", "--no-host",
               "--cpu-seconds", str(args.sub_cpu_seconds)]
        t0 = time.time()
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=None, timeout=args.sub_timeout, text=True,
                               env=dict(os.environ, TB_BENCH_SUB="1"))
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not lines:
                out[key] = {"error": f"exit {r.returncode}", "argv": argv}
                continue
            d = json.loads(lines[-1])
        except subprocess.TimeoutExpired:
            out[key] = {"error": f"timeout {args.sub_timeout}s", "argv": argv}
            continue
        for k in SUB_DROP:
            d.pop(k, None)
        if isinstance(d.get("roofline"), dict):
            d["roofline"].pop("phase_ms_per_step", None)
        d["argv"] = " ".join(argv)
        d["wall_s"] = round(time.time() - t0, 1)
        out[key] = d
        log(f"[bench] {key}: {d.get('value')} transfers/s ({d['wall_s']} s)")
    return out


def spawn_ranks(n: int) -> None:
    """`--gpus N` without a launcher: start N rank processes (one per GPU, RCCL over
    127.0.0.1) before this process touches the GPU, pass rank 0's result line through
    and exit with the first failing rank's code.  (Children, never exec: this process
    has not initialised the GPU, but a child keeps the rule simple.)"""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    sys.exit(rc)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE, else 1).  Without a launcher, N > 1 starts "
                         "the N rank processes itself; under a launcher it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=None, help="default 3 (config 5: 14, ~the whole shard)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=None, choices=(1, 2, 3, 4, 5),
                    help="default 2 on one GPU, 4 (routed) on several.  4: 1000 ledgers x 10k accounts with "
                         "1%% cross-ledger linked pairs; 5: 100M accounts, one 1/8 ledger shard of 1B transfers "
                         "per GPU (generated in HBM)")
    ap.add_argument("--routed", action="store_true",
                    help="config 4 through the ledger router even on one GPU (a one-rank RCCL group)")
    ap.add_argument("--pipelined", dest="pipelined", action="store_true", default=None,
                    help="routed: step k + 1's all-to-all runs while step k commits (the default on N > 1 GPUs; "
                         "a one-rank group has nothing to exchange)")
    ap.add_argument("--no-pipelined", dest="pipelined", action="store_false")
    ap.add_argument("--unrouted", action="store_true",
                    help="N > 1: every rank commits its own pre-routed ledger shard (no all-to-all)")
    ap.add_argument("--force-general", action="store_true", help="disable the fast path (measure the fixed point)")
    ap.add_argument("--batches-per-step", type=int, default=None,
                    help="default 1000 (config 1/2: a whole BASELINE config-2 run per call), 60 for config 3")
    ap.add_argument("--accounts", type=int, default=None)
    ap.add_argument("--id-order", default="sequential", choices=("sequential", "random", "reversed"),
                    help="configs 1 and 2: the reference benchmark's --id-order (src/tigerbeetle/cli.zig:205, "
                         "IdPermutation, src/testing/id.zig:28-48) for account and transfer ids")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-queries", action="store_true", help="skip the query phase (after the timed region)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-buffer (drop-in call) measurement")
    ap.add_argument("--host-batches", type=int, default=None,
                    help="batches for the host-buffer measurement (default 64 single calls + 256 streamed)")
    ap.add_argument("--verify", action="store_true",
                    help="after the timed region, replay the same stream through the CPU oracle and compare "
                         "every reply and the final state bit for bit (configs 1-4)")
    ap.add_argument("--no-subconfigs", action="store_true",
                    help="the default one-GPU run: skip the config-1 / config-3 / routed N = 1 sub-measurements")
    ap.add_argument("--sub-cpu-seconds", type=float, default=5.0, help="CPU-baseline sample of each sub-measurement")
    ap.add_argument("--sub-timeout", type=float, default=240.0, help="seconds allowed to each sub-measurement")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world or 1)
    if env_world is None and args.gpus > 1:
        spawn_ranks(args.gpus)  # does not return
    subs = None
    # (not under a profiler: its preloaded library has initialised the GPU in this
    # process already, and the sub-measurements are children of it)
    profiled = "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)
    if (env_world is None and args.gpus == 1 and args.config is None and not args.routed and not args.no_subconfigs
            and not os.environ.get("TB_BENCH_SUB") and not profiled):
        subs = run_subconfigs(args)  # before this process touches the GPU
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU", file=sys.stderr)
        sys.exit(2)
    # Under a launcher (torchrun, or spawn_ranks) every N, N = 1 included, times the
    # same workload: BASELINE config 4 through the ledger router.  A plain one-process
    # run times BASELINE config 2 (configs[1], the metric's own configuration).
    launched = env_world is not None
    _claim_stdout()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("TB_DIST_BACKEND", "nccl") != "nccl":
        import torch
        local_rank %= max(torch.cuda.device_count(), 1)  # rehearsal: ranks may share a GPU

    import torch  # device memory + torch.distributed plumbing (loaded before libtbgpu: one HIP runtime)
    import torch.distributed as dist
    from tigerbeetle_amd import workload
    from tigerbeetle_amd.engine import PHASES, Engine
    from tigerbeetle_amd.types import BATCH_MAX

    torch.cuda.set_device(local_rank)
    backend = os.environ.get("TB_DIST_BACKEND", "nccl")  # gloo: a CPU-collective rehearsal on one GPU
    if launched and world == 1:
        args.routed = True  # the scaling family's N = 1 point
    if world == 1 and args.routed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or args.routed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    if args.config is None:
        args.config = 4 if (world > 1 or args.routed) else 2
    if args.pipelined is None:
        args.pipelined = world > 1

    if args.batches_per_step is None:
        args.batches_per_step = 60 if args.config == 3 else 1000
    if args.steps is None:
        args.steps = 14 if args.config == 5 else 3
    B, K, W = args.batches_per_step, args.steps, args.warmup
    if (world > 1 or args.routed) and args.config == 4 and not args.unrouted:
        return routed_bench(args, rank, world, local_rank, torch, dist, backend)
    host_nb = (0, 0, 0, 0) if (args.no_host or world > 1 or args.config == 5) else \
        ((args.host_batches or 136, args.host_batches or 136, args.host_batches or 136, (args.host_batches or 64) * 4)
         if args.config != 3 else (16, 16, 16, 48))
    n_batches = (K + W) * B + sum(host_nb)
    n_transfers = n_batches * BATCH_MAX
    t_gen = time.time()
    c5 = None
    cache = os.environ.get("TB_BENCH_CACHE")  # diagnostics only: reuse a generated workload across runs
    ckey = f"c{args.config}_{args.accounts}_{n_batches}_{42 + rank}_{args.id_order}"
    if cache and args.config != 5 and os.path.exists(os.path.join(cache, ckey + ".npz")):
        z = np.load(os.path.join(cache, ckey + ".npz"))
        w = workload.Workload(str(z["name"]), z["accounts"], z["account_counts"], z["transfers"], z["transfer_counts"],
                              ticks={int(k): int(v) for k, v in z["ticks"]})
        acc_n = args.accounts or {1: 10_000, 2: 1_000_000, 3: 10_000, 4: 10_000_000}[args.config]
        n_batches = len(w.transfer_counts)
    elif args.config == 5:
        c5 = workload.config5(shard=rank, shards=8)
        acc_n = c5.accounts
        w = None
    elif args.config == 2:
        acc_n = args.accounts or 1_000_000
        w = workload.config2(transfer_count=n_transfers, account_count=acc_n, seed=42 + rank, id_order=args.id_order)
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
        w = workload.config1(transfer_count=n_transfers, account_count=acc_n, seed=42 + rank, id_order=args.id_order)
    log(f"[rank {rank}] generated {n_transfers} transfers / {acc_n} accounts in {time.time() - t_gen:.1f}s")
    if cache and w is not None and not os.path.exists(os.path.join(cache, ckey + ".npz")):
        os.makedirs(cache, exist_ok=True)
        np.savez(os.path.join(cache, ckey + ".npz"), name=w.name, accounts=w.accounts,
                 account_counts=w.account_counts, transfers=w.transfers, transfer_counts=w.transfer_counts,
                 ticks=np.array(sorted(w.ticks.items()), dtype=np.int64).reshape(-1, 2))

    dev = torch.device("cuda", local_rank)
    if c5 is not None:
        # config 5: the load is generated in HBM (workload.DeviceLoad, csrc/loadgen.hip)
        from tigerbeetle_amd.engine import generate_accounts, generate_transfers
        counts = c5.transfer_batches()[:n_batches]
        n_batches = len(counts)
        ats, tts = c5.timestamps()
        # a ledger shard (tbgpu_options.shard_world = 8): the directory knows all 100M
        # accounts, the 128-byte rows are this shard's 12.5M (ledger % 8 == rank)
        eng = Engine(device=local_rank, accounts_max=c5.owned_accounts(), directory_max=acc_n, hashed_max=1024,
                     transfers_max=int(counts.sum()) + 1024, history_max=1024, events_per_call_max=B * BATCH_MAX,
                     force_general=args.force_general, pinned_input=True, shard_world=c5.shards,
                     shard_rank=c5.shard)
        ab = c5.account_batches()
        buf = torch.empty(1221 * BATCH_MAX * 128, dtype=torch.uint8, device=dev)
        res = torch.empty(1221 * BATCH_MAX * 8, dtype=torch.uint8, device=dev)
        first = 1
        acc_ms, acc_wall = 0.0, 0.0
        eng.set_profiling(True)
        for b0 in range(0, len(ab), 1221):
            cnt = ab[b0:b0 + 1221]
            generate_accounts(local_rank, first, int(cnt.sum()), c5.accounts_per_ledger, buf.data_ptr())
            torch.cuda.synchronize()
            ta = time.perf_counter()
            tot, _ = eng.create_accounts_batches_device(ats[b0:b0 + len(cnt)], cnt, buf.data_ptr(), res.data_ptr())
            acc_wall += time.perf_counter() - ta
            acc_ms += eng.stats().device_ms
            if int(tot) != 0:
                raise RuntimeError("account creation failed")
            first += int(cnt.sum())
        eng.set_profiling(False)
        # the 100M accounts as 10M-account calls (1221 batches of 8190 each)
        acc_line = accounts_line(acc_n, len(ab), acc_ms, acc_wall)
        del buf, res
        ev_dev = torch.empty(int(counts.sum()) * 128, dtype=torch.uint8, device=dev)
        generate_transfers(local_rank, c5.first_transfer_id, int(counts.sum()), c5.seed, c5.ledger0, c5.ledgers,
                           c5.accounts_per_ledger, ev_dev.data_ptr(), ledger_stride=c5.ledger_stride)
        log(f"[rank {rank}] config 5: {acc_n} accounts created, {int(counts.sum())} transfers generated in HBM "
            f"in {time.time() - t_gen:.1f}s")
    else:
        eng = Engine(device=local_rank, accounts_max=acc_n, transfers_max=int(w.transfer_counts.sum()) + 1024,
                     history_max=int(w.transfer_counts.sum()) + 1024 if args.config == 3 else 1024,
                     events_per_call_max=B * BATCH_MAX, force_general=args.force_general,
                     pinned_input=True,  # host_path's buffers are page-locked (TBGPU_OPT_PINNED_INPUT)
                     # config 4 numbers its accounts ledger << 32 | k: the blocked directory
                     dense_block_span=acc_n // 1000 if args.config == 4 else 0)
        ats, tts = w.timestamps()
        acc_line = create_accounts_device(eng, torch, dev, ats, w.account_counts, w.accounts, rank)
        ev_dev = eng.to_device(w.transfers, dev)  # HBM-resident events, written by the engine's copy kernel
        counts = w.transfer_counts
    res_dev = torch.empty(B * BATCH_MAX * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ev_base = ev_dev.data_ptr()
    res_ptr = res_dev.data_ptr()

    replies = []  # --verify: every step's replies (copied after the step, outside nothing timed by HIP events)

    def step(k):
        b0 = k * B
        off = int(counts[:b0].sum()) * 128
        total, rcs = eng.create_transfers_batches_device(tts[b0:b0 + B], counts[b0:b0 + B], ev_base + off, res_ptr)
        if args.verify:
            replies.append((np.array(rcs, dtype=np.uint32).copy(), res_dev[:int(total) * 8].cpu().numpy().copy()))
        return int(total)

    prewarm = float(os.environ.get("TB_BENCH_PREWARM_S", "0"))  # diagnostics only: untimed device load first
    if prewarm > 0:
        a = torch.empty(1 << 28, dtype=torch.int32, device=dev)
        t_pw = time.time()
        while time.time() - t_pw < prewarm:
            a.add_(1)
        torch.cuda.synchronize()
        del a
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
    paths = []
    step_phase_ms = []  # per step: every phase's HIP-event time (the dominant one's spread is reported)
    non_ok = 0
    t0 = time.perf_counter()
    for k in range(W, W + K):
        non_ok += step(k)
        st = eng.stats()
        step_phase_ms.append(np.array(st.phase_ms[:8], dtype=np.float64))
        phase += np.array(st.phase_ms[:8])
        dev_ms += st.device_ms
        iters.append(st.iterations)
        sorts.append(st.sorts)
        paths.append(st.path)
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

    # Roofline.  Fast path (configs 1, 2, 4): the dominant kernel is fp_commit (the
    # single-pass create_transfers, fast.hip); its algorithmic bytes per transfer are
    # SURVEY.md §8d's 680 B minus the 24-B id-index insert done by fp_index; its
    # duration is the "classify" phase: HIP events recorded on the engine's stream
    # around each launch in the timed region.  General path (config 3): no single
    # kernel dominates (sort, scan, evaluate, classify, apply are each 10-30 %), so
    # the roofline is that of the whole path per call: §8d's algorithmic bytes of the
    # call's events (680 B per transfer, 824 B per post/void, +8 B per non-ok reply)
    # over the call's device time (HIP events around the call on the engine stream).
    names = list(PHASES)
    dom = int(np.argmax(phase[:len(names)]))
    step_dom_ms = [float(p[dom]) for p in step_phase_ms]  # the dominant phase, step by step
    phase_ms_per_step = {names[i]: round(phase[i] / K, 4) for i in range(len(names))}
    e2e_gbps = value / world * ALGO_BYTES_PER_TRANSFER / 1e9
    if w is not None:
        timed = w.transfers[int(counts[:W * B].sum()):int(counts[:(W + K) * B].sum())]
        n_pv = int(((timed["flags"] & 12) != 0).sum())
    else:
        n_pv = 0  # config 5: plain transfers
    fast = max(paths) == 1 and min(paths) == 1
    if fast:
        commit_ms = phase[names.index("classify")] / K
        achieved = per_rank / K * COMMIT_BYTES_PER_TRANSFER / (commit_ms * 1e-3) / 1e9 if commit_ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(args.config, acc_n, kernel="fp_commit", id_order=args.id_order)
        kernel = "fp_commit"
        basis = (f"{COMMIT_BYTES_PER_TRANSFER} B/transfer x {B * BATCH_MAX} transfers per launch "
                 f"/ fp_commit launch time ({commit_ms:.4f} ms, HIP events on the engine stream)")
    else:
        call_ms = dev_ms / K
        algo = (per_rank - n_pv) * ALGO_BYTES_PER_TRANSFER + n_pv * PV_BYTES + 8 * non_ok // world
        achieved = algo / K / (call_ms * 1e-3) / 1e9 if call_ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(args.config, acc_n, kernel=None, id_order=args.id_order)
        kernel = "general path (every kernel of the call)"
        basis = (f"{ALGO_BYTES_PER_TRANSFER} B x {per_rank - n_pv} transfers + {PV_BYTES} B x {n_pv} posts/voids "
                 f"+ 8 B x {non_ok // world} non-ok replies over {K} calls / call device time "
                 f"({call_ms:.4f} ms, HIP events on the engine stream)")
    # the same launch time priced with the measured HBM bytes instead of the algorithmic ones
    t_ms = commit_ms if fast else dev_ms / K
    traffic_gbps = traffic / (t_ms * 1e-3) / 1e9 if traffic and t_ms > 0 else None
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 5),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "traffic_achieved": round(traffic_gbps, 2) if traffic_gbps else None,
        "traffic_frac": round(traffic_gbps / HBM_PEAK_GBPS, 5) if traffic_gbps else None,
        "kernel": kernel,
        "basis": basis,
        "end_to_end": {"achieved": round(e2e_gbps, 2), "frac": round(e2e_gbps / HBM_PEAK_GBPS, 5),
                       "basis": f"{ALGO_BYTES_PER_TRANSFER} B/transfer x per-GPU committed transfers/s"},
        "dominant_phase": names[dom],
        "dominant_ms_per_step": {"phase": names[dom], "min": round(min(step_dom_ms), 4),
                                 "median": round(float(np.median(step_dom_ms)), 4),
                                 "max": round(max(step_dom_ms), 4),
                                 "first": round(step_dom_ms[0], 4), "last": round(step_dom_ms[-1], 4)},
        "phase_ms_per_step": phase_ms_per_step,
        "device_ms_per_step": round(dev_ms / K, 4),
    }

    verify = None
    if args.verify and w is not None:
        verify = verify_stream(eng, w, ats, tts, counts, B, W + K, replies, acc_n)
        log(f"[rank {rank}] verify: {verify}")

    queries = None
    if rank == 0 and not args.no_queries and w is not None:
        queries = query_phase(eng, w, acc_n, torch, dev)

    host = None
    if rank == 0 and world == 1 and not args.no_host and w is not None and sum(host_nb):
        host = host_path(eng, w, tts, counts, (W + K) * B, host_nb, torch)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        if w is not None:
            cpu = cpu_baseline_leg(args, acc_n, acc_n, ats, w.account_counts, w.accounts, tts, counts, w.transfers)
        else:
            # config 5: the leading 1024 batches, with the accounts they touch (the sample
            # need not create all 100M): their results do not depend on the others
            from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE
            nh = int(counts[:1024].sum())
            host_events = ev_dev[:nh * 128].cpu().numpy().view(TRANSFER_DTYPE)
            ids = np.unique(np.concatenate([host_events["debit_account_id_lo"], host_events["credit_account_id_lo"]]))
            acc = np.zeros(len(ids), dtype=ACCOUNT_DTYPE)
            acc["id_lo"] = ids
            acc["ledger"] = ((ids - 1) // c5.accounts_per_ledger + 1).astype(np.uint32)
            acc["code"] = 1
            cpu = cpu_baseline_leg(args, acc_n, len(ids), np.array([ats[-1]], np.uint64),
                                   np.array([len(acc)], np.uint32), acc, tts, counts[:1024], host_events)

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
                                         "linked pairs (ids ledger << 32 | k: the blocked directory)",
                                      5: "1000 ledgers, one 1/8 ledger shard of 1B transfers (the per-GPU shard), "
                                         "uniform pairs within a ledger, generated in HBM"}[args.config]
                                   + ("" if args.id_order == "sequential" else
                                      f", --id-order={args.id_order} account and transfer ids (IdPermutation)")
                                   + f", {B} x 8190-transfer batches per step (streamed, HBM-resident)",
                       "batches_per_step": B, "transfers_per_step_per_gpu": B * BATCH_MAX,
                       "parallelism": f"ledger-shard x{world}"},
            "non_ok_results": non_ok,
            "non_ok_rate": round(non_ok / total, 5) if total else 0.0,
            "fixed_point_passes": max(iters) if iters else 0,
            "fixed_point_sorts": max(sorts) if sorts else 0,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "create_accounts": acc_line,
            "host_path": host,
            "queries": queries,
            "verify": verify,
        }
        if subs is not None:
            line["configs"] = {k: v for k, v in subs.items() if k != "scaling_n1"}
            line["scaling_n1"] = subs.get("scaling_n1")
        emit(line)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
