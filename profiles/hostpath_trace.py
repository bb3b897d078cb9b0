"""Kernel timeline of the drop-in call (run under rocprofv3 --kernel-trace): 100k accounts,
then 120 single tbgpu_create_transfers calls of one 8190-transfer batch each from page-locked
host memory, the last 60 after tbgpu_prefetch_transfers + wait (bench.py host_path's legs)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.engine import Engine  # noqa: E402
from tigerbeetle_amd.types import TRANSFER_DTYPE  # noqa: E402

w = workload.config2(transfer_count=8190 * 130, account_count=100_000, seed=7)
eng = Engine(accounts_max=100_000, transfers_max=8190 * 131, history_max=1024, events_per_call_max=8190,
             pinned_input=True)
ats, tts = w.timestamps()
eng.create_accounts_batches(ats, w.account_counts, w.accounts)
pinned = torch.empty(len(w.transfers) * 128, dtype=torch.uint8, pin_memory=True)
view = pinned.numpy().view(TRANSFER_DTYPE)
view[:] = w.transfers
offs = np.concatenate([[0], np.cumsum(w.transfer_counts.astype(np.int64))])
# argv[1]: "single" / "prefetched" (one kind of call only, e.g. for TBGPU_HOST_TRACE=1,
# whose averages are printed at close), default both
mode = sys.argv[1] if len(sys.argv) > 1 else "both"
lat = []
for k in range(120):
    ev = view[offs[k]:offs[k + 1]]
    t0 = time.perf_counter()
    pre = mode == "prefetched" or (mode == "both" and k >= 60)
    if pre:
        eng.prefetch_transfers(ev)
        eng.prefetch_wait()
    t1 = time.perf_counter()
    eng.create_transfers(int(tts[k]), ev)
    lat.append((time.perf_counter() - t1) * 1e6)
if mode == "both":
    print("single p50 %.1f us, prefetched commit p50 %.1f us" % (np.median(lat[10:60]), np.median(lat[70:])))
else:
    print("%s p50 %.1f us, p99 %.1f us" % (mode, np.median(lat[10:]), np.percentile(lat[10:], 99)))
eng.close()
