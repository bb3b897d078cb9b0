"""The drop-in call's timeline: one 8190-event tbgpu_create_transfers per call from
pinned host memory (INTEGRATION.md's Zig shim), config-2 load; prints per-call latency.
Run under `rocprofv3 --kernel-trace` to see where a call's time goes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402  (device memory, pinned buffers)

from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.engine import Engine  # noqa: E402
from tigerbeetle_amd.types import TRANSFER_DTYPE  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 64
w = workload.config2(transfer_count=calls * 8190, account_count=1_000_000, seed=5)
ats, tts = w.timestamps()
eng = Engine(device=0, accounts_max=1_000_000, transfers_max=calls * 8190 + 1024, history_max=1024,
             events_per_call_max=8190 * 4, pinned_input=True)
eng.create_accounts_batches(ats, w.account_counts, w.accounts)
pinned = torch.empty(calls * 8190 * 128, dtype=torch.uint8, pin_memory=True)
view = pinned.numpy().view(TRANSFER_DTYPE)
view[:] = w.transfers
lat = []
for k in range(calls):
    ev = view[k * 8190:(k + 1) * 8190]
    t0 = time.perf_counter()
    eng.create_transfers(int(tts[k]), ev)
    lat.append(time.perf_counter() - t0)
lat = np.array(lat[4:]) * 1e6
print(f"single call: p50 {np.percentile(lat, 50):.1f} us, p99 {np.percentile(lat, 99):.1f} us, "
      f"{8190 / np.percentile(lat, 50) * 1e6 / 1e6:.1f} M transfers/s at p50", flush=True)
eng.close()
