"""The primary's staged sequence (tbgpu_bench_host_staged: stage at prepare, a gap for the
replication round trip, prefetch + wait, commit) at several gaps, and the prefetched
sequence for comparison: p50 of prefetch and commit, from C.  Shows what the gap (an
idle GPU between ops) costs the commit.  1M accounts, config-2 batches, page-locked."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.engine import Engine  # noqa: E402
from tigerbeetle_amd.types import TRANSFER_DTYPE  # noqa: E402

gaps = [float(x) for x in (sys.argv[1:] or ["0", "20", "200", "1000"])]
per = 72
nb = per * (len(gaps) + 1)
w = workload.config2(transfer_count=8190 * nb, account_count=1_000_000, seed=7)
eng = Engine(accounts_max=1_000_000, transfers_max=8190 * (nb + 1), history_max=1024, events_per_call_max=8190,
             pinned_input=True)
ats, tts = w.timestamps()
eng.create_accounts_batches(ats, w.account_counts, w.accounts)
pinned = torch.empty(len(w.transfers) * 128, dtype=torch.uint8, pin_memory=True)
view = pinned.numpy().view(TRANSFER_DTYPE)
view[:] = w.transfers
offs = np.concatenate([[0], np.cumsum(w.transfer_counts.astype(np.int64))])
cnt = w.transfer_counts
p50 = lambda x: float(np.median(np.asarray(x)[8:]))
b = 0
com, pre = eng.bench_host_calls(1, tts[b:b + per], cnt[b:b + per], view[offs[b]:offs[b + per]])
print(f"prefetched         prefetch {p50(pre):6.1f} us  commit {p50(com):6.1f} us  sum {p50(pre + com):6.1f} us",
      flush=True)
b += per
for g in gaps:
    st, spre, scom = eng.bench_host_staged(tts[b:b + per], cnt[b:b + per], view[offs[b]:offs[b + per]], g)
    print(f"staged gap {g:6.0f}  prefetch {p50(spre):6.1f} us  commit {p50(scom):6.1f} us  "
          f"sum {p50(spre + scom):6.1f} us  (stage {p50(st):.1f} us)", flush=True)
    b += per
eng.close()
