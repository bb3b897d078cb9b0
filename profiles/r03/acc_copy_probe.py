"""Round 3 diagnosis: create_accounts on a fresh ctx whose buffers start zeroed reads
zero ids for scattered events (tests/test_gpu_general.py relay chain).  Which input
path shows it: pageable host memory (runtime-staged copy), page-locked host memory
(a plain DMA copy), or events already in device memory (no copy)?

    python profiles/r03/acc_copy_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from tigerbeetle_amd import workload
from tigerbeetle_amd.engine import Engine
from tigerbeetle_amd.types import ACCOUNT_DTYPE, RESULT_DTYPE, AccountFlags


def accounts(n):
    a = workload.make_accounts(np.arange(1, n + 1, dtype=np.uint64), ledger=1,
                               flags=int(AccountFlags.debits_must_not_exceed_credits))
    a[-1]["flags"] = 0
    return a


def engine(n):
    return Engine(accounts_max=max(n, 1024), transfers_max=n + 1024, history_max=n + 1024,
                  events_per_call_max=2 * 8190)


def run(kind, n):
    acc = accounts(n)
    e = engine(n)
    try:
        ts = np.array([1 << 40], dtype=np.uint64)
        cs = np.array([n], dtype=np.uint32)
        if kind == "pageable":
            out, rc = e.create_accounts_batches(ts, cs, acc)
            res = out[:int(rc.sum())]
        elif kind == "pinned":
            buf = torch.empty(n * 128, dtype=torch.uint8, pin_memory=True)
            view = buf.numpy().view(ACCOUNT_DTYPE)
            view[:] = acc
            out, rc = e.create_accounts_batches(ts, cs, view)
            res = out[:int(rc.sum())]
        else:  # device
            dev = torch.from_numpy(acc.view(np.uint8).copy()).cuda()
            rdev = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            total, rc = e.create_accounts_batches_device(ts, cs, dev.data_ptr(), rdev.data_ptr())
            res = rdev[:total * 8].cpu().numpy().view(RESULT_DTYPE)
        bad = res[res["result"] != 0]
        idx = [int(x) for x in bad["index"][:12]]
        print(f"{kind:9s} n={n}: {len(bad)} failures {idx}", flush=True)
    finally:
        e.close()


if __name__ == "__main__":
    for rep in range(2):
        for kind in ("pageable", "pinned", "device"):
            run(kind, 8191)
    run("pageable", 8190)
    run("pageable", 4096)
    run("pageable", 16380)
