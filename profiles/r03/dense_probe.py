"""Round 3 diagnosis: tests/test_gpu_parity.py::test_dense_directory_boundaries failed once
(an account's balances behind the oracle's, every reply equal).  Run its workload a few
times on each path and report which path and how often the state differs.

    python profiles/r03/dense_probe.py [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402  (the checker)
from parity import per_batch_results, run_workload, sort_accounts  # noqa: E402
from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.engine import Engine  # noqa: E402
from tigerbeetle_amd.types import AccountFlags  # noqa: E402


def dense_workload():
    amax = 1000
    rng = np.random.default_rng(5)
    ids = [k for k in range(1, 600) if k % 7] + [998, 999, 1000, 1001, 1002, 5000] + \
          [(1 << 64) + k for k in range(1, 50)] + [(k << 70) | 3 for k in range(1, 30)]
    ids = ids[:amax]
    acc = workload.make_accounts(np.zeros(len(ids), dtype=np.uint64), ledger=1)
    for j, v in enumerate(ids):
        acc[j]["id_lo"], acc[j]["id_hi"] = v & ((1 << 64) - 1), v >> 64
    roll = rng.random(len(ids))
    acc["flags"] = np.where(roll < 0.1, int(AccountFlags.debits_must_not_exceed_credits),
                            np.where(roll < 0.15, int(AccountFlags.history), 0)).astype(np.uint16)
    pool = ids + [7, 14, 700, 1003, (1 << 64) + 77]
    n = 12_000
    t = np.zeros(n, dtype=workload.TRANSFER_DTYPE)
    t["id_lo"] = np.arange(1, n + 1)
    for i in range(n):
        d, c = pool[int(rng.integers(0, len(pool)))], pool[int(rng.integers(0, len(pool)))]
        t[i]["debit_account_id_lo"], t[i]["debit_account_id_hi"] = d & ((1 << 64) - 1), d >> 64
        t[i]["credit_account_id_lo"], t[i]["credit_account_id_hi"] = c & ((1 << 64) - 1), c >> 64
    t["amount_lo"] = rng.integers(1, 100, n)
    t["ledger"] = 1
    t["code"] = 1
    return workload.Workload("dense", acc, np.array([len(acc)], dtype=np.uint32), t,
                             np.array([3000] * 4, dtype=np.uint32)), amax


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    w, amax = dense_workload()
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    oa_res, ot_res = run_workload(orc, w)
    oacc = sort_accounts(orc.export_accounts())
    for fg in (False, True):
        for r in range(reps):
            gpu = Engine(accounts_max=amax, transfers_max=1 << 21, history_max=1 << 18, events_per_call_max=1 << 17,
                         force_general=fg)
            try:
                ga_res, gt_res = run_workload(gpu, w)
                same_replies = all(a.tobytes() == b.tobytes() for a, b in zip(gt_res, ot_res))
                gacc = sort_accounts(gpu.export_accounts())
                again = sort_accounts(gpu.export_accounts())
                bad = np.nonzero(gacc != oacc)[0]
                st = gpu.stats()
                print(f"general={fg} rep {r}: replies equal {same_replies}, accounts differing {len(bad)}"
                      f" {list(bad[:4])}, second export equal to first {gacc.tobytes() == again.tobytes()},"
                      f" path {st.path} passes {st.iterations}", flush=True)
                if len(bad):
                    print("   gpu", gacc[bad[:2]], "\n   orc", oacc[bad[:2]], flush=True)
            finally:
                gpu.close()


if __name__ == "__main__":
    main()
