"""Debug: the walk (TBGPU_OPT_WALK_EARLY) vs the oracle on test_walk_matches_the_passes[config3]."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle
from parity import run_workload
from tigerbeetle_amd import workload
from tigerbeetle_amd.engine import Engine
from tigerbeetle_amd.types import BATCH_MAX

for rep, mk in [(0, workload.config3), (1, workload.config3), (2, workload.config3_stress), (3, workload.config3)]:
  w = mk(batches=6, account_count=2_000, seed=21)
  n = len(w.transfers)
  for walk in (True,):
    print("rep", rep, mk.__name__)
    orc = oracle.Oracle(len(w.accounts), n)
    gpu = Engine(accounts_max=max(len(w.accounts), 1024), transfers_max=n + 1024, history_max=n + 1024,
                 events_per_call_max=max(int(w.transfer_counts.max()) * 2, min(n, 210 * BATCH_MAX)),
                 force_general=True, walk_early=walk)
    oa, ot = run_workload(orc, w)
    ga, gt = run_workload(gpu, w, split=2)
    print("walk", walk, "walks", gpu.stats().walks)
    off = 0
    for b, (g, o) in enumerate(zip(gt, ot)):
        gd = {int(x["index"]): int(x["result"]) for x in g}
        od = {int(x["index"]): int(x["result"]) for x in o}
        diff = sorted(set(gd) | set(od))
        diff = [i for i in diff if gd.get(i, 0) != od.get(i, 0)]
        if diff:
            print(f" batch {b}: {len(diff)} differ; first: {[(i, gd.get(i, 0), od.get(i, 0)) for i in diff[:12]]}")
            for i in diff[:4]:
                t = w.transfers[off + i]
                print("   ev", i, "flags", int(t["flags"]), "dr", int(t["debit_account_id_lo"]), "cr", int(t["credit_account_id_lo"]),
                      "amt", int(t["amount_lo"]), "pend", int(t["pending_id_lo"]), "id", int(t["id_lo"]))
        off += int(w.transfer_counts[b])
    gpu.close(); orc.close()
