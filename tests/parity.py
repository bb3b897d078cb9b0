"""Helpers comparing the GPU engine with the CPU oracle (bit-exact)."""
from __future__ import annotations

import numpy as np

from tigerbeetle_amd.types import RESULT_DTYPE


def sort_accounts(a: np.ndarray) -> np.ndarray:
    return a[np.lexsort((a["id_lo"], a["id_hi"]))]


def per_batch_results(results: np.ndarray, counts, result_counts):
    out, off = [], 0
    for c, rc in zip(counts, result_counts):
        out.append(results[off:off + int(rc)].copy())
        off += int(c)
    return out


def assert_results_equal(got, want, what="results"):
    for b, (g, w) in enumerate(zip(got, want)):
        if g.tobytes() != w.tobytes():
            gl = [(int(x["index"]), int(x["result"])) for x in g[:20]]
            wl = [(int(x["index"]), int(x["result"])) for x in w[:20]]
            raise AssertionError(f"{what}: batch {b} differs (len {len(g)} vs {len(w)}):\n got {gl}\nwant {wl}")


def assert_state_equal(gpu, orc):
    ga, oa = sort_accounts(gpu.export_accounts()), sort_accounts(orc.export_accounts())
    assert len(ga) == len(oa), (len(ga), len(oa))
    if ga.tobytes() != oa.tobytes():
        bad = np.nonzero(ga != oa)[0][:5]
        raise AssertionError(f"accounts differ at {bad}: gpu={ga[bad]} oracle={oa[bad]}")
    assert gpu.transfer_count() == orc.transfer_count(), (gpu.transfer_count(), orc.transfer_count())
    gt, ot = gpu.export_transfers(), orc.export_transfers()
    if gt.tobytes() != ot.tobytes():
        bad = np.nonzero(gt != ot)[0][:5]
        raise AssertionError(f"stored transfers differ at rows {bad}: gpu={gt[bad]} oracle={ot[bad]}")
    assert gpu.history_count() == orc.history_count()
    if gpu.export_history().tobytes() != orc.export_history().tobytes():
        raise AssertionError("account history differs")
    assert gpu.commit_timestamp() == orc.commit_timestamp(), (gpu.commit_timestamp(), orc.commit_timestamp())


def run_workload(backend, w, split=None):
    """Commit a workload's accounts then transfers; returns per-batch transfer results."""
    ats, tts = w.timestamps()
    r, rc = backend.create_accounts_batches(ats, w.account_counts, w.accounts)
    acc_res = per_batch_results(r, w.account_counts, rc)
    if split is None:
        res, rcs, _ = backend.create_transfers_batches(tts, w.transfer_counts, w.transfers)
        return acc_res, per_batch_results(res, w.transfer_counts, rcs)
    out, off, b = [], 0, 0
    counts = list(w.transfer_counts)
    while b < len(counts):
        k = min(split, len(counts) - b)
        n = int(sum(counts[b:b + k]))
        res, rcs, _ = backend.create_transfers_batches(tts[b:b + k], counts[b:b + k], w.transfers[off:off + n])
        out += per_batch_results(res, counts[b:b + k], rcs)
        off += n
        b += k
    return acc_res, out


EMPTY = np.zeros(0, dtype=RESULT_DTYPE)
