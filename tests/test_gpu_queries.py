"""get_account_transfers / get_account_history on the GPU (query.hip) against the
CPU oracle, bit for bit, with queries interleaved between commits so that the
account-transfers index holds several runs and merges them (tbgpu_compact)."""
import numpy as np
import pytest

import oracle
from query_filters import random_filters
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import FILTER_DTYPE, QUERY_MAX, TRANSFER_DTYPE, account_filter

pytestmark = pytest.mark.gpu


def _engine(w, **kw):
    from tigerbeetle_amd.engine import Engine
    args = dict(accounts_max=len(w.accounts) + 16, transfers_max=len(w.transfers) + 1024,
                history_max=len(w.transfers) + 1024, events_per_call_max=1 << 17)
    args.update(kw)
    return Engine(**args)


def _rows(t):
    """(id, debit account, credit account, timestamp, flags) of each row, for failure messages."""
    return [(int(x["id_lo"]), int(x["debit_account_id_lo"]), int(x["credit_account_id_lo"]), int(x["timestamp"]),
             int(x["flags"])) for x in t[:4]]


def _interleaved(w, rounds, n_filters, seed, history_ids=None):
    orc, gpu = oracle.Oracle(len(w.accounts), len(w.transfers)), _engine(w)
    rng = np.random.default_rng(seed)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            _, rc = be.create_accounts_batches(ats, w.account_counts, w.accounts)
            assert int(rc.sum()) == 0
        counts = list(w.transfer_counts)
        cuts = np.linspace(0, len(counts), rounds + 1).astype(int)
        off = 0
        checked = 0
        for r in range(rounds):
            b0, b1 = cuts[r], cuts[r + 1]
            n = int(sum(counts[b0:b1]))
            for be in (orc, gpu):
                be.create_transfers_batches(tts[b0:b1], counts[b0:b1], w.transfers[off:off + n])
            off += n
            rows = orc.export_transfers()
            for f in random_filters(rng, w.accounts["id_lo"], rows, n_filters):
                g, o = gpu.get_account_transfers(f), orc.get_account_transfers(f)
                assert g.tobytes() == o.tobytes(), (r, f, _rows(g), _rows(o), _rows(gpu.lookup_transfers(
                    o["id_lo"].astype(object) + (o["id_hi"].astype(object) << 64))) if len(o) else None)
                checked += len(o) > 0
            if history_ids is not None:
                for f in random_filters(rng, history_ids, rows, n_filters // 2):
                    g, o = gpu.get_account_history(f), orc.get_account_history(f)
                    assert g.tobytes() == o.tobytes(), (r, f, len(g), len(o))
        assert checked > n_filters
        return gpu, orc
    except Exception:
        gpu.close()
        raise


def test_queries_flag_mix_with_history():
    w = workload.config3(batches=6, batch=2000, account_count=150, seed=21)
    hist = w.accounts["id_lo"][(w.accounts["flags"] & 8) != 0]
    assert len(hist) > 0
    gpu, _ = _interleaved(w, rounds=5, n_filters=120, seed=1, history_ids=hist)
    gpu.close()


def test_queries_long_segments_and_limit():
    """Few accounts, many transfers each: segments span many 256-entry chunks and
    exceed batch_max, so the limit cut and reversed order are exercised."""
    w = workload.config1(transfer_count=120_000, account_count=12, seed=5)
    gpu, orc = _interleaved(w, rounds=3, n_filters=60, seed=2)
    try:
        aid = int(w.accounts["id_lo"][3])
        for flags in (1, 2, 3, 5, 6, 7):
            f = account_filter(aid, flags=flags)
            g = gpu.get_account_transfers(f)
            assert len(g) == QUERY_MAX
            assert g.tobytes() == orc.get_account_transfers(f).tobytes()
    finally:
        gpu.close()


def test_queries_device_batch_matches_single():
    import torch
    w = workload.config1(transfer_count=40_000, account_count=300, seed=8)
    gpu, orc = _interleaved(w, rounds=2, n_filters=40, seed=3)
    try:
        rows = orc.export_transfers()
        fl = random_filters(np.random.default_rng(9), w.accounts["id_lo"], rows, 200)
        filters = np.concatenate(fl).astype(FILTER_DTYPE)
        stride = 256
        fd = gpu.to_device(filters)
        out = torch.empty(len(fl) * stride * 128, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        total, rc = gpu.query_device(fd.data_ptr(), len(fl), stride, out.data_ptr())
        host = out.cpu().numpy().view(TRANSFER_DTYPE).reshape(len(fl), stride)
        for q, f in enumerate(fl):
            f2 = f.copy()
            f2["limit"] = min(int(f["limit"][0]), stride)
            want = orc.get_account_transfers(f2)
            assert int(rc[q]) == len(want)
            assert host[q][:len(want)].tobytes() == want.tobytes()
        assert total == int(rc.sum())
    finally:
        gpu.close()


def test_queries_on_empty_state():
    w = workload.config1(transfer_count=10, account_count=4, seed=1)
    gpu = _engine(w)
    try:
        ats, _ = w.timestamps()
        gpu.create_accounts_batches(ats, w.account_counts, w.accounts)
        assert len(gpu.get_account_transfers(account_filter(1))) == 0
        assert len(gpu.get_account_history(account_filter(1))) == 0
        assert gpu.compact() == 0
    finally:
        gpu.close()
