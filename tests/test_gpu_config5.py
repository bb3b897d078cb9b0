"""BASELINE config 5 at its per-GPU size on one MI355X.

100M accounts and one shard's 125M transfers (1B over 8 ledger shards), streamed as
back-to-back 8190-transfer batches, the load generated in HBM (workload.config5,
csrc/loadgen.hip), on a ledger-shard ctx (tbgpu_options.shard_world = 8): the
directory knows all 100M accounts, the 128-byte rows are the shard's own 12.5M.
Checked over the whole state:

- capacity: 100M accounts in the direct-mapped directory (row + 1 in 29 bits, rows
  only for the shard's ledgers) and 125M stored rows in the transfer-id index;
- every transfer is accepted (all accounts exist, ids are new) and stored;
- conservation: total debits_posted == total credits_posted == the sum of the
  amounts, and accounts outside the shard's ledgers never move;
- idempotence: re-submitting a committed batch answers `exists` for every event
  and changes nothing;
- oracle parity on the leading batches: the CPU oracle, given the accounts those
  batches touch, returns the same replies, balances and stored rows
  (src/state_machine.zig:1239-1368).
"""
import numpy as np
import pytest

import oracle
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import ACCOUNT_DTYPE, BATCH_MAX, TRANSFER_DTYPE

pytestmark = pytest.mark.gpu

EXISTS = 46  # CreateTransferResult.exists (src/tigerbeetle.zig:165-245)


def _sum128(lo, hi):
    return int(lo.astype(object).sum()) + (int(hi.astype(object).sum()) << 64)


def test_config5_per_gpu_shard():
    import torch
    from tigerbeetle_amd import engine as E

    dev = torch.device("cuda", 0)
    c5 = workload.config5(shard=0)
    assert c5.accounts < (1 << 29) - 1, "the directory's row field is 29 bits"
    assert c5.transfers < (1 << 31) - 1, "the transfer-id index holds u32 row + 1"
    per_call = 1000  # batches per streamed call
    owned = c5.owned_accounts()
    eng = E.Engine(accounts_max=owned, directory_max=c5.accounts, hashed_max=1024,
                   transfers_max=c5.transfers + 2 * BATCH_MAX, history_max=1024,
                   events_per_call_max=per_call * BATCH_MAX, shard_world=c5.shards, shard_rank=c5.shard)
    try:
        ats, tts = c5.timestamps()
        # accounts, 10M per generated slice
        ab = c5.account_batches()
        slice_batches = 1221  # 10,000,890 accounts
        buf = torch.empty(slice_batches * BATCH_MAX * 128, dtype=torch.uint8, device=dev)
        res = torch.empty(slice_batches * BATCH_MAX * 8, dtype=torch.uint8, device=dev)
        first = 1
        for b0 in range(0, len(ab), slice_batches):
            cnt = ab[b0:b0 + slice_batches]
            n = int(cnt.sum())
            E.generate_accounts(0, first, n, c5.accounts_per_ledger, buf.data_ptr())
            total, _ = eng.create_accounts_batches_device(ats[b0:b0 + len(cnt)], cnt, buf.data_ptr(), res.data_ptr())
            assert total == 0, "account creation failed"
            first += n
        assert eng.account_count() == owned  # rows: this shard's ledgers only
        del buf, res

        tb = c5.transfer_batches()
        offs = np.concatenate([[0], np.cumsum(tb.astype(np.int64))])
        ev = torch.empty(per_call * BATCH_MAX * 128, dtype=torch.uint8, device=dev)
        res = torch.empty(per_call * BATCH_MAX * 8, dtype=torch.uint8, device=dev)
        amount_sum = 0

        # leading batches: their own call, then checked against the oracle
        lead = 4
        n_lead = int(offs[lead])
        E.generate_transfers(0, c5.first_transfer_id, n_lead, c5.seed, c5.ledger0, c5.ledgers,
                             c5.accounts_per_ledger, ev.data_ptr(), ledger_stride=c5.ledger_stride)
        lead_ev = ev[:n_lead * 128].cpu().numpy().view(TRANSFER_DTYPE).copy()
        total, rc = eng.create_transfers_batches_device(tts[:lead], tb[:lead], ev.data_ptr(), res.data_ptr())
        assert total == 0
        amount_sum += int(lead_ev["amount_lo"].astype(np.uint64).astype(object).sum())
        ids = np.unique(np.concatenate([lead_ev["debit_account_id_lo"], lead_ev["credit_account_id_lo"]]))
        acc = np.zeros(len(ids), dtype=ACCOUNT_DTYPE)
        acc["id_lo"] = ids
        acc["ledger"] = ((ids - 1) // c5.accounts_per_ledger + 1).astype(np.uint32)
        acc["code"] = 1
        orc = oracle.Oracle(len(ids), n_lead)
        try:
            orc.create_accounts_batches(np.array([ats[-1]], dtype=np.uint64), np.array([len(acc)], np.uint32), acc)
            o, orc_rc, _ = orc.create_transfers_batches(tts[:lead], tb[:lead], lead_ev)
            assert int(orc_rc.sum()) == 0 and np.array_equal(rc, orc_rc)
            g_acc = eng.lookup_accounts([int(x) for x in ids])
            o_acc = orc.lookup_accounts([int(x) for x in ids])
            for f in ("id", "debits_pending", "debits_posted", "credits_pending", "credits_posted"):
                for part in ("_lo", "_hi"):
                    assert np.array_equal(g_acc[f + part], o_acc[f + part]), f
            assert eng.export_transfers(0, n_lead).tobytes() == orc.export_transfers().tobytes()
        finally:
            orc.close()

        # the rest of the shard's transfers, streamed in calls of 1000 batches
        b = lead
        while b < len(tb):
            k = min(per_call, len(tb) - b)
            n = int(offs[b + k] - offs[b])
            E.generate_transfers(0, c5.first_transfer_id + int(offs[b]), n, c5.seed, c5.ledger0, c5.ledgers,
                                 c5.accounts_per_ledger, ev.data_ptr(), ledger_stride=c5.ledger_stride)
            amount_sum += int(ev[:n * 128].view(torch.int64).view(n, 16)[:, 6].sum().item())
            total, _ = eng.create_transfers_batches_device(tts[b:b + k], tb[b:b + k], ev.data_ptr(), res.data_ptr())
            assert total == 0, f"calls at batch {b}: {total} failures"
            b += k
        assert eng.transfer_count() == c5.transfers

        # conservation over the whole state
        a = eng.export_accounts()
        assert len(a) == owned
        assert (a["ledger"] % c5.shards == c5.shard).all()
        dpo = _sum128(a["debits_posted_lo"], a["debits_posted_hi"])
        cpo = _sum128(a["credits_posted_lo"], a["credits_posted_hi"])
        assert dpo == cpo == amount_sum
        assert not a["debits_pending_lo"].any() and not a["credits_pending_lo"].any()
        del a
        # another shard's account: in the directory (a transfer naming it with this
        # shard's ledger fails on the ledger, not as not-found), but no row here
        other = c5.accounts_per_ledger + 1  # ledger 2 (shard 2 of 8)
        assert len(eng.lookup_accounts([other])) == 0

        # idempotence: the first batch again (a new prepare timestamp)
        E.generate_transfers(0, c5.first_transfer_id, BATCH_MAX, c5.seed, c5.ledger0, c5.ledgers,
                             c5.accounts_per_ledger, ev.data_ptr(), ledger_stride=c5.ledger_stride)
        before = eng.lookup_accounts([int(x) for x in ids[:1000]])
        total, rc = eng.create_transfers_batches_device(np.array([tts[-1] + BATCH_MAX + 1], np.uint64),
                                                        np.array([BATCH_MAX], np.uint32), ev.data_ptr(),
                                                        res.data_ptr())
        assert total == BATCH_MAX
        r = res[:BATCH_MAX * 8].cpu().numpy().view(np.uint32).reshape(-1, 2)
        assert (r[:, 1] == EXISTS).all() and np.array_equal(r[:, 0], np.arange(BATCH_MAX))
        assert eng.transfer_count() == c5.transfers
        assert eng.lookup_accounts([int(x) for x in ids[:1000]]).tobytes() == before.tobytes()
    finally:
        eng.close()
