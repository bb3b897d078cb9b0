"""Bit-exact parity of the HIP engine with the CPU oracle on seeded workloads.

Compares, per batch, the sparse results, then the whole state: every account row,
every stored transfer row in commit order, the account-history rows, the posted
groove and commit_timestamp.
"""
import numpy as np
import pytest

import oracle
from parity import assert_results_equal, assert_state_equal, per_batch_results, run_workload
from tigerbeetle_amd import workload

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from tigerbeetle_amd.engine import Engine
    args = dict(accounts_max=1 << 17, transfers_max=1 << 21, history_max=1 << 18, events_per_call_max=1 << 17)
    args.update(kw)
    return Engine(**args)


@pytest.fixture(params=[False, True], ids=["auto", "general"])
def force_general(request):
    return request.param


def _parity(w, split=None, **kw):
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    gpu = _engine(**kw)
    try:
        oa, ot = run_workload(orc, w)
        ga, gt = run_workload(gpu, w, split=split)
        assert_results_equal(ga, oa, "create_accounts")
        assert_results_equal(gt, ot, "create_transfers")
        assert_state_equal(gpu, orc)
        return gpu.stats()
    finally:
        gpu.close()


def test_config1_small(force_general):
    _parity(workload.config1(transfer_count=50_000, account_count=1000), force_general=force_general)


def test_config1_batch_by_batch(force_general):
    _parity(workload.config1(transfer_count=20_000, account_count=500), split=1, force_general=force_general)


def test_config2_small_zipf(force_general):
    _parity(workload.config2(transfer_count=100_000, account_count=20_000), force_general=force_general)


def test_config3_flag_mix(force_general):
    _parity(workload.config3(batches=6, batch=2000, account_count=2000), force_general=force_general)


def test_config3_batch_by_batch(force_general):
    _parity(workload.config3(batches=4, batch=1000, account_count=500, seed=7), split=1, force_general=force_general)


def test_config3_full_batches(force_general):
    _parity(workload.config3(batches=4, account_count=10_000, seed=3), force_general=force_general)


def test_config3_stress_flag_mix(force_general):
    _parity(workload.config3_stress(batches=6, batch=2000, account_count=2000), force_general=force_general)


def test_config3_stress_batch_by_batch(force_general):
    _parity(workload.config3_stress(batches=4, batch=1000, account_count=500, seed=7), split=1,
            force_general=force_general)


def test_posted_groove():
    w = workload.config3(batches=3, batch=1500, account_count=800, seed=11)
    orc = oracle.Oracle()
    gpu = _engine()
    try:
        run_workload(orc, w)
        run_workload(gpu, w)
        pend = w.transfers[(w.transfers["flags"] & 2) != 0]["id_lo"][:500]
        for pid in pend:
            assert gpu.get_posted(int(pid)) == orc.get_posted(int(pid))
    finally:
        gpu.close()


def test_lookups_match():
    w = workload.config1(transfer_count=5000, account_count=300)
    orc, gpu = oracle.Oracle(), _engine()
    try:
        run_workload(orc, w)
        run_workload(gpu, w)
        ids = list(range(0, 400)) + [(1 << 128) - 1]
        assert gpu.lookup_accounts(ids).tobytes() == orc.lookup_accounts(ids).tobytes()
        tids = list(range(0, 6000, 7)) + [(1 << 128) - 1]
        assert gpu.lookup_transfers(tids).tobytes() == orc.lookup_transfers(tids).tobytes()
    finally:
        gpu.close()


def test_fast_path_is_taken_for_plain_batches():
    w = workload.config2(transfer_count=30_000, account_count=5_000)
    gpu = _engine()
    try:
        run_workload(gpu, w)
        st = gpu.stats()
        assert st.path == 1 and st.iterations == 1
    finally:
        gpu.close()


def test_fast_path_falls_back_exactly():
    """Plain batches followed by one duplicate id: the fast attempt undoes its deltas."""
    w = workload.config1(transfer_count=20_000, account_count=300, seed=9)
    t = w.transfers.copy()
    t[15_000]["id_lo"] = t[14_000]["id_lo"]  # duplicate inside one call
    t[16_000]["amount_lo"] = 0               # a static failure next to it
    w.transfers = t
    _parity(w)


def test_fallback_keeps_commit_timestamp():
    """The last event of a call repeats an earlier id of the same call: the fast
    attempt classified it ok against the pre-call state (and saw its timestamp), but
    sequentially it is `exists`, so commit_timestamp stays at the previous event's
    (src/state_machine.zig:1366 only advances on ok).  Also with a post as the last
    event, whose id a plain transfer took earlier in the call."""
    for seed in (1, 2):
        w = workload.config1(transfer_count=9_000, account_count=200, seed=seed)
        t = w.transfers.copy()
        t[-1]["id_lo"] = t[-3]["id_lo"]  # exists_with_different_* at the very end
        w.transfers = t
        _parity(w)
        _parity(w, split=1)


def test_overflow_guard_routes_to_general():
    """Huge balances (high words >= 2^62) are never handled by the fast path."""
    from table import check
    text = """
account A1 0 0 0 0 _ _ _ _ L1 C1 _ _ _ _ _ ok
account A2 0 0 0 0 _ _ _ _ L1 C1 _ _ _ _ _ ok
commit create_accounts
setup A1 0 -10 0 0
setup A2 0 0 0 -20
transfer T1 A1 A2 5 _ _ _ _ _ L1 C1 _ _ _ _ _ _ _ _ ok
transfer T2 A1 A2 6 _ _ _ _ _ L1 C1 _ _ _ _ _ _ _ _ overflows_debits_posted
transfer T3 A2 A1 9 _ _ _ _ _ L1 C1 _ _ _ _ _ _ _ _ ok
commit create_transfers
lookup_account A1 0 -5 0 9
commit lookup_accounts
"""
    gpu = _engine()
    try:
        check(gpu, text)
    finally:
        gpu.close()


def _h64_table(last_amount: int) -> str:
    """Eight accounts just under 2^61 (the 64-bit headroom form's entry bound) whose
    balancing debits pile their headroom onto A9 inside one call: A9's figures leave
    +-2^63 during the fixed point.  (No transfer takes an account across 2^61 before the
    call's fixed point: the fast path's attempt, undone, would set the guard bit.)"""
    top = (1 << 61) - 1
    lines = [f"account A{k} 0 0 0 0 _ _ _ _ L1 C1 _ _ _ _ _ ok" for k in range(1, 11)]
    lines.append("commit create_accounts")
    lines += [f"setup A{k} 0 0 0 {top}" for k in range(1, 9)]
    lines += [f"transfer T{k} A{k} A9 0 _ _ _ _ _ L1 C1 _ _ _ _ BDR _ _ _ ok" for k in range(1, 9)]
    lines.append("transfer T9 A9 A10 5 _ _ _ _ _ L1 C1 _ _ _ _ _ _ _ _ ok")
    lines.append(f"transfer T10 A10 A9 {last_amount} _ _ _ _ _ L1 C1 _ _ _ _ _ _ _ _ ok")
    lines.append("commit create_transfers")
    lines += [f"lookup_account A{k} 0 {top} 0 {top}" for k in range(1, 9)]
    lines.append(f"lookup_account A9 0 5 0 {8 * top + last_amount}")
    lines.append(f"lookup_account A10 0 {last_amount} 0 5")
    lines.append("commit lookup_accounts")
    return "\n".join(lines)


@pytest.mark.parametrize("big_amount", [False, True], ids=["h64-redo", "wide64"])
def test_h64_headroom_overflow_redoes_the_chunk(big_amount):
    """A chunk in the 64-bit headroom form (amounts < 2^40, balances < 2^61) whose
    balancing transfers carry one account's figures past +-2^63 raises FL_H64_OVER,
    applies nothing and is redone in the u128 form, with the oracle's results.  With an
    amount >= 2^40 in the call the chunk never takes the 64-bit form."""
    from table import check
    text = _h64_table(1 << 40 if big_amount else 1)
    orc = oracle.Oracle(64, 64)
    try:
        check(orc, text)
    finally:
        orc.close()
    gpu = _engine()
    try:
        check(gpu, text)
        assert gpu.stats().h64_redos == (0 if big_amount else 1), gpu.stats().h64_redos
    finally:
        gpu.close()


def test_h64_long_segments_keep_the_form():
    """Zipf-hot accounts on the general path: their segments outgrow the fused scan's
    window, so the passes switch to the three-launch Bal4 scan, which reads the chunk's
    64-bit delta records (no redo: no balance nears 2^62)."""
    st = _parity(workload.config2(transfer_count=100_000, account_count=20_000, seed=5), force_general=True)
    assert st.h64_redos == 0, st.h64_redos


@pytest.mark.parametrize("order", ["increasing", "random"])
def test_guarded_fast_path_many_calls(order):
    """Once any balance's high word reaches 2^62 every event takes the guarded
    classification.  Many consecutive calls must stay on the fast path (no claim of
    the in-call duplicate table may leak from one call into the next) and match the
    oracle, with ids in order and in random order."""
    w = workload.config1(transfer_count=12 * 4000, account_count=300, seed=31, batch=4000)
    extra = workload.make_accounts(np.array([10_000], dtype=np.uint64), ledger=2)  # never transferred
    w.accounts = np.concatenate([w.accounts, extra])
    w.account_counts = np.array([len(w.accounts)], dtype=np.uint32)
    if order == "random":
        t = w.transfers.copy()
        t["id_lo"] = np.random.default_rng(2).permutation(t["id_lo"])
        w.transfers = t
    orc, gpu = oracle.Oracle(), _engine(events_per_call_max=1 << 14)
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
            be.set_balances(10_000, 0, 1 << 127, 0, 0)
        off = 0
        for b, c in enumerate(w.transfer_counts):
            ev = w.transfers[off:off + int(c)]
            g = gpu.create_transfers(int(tts[b]), ev)
            o = orc.create_transfers(int(tts[b]), ev)
            assert g.tobytes() == o.tobytes(), f"call {b}"
            assert gpu.stats().path == 1, f"call {b} left the fast path"
            off += int(c)
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_random_id_order():
    """Ids in random order (benchmark --id-order=random): the fast path must run its
    in-call duplicate check and still match the oracle, with and without repeats."""
    w = workload.config1(transfer_count=40_000, account_count=700, seed=13)
    rng = np.random.default_rng(1)
    t = w.transfers.copy()
    t["id_lo"] = rng.permutation(t["id_lo"])
    w.transfers = t
    st = _parity(w)
    assert st.path == 1
    t2 = t.copy()
    t2[30_000]["id_lo"] = t2[29_999]["id_lo"]  # a repeat inside the last call
    w.transfers = t2
    _parity(w)


def test_withdrawn_id_claims_rebuild_the_index():
    """Random ids (eager claims in fp_commit) in linked pairs whose second member fails
    four times in five: each broken pair withdraws its first member's claim, leaving a
    tombstone in the transfer-id index.  Past 1/16 of the slots the engine rebuilds the
    index from the stored rows (xidx_tombs_check); replies, state and lookups still
    match the oracle."""
    from tigerbeetle_amd.types import TransferFlags
    w = workload.config1(transfer_count=40 * 256, account_count=300, seed=31, batch=256, id_order="random")
    rng = np.random.default_rng(31)
    t = w.transfers
    for i in range(0, len(t) - 1, 2):
        t[i]["flags"] |= np.uint16(int(TransferFlags.linked))
        if rng.random() < 0.8:
            t[i + 1]["credit_account_id_lo"] ^= np.uint64(0x5A5A)  # no such account
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    # (load <= 1/2: the tombstones reach 1/16 of the slots within the workload)
    gpu = _engine(transfers_max=1 << 13, history_max=1 << 10, events_per_call_max=1 << 12, dense_indexes=True)
    try:
        oa, ot = run_workload(orc, w)
        ga, gt = run_workload(gpu, w, split=1)
        assert_results_equal(gt, ot, "create_transfers")
        assert_state_equal(gpu, orc)
        assert gpu.stats().index_rebuilds > 0, gpu.stats().index_rebuilds
        # every id through the rebuilt index: the stored ones found, the withdrawn not
        q = t[["id_lo", "id_hi"]]
        ids = [(int(h) << 64) | int(lo) for lo, h in zip(q["id_lo"], q["id_hi"])]
        for c0 in range(0, len(ids), 4096):
            got = gpu.lookup_transfers(ids[c0:c0 + 4096])
            want = orc.lookup_transfers(ids[c0:c0 + 4096])
            assert got.tobytes() == want.tobytes(), (c0, len(got), len(want))
        # later calls still claim and find ids after the rebuild
        w2 = workload.config1(transfer_count=4 * 256, account_count=300, seed=32, batch=256, id_order="random")
        t2 = w2.transfers
        t2[100] = t[0]  # an id seen before the rebuild (stored or withdrawn)
        ts = int(orc.commit_timestamp()) + 10_000
        for b in range(4):
            ev = np.ascontiguousarray(t2[b * 256:(b + 1) * 256])
            assert gpu.create_transfers(ts + b * 1000, ev).tobytes() == orc.create_transfers(ts + b * 1000, ev).tobytes()
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_eager_claim_of_a_broken_chain_is_not_an_existing_id():
    """Random ids, eager claims (the ctx saw non-rising ids in its first call): the second
    call, 1M events in one streamed call (≈2000 tiles of fp_commit, more than the chip
    holds at once), starts with an event linked to a partner that fails, so its claim is
    withdrawn after fp_commit; the call's last events repeat its id.  If their tiles
    classify after the first tile claimed the id and stored its optimistic row, a probe
    that compared this call's claimed rows would answer `exists` (fp_classify probes only
    rows committed before the call, xidx_committed); the sequential answer is `ok` for
    the first repeat (the first event failed) and `exists_with_different_amount` for the
    second."""
    from tigerbeetle_amd.types import TransferFlags
    nb = 1 + 122
    w = workload.config1(transfer_count=nb * 8190, account_count=500, seed=41, id_order="random")
    t = w.transfers
    a = 8190  # the second call's first event
    t[a]["flags"] |= np.uint16(int(TransferFlags.linked))
    t[a + 1]["credit_account_id_lo"] ^= np.uint64(0x77)  # no such account: the chain breaks
    last = len(t) - 1
    for b in (last - 2, last):
        t[b]["id_lo"], t[b]["id_hi"] = t[a]["id_lo"], t[a]["id_hi"]
    t[last]["amount_lo"] += np.uint64(1)
    orc = oracle.Oracle(len(w.accounts), len(w.transfers))
    gpu = _engine(transfers_max=1 << 21, events_per_call_max=1 << 20)  # the second call is one chunk
    try:
        ats, tts = w.timestamps()
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        got, want = [], []
        for b0, b1 in ((0, 1), (1, nb)):
            e0, e1 = b0 * 8190, b1 * 8190
            for be, out in ((gpu, got), (orc, want)):
                res, rc, _ = be.create_transfers_batches(tts[b0:b1], w.transfer_counts[b0:b1], t[e0:e1])
                out.append(res[:int(rc.sum())].copy())
        assert_results_equal(got, want, "create_transfers")
        assert_state_equal(gpu, orc)
    finally:
        gpu.close()


def test_fast_path_with_failures():
    """Static failures, unknown accounts and re-submitted ids stay on the fast path:
    rows are re-placed at their ranks (fp_fix) and the replies are exact."""
    w = workload.config1(transfer_count=30_000, account_count=400, seed=21)
    t = w.transfers.copy()
    t[100]["amount_lo"] = 0                          # amount_must_not_be_zero
    t[9_000]["debit_account_id_lo"] = 10_000_000     # debit_account_not_found
    t[12_345]["ledger"] = 0                          # ledger_must_not_be_zero
    t[29_000:29_100] = t[0:100]                      # exists (same ids, earlier calls)
    t[29_100]["id_lo"] = t[5]["id_lo"]               # exists_with_different_* (other fields)
    w.transfers = t
    st = _parity(w, split=1)
    assert st.path == 1
    st = _parity(w, split=2)


def _chainy_config1(seed, n=40_000, accounts=800):
    """config 1 with linked chains of 2-6 events, some with a failing member (unknown
    account, amount 0, a repeated id) and open chains at batch ends."""
    from tigerbeetle_amd.types import TransferFlags
    w = workload.config1(transfer_count=n, account_count=accounts, seed=seed)
    rng = np.random.default_rng(seed)
    t = w.transfers
    i = 0
    while i < n - 1:
        if rng.random() < 0.15:
            ln = int(rng.integers(2, 7))
            for q in range(i, min(i + ln - 1, n - 1)):
                t[q]["flags"] |= np.uint16(int(TransferFlags.linked))
            if rng.random() < 0.2:
                v = i + int(rng.integers(0, ln))
                if v < n:
                    kind = int(rng.integers(0, 3))
                    if kind == 0:
                        t[v]["debit_account_id_lo"] = accounts + 5
                    elif kind == 1:
                        t[v]["amount_lo"] = 0
                    elif v > 0:
                        t[v]["id_lo"] = t[v - 1]["id_lo"]
            i += ln
        else:
            i += 1
    ends = np.cumsum(w.transfer_counts) - 1
    for e in ends[rng.random(len(ends)) < 0.3]:
        t[e]["flags"] |= np.uint16(int(TransferFlags.linked))
    return w


def test_fast_path_linked_chains():
    st = _parity(_chainy_config1(3))
    assert st.path in (0, 1)


def test_fast_path_linked_chains_batch_by_batch():
    _parity(_chainy_config1(4, n=12_000, accounts=300), split=1)


def test_config4_cross_ledger_pairs_on_fast_path():
    w = workload.config4(transfer_count=60_000, ledgers=20, accounts_per_ledger=200, seed=9, cross_ledger_pairs=0.02)
    st = _parity(w)
    assert st.path == 1, "config 4 (valid linked pairs) should stay on the single-pass path"


def test_dense_directory_boundaries():
    """Account ids 1..accounts_max use the direct-mapped directory, others the hash
    index: mix both in every batch, with ids on either side of the boundary, ids in
    range that were never created, u128 ids, and limit/history flags read through
    the directory."""
    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.types import AccountFlags
    amax = 1000  # engine accounts_max: the directory covers ids 1..1000
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
    pool = ids + [7, 14, 700, 1003, (1 << 64) + 77]  # never created: in range and out of it
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
    w = workload.Workload("dense", acc, np.array([len(acc)], dtype=np.uint32), t,
                          np.array([3000] * 4, dtype=np.uint32))
    plain = w.transfers.copy()
    for fg in (False, True):
        _parity(w, accounts_max=amax, force_general=fg)
        _parity(w, split=1, accounts_max=amax, force_general=fg)
    # without flagged accounts every call stays on the fast path
    w.accounts = acc.copy()
    w.accounts["flags"] = 0
    w.transfers = plain
    st = _parity(w, accounts_max=amax)
    assert st.path == 1


def test_blocked_dense_directory(force_general):
    """tbgpu_options.dense_block_span: ledger-major ids (ledger << 32 | k) in the
    direct-mapped directory (config 4's numbering), with ids past the span, in block
    0, beyond the last block and never created mixed in, plus limit flags read
    through the directory; and the config-4 workload itself with the span set."""
    from tigerbeetle_amd.types import AccountFlags
    span, ledgers = 50, 8
    rng = np.random.default_rng(17)
    ids = [(l << 32) | k for l in range(1, ledgers + 1) for k in range(1, span + 1) if (l + k) % 5] + \
          [(1 << 32) | (span + 1), (2 << 32) | (span + 7), 3, span, ((ledgers + 9) << 32) | 1, (1 << 64) | 5]
    acc = workload.make_accounts(np.zeros(len(ids), dtype=np.uint64), ledger=1)
    for j, v in enumerate(ids):
        acc[j]["id_lo"], acc[j]["id_hi"] = v & ((1 << 64) - 1), v >> 64
    acc["flags"] = np.where(rng.random(len(ids)) < 0.1, int(AccountFlags.debits_must_not_exceed_credits),
                            0).astype(np.uint16)
    pool = ids + [(1 << 32) | 5, (4 << 32), ((ledgers + 1) << 32) | 3, (2 << 32) | (span + 2)]  # never created
    n = 9_000
    t = np.zeros(n, dtype=workload.TRANSFER_DTYPE)
    t["id_lo"] = np.arange(1, n + 1)
    for i in range(n):
        d, c = pool[int(rng.integers(0, len(pool)))], pool[int(rng.integers(0, len(pool)))]
        t[i]["debit_account_id_lo"], t[i]["debit_account_id_hi"] = d & ((1 << 64) - 1), d >> 64
        t[i]["credit_account_id_lo"], t[i]["credit_account_id_hi"] = c & ((1 << 64) - 1), c >> 64
    t["amount_lo"] = rng.integers(1, 100, n)
    t["ledger"] = 1
    t["code"] = 1
    w = workload.Workload("blocked", acc, np.array([len(acc)], dtype=np.uint32), t,
                          np.array([3000] * 3, dtype=np.uint32))
    _parity(w, accounts_max=ledgers * span, dense_block_span=span, force_general=force_general)
    w4 = workload.config4(transfer_count=40_000, ledgers=20, accounts_per_ledger=200, seed=3, cross_ledger_pairs=0.02)
    st = _parity(w4, accounts_max=20 * 200, dense_block_span=200, force_general=force_general)
    assert force_general or st.path == 1


def test_sorted_run_id_index():
    """The id index's sorted run (engine.h xrun): monotone fast calls extend it
    without hashing; then ids replayed from it answer `exists` (binary search),
    posts and voids find pendings that live only in the run, a non-monotone call and
    a call after a frozen run hash their ids, lookups see both, and a checkpoint
    restores everything into the hash index -- all bit-exact vs the oracle."""
    from tigerbeetle_amd.types import TRANSFER_DTYPE, TransferFlags
    rng = np.random.default_rng(17)
    w = workload.config1(transfer_count=8 * 8190, account_count=500, seed=3)
    t = w.transfers
    t["flags"][::5] = int(TransferFlags.pending)  # pendings that only the run will hold
    ats, tts = w.timestamps()
    calls = []
    # 1-2: monotone plain calls (the run starts, then grows)
    calls.append(t[:2 * 8190].copy())
    calls.append(t[2 * 8190:4 * 8190].copy())
    # 3: replays of run ids (exists / exists_with_different_*) next to new ids
    c3 = t[4 * 8190:5 * 8190].copy()
    rep = rng.choice(4 * 8190, 600, replace=False)
    c3[:600] = t[rep]
    c3["amount_lo"][:300] += 1
    calls.append(c3)
    # 4: posts and voids of pendings committed in the run (the general path)
    pend = np.nonzero(t["flags"][:4 * 8190] == int(TransferFlags.pending))[0][:4000]
    c4 = np.zeros(len(pend), dtype=TRANSFER_DTYPE)
    c4["id_lo"] = 10_000_000 + np.arange(len(pend))
    c4["pending_id_lo"] = t["id_lo"][pend]
    c4["flags"] = np.where(np.arange(len(pend)) % 2 == 0, int(TransferFlags.post_pending_transfer),
                           int(TransferFlags.void_pending_transfer))
    calls.append(c4)
    # 5: monotone again (the run is frozen: hashed); 6: non-monotone ids
    calls.append(t[5 * 8190:6 * 8190].copy())
    c6 = t[6 * 8190:8 * 8190].copy()
    rng.shuffle(c6)
    calls.append(c6)
    orc = oracle.Oracle(len(w.accounts), 1 << 20)
    gpu = _engine()
    try:
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        ts = int(ats[-1])
        for k, ev in enumerate(calls):
            counts = np.full(len(ev) // 8190, 8190, dtype=np.uint32)
            if len(ev) % 8190:
                counts = np.append(counts, len(ev) % 8190).astype(np.uint32)
            bts = ts + np.cumsum(counts.astype(np.uint64) + 1)
            ts = int(bts[-1])
            go, gr, _ = gpu.create_transfers_batches(bts, counts, ev)
            oo, orr, _ = orc.create_transfers_batches(bts, counts, ev)
            assert np.array_equal(gr, orr), k
            assert_results_equal(per_batch_results(go, counts, gr), per_batch_results(oo, counts, orr), f"call {k}")
            if k == 2:
                assert int(gr.sum()) >= 600  # every replayed id answered from the run
        assert_state_equal(gpu, orc)
        ids = t["id_lo"][::7].tolist() + c4["id_lo"][::5].tolist() + [0, 99_999_999]
        assert gpu.lookup_transfers(ids).tobytes() == orc.lookup_transfers(ids).tobytes()
        image = gpu.checkpoint()
        gpu2 = _engine()
        try:
            assert gpu2.open(image) == 0
            assert gpu2.lookup_transfers(ids).tobytes() == orc.lookup_transfers(ids).tobytes()
            again = t[:8190].copy()  # all exist, now through the rebuilt hash index
            bts = np.array([ts + 8191], dtype=np.uint64)
            go, gr, _ = gpu2.create_transfers_batches(bts, np.array([8190], np.uint32), again)
            oo, orr, _ = orc.create_transfers_batches(bts, np.array([8190], np.uint32), again)
            assert np.array_equal(gr, orr) and int(gr[0]) == 8190
            assert go[:8190].tobytes() == oo[:8190].tobytes()
        finally:
            gpu2.close()
    finally:
        gpu.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sorted_run_random_call_mix(seed):
    """Random sequences of calls against the oracle, each call one of: fresh rising ids
    (the run grows), rising ids with failures (exists / invalid fields: hashed), a
    shuffled call (non-monotone: hashed), replays of earlier ids, posts and voids of
    earlier pendings (general path), linked pairs (fp_chains): the sorted run and the
    hash index together must answer every `exists`, every pending lookup and every
    lookup exactly as the oracle's single map does."""
    from tigerbeetle_amd.types import TRANSFER_DTYPE, TransferFlags
    rng = np.random.default_rng(100 + seed)
    acc_n = 300
    w = workload.config1(transfer_count=1, account_count=acc_n, seed=seed)
    ats, _ = w.timestamps()
    orc = oracle.Oracle(acc_n, 1 << 20)
    gpu = _engine()
    next_id = 1
    committed = []  # ids and flags of events sent so far
    try:
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        ts = int(ats[-1])
        for k in range(24):
            kind = rng.choice(["fresh", "fresh", "fail", "shuffle", "replay", "postvoid", "linked"])
            n = int(rng.integers(1, 3 * 8190))
            ev = np.zeros(n, dtype=TRANSFER_DTYPE)
            ev["id_lo"] = np.arange(next_id, next_id + n)
            next_id += n + int(rng.integers(0, 3))
            d = rng.integers(1, acc_n + 1, n)
            c = rng.integers(1, acc_n, n)
            c = np.where(c >= d, c + 1, c)
            ev["debit_account_id_lo"], ev["credit_account_id_lo"] = d, c
            ev["amount_lo"] = rng.integers(1, 1000, n)
            ev["ledger"], ev["code"] = 2, 1
            ev["flags"] = np.where(rng.random(n) < 0.2, int(TransferFlags.pending), 0)
            if kind == "fail":
                bad = rng.random(n) < 0.05
                ev["code"][bad] = 0
            elif kind == "shuffle":
                rng.shuffle(ev)
            elif kind == "replay" and committed:
                old = np.concatenate(committed)
                pick = old[rng.integers(0, len(old), min(n, 2000))]
                ev[:len(pick)] = pick
                ev["amount_lo"][:len(pick) // 2] += 1
            elif kind == "postvoid" and committed:
                old = np.concatenate(committed)
                pend = old[old["flags"] == int(TransferFlags.pending)]
                if len(pend):
                    m = min(n, len(pend))
                    sel = pend[rng.choice(len(pend), m, replace=False)]
                    ev = ev[:m]
                    ev["pending_id_lo"] = sel["id_lo"]
                    ev["debit_account_id_lo"] = 0
                    ev["credit_account_id_lo"] = 0
                    ev["amount_lo"] = 0
                    ev["ledger"], ev["code"] = 0, 0
                    ev["flags"] = np.where(rng.random(m) < 0.5, int(TransferFlags.post_pending_transfer),
                                           int(TransferFlags.void_pending_transfer))
            elif kind == "linked":
                ev["flags"][0:n - 1:2] |= int(TransferFlags.linked)
            counts = np.full(len(ev) // 8190, 8190, dtype=np.uint32)
            if len(ev) % 8190:
                counts = np.append(counts, len(ev) % 8190).astype(np.uint32)
            bts = ts + np.cumsum(counts.astype(np.uint64) + 1)
            ts = int(bts[-1])
            go, gr, _ = gpu.create_transfers_batches(bts, counts, ev)
            oo, orr, _ = orc.create_transfers_batches(bts, counts, ev)
            assert np.array_equal(gr, orr), (k, kind)
            assert_results_equal(per_batch_results(go, counts, gr), per_batch_results(oo, counts, orr), f"{k} {kind}")
            committed.append(ev.copy())
        assert_state_equal(gpu, orc)
        ids = np.concatenate(committed)["id_lo"][::11].tolist() + [0, next_id + 5]
        assert gpu.lookup_transfers(ids).tobytes() == orc.lookup_transfers(ids).tobytes()
    finally:
        gpu.close()


@pytest.mark.parametrize("n", [1, 2, 511, 513, 8190, 16383, 16384, 16385])
def test_small_call_tail_boundary(n):
    """Calls on both sides of FP_TAIL_MAX (16384 events, fast.h): at most that many run
    everything after fp_commit in one workgroup (fp_tail), more run the launch
    sequence.  Each size goes through the kinds fp_tail has phases for: all accepted
    with rising ids (the sorted run takes the rows), failures (fix ranks and replies),
    linked chains with a failing member (fp_chains), shuffled ids (dupcheck, hash
    index) and an id repeated within the call (the fallback to the general path)."""
    from tigerbeetle_amd.types import TRANSFER_DTYPE, TransferFlags
    rng = np.random.default_rng(n)
    acc_n = 200
    w = workload.config1(transfer_count=1, account_count=acc_n, seed=5)
    ats, _ = w.timestamps()
    orc = oracle.Oracle(acc_n, 1 << 20)
    gpu = _engine()
    next_id = 1
    try:
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        ts = int(ats[-1])
        for k, kind in enumerate(("fresh", "fail", "linked", "shuffle", "repeat", "fresh")):
            ev = np.zeros(n, dtype=TRANSFER_DTYPE)
            ev["id_lo"] = np.arange(next_id, next_id + n)
            next_id += n + 1
            d = rng.integers(1, acc_n + 1, n)
            c = rng.integers(1, acc_n, n)
            ev["debit_account_id_lo"], ev["credit_account_id_lo"] = d, np.where(c >= d, c + 1, c)
            ev["amount_lo"] = rng.integers(1, 1000, n)
            ev["ledger"], ev["code"] = 2, 1
            if kind in ("fail", "linked"):
                ev["code"][rng.random(n) < 0.03] = 0
            if kind == "linked":
                ev["flags"][0:n - 1:3] |= int(TransferFlags.linked)
                ev["flags"][1:n - 1:3] |= int(TransferFlags.linked)
            if kind == "shuffle":
                rng.shuffle(ev)
            if kind == "repeat" and n > 1:
                ev["id_lo"][-1] = ev["id_lo"][0]
            counts = np.full(n // 8190, 8190, dtype=np.uint32)
            if n % 8190:
                counts = np.append(counts, n % 8190).astype(np.uint32)
            bts = ts + np.cumsum(counts.astype(np.uint64) + 1)
            ts = int(bts[-1])
            go, gr, _ = gpu.create_transfers_batches(bts, counts, ev)
            oo, orr, _ = orc.create_transfers_batches(bts, counts, ev)
            assert np.array_equal(gr, orr), kind
            assert_results_equal(per_batch_results(go, counts, gr), per_batch_results(oo, counts, orr), f"{n} {kind}")
            if k < 4 and kind != "linked":
                assert gpu.stats().path == 1, kind  # the fast path stood (before any fallback)
        assert_state_equal(gpu, orc)
        assert gpu.commit_timestamp() == orc.commit_timestamp()
        ids = list(range(1, next_id, max(1, n // 50))) + [next_id + 3]
        assert gpu.lookup_transfers(ids).tobytes() == orc.lookup_transfers(ids).tobytes()
    finally:
        gpu.close()


def test_pinned_host_events_read_in_place():
    """Small one-chunk calls whose events sit in page-locked host memory (here a pinned
    torch buffer, at offsets inside it) are read by the kernels in place, without a
    copy (engine.hip transfers_batches, zero copy): same results and state as the
    oracle for accepted calls, calls with failures, chains, and a repeated id (the
    fallback redoes the call from a copy)."""
    import torch
    from tigerbeetle_amd.types import TRANSFER_DTYPE, TransferFlags
    rng = np.random.default_rng(77)
    acc_n = 150
    w = workload.config1(transfer_count=1, account_count=acc_n, seed=9)
    ats, _ = w.timestamps()
    orc = oracle.Oracle(acc_n, 1 << 20)
    gpu = _engine(pinned_input=True)  # the buffers below are page-locked (TBGPU_OPT_PINNED_INPUT)
    n = 8190
    kinds = ("fresh", "fail", "linked", "repeat", "fresh", "fresh")
    pinned = torch.empty((len(kinds) + 1) * n * 128, dtype=torch.uint8, pin_memory=True)
    view = pinned.numpy().view(TRANSFER_DTYPE)
    next_id = 1
    try:
        for be in (orc, gpu):
            be.create_accounts_batches(ats, w.account_counts, w.accounts)
        ts = int(ats[-1])
        for k, kind in enumerate(kinds):
            m = n - 7 * k  # ragged sizes at offsets inside the pinned buffer
            ev = view[k * n + 3:k * n + 3 + m]
            ev[:] = np.zeros(m, dtype=TRANSFER_DTYPE)
            ev["id_lo"] = np.arange(next_id, next_id + m)
            next_id += m
            d = rng.integers(1, acc_n + 1, m)
            c = rng.integers(1, acc_n, m)
            ev["debit_account_id_lo"], ev["credit_account_id_lo"] = d, np.where(c >= d, c + 1, c)
            ev["amount_lo"] = rng.integers(1, 1000, m)
            ev["ledger"], ev["code"] = 2, 1
            if kind in ("fail", "linked"):
                ev["code"][rng.random(m) < 0.02] = 0
            if kind == "linked":
                ev["flags"][0:m - 1:2] |= int(TransferFlags.linked)
            if kind == "repeat":
                ev["id_lo"][m // 2] = ev["id_lo"][1]
            ts += m + 1
            gr = gpu.create_transfers(ts, ev)
            orr = orc.create_transfers(ts, np.array(ev))
            assert gr.tobytes() == orr.tobytes(), (k, kind)
        assert_state_equal(gpu, orc)
        assert gpu.commit_timestamp() == orc.commit_timestamp()
        ids = list(range(1, next_id, 97)) + [next_id + 1]
        assert gpu.lookup_transfers(ids).tobytes() == orc.lookup_transfers(ids).tobytes()
    finally:
        gpu.close()


@pytest.mark.parametrize("order", ["shuffled_directory", "random_u128"])
def test_create_accounts_unordered_ids(order):
    """The clean call with ids that do not rise (the benchmark's --id-order=random /
    reversed, IdPermutation, src/testing/id.zig:28-48): ac_fast_dup claims every id in a
    call-local table.  Clean shuffled calls stay on the two-pass path; a repeat within
    the call (adjacent or far apart), an existing id and an invalid field each hand the
    call to the general path; every reply and row equals the oracle's, and the claim
    table is left clean for the calls after (and for create_transfers' own use of it)."""
    rng = np.random.default_rng(21)
    calls, used = [], 0

    def fresh(n):
        nonlocal used
        a = workload.make_accounts(np.arange(used + 1, used + 1 + n, dtype=np.uint64),
                                   ledger=rng.integers(1, 3, n).astype(np.uint32))
        used += n
        if order == "random_u128":
            a["id_lo"] = rng.integers(1, 1 << 63, n, dtype=np.uint64)
            a["id_hi"] = rng.integers(1, 1 << 63, n, dtype=np.uint64)
        else:
            a = a[rng.permutation(n)]
        return np.ascontiguousarray(a)

    calls.append(fresh(4000))                     # clean, unordered
    c = fresh(3000)
    c[2999] = c[17]                               # a repeat far apart
    calls.append(c)
    calls.append(fresh(2500))                     # clean again (the claims were cleared)
    c = fresh(1800)
    c[901] = c[900]                               # an adjacent repeat
    calls.append(c)
    c = fresh(1500)
    c[40] = calls[0][1234]                        # an existing id
    calls.append(c)
    c = fresh(1200)
    c[5]["ledger"] = 0                            # an invalid field
    calls.append(c)
    calls.append(fresh(8190))                     # a full clean batch
    orc, gpu = oracle.Oracle(40000, 30000), _engine(accounts_max=40000, transfers_max=30000)
    try:
        ts = 0
        for c in calls:
            ts += 1 + len(c)
            want = orc.create_accounts(ts, c)
            got = gpu.create_accounts(ts, c)
            assert got.tobytes() == want.tobytes(), (got[:5], want[:5])
        # transfers between the created accounts, after the account calls used the table
        accs = np.concatenate(calls)
        t = np.zeros(6000, dtype=workload.TRANSFER_DTYPE)
        t["id_lo"] = rng.permutation(6000).astype(np.uint64) + 1
        pick = rng.integers(0, len(accs), (6000, 2))
        t["debit_account_id_lo"], t["debit_account_id_hi"] = accs["id_lo"][pick[:, 0]], accs["id_hi"][pick[:, 0]]
        t["credit_account_id_lo"], t["credit_account_id_hi"] = accs["id_lo"][pick[:, 1]], accs["id_hi"][pick[:, 1]]
        t["ledger"] = accs["ledger"][pick[:, 0]]
        t["code"] = 1
        t["amount_lo"] = 3
        ts += 6001
        assert gpu.create_transfers(ts, t).tobytes() == orc.create_transfers(ts, t).tobytes()
        assert_state_equal(gpu, orc)
        q = [int(a["id_lo"]) | (int(a["id_hi"]) << 64) for a in accs[::61]]
        assert gpu.lookup_accounts(q).tobytes() == orc.lookup_accounts(q).tobytes()
    finally:
        gpu.close()


@pytest.mark.parametrize("dense", [True, False], ids=["directory", "hashed"])
def test_create_accounts_clean_and_dirty_calls(dense):
    """create_accounts' two-pass clean call (accounts.hip ac_fast_*: rising ids, every
    field valid, no chain, no existing id) and its hand-over to the general path: a
    call with one existing id, one invalid field or falling ids in the middle commits
    nothing through the clean pass (its optimistic rows lie past the committed ones)
    and answers exactly like the oracle; clean calls before and after stay exact."""
    rng = np.random.default_rng(11)
    hi = 0 if dense else 64  # ids 1..N sit in the direct-mapped directory; (64 << 64) | k are hashed
    calls = []
    nxt = 0

    def fresh(n):
        nonlocal nxt
        a = workload.make_accounts(np.arange(nxt + 1, nxt + 1 + n, dtype=np.uint64),
                                   ledger=rng.integers(1, 4, n).astype(np.uint32))
        a["id_hi"] = hi
        a["user_data_64"] = rng.integers(0, 1 << 40, n, dtype=np.uint64)
        nxt += n
        return a

    calls.append(fresh(3000))                     # clean
    c = fresh(2000)
    c[700] = calls[0][5]                          # an existing id in the middle
    calls.append(c)
    c = fresh(1500)
    c[20]["code"] = 0                             # an invalid field
    calls.append(c)
    c = fresh(1200)
    c[[100, 101]] = c[[101, 100]]                 # ids falling once (no repeat)
    calls.append(c)
    c = fresh(1000)
    c[999] = c[3]                                 # a repeat within the call
    calls.append(c)
    calls.append(fresh(2500))                     # clean again
    orc, gpu = oracle.Oracle(20000, 1024), _engine(accounts_max=20000)
    try:
        ts = 0
        for c in calls:
            ts += 1 + len(c)
            want = orc.create_accounts(ts, c)
            got = gpu.create_accounts(ts, c)
            assert got.tobytes() == want.tobytes(), (got[:5], want[:5])
        assert_state_equal(gpu, orc)
        ids = np.concatenate([c["id_lo"] for c in calls])
        q = [int(x) | (hi << 64) for x in ids[::97]]
        assert gpu.lookup_accounts(q).tobytes() == orc.lookup_accounts(q).tobytes()
    finally:
        gpu.close()
