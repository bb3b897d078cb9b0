"""Sharded commit with the HIP engine as every rank's shard backend (2 ranks on one
GPU, gloo for the router's collectives): tbgpu_create_transfers_routed with chain
control and dry runs, and tbgpu_import_transfers, against the single CPU state
machine over the router's global order (tests/test_shard.py for the protocol)."""
import pytest

from tests.test_shard import _check


@pytest.mark.gpu
def test_gpu_sharded_flag_mix():
    stats = _check(("mix", 21, 2, 3, 2), 2, kind="gpu")
    assert stats["dry_rounds"] > 0


@pytest.mark.gpu
def test_gpu_sharded_config4():
    stats = _check(("c4", 5, 2, 2, 2), 2, kind="gpu")
    assert stats["dry_rounds"] > 0


@pytest.mark.gpu
def test_gpu_device_step_config4():
    """The device-resident routed step with the HIP engine behind every rank (the
    engine's tbgpu_create_transfers_routed_device, fast path with chain control
    and dry runs)."""
    stats = _check(("c4", 17, 2, 3, 2), 2, kind="gpu", device_step=True)
    assert stats["preruns"] > 0 and stats["dry_rounds"] == 0 and stats["splits"] == 0


@pytest.mark.gpu
def test_gpu_device_step_breaking_chains():
    """Cross-shard pairs that break: the one-dry-run settlement (static failures) and
    dry rounds (balance-limited accounts) with the HIP engine behind every rank."""
    stats = _check(("c4f", 19, 2, 3, 2), 2, kind="gpu", device_step=True)
    assert stats["preruns"] > 0 and stats["dry_rounds"] == 0
    stats = _check(("c4l", 23, 2, 3, 2), 2, kind="gpu", device_step=True)
    assert stats["dry_rounds"] > 0


@pytest.mark.gpu
def test_route_scatter_matches_torch_partition():
    """tbgpu_route_scatter (csrc/route.hip) against the router's torch partition:
    identical send buffers, side records and per-owner counts, with empty batches,
    chains (some spanning owners, some open at a batch end) and 1..256 owners."""
    import numpy as np
    import torch

    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.shard import partition_torch
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    rng = np.random.default_rng(3)
    counts = [8190, 17, 0, 1000, 1, 0, 8190, 333]
    n = sum(counts)
    t = np.zeros(n, dtype=TRANSFER_DTYPE)
    t["id_lo"] = np.arange(1, n + 1)
    t["ledger"] = rng.integers(0, 5000, n)
    t["flags"] = np.where(rng.random(n) < 0.3, 1, 0) | np.where(rng.random(n) < 0.1, 2, 0)
    dev = torch.device("cuda", 0)
    ev = torch.from_numpy(t.view(np.uint8).copy()).to(dev)
    bts = np.cumsum(np.array(counts, dtype=np.uint64) + 1) + 1000
    eng = Engine(device=0, accounts_max=16, transfers_max=16, events_per_call_max=1 << 12)
    try:
        for W in (1, 2, 3, 8, 256):
            e_t, s_t, c_t, b_t, p_t = partition_torch(torch, ev, counts, bts, 5, W, dev, detail=True)
            # the scatter on its own, and after tbgpu_route_prepare ranked the events
            for prepared in (False, True):
                if prepared:
                    eng.route_stats(ev, n, world=W)
                e_n = torch.empty((n, 128), dtype=torch.uint8, device=dev)
                s_n = torch.empty(n, dtype=torch.int64, device=dev)
                c_n, b_n, p_n = eng.route_scatter(W, counts, bts, 5, ev, e_n, s_n, detail=True)
                assert c_n.tolist() == c_t.cpu().tolist(), (W, prepared)
                assert b_n.tolist() == b_t.cpu().tolist(), (W, prepared)
                assert p_n.tolist() == p_t.cpu().tolist(), (W, prepared)
                assert torch.equal(e_n, e_t), (W, prepared)
                assert torch.equal(s_n, s_t), (W, prepared)
        # the owner side: timestamps from the records (global batches 5.. of this rank)
        e_t, s_t, _ = partition_torch(torch, ev, counts, bts, 5, 3, dev)
        tsb = torch.tensor([0] * 5 + [int(b) - c for b, c in zip(bts, counts)], dtype=torch.int64, device=dev)
        ts_n = torch.empty(n, dtype=torch.int64, device=dev)
        eng.route_unpack(s_t, tsb, ts_n)
        assert torch.equal(ts_n, tsb[s_t >> 32] + (s_t & 0x1FFF) + 1)
        with pytest.raises(ValueError):
            eng.route_unpack(s_t, tsb[:7], ts_n)  # a record of batch 12 > the table
    finally:
        eng.close()


@pytest.mark.gpu
def test_route_packed_wire_format_round_trip():
    """tbgpu_route_scatter_packed + tbgpu_route_unpack_packed (the all-to-all's wire
    format: the step's nonzero 4-byte words, then the record's low word) give back exactly the
    torch partition's rows, records and timestamps, for masks from the events' own
    nonzero words (tbgpu_route_stats) to all 32; a mask missing a nonzero word fails."""
    import numpy as np
    import torch

    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.shard import partition_torch
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    rng = np.random.default_rng(5)
    counts = [8190, 17, 0, 1000, 1, 0, 8190, 333, 4095]
    n = sum(counts)
    t = np.zeros(n, dtype=TRANSFER_DTYPE)
    t["id_lo"] = np.arange(1, n + 1)
    t["debit_account_id_lo"] = rng.integers(1, 1 << 40, n)
    t["credit_account_id_lo"] = rng.integers(1, 1 << 40, n)
    t["amount_lo"] = rng.integers(1, 1 << 20, n)
    t["user_data_64"] = rng.integers(0, 1 << 63, n)
    t["ledger"] = rng.integers(0, 5000, n)
    t["code"] = 1
    t["flags"] = np.where(rng.random(n) < 0.3, 1, 0) | np.where(rng.random(n) < 0.1, 2, 0)
    t["timeout"][::97] = 3  # a word that is nonzero in few events
    dev = torch.device("cuda", 0)
    ev = torch.from_numpy(t.view(np.uint8).copy()).to(dev)
    bts = np.cumsum(np.array(counts, dtype=np.uint64) + 1) + 1000
    tsb = torch.tensor([0] * 5 + [int(b) - c for b, c in zip(bts, counts)], dtype=torch.int64, device=dev)
    w32 = t.view(np.uint32).reshape(n, 32)
    want_mask = sum(1 << w for w in range(32) if w32[:, w].any())
    eng = Engine(device=0, accounts_max=16, transfers_max=16, events_per_call_max=1 << 12)
    try:
        *_, got_mask = eng.route_stats(ev, n, world=3, word_mask=True)
        assert got_mask == want_mask
        for W in (1, 3, 8):
            e_t, s_t, c_t, b_t, p_t = partition_torch(torch, ev, counts, bts, 5, W, dev, detail=True)
            # the whole send buffer as one owner's input: sub-batches owner-major, then by batch
            bcn = b_t.cpu().numpy()
            sub_c = [int(bcn[o, b]) for o in range(W) for b in range(len(counts)) if bcn[o, b]]
            sub_g = [5 + b for o in range(W) for b in range(len(counts)) if bcn[o, b]]
            sub_off = torch.tensor(np.concatenate([[0], np.cumsum(sub_c)]), dtype=torch.int32, device=dev)
            sub_gt = torch.tensor(sub_g, dtype=torch.int32, device=dev)
            for mask in (want_mask, want_mask | 0x80000001, 0xFFFFFFFF):
                k = bin(mask).count("1") + 1
                send = torch.empty((n, k), dtype=torch.int32, device=dev)
                c_n, b_n, p_n = eng.route_scatter_packed(W, counts, 5, ev, mask, send)
                assert c_n.tolist() == c_t.cpu().tolist() and b_n.tolist() == b_t.cpu().tolist()
                assert p_n.tolist() == p_t.cpu().tolist()
                e_n = torch.empty((n, 128), dtype=torch.uint8, device=dev)
                s_n = torch.empty(n, dtype=torch.int64, device=dev)
                ts_n = torch.empty(n, dtype=torch.int64, device=dev)
                eng.route_unpack_packed(send, mask, sub_off, sub_gt, tsb, e_n, s_n, ts_n)
                assert torch.equal(e_n, e_t), (W, mask)
                assert torch.equal(s_n, s_t), (W, mask)
                assert torch.equal(ts_n, tsb[s_t >> 32] + (s_t & 0x1FFF) + 1), (W, mask)
        with pytest.raises(ValueError):
            send = torch.empty((n, 32), dtype=torch.int32, device=dev)
            eng.route_scatter_packed(3, counts, 5, ev, want_mask & ~(1 << 27), send)  # drops the timeouts
    finally:
        eng.close()


@pytest.mark.gpu
def test_route_stats_matches_numpy():
    """tbgpu_route_stats (csrc/route.hip) against numpy over the same events."""
    import numpy as np
    import torch

    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    rng = np.random.default_rng(11)
    eng = Engine(device=0, accounts_max=16, transfers_max=16, events_per_call_max=1 << 12)
    try:
        for n, mono, pv, big in ((1, True, False, False), (1000, True, False, False), (77_777, True, False, True),
                                 (50_001, False, True, False), (8190 * 3, True, False, False)):
            t = np.zeros(n, dtype=TRANSFER_DTYPE)
            ids = np.sort(rng.choice(1 << 40, size=n, replace=False)).astype(np.uint64) + 1
            if not mono:
                ids[n // 2], ids[n // 2 + 1] = ids[n // 2 + 1], ids[n // 2]
            t["id_lo"] = ids
            t["amount_lo"] = rng.integers(0, 1 << 63, n, dtype=np.uint64) * 2
            if big:
                t["amount_hi"][n // 3] = 1
            if pv:
                t["flags"][n - 1] = 4
            ev = torch.from_numpy(t.view(np.uint8).copy()).to("cuda:0")
            want = sum(int(x) for x in t["amount_lo"]) + (sum(int(x) for x in t["amount_hi"]) << 64)
            for world in (0, 1, 5):  # tbgpu_route_stats, and tbgpu_route_prepare's fused pass
                mn, mx, mo, ids_ok, has_pv, has_big, asum = eng.route_stats(ev, n, world=world)
                assert (mn, mx) == (int(ids.min()), int(ids.max())), world
                assert mo == mono and ids_ok and has_pv == pv and has_big == big, world
                assert asum == want % (1 << 128), world
    finally:
        eng.close()


@pytest.mark.gpu
def test_route_directory_matches_the_host_form():
    """tbgpu_route_directory_owners + tbgpu_route_directory (csrc/directory.hip, the
    general step's directory on the device) against shard_vec's host form of the same
    rule (a stable sort by key): committed ids and pendings (owner = ledger % world),
    ids first seen in the step and their repeats, pendings created earlier in the step
    with each kind of route hint, unknown pendings, u128 keys."""
    import numpy as np
    import torch

    from tigerbeetle_amd import workload
    from tigerbeetle_amd.engine import Engine
    from tigerbeetle_amd.shard_vec import ANY, DUP, EXISTS, INF, NEW, PEND, PEND_HAZARD, PEND_NONE, PV
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    rng = np.random.default_rng(11)
    W = 3
    eng = Engine(device=0, accounts_max=64, transfers_max=4096, history_max=16, events_per_call_max=1 << 12)
    try:
        ids = np.arange(1, 61, dtype=np.uint64)
        eng.create_accounts(10, workload.make_accounts(ids, ledger=(ids - 1) // 10 + 1))
        k = 500
        t = np.zeros(k, dtype=TRANSFER_DTYPE)
        t["id_lo"] = np.arange(1000, 1000 + k)
        led = rng.integers(1, 7, k)
        t["debit_account_id_lo"] = (led - 1) * 10 + 1 + rng.integers(0, 5, k)
        t["credit_account_id_lo"] = (led - 1) * 10 + 6 + rng.integers(0, 5, k)
        t["amount_lo"] = 1
        t["ledger"] = led
        t["code"] = 1
        assert len(eng.create_transfers(1000, t)) == 0
        committed = {1000 + j: int(led[j]) % W for j in range(k)}
        # the step's records: ids (kind 0, unique positions) and pending ids (kind 1)
        n = 3000
        pool = np.concatenate([np.arange(1000, 1500), np.arange(5000, 5300), [2**64 + 7, 2**65 + 9]]).astype(object)
        key = [int(pool[j]) for j in rng.integers(0, len(pool), n)]
        kind = rng.integers(0, 2, n)
        pos = np.where(kind == 0, np.arange(n) * 2, rng.integers(0, 2 * n, n)).astype(np.int64)
        hint = rng.choice([ANY, PV, 0, 1, 2], n).astype(np.int64)
        R = np.zeros((n, 5), dtype=np.int64)
        R[:, 0], R[:, 1], R[:, 4] = pos, kind, hint
        R[:, 2] = np.array([x & (2**64 - 1) for x in key], dtype=np.uint64).view(np.int64)
        R[:, 3] = np.array([x >> 64 for x in key], dtype=np.uint64).view(np.int64)
        dev = torch.device("cuda", 0)
        A = torch.from_numpy(R).to(dev)
        owners = torch.empty(n, dtype=torch.int64, device=dev)
        eng.route_directory_owners(W, A, owners)
        out = torch.empty((n, 3), dtype=torch.int64, device=dev)
        eng.route_directory(A, owners, out)
        got = out.cpu().numpy()
        cown = np.array([committed.get(x, -1) for x in key], dtype=np.int64)
        assert np.array_equal(owners.cpu().numpy(), cown)
        # the host form (shard_vec._directory_host) on the same records
        k0 = kind == 0
        cand = k0 & (cown < 0)
        first_p, first_h = {}, {}
        for j in np.argsort(pos, kind="stable"):
            if cand[j] and key[j] not in first_p:
                first_p[key[j]], first_h[key[j]] = int(pos[j]), int(hint[j])
        fP = np.array([first_p.get(x, INF) for x in key], dtype=np.int64)
        fH = np.array([first_h.get(x, ANY) for x in key], dtype=np.int64)
        isfirst = cand & (pos == fP)
        typ = np.where(k0, np.where(cown >= 0, EXISTS, np.where(isfirst, NEW, DUP)),
                       np.where(cown >= 0, PEND, np.where(fP < pos, np.where((fH == ANY) | (fH == PV), PEND_HAZARD,
                                                                              PEND), PEND_NONE)))
        assert np.array_equal(got[:, 0], typ)
        assert np.array_equal(got[:, 1], np.where(cown >= 0, cown, fH))
        assert np.array_equal(got[:, 2], fP)
        assert {int(x) for x in typ} >= {NEW, DUP, EXISTS, PEND, PEND_NONE, PEND_HAZARD}
    finally:
        eng.close()
