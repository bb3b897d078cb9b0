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
