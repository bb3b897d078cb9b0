"""The drop-in boundary: libtbgpu.so loads and exports the whole C-ABI (no GPU needed)."""
import ctypes
import re

from tigerbeetle_amd import engine
from tigerbeetle_amd.types import ACCOUNT_DTYPE, HISTORY_DTYPE, TRANSFER_DTYPE


def test_library_exports_every_header_symbol():
    L = engine.lib()
    syms = engine.header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"libtbgpu.so does not export {s}"


def test_header_declares_the_reference_entry_points():
    syms = set(engine.header_symbols())
    for s in ("tbgpu_init", "tbgpu_deinit", "tbgpu_create_accounts", "tbgpu_create_transfers",
              "tbgpu_lookup_accounts", "tbgpu_lookup_transfers", "tbgpu_test_set_balances",
              "tbgpu_last_error"):
        assert s in syms


def _offsets_from_header(struct):
    text = open(engine.HEADER).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (struct, struct), text, re.S).group(1)
    size = {"tb_uint128_t": 16, "uint64_t": 8, "uint32_t": 4, "uint16_t": 2}
    off, out = 0, {}
    for line in body.split(";"):
        m = re.match(r"\s*(\w+)\s+(\w+)", line)
        if not m:
            continue
        ty, name = m.groups()
        if ty not in size:
            continue
        out[name] = off
        off += size[ty]
    return out, off


def test_struct_layouts_match_numpy_views():
    for struct, dt in (("tb_account_t", ACCOUNT_DTYPE), ("tb_transfer_t", TRANSFER_DTYPE)):
        offs, size = _offsets_from_header(struct)
        assert size == dt.itemsize == 128
        for name, off in offs.items():
            key = name + "_lo" if name + "_lo" in dt.fields else name
            assert dt.fields[key][1] == off, (struct, name)
    assert HISTORY_DTYPE.itemsize == 256


def test_init_without_gpu_fails_loudly():
    """No GPU here: tbgpu_init must refuse rather than fall back to the CPU."""
    import pytest
    try:
        import torch  # noqa: F401
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        engine.Engine()
