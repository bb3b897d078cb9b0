"""The drop-in boundary: libtbgpu.so loads and exports the whole C-ABI (no GPU needed)."""
import ctypes
import re

import pytest

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
    size = {"tbgpu_uint128_t": 16, "uint64_t": 8, "uint32_t": 4, "uint16_t": 2}
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
    for struct, dt in (("tbgpu_account_t", ACCOUNT_DTYPE), ("tbgpu_transfer_t", TRANSFER_DTYPE)):
        offs, size = _offsets_from_header(struct)
        assert size == dt.itemsize == 128
        for name, off in offs.items():
            key = name + "_lo" if name + "_lo" in dt.fields else name
            assert dt.fields[key][1] == off, (struct, name)
    assert HISTORY_DTYPE.itemsize == 256


REF_CLIENT_HEADER = "/root/reference/src/clients/c/tb_client.h"


def test_header_coexists_with_reference_client_header(tmp_path):
    """include/tbgpu.h and the reference's tb_client.h compile in one C translation unit
    (distinct type and enumerator names), with identical struct sizes and every result
    code and flag of tbgpu.h equal to its tb_client.h counterpart.  Runs only where the
    reference checkout is present (this container); nothing of it is copied."""
    import os
    import shutil
    import subprocess

    import pytest
    if not os.path.exists(REF_CLIENT_HEADER) or not shutil.which("gcc"):
        pytest.skip("reference client header or gcc not available")
    ours = open(engine.HEADER).read()
    names = sorted(set(re.findall(r"\bTBGPU_((?:CREATE_ACCOUNT|CREATE_TRANSFER|ACCOUNT|TRANSFER)_[A-Z0-9_]+)\s*=",
                                  ours)))
    assert len(names) > 90
    src = [f'#include "{REF_CLIENT_HEADER}"', f'#include "{engine.HEADER}"']
    for a, b in (("tb_account_t", "tbgpu_account_t"), ("tb_transfer_t", "tbgpu_transfer_t"),
                 ("tb_create_transfers_result_t", "tbgpu_create_transfers_result_t"),
                 ("tb_create_accounts_result_t", "tbgpu_create_accounts_result_t"),
                 ("tb_account_filter_t", "tbgpu_account_filter_t"),
                 ("tb_account_balance_t", "tbgpu_account_balance_t")):
        src.append(f'_Static_assert(sizeof({a}) == sizeof({b}), "{a}");')
    for n in names:
        src.append(f'_Static_assert((int)TB_{n} == (int)TBGPU_{n}, "{n}");')
    src.append("int main(void) { return 0; }")
    c = tmp_path / "both.c"
    c.write_text("\n".join(src) + "\n")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-c", str(c), "-o", str(tmp_path / "both.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


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


@pytest.mark.parametrize("ctype,mirror", [("tbgpu_stats", "Stats"), ("tbgpu_options", "Options")])
def test_structs_match_the_python_mirrors(tmp_path, ctype, mirror):
    """tbgpu_stats / tbgpu_options as the C compiler lays them out (include/tbgpu.h)
    against the ctypes mirrors the Python host passes and reads: size and every field's
    offset."""
    import os
    import subprocess
    M = getattr(engine, mirror)
    fields = [name for name, _ in M._fields_]
    src = tmp_path / "stats.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "tbgpu.h"\nint main(void) {\n'
                   f'    printf("size %zu\\n", sizeof({ctype}));\n'
                   + "".join(f'    printf("{f} %zu\\n", offsetof({ctype}, {f}));\n' for f in fields)
                   + "    return 0;\n}\n")
    exe = tmp_path / "stats"
    inc = os.path.join(os.path.dirname(engine.HEADER))
    subprocess.run(["gcc", "-std=c11", "-I", inc, str(src), "-o", str(exe)], check=True)
    out = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                       text=True).stdout.splitlines())
    assert int(out["size"]) == ctypes.sizeof(M)
    for f in fields:
        assert int(out[f]) == getattr(M, f).offset, f
