"""The HIP engine against the reference's known-answer tables (through the C-ABI)."""
import os

import pytest

from conftest import GOLDEN_DIR, golden_tables
from table import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine_factory():
    from tigerbeetle_amd.engine import Engine

    def make():
        return Engine(accounts_max=1 << 10, transfers_max=1 << 12, history_max=1 << 10,
                      events_per_call_max=1 << 14)
    return make


@pytest.mark.parametrize("name", golden_tables())
def test_golden_table_gpu(name, engine_factory):
    eng = engine_factory()
    try:
        assert check(eng, open(os.path.join(GOLDEN_DIR, name)).read()) >= 1
    finally:
        eng.close()
