import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
# a fatal engine error aborts the process before pytest shows the captured stderr:
# the engine also appends its message here (csrc/engine.hip tbgpu_fatal)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
os.environ.setdefault("TBGPU_FATAL_LOG", os.path.join(ROOT, "gpurun_out", "tbgpu_fatal.log"))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtbgpu.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running parity case")


GOLDEN_DIR = os.path.join(TESTS, "golden")


def golden_tables():
    return sorted(f for f in os.listdir(GOLDEN_DIR) if f.endswith(".tbl"))


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN_DIR
