"""tigerbeetle_amd — MI355X-native commit engine for TigerBeetle's create_accounts /
create_transfers hot path (reference: src/state_machine.zig:894-1573).

The product is ``libtbgpu.so`` (HIP kernels for gfx950 + a C-ABI, include/tbgpu.h).
This package holds its sources (``csrc/``), the ctypes binding (``engine``), the
host-side mirror of the reference ``StateMachine`` interface (``state_machine``) and
the synthetic workload generators used by the tests and bench (``workload``).
"""
from . import types  # noqa: F401

__all__ = ["types"]
