"""ctypes binding of libtbgpu.so — the C-ABI in include/tbgpu.h.

This is the product path: every call goes to the HIP engine on the GPU.  There
is no CPU fallback; loading fails loudly when the library is missing and
``Engine()`` fails loudly when no GPU is visible.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

from .types import (ACCOUNT_DTYPE, BALANCE_DTYPE, FILTER_DTYPE, HISTORY_DTYPE, INDEX_FILTER_DTYPE, QUERY_MAX,
                    RESULT_DTYPE, TRANSFER_DTYPE, U128_DTYPE, U64_MAX, u128_array)

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# TBGPU_LIB: a timing variant built by build.build_variant (experiments only)
LIB_PATH = os.environ.get("TBGPU_LIB") or os.path.join(PKG, "libtbgpu.so")
HEADER = os.path.join(ROOT, "include", "tbgpu.h")
_lib = None


class U128(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


def u128(v: int) -> U128:
    return U128(v & U64_MAX, v >> 64)


class Options(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("reserved0", ctypes.c_uint32), ("accounts_max", ctypes.c_uint64),
                ("transfers_max", ctypes.c_uint64), ("history_max", ctypes.c_uint64),
                ("events_per_call_max", ctypes.c_uint64), ("flags", ctypes.c_uint32),
                ("dense_block_span", ctypes.c_uint32), ("directory_max", ctypes.c_uint64),
                ("hashed_max", ctypes.c_uint64), ("shard_world", ctypes.c_uint32), ("shard_rank", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("events", ctypes.c_uint64), ("iterations", ctypes.c_uint32), ("path", ctypes.c_uint32),
                ("sorts", ctypes.c_uint64), ("device_ms", ctypes.c_double), ("phase_ms", ctypes.c_double * 8),
                ("walks", ctypes.c_uint64), ("index_rebuilds", ctypes.c_uint64),
                ("h64_redos", ctypes.c_uint64)]

PHASES = ("upload", "classify", "sort", "scan", "evaluate", "apply", "index", "prep")


OPT_FORCE_GENERAL = 1
OPT_WALK_EARLY = 2  # include/tbgpu.h TBGPU_OPT_WALK_EARLY (tests)
OPT_PINNED_INPUT = 4  # include/tbgpu.h TBGPU_OPT_PINNED_INPUT: host event buffers are page-locked
OPT_DENSE_INDEXES = 8  # include/tbgpu.h TBGPU_OPT_DENSE_INDEXES: hash indexes at load <= 1/2


def header_symbols() -> list[str]:
    """Every function the C-ABI header declares."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(tbgpu_[a-z0-9_]+)\s*\(", text)))


def lib():
    """Load libtbgpu.so (built in-tree by tigerbeetle_amd.build)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `python -m tigerbeetle_amd.build` (no CPU fallback)")
    try:
        # torch ships its own HIP runtime: load it first so that libtbgpu.so binds to
        # the same one (one runtime per process; torch cannot see the GPU if ours
        # initialised first).  torch is plumbing here: device buffers, streams, RCCL.
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    L.tbgpu_init.restype = ctypes.c_int
    L.tbgpu_init.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(Options)]
    L.tbgpu_deinit.argtypes = [vp]
    L.tbgpu_reset.argtypes = [vp]
    for name in ("tbgpu_create_accounts", "tbgpu_create_transfers"):
        getattr(L, name).restype = u32
        getattr(L, name).argtypes = [vp, u64, vp, u32, vp]
    for name in ("tbgpu_create_transfers_batches", "tbgpu_create_accounts_batches",
                 "tbgpu_create_transfers_batches_device", "tbgpu_create_accounts_batches_device"):
        getattr(L, name).restype = u64
        getattr(L, name).argtypes = [vp, u32, vp, vp, vp, vp, vp]
    for name in ("tbgpu_lookup_accounts", "tbgpu_lookup_transfers"):
        getattr(L, name).restype = u32
        getattr(L, name).argtypes = [vp, vp, u32, vp]
    L.tbgpu_copy_to_device.restype = ctypes.c_int
    L.tbgpu_copy_to_device.argtypes = [vp, vp, vp, u64]
    L.tbgpu_prefetch_transfers.restype = ctypes.c_int
    L.tbgpu_prefetch_transfers.argtypes = [vp, vp, u32]
    L.tbgpu_prefetch_wait.restype = ctypes.c_int
    L.tbgpu_prefetch_wait.argtypes = [vp]
    L.tbgpu_bench_host_calls.restype = ctypes.c_int
    L.tbgpu_bench_host_calls.argtypes = [vp, ctypes.c_int, u32, vp, vp, vp, vp, vp, vp]
    L.tbgpu_stage_transfers.restype = ctypes.c_int
    L.tbgpu_stage_transfers.argtypes = [vp, U128, vp, u32]
    L.tbgpu_prefetch_transfers_staged.restype = ctypes.c_int
    L.tbgpu_prefetch_transfers_staged.argtypes = [vp, U128, vp, u32]
    L.tbgpu_bench_host_staged.restype = ctypes.c_int
    L.tbgpu_bench_host_staged.argtypes = [vp, u32, vp, vp, vp, vp, ctypes.c_double, vp, vp, vp]
    L.tbgpu_test_set_balances.restype = ctypes.c_int
    L.tbgpu_test_set_balances.argtypes = [vp, U128, U128, U128, U128, U128]
    for name in ("tbgpu_account_count", "tbgpu_transfer_count", "tbgpu_history_count", "tbgpu_commit_timestamp"):
        getattr(L, name).restype = u64
        getattr(L, name).argtypes = [vp]
    L.tbgpu_export_transfers.restype = u64
    L.tbgpu_export_transfers.argtypes = [vp, u64, u64, vp]
    L.tbgpu_export_history.restype = u64
    L.tbgpu_export_history.argtypes = [vp, u64, u64, vp]
    L.tbgpu_export_accounts.restype = u64
    L.tbgpu_export_accounts.argtypes = [vp, vp, u64]
    L.tbgpu_get_posted.restype = ctypes.c_int
    L.tbgpu_get_posted.argtypes = [vp, U128]
    L.tbgpu_last_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    L.tbgpu_set_profiling.argtypes = [vp, ctypes.c_int]
    L.tbgpu_create_transfers_routed.restype = u64
    L.tbgpu_create_transfers_routed.argtypes = [vp, u32, vp, vp, vp, vp, ctypes.c_int, vp, vp,
                                                ctypes.POINTER(ctypes.c_uint64)]
    L.tbgpu_create_transfers_routed_device.restype = u64
    L.tbgpu_create_transfers_routed_device.argtypes = [vp, u32, vp, vp, vp, vp, ctypes.c_int, vp, vp,
                                                       ctypes.POINTER(ctypes.c_uint64)]
    L.tbgpu_route_scatter.restype = ctypes.c_int
    L.tbgpu_route_scatter.argtypes = [vp, u32, u32, vp, vp, u64, vp, vp, vp, vp, vp, vp]
    L.tbgpu_route_stats.restype = ctypes.c_int
    L.tbgpu_route_stats.argtypes = [vp, vp, u64, vp]
    L.tbgpu_route_prepare.restype = ctypes.c_int
    L.tbgpu_route_prepare.argtypes = [vp, u32, vp, u64, vp]
    L.tbgpu_route_scatter_packed.restype = ctypes.c_int
    L.tbgpu_route_scatter_packed.argtypes = [vp, u32, u32, vp, u64, vp, u32, vp, vp, vp, vp]
    L.tbgpu_route_unpack_packed.restype = ctypes.c_int
    L.tbgpu_route_unpack_packed.argtypes = [vp, vp, u64, u32, u32, vp, vp, vp, u64, vp, vp, vp]
    L.tbgpu_route_unpack.restype = ctypes.c_int
    L.tbgpu_route_unpack.argtypes = [vp, vp, u64, vp, u64, vp]
    L.tbgpu_route_directory_owners.restype = ctypes.c_int
    L.tbgpu_route_directory_owners.argtypes = [vp, u32, vp, u64, vp]
    L.tbgpu_route_directory.restype = ctypes.c_int
    L.tbgpu_route_directory.argtypes = [vp, vp, vp, u64, vp]
    L.tbgpu_import_transfers.restype = ctypes.c_int
    L.tbgpu_import_transfers.argtypes = [vp, vp, u32]
    L.tbgpu_advance_commit_timestamp.argtypes = [vp, u64]
    L.tbgpu_checkpoint_size.restype = u64
    L.tbgpu_checkpoint_size.argtypes = [vp]
    L.tbgpu_checkpoint.restype = u64
    L.tbgpu_checkpoint.argtypes = [vp, vp, u64]
    L.tbgpu_open.restype = ctypes.c_int
    L.tbgpu_open.argtypes = [vp, vp, u64]
    L.tbgpu_compact.restype = u64
    L.tbgpu_compact.argtypes = [vp]
    for name in ("tbgpu_get_account_transfers", "tbgpu_get_account_history"):
        getattr(L, name).restype = u32
        getattr(L, name).argtypes = [vp, vp, vp]
    for name in ("tbgpu_scan_transfers", "tbgpu_scan_accounts"):
        getattr(L, name).restype = u32
        getattr(L, name).argtypes = [vp, vp, vp]
    for name in ("tbgpu_get_account_transfers_device", "tbgpu_get_account_history_device"):
        getattr(L, name).restype = u64
        getattr(L, name).argtypes = [vp, u32, vp, u32, vp, vp]
    L.tbgpu_bench_generate_accounts.restype = ctypes.c_int
    L.tbgpu_bench_generate_accounts.argtypes = [ctypes.c_int, u64, u64, u32, vp]
    L.tbgpu_bench_generate_transfers.restype = ctypes.c_int
    L.tbgpu_bench_generate_transfers.argtypes = [ctypes.c_int, u64, u64, u64, u32, u32, u32, u32, vp]
    L.tbgpu_last_error.restype = ctypes.c_int
    L.tbgpu_last_error.argtypes = [vp, ctypes.c_char_p, u32]
    _lib = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Engine:
    """One commit-engine context on one GPU (a StateMachine's hot-path state)."""

    name = "gpu"

    def __init__(self, device: int = 0, accounts_max: int = 1 << 16, transfers_max: int = 1 << 20,
                 history_max: int = 1 << 16, events_per_call_max: int = 1 << 17, force_general: bool = False,
                 dense_block_span: int = 0, walk_early: bool = False, pinned_input: bool = False,
                 directory_max: int = 0, hashed_max: int = 0, shard_world: int = 0, shard_rank: int = 0,
                 dense_indexes: bool = False):
        """dense_block_span = S > 0: account ids of the form (b << 32) | k with 1 <= k <= S
        (e.g. ledger-major numbering) are looked up in the direct-mapped directory, one
        8-byte read; other ids use the hash index.  0: the directory covers ids
        1..directory_max (the reference benchmark's numbering).
        shard_world = N >= 2: a ledger shard (include/tbgpu.h): rows only for accounts of
        ledgers with ledger % N == shard_rank (accounts_max of them), a directory entry
        for each of the directory_max accounts."""
        self._L = lib()
        opt = Options(device=device, accounts_max=accounts_max, transfers_max=transfers_max,
                      history_max=history_max, events_per_call_max=events_per_call_max,
                      flags=(OPT_FORCE_GENERAL if force_general else 0) | (OPT_WALK_EARLY if walk_early else 0)
                      | (OPT_PINNED_INPUT if pinned_input else 0) | (OPT_DENSE_INDEXES if dense_indexes else 0),
                      dense_block_span=dense_block_span, directory_max=directory_max, hashed_max=hashed_max,
                      shard_world=shard_world, shard_rank=shard_rank)
        self.device = device
        self.shard_world, self.shard_rank = shard_world, shard_rank
        h = ctypes.c_void_p()
        rc = self._L.tbgpu_init(ctypes.byref(h), ctypes.byref(opt))
        if rc != 0:
            raise RuntimeError(f"tbgpu_init failed ({rc}): no usable GPU (the engine has no CPU fallback)")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.tbgpu_deinit(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        self._L.tbgpu_reset(self._h)

    # -- commit -------------------------------------------------------------
    def create_accounts(self, timestamp: int, events: np.ndarray) -> np.ndarray:
        events = np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE)
        out = np.zeros(max(len(events), 1), dtype=RESULT_DTYPE)
        n = self._L.tbgpu_create_accounts(self._h, timestamp, _ptr(events), len(events), _ptr(out))
        return out[:n].copy()

    def create_transfers(self, timestamp: int, events: np.ndarray) -> np.ndarray:
        events = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE)
        out = np.empty(max(len(events), 1), dtype=RESULT_DTYPE)  # (the first n are written)
        n = self._L.tbgpu_create_transfers(self._h, timestamp, _ptr(events), len(events), _ptr(out))
        return out[:n].copy()

    def to_device(self, host, torch_device=None):
        """A device copy (torch uint8 tensor) of a numpy array / bytes, written by the
        engine's copy kernel (tbgpu_copy_to_device) rather than a copy engine: the way
        to hand the *_device entry points their inputs."""
        import torch
        a = np.ascontiguousarray(np.frombuffer(host, dtype=np.uint8) if isinstance(host, (bytes, bytearray))
                                 else np.asarray(host)).view(np.uint8).reshape(-1)
        out = torch.empty(max(len(a), 1), dtype=torch.uint8, device=torch_device or f"cuda:{self.device}")
        torch.cuda.current_stream(out.device).synchronize()  # the allocation's previous users are done
        if len(a):
            self._L.tbgpu_copy_to_device(self._h, ctypes.c_void_p(out.data_ptr()), _ptr(a), len(a))
        return out[:len(a)]

    def prefetch_transfers(self, events: np.ndarray) -> None:
        """StateMachine.prefetch for create_transfers (tbgpu_prefetch_transfers): the
        batch's copy to HBM is enqueued; create_transfers on the same array commits from
        it.  `events` must be contiguous TRANSFER_DTYPE and unchanged until that commit."""
        if events.dtype != TRANSFER_DTYPE or not events.flags["C_CONTIGUOUS"]:
            raise ValueError("prefetch_transfers needs the contiguous event array create_transfers will get")
        if self._L.tbgpu_prefetch_transfers(self._h, _ptr(events), len(events)) != 0:
            raise ValueError("prefetch_transfers: more events than a batch")

    def stage_transfers(self, key: int, events: np.ndarray) -> None:
        """StateMachine.prepare for create_transfers (tbgpu_stage_transfers): the body's
        copy to HBM starts now, keyed by `key` (the shim's checksum_body); a later
        prefetch_transfers(events, key=key) finds it there.  `events` must stay unchanged
        until that prefetch."""
        if events.dtype != TRANSFER_DTYPE or not events.flags["C_CONTIGUOUS"]:
            raise ValueError("stage_transfers needs a contiguous TRANSFER_DTYPE array")
        if self._L.tbgpu_stage_transfers(self._h, u128(key), _ptr(events), len(events)) != 0:
            raise ValueError("stage_transfers: more events than a batch")

    def prefetch_transfers_staged(self, key: int, events: np.ndarray) -> None:
        """tbgpu_prefetch_transfers_staged: prefetch of a body that may have been staged
        under `key` (then nothing is copied); create_transfers on the same array commits it."""
        if events.dtype != TRANSFER_DTYPE or not events.flags["C_CONTIGUOUS"]:
            raise ValueError("prefetch_transfers_staged needs the contiguous event array create_transfers will get")
        if self._L.tbgpu_prefetch_transfers_staged(self._h, u128(key), _ptr(events), len(events)) != 0:
            raise ValueError("prefetch_transfers_staged: more events than a batch")

    def bench_host_staged(self, timestamps, counts, events, gap_us: float):
        """tbgpu_bench_host_staged: stage, a gap of gap_us, prefetch (staged) + wait,
        commit, per batch, timed from C.  Returns (stage, prefetch, commit) microseconds."""
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        if events.dtype != TRANSFER_DTYPE or not events.flags["C_CONTIGUOUS"]:
            raise ValueError("bench_host_staged needs contiguous TRANSFER_DTYPE events")
        out = np.zeros(max(int(cs.max()) if len(cs) else 1, 1), dtype=RESULT_DTYPE)
        st, pre, com = (np.zeros(len(cs), dtype=np.float64) for _ in range(3))
        rc = self._L.tbgpu_bench_host_staged(self._h, len(cs), _ptr(events), _ptr(cs), _ptr(ts), _ptr(out),
                                             float(gap_us), _ptr(st), _ptr(pre), _ptr(com))
        if rc != 0:
            raise ValueError(f"bench_host_staged: {rc}")
        return st, pre, com

    def bench_host_calls(self, mode: int, timestamps, counts, events):
        """tbgpu_bench_host_calls: the drop-in call timed from C (mode 0 one
        tbgpu_create_transfers per batch, 1 prefetch + wait + commit).  Returns the per-call
        commit and prefetch wall times in microseconds."""
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        if events.dtype != TRANSFER_DTYPE or not events.flags["C_CONTIGUOUS"]:
            raise ValueError("bench_host_calls needs contiguous TRANSFER_DTYPE events")
        out = np.zeros(max(int(cs.max()) if len(cs) else 1, 1), dtype=RESULT_DTYPE)
        com = np.zeros(len(cs), dtype=np.float64)
        pre = np.zeros(len(cs), dtype=np.float64)
        rc = self._L.tbgpu_bench_host_calls(self._h, int(mode), len(cs), _ptr(events), _ptr(cs), _ptr(ts), _ptr(out),
                                            _ptr(com), _ptr(pre))
        if rc != 0:
            raise ValueError(f"bench_host_calls: {rc}")
        return com, pre

    def prefetch_wait(self) -> None:
        """The prefetch's completion (the reference's prefetch callback point)."""
        self._L.tbgpu_prefetch_wait(self._h)

    def create_transfers_batches(self, timestamps, counts, events):
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        events = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE)
        out = np.zeros(max(len(events), 1), dtype=RESULT_DTYPE)
        rc = np.zeros(len(cs), dtype=np.uint32)
        self._L.tbgpu_create_transfers_batches(self._h, len(cs), _ptr(ts), _ptr(cs), _ptr(events), _ptr(out),
                                               _ptr(rc))
        return out, rc, self.stats().device_ms / 1e3

    def create_transfers_batches_device(self, timestamps, counts, events_ptr: int, results_ptr: int):
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        rc = np.zeros(len(cs), dtype=np.uint32)
        total = self._L.tbgpu_create_transfers_batches_device(self._h, len(cs), _ptr(ts), _ptr(cs),
                                                              ctypes.c_void_p(events_ptr),
                                                              ctypes.c_void_p(results_ptr), _ptr(rc))
        return total, rc

    def create_transfers_routed(self, counts, events, event_ts, ctl=None, dry_run=False):
        """Owner sub-batches of a routed step (tbgpu_create_transfers_routed): returns
        (results at each sub-batch's event offset, result_counts, commit_timestamp)."""
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        events = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE)
        ts = np.ascontiguousarray(event_ts, dtype=np.uint64)
        c = None if ctl is None else np.ascontiguousarray(ctl, dtype=np.uint8)
        out = np.zeros(max(len(events), 1), dtype=RESULT_DTYPE)
        rc = np.zeros(len(cs), dtype=np.uint32)
        cts = ctypes.c_uint64(0)
        self._L.tbgpu_create_transfers_routed(self._h, len(cs), _ptr(cs), _ptr(events), _ptr(ts),
                                              None if c is None else _ptr(c), int(bool(dry_run)), _ptr(out),
                                              _ptr(rc), ctypes.byref(cts))
        return out, rc, cts.value

    def create_transfers_routed_tensors(self, counts, events, event_ts, ctl, dry_run, results, sync_inputs=True):
        """Routed sub-batches with every array a device tensor (torch, on this engine's
        GPU): events uint8 [n*128], event_ts int64 [n], ctl uint8 [n] or None, results
        a uint8 tensor of >= 8*n bytes that receives the concatenated sparse replies.
        Returns (result_counts per sub-batch, commit_timestamp)."""
        host_results = None
        if events.is_cuda:
            # the tensors were produced on torch's current stream; the engine runs on
            # its own, so wait for them (the call itself returns after its stream drained);
            # a caller on another thread synchronizes before handing them over
            if sync_inputs:
                import torch
                torch.cuda.current_stream(events.device).synchronize()
        else:  # CPU tensors (the gloo-routed tests): stage them in HBM
            dev = f"cuda:{self.device}"
            events, event_ts = events.to(dev), event_ts.to(dev)
            ctl = None if ctl is None else ctl.to(dev)
            host_results, results = results, results.to(dev)
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        rc = np.zeros(len(cs), dtype=np.uint32)
        cts = ctypes.c_uint64(0)
        self._L.tbgpu_create_transfers_routed_device(
            self._h, len(cs), _ptr(cs), ctypes.c_void_p(events.data_ptr()), ctypes.c_void_p(event_ts.data_ptr()),
            None if ctl is None else ctypes.c_void_p(ctl.data_ptr()), int(bool(dry_run)),
            ctypes.c_void_p(results.data_ptr()), _ptr(rc), ctypes.byref(cts))
        if host_results is not None:
            host_results.copy_(results.cpu())
        return rc, cts.value

    def import_transfers(self, rows: np.ndarray) -> None:
        rows = np.ascontiguousarray(rows, dtype=TRANSFER_DTYPE)
        if len(rows):
            self._L.tbgpu_import_transfers(self._h, _ptr(rows), len(rows))

    def route_scatter(self, world: int, counts, batch_timestamps, first_global_batch: int, events, send_events,
                      send_records, detail: bool = False):
        """The send side of a routed step (tbgpu_route_scatter): `events` (uint8 device
        tensor, n*128 B) to owner-major `send_events` (n*128 B) with 8-byte records
        (TBGPU_ROUTE_REC_*, shard.py REC_*) in `send_records` (n int64).  Returns the
        events per owner; with `detail`, also the events per (owner, batch) and the
        spanning events per owner."""
        import torch
        torch.cuda.current_stream(events.device).synchronize()
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        ts = np.ascontiguousarray(batch_timestamps, dtype=np.uint64)
        out = np.zeros(world, dtype=np.uint64)
        bc = np.zeros((world, max(len(cs), 1)), dtype=np.uint32)
        sp = np.zeros(world, dtype=np.uint32)
        rc = self._L.tbgpu_route_scatter(self._h, world, len(cs), _ptr(cs), _ptr(ts), int(first_global_batch),
                                         ctypes.c_void_p(events.data_ptr()), ctypes.c_void_p(send_events.data_ptr()),
                                         ctypes.c_void_p(send_records.data_ptr()), _ptr(out), _ptr(bc), _ptr(sp))
        if rc != 0:
            raise ValueError(f"tbgpu_route_scatter failed ({rc})")
        return (out, bc[:, :len(cs)], sp) if detail else out

    def route_scatter_packed(self, world: int, counts, first_global_batch: int, events, word_mask: int, send):
        """tbgpu_route_scatter_packed: `events` (uint8 device tensor, n*128 B) to the
        owner-major packed rows of `send` (int32 device tensor [n, popcount(mask) + 1]:
        the event's 4-byte words of `word_mask`, then its record's low word).  Returns
        (events per owner, events per (owner, batch), spanning events per owner)."""
        import torch
        torch.cuda.current_stream(events.device).synchronize()
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        out = np.zeros(world, dtype=np.uint64)
        bc = np.zeros((world, max(len(cs), 1)), dtype=np.uint32)
        sp = np.zeros(world, dtype=np.uint32)
        rc = self._L.tbgpu_route_scatter_packed(self._h, world, len(cs), _ptr(cs), int(first_global_batch),
                                                ctypes.c_void_p(events.data_ptr()), int(word_mask),
                                                ctypes.c_void_p(send.data_ptr()), _ptr(out), _ptr(bc), _ptr(sp))
        if rc != 0:
            raise ValueError(f"tbgpu_route_scatter_packed failed ({rc}): an event word outside mask {word_mask:#x}?")
        return out, bc[:, :len(cs)], sp

    def route_unpack_packed(self, packed, word_mask: int, sub_offsets, sub_batches, ts_base, events, records,
                            timestamps) -> None:
        """tbgpu_route_unpack_packed: received packed rows (int32 device tensor [m, K]) of
        the sub-batches starting at rows `sub_offsets` (int32 device tensor, + the end)
        of global batches `sub_batches` back to events (uint8 [m*128]), records and
        timestamps (int64 [m])."""
        import torch
        torch.cuda.current_stream(packed.device).synchronize()
        rc = self._L.tbgpu_route_unpack_packed(self._h, ctypes.c_void_p(packed.data_ptr()), int(packed.shape[0]),
                                               int(word_mask), int(sub_batches.numel()),
                                               ctypes.c_void_p(sub_offsets.data_ptr()),
                                               ctypes.c_void_p(sub_batches.data_ptr()),
                                               ctypes.c_void_p(ts_base.data_ptr()),
                                               int(ts_base.numel()), ctypes.c_void_p(events.data_ptr()),
                                               ctypes.c_void_p(records.data_ptr()),
                                               ctypes.c_void_p(timestamps.data_ptr()))
        if rc != 0:
            raise ValueError("tbgpu_route_unpack_packed: bad mask, or a record names an unknown batch")

    def route_stats(self, events, n: int, world: int = 0, word_mask: bool = False):
        """tbgpu_route_stats over n events of a uint8 device tensor: (min id, max id,
        monotone, plain ids, any post/void, any amount >= 2^64, amount sum).  With
        `world`, tbgpu_route_prepare: the same figures from the pass that also ranks the
        events for a route_scatter of them to `world` owners (which then skips it).
        With `word_mask`, also the mask of the 4-byte words nonzero in some event."""
        import torch
        torch.cuda.current_stream(events.device).synchronize()
        out = np.zeros(5, dtype=np.uint64)
        if world:
            rc = self._L.tbgpu_route_prepare(self._h, int(world), ctypes.c_void_p(events.data_ptr()), int(n), _ptr(out))
            if rc != 0:
                raise ValueError(f"tbgpu_route_prepare failed ({rc})")
        else:
            self._L.tbgpu_route_stats(self._h, ctypes.c_void_p(events.data_ptr()), int(n), _ptr(out))
        fl = int(out[2])
        r = (int(out[0]), int(out[1]), not (fl & 1), not (fl & 2), bool(fl & 4), bool(fl & 8),
             int(out[3]) | (int(out[4]) << 64))
        return r + ((fl >> 16) & 0xFFFFFFFF,) if word_mask else r

    def route_unpack(self, records, ts_base, timestamps) -> None:
        """tbgpu_route_unpack: event timestamps (int64 device tensor) from received
        records and the per-global-batch T - n table `ts_base` (int64 device tensor)."""
        import torch
        torch.cuda.current_stream(records.device).synchronize()
        rc = self._L.tbgpu_route_unpack(self._h, ctypes.c_void_p(records.data_ptr()), int(records.numel()),
                                        ctypes.c_void_p(ts_base.data_ptr()), int(ts_base.numel()),
                                        ctypes.c_void_p(timestamps.data_ptr()))
        if rc != 0:
            raise ValueError("tbgpu_route_unpack: a record names an unknown batch")

    def route_directory_owners(self, world: int, records, owners) -> None:
        """tbgpu_route_directory_owners: per record (int64 device tensor [k, 5]: position,
        kind, key lo, key hi, hint) the owner of this shard's committed transfer with that
        key, or -1, into `owners` (int64 device tensor [k])."""
        import torch
        torch.cuda.current_stream(records.device).synchronize()
        rc = self._L.tbgpu_route_directory_owners(self._h, int(world), ctypes.c_void_p(records.data_ptr()),
                                                  int(records.shape[0]), ctypes.c_void_p(owners.data_ptr()))
        if rc != 0:
            raise ValueError("tbgpu_route_directory_owners: bad arguments")

    def route_directory(self, records, owners, out) -> None:
        """tbgpu_route_directory: each record's (type, hint, first position) into `out`
        (int64 device tensor [k, 3]), from the records and their all-reduced owners."""
        import torch
        torch.cuda.current_stream(records.device).synchronize()
        rc = self._L.tbgpu_route_directory(self._h, ctypes.c_void_p(records.data_ptr()),
                                           ctypes.c_void_p(owners.data_ptr()), int(records.shape[0]),
                                           ctypes.c_void_p(out.data_ptr()))
        if rc != 0:
            raise ValueError("tbgpu_route_directory: bad arguments")

    def advance_commit_timestamp(self, ts: int) -> None:
        self._L.tbgpu_advance_commit_timestamp(self._h, int(ts))

    def create_accounts_batches_device(self, timestamps, counts, events_ptr: int, results_ptr: int):
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        rc = np.zeros(len(cs), dtype=np.uint32)
        total = self._L.tbgpu_create_accounts_batches_device(self._h, len(cs), _ptr(ts), _ptr(cs),
                                                             ctypes.c_void_p(events_ptr),
                                                             ctypes.c_void_p(results_ptr), _ptr(rc))
        return total, rc

    def create_accounts_batches(self, timestamps, counts, events):
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        cs = np.ascontiguousarray(counts, dtype=np.uint32)
        events = np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE)
        out = np.zeros(max(len(events), 1), dtype=RESULT_DTYPE)
        rc = np.zeros(len(cs), dtype=np.uint32)
        self._L.tbgpu_create_accounts_batches(self._h, len(cs), _ptr(ts), _ptr(cs), _ptr(events), _ptr(out),
                                              _ptr(rc))
        return out, rc

    # -- queries --------------------------------------------------------------
    def lookup_accounts(self, ids) -> np.ndarray:
        q = u128_array(list(ids))
        out = np.zeros(max(len(q), 1), dtype=ACCOUNT_DTYPE)
        n = self._L.tbgpu_lookup_accounts(self._h, _ptr(q), len(q), _ptr(out))
        return out[:n].copy()

    def lookup_transfers(self, ids) -> np.ndarray:
        q = ids if isinstance(ids, np.ndarray) and ids.dtype == U128_DTYPE else u128_array(list(ids))
        out = np.zeros(max(len(q), 1), dtype=TRANSFER_DTYPE)
        n = self._L.tbgpu_lookup_transfers(self._h, _ptr(q), len(q), _ptr(out))
        return out[:n].copy()

    def checkpoint(self) -> np.ndarray:
        """tbgpu_checkpoint: the durable image of the ctx's state (uint8 array)."""
        out = np.zeros(self._L.tbgpu_checkpoint_size(self._h), dtype=np.uint8)
        n = self._L.tbgpu_checkpoint(self._h, _ptr(out), len(out))
        assert n == len(out)
        return out

    def open(self, image: np.ndarray) -> int:
        """tbgpu_open: replace the state by a checkpoint image; 0 or a negative errno."""
        image = np.ascontiguousarray(image, dtype=np.uint8)
        return self._L.tbgpu_open(self._h, _ptr(image), len(image))

    def compact(self) -> int:
        """tbgpu_compact: index the rows stored since the last compaction."""
        return self._L.tbgpu_compact(self._h)

    def get_account_transfers(self, filt: np.ndarray) -> np.ndarray:
        f = np.ascontiguousarray(filt, dtype=FILTER_DTYPE).reshape(1)
        out = np.zeros(QUERY_MAX, dtype=TRANSFER_DTYPE)
        n = self._L.tbgpu_get_account_transfers(self._h, _ptr(f), _ptr(out))
        return out[:n].copy()

    def get_account_history(self, filt: np.ndarray) -> np.ndarray:
        f = np.ascontiguousarray(filt, dtype=FILTER_DTYPE).reshape(1)
        out = np.zeros(QUERY_MAX, dtype=BALANCE_DTYPE)
        n = self._L.tbgpu_get_account_history(self._h, _ptr(f), _ptr(out))
        return out[:n].copy()

    def scan_transfers(self, filt: np.ndarray) -> np.ndarray:
        """tbgpu_scan_transfers: one scan of a transfers index tree (INDEX_FILTER_DTYPE)."""
        f = np.ascontiguousarray(filt, dtype=INDEX_FILTER_DTYPE).reshape(1)
        out = np.zeros(QUERY_MAX, dtype=TRANSFER_DTYPE)
        n = self._L.tbgpu_scan_transfers(self._h, _ptr(f), _ptr(out))
        return out[:n].copy()

    def scan_accounts(self, filt: np.ndarray) -> np.ndarray:
        """tbgpu_scan_accounts: one scan of an accounts index tree (INDEX_FILTER_DTYPE)."""
        f = np.ascontiguousarray(filt, dtype=INDEX_FILTER_DTYPE).reshape(1)
        out = np.zeros(QUERY_MAX, dtype=ACCOUNT_DTYPE)
        n = self._L.tbgpu_scan_accounts(self._h, _ptr(f), _ptr(out))
        return out[:n].copy()

    def query_device(self, filters_ptr: int, count: int, stride: int, out_ptr: int, history: bool = False):
        """Batched queries with filters and results in device memory; returns (total, counts)."""
        rc = np.zeros(max(count, 1), dtype=np.uint32)
        fn = self._L.tbgpu_get_account_history_device if history else self._L.tbgpu_get_account_transfers_device
        total = fn(self._h, count, ctypes.c_void_p(filters_ptr), stride, ctypes.c_void_p(out_ptr), _ptr(rc))
        return total, rc[:count]

    def set_balances(self, id_, dp, dpo, cp, cpo) -> None:
        rc = self._L.tbgpu_test_set_balances(self._h, u128(id_), u128(dp), u128(dpo), u128(cp), u128(cpo))
        assert rc == 0, "setup: account not found"

    def account_count(self) -> int:
        return self._L.tbgpu_account_count(self._h)

    def transfer_count(self) -> int:
        return self._L.tbgpu_transfer_count(self._h)

    def history_count(self) -> int:
        return self._L.tbgpu_history_count(self._h)

    def commit_timestamp(self) -> int:
        return self._L.tbgpu_commit_timestamp(self._h)

    def export_accounts(self) -> np.ndarray:
        n = self.account_count()
        out = np.zeros(max(n, 1), dtype=ACCOUNT_DTYPE)
        k = self._L.tbgpu_export_accounts(self._h, _ptr(out), n)
        return out[:k]

    def export_transfers(self, first: int = 0, count: int | None = None) -> np.ndarray:
        total = self.transfer_count()
        count = total - first if count is None else count
        out = np.zeros(max(count, 1), dtype=TRANSFER_DTYPE)
        n = self._L.tbgpu_export_transfers(self._h, first, count, _ptr(out))
        return out[:n]

    def export_history(self) -> np.ndarray:
        n = self.history_count()
        out = np.zeros(max(n, 1), dtype=HISTORY_DTYPE)
        self._L.tbgpu_export_history(self._h, 0, n, _ptr(out))
        return out[:n]

    def get_posted(self, pending_id: int) -> int:
        return self._L.tbgpu_get_posted(self._h, u128(pending_id))

    def set_profiling(self, enable: bool) -> None:
        self._L.tbgpu_set_profiling(self._h, 1 if enable else 0)

    def stats(self) -> Stats:
        s = Stats()
        self._L.tbgpu_last_stats(self._h, ctypes.byref(s))
        return s


def generate_accounts(device: int, first_id: int, count: int, accounts_per_ledger: int, out_ptr: int) -> None:
    """The benchmark's accounts in device memory (tbgpu_bench_generate_accounts)."""
    rc = lib().tbgpu_bench_generate_accounts(device, first_id, count, accounts_per_ledger, ctypes.c_void_p(out_ptr))
    if rc != 0:
        raise RuntimeError(f"tbgpu_bench_generate_accounts failed ({rc})")


def generate_transfers(device: int, first_id: int, count: int, seed: int, ledger0: int, ledgers: int,
                       accounts_per_ledger: int, out_ptr: int, ledger_stride: int = 1) -> None:
    """The benchmark's transfers in device memory (tbgpu_bench_generate_transfers): ledgers
    ledger0 + ledger_stride * [0, ledgers)."""
    rc = lib().tbgpu_bench_generate_transfers(device, first_id, count, seed, ledger0, ledgers, ledger_stride,
                                              accounts_per_ledger, ctypes.c_void_p(out_ptr))
    if rc != 0:
        raise RuntimeError(f"tbgpu_bench_generate_transfers failed ({rc})")
