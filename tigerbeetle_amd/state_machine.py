"""Host-side mirror of the reference ``StateMachine`` interface for the hot path.

The reference replica drives its state machine through ``prepare`` / ``prefetch`` /
``commit`` (src/state_machine.zig:503-928).  This class keeps those names, argument
meanings and reply format, and routes create_accounts / create_transfers and the two
lookups to the HIP engine (libtbgpu.so).  Inputs and outputs are raw message bodies
(``bytes`` of 128-byte events / 8-byte results), exactly like the reference.
"""
from __future__ import annotations

import hashlib

import numpy as np

from .engine import Engine
from .types import ACCOUNT_DTYPE, FILTER_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE, U128_DTYPE, Operation

MESSAGE_BODY_SIZE_MAX = (1 << 20) - 256  # constants.message_body_size_max (src/constants.zig:204)


class StateMachine:
    """``StateMachineType(Storage, config)`` for the operations this engine owns."""

    Operation = Operation

    def __init__(self, engine: Engine | None = None, **engine_options):
        self.engine = engine or Engine(**engine_options)
        self.prepare_timestamp = 0
        self.commit_timestamp = 0
        self._prefetched = None  # the create_transfers body prefetch staged (its array view)
        self._staged = {}        # content key -> the staged body's array (alive while its copy may run)

    @staticmethod
    def body_key(input: bytes) -> int:
        """The body's content key (the Zig shim passes the header's checksum_body; the
        mirror has no header, so a 128-bit hash of the same bytes)."""
        return int.from_bytes(hashlib.blake2b(input, digest_size=16).digest(), "little")

    # src/state_machine.zig:503-512; the primary calls it from primary_pipeline_prepare
    # (src/vsr/replica.zig:5159-5167), before the prepare is replicated: a create_transfers
    # body is staged in HBM then and its commit prepared (tbgpu_stage_transfers)
    def prepare(self, operation: Operation, input: bytes) -> None:
        if operation in (Operation.create_accounts, Operation.create_transfers):
            self.prepare_timestamp += len(input) // 128
        if operation == Operation.create_transfers and input:
            key = self.body_key(input)
            events = np.frombuffer(input, dtype=TRANSFER_DTYPE)
            self.engine.stage_transfers(key, events)
            self._staged[key] = events
            while len(self._staged) > 16:
                self._staged.pop(next(iter(self._staged)))

    # src/state_machine.zig:930-955: the LSM compaction beat; here the account-transfers
    # index folds in the rows committed since the previous beat.
    def compact(self, callback, op: int) -> None:
        self.engine.compact()
        callback(self)

    # src/state_machine.zig:514-655 — the tables are HBM-resident, so prefetch has only
    # the batch's host-to-device copy left to do, and none when prepare staged the body:
    # create_transfers finds it by its content key (tbgpu_prefetch_transfers_staged;
    # a backup, which never prepares, copies it now) and the commit of the same body
    # skips its copy.  The callback runs once the copy has landed (the reference delivers
    # it asynchronously via the grid's next tick).
    def prefetch(self, callback, op: int, operation: Operation, input: bytes) -> None:
        if operation == Operation.create_transfers and input:
            self._prefetched = np.frombuffer(input, dtype=TRANSFER_DTYPE)
            key = self.body_key(input)
            self.engine.prefetch_transfers_staged(key, self._prefetched)
            self.engine.prefetch_wait()
            self._staged.pop(key, None)
        callback(self)

    # src/state_machine.zig:894-928
    def commit(self, client: int, op: int, timestamp: int, operation: Operation, input: bytes) -> bytes:
        assert op != 0
        assert timestamp > self.commit_timestamp
        if operation == Operation.create_accounts:
            events = np.frombuffer(input, dtype=ACCOUNT_DTYPE)
            out = self.engine.create_accounts(timestamp, events)
        elif operation == Operation.create_transfers:
            pre = getattr(self, "_prefetched", None)
            # the prefetched view of this very body (same buffer): the staged copy is used
            events = pre if pre is not None and pre.base is not None and pre.base is input else \
                np.frombuffer(input, dtype=TRANSFER_DTYPE)
            self._prefetched = None
            out = self.engine.create_transfers(timestamp, events)
        elif operation == Operation.lookup_accounts:
            ids = np.frombuffer(input, dtype=U128_DTYPE)
            out = self.engine.lookup_accounts([(int(x["hi"]) << 64) | int(x["lo"]) for x in ids])
            out = out[:MESSAGE_BODY_SIZE_MAX // 128]
        elif operation == Operation.lookup_transfers:
            ids = np.frombuffer(input, dtype=U128_DTYPE)
            out = self.engine.lookup_transfers([(int(x["hi"]) << 64) | int(x["lo"]) for x in ids])
            out = out[:MESSAGE_BODY_SIZE_MAX // 128]
        elif operation in (Operation.get_account_transfers, Operation.get_account_history):
            # parse_filter_from_input (src/state_machine.zig:812-820): a body that is not
            # exactly one AccountFilter reads as the zeroed (invalid) filter
            f = np.frombuffer(input, dtype=FILTER_DTYPE) if len(input) == FILTER_DTYPE.itemsize \
                else np.zeros(1, dtype=FILTER_DTYPE)
            out = (self.engine.get_account_transfers(f) if operation == Operation.get_account_transfers
                   else self.engine.get_account_history(f))
        else:
            raise NotImplementedError(f"{operation.name} is not served by the GPU engine")
        self.commit_timestamp = max(self.commit_timestamp, self.engine.commit_timestamp())
        return out.tobytes()

    @staticmethod
    def results(reply: bytes) -> np.ndarray:
        return np.frombuffer(reply, dtype=RESULT_DTYPE)


class Demuxer:
    """DemuxerType (src/state_machine.zig:126-165): splits one create_* reply (sparse
    results of several client requests batched together) back into per-request
    replies, in place.  decode() ranges must be disjoint and increasing."""

    def __init__(self, reply: np.ndarray):
        self.results = reply.view(RESULT_DTYPE)

    def decode(self, event_offset: int, event_count: int) -> np.ndarray:
        n = 0
        for r in self.results:
            if r["index"] < event_offset or r["index"] >= event_offset + event_count:
                break
            r["index"] -= event_offset
            n += 1
        out, self.results = self.results[:n], self.results[n:]
        return out
