"""ABI data types (numpy views of the 128-byte extern structs).

Layouts follow the reference exactly:
  Account   src/tigerbeetle.zig:7-40   Transfer  src/tigerbeetle.zig:80-105
  CreateAccountsResult / CreateTransfersResult  src/tigerbeetle.zig:247-265
  AccountHistoryGrooveValue  src/state_machine.zig:275-294
u128 fields are stored as two little-endian u64 words (``<name>_lo``, ``<name>_hi``).
"""
from __future__ import annotations

import enum

import numpy as np

U128_MAX = (1 << 128) - 1
U64_MAX = (1 << 64) - 1


def _u128(name):
    return [(name + "_lo", "<u8"), (name + "_hi", "<u8")]


ACCOUNT_DTYPE = np.dtype(
    _u128("id") + _u128("debits_pending") + _u128("debits_posted") + _u128("credits_pending")
    + _u128("credits_posted") + _u128("user_data_128")
    + [("user_data_64", "<u8"), ("user_data_32", "<u4"), ("reserved", "<u4"), ("ledger", "<u4"),
       ("code", "<u2"), ("flags", "<u2"), ("timestamp", "<u8")],
    align=False,
)
TRANSFER_DTYPE = np.dtype(
    _u128("id") + _u128("debit_account_id") + _u128("credit_account_id") + _u128("amount")
    + _u128("pending_id") + _u128("user_data_128")
    + [("user_data_64", "<u8"), ("user_data_32", "<u4"), ("timeout", "<u4"), ("ledger", "<u4"),
       ("code", "<u2"), ("flags", "<u2"), ("timestamp", "<u8")],
    align=False,
)
RESULT_DTYPE = np.dtype([("index", "<u4"), ("result", "<u4")])
HISTORY_DTYPE = np.dtype(
    _u128("dr_account_id") + _u128("dr_debits_pending") + _u128("dr_debits_posted")
    + _u128("dr_credits_pending") + _u128("dr_credits_posted") + _u128("cr_account_id")
    + _u128("cr_debits_pending") + _u128("cr_debits_posted") + _u128("cr_credits_pending")
    + _u128("cr_credits_posted") + [("timestamp", "<u8"), ("reserved", "u1", (88,))]
)
U128_DTYPE = np.dtype([("lo", "<u8"), ("hi", "<u8")])
# AccountFilter (src/tigerbeetle.zig:268-302) and AccountBalance (:65-78)
FILTER_DTYPE = np.dtype(_u128("account_id") + [("timestamp_min", "<u8"), ("timestamp_max", "<u8"),
                                               ("limit", "<u4"), ("flags", "<u4"), ("reserved", "u1", (24,))])
BALANCE_DTYPE = np.dtype(_u128("debits_pending") + _u128("debits_posted") + _u128("credits_pending")
                         + _u128("credits_posted") + [("timestamp", "<u8"), ("reserved", "u1", (56,))])
QUERY_MAX = 8190  # constants.batch_max.get_account_transfers / _history (src/state_machine.zig:53-76)
# tbgpu_index_filter_t (include/tbgpu.h): a scan of one groove index tree
INDEX_FILTER_DTYPE = np.dtype(_u128("value") + [("timestamp_min", "<u8"), ("timestamp_max", "<u8"),
                                               ("limit", "<u4"), ("field", "<u4"), ("flags", "<u4"),
                                               ("reserved", "<u4")])


class IndexField(enum.IntEnum):
    """tbgpu_index_field: the grooves' index trees (src/state_machine.zig:1575-1641)."""
    debit_account_id = 0
    credit_account_id = 1
    user_data_128 = 2
    user_data_64 = 3
    user_data_32 = 4
    pending_id = 5
    timeout = 6
    ledger = 7
    code = 8
    amount = 9


TRANSFER_INDEX_FIELDS = tuple(IndexField)
ACCOUNT_INDEX_FIELDS = (IndexField.user_data_128, IndexField.user_data_64, IndexField.user_data_32,
                        IndexField.ledger, IndexField.code)

assert ACCOUNT_DTYPE.itemsize == 128
assert TRANSFER_DTYPE.itemsize == 128
assert RESULT_DTYPE.itemsize == 8
assert HISTORY_DTYPE.itemsize == 256
assert FILTER_DTYPE.itemsize == 64
assert BALANCE_DTYPE.itemsize == 128
assert INDEX_FILTER_DTYPE.itemsize == 48

ACCOUNT_U128_FIELDS = ("id", "debits_pending", "debits_posted", "credits_pending", "credits_posted",
                       "user_data_128")
TRANSFER_U128_FIELDS = ("id", "debit_account_id", "credit_account_id", "amount", "pending_id",
                        "user_data_128")


class AccountFlags(enum.IntFlag):
    """src/tigerbeetle.zig:42-63"""
    linked = 1 << 0
    debits_must_not_exceed_credits = 1 << 1
    credits_must_not_exceed_debits = 1 << 2
    history = 1 << 3


class TransferFlags(enum.IntFlag):
    """src/tigerbeetle.zig:107-120"""
    linked = 1 << 0
    pending = 1 << 1
    post_pending_transfer = 1 << 2
    void_pending_transfer = 1 << 3
    balancing_debit = 1 << 4
    balancing_credit = 1 << 5


class AccountFilterFlags(enum.IntFlag):
    """src/tigerbeetle.zig:289-302"""
    debits = 1 << 0
    credits = 1 << 1
    reversed = 1 << 2


class CreateAccountResult(enum.IntEnum):
    """src/tigerbeetle.zig:125-160 (value == precedence index)."""
    ok = 0
    linked_event_failed = 1
    linked_event_chain_open = 2
    timestamp_must_be_zero = 3
    reserved_field = 4
    reserved_flag = 5
    id_must_not_be_zero = 6
    id_must_not_be_int_max = 7
    flags_are_mutually_exclusive = 8
    debits_pending_must_be_zero = 9
    debits_posted_must_be_zero = 10
    credits_pending_must_be_zero = 11
    credits_posted_must_be_zero = 12
    ledger_must_not_be_zero = 13
    code_must_not_be_zero = 14
    exists_with_different_flags = 15
    exists_with_different_user_data_128 = 16
    exists_with_different_user_data_64 = 17
    exists_with_different_user_data_32 = 18
    exists_with_different_ledger = 19
    exists_with_different_code = 20
    exists = 21


class CreateTransferResult(enum.IntEnum):
    """src/tigerbeetle.zig:165-245 (value == precedence index)."""
    ok = 0
    linked_event_failed = 1
    linked_event_chain_open = 2
    timestamp_must_be_zero = 3
    reserved_flag = 4
    id_must_not_be_zero = 5
    id_must_not_be_int_max = 6
    flags_are_mutually_exclusive = 7
    debit_account_id_must_not_be_zero = 8
    debit_account_id_must_not_be_int_max = 9
    credit_account_id_must_not_be_zero = 10
    credit_account_id_must_not_be_int_max = 11
    accounts_must_be_different = 12
    pending_id_must_be_zero = 13
    pending_id_must_not_be_zero = 14
    pending_id_must_not_be_int_max = 15
    pending_id_must_be_different = 16
    timeout_reserved_for_pending_transfer = 17
    amount_must_not_be_zero = 18
    ledger_must_not_be_zero = 19
    code_must_not_be_zero = 20
    debit_account_not_found = 21
    credit_account_not_found = 22
    accounts_must_have_the_same_ledger = 23
    transfer_must_have_the_same_ledger_as_accounts = 24
    pending_transfer_not_found = 25
    pending_transfer_not_pending = 26
    pending_transfer_has_different_debit_account_id = 27
    pending_transfer_has_different_credit_account_id = 28
    pending_transfer_has_different_ledger = 29
    pending_transfer_has_different_code = 30
    exceeds_pending_transfer_amount = 31
    pending_transfer_has_different_amount = 32
    pending_transfer_already_posted = 33
    pending_transfer_already_voided = 34
    pending_transfer_expired = 35
    exists_with_different_flags = 36
    exists_with_different_debit_account_id = 37
    exists_with_different_credit_account_id = 38
    exists_with_different_amount = 39
    exists_with_different_pending_id = 40
    exists_with_different_user_data_128 = 41
    exists_with_different_user_data_64 = 42
    exists_with_different_user_data_32 = 43
    exists_with_different_timeout = 44
    exists_with_different_code = 45
    exists = 46
    overflows_debits_pending = 47
    overflows_credits_pending = 48
    overflows_debits_posted = 49
    overflows_credits_posted = 50
    overflows_debits = 51
    overflows_credits = 52
    overflows_timeout = 53
    exceeds_credits = 54
    exceeds_debits = 55


class Operation(enum.IntEnum):
    """StateMachine.Operation (src/state_machine.zig:318-326), vsr_operations_reserved = 128."""
    create_accounts = 128
    create_transfers = 129
    lookup_accounts = 130
    lookup_transfers = 131
    get_account_transfers = 132
    get_account_history = 133


BATCH_MAX = 8190  # constants.batch_max.create_transfers (src/state_machine.zig:53-76)


def set_u128(arr, field, value):
    """Assign python int(s) to a u128 field of a structured array (or record)."""
    if isinstance(value, int):
        arr[field + "_lo"] = value & U64_MAX
        arr[field + "_hi"] = value >> 64
    else:
        v = [int(x) for x in value]
        arr[field + "_lo"] = np.array([x & U64_MAX for x in v], dtype=np.uint64)
        arr[field + "_hi"] = np.array([x >> 64 for x in v], dtype=np.uint64)


def get_u128(rec, field) -> int:
    return (int(rec[field + "_hi"]) << 64) | int(rec[field + "_lo"])


def u128_array(values) -> np.ndarray:
    out = np.zeros(len(values), dtype=U128_DTYPE)
    for i, v in enumerate(values):
        out[i]["lo"] = v & U64_MAX
        out[i]["hi"] = v >> 64
    return out


def account(**kw) -> np.ndarray:
    """One Account record from keyword fields (u128 fields given as python ints)."""
    a = np.zeros(1, dtype=ACCOUNT_DTYPE)
    for k, v in kw.items():
        if k in ACCOUNT_U128_FIELDS:
            set_u128(a, k, int(v))
        else:
            a[k] = v
    return a


def transfer(**kw) -> np.ndarray:
    t = np.zeros(1, dtype=TRANSFER_DTYPE)
    for k, v in kw.items():
        if k in TRANSFER_U128_FIELDS:
            set_u128(t, k, int(v))
        else:
            t[k] = v
    return t


def account_filter(account_id: int, timestamp_min: int = 0, timestamp_max: int = 0, limit: int = QUERY_MAX,
                   flags: int = 3) -> np.ndarray:
    """One AccountFilter record (flags: AccountFilterFlags bits; 3 = debits | credits)."""
    f = np.zeros(1, dtype=FILTER_DTYPE)
    set_u128(f, "account_id", int(account_id))
    f["timestamp_min"] = timestamp_min
    f["timestamp_max"] = timestamp_max
    f["limit"] = limit
    f["flags"] = flags
    return f
