"""Known-answer table harness.

Parses the golden tables (tests/golden/*.tbl) with the row grammar of the
reference's table parser (src/testing/table.zig:8-100: a leading letter is a
visual tag, ``-N`` on an unsigned column is ``maxInt - N``, ``_`` selects the
column default, a trailing ``//`` starts a comment) and replays them exactly as
the reference harness ``check()`` does (src/state_machine.zig:1867-2030):

* ``setup``  overwrites an account's four balances (:1892-1908);
* ``tick n`` adds n to prepare_timestamp (:1910-1913);
* ``commit op``: prepare_timestamp += 1, prepare() adds the event count,
  timestamp = prepare_timestamp, commit, then compare the sparse results
  (create_*) or the looked-up rows with timestamps zeroed (lookup_*) (:1973-2023).

``backend`` is anything with the engine/oracle method set (create_accounts,
create_transfers, lookup_accounts, lookup_transfers, set_balances).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from tigerbeetle_amd.types import (ACCOUNT_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE, CreateAccountResult,
                                   CreateTransferResult, account, transfer)

_MAX = {"u128": (1 << 128) - 1, "u64": (1 << 64) - 1, "u32": (1 << 32) - 1, "u16": (1 << 16) - 1,
        "u12": (1 << 12) - 1, "u10": (1 << 10) - 1, "u1": 1}
_NODEF = object()

# (name, type, default) — field order of TestCreateAccount (src/state_machine.zig:1777-1795)
ACCOUNT_COLUMNS = [
    ("id", "u128", _NODEF), ("debits_pending", "u128", 0), ("debits_posted", "u128", 0),
    ("credits_pending", "u128", 0), ("credits_posted", "u128", 0), ("user_data_128", "u128", 0),
    ("user_data_64", "u64", 0), ("user_data_32", "u32", 0), ("reserved", "u1", 0),
    ("ledger", "u32", _NODEF), ("code", "u16", _NODEF),
    ("flags_linked", ("LNK",), None), ("flags_dnec", ("D<C",), None), ("flags_cned", ("C<D",), None),
    ("flags_padding", "u12", 0), ("timestamp", "u64", 0), ("result", "enum_account", _NODEF),
]
# TestCreateTransfer (src/state_machine.zig:1822-1865)
TRANSFER_COLUMNS = [
    ("id", "u128", _NODEF), ("debit_account_id", "u128", _NODEF), ("credit_account_id", "u128", _NODEF),
    ("amount", "u128", 0), ("pending_id", "u128", 0), ("user_data_128", "u128", 0),
    ("user_data_64", "u64", 0), ("user_data_32", "u32", 0), ("timeout", "u32", 0),
    ("ledger", "u32", _NODEF), ("code", "u16", _NODEF),
    ("flags_linked", ("LNK",), None), ("flags_pending", ("PEN",), None), ("flags_post", ("POS",), None),
    ("flags_void", ("VOI",), None), ("flags_bdr", ("BDR",), None), ("flags_bcr", ("BCR",), None),
    ("flags_padding", "u10", 0), ("timestamp", "u64", 0), ("result", "enum_transfer", _NODEF),
]


def parse_int(tok: str, ty: str) -> int:
    off = 1 if tok[0].isalpha() else 0
    if tok[off] == "-":
        return _MAX[ty] - int(tok[off + 1:])
    return int(tok[off:])


class _Tokens:
    def __init__(self, toks):
        self.toks, self.i = toks, 0

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else None


def _parse_struct(cols, tk: _Tokens) -> dict:
    out = {}
    for name, ty, default in cols:
        if default is not _NODEF and tk.peek() == "_":
            tk.next()
            out[name] = default
            continue
        tok = tk.next()
        if isinstance(ty, tuple):
            assert tok in ty, (name, tok)
            out[name] = tok
        elif ty == "enum_account":
            out[name] = CreateAccountResult[tok]
        elif ty == "enum_transfer":
            out[name] = CreateTransferResult[tok]
        else:
            out[name] = parse_int(tok, ty)
    return out


@dataclass
class Action:
    kind: str
    data: dict = field(default_factory=dict)


def parse(text: str) -> list[Action]:
    actions = []
    for line in text.split("\n"):
        line = line.split("#")[0] if line.startswith("#") else line
        toks = line.split()
        if not toks:
            continue
        if "//" in toks:
            toks = toks[:toks.index("//")]
        tk = _Tokens(toks[1:])
        kind = toks[0]
        if kind == "setup":
            d = {k: parse_int(tk.next(), "u128") for k in ("account", "dp", "dpo", "cp", "cpo")}
        elif kind == "tick":
            d = {"ticks": parse_int(tk.next(), "u64")}
        elif kind == "commit":
            d = {"operation": tk.next()}
        elif kind == "account":
            d = _parse_struct(ACCOUNT_COLUMNS, tk)
        elif kind == "transfer":
            d = _parse_struct(TRANSFER_COLUMNS, tk)
        elif kind == "lookup_account":
            d = {"id": parse_int(tk.next(), "u128")}
            if tk.peek() == "_":
                tk.next()
                d["balance"] = None
            else:
                d["balance"] = tuple(parse_int(tk.next(), "u128") for _ in range(4))
        elif kind == "lookup_transfer":
            d = {"id": parse_int(tk.next(), "u128")}
            variant = tk.next()
            if variant == "exists":
                v = tk.next()
                d["exists"] = v in ("1", "true", "T")
                assert v in ("0", "1", "true", "false", "T", "F")
            else:
                assert variant == "amount"
                d["amount"] = parse_int(tk.next(), "u128")
        else:
            raise ValueError(f"unknown action {kind!r}")
        assert tk.peek() is None, f"trailing tokens in {line!r}"
        actions.append(Action(kind, d))
    return actions


def account_event(a: dict) -> np.ndarray:
    """TestCreateAccount.event (src/state_machine.zig:1797-1818)."""
    flags = ((a["flags_linked"] is not None) << 0 | (a["flags_dnec"] is not None) << 1
             | (a["flags_cned"] is not None) << 2 | (a["flags_padding"] << 4))
    return account(id=a["id"], debits_pending=a["debits_pending"], debits_posted=a["debits_posted"],
                   credits_pending=a["credits_pending"], credits_posted=a["credits_posted"],
                   user_data_128=a["user_data_128"], user_data_64=a["user_data_64"],
                   user_data_32=a["user_data_32"], reserved=a["reserved"], ledger=a["ledger"],
                   code=a["code"], flags=flags, timestamp=a["timestamp"])


def transfer_event(t: dict) -> np.ndarray:
    """TestCreateTransfer.event (src/state_machine.zig:1843-1865)."""
    flags = ((t["flags_linked"] is not None) << 0 | (t["flags_pending"] is not None) << 1
             | (t["flags_post"] is not None) << 2 | (t["flags_void"] is not None) << 3
             | (t["flags_bdr"] is not None) << 4 | (t["flags_bcr"] is not None) << 5
             | (t["flags_padding"] << 6))
    return transfer(id=t["id"], debit_account_id=t["debit_account_id"],
                    credit_account_id=t["credit_account_id"], amount=t["amount"],
                    pending_id=t["pending_id"], user_data_128=t["user_data_128"],
                    user_data_64=t["user_data_64"], user_data_32=t["user_data_32"], timeout=t["timeout"],
                    ledger=t["ledger"], code=t["code"], flags=flags, timestamp=t["timestamp"])


class CheckFailure(AssertionError):
    pass


def check(backend, text: str) -> int:
    """Replay one table against `backend`; returns the number of commits verified."""
    accounts: dict[int, np.ndarray] = {}
    transfers: dict[int, np.ndarray] = {}
    request: list = []
    reply: list = []
    operation = None
    prepare_timestamp = 0
    commits = 0
    for act in parse(text):
        d = act.data
        if act.kind == "setup":
            assert operation is None
            backend.set_balances(d["account"], d["dp"], d["dpo"], d["cp"], d["cpo"])
        elif act.kind == "tick":
            prepare_timestamp += d["ticks"]
        elif act.kind == "account":
            assert operation in (None, "create_accounts")
            operation = "create_accounts"
            ev = account_event(d)
            request.append(ev)
            if d["result"] == CreateAccountResult.ok:
                accounts[d["id"]] = ev
            else:
                reply.append((len(request) - 1, int(d["result"])))
        elif act.kind == "transfer":
            assert operation in (None, "create_transfers")
            operation = "create_transfers"
            ev = transfer_event(d)
            request.append(ev)
            if d["result"] == CreateTransferResult.ok:
                transfers[d["id"]] = ev
            else:
                reply.append((len(request) - 1, int(d["result"])))
        elif act.kind == "lookup_account":
            assert operation in (None, "lookup_accounts")
            operation = "lookup_accounts"
            request.append(d["id"])
            if d["balance"] is not None:
                a = accounts[d["id"]].copy()
                from tigerbeetle_amd.types import set_u128
                for f, v in zip(("debits_pending", "debits_posted", "credits_pending", "credits_posted"),
                                d["balance"]):
                    set_u128(a, f, v)
                reply.append(a)
        elif act.kind == "lookup_transfer":
            assert operation in (None, "lookup_transfers")
            operation = "lookup_transfers"
            request.append(d["id"])
            if "exists" in d:
                if d["exists"]:
                    reply.append(transfers[d["id"]].copy())
            else:
                from tigerbeetle_amd.types import set_u128
                t = transfers[d["id"]].copy()
                set_u128(t, "amount", d["amount"])
                reply.append(t)
        elif act.kind == "commit":
            op = d["operation"]
            assert operation in (None, op)
            prepare_timestamp += 1
            if op in ("create_accounts", "create_transfers"):
                prepare_timestamp += len(request)  # StateMachine.prepare (src/state_machine.zig:503-512)
            timestamp = prepare_timestamp
            if op == "create_accounts":
                evs = np.concatenate(request) if request else np.zeros(0, dtype=ACCOUNT_DTYPE)
                got = backend.create_accounts(timestamp, evs)
                want = np.array(reply, dtype=RESULT_DTYPE)
                _cmp_results(got, want, op)
            elif op == "create_transfers":
                evs = np.concatenate(request) if request else np.zeros(0, dtype=TRANSFER_DTYPE)
                got = backend.create_transfers(timestamp, evs)
                want = np.array(reply, dtype=RESULT_DTYPE)
                _cmp_results(got, want, op)
            elif op == "lookup_accounts":
                got = backend.lookup_accounts(request).copy()
                got["timestamp"] = 0
                want = np.concatenate(reply) if reply else np.zeros(0, dtype=ACCOUNT_DTYPE)
                if got.tobytes() != want.tobytes():
                    raise CheckFailure(f"lookup_accounts mismatch:\n got={got}\nwant={want}")
            elif op == "lookup_transfers":
                got = backend.lookup_transfers(request).copy()
                got["timestamp"] = 0
                want = np.concatenate(reply) if reply else np.zeros(0, dtype=TRANSFER_DTYPE)
                if got.tobytes() != want.tobytes():
                    raise CheckFailure(f"lookup_transfers mismatch:\n got={got}\nwant={want}")
            else:
                raise ValueError(op)
            commits += 1
            request, reply, operation = [], [], None
    assert operation is None and not request and not reply
    return commits


def _cmp_results(got, want, op):
    if got.tobytes() != want.tobytes():
        g = [(int(r["index"]), int(r["result"])) for r in got]
        w = [(int(r["index"]), int(r["result"])) for r in want]
        raise CheckFailure(f"{op} results mismatch:\n got={g}\nwant={w}")
