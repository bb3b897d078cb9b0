"""Multi-ledger flag-heavy workload for the sharded-commit tests.

Everything that couples shards appears: linked chains whose members sit on
different ledgers (the currency-exchange pattern, docs/reference/transfers.md:282),
post/void of pendings created in earlier batches of any rank (including the same
step), transfer ids reused across ledgers (committed and within a step), pending
ids that name a post/void, limit accounts, balancing, invalid fields and chains
left open at a batch end.  Batches are laid out per step and rank: step s, rank r
gets batches [s*W*B + r*B, s*W*B + (r+1)*B) of the global sequence, which is the
router's global order.
"""
from __future__ import annotations

import numpy as np

from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, AccountFlags, TransferFlags
from tigerbeetle_amd.workload import make_accounts


class ShardWorkload:
    def __init__(self, seed: int, world: int, steps: int, batches_per_rank: int, batch: int = 64,
                 ledgers: int = 5, accounts_per_ledger: int = 24):
        rng = np.random.default_rng(seed)
        self.world, self.steps, self.B = world, steps, batches_per_rank
        L, A = ledgers, accounts_per_ledger
        led = np.repeat(np.arange(1, L + 1, dtype=np.uint64), A)
        k = np.tile(np.arange(1, A + 1, dtype=np.uint64), L)
        roll = rng.random(L * A)
        aflags = np.where(roll < 0.2, int(AccountFlags.debits_must_not_exceed_credits),
                          np.where(roll < 0.3, int(AccountFlags.credits_must_not_exceed_debits), 0))
        aflags = (aflags | np.where(rng.random(L * A) < 0.05, int(AccountFlags.history), 0)).astype(np.uint16)
        ids = (led << np.uint64(32)) | k
        self.accounts = make_accounts(ids, ledger=led.astype(np.uint32), flags=aflags)
        self.account_batches = [self.accounts[i:i + 50] for i in range(0, len(self.accounts), 50)]

        def acct(l, j):
            return (int(l) << 32) | (int(j) + 1)

        next_id = [1]
        pendings: list[tuple[int, int, int]] = []  # (id, amount, ledger)
        recent: list[int] = []
        postvoids: list[int] = []
        total = steps * world * batches_per_rank
        self.batches = []
        for b in range(total):
            t = np.zeros(batch, dtype=TRANSFER_DTYPE)
            new_p = []
            for j in range(batch):
                r = t[j]
                tid = next_id[0]
                next_id[0] += 1
                u = rng.random()
                if u < 0.03 and recent:
                    tid = recent[int(rng.integers(0, len(recent)))]      # id reuse (any ledger)
                elif u < 0.04 and postvoids:
                    tid = postvoids[int(rng.integers(0, len(postvoids)))]
                r["id_lo"] = tid & 0xFFFFFFFFFFFFFFFF
                r["id_hi"] = tid >> 64
                l = int(rng.integers(1, L + 1))
                d = int(rng.integers(0, A))
                c = int(rng.integers(0, A - 1))
                c = c + 1 if c >= d else c
                kind = rng.choice(6, p=[0.45, 0.2, 0.15, 0.1, 0.05, 0.05])
                r["ledger"] = l
                r["code"] = int(rng.integers(1, 5))
                r["user_data_64"] = int(rng.integers(0, 2))
                amt = int(rng.integers(1, 3000))
                if kind in (2, 3) and pendings:
                    if rng.random() < 0.05 and postvoids:
                        pid, pamt, pl = postvoids[int(rng.integers(0, len(postvoids)))], 10, l
                    else:
                        pid, pamt, pl = pendings[int(rng.integers(0, len(pendings)))]
                    r["pending_id_lo"] = pid
                    r["flags"] = int(TransferFlags.post_pending_transfer if kind == 2
                                     else TransferFlags.void_pending_transfer)
                    r["amount_lo"] = 0 if rng.random() < 0.4 else int(rng.integers(1, pamt + 2))
                    r["ledger"] = 0 if rng.random() < 0.6 else pl
                    r["code"] = 0
                    postvoids.append(tid)
                else:
                    r["debit_account_id_lo"] = acct(l, d)
                    r["credit_account_id_lo"] = acct(l, c)
                    r["amount_lo"] = amt
                    if kind == 1:
                        r["flags"] = int(TransferFlags.pending)
                        r["timeout"] = 0 if rng.random() < 0.7 else int(rng.integers(1, 100))
                        new_p.append((tid, amt, l))
                    elif kind == 4:
                        r["flags"] = int(TransferFlags.balancing_debit)
                        r["amount_lo"] = 0 if rng.random() < 0.5 else amt
                    elif kind == 5:
                        r["flags"] = int(TransferFlags.balancing_credit)
                        r["amount_lo"] = 0 if rng.random() < 0.5 else amt
                    if rng.random() < 0.03:   # accounts on another ledger
                        r["credit_account_id_lo"] = acct(l % L + 1, c)
                    if rng.random() < 0.02:
                        r["ledger"] = l % L + 1
                if rng.random() < 0.01:
                    r["debit_account_id_lo"] = acct(L + 3, 0)   # unknown account
                if rng.random() < 0.01:
                    r["code"] = 0
                recent.append(tid)
            # chains, half of them spanning ledgers (consecutive events, different ledgers)
            j = 0
            while j < batch - 1:
                if rng.random() < 0.12:
                    ln = min(int(rng.integers(2, 6)), batch - j)
                    for q in range(j, j + ln - 1):
                        t[q]["flags"] |= int(TransferFlags.linked)
                    j += ln
                else:
                    j += 1
            if rng.random() < 0.1:
                t[batch - 1]["flags"] |= int(TransferFlags.linked)       # open chain
            self.batches.append(t)
            pendings.extend(new_p)
            recent = recent[-400:]
            postvoids = postvoids[-100:]

    def step_batches(self, step: int, rank: int) -> list[np.ndarray]:
        base = step * self.world * self.B + rank * self.B
        return self.batches[base:base + self.B]

    def global_sequence(self):
        return self.batches


def config4_small(seed: int, world: int, steps: int, batches_per_rank: int, batch: int = 256,
                  ledgers: int = 16, accounts_per_ledger: int = 64, cross: float = 0.02):
    """BASELINE config 4 in miniature (uniform pairs within a ledger + cross-ledger
    linked pairs), laid out like ShardWorkload."""
    from tigerbeetle_amd import workload
    total = steps * world * batches_per_rank * batch
    w = workload.config4(transfer_count=total, ledgers=ledgers, accounts_per_ledger=accounts_per_ledger,
                         seed=seed, cross_ledger_pairs=cross, batch=batch)
    sw = ShardWorkload.__new__(ShardWorkload)
    sw.world, sw.steps, sw.B = world, steps, batches_per_rank
    sw.accounts = w.accounts
    sw.account_batches = [w.accounts[i:i + 4096] for i in range(0, len(w.accounts), 4096)]
    sw.batches = [w.transfers[i:i + batch] for i in range(0, total, batch)]
    return sw


def config4_failing(seed: int, world: int, steps: int, batches_per_rank: int, batch: int = 256,
                    limits: bool = False):
    """config4_small whose cross-ledger pairs sometimes break: a member with code 0 or an
    unknown debit account fails by itself (`limits` = False: every outcome is
    independent of other transfers, the device step's one-dry-run case), or, with
    `limits`, some accounts carry debits_must_not_exceed_credits with little credit,
    so members fail on balances written by other transfers (the dry-round case)."""
    from tigerbeetle_amd.types import AccountFlags, TransferFlags
    sw = config4_small(seed, world, steps, batches_per_rank, batch=batch, cross=0.1)
    rng = np.random.default_rng(seed + 1000)
    if limits:
        acc = sw.accounts.copy()
        lim = rng.random(len(acc)) < 0.3
        acc["flags"][lim] |= np.uint16(int(AccountFlags.debits_must_not_exceed_credits))
        sw.accounts = acc
        sw.account_batches = [acc[i:i + 4096] for i in range(0, len(acc), 4096)]
    out = []
    for b in sw.batches:
        b = b.copy()
        linked = (b["flags"] & int(TransferFlags.linked)) != 0
        pairs = np.nonzero(linked)[0]
        for j in pairs:
            u = rng.random()
            k = j + int(rng.integers(0, 2))
            if u < 0.15:
                b[k]["code"] = 0
            elif u < 0.25:
                b[k]["debit_account_id_hi"] = 7  # unknown account
        out.append(b)
    sw.batches = out
    return sw


def random_u128_ids(sw: ShardWorkload, seed: int) -> ShardWorkload:
    """The same workload with every transfer id (and every pending id naming one) mapped
    through a random bijection into the whole u128 space: ids neither rise along the
    global order nor fit 64 bits (the general step's directory, not the fast step's
    key-range filter, decides every `exists` and every pending)."""
    rng = np.random.default_rng(seed)
    vals = set()
    for b in sw.batches:
        for f in ("id", "pending_id"):
            v = (b[f + "_hi"].astype(object) << 64) | b[f + "_lo"].astype(object)
            vals.update(int(x) for x in v if x)
    vals = sorted(vals)
    out = set()
    while len(out) < len(vals):
        out.add((int(rng.integers(1, 1 << 63)) << 65) ^ int(rng.integers(1, 1 << 63)))
    m = dict(zip(vals, rng.permutation(sorted(out)).tolist()))
    batches = []
    for b in sw.batches:
        b = b.copy()
        for f in ("id", "pending_id"):
            v = (b[f + "_hi"].astype(object) << 64) | b[f + "_lo"].astype(object)
            new = [m.get(int(x), 0) for x in v]
            b[f + "_lo"] = np.array([x & 0xFFFFFFFFFFFFFFFF for x in new], dtype=np.uint64)
            b[f + "_hi"] = np.array([x >> 64 for x in new], dtype=np.uint64)
        batches.append(b)
    sw.batches = batches
    return sw
