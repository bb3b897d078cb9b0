/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h for who may use it).
 *
 * A sequential, one-event-at-a-time restatement of the reference commit path:
 *
 *   execute                          src/state_machine.zig:1002-1088
 *   create_account / _exists         src/state_machine.zig:1198-1237
 *   create_transfer / _exists        src/state_machine.zig:1239-1389
 *   post_or_void_pending_transfer    src/state_machine.zig:1391-1498
 *   post_or_void_pending_..._exists  src/state_machine.zig:1500-1561
 *   get_transfer / get_posted        src/state_machine.zig:1563-1573
 *   sum_overflows                    src/state_machine.zig:1645-1650
 *   lookup_accounts / _transfers     src/state_machine.zig:1091-1126
 *   get_account_transfers / _history src/state_machine.zig:693-885, :1128-1196
 *
 * State is three maps (accounts, transfers, posted) plus the account-history
 * log.  Linked-chain scopes (scope_open/scope_close, :972-1000) are an undo log
 * replayed in reverse on discard — the observable semantics of the groove
 * scope (src/lsm/groove.zig:1036-1060, src/lsm/cache_map.zig:254-301).  The
 * groove object caches and prefetch are cache fills only and do not change
 * results (src/lsm/groove.zig:441-469), so they have no counterpart here.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <assert.h>

typedef unsigned __int128 u128;
#define U128_MAX (~(u128)0)

static inline u128 u128_of(tbgpu_uint128_t x) { return ((u128)x.hi << 64) | x.lo; }
static inline tbgpu_uint128_t tb_of(u128 x) {
    tbgpu_uint128_t r = {(uint64_t)x, (uint64_t)(x >> 64)};
    return r;
}
#define G(x) u128_of(x)

/* sum_overflows: std.math.add overflow → true (src/state_machine.zig:1645-1650). */
static inline int sum_overflows_u128(u128 a, u128 b) { return a + b < a; }
static inline int sum_overflows_u64(uint64_t a, uint64_t b) { return (uint64_t)(a + b) < a; }

/* ---------------------------------------------------------------- maps ---- */

static inline uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 27; z *= 0x94d049bb133111ebull;
    z ^= z >> 31; return z;
}

/* Open addressing (linear probing, backward-shift delete), key u128 -> u64 value. */
typedef struct {
    u128* keys;
    uint64_t* vals;
    uint8_t* used;
    uint64_t cap, len;
} map_t;

static void map_init(map_t* m, uint64_t cap_hint) {
    uint64_t cap = 16;
    while (cap < cap_hint * 2) cap <<= 1;
    m->cap = cap;
    m->len = 0;
    m->keys = (u128*)calloc(cap, sizeof(u128));
    m->vals = (uint64_t*)calloc(cap, sizeof(uint64_t));
    m->used = (uint8_t*)calloc(cap, 1);
}
static void map_free(map_t* m) { free(m->keys); free(m->vals); free(m->used); }
static inline uint64_t map_hash(u128 k) { return mix64((uint64_t)k ^ mix64((uint64_t)(k >> 64))); }

static int map_get(const map_t* m, u128 k, uint64_t* v) {
    uint64_t mask = m->cap - 1, i = map_hash(k) & mask;
    while (m->used[i]) {
        if (m->keys[i] == k) { if (v) *v = m->vals[i]; return 1; }
        i = (i + 1) & mask;
    }
    return 0;
}
static void map_put_new(map_t* m, u128 k, uint64_t v);
static void map_grow(map_t* m) {
    map_t n;
    map_init(&n, m->cap);  /* doubles */
    for (uint64_t i = 0; i < m->cap; i++)
        if (m->used[i]) map_put_new(&n, m->keys[i], m->vals[i]);
    map_free(m);
    *m = n;
}
static void map_put_new(map_t* m, u128 k, uint64_t v) {
    if ((m->len + 1) * 2 > m->cap) map_grow(m);
    uint64_t mask = m->cap - 1, i = map_hash(k) & mask;
    while (m->used[i]) { assert(m->keys[i] != k); i = (i + 1) & mask; }
    m->used[i] = 1; m->keys[i] = k; m->vals[i] = v; m->len++;
}
static void map_remove(map_t* m, u128 k) {
    uint64_t mask = m->cap - 1, i = map_hash(k) & mask;
    while (m->used[i] && m->keys[i] != k) i = (i + 1) & mask;
    assert(m->used[i]);
    m->used[i] = 0; m->len--;
    uint64_t j = i;
    for (;;) {  /* backward-shift deletion */
        j = (j + 1) & mask;
        if (!m->used[j]) break;
        uint64_t h = map_hash(m->keys[j]) & mask;
        /* entry at j may move to i iff its home h is not in (i, j] cyclically */
        int in_range = (i <= j) ? (h > i && h <= j) : (h > i || h <= j);
        if (!in_range) {
            m->keys[i] = m->keys[j]; m->vals[i] = m->vals[j]; m->used[i] = 1;
            m->used[j] = 0; i = j;
        }
    }
}

/* ---------------------------------------------------------------- state --- */

enum { UNDO_ACCOUNT_INSERT, UNDO_ACCOUNT_UPDATE, UNDO_TRANSFER_INSERT, UNDO_POSTED_INSERT,
       UNDO_HISTORY_INSERT };
typedef struct { int kind; uint64_t index; tbgpu_account_t old; u128 key; } undo_t;

enum { FULFILLMENT_POSTED = 0, FULFILLMENT_VOIDED = 1 };  /* src/state_machine.zig:235-248 */

struct orc {
    map_t account_map;  /* id -> index into accounts */
    tbgpu_account_t* accounts; uint64_t accounts_len, accounts_cap;
    map_t transfer_map; /* id -> index into transfers */
    tbgpu_transfer_t* transfers; uint64_t transfers_len, transfers_cap;
    map_t posted_map;   /* pending timestamp -> fulfillment */
    tbgpu_account_history_t* history; uint64_t history_len, history_cap;
    uint64_t commit_timestamp;
    uint64_t* imp; uint64_t imp_len, imp_cap;  /* rows imported from other shards, ascending */
    /* scope (at most one open at a time: chains do not nest) */
    int scope_open;
    undo_t* undo; uint64_t undo_len, undo_cap;
};

static void* grow(void* p, uint64_t* cap, uint64_t need, size_t elem) {
    if (need <= *cap) return p;
    uint64_t c = *cap ? *cap : 1024;
    while (c < need) c *= 2;
    p = realloc(p, c * elem);
    *cap = c;
    return p;
}

static void undo_push(orc_t* o, int kind, uint64_t index, const tbgpu_account_t* old, u128 key) {
    if (!o->scope_open) return;
    o->undo = (undo_t*)grow(o->undo, &o->undo_cap, o->undo_len + 1, sizeof(undo_t));
    undo_t* u = &o->undo[o->undo_len++];
    u->kind = kind; u->index = index; u->key = key;
    if (old) u->old = *old;
}

/* scope_open / scope_close (src/state_machine.zig:972-1000). */
static void scope_open(orc_t* o) { assert(!o->scope_open); o->scope_open = 1; o->undo_len = 0; }
static void scope_close(orc_t* o, int discard) {
    assert(o->scope_open);
    if (discard) {
        while (o->undo_len > 0) {  /* LIFO replay */
            undo_t* u = &o->undo[--o->undo_len];
            switch (u->kind) {
            case UNDO_ACCOUNT_INSERT:
                map_remove(&o->account_map, u->key);
                assert(u->index == o->accounts_len - 1);
                o->accounts_len--;
                break;
            case UNDO_ACCOUNT_UPDATE: o->accounts[u->index] = u->old; break;
            case UNDO_TRANSFER_INSERT:
                map_remove(&o->transfer_map, u->key);
                assert(u->index == o->transfers_len - 1);
                o->transfers_len--;
                break;
            case UNDO_POSTED_INSERT: map_remove(&o->posted_map, u->key); break;
            case UNDO_HISTORY_INSERT: o->history_len--; break;
            }
        }
    }
    o->undo_len = 0;
    o->scope_open = 0;
}

static tbgpu_account_t* get_account(orc_t* o, u128 id) {
    uint64_t i;
    return map_get(&o->account_map, id, &i) ? &o->accounts[i] : NULL;
}
/* get_transfer (src/state_machine.zig:1563-1565) */
static tbgpu_transfer_t* get_transfer(orc_t* o, u128 id) {
    uint64_t i;
    return map_get(&o->transfer_map, id, &i) ? &o->transfers[i] : NULL;
}
/* get_posted (src/state_machine.zig:1568-1573): -1 when absent. */
static int get_posted(orc_t* o, uint64_t pending_timestamp) {
    uint64_t v;
    return map_get(&o->posted_map, (u128)pending_timestamp, &v) ? (int)v : -1;
}

static void accounts_insert(orc_t* o, const tbgpu_account_t* a) {
    o->accounts = (tbgpu_account_t*)grow(o->accounts, &o->accounts_cap, o->accounts_len + 1, sizeof(tbgpu_account_t));
    uint64_t i = o->accounts_len++;
    o->accounts[i] = *a;
    map_put_new(&o->account_map, G(a->id), i);
    undo_push(o, UNDO_ACCOUNT_INSERT, i, NULL, G(a->id));
}
static void accounts_update(orc_t* o, tbgpu_account_t* old, const tbgpu_account_t* new_) {
    uint64_t i = (uint64_t)(old - o->accounts);
    undo_push(o, UNDO_ACCOUNT_UPDATE, i, old, 0);
    o->accounts[i] = *new_;
}
static void transfers_insert(orc_t* o, const tbgpu_transfer_t* t) {
    o->transfers = (tbgpu_transfer_t*)grow(o->transfers, &o->transfers_cap, o->transfers_len + 1, sizeof(tbgpu_transfer_t));
    uint64_t i = o->transfers_len++;
    o->transfers[i] = *t;
    map_put_new(&o->transfer_map, G(t->id), i);
    undo_push(o, UNDO_TRANSFER_INSERT, i, NULL, G(t->id));
}
static void posted_insert(orc_t* o, uint64_t timestamp, int fulfillment) {
    map_put_new(&o->posted_map, (u128)timestamp, (uint64_t)fulfillment);
    undo_push(o, UNDO_POSTED_INSERT, 0, NULL, (u128)timestamp);
}
static void history_insert(orc_t* o, const tbgpu_account_history_t* h) {
    o->history = (tbgpu_account_history_t*)grow(o->history, &o->history_cap, o->history_len + 1, sizeof(*h));
    o->history[o->history_len++] = *h;
    undo_push(o, UNDO_HISTORY_INSERT, 0, NULL, 0);
}

/* ------------------------------------------------------ create_account ---- */

/* create_account_exists (src/state_machine.zig:1227-1237) */
static uint32_t create_account_exists(const tbgpu_account_t* a, const tbgpu_account_t* e) {
    if (a->flags != e->flags) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (G(a->user_data_128) != G(e->user_data_128)) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (a->user_data_64 != e->user_data_64) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (a->user_data_32 != e->user_data_32) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (a->ledger != e->ledger) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_LEDGER;
    if (a->code != e->code) return TBGPU_CREATE_ACCOUNT_EXISTS_WITH_DIFFERENT_CODE;
    return TBGPU_CREATE_ACCOUNT_EXISTS;
}

/* create_account (src/state_machine.zig:1198-1225) */
static uint32_t create_account(orc_t* o, const tbgpu_account_t* a) {
    if (a->reserved != 0) return TBGPU_CREATE_ACCOUNT_RESERVED_FIELD;
    if (a->flags & 0xFFF0u) return TBGPU_CREATE_ACCOUNT_RESERVED_FLAG;
    if (G(a->id) == 0) return TBGPU_CREATE_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (G(a->id) == U128_MAX) return TBGPU_CREATE_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if ((a->flags & TBGPU_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
        (a->flags & TBGPU_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
        return TBGPU_CREATE_ACCOUNT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (G(a->debits_pending) != 0) return TBGPU_CREATE_ACCOUNT_DEBITS_PENDING_MUST_BE_ZERO;
    if (G(a->debits_posted) != 0) return TBGPU_CREATE_ACCOUNT_DEBITS_POSTED_MUST_BE_ZERO;
    if (G(a->credits_pending) != 0) return TBGPU_CREATE_ACCOUNT_CREDITS_PENDING_MUST_BE_ZERO;
    if (G(a->credits_posted) != 0) return TBGPU_CREATE_ACCOUNT_CREDITS_POSTED_MUST_BE_ZERO;
    if (a->ledger == 0) return TBGPU_CREATE_ACCOUNT_LEDGER_MUST_NOT_BE_ZERO;
    if (a->code == 0) return TBGPU_CREATE_ACCOUNT_CODE_MUST_NOT_BE_ZERO;

    tbgpu_account_t* e = get_account(o, G(a->id));
    if (e) return create_account_exists(a, e);

    accounts_insert(o, a);
    o->commit_timestamp = a->timestamp;
    return TBGPU_CREATE_ACCOUNT_OK;
}

/* ----------------------------------------------------- create_transfer ---- */

/* create_transfer_exists (src/state_machine.zig:1370-1389) */
static uint32_t create_transfer_exists(const tbgpu_transfer_t* t, const tbgpu_transfer_t* e) {
    if (t->flags != e->flags) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_FLAGS;
    if (G(t->debit_account_id) != G(e->debit_account_id)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (G(t->credit_account_id) != G(e->credit_account_id)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (G(t->amount) != G(e->amount)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_AMOUNT;
    if (G(t->user_data_128) != G(e->user_data_128)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (t->user_data_64 != e->user_data_64) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (t->user_data_32 != e->user_data_32) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (t->timeout != e->timeout) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_TIMEOUT;
    if (t->code != e->code) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_CODE;
    return TBGPU_CREATE_TRANSFER_EXISTS;
}

/* post_or_void_pending_transfer_exists (src/state_machine.zig:1500-1561) */
static uint32_t post_or_void_pending_transfer_exists(const tbgpu_transfer_t* t, const tbgpu_transfer_t* e,
                                                     const tbgpu_transfer_t* p) {
    if (t->flags != e->flags) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_FLAGS;
    if (G(t->amount) == 0) {
        if (G(e->amount) != G(p->amount)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_AMOUNT;
    } else {
        if (G(t->amount) != G(e->amount)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_AMOUNT;
    }
    if (G(t->pending_id) != G(e->pending_id)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_PENDING_ID;
    if (G(t->user_data_128) == 0) {
        if (G(e->user_data_128) != G(p->user_data_128)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    } else {
        if (G(t->user_data_128) != G(e->user_data_128)) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    }
    if (t->user_data_64 == 0) {
        if (e->user_data_64 != p->user_data_64) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    } else {
        if (t->user_data_64 != e->user_data_64) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    }
    if (t->user_data_32 == 0) {
        if (e->user_data_32 != p->user_data_32) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    } else {
        if (t->user_data_32 != e->user_data_32) return TBGPU_CREATE_TRANSFER_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    }
    return TBGPU_CREATE_TRANSFER_EXISTS;
}

#define NS_PER_S 1000000000ull

/* post_or_void_pending_transfer (src/state_machine.zig:1391-1498) */
static uint32_t post_or_void_pending_transfer(orc_t* o, const tbgpu_transfer_t* t) {
    const uint16_t f = t->flags;
    const int post = (f & TBGPU_TRANSFER_POST_PENDING_TRANSFER) != 0;
    const int void_ = (f & TBGPU_TRANSFER_VOID_PENDING_TRANSFER) != 0;
    if (post && void_) return TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TBGPU_TRANSFER_PENDING) return TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TBGPU_TRANSFER_BALANCING_DEBIT) return TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TBGPU_TRANSFER_BALANCING_CREDIT) return TBGPU_CREATE_TRANSFER_FLAGS_ARE_MUTUALLY_EXCLUSIVE;

    if (G(t->pending_id) == 0) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_ZERO;
    if (G(t->pending_id) == U128_MAX) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_NOT_BE_INT_MAX;
    if (G(t->pending_id) == G(t->id)) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_DIFFERENT;
    if (t->timeout != 0) return TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;

    tbgpu_transfer_t* pp = get_transfer(o, G(t->pending_id));
    if (!pp) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_FOUND;
    const tbgpu_transfer_t p = *pp; /* copy: inserts below may move the array */
    if (!(p.flags & TBGPU_TRANSFER_PENDING)) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_NOT_PENDING;

    tbgpu_account_t* dr = get_account(o, G(p.debit_account_id));
    tbgpu_account_t* cr = get_account(o, G(p.credit_account_id));
    assert(dr && cr);
    assert(G(p.amount) > 0);

    if (G(t->debit_account_id) > 0 && G(t->debit_account_id) != G(p.debit_account_id))
        return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (G(t->credit_account_id) > 0 && G(t->credit_account_id) != G(p.credit_account_id))
        return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t->ledger > 0 && t->ledger != p.ledger) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
    if (t->code > 0 && t->code != p.code) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_CODE;

    const u128 amount = G(t->amount) > 0 ? G(t->amount) : G(p.amount);
    if (amount > G(p.amount)) return TBGPU_CREATE_TRANSFER_EXCEEDS_PENDING_TRANSFER_AMOUNT;
    if (void_ && amount < G(p.amount)) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;

    tbgpu_transfer_t* e = get_transfer(o, G(t->id));
    if (e) return post_or_void_pending_transfer_exists(t, e, &p);

    const int posted = get_posted(o, p.timestamp);
    if (posted == FULFILLMENT_POSTED) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_ALREADY_POSTED;
    if (posted == FULFILLMENT_VOIDED) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_ALREADY_VOIDED;

    assert(p.timestamp < t->timestamp);
    if (p.timeout > 0) {
        const uint64_t timeout_ns = (uint64_t)p.timeout * NS_PER_S;
        if (t->timestamp >= p.timestamp + timeout_ns) return TBGPU_CREATE_TRANSFER_PENDING_TRANSFER_EXPIRED;
    }

    tbgpu_transfer_t s;
    memset(&s, 0, sizeof s);
    s.id = t->id;
    s.debit_account_id = p.debit_account_id;
    s.credit_account_id = p.credit_account_id;
    s.user_data_128 = G(t->user_data_128) > 0 ? t->user_data_128 : p.user_data_128;
    s.user_data_64 = t->user_data_64 > 0 ? t->user_data_64 : p.user_data_64;
    s.user_data_32 = t->user_data_32 > 0 ? t->user_data_32 : p.user_data_32;
    s.ledger = p.ledger;
    s.code = p.code;
    s.pending_id = t->pending_id;
    s.timeout = 0;
    s.timestamp = t->timestamp;
    s.flags = t->flags;
    s.amount = tb_of(amount);
    transfers_insert(o, &s);

    posted_insert(o, p.timestamp, post ? FULFILLMENT_POSTED : FULFILLMENT_VOIDED);

    tbgpu_account_t dr_new = *dr, cr_new = *cr;
    dr_new.debits_pending = tb_of(G(dr_new.debits_pending) - G(p.amount));
    cr_new.credits_pending = tb_of(G(cr_new.credits_pending) - G(p.amount));
    if (post) {
        assert(amount > 0 && amount <= G(p.amount));
        dr_new.debits_posted = tb_of(G(dr_new.debits_posted) + amount);
        cr_new.credits_posted = tb_of(G(cr_new.credits_posted) + amount);
    }
    accounts_update(o, dr, &dr_new);
    accounts_update(o, cr, &cr_new);

    o->commit_timestamp = t->timestamp;
    return TBGPU_CREATE_TRANSFER_OK;
}

/* Account.debits_exceed_credits / credits_exceed_debits (src/tigerbeetle.zig:31-39) */
static int debits_exceed_credits(const tbgpu_account_t* a, u128 amount) {
    return (a->flags & TBGPU_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
           G(a->debits_pending) + G(a->debits_posted) + amount > G(a->credits_posted);
}
static int credits_exceed_debits(const tbgpu_account_t* a, u128 amount) {
    return (a->flags & TBGPU_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) &&
           G(a->credits_pending) + G(a->credits_posted) + amount > G(a->debits_posted);
}

/* create_transfer (src/state_machine.zig:1239-1368) */
static uint32_t create_transfer(orc_t* o, const tbgpu_transfer_t* t) {
    const uint16_t f = t->flags;
    if (f & 0xFFC0u) return TBGPU_CREATE_TRANSFER_RESERVED_FLAG;
    if (G(t->id) == 0) return TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_ZERO;
    if (G(t->id) == U128_MAX) return TBGPU_CREATE_TRANSFER_ID_MUST_NOT_BE_INT_MAX;

    if (f & (TBGPU_TRANSFER_POST_PENDING_TRANSFER | TBGPU_TRANSFER_VOID_PENDING_TRANSFER))
        return post_or_void_pending_transfer(o, t);

    if (G(t->debit_account_id) == 0) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (G(t->debit_account_id) == U128_MAX) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (G(t->credit_account_id) == 0) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (G(t->credit_account_id) == U128_MAX) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (G(t->credit_account_id) == G(t->debit_account_id)) return TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_BE_DIFFERENT;

    if (G(t->pending_id) != 0) return TBGPU_CREATE_TRANSFER_PENDING_ID_MUST_BE_ZERO;
    if (!(f & TBGPU_TRANSFER_PENDING)) {
        if (t->timeout != 0) return TBGPU_CREATE_TRANSFER_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    }
    const int bdr = (f & TBGPU_TRANSFER_BALANCING_DEBIT) != 0;
    const int bcr = (f & TBGPU_TRANSFER_BALANCING_CREDIT) != 0;
    if (!bdr && !bcr) {
        if (G(t->amount) == 0) return TBGPU_CREATE_TRANSFER_AMOUNT_MUST_NOT_BE_ZERO;
    }
    if (t->ledger == 0) return TBGPU_CREATE_TRANSFER_LEDGER_MUST_NOT_BE_ZERO;
    if (t->code == 0) return TBGPU_CREATE_TRANSFER_CODE_MUST_NOT_BE_ZERO;

    tbgpu_account_t* dr = get_account(o, G(t->debit_account_id));
    if (!dr) return TBGPU_CREATE_TRANSFER_DEBIT_ACCOUNT_NOT_FOUND;
    tbgpu_account_t* cr = get_account(o, G(t->credit_account_id));
    if (!cr) return TBGPU_CREATE_TRANSFER_CREDIT_ACCOUNT_NOT_FOUND;

    if (dr->ledger != cr->ledger) return TBGPU_CREATE_TRANSFER_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t->ledger != dr->ledger) return TBGPU_CREATE_TRANSFER_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;

    tbgpu_transfer_t* e = get_transfer(o, G(t->id));
    if (e) return create_transfer_exists(t, e);

    u128 amount = G(t->amount);
    if (bdr || bcr) {
        if (amount == 0) amount = (u128)UINT64_MAX; /* std.math.maxInt(u64) */
    }
    if (bdr) {
        const u128 dr_balance = G(dr->debits_posted) + G(dr->debits_pending);
        const u128 cpo = G(dr->credits_posted);
        const u128 avail = cpo > dr_balance ? cpo - dr_balance : 0; /* -| saturating */
        if (avail < amount) amount = avail;
        if (amount == 0) return TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS;
    }
    if (bcr) {
        const u128 cr_balance = G(cr->credits_posted) + G(cr->credits_pending);
        const u128 dpo = G(cr->debits_posted);
        const u128 avail = dpo > cr_balance ? dpo - cr_balance : 0;
        if (avail < amount) amount = avail;
        if (amount == 0) return TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS;
    }

    if (f & TBGPU_TRANSFER_PENDING) {
        if (sum_overflows_u128(amount, G(dr->debits_pending))) return TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS_PENDING;
        if (sum_overflows_u128(amount, G(cr->credits_pending))) return TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS_PENDING;
    }
    if (sum_overflows_u128(amount, G(dr->debits_posted))) return TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS_POSTED;
    if (sum_overflows_u128(amount, G(cr->credits_posted))) return TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS_POSTED;
    if (sum_overflows_u128(amount, G(dr->debits_pending) + G(dr->debits_posted))) return TBGPU_CREATE_TRANSFER_OVERFLOWS_DEBITS;
    if (sum_overflows_u128(amount, G(cr->credits_pending) + G(cr->credits_posted))) return TBGPU_CREATE_TRANSFER_OVERFLOWS_CREDITS;

    if (sum_overflows_u64(t->timestamp, (uint64_t)t->timeout * NS_PER_S)) return TBGPU_CREATE_TRANSFER_OVERFLOWS_TIMEOUT;
    if (debits_exceed_credits(dr, amount)) return TBGPU_CREATE_TRANSFER_EXCEEDS_CREDITS;
    if (credits_exceed_debits(cr, amount)) return TBGPU_CREATE_TRANSFER_EXCEEDS_DEBITS;

    tbgpu_transfer_t t2 = *t;
    t2.amount = tb_of(amount);
    transfers_insert(o, &t2);

    tbgpu_account_t dr_new = *dr, cr_new = *cr;
    if (f & TBGPU_TRANSFER_PENDING) {
        dr_new.debits_pending = tb_of(G(dr_new.debits_pending) + amount);
        cr_new.credits_pending = tb_of(G(cr_new.credits_pending) + amount);
    } else {
        dr_new.debits_posted = tb_of(G(dr_new.debits_posted) + amount);
        cr_new.credits_posted = tb_of(G(cr_new.credits_posted) + amount);
    }
    accounts_update(o, dr, &dr_new);
    accounts_update(o, cr, &cr_new);

    if ((dr_new.flags & TBGPU_ACCOUNT_HISTORY) || (cr_new.flags & TBGPU_ACCOUNT_HISTORY)) {
        tbgpu_account_history_t h;
        memset(&h, 0, sizeof h);
        h.timestamp = t2.timestamp;
        if (dr_new.flags & TBGPU_ACCOUNT_HISTORY) {
            h.dr_account_id = dr_new.id;
            h.dr_debits_pending = dr_new.debits_pending;
            h.dr_debits_posted = dr_new.debits_posted;
            h.dr_credits_pending = dr_new.credits_pending;
            h.dr_credits_posted = dr_new.credits_posted;
        }
        if (cr_new.flags & TBGPU_ACCOUNT_HISTORY) {
            h.cr_account_id = cr_new.id;
            h.cr_debits_pending = cr_new.debits_pending;
            h.cr_debits_posted = cr_new.debits_posted;
            h.cr_credits_pending = cr_new.credits_pending;
            h.cr_credits_posted = cr_new.credits_posted;
        }
        history_insert(o, &h);
    }

    o->commit_timestamp = t->timestamp;
    return TBGPU_CREATE_TRANSFER_OK;
}

/* -------------------------------------------------------------- execute --- */

/* execute (src/state_machine.zig:1002-1088), generic over the event kind. */
typedef uint32_t (*create_fn)(orc_t*, const void* event);
static uint32_t create_account_v(orc_t* o, const void* e) { return create_account(o, (const tbgpu_account_t*)e); }
static uint32_t create_transfer_v(orc_t* o, const void* e) { return create_transfer(o, (const tbgpu_transfer_t*)e); }

/* `ev_ts` / `ctl` (may be NULL): the routed form used by the sharded commit
 * (include/tbgpu.h, tbgpu_create_transfers_routed) -- per-event timestamps and
 * TBGPU_CTL_* chain control.  NULL reproduces execute exactly. */
static uint32_t execute_ex(orc_t* o, uint64_t timestamp, const uint8_t* events, uint32_t n, size_t size,
                           create_fn create, uint32_t* results /* pairs {index,result} */,
                           const uint64_t* ev_ts, const uint8_t* ctl) {
    uint32_t count = 0;
    int64_t chain = -1;
    int chain_broken = 0;
    uint8_t event[128] __attribute__((aligned(16)));
    for (uint32_t index = 0; index < n; index++) {
        memcpy(event, events + (size_t)index * size, size);
        /* flags and timestamp share the layout tail for both structs */
        uint16_t flags; memcpy(&flags, event + 118, 2);
        uint64_t ts; memcpy(&ts, event + 120, 8);
        /* AccountFlags.linked / TransferFlags.linked; a routed chain part ends where
         * the router closed it (the chain continues on another shard) */
        const int linked = (flags & 1) && !(ctl && (ctl[index] & TBGPU_CTL_CHAIN_END));
        const int doom = ctl && (ctl[index] & TBGPU_CTL_DOOM);
        uint32_t result;
        if ((linked || doom) && chain < 0) { chain = index; assert(!chain_broken); scope_open(o); }
        if (linked && index == n - 1) {
            result = TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN; /* == account code 2 */
        } else if (chain_broken || (ctl && (ctl[index] & TBGPU_CTL_SKIP))) {
            result = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
        } else if (ts != 0) {
            result = TBGPU_CREATE_TRANSFER_TIMESTAMP_MUST_BE_ZERO;
        } else {
            ts = ev_ts ? ev_ts[index] : timestamp - n + index + 1;
            memcpy(event + 120, &ts, 8);
            result = create(o, event);
            /* the chain breaks on another shard right after this member */
            if (doom && result == 0) result = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
        }
        if (result != 0) {
            if (chain >= 0) {
                if (!chain_broken) {
                    chain_broken = 1;
                    scope_close(o, 1);
                    for (uint32_t ci = (uint32_t)chain; ci < index; ci++) {
                        results[2 * count] = ci;
                        results[2 * count + 1] = TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED;
                        count++;
                    }
                } else {
                    assert(result == TBGPU_CREATE_TRANSFER_LINKED_EVENT_FAILED ||
                           result == TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN);
                }
            }
            results[2 * count] = index;
            results[2 * count + 1] = result;
            count++;
        }
        if (chain >= 0 && (!linked || result == TBGPU_CREATE_TRANSFER_LINKED_EVENT_CHAIN_OPEN)) {
            if (!chain_broken) scope_close(o, 0);
            chain = -1;
            chain_broken = 0;
        }
    }
    assert(chain < 0 && !chain_broken);
    return count;
}

static uint32_t execute(orc_t* o, uint64_t timestamp, const uint8_t* events, uint32_t n, size_t size,
                        create_fn create, uint32_t* results) {
    return execute_ex(o, timestamp, events, n, size, create, results, NULL, NULL);
}

/* ------------------------------------------------------------------ API --- */

orc_t* orc_new(uint64_t accounts_hint, uint64_t transfers_hint) {
    orc_t* o = (orc_t*)calloc(1, sizeof(orc_t));
    map_init(&o->account_map, accounts_hint ? accounts_hint : 1024);
    map_init(&o->transfer_map, transfers_hint ? transfers_hint : 1024);
    map_init(&o->posted_map, 1024);
    o->accounts = (tbgpu_account_t*)grow(NULL, &o->accounts_cap, accounts_hint ? accounts_hint : 1024, sizeof(tbgpu_account_t));
    o->transfers = (tbgpu_transfer_t*)grow(NULL, &o->transfers_cap, transfers_hint ? transfers_hint : 1024, sizeof(tbgpu_transfer_t));
    return o;
}

void orc_free(orc_t* o) {
    if (!o) return;
    map_free(&o->account_map); map_free(&o->transfer_map); map_free(&o->posted_map);
    free(o->accounts); free(o->transfers); free(o->history); free(o->undo); free(o->imp);
    free(o);
}

uint32_t orc_create_accounts(orc_t* o, uint64_t timestamp, const tbgpu_account_t* events, uint32_t count,
                             tbgpu_create_accounts_result_t* results) {
    return execute(o, timestamp, (const uint8_t*)events, count, sizeof(tbgpu_account_t), create_account_v,
                   (uint32_t*)results);
}
uint32_t orc_create_transfers(orc_t* o, uint64_t timestamp, const tbgpu_transfer_t* events, uint32_t count,
                              tbgpu_create_transfers_result_t* results) {
    return execute(o, timestamp, (const uint8_t*)events, count, sizeof(tbgpu_transfer_t), create_transfer_v,
                   (uint32_t*)results);
}

uint64_t orc_create_transfers_batches(orc_t* o, uint32_t batch_count, const uint64_t* timestamps,
                                      const uint32_t* counts, const tbgpu_transfer_t* events,
                                      tbgpu_create_transfers_result_t* results, uint32_t* result_counts,
                                      double* elapsed_s) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint64_t off = 0, total = 0;
    for (uint32_t b = 0; b < batch_count; b++) {
        uint32_t c = orc_create_transfers(o, timestamps[b], events + off, counts[b], results + off);
        if (result_counts) result_counts[b] = c;
        total += c;
        off += counts[b];
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (elapsed_s) *elapsed_s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return total;
}

uint64_t orc_create_accounts_batches(orc_t* o, uint32_t batch_count, const uint64_t* timestamps,
                                     const uint32_t* counts, const tbgpu_account_t* events,
                                     tbgpu_create_accounts_result_t* results, uint32_t* result_counts) {
    uint64_t off = 0, total = 0;
    for (uint32_t b = 0; b < batch_count; b++) {
        uint32_t c = orc_create_accounts(o, timestamps[b], events + off, counts[b], results + off);
        if (result_counts) result_counts[b] = c;
        total += c;
        off += counts[b];
    }
    return total;
}

/* execute_lookup_accounts (src/state_machine.zig:1091-1107) */
uint32_t orc_lookup_accounts(orc_t* o, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_account_t* out) {
    uint32_t n = 0;
    for (uint32_t i = 0; i < count; i++) {
        tbgpu_account_t* a = get_account(o, G(ids[i]));
        if (a) out[n++] = *a;
    }
    return n;
}
/* execute_lookup_transfers (src/state_machine.zig:1110-1126) */
uint32_t orc_lookup_transfers(orc_t* o, const tbgpu_uint128_t* ids, uint32_t count, tbgpu_transfer_t* out) {
    uint32_t n = 0;
    for (uint32_t i = 0; i < count; i++) {
        tbgpu_transfer_t* t = get_transfer(o, G(ids[i]));
        if (t) out[n++] = *t;
    }
    return n;
}

/* Test harness `setup` (src/state_machine.zig:1892-1908). */
int orc_set_balances(orc_t* o, tbgpu_uint128_t id, tbgpu_uint128_t dp, tbgpu_uint128_t dpo, tbgpu_uint128_t cp,
                     tbgpu_uint128_t cpo) {
    tbgpu_account_t* a = get_account(o, G(id));
    if (!a) return -1;
    a->debits_pending = dp; a->debits_posted = dpo; a->credits_pending = cp; a->credits_posted = cpo;
    return 0;
}

uint64_t orc_account_count(orc_t* o) { return o->accounts_len; }
uint64_t orc_transfer_count(orc_t* o) { return o->transfers_len; }
uint64_t orc_history_count(orc_t* o) { return o->history_len; }
uint64_t orc_export_accounts(orc_t* o, tbgpu_account_t* out, uint64_t capacity) {
    uint64_t n = o->accounts_len < capacity ? o->accounts_len : capacity;
    memcpy(out, o->accounts, n * sizeof(tbgpu_account_t));
    return n;
}
uint64_t orc_export_transfers(orc_t* o, uint64_t first, uint64_t count, tbgpu_transfer_t* out) {
    if (first >= o->transfers_len) return 0;
    if (first + count > o->transfers_len) count = o->transfers_len - first;
    memcpy(out, o->transfers + first, count * sizeof(tbgpu_transfer_t));
    return count;
}
uint64_t orc_export_history(orc_t* o, uint64_t first, uint64_t count, tbgpu_account_history_t* out) {
    if (first >= o->history_len) return 0;
    if (first + count > o->history_len) count = o->history_len - first;
    memcpy(out, o->history + first, count * sizeof(tbgpu_account_history_t));
    return count;
}
int orc_get_posted(orc_t* o, tbgpu_uint128_t pending_id) {
    tbgpu_transfer_t* p = get_transfer(o, G(pending_id));
    if (!p) return -1;
    return get_posted(o, p->timestamp);
}
uint64_t orc_commit_timestamp(orc_t* o) { return o->commit_timestamp; }

int orc_sum_overflows_u64(uint64_t a, uint64_t b) { return sum_overflows_u64(a, b); }
int orc_sum_overflows_u128(tbgpu_uint128_t a, tbgpu_uint128_t b) { return sum_overflows_u128(G(a), G(b)); }

/* ------------------------------------------------------- sharded commit --- */

static void map_copy(map_t* dst, const map_t* src) {
    *dst = *src;
    dst->keys = (u128*)malloc(src->cap * sizeof(u128));
    dst->vals = (uint64_t*)malloc(src->cap * sizeof(uint64_t));
    dst->used = (uint8_t*)malloc(src->cap);
    memcpy(dst->keys, src->keys, src->cap * sizeof(u128));
    memcpy(dst->vals, src->vals, src->cap * sizeof(uint64_t));
    memcpy(dst->used, src->used, src->cap);
}

static void* dup_array(const void* p, uint64_t cap, size_t elem) {
    void* q = malloc((cap ? cap : 1) * elem);
    if (p && cap) memcpy(q, p, cap * elem);
    return q;
}

/* Deep copy: a dry run executes on a clone (tbgpu_create_transfers_routed). */
static orc_t* orc_clone(const orc_t* o) {
    orc_t* c = (orc_t*)calloc(1, sizeof(orc_t));
    *c = *o;
    map_copy(&c->account_map, &o->account_map);
    map_copy(&c->transfer_map, &o->transfer_map);
    map_copy(&c->posted_map, &o->posted_map);
    c->accounts = (tbgpu_account_t*)dup_array(o->accounts, o->accounts_cap, sizeof(tbgpu_account_t));
    c->transfers = (tbgpu_transfer_t*)dup_array(o->transfers, o->transfers_cap, sizeof(tbgpu_transfer_t));
    c->history = (tbgpu_account_history_t*)dup_array(o->history, o->history_cap, sizeof(tbgpu_account_history_t));
    c->undo = (undo_t*)dup_array(o->undo, o->undo_cap, sizeof(undo_t));
    c->imp = (uint64_t*)dup_array(o->imp, o->imp_cap, sizeof(uint64_t));
    return c;
}

uint64_t orc_create_transfers_routed(orc_t* o, uint32_t batch_count, const uint32_t* counts,
                                     const tbgpu_transfer_t* events, const uint64_t* event_ts, const uint8_t* ctl,
                                     int dry_run, tbgpu_create_transfers_result_t* results, uint32_t* result_counts,
                                     uint64_t* commit_timestamp) {
    orc_t* x = dry_run ? orc_clone(o) : o;
    uint64_t off = 0, total = 0;
    for (uint32_t b = 0; b < batch_count; b++) {
        uint32_t c = execute_ex(x, 0, (const uint8_t*)(events + off), counts[b], sizeof(tbgpu_transfer_t),
                                create_transfer_v, (uint32_t*)(results + off), event_ts + off,
                                ctl ? ctl + off : NULL);
        result_counts[b] = c;
        total += c;
        off += counts[b];
    }
    if (commit_timestamp) *commit_timestamp = x->commit_timestamp;
    if (dry_run) orc_free(x);
    return total;
}

int orc_import_transfers(orc_t* o, const tbgpu_transfer_t* rows, uint32_t count) {
    for (uint32_t i = 0; i < count; i++) {
        if (map_get(&o->transfer_map, G(rows[i].id), NULL)) continue;  /* already held */
        o->transfers = (tbgpu_transfer_t*)grow(o->transfers, &o->transfers_cap, o->transfers_len + 1,
                                            sizeof(tbgpu_transfer_t));
        o->transfers[o->transfers_len] = rows[i];
        map_put_new(&o->transfer_map, G(rows[i].id), o->transfers_len);
        o->imp = (uint64_t*)grow(o->imp, &o->imp_cap, o->imp_len + 1, sizeof(uint64_t));
        o->imp[o->imp_len++] = o->transfers_len;  /* another shard's transfer: never queried here */
        o->transfers_len++;
    }
    return 0;
}

void orc_advance_commit_timestamp(orc_t* o, uint64_t timestamp) {
    if (timestamp > o->commit_timestamp) o->commit_timestamp = timestamp;
}

/* ------------------------------------------------------------- queries --- */

#define QUERY_MAX 8190u /* constants.batch_max.get_account_transfers / _history (src/state_machine.zig:53-76) */

/* get_scan_from_filter's validity test (src/state_machine.zig:822-833). */
static int filter_valid(const tbgpu_account_filter_t* f) {
    const u128 id = G(f->account_id);
    for (int k = 0; k < 24; k++)
        if (f->reserved[k]) return 0;
    return id != 0 && id != U128_MAX && f->timestamp_min != UINT64_MAX && f->timestamp_max != UINT64_MAX &&
           (f->timestamp_max == 0 || f->timestamp_min <= f->timestamp_max) && f->limit != 0 &&
           (f->flags & (TBGPU_ACCOUNT_FILTER_DEBITS | TBGPU_ACCOUNT_FILTER_CREDITS)) != 0 && (f->flags >> 3) == 0;
}

static int row_imported(const orc_t* o, uint64_t row) {
    uint64_t lo = 0, hi = o->imp_len;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (o->imp[mid] < row) lo = mid + 1; else hi = mid;
    }
    return lo < o->imp_len && o->imp[lo] == row;
}

/* The account-history row stored under `timestamp` (rows ascend in timestamp). */
static const tbgpu_account_history_t* history_at(const orc_t* o, uint64_t timestamp) {
    uint64_t lo = 0, hi = o->history_len;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (o->history[mid].timestamp < timestamp) lo = mid + 1; else hi = mid;
    }
    return lo < o->history_len && o->history[lo].timestamp == timestamp ? &o->history[lo] : NULL;
}

/* The scan behind both queries: the union of the debit_account_id and
 * credit_account_id prefix scans (:850-884) over the stored transfers -- in
 * timestamp order, which is their insertion order -- restricted to
 * [timestamp_min, timestamp_max] (0 = TimestampRange.timestamp_min / _max,
 * src/lsm/timestamp_range.zig:4-5), descending when reversed, and cut at
 * min(limit, batch_max) objects (:710-713).  get_account_history then looks up
 * the history row of each timestamp (:769-779); a post/void transfer has none
 * (only create_transfer stores one, :1342-1364) and the reference's lookup would
 * assert (src/lsm/scan_lookup.zig:179, :215): it is skipped here. */
static uint32_t scan_account(orc_t* o, const tbgpu_account_filter_t* f, int history, void* out) {
    const u128 id = G(f->account_id);
    const uint32_t limit = f->limit < QUERY_MAX ? f->limit : QUERY_MAX;
    const uint64_t tlo = f->timestamp_min ? f->timestamp_min : 1;
    const uint64_t thi = f->timestamp_max ? f->timestamp_max : UINT64_MAX - 1;
    const int rev = (f->flags & TBGPU_ACCOUNT_FILTER_REVERSED) != 0;
    const int dr = (f->flags & TBGPU_ACCOUNT_FILTER_DEBITS) != 0, cr = (f->flags & TBGPU_ACCOUNT_FILTER_CREDITS) != 0;
    uint32_t n = 0;
    for (uint64_t k = 0; k < o->transfers_len && n < limit; k++) {
        const uint64_t i = rev ? o->transfers_len - 1 - k : k;
        const tbgpu_transfer_t* t = &o->transfers[i];
        if (t->timestamp < tlo || t->timestamp > thi) continue;
        if (!((dr && G(t->debit_account_id) == id) || (cr && G(t->credit_account_id) == id))) continue;
        if (row_imported(o, i)) continue;
        if (!history) {
            ((tbgpu_transfer_t*)out)[n++] = *t;
            continue;
        }
        const tbgpu_account_history_t* h = history_at(o, t->timestamp);
        if (!h) continue;
        /* execute_get_account_history (:1171-1192) */
        tbgpu_account_balance_t b;
        memset(&b, 0, sizeof b);
        if (G(h->dr_account_id) == id) {
            b.debits_pending = h->dr_debits_pending; b.debits_posted = h->dr_debits_posted;
            b.credits_pending = h->dr_credits_pending; b.credits_posted = h->dr_credits_posted;
        } else {
            b.debits_pending = h->cr_debits_pending; b.debits_posted = h->cr_debits_posted;
            b.credits_pending = h->cr_credits_pending; b.credits_posted = h->cr_credits_posted;
        }
        b.timestamp = h->timestamp;
        ((tbgpu_account_balance_t*)out)[n++] = b;
    }
    return n;
}

/* execute_get_account_transfers (src/state_machine.zig:693-734, :1128-1147) */
uint32_t orc_get_account_transfers(orc_t* o, const tbgpu_account_filter_t* f, tbgpu_transfer_t* out) {
    return filter_valid(f) ? scan_account(o, f, 0, out) : 0;
}

/* execute_get_account_history (src/state_machine.zig:736-808, :1149-1196): only for
 * an existing account with flags.history (:759-761). */
uint32_t orc_get_account_history(orc_t* o, const tbgpu_account_filter_t* f, tbgpu_account_balance_t* out) {
    if (!filter_valid(f)) return 0;
    const tbgpu_account_t* a = get_account(o, G(f->account_id));
    if (!a || !(a->flags & TBGPU_ACCOUNT_HISTORY)) return 0;
    return scan_account(o, f, 1, out);
}
