"""CPU ORACLE -- test infrastructure only (same rules as oracle/gat_oracle.py: imported by
tests/ and tools' CPU baselines only, never by the product package).

``bpr_sample`` restates libppgat's BPR triple sampler (csrc/ppgat_sample.hip) in numpy,
bit for bit: the counter-based stream (splitmix64 finaliser over (seed, t, draw)), the
128-bit multiply-high range reduction and the rejection of negatives that are positives.
The sampling RULE it implements is the reference's sample_bpr_epoch
(scripts/train_gat_pyg.py:179-190): u uniform over users with >= 1 train item
(``random.choice(users)``, :183), i uniform over the positions of u's train list
(``random.choice(train_pos_idx[u])``, :184), j ~ randrange(n_items) redrawn while j is a
positive of u (:185-188).  The reference's stream is Python's Mersenne twister, so triples
are not comparable one to one; the distribution is, and tests/test_sampler.py checks it
against ``data.sample_bpr_epoch`` (which reproduces the reference's exact stream and is
itself pinned by tests/golden/config1_plumbing.npz).
"""
from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
M32 = np.uint64(0xFFFFFFFF)
MAX_NEG_DRAWS = 1024


def _u64(x):
    return np.asarray(x, dtype=np.uint64)


def draw64(seed: int, t: np.ndarray, k: int) -> np.ndarray:
    """csrc/ppgat_sample.hip draw64 (uint64 arithmetic wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        z = _u64(seed) + (_u64(t) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z ^= np.uint64((k + 1) * 0xD1B54A32D192ED03 & 0xFFFFFFFFFFFFFFFF)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def below(r: np.ndarray, n) -> np.ndarray:
    """High 64 bits of r * n (__umul64hi), i.e. floor(r * n / 2^64)."""
    r = _u64(r)
    n = _u64(n)
    a_lo, a_hi = r & M32, r >> np.uint64(32)
    b_lo, b_hi = n & M32, n >> np.uint64(32)
    p0, p1, p2, p3 = a_lo * b_lo, a_lo * b_hi, a_hi * b_lo, a_hi * b_hi
    mid = (p0 >> np.uint64(32)) + (p1 & M32) + (p2 & M32)
    return (p3 + (p1 >> np.uint64(32)) + (p2 >> np.uint64(32)) + (mid >> np.uint64(32))).astype(np.int64)


def prepare(user_ptr: np.ndarray, user_items: np.ndarray):
    """Each user's items ascending + the users that have items (ppgat_bpr_sampler_prepare)."""
    user_ptr = np.asarray(user_ptr, dtype=np.int64)
    items = np.asarray(user_items, dtype=np.int64)
    deg = np.diff(user_ptr)
    owner = np.repeat(np.arange(len(deg), dtype=np.int64), deg)
    order = np.lexsort((items, owner))
    return items[order], np.flatnonzero(deg > 0).astype(np.int64)


def bpr_sample(user_ptr: np.ndarray, user_items: np.ndarray, n_items: int, S: int, seed: int, t0: int = 0):
    """-> (u, i, j, bad) exactly as ppgat_bpr_sample writes them."""
    user_ptr = np.asarray(user_ptr, dtype=np.int64)
    items_sorted, eligible = prepare(user_ptr, user_items)
    t = np.arange(t0, t0 + S, dtype=np.uint64)
    if len(eligible) == 0 or n_items <= 0:
        z = np.zeros(S, dtype=np.int64)
        return z, z.copy(), z.copy(), (1 if S > 0 else 0)
    u = eligible[below(draw64(seed, t, 0), len(eligible))]
    lo, hi = user_ptr[u], user_ptr[u + 1]
    i = items_sorted[lo + below(draw64(seed, t, 1), hi - lo)]
    # membership by searching the (user, item) key in the sorted key array
    owner = np.repeat(np.arange(len(user_ptr) - 1, dtype=np.int64), np.diff(user_ptr))
    keys = owner * np.int64(n_items) + items_sorted
    j = np.full(S, -1, dtype=np.int64)
    open_ = np.arange(S)
    for k in range(MAX_NEG_DRAWS):
        if open_.size == 0:
            break
        c = below(draw64(seed, t[open_], 2 + k), n_items)
        q = u[open_] * np.int64(n_items) + c
        pos = np.minimum(np.searchsorted(keys, q), max(len(keys) - 1, 0))
        hit = keys[pos] == q if len(keys) else np.zeros(len(q), dtype=bool)
        j[open_[~hit]] = c[~hit]
        open_ = open_[hit]
    bad = 0
    if open_.size:
        j[open_] = 0
        bad = 2
    return u, i.astype(np.int64), j, bad


def eval_sample(user_ptr: np.ndarray, user_items: np.ndarray, users: np.ndarray, pos: np.ndarray, n_items: int,
                n_neg: int, seed: int):
    """ppgat_eval_sample restated (csrc/ppgat_sample.hip k_eval_sample) -> (cands [B, n_neg+1], bad).
    Rule of eval_sampled (scripts/train_gat_pyg.py:157-167): negatives uniform over the items
    outside the user's train list and != the held-out positive, drawn independently."""
    user_ptr = np.asarray(user_ptr, dtype=np.int64)
    items_sorted, _ = prepare(user_ptr, user_items)
    users = np.asarray(users, np.int64)
    pos = np.asarray(pos, np.int64)
    B = len(users)
    owner = np.repeat(np.arange(len(user_ptr) - 1, dtype=np.int64), np.diff(user_ptr))
    keys = owner * np.int64(n_items) + items_sorted
    t = (np.arange(B, dtype=np.int64)[:, None] * n_neg + np.arange(n_neg, dtype=np.int64)[None, :]).reshape(-1)
    ub = np.repeat(users, n_neg)
    pb = np.repeat(pos, n_neg)
    neg = np.full(B * n_neg, -1, np.int64)
    open_ = np.arange(B * n_neg)
    for d in range(MAX_NEG_DRAWS):
        if open_.size == 0:
            break
        c = below(draw64(seed, t[open_].astype(np.uint64), d), n_items)
        q = ub[open_] * np.int64(n_items) + c
        ix = np.minimum(np.searchsorted(keys, q), max(len(keys) - 1, 0))
        hit = (keys[ix] == q) if len(keys) else np.zeros(len(q), dtype=bool)
        hit |= c == pb[open_]
        neg[open_[~hit]] = c[~hit]
        open_ = open_[hit]
    bad = 0
    if open_.size:
        neg[open_] = 0
        bad = 2
    return np.concatenate([pos[:, None], neg.reshape(B, n_neg)], 1), bad
