"""BPR triple sampler (scripts/train_gat_pyg.py:179-190).

CPU: the oracle's counter stream (oracle/sampler_oracle.py) against the reference's sampling
rule -- the reference's own stream (data.sample_bpr_epoch, golden-pinned) and the exact
probabilities of the rule agree with the oracle's frequencies; range reduction checked
against Python integers.  GPU: ppgat_bpr_sample equals the oracle bit for bit (small ragged
graph with duplicates / empty users / a dense user, and the config-2 graph at the reference's
200k samples), draws are invariant to how an epoch is cut into calls, and the failure flags
raise."""
import random
from collections import Counter

import numpy as np
import pytest

from oracle import sampler_oracle as so

# user 1 has no items, user 2 has a duplicate, user 4 holds 11 of the 12 items
N_ITEMS = 12
LISTS = [[0, 5, 7], [], [3, 3, 9], [11], [i for i in range(N_ITEMS) if i != 6], [2, 4, 6, 8, 10]]


def _csr(lists):
    ptr = np.zeros(len(lists) + 1, dtype=np.int64)
    ptr[1:] = np.cumsum([len(x) for x in lists])
    items = np.array([v for x in lists for v in x], dtype=np.int64)
    return ptr, items


def _rule_probs(lists, n_items):
    """Exact probabilities of the reference's rule: P(u), P(i | u), P(j | u)."""
    elig = [u for u, x in enumerate(lists) if x]
    pu = {u: 1 / len(elig) for u in elig}
    pi = {(u, i): c / len(lists[u]) for u in elig for i, c in Counter(lists[u]).items()}
    pj = {(u, j): 1 / (n_items - len(set(lists[u]))) for u in elig for j in range(n_items) if j not in set(lists[u])}
    return pu, pi, pj


def _freqs(u, i, j):
    S = len(u)
    fu = Counter(u.tolist())
    fi = Counter(zip(u.tolist(), i.tolist()))
    fj = Counter(zip(u.tolist(), j.tolist()))
    return ({k: v / S for k, v in fu.items()}, {k: v / fu[k[0]] for k, v in fi.items()},
            {k: v / fu[k[0]] for k, v in fj.items()})


def _max_dev(freq, prob):
    keys = set(freq) | set(prob)
    return max(abs(freq.get(k, 0.0) - prob.get(k, 0.0)) for k in keys)


def test_oracle_and_reference_stream_follow_the_rule(pkg):
    S = 60_000
    pu, pi, pj = _rule_probs(LISTS, N_ITEMS)
    ptr, items = _csr(LISTS)
    u, i, j, bad = so.bpr_sample(ptr, items, N_ITEMS, S, seed=3)
    assert bad == 0
    random.seed(0)
    tr = {uu: np.array(x) for uu, x in enumerate(LISTS) if x}
    ru, ri, rj = pkg.data.sample_bpr_epoch(tr, N_ITEMS, S)
    # conditional frequencies over ~12k draws per user: 5-sigma ~ 0.02
    for fr in (_freqs(u, i, j), _freqs(ru, ri, rj)):
        assert _max_dev(fr[0], pu) < 0.01
        assert _max_dev(fr[1], pi) < 0.02
        assert _max_dev(fr[2], pj) < 0.02
    # no sample ever violates the rule
    for uu, ii, jj in zip(u.tolist(), i.tolist(), j.tolist()):
        assert ii in LISTS[uu] and jj not in LISTS[uu] and 0 <= jj < N_ITEMS


def test_oracle_offset_invariance():
    ptr, items = _csr(LISTS)
    a = so.bpr_sample(ptr, items, N_ITEMS, 1000, seed=9)
    b = so.bpr_sample(ptr, items, N_ITEMS, 400, seed=9, t0=600)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x[600:], y)


def test_oracle_range_reduction_exact():
    rng = np.random.default_rng(0)
    r = rng.integers(0, 2**63, 2000, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, 2000, dtype=np.uint64)
    for n in (1, 7, 63_001, 2**31 - 1, 5_000_000):
        got = so.below(r, n)
        ref = np.array([(int(x) * n) >> 64 for x in r], dtype=np.int64)
        assert np.array_equal(got, ref)
    # draw64 against Python integers mod 2^64
    M = (1 << 64) - 1

    def ref_draw(seed, t, k):
        z = (seed + (t + 1) * 0x9E3779B97F4A7C15) & M
        z ^= ((k + 1) * 0xD1B54A32D192ED03) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)
    t = np.array([0, 1, 2, 12345, 2**40 + 7], dtype=np.uint64)
    for seed in (0, 42, 2**64 - 1):
        for k in (0, 1, 2, 1000):
            assert [int(x) for x in so.draw64(seed, t, k)] == [ref_draw(seed, int(x), k) for x in t]


def test_oracle_flags():
    ptr, items = _csr([[], []])
    assert so.bpr_sample(ptr, items, 5, 10, seed=1)[3] == 1
    ptr, items = _csr([[0, 1, 2]])
    assert so.bpr_sample(ptr, items, 3, 10, seed=1)[3] == 2


# ---------------------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 42, 2**64 - 5])
def test_gpu_small_equals_oracle(pkg, cuda, seed):
    import torch
    ptr, items = _csr(LISTS)
    smp = pkg.sampler.BPRSampler(torch.from_numpy(ptr), torch.from_numpy(items), N_ITEMS, device=cuda)
    u, i, j = smp.sample(50_000, seed=seed)
    ou, oi, oj, bad = so.bpr_sample(ptr, items, N_ITEMS, 50_000, seed=seed)
    assert bad == 0
    assert np.array_equal(u.cpu().numpy(), ou)
    assert np.array_equal(i.cpu().numpy(), oi)
    assert np.array_equal(j.cpu().numpy(), oj)


@pytest.mark.gpu
def test_gpu_config2_equals_oracle(pkg, cuda):
    """Config 2's U-I graph, the reference's 200k samples per epoch (train_gat_pyg.py:300)."""
    g = pkg.data.synthetic_ui_graph()
    smp = pkg.sampler.BPRSampler(g.user_ptr, g.user_items, g.n_items, device=cuda)
    u, i, j = (t.cpu().numpy() for t in smp.sample(200_000, seed=42))
    ou, oi, oj, bad = so.bpr_sample(g.user_ptr, g.user_items, g.n_items, 200_000, seed=42)
    assert bad == 0
    assert np.array_equal(u, ou) and np.array_equal(i, oi) and np.array_equal(j, oj)
    # properties straight from the rule
    key = np.repeat(np.arange(g.n_users), np.diff(g.user_ptr)) * g.n_items + g.user_items
    key.sort()
    assert np.all(np.isin(u * g.n_items + i, key))
    assert not np.any(np.isin(u * g.n_items + j, key))
    assert j.min() >= 0 and j.max() < g.n_items


@pytest.mark.gpu
def test_gpu_epoch_in_pieces(pkg, cuda):
    import torch
    g = pkg.data.synthetic_ui_graph(n_users=3000, n_items=800, n_interactions=40_000, seed=5)
    smp = pkg.sampler.BPRSampler(g.user_ptr, g.user_items, g.n_items, device=cuda)
    whole = torch.stack(smp.sample(10_000, seed=7))
    parts = torch.cat([torch.stack(smp.sample(n, seed=7, offset=o)) for o, n in ((0, 3333), (3333, 1), (3334, 6666))],
                      dim=1)
    assert torch.equal(whole, parts)
    again = torch.stack(smp.sample(10_000, seed=7))
    assert torch.equal(whole, again)


@pytest.mark.gpu
def test_gpu_flags_raise(pkg, cuda):
    import torch
    ptr, items = _csr([[], []])
    with pytest.raises(ValueError, match="no user"):
        pkg.sampler.BPRSampler(torch.from_numpy(ptr), torch.from_numpy(items), 5, device=cuda).sample(10)
    ptr, items = _csr([[0, 1, 2], [1]])
    smp = pkg.sampler.BPRSampler(torch.from_numpy(ptr), torch.from_numpy(items), 3, device=cuda)
    with pytest.raises(ValueError, match="every item"):
        smp.sample(100, seed=1)
    assert smp.sample(0)[0].numel() == 0


# ---------------------------------------------------------------------------
# eval_sampled candidates (scripts/train_gat_pyg.py:157-167; ppgat_eval_sample)
# ---------------------------------------------------------------------------
def _eval_rule_probs(lists, users, pos, n_items):
    """P(negative = c | row b): uniform over items outside train(u) and != pos."""
    out = []
    for u, p in zip(users, pos):
        allowed = [c for c in range(n_items) if c not in set(lists[u]) and c != p]
        out.append({c: 1 / len(allowed) for c in allowed})
    return out


def test_eval_candidates_oracle_and_reference_stream_follow_the_rule(pkg):
    """The oracle's eval negatives and the reference's own np.random draw
    (evaluation.sample_eval_candidates, the reference's call sequence) both follow the rule."""
    ev = pkg.evaluation
    lists = [[0, 5, 7], [], [3, 3, 9], [11], [2, 4, 6, 8, 10]]
    users = np.array([0, 1, 2, 3, 4])
    pos = np.array([1, 2, 4, 0, 3])
    n_neg = 20_000
    probs = _eval_rule_probs(lists, users, pos, N_ITEMS)
    ptr, items = _csr(lists)
    cands, bad = so.eval_sample(ptr, items, users, pos, N_ITEMS, n_neg, seed=11)
    assert bad == 0 and cands.shape == (5, n_neg + 1)
    assert np.array_equal(cands[:, 0], pos)
    np.random.seed(0)
    tr = {uu: np.array(x) for uu, x in enumerate(lists) if x}
    _, ref = ev.sample_eval_candidates(tr, dict(zip(users.tolist(), pos.tolist())), N_ITEMS, n_neg)
    for b in range(5):
        for arr in (cands[b, 1:], ref[b, 1:]):
            f = Counter(arr.tolist())
            assert set(f) <= set(probs[b])  # never a train item nor the positive
            assert max(abs(f.get(c, 0) / n_neg - p) for c, p in probs[b].items()) < 0.012


@pytest.mark.gpu
def test_eval_candidates_gpu_bit_exact(pkg, cuda):
    import torch
    rng = np.random.default_rng(4)
    n_users, n_items = 3000, 900
    lens = rng.integers(0, 30, n_users)
    lens[7] = 0
    lists = [rng.choice(n_items, int(k), replace=True).tolist() for k in lens]
    ptr, items = _csr(lists)
    users = rng.permutation(n_users)[:2000]
    pos = rng.integers(0, n_items, 2000)
    s = pkg.sampler.BPRSampler(ptr, items, n_items, device=cuda)
    got = s.eval_candidates(torch.from_numpy(users), torch.from_numpy(pos), 100, seed=77).cpu().numpy()
    ref, bad = so.eval_sample(ptr, items, users, pos, n_items, 100, seed=77)
    assert bad == 0
    assert np.array_equal(got, ref)
