"""CPU ORACLE -- test infrastructure only (same rules as oracle/gat_oracle.py: imported by
tests/ and tools' CPU baselines only, never by the product package).

``ii_knn`` restates the I-I kNN build of graphs/build_ii_knn.py:56-99 with the same
libraries the reference uses (numpy + sklearn.metrics.pairwise.cosine_similarity):
  rows L2-normalised as embeddings / (norm + 1e-8)              (:57-59)
  per batch: cosine_similarity(batch, all) (sklearn normalises both again),
  self similarity -> -inf, argpartition top-k, sorted descending (:76-90),
  kept where sim >= min_similarity (:93-95), appended in item order (:98-101).
Pinned against the reference itself: tests/golden/knn_small.npz is the output of
build_ii_knn.py main() run by tests/golden/make_golden.py (tests/test_knn.py).
"""
from __future__ import annotations

import numpy as np


def ii_knn(embeddings: np.ndarray, k: int = 20, min_similarity: float = 0.3, batch_size: int = 1000):
    from sklearn.metrics.pairwise import cosine_similarity

    emb = np.asarray(embeddings)
    n = emb.shape[0]
    norms = np.linalg.norm(emb, axis=1, keepdims=True)
    en = emb / (norms + 1e-8)
    rows, cols, sims = [], [], []
    for s0 in range(0, n, batch_size):
        s1 = min(s0 + batch_size, n)
        sim = cosine_similarity(en[s0:s1], en)
        for i, item in enumerate(range(s0, s1)):
            v = sim[i]
            v[item] = -np.inf
            top = np.argpartition(v, -k)[-k:]
            top = top[np.argsort(v[top])[::-1]]
            tv = v[top]
            keep = tv >= min_similarity
            rows.extend([item] * int(keep.sum()))
            cols.extend(top[keep])
            sims.extend(tv[keep])
    return (np.asarray(rows, np.int32), np.asarray(cols, np.int32), np.asarray(sims, np.float32))
