"""Consumers of the inference forward.

* ``eval_sampled``        -- scripts/train_gat_pyg.py:150-176 (identical custom :184-210):
  no-grad forward, 1 held-out positive + ``eval_neg_k`` rejection-sampled negatives per
  user, rank = #(score > positive's score) + 1, Recall@K / NDCG@K means.  The negatives
  are drawn with the reference's exact ``np.random`` call sequence (so a seeded run
  evaluates the same candidates); the scoring of all users is ONE device pass
  (``ppgat_sampled_rank``) instead of a GEMV + device->host sync per user.
  ``sampler=`` (a sampler.BPRSampler over the train lists) draws the candidates on the
  device too (``ppgat_eval_sample``: same rule, counter-based stream), so the whole
  evaluation is two kernels and one copy of the ranks; ``fast=True`` draws the same
  distribution with vectorised numpy (different stream).
* ``export_item_embeddings`` -- tools/export_item_embeddings.py:139-145.
* ``top_k_for_user_items`` / ``top_k_batch`` -- serving/runtime.py:56-76 on the device
  (``ppgat_serve_topk``): user vector = mean of history rows, history masked to -1e9,
  the k best descending with ties by smaller item index.
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, Sequence

import numpy as np
import torch

from . import _lib


def sample_eval_candidates(train_pos_idx: Dict[int, np.ndarray], eval_pos: Dict[int, int], n_items: int,
                           eval_neg_k: int):
    """The reference's candidate draw (train_gat_pyg.py:157-167), same np.random sequence."""
    user_pos_sets = {u: set(pos) for u, pos in train_pos_idx.items()}
    users = np.empty(len(eval_pos), np.int64)
    cands = np.empty((len(eval_pos), eval_neg_k + 1), np.int64)
    for t, (u, pos_i) in enumerate(eval_pos.items()):
        avoid = user_pos_sets.get(u, set()) | {pos_i}
        negs = []
        while len(negs) < eval_neg_k:
            cand = np.random.randint(0, n_items)
            if cand not in avoid:
                negs.append(cand)
        users[t] = u
        cands[t, 0] = pos_i
        cands[t, 1:] = negs
    return users, cands


def sample_eval_candidates_fast(train_pos_idx: Dict[int, np.ndarray], eval_pos: Dict[int, int], n_items: int,
                                eval_neg_k: int, seed: int = 0):
    """Same distribution (uniform over items not in train history + positive), vectorised."""
    rng = np.random.default_rng(seed)
    users = np.fromiter(eval_pos.keys(), np.int64, len(eval_pos))
    pos = np.fromiter(eval_pos.values(), np.int64, len(eval_pos))
    negs = rng.integers(0, n_items, (len(users), eval_neg_k))
    for _ in range(64):
        bad = negs == pos[:, None]
        for t, u in enumerate(users):
            hist = train_pos_idx.get(int(u))
            if hist is not None and len(hist):
                bad[t] |= np.isin(negs[t], hist)
        if not bad.any():
            break
        negs[bad] = rng.integers(0, n_items, int(bad.sum()))
    return users, np.concatenate([pos[:, None], negs], 1)


def sampled_rank(Z: torch.Tensor, n_users: int, users: np.ndarray, cands: np.ndarray, row_map=None) -> np.ndarray:
    """rank[b] = #(scores > positive score) + 1 for candidate lists (column 0 = positive)."""
    lib = _lib.load()
    if not Z.is_cuda or Z.dtype != torch.float32:
        raise RuntimeError("sampled_rank: fp32 ROCm tensor required (no CPU path)")
    Z = Z.contiguous()
    dev = Z.device
    n_rows, C = Z.shape
    n_items = (n_rows - n_users) if row_map is None else int(row_map.numel()) - n_users
    u = torch.as_tensor(users, dtype=torch.int64).to(dev).contiguous()
    c = torch.as_tensor(cands, dtype=torch.int64).to(dev).contiguous()
    rank = torch.empty(len(u), dtype=torch.int32, device=dev)
    _lib.check(lib.ppgat_sampled_rank(Z.data_ptr(), n_rows, n_users, n_items, _lib.ptr(row_map), C, u.data_ptr(),
                                      c.data_ptr(), len(u), c.size(1), rank.data_ptr(), _lib.stream_handle(dev)),
               "sampled_rank")
    return rank.cpu().numpy()


def metrics_from_ranks(ranks: np.ndarray, Ks: Sequence[int] = (10, 20)) -> Dict[str, float]:
    """train_gat_pyg.py:158-176 aggregation (key order recall@K..., ndcg@K...)."""
    metrics = {f"recall@{k}": [] for k in Ks}
    metrics.update({f"ndcg@{k}": [] for k in Ks})
    for r in ranks.tolist():
        for k in Ks:
            hit = 1.0 if r <= k else 0.0
            metrics[f"recall@{k}"].append(hit)
            metrics[f"ndcg@{k}"].append((1.0 / math.log2(r + 1)) if hit else 0.0)
    return {m: float(np.mean(v)) if v else 0.0 for m, v in metrics.items()}


def eval_sampled(model, cfg, item_feats: torch.Tensor, edge_index: torch.Tensor,
                 train_pos_idx: Dict[int, np.ndarray], eval_pos: Dict[int, int], Ks=(10, 20), fast: bool = False,
                 sampler=None, seed: int = 0):
    """Mirror of eval_sampled (train_gat_pyg.py:150-176); ``cfg.eval_neg_k`` negatives."""
    with torch.no_grad():
        Z = model(item_feats, edge_index)
    if sampler is not None:
        if not eval_pos:
            return metrics_from_ranks(np.zeros(0, np.int64), Ks)
        users = np.fromiter(eval_pos.keys(), np.int64, len(eval_pos))
        pos = np.fromiter(eval_pos.values(), np.int64, len(eval_pos))
        cands = sampler.eval_candidates(users, pos, cfg.eval_neg_k, seed)
        return metrics_from_ranks(sampled_rank(Z, model.n_users, users, cands), Ks)
    if fast:
        users, cands = sample_eval_candidates_fast(train_pos_idx, eval_pos, model.n_items, cfg.eval_neg_k)
    else:
        users, cands = sample_eval_candidates(train_pos_idx, eval_pos, model.n_items, cfg.eval_neg_k)
    if len(users) == 0:
        return metrics_from_ranks(np.zeros(0, np.int64), Ks)
    ranks = sampled_rank(Z, model.n_users, users, cands)
    return metrics_from_ranks(ranks, Ks)


def export_item_embeddings(model, item_feats: torch.Tensor, edge_index: torch.Tensor) -> np.ndarray:
    """tools/export_item_embeddings.py:139-142: eval-mode no-grad forward, items' rows."""
    model.eval()
    with torch.no_grad():
        Z = model(item_feats, edge_index)
        return Z[model.n_users:].detach().cpu().numpy().astype(np.float32)


def top_k_batch(item_vecs: torch.Tensor, histories: Sequence[Sequence[int]], k: int = 20):
    """serving/runtime.py:56-76 for a batch of users on the device (ppgat_serve_topk): per
    history, the mean of its rows, scores over every item, the history masked to -1e9, the
    k best descending (ties by smaller index).  Returns (indices [B, k] int64, scores [B, k])."""
    lib = _lib.load()
    if not item_vecs.is_cuda or item_vecs.dtype != torch.float32:
        raise RuntimeError("top_k_batch: fp32 ROCm item vectors required (no CPU path)")
    iv = item_vecs.contiguous()
    n_items, C = iv.shape
    dev = iv.device
    idx_out, sc_out = [], []
    for b0 in range(0, len(histories), 256):
        chunk = histories[b0:b0 + 256]
        for h in chunk:
            assert len(h) > 0, "Need at least one item id from user history"
        lens = np.array([len(h) for h in chunk], np.int64)
        ptr = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).to(dev)
        hist = torch.from_numpy(np.concatenate([np.asarray(h, np.int64) for h in chunk])).to(dev)
        B = len(chunk)
        nbytes = ctypes.c_size_t(0)
        _lib.check(lib.ppgat_serve_topk_workspace_bytes(n_items, C, B, ctypes.byref(nbytes)), "serve_topk_ws")
        ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev)
        oi = torch.empty(B, k, dtype=torch.int32, device=dev)
        os_ = torch.empty(B, k, dtype=torch.float32, device=dev)
        _lib.check(lib.ppgat_serve_topk(iv.data_ptr(), n_items, C, ptr.data_ptr(), hist.data_ptr(), int(lens.max()), B,
                                        int(k), oi.data_ptr(), os_.data_ptr(), ws.data_ptr(), nbytes.value,
                                        _lib.stream_handle(dev)), "serve_topk")
        idx_out.append(oi.long())
        sc_out.append(os_)
    return torch.cat(idx_out), torch.cat(sc_out)


def top_k_for_user_items(item_vecs: torch.Tensor, item_ids, k: int = 20):
    """serving/runtime.py:56-76 on the device: (indices, scores) of the top-k items for the
    mean of the history rows, history excluded, descending (ppgat_serve_topk)."""
    assert len(item_ids) > 0, "Need at least one item id from user history"
    idx, sc = top_k_batch(item_vecs, [list(item_ids)], k)
    return idx[0].cpu().numpy(), sc[0].cpu().numpy()
