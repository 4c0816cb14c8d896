"""Recommender models around the drop-in layers, same structure and state_dict keys
as the reference so checkpoints ({"state_dict", "config"}) load both ways:

``PyGGAT``    -- scripts/train_gat_pyg.py:68-88  (user_emb, item_proj, convs.{l})
``CustomGAT`` -- scripts/train_gat_custom.py:96-115 (user_emb, item_proj, layers.{l})

node_features = cat(user_emb.weight, item_proj(item_feats)); L stacked layers with no
nonlinearity in between (train_gat_pyg.py:86-87).  forward() hands the two row blocks to
the first layer separately (``forward_segments``), so the concatenation is never
materialised; ``node_features`` still returns it for callers that want it.  The two blocks
live back to back in one node table (``node_table``: the user embedding's storage is its
first rows, the item projection writes the rest), so a layer that does need them as one
tensor (the aggregate-then-transform layer of config 5) gets it without a copy.
"""
from __future__ import annotations

import os

import torch

from . import hip_ops
from .conv import GATConv, SimpleGATLayer


def node_table(model: torch.nn.Module, n_items: int) -> torch.Tensor:
    """[n_users + n_items, hidden]: rows [0, n_users) ARE model.user_emb.weight's storage
    (re-pointed here once, values kept; optimisers hold the same Parameter object), rows
    [n_users, N) take the item projection each forward.  Rebuilt if the weight moved (.to(),
    a new device) or the item count changed."""
    w = model.user_emb.weight
    t = getattr(model, "_node_rows", None)
    if (t is None or t.device != w.device or t.dtype != w.dtype or t.shape != (w.size(0) + n_items, w.size(1))
            or w.data_ptr() != t.data_ptr()):
        t = torch.empty(w.size(0) + n_items, w.size(1), dtype=w.dtype, device=w.device)
        t[:w.size(0)].copy_(w.detach())
        w.data = t[:w.size(0)]
        model._node_rows = t
    return t


class _TableGuard(torch.autograd.Function):
    """Identity on the node table's item rows, whose backward checks that no later forward
    rewrote them.  The item projection writes them through a raw pointer each forward (no
    version-counter bump: a bump would trip autograd's view checks on the table's views), so a
    graph whose backward runs after another forward -- its layers saved those rows -- would
    otherwise take the new rows' values silently; here it raises instead.  (One forward in
    flight per model: the node table is a per-model buffer.)"""

    @staticmethod
    def forward(ctx, v, holder, gen: int):
        ctx.holder, ctx.gen = holder, gen
        return v.view_as(v)

    @staticmethod
    def backward(ctx, g):
        if ctx.holder[0]._node_rows_gen != ctx.gen:
            raise RuntimeError("ppgat node table: the item rows this graph saved were rewritten by a later "
                               "forward of the same model; run backward before the next forward "
                               "(or PPGAT_NODE_TABLE=0)")
        return g, None, None


def _unalias_state(module, state_dict, prefix, local_metadata):
    """state_dict hook: the user embedding shares the node table's storage; hand out its own copy
    (torch.save would otherwise write the whole table)."""
    k = prefix + "user_emb.weight"
    v = state_dict.get(k)
    if v is not None and v.untyped_storage().nbytes() > v.numel() * v.element_size():
        state_dict[k] = v.clone()


def _stack(model, item_proj, item_feats, layers, edge_index):
    user_w = model.user_emb.weight
    if user_w.is_cuda and os.environ.get("PPGAT_NODE_TABLE", "1") != "0":
        table = node_table(model, item_feats.size(0))
        v = hip_ops.linear(item_feats, item_proj.weight, item_proj.bias, out=table[user_w.size(0):])
        gen = getattr(model, "_node_rows_gen", 0) + 1
        model._node_rows_gen = gen
        if torch.is_grad_enabled() and v.requires_grad:
            v = _TableGuard.apply(v, [model], gen)
    else:
        v = hip_ops.linear(item_feats, item_proj.weight, item_proj.bias)
    if len(layers) == 0:
        return torch.cat([user_w, v], dim=0)
    x = layers[0].forward_segments(user_w, v, edge_index)
    for layer in list(layers)[1:]:
        x = layer(x, edge_index)
    return x


class PyGGAT(torch.nn.Module):
    def __init__(self, n_users: int, n_items: int, item_feat_dim: int, hidden: int, layers: int, heads: int,
                 attn_dropout: float):
        super().__init__()
        self.n_users, self.n_items = n_users, n_items
        self.user_emb = torch.nn.Embedding(n_users, hidden)
        torch.nn.init.normal_(self.user_emb.weight, std=0.1)
        self.item_proj = torch.nn.Linear(item_feat_dim, hidden)
        self.convs = torch.nn.ModuleList()
        for _ in range(layers):
            self.convs.append(GATConv(hidden, hidden, heads=heads, dropout=attn_dropout, add_self_loops=False,
                                      concat=False))
        self._register_state_dict_hook(_unalias_state)

    def node_features(self, item_feats: torch.Tensor) -> torch.Tensor:
        u = self.user_emb.weight
        v = hip_ops.linear(item_feats, self.item_proj.weight, self.item_proj.bias)
        return torch.cat([u, v], dim=0)

    def forward(self, item_feats: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        return _stack(self, self.item_proj, item_feats, self.convs, edge_index)


class CustomGAT(torch.nn.Module):
    def __init__(self, n_users: int, n_items: int, item_feat_dim: int, hidden: int, layers: int):
        super().__init__()
        self.n_users, self.n_items = n_users, n_items
        self.user_emb = torch.nn.Embedding(n_users, hidden)
        torch.nn.init.normal_(self.user_emb.weight, std=0.1)
        self.item_proj = torch.nn.Linear(item_feat_dim, hidden)
        self.layers = torch.nn.ModuleList([SimpleGATLayer(hidden, hidden) for _ in range(layers)])
        self._register_state_dict_hook(_unalias_state)

    def node_features(self, item_feats: torch.Tensor) -> torch.Tensor:
        u = self.user_emb.weight
        v = hip_ops.linear(item_feats, self.item_proj.weight, self.item_proj.bias)
        return torch.cat([u, v], dim=0)

    def forward(self, item_feats: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        return _stack(self, self.item_proj, item_feats, self.layers, edge_index)


def bpr_loss(Z: torch.Tensor, n_users: int, u, i, j, loss: str = "bpr", prepared=None) -> torch.Tensor:
    """Loss of the train step, scripts/train_gat_pyg.py:313-322 (BPR or BCE), fused on the
    device (ppgat_bpr_fwd / ppgat_bpr_bwd; with ``prepared`` from ``hip_ops.bpr_prepare`` the
    backward's triple sort has already run beside the forward)."""
    return hip_ops.bpr_loss(Z, n_users, u, i, j, loss, prepared=prepared)
