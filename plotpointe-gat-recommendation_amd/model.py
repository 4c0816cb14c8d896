"""Recommender models around the drop-in layers, same structure and state_dict keys
as the reference so checkpoints ({"state_dict", "config"}) load both ways:

``PyGGAT``    -- scripts/train_gat_pyg.py:68-88  (user_emb, item_proj, convs.{l})
``CustomGAT`` -- scripts/train_gat_custom.py:96-115 (user_emb, item_proj, layers.{l})

node_features = cat(user_emb.weight, item_proj(item_feats)); L stacked layers with no
nonlinearity in between (train_gat_pyg.py:86-87).  forward() hands the two row blocks to
the first layer separately (``forward_segments``), so the concatenation is never
materialised; ``node_features`` still returns it for callers that want it.
"""
from __future__ import annotations

import torch

from . import hip_ops
from .conv import GATConv, SimpleGATLayer


def _stack(user_w, item_proj, item_feats, layers, edge_index):
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

    def node_features(self, item_feats: torch.Tensor) -> torch.Tensor:
        u = self.user_emb.weight
        v = hip_ops.linear(item_feats, self.item_proj.weight, self.item_proj.bias)
        return torch.cat([u, v], dim=0)

    def forward(self, item_feats: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        return _stack(self.user_emb.weight, self.item_proj, item_feats, self.convs, edge_index)


class CustomGAT(torch.nn.Module):
    def __init__(self, n_users: int, n_items: int, item_feat_dim: int, hidden: int, layers: int):
        super().__init__()
        self.n_users, self.n_items = n_users, n_items
        self.user_emb = torch.nn.Embedding(n_users, hidden)
        torch.nn.init.normal_(self.user_emb.weight, std=0.1)
        self.item_proj = torch.nn.Linear(item_feat_dim, hidden)
        self.layers = torch.nn.ModuleList([SimpleGATLayer(hidden, hidden) for _ in range(layers)])

    def node_features(self, item_feats: torch.Tensor) -> torch.Tensor:
        u = self.user_emb.weight
        v = hip_ops.linear(item_feats, self.item_proj.weight, self.item_proj.bias)
        return torch.cat([u, v], dim=0)

    def forward(self, item_feats: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        return _stack(self.user_emb.weight, self.item_proj, item_feats, self.layers, edge_index)


def bpr_loss(Z: torch.Tensor, n_users: int, u, i, j, loss: str = "bpr", prepared=None) -> torch.Tensor:
    """Loss of the train step, scripts/train_gat_pyg.py:313-322 (BPR or BCE), fused on the
    device (ppgat_bpr_fwd / ppgat_bpr_bwd; with ``prepared`` from ``hip_ops.bpr_prepare`` the
    backward's triple sort has already run beside the forward)."""
    return hip_ops.bpr_loss(Z, n_users, u, i, j, loss, prepared=prepared)
