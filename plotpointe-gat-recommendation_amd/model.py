"""Recommender models around the drop-in layers, same structure and state_dict keys
as the reference so checkpoints ({"state_dict", "config"}) load both ways:

``PyGGAT``    -- scripts/train_gat_pyg.py:68-88  (user_emb, item_proj, convs.{l})
``CustomGAT`` -- scripts/train_gat_custom.py:96-115 (user_emb, item_proj, layers.{l})

node_features = cat(user_emb.weight, item_proj(item_feats)); L stacked layers with no
nonlinearity in between (train_gat_pyg.py:86-87).
"""
from __future__ import annotations

import torch

from . import hip_ops
from .conv import GATConv, SimpleGATLayer


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
        x = self.node_features(item_feats)
        for conv in self.convs:
            x = conv(x, edge_index)
        return x


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
        x = self.node_features(item_feats)
        for gat in self.layers:
            x = gat(x, edge_index)
        return x


def bpr_loss(Z: torch.Tensor, n_users: int, u, i, j, loss: str = "bpr") -> torch.Tensor:
    """Loss of the train step, scripts/train_gat_pyg.py:313-322 (BPR or BCE), fused on the
    device (ppgat_bpr_fwd / ppgat_bpr_bwd)."""
    return hip_ops.bpr_loss(Z, n_users, u, i, j, loss)
