"""Drop-in GAT layers backed by the fused HIP kernels.

``GATConv``        -- torch_geometric.nn.GATConv as the reference constructs it
                      (scripts/train_gat_pyg.py:77: heads=H, dropout=p,
                      add_self_loops=False, concat=False); same constructor names,
                      ``forward(x, edge_index)``, and state_dict keys
                      (``lin.weight`` [H*C, F], ``att_src``/``att_dst`` [1, H, C],
                      ``bias`` [C]; the older ``lin_src.weight``/``lin_dst.weight`` keys load too).
``SimpleGATLayer`` -- scripts/train_gat_custom.py:63-93, same constructor
                      ``(in_dim, out_dim, attn_dropout=0.1)``, same parameter creation
                      order (so a seeded construction yields the reference's weights)
                      and keys (``lin.weight``, ``a_src``, ``a_dst``).

Both run the layer as ``hip_ops.gat_layer``, entirely in ``libppgat.so``: ``h = lin(x)``
on the fp32 matrix cores with the node attention terms in the GEMM epilogue, the fused
edge kernels, and a backward that folds the attention terms into the projection GEMMs;
multi-head layers wider than their input (config 5) run aggregate-then-transform
(``hip_ops.GATLayerX``: x_j gathered once per edge, one transform GEMM).  Dropout on alpha is the counter-hash mask of
include/ppgat.h, drawn fresh per training forward from torch's CPU generator.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from .hip_ops import gat_layer, graph_cache


def _dropout_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def _glorot_(t: torch.Tensor):
    """PyG inits.glorot: U(+-sqrt(6 / (size(-2) + size(-1))))."""
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)
    return t


class GATConv(torch.nn.Module):
    """MI355X-native ``GATConv`` (PyG semantics)."""

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 negative_slope: float = 0.2, dropout: float = 0.0, add_self_loops: bool = True,
                 edge_dim=None, fill_value="mean", bias: bool = True, residual: bool = False, **kwargs):
        super().__init__()
        if isinstance(in_channels, (tuple, list)):
            raise NotImplementedError("bipartite (tuple) in_channels not implemented")
        if concat:
            raise NotImplementedError("GATConv(concat=True) not implemented; the reference uses concat=False")
        if add_self_loops:
            raise NotImplementedError("GATConv(add_self_loops=True) not implemented; the reference passes False")
        if edge_dim is not None:
            raise NotImplementedError("edge_dim (edge features) not implemented")
        if residual:
            raise NotImplementedError("residual=True not implemented")
        if not _lib.load().ppgat_supported_channels(int(out_channels)):
            raise NotImplementedError(f"out_channels={out_channels}: fused kernels take C in 4*2^k <= 256")
        if heads > 8:
            raise NotImplementedError("heads > 8 not implemented")
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.dropout = concat, negative_slope, dropout
        self.add_self_loops = add_self_loops
        self.lin = torch.nn.Linear(in_channels, heads * out_channels, bias=False)
        self.att_src = torch.nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = torch.nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = torch.nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        _glorot_(self.lin.weight)
        _glorot_(self.att_src)
        _glorot_(self.att_dst)
        if self.bias is not None:
            torch.nn.init.zeros_(self.bias)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        # older PyG: lin_src / lin_dst share one weight (in_channels is an int)
        old = prefix + "lin_src.weight"
        if old in state_dict and prefix + "lin.weight" not in state_dict:
            state_dict[prefix + "lin.weight"] = state_dict.pop(old)
            state_dict.pop(prefix + "lin_dst.weight", None)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, return_attention_weights=None) -> torch.Tensor:
        if return_attention_weights:
            raise NotImplementedError("return_attention_weights not implemented")
        graph = graph_cache.get(edge_index, x.size(0))
        p = float(self.dropout) if self.training else 0.0
        seed = _dropout_seed() if p > 0 else 0
        return gat_layer(x, self.lin.weight, self.att_src, self.att_dst, self.bias, graph, self.heads,
                         self.out_channels, _lib.MODE_PYG, float(self.negative_slope), p, seed)

    def forward_segments(self, x: torch.Tensor, x_items: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        """forward(cat(x, x_items), edge_index) without materialising the concatenation
        (the model's node features, train_gat_pyg.py:79-82)."""
        graph = graph_cache.get(edge_index, x.size(0) + x_items.size(0))
        p = float(self.dropout) if self.training else 0.0
        seed = _dropout_seed() if p > 0 else 0
        return gat_layer(x, self.lin.weight, self.att_src, self.att_dst, self.bias, graph, self.heads,
                         self.out_channels, _lib.MODE_PYG, float(self.negative_slope), p, seed, x_items=x_items)

    def __repr__(self):
        return (f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, heads={self.heads}, "
                f"backend=hip)")


class SimpleGATLayer(torch.nn.Module):
    """MI355X-native ``SimpleGATLayer`` (scripts/train_gat_custom.py:63-93)."""

    def __init__(self, in_dim: int, out_dim: int, attn_dropout: float = 0.1):
        super().__init__()
        if not _lib.load().ppgat_supported_channels(int(out_dim)):
            raise NotImplementedError(f"out_dim={out_dim}: fused kernels take C in 4*2^k <= 256")
        # creation/initialisation order identical to the reference (RNG-consuming calls)
        self.lin = torch.nn.Linear(in_dim, out_dim, bias=False)
        self.a_src = torch.nn.Parameter(torch.empty(out_dim))
        self.a_dst = torch.nn.Parameter(torch.empty(out_dim))
        torch.nn.init.xavier_uniform_(self.lin.weight)
        torch.nn.init.xavier_uniform_(self.a_src.unsqueeze(0))
        torch.nn.init.xavier_uniform_(self.a_dst.unsqueeze(0))
        self.leaky = torch.nn.LeakyReLU(0.2)
        self.drop = torch.nn.Dropout(attn_dropout)
        self.out_dim = out_dim

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        graph = graph_cache.get(edge_index, x.size(0))
        p = float(self.drop.p) if self.training else 0.0
        seed = _dropout_seed() if p > 0 else 0
        return gat_layer(x, self.lin.weight, self.a_src, self.a_dst, None, graph, 1, self.out_dim, _lib.MODE_CUSTOM,
                         float(self.leaky.negative_slope), p, seed)

    def forward_segments(self, x: torch.Tensor, x_items: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        """forward(cat(x, x_items), edge_index) without materialising the concatenation."""
        graph = graph_cache.get(edge_index, x.size(0) + x_items.size(0))
        p = float(self.drop.p) if self.training else 0.0
        seed = _dropout_seed() if p > 0 else 0
        return gat_layer(x, self.lin.weight, self.a_src, self.a_dst, None, graph, 1, self.out_dim, _lib.MODE_CUSTOM,
                         float(self.leaky.negative_slope), p, seed, x_items=x_items)
