"""``torch.ops.ppgat.*``: the GAT layer's device ops in the PyTorch dispatcher.

``libppgat_torch.so`` (csrc/ppgat_torch.cpp) registers them with ``TORCH_LIBRARY(ppgat)``
over the C ABI of libppgat.so (include/ppgat.h), so torch.compile, TorchScript and C++
callers see them as ordinary operators:

    torch.ops.ppgat.csr_build(edge_index, n_nodes)
    torch.ops.ppgat.schedule_build(ptr, n_edges, max_edges=256)
    torch.ops.ppgat.node_scores(h, att_src, att_dst, heads, channels)
    torch.ops.ppgat.gat_fwd(h, s_src, s_dst, bias, col, csr_eid, <schedule>, sched, heads, channels,
                            mode, slope, dropout_p, seed, want_agg)
    torch.ops.ppgat.gat_bwd(...)

``load()`` loads the library once and registers fake (meta) implementations of the
shape-static ops for torch.compile's tracing.  ``schedule_args(sched)`` turns a
hip_ops.Schedule into the op's schedule arguments.
"""
from __future__ import annotations

from pathlib import Path

import torch

from . import _lib

LIB_PATH = Path(__file__).resolve().parent / "libppgat_torch.so"
_loaded = False


def load():
    """Load libppgat_torch.so (raises RuntimeError if it is missing) and register the fakes."""
    global _loaded
    if _loaded:
        return torch.ops.ppgat
    _lib.load()
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} not found; build it with make -C {LIB_PATH.parent / 'csrc'}")
    torch.ops.load_library(str(LIB_PATH))
    _register_fakes()
    _loaded = True
    return torch.ops.ppgat


def _register_fakes():
    @torch.library.register_fake("ppgat::node_scores")
    def _scores(h, att_src, att_dst, heads, channels):
        return h.new_empty(h.size(0), heads), h.new_empty(h.size(0), heads)

    @torch.library.register_fake("ppgat::gat_fwd")
    def _fwd(h, s_src, s_dst, bias, col, csr_eid, item_row, item_beg, item_end, hub_row, hub_ptr, sched, heads,
             channels, mode, slope, dropout_p, seed, want_agg):
        n = s_dst.size(0)
        agg = h.new_empty(n, heads, channels) if want_agg else h.new_empty(0)
        return (h.new_empty(n, channels), h.new_empty(n, heads), h.new_empty(n, heads), agg,
                h.new_empty(1, dtype=torch.int64))

    @torch.library.register_fake("ppgat::gat_bwd")
    def _bwd(h, s_src, s_dst, att_src, att_dst, bias, out, agg, m, inv_l, grad_out, rowptr, row, csc_eid, csc2csr,
             item_row, item_beg, item_end, hub_row, hub_ptr, sched, heads, channels, mode, slope, dropout_p, seed,
             seed_used, want_bias_grad):
        return (h.new_empty(h.size(0), heads * channels), h.new_empty(heads, channels), h.new_empty(heads, channels),
                h.new_empty(channels) if want_bias_grad else h.new_empty(0))


def schedule_args(sched):
    """(item_row, item_beg, item_end, hub_row, hub_ptr, [n_items, n_hub_items, n_hubs, n_long_items])"""
    return (sched.item_row, sched.item_beg, sched.item_end, sched.hub_row, sched.hub_ptr,
            [int(sched.n_items), int(sched.n_hub_items), int(sched.n_hubs), int(sched.n_long_items)])
