"""torch.ops.ppgat.* (TORCH_LIBRARY registration, csrc/ppgat_torch.cpp) -- CPU: the library
loads and registers every op with its schema and refuses CPU tensors; GPU: each op returns
exactly what the ctypes path returns (same kernels), and the ops trace through torch.compile
(fake implementations) and TorchScript."""
import importlib

import numpy as np
import pytest
import torch


def _tops():
    return importlib.import_module("plotpointe-gat-recommendation_amd.torch_ops")


def test_ops_registered_with_schemas(pkg):
    ops = _tops().load()
    for name in ("csr_build", "schedule_build", "node_scores", "gat_fwd", "gat_bwd"):
        assert getattr(ops, name).default._schema.name == f"ppgat::{name}"
    # only a CUDA (= HIP) kernel is registered: the dispatcher refuses CPU tensors (no CPU path)
    with pytest.raises(NotImplementedError, match="CPU"):
        ops.node_scores(torch.zeros(4, 8), torch.zeros(1, 8), torch.zeros(1, 8), 1, 8)


def _graph_inputs(cuda, n=900, e=9000, C=128, H=1, seed=0):
    rng = np.random.default_rng(seed)
    ei = torch.from_numpy(np.stack([rng.integers(0, n, e), rng.integers(0, n, e)]).astype(np.int64)).to(cuda)
    h = torch.randn(n, H * C, device=cuda)
    a_s = torch.randn(H, C, device=cuda) * 0.1
    a_d = torch.randn(H, C, device=cuda) * 0.1
    return ei, h, a_s, a_d


@pytest.mark.gpu
@pytest.mark.parametrize("H,C", [(1, 128), (2, 64)])
def test_ops_equal_ctypes_path(pkg, cuda, H, C):
    tops = _tops()
    ops = tops.load()
    ho = pkg.hip_ops
    ei, h, a_s, a_d = _graph_inputs(cuda, C=C, H=H)
    n = h.size(0)
    bias = torch.randn(C, device=cuda) * 0.1
    g = ho.csr_build(ei, n)
    res = ops.csr_build(ei, n)
    for a, b in zip(res, (g.rowptr, g.col, g.csr_eid, g.colptr, g.row, g.csc_eid, g.csc2csr)):
        assert torch.equal(a, b)
    s_src, s_dst = ops.node_scores(h, a_s, a_d, H, C)
    r_src, r_dst = ho.node_scores(h, a_s, a_d, H, C)
    assert torch.equal(s_src, r_src) and torch.equal(s_dst, r_dst)
    out, m, inv_l, agg, seed_used = ops.gat_fwd(h, s_src, s_dst, bias, g.col, g.csr_eid,
                                                *tops.schedule_args(g.fwd_sched), H, C, 0, 0.2, 0.2, 1234, H > 1)
    sb = ho.seed_buffer(0.2, cuda)
    o2, m2, l2, a2 = ho.gat_fwd(g, h, s_src, s_dst, bias, H, C, 0, 0.2, 0.2, 1234, H > 1, seed_buf=sb)
    assert torch.equal(out, o2) and torch.equal(m, m2) and torch.equal(inv_l, l2) and torch.equal(seed_used, sb)
    G = torch.randn(n, C, device=cuda)
    gh, ds, dd, db = ops.gat_bwd(h, s_src, s_dst, a_s, a_d, bias, out, agg if H > 1 else None, m, inv_l, G, g.rowptr,
                                 g.row, g.csc_eid, g.csc2csr, *tops.schedule_args(g.bwd_sched), H, C, 0, 0.2, 0.2,
                                 1234, seed_used, True)
    r = ho.gat_bwd(g, h, s_src, s_dst, a_s, a_d, bias, out, agg if H > 1 else None, m, inv_l, G, H, C, 0, 0.2, 0.2,
                   1234, want_bias_grad=True, seed_buf=seed_used)
    for a, b in zip((gh, ds, dd, db), r):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_ops_trace_through_compile_and_torchscript(pkg, cuda):
    tops = _tops()
    ops = tops.load()
    ei, h, a_s, a_d = _graph_inputs(cuda)
    g = pkg.hip_ops.csr_build(ei, h.size(0))
    sargs = tops.schedule_args(g.fwd_sched)

    def layer(h, a_s, a_d, col, eid, r0, r1, r2, r3, r4):
        s_src, s_dst = torch.ops.ppgat.node_scores(h, a_s, a_d, 1, 128)
        out = torch.ops.ppgat.gat_fwd(h, s_src, s_dst, None, col, eid, r0, r1, r2, r3, r4, sargs[5], 1, 128, 0, 0.2,
                                      0.0, 0, False)[0]
        return out * 2.0 + 1.0

    eager = layer(h, a_s, a_d, g.col, g.csr_eid, *sargs[:5])
    compiled = torch.compile(layer, backend="aot_eager", fullgraph=True)
    assert torch.equal(compiled(h, a_s, a_d, g.col, g.csr_eid, *sargs[:5]), eager)

    @torch.jit.script
    def scores(h: torch.Tensor, a_s: torch.Tensor, a_d: torch.Tensor):
        return torch.ops.ppgat.node_scores(h, a_s, a_d, 1, 128)

    s1, s2 = scores(h, a_s, a_d)
    r1, r2 = pkg.hip_ops.node_scores(h, a_s, a_d, 1, 128)
    assert torch.equal(s1, r1) and torch.equal(s2, r2)
