"""The CPU oracle, pinned against the real reference (tests/golden, made by importing
scripts/train_gat_custom.py) -- CPU only."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN

CASES = ["small_c8", "uniform_c128", "skewed_c128", "clamp_c128"]


def _load(name):
    return dict(np.load(GOLDEN / f"layer_{name}.npz"))


def _rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("name", CASES)
def test_custom_oracle_matches_reference_golden(oracle, name):
    g = _load(name)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    W = torch.from_numpy(g["lin_weight"]).requires_grad_(True)
    a_s = torch.from_numpy(g["a_src"]).requires_grad_(True)
    a_d = torch.from_numpy(g["a_dst"]).requires_grad_(True)
    out = oracle.custom_gat_layer(x, torch.from_numpy(g["edge_index"]), W, a_s, a_d)
    (out * torch.from_numpy(g["G"])).sum().backward()
    # same op order as the reference on the same CPU -> (near) bitwise
    assert _rel(out.detach(), g["out"]) <= 1e-6
    assert _rel(x.grad, g["dx"]) <= 1e-5
    assert _rel(W.grad, g["dW"]) <= 1e-5
    assert _rel(a_s.grad, g["da_src"]) <= 1e-5
    assert _rel(a_d.grad, g["da_dst"]) <= 1e-5


@pytest.mark.parametrize("name", ["small_c8", "uniform_c128", "skewed_c128"])
def test_pyg_restatement_equals_reference_custom_layer(oracle, name):
    """PyG GATConv restatement == imported custom reference when H=1, bias=0, |e|<10
    (SURVEY.md 8(c) partial pin), forward and all gradients, fp64."""
    g = _load(name)
    assert float(g["emax"]) < 10.0
    d = torch.float64
    x = torch.from_numpy(g["x"]).to(d).requires_grad_(True)
    W = torch.from_numpy(g["lin_weight"]).to(d).requires_grad_(True)
    a_s = torch.from_numpy(g["a_src"]).to(d).requires_grad_(True)
    a_d = torch.from_numpy(g["a_dst"]).to(d).requires_grad_(True)
    ei = torch.from_numpy(g["edge_index"])
    Gt = torch.from_numpy(g["G"]).to(d)
    out = oracle.pyg_gat_conv(x, ei, W, a_s.view(1, 1, -1), a_d.view(1, 1, -1), None, heads=1)
    (out * Gt).sum().backward()
    grads = [t.grad.clone() for t in (x, W, a_s, a_d)]
    for t in (x, W, a_s, a_d):
        t.grad = None
    ref = oracle.custom_gat_layer(x, ei, W, a_s, a_d)
    (ref * Gt).sum().backward()
    # the only difference is the softmax eps (custom 1e-9 vs PyG 1e-16): ~1e-9 relative
    assert _rel(out.detach(), ref.detach()) <= 1e-8
    for a, t in zip(grads, (x, W, a_s, a_d)):
        assert _rel(a, t.grad) <= 1e-7
    # and against the fp32 reference output itself
    assert _rel(out.detach(), g["out"]) <= 1e-5


def test_dropout_mask_properties(oracle):
    eid = np.arange(200_000)
    m = oracle.dropout_scale(1234, eid, 0, 0.1)
    keep = (m > 0).mean()
    assert abs(keep - 0.9) < 0.005
    assert np.allclose(m[m > 0], 1 / 0.9)
    assert np.array_equal(m, oracle.dropout_scale(1234, eid, 0, 0.1))
    assert not np.array_equal(m, oracle.dropout_scale(1234, eid, 1, 0.1))
    assert not np.array_equal(m, oracle.dropout_scale(1235, eid, 0, 0.1))
    assert np.all(oracle.dropout_scale(1, eid, 0, 0.0) == 1)


def test_csr_oracle_simple(oracle):
    ei = np.array([[0, 2, 1, 2, 0], [1, 1, 0, 2, 1]])
    rowptr, col, eid, colptr, row, ceid, c2r = oracle.csr_from_edge_index(ei, 4)
    assert rowptr.tolist() == [0, 1, 4, 5, 5]
    assert eid.tolist() == [2, 0, 1, 4, 3]
    assert col.tolist() == [1, 0, 2, 0, 2]
    assert colptr.tolist() == [0, 2, 3, 5, 5]
    assert ceid.tolist() == [0, 4, 2, 1, 3]
    assert row.tolist() == [1, 1, 0, 1, 2]
    assert all(eid[c2r[k]] == ceid[k] for k in range(5))


def test_serving_topk_and_rank(oracle):
    v = np.eye(10, dtype=np.float32)
    idx, sc = oracle.serving_topk(v, [0, 1], 3)
    assert 0 not in idx and 1 not in idx and len(idx) == 3
    assert all(sc[i] >= sc[i + 1] for i in range(2))
    assert oracle.sampled_rank(np.array([1.0, 2.0, 1.0, 0.5])) == 2


def test_fusion_train_loss_oracle_matches_reference_golden(oracle):
    """fusion_train_loss (fp64) at dropout 0 vs the reference's own contrastive_fusion_loss and
    autograd gradients on the golden batch (tests/golden/fusion_mlp.npz, first 256 rows)."""
    g = dict(np.load(GOLDEN / "fusion_mlp.npz"))
    P = {k[4:]: torch.from_numpy(v).double().requires_grad_(True) for k, v in g.items() if k.startswith("sd__")}
    loss, lt, li = oracle.fusion_train_loss(P, torch.from_numpy(g["txt"][:256]).double(),
                                            torch.from_numpy(g["img"][:256]).double())
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 1e-5 * float(g["loss"])
    assert abs(float(lt) - float(g["loss_txt"])) <= 1e-5 * float(g["loss_txt"])
    assert abs(float(li) - float(g["loss_img"])) <= 1e-5 * float(g["loss_img"])
    for k, p in P.items():
        ref = torch.from_numpy(g["grad__" + k]).double()
        assert float((p.grad - ref).abs().max() / ref.abs().max()) <= 1e-4, k


def test_mlp_dropout_mask_properties(oracle):
    m = oracle.mlp_dropout_scale(77, 200_000, 0.1)
    assert np.array_equal(m, oracle.mlp_dropout_scale(77, 200_000, 0.1))
    assert abs(float((m == 0).mean()) - 0.1) < 0.005
    assert set(np.unique(m).tolist()) == {0.0, float(np.float32(1) / np.float32(0.9))}
    assert not np.array_equal(m, oracle.mlp_dropout_scale(78, 200_000, 0.1))
    assert np.all(oracle.mlp_dropout_scale(77, 1000, 0.0) == 1.0)


def test_chunked_oracle_equals_whole_graph(oracle):
    """pyg_gat_conv_chunked (destination blocks, used as the config-5 full-size checker) gives
    the whole-graph oracle's output, dx and parameter gradients, with dropout and hub rows."""
    g = _load("skewed_c128")
    rng = np.random.default_rng(4)
    H, C, Cin = 2, 16, 24
    n = g["x"].shape[0]
    ei = torch.from_numpy(g["edge_index"])
    x = torch.from_numpy(rng.standard_normal((n, Cin))).double()
    G = torch.from_numpy(rng.standard_normal((n, C))).double()
    P = {"lin.weight": torch.from_numpy(rng.standard_normal((H * C, Cin)) * 0.2),
         "att_src": torch.from_numpy(rng.standard_normal((1, H, C)) * 0.2),
         "att_dst": torch.from_numpy(rng.standard_normal((1, H, C)) * 0.2),
         "bias": torch.from_numpy(rng.standard_normal(C) * 0.1)}
    out_c, dx_c, gr_c = oracle.pyg_gat_conv_chunked(P, x, ei, G, H, 0.1, 77, max_edges=700)
    Q = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    xw = x.clone().requires_grad_(True)
    out = oracle.pyg_gat_conv(xw, ei, Q["lin.weight"], Q["att_src"], Q["att_dst"], Q["bias"], H, dropout_p=0.1,
                              seed=77)
    (out * G).sum().backward()
    assert _rel(out_c, out.detach()) <= 1e-12
    assert _rel(dx_c, xw.grad) <= 1e-12
    for k in P:
        assert _rel(gr_c[k], Q[k].grad) <= 1e-11, k
    # the gradient-path split behind the config-5 per-row dx bound: the message path (attention
    # weights detached) and the attention path (h detached in the message) add up to dx
    _, dx_c2, _, dxm_c = oracle.pyg_gat_conv_chunked(P, x, ei, G, H, 0.1, 77, max_edges=700, dx_message=True)
    assert torch.equal(dx_c2, dx_c)
    parts = []
    for det in ("alpha", "msg_h"):
        xp = x.clone().requires_grad_(True)
        o = oracle.pyg_gat_conv(xp, ei, P["lin.weight"], P["att_src"], P["att_dst"], P["bias"], H, dropout_p=0.1,
                                seed=77, detach=det)
        assert torch.equal(o, out.detach())                 # the same forward value
        parts.append(torch.autograd.grad((o * G).sum(), xp)[0])
    assert _rel(dxm_c, parts[0]) <= 1e-12
    assert _rel(parts[0] + parts[1], xw.grad) <= 1e-12
    assert float((parts[1]).abs().max()) > 1e-3 * float(parts[0].abs().max())  # both paths carry weight
    # the attention path's pre-cancellation scale bounds its value on every row, and stays
    # nonzero on a destination with a single in-edge whose own softmax piece cancels exactly
    U = oracle.pyg_dx_attention_scale(P, x, ei, G, H, 0.1, 77, max_edges=1000)
    assert U.shape == (n,) and bool((parts[1].norm(dim=1) <= U * (1 + 1e-9) + 1e-300).all())
    indeg = torch.bincount(ei[1], minlength=n)
    one = int(torch.nonzero(indeg == 1)[0])
    assert float(U[one]) > 0


def test_rows_oracle_equals_whole_graph(oracle):
    """pyg_gat_conv_rows (the full-graph test's checker: the layer restricted to sampled
    destination rows, the upstream gradient zero elsewhere) gives the chunked whole-graph
    oracle's rows, dx and parameter gradients -- with the heaviest row on the scatter-free
    single-destination path (``heavy`` below its in-degree) and on the general one, with kink
    sides given."""
    g = _load("skewed_c128")
    rng = np.random.default_rng(5)
    H, C, Cin = 2, 16, 24
    n = g["x"].shape[0]
    ei = torch.from_numpy(g["edge_index"])
    x = torch.from_numpy(rng.standard_normal((n, Cin))).double()
    P = {"lin.weight": torch.from_numpy(rng.standard_normal((H * C, Cin)) * 0.2),
         "att_src": torch.from_numpy(rng.standard_normal((1, H, C)) * 0.2),
         "att_dst": torch.from_numpy(rng.standard_normal((1, H, C)) * 0.2),
         "bias": torch.from_numpy(rng.standard_normal(C) * 0.1)}
    indeg = torch.bincount(ei[1], minlength=n)
    hub = int(torch.argmax(indeg))
    rows = torch.tensor([hub] + [r for r in range(5, n, max(1, n // 7)) if r != hub][:6])
    Gr = torch.from_numpy(rng.standard_normal((rows.numel(), C)))
    G = torch.zeros(n, C, dtype=torch.float64)
    G[rows] = Gr
    out_c, dx_c, gr_c = oracle.pyg_gat_conv_chunked(P, x, ei, G, H, 0.1, 77, max_edges=700)
    cols = torch.nonzero(torch.isin(ei[1], rows)).squeeze(1)
    for heavy in (int(indeg[hub]) + 1, int(indeg[hub]) - 1):
        o, nodes, dxn, gr = oracle.pyg_gat_conv_rows(P, x, ei, cols, rows, Gr, H, 0.1, 77, heavy=heavy)
        assert _rel(o, out_c[rows]) <= 1e-12, heavy
        assert _rel(dxn, dx_c[nodes]) <= 1e-12, heavy
        dx_c_off = dx_c.clone()
        dx_c_off[nodes] = 0
        assert float(dx_c_off.abs().max()) == 0.0    # no other row carries a gradient
        for k in P:
            assert _rel(gr[k], gr_c[k]) <= 1e-11, (heavy, k)
    kp = torch.from_numpy(rng.random((ei.shape[1], H)) > 0.5)
    a, b = [], []
    ra = oracle.pyg_gat_conv_rows(P, x, ei, cols, rows, Gr, H, 0.1, 77, kink_pos=kp, kink_stats=a,
                                  heavy=int(indeg[hub]) + 1)
    rb = oracle.pyg_gat_conv_rows(P, x, ei, cols, rows, Gr, H, 0.1, 77, kink_pos=kp, kink_stats=b,
                                  heavy=int(indeg[hub]) - 1)
    assert _rel(ra[0], rb[0]) <= 1e-12 and _rel(ra[2], rb[2]) <= 1e-12
    assert sum(s[0] for s in a) == sum(s[0] for s in b) > 0


def test_kink_sides_option(oracle):
    """kink_pos = the fp64 signs leaves the layer unchanged (bitwise) and reports no tie; all
    sides forced to slope 1 gives the layer without the LeakyReLU; flipped sides are reported."""
    g = _load("uniform_c128")
    x = torch.from_numpy(g["x"]).double()
    ei = torch.from_numpy(g["edge_index"])
    W = torch.from_numpy(g["lin_weight"]).double()
    a_s = torch.from_numpy(g["a_src"]).double().view(1, 1, -1)
    a_d = torch.from_numpy(g["a_dst"]).double().view(1, 1, -1)
    b = torch.zeros(W.size(0), dtype=torch.float64)
    h = x @ W.t()
    z = (h @ a_s.view(-1))[ei[0]] + (h @ a_d.view(-1))[ei[1]]
    base = oracle.pyg_gat_conv(x, ei, W, a_s, a_d, b, 1)
    st = []
    same = oracle.pyg_gat_conv(x, ei, W, a_s, a_d, b, 1, kink_pos=(z > 0).view(-1, 1), kink_stats=st)
    assert torch.equal(base, same) and st == [(0, 0.0, 0.0)]
    lin = oracle.pyg_gat_conv(x, ei, W, a_s, a_d, b, 1, kink_pos=torch.ones(ei.size(1), 1, dtype=torch.bool))
    ref = oracle.pyg_gat_conv(x, ei, W, a_s, a_d, b, 1, negative_slope=1.0)
    assert torch.allclose(lin, ref, rtol=0, atol=1e-12)
    st = []
    flip = (z > 0).view(-1, 1).clone()
    flip[:3] = ~flip[:3]
    oracle.pyg_gat_conv(x, ei, W, a_s, a_d, b, 1, kink_pos=flip, kink_stats=st)
    assert st[0][0] == 3 and st[0][1] > 0 and st[0][2] > 1.0  # real flips, far beyond an fp32 tie
