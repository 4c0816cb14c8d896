"""Training-step kernels around the GAT layers (GPU): the MFMA weight-gradient GEMM and
the fused BPR/BCE loss, against fp64 torch restatements (oracle.bpr_loss follows
scripts/train_gat_pyg.py:313-322).  Tolerance: max-abs error / max-abs reference <= 1e-5."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("N,M,K", [(1000, 128, 128), (255_404, 128, 128), (63_001, 128, 384), (5000, 1024, 256),
                                   (37, 8, 16), (300, 200, 72), (1, 128, 128)])
def test_gemm_tn_vs_fp64(pkg, cuda, N, M, K):
    from importlib import import_module
    ops = import_module("plotpointe-gat-recommendation_amd.hip_ops")
    g = torch.Generator().manual_seed(N + M + K)
    A = torch.randn(N, M, generator=g, dtype=torch.float64)
    B = torch.randn(N, K, generator=g, dtype=torch.float64)
    V = torch.randn(N, 2, generator=g, dtype=torch.float64)
    out, cs, vo = ops.gemm_tn(A.float().to(cuda), B.float().to(cuda), want_colsum=True, V=V.float().to(cuda))
    assert rel(out, A.t() @ B) <= 1e-5
    assert rel(cs, A.sum(0)) <= 1e-5
    assert rel(vo, V.t() @ B) <= 1e-5
    out2, _, _ = ops.gemm_tn(A.float().to(cuda), B.float().to(cuda))  # M <= 16: the skinny kernel
    assert rel(out2, A.t() @ B) <= 1e-5
    out3, _, _ = ops.gemm_tn(A.float().to(cuda), B.float().to(cuda))
    assert torch.equal(out2, out3)
    assert torch.equal(out, out2)  # same kernel and order with or without the extras (M <= 16 too)


@pytest.mark.parametrize("N,M,K", [(489, 489, 128), (45, 45, 45), (301, 13, 130)])
def test_gemm_tn_unaligned_rows(pkg, cuda, N, M, K):
    """Operands whose rows are not 16-byte aligned (e.g. the [B, B] InfoNCE logit gradient of
    a ragged last batch) are zero-padded to a multiple of 4 columns, not refused."""
    from importlib import import_module
    ops = import_module("plotpointe-gat-recommendation_amd.hip_ops")
    g = torch.Generator().manual_seed(N * M + K)
    A = torch.randn(N, M, generator=g, dtype=torch.float64)
    B = torch.randn(N, K, generator=g, dtype=torch.float64)
    out, cs, _ = ops.gemm_tn(A.float().to(cuda), B.float().to(cuda), want_colsum=True)
    assert out.shape == (M, K) and cs.shape == (M,)
    assert rel(out, A.t() @ B) <= 1e-5
    assert rel(cs, A.sum(0)) <= 1e-5


def test_gemm_tn_strided_operands(pkg, cuda):
    """A and V as column slices of one [N, ld] buffer (the fused backward's D = [dh | ds])."""
    from importlib import import_module
    ops = import_module("plotpointe-gat-recommendation_amd.hip_ops")
    g = torch.Generator().manual_seed(9)
    N, HC, H = 20_000, 128, 2
    D = torch.randn(N, HC + 8, generator=g, dtype=torch.float64)
    x = torch.randn(N, 96, generator=g, dtype=torch.float64)
    Dd = D.float().to(cuda)
    out, _, vo = ops.gemm_tn(Dd[:, :HC], x.float().to(cuda), V=Dd[:, HC:HC + 2 * H])
    assert rel(out, D[:, :HC].t() @ x) <= 1e-5
    assert rel(vo, D[:, HC:HC + 2 * H].t() @ x) <= 1e-5


def test_linear_grads(pkg, cuda):
    from importlib import import_module
    ops = import_module("plotpointe-gat-recommendation_amd.hip_ops")
    torch.manual_seed(0)
    x64 = torch.randn(4000, 96, dtype=torch.float64, requires_grad=True)
    W64 = torch.randn(128, 96, dtype=torch.float64, requires_grad=True)
    b64 = torch.randn(128, dtype=torch.float64, requires_grad=True)
    G = torch.randn(4000, 128, dtype=torch.float64)
    x, W, b = (t.detach().float().to(cuda).requires_grad_(True) for t in (x64, W64, b64))
    (ops.linear(x, W, b) * G.float().to(cuda)).sum().backward()
    (torch.nn.functional.linear(x64, W64, b64) * G).sum().backward()
    assert rel(x.grad, x64.grad) <= 1e-5
    assert rel(W.grad, W64.grad) <= 1e-5
    assert rel(b.grad, b64.grad) <= 1e-5


@pytest.mark.parametrize("loss", ["bpr", "bce"])
@pytest.mark.parametrize("C", [32, 128, 256])
def test_bpr_loss_vs_oracle(pkg, oracle, cuda, loss, C):
    rng = np.random.default_rng(C)
    n_users, n_items, S = 3000, 500, 20_000
    # skewed items (a few appear in > 1000 triples -> rows spanning many 32-entry chunks)
    w = np.arange(1, n_items + 1, dtype=np.float64) ** -1.1
    w /= w.sum()
    u = torch.from_numpy(rng.integers(0, n_users, S))
    i = torch.from_numpy(rng.choice(n_items, S, p=w))
    j = torch.from_numpy(rng.choice(n_items, S, p=w))
    Z64 = torch.from_numpy(rng.standard_normal((n_users + n_items, C)) * 0.3).requires_grad_(True)
    Zd = Z64.detach().float().to(cuda).requires_grad_(True)
    L = pkg.bpr_loss(Zd, n_users, u.to(cuda), i.to(cuda), j.to(cuda), loss)
    (L * 3.0).backward()
    Lr = oracle.bpr_loss(Z64, n_users, u, i, j, loss)
    (Lr * 3.0).backward()
    assert abs(L.item() - Lr.item()) <= 1e-5 * abs(Lr.item())
    assert rel(Zd.grad, Z64.grad) <= 1e-5
    # deterministic
    g1 = Zd.grad.clone()
    Zd.grad = None
    (pkg.bpr_loss(Zd, n_users, u.to(cuda), i.to(cuda), j.to(cuda), loss) * 3.0).backward()
    assert torch.equal(g1, Zd.grad)


def test_bpr_single_row_everything(pkg, oracle, cuda):
    """All triples on one user and one item pair: one destination spans every chunk.  Each
    gradient row is a sum of 10,000 identical fp32 terms, whose rounding errors do not
    cancel: tolerance 5e-5 here (seeded input; 1e-5 everywhere else)."""
    n_users, n_items, S = 4, 3, 5000
    u = torch.zeros(S, dtype=torch.long)
    i = torch.ones(S, dtype=torch.long)
    j = torch.full((S,), 2, dtype=torch.long)
    g = torch.Generator().manual_seed(17)
    Z64 = torch.randn(n_users + n_items, 128, dtype=torch.float64, generator=g).requires_grad_(True)
    Zd = Z64.detach().float().to(cuda).requires_grad_(True)
    pkg.bpr_loss(Zd, n_users, u.to(cuda), i.to(cuda), j.to(cuda)).backward()
    oracle.bpr_loss(Z64, n_users, u, i, j).backward()
    assert rel(Zd.grad, Z64.grad) <= 5e-5


def test_bpr_bad_index_raises(pkg, cuda):
    from importlib import import_module
    ops = import_module("plotpointe-gat-recommendation_amd.hip_ops")
    Z = torch.randn(10, 128, device=cuda, requires_grad=True)
    u = torch.tensor([0, 1], device=cuda)
    i = torch.tensor([0, 7], device=cuda)   # 7 >= n_items = 4
    j = torch.tensor([1, 2], device=cuda)
    pkg.bpr_loss(Z, 6, u, i, j)
    with pytest.raises(IndexError):
        ops.check_bpr_indices()
    pkg.bpr_loss(Z, 6, u, torch.tensor([0, 3], device=cuda), j)
    ops.check_bpr_indices()


@pytest.mark.gpu
def test_bpr_large_row_space(pkg, oracle, cuda):
    """N > 2^20 rows: the contribution sort takes three radix passes (21 key bits)."""
    rng = np.random.default_rng(7)
    n_users, n_items, S, C = 1_100_000, 2_000, 30_000, 32
    u = torch.from_numpy(rng.integers(0, n_users, S))
    i = torch.from_numpy(rng.integers(0, n_items, S))
    j = torch.from_numpy(rng.integers(0, n_items, S))
    Z64 = torch.from_numpy(rng.standard_normal((n_users + n_items, C)) * 0.3).requires_grad_(True)
    Zd = Z64.detach().float().to(cuda).requires_grad_(True)
    pkg.bpr_loss(Zd, n_users, u.to(cuda), i.to(cuda), j.to(cuda)).backward()
    oracle.bpr_loss(Z64, n_users, u, i, j).backward()
    assert rel(Zd.grad, Z64.grad) <= 1e-5


@pytest.mark.gpu
def test_bpr_sparse_keys_zero_untouched_rows(pkg, oracle, cuda):
    """Three triples over 500k rows: almost every row of dZ is reached by no contribution and
    must be written as zero (k_bpr_zero_untouched, row-parallel) -- on memory the caching
    allocator hands back dirty (NaN-filled) on purpose."""
    rng = np.random.default_rng(3)
    n_users, n_items, S, C = 400_000, 100_000, 3, 128
    dirty = torch.full(((n_users + n_items) * C * 2,), float("nan"), device=cuda)
    del dirty
    u = torch.from_numpy(rng.integers(0, n_users, S))
    i = torch.from_numpy(rng.integers(0, n_items, S))
    j = torch.from_numpy(rng.integers(0, n_items, S))
    Z64 = torch.from_numpy(rng.standard_normal((n_users + n_items, C)) * 0.3).requires_grad_(True)
    Zd = Z64.detach().float().to(cuda).requires_grad_(True)
    pkg.bpr_loss(Zd, n_users, u.to(cuda), i.to(cuda), j.to(cuda)).backward()
    oracle.bpr_loss(Z64, n_users, u, i, j).backward()
    assert torch.isfinite(Zd.grad).all()
    assert rel(Zd.grad, Z64.grad) <= 1e-5
    assert int((Zd.grad != 0).any(1).sum()) <= 3 * S


@pytest.mark.parametrize("n_users,n_items,S,C,mapped", [(3000, 500, 20_000, 128, False), (1_100_000, 2_000, 30_000, 32,
                                                                                        False),
                                                         (3000, 500, 20_000, 256, True), (50, 40, 0, 64, False),
                                                         (7, 5, 1, 32, True)])
def test_bpr_prepared_bitwise(pkg, cuda, n_users, n_items, S, C, mapped):
    """ppgat_bpr_bwd_prepare on a side stream (started before Z exists) + ppgat_bpr_bwd_prepared
    == the one-call ppgat_bpr_bwd, bit for bit: 2- and 3-pass sorts (odd/even pass parity of the
    sorted pairs' home), a row map with unheld users (-1), no triples at all."""
    from importlib import import_module
    ops = import_module("plotpointe-gat-recommendation_amd.hip_ops")
    rng = np.random.default_rng(S + C)
    u, i, j = (torch.from_numpy(rng.integers(0, n, S)).to(cuda) for n in (n_users, n_items, n_items))
    N = n_users + n_items
    row_map = None
    if mapped:
        perm = rng.permutation(N + 3)[:N].astype(np.int32)
        perm[rng.random(N) < 0.2] = -1                     # users not held here
        perm[n_users:] = np.abs(perm[n_users:])          # items always held
        row_map = torch.from_numpy(perm).to(cuda)
        n_rows = N + 3
    else:
        n_rows = N
    Z0 = torch.from_numpy(rng.standard_normal((n_rows, C)).astype(np.float32) * 0.3).to(cuda)
    grads, losses = [], []
    for use_prep in (False, True):
        Z = Z0.clone()
        prep = ops.bpr_prepare(n_rows, n_users, n_items, C, u, i, j, row_map) if use_prep else None
        torch.cuda._sleep(2_000_000) if use_prep else None   # the forward still running on the main stream
        Z = (Z * 1.0).requires_grad_(True)
        L = (ops.bpr_loss_mapped(Z, n_users, n_items, row_map, u, i, j, prepared=prep) if mapped
             else ops.bpr_loss(Z, n_users, u, i, j, prepared=prep))
        (L * 2.0).backward()
        grads.append(Z.grad.clone())
        losses.append(L.detach().clone())
    assert torch.equal(grads[0], grads[1]) and torch.equal(losses[0], losses[1])
    prep = ops.bpr_prepare(n_rows, n_users, n_items, C, u, i, j, row_map)
    with pytest.raises(RuntimeError):                      # other triples / sizes than prepared
        ops.bpr_loss_mapped(Z0, n_users, n_items + 1 if S == 0 else n_items, row_map, u.clone(), i, j, prepared=prep)
    torch.cuda.synchronize()


@pytest.mark.parametrize("n_users,n_items,S,C,with_bias", [(3000, 500, 20_000, 128, True), (2000, 300, 5000, 256, True),
                                                           (400, 100, 3000, 32, False), (50, 40, 0, 128, True),
                                                           (4, 3, 5000, 64, True)])
def test_bpr_bwd_producer(pkg, cuda, n_users, n_items, S, C, with_bias):
    """ppgat_bpr_bwd_producer: grad_Z bit for bit that of ppgat_bpr_bwd, plus the producing
    layer's prologue -- nstate = {s_dst, m, inv_l, <dZ_r, Z_r - b>} from the forward's dot
    products and dbias = sum_r dZ_r -- against fp64 of the same dZ (per-row bound relative to
    the pre-cancellation size sum |dZ| |Z - b|); rows spanning many chunks (one user, one item
    pair); no triples at all."""
    import ctypes
    lib = pkg._lib.load()
    rng = np.random.default_rng(S + C)
    u, i, j = (torch.from_numpy(rng.integers(0, n, S)).to(cuda) for n in (n_users, n_items, n_items))
    N = n_users + n_items
    Z = torch.from_numpy(rng.standard_normal((N, C)).astype(np.float32) * 0.3).to(cuda)
    b = torch.from_numpy(rng.standard_normal(C).astype(np.float32) * 0.1).to(cuda)
    sd, m, il = (torch.from_numpy(rng.standard_normal(N).astype(np.float32)).to(cuda) for _ in range(3))
    nbytes = ctypes.c_size_t(0)
    pkg._lib.check(lib.ppgat_bpr_workspace_bytes(N, S, C, ctypes.byref(nbytes)), "ws")
    st = pkg._lib.stream_handle(cuda)
    gl = torch.tensor([1.7], device=cuda)
    res = []
    for producer in (False, True):
        ws = torch.full((int(nbytes.value),), 255, dtype=torch.uint8, device=cuda)
        loss = torch.empty(1, device=cuda)
        coef = torch.empty(max(S, 1), 2, device=cuda)
        pkg._lib.check(lib.ppgat_bpr_fwd(Z.data_ptr(), N, n_users, n_items, None, C, u.data_ptr(), i.data_ptr(),
                                         j.data_ptr(), S, 0, loss.data_ptr(), coef.data_ptr(), None, ws.data_ptr(),
                                         nbytes.value, st), "fwd")
        dZ = torch.full((N, C), float("nan"), device=cuda)
        ns = torch.full((N, 4), float("nan"), device=cuda)
        db = torch.full((C,), float("nan"), device=cuda)
        if producer:
            pkg._lib.check(lib.ppgat_bpr_bwd_producer(
                Z.data_ptr(), N, n_users, n_items, C, u.data_ptr(), i.data_ptr(), j.data_ptr(), S, coef.data_ptr(),
                gl.data_ptr(), dZ.data_ptr(), b.data_ptr() if with_bias else None, sd.data_ptr(), m.data_ptr(),
                il.data_ptr(), 1.0, ns.data_ptr(), db.data_ptr() if with_bias else None, ws.data_ptr(), nbytes.value,
                st), "bwd_producer")
        else:
            pkg._lib.check(lib.ppgat_bpr_bwd(Z.data_ptr(), N, n_users, n_items, None, C, u.data_ptr(), i.data_ptr(),
                                             j.data_ptr(), S, coef.data_ptr(), gl.data_ptr(), dZ.data_ptr(),
                                             ws.data_ptr(), nbytes.value, st), "bwd")
        res.append((dZ, ns, db))
    (dZ0, _, _), (dZ1, ns, db) = res
    assert torch.equal(dZ0, dZ1)
    dz64, z64 = dZ1.double().cpu(), Z.double().cpu()
    zb = z64 - (b.double().cpu() if with_bias else 0.0)
    Dref = (dz64 * zb).sum(1)
    scale = (dz64.abs() * zb.abs()).sum(1)
    err = (ns[:, 3].double().cpu() - Dref).abs()
    assert bool((err <= 1e-5 * scale + 1e-30).all()), float((err / scale.clamp_min(1e-30)).max())
    assert torch.equal(ns[:, :3].cpu(), torch.stack([sd, m, il], 1).cpu())
    if with_bias:
        ref = dz64.sum(0)
        assert float((db.double().cpu() - ref).abs().max()) <= 1e-5 * max(float(dz64.abs().sum(0).max()), 1e-30)


def _two_layer_grads(pkg, cuda, steps=1, zero=True):
    g = pkg.data.synthetic_ui_graph(n_users=3000, n_items=800, n_interactions=40_000, seed=5)
    ei = torch.from_numpy(g.edge_index_numpy()).to(cuda)
    feats = torch.from_numpy(pkg.data.synthetic_item_features(g.n_items, 64, seed=5)).to(cuda)
    torch.manual_seed(0)
    model = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=64, hidden=128, layers=2, heads=1,
                       attn_dropout=0.1).to(cuda).train()
    u, i, j = (torch.from_numpy(a).to(cuda) for a in pkg.data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items,
                                                                                 20_000, seed=1))
    for s in range(steps):
        if zero:
            model.zero_grad(set_to_none=True)
        torch.manual_seed(100 + s)
        pkg.bpr_loss(model(feats, ei), g.n_users, u, i, j).backward()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def test_side_stream_weight_grads_bitwise(pkg, cuda, monkeypatch):
    """Layer weight gradients on the side stream (joined at the end of backward) equal the
    in-order path bit for bit, read straight after backward() without a sync; a second
    backward into existing .grad takes the in-order path (accumulation)."""
    monkeypatch.setenv("PPGAT_FUSED_DXW", "0")  # the side stream runs the two-kernel products
    monkeypatch.setenv("PPGAT_ASYNC_WGRAD", "0")
    ref = _two_layer_grads(pkg, cuda)
    acc_ref = _two_layer_grads(pkg, cuda, steps=2, zero=False)
    monkeypatch.setenv("PPGAT_ASYNC_WGRAD", "1")
    got = _two_layer_grads(pkg, cuda)
    acc = _two_layer_grads(pkg, cuda, steps=2, zero=False)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
        assert torch.equal(acc[k], acc_ref[k]), k
    assert pkg.hip_ops._PENDING_JOINS == []
