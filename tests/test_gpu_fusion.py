"""A11 FusionMLP (GPU): the fused fp32-MFMA inference kernel vs the reference golden
(embeddings/fuse_modal.py imported in make_golden.py) and vs an fp64 restatement, with the
mean-image fallback path; InfoNCE training step vs the reference's loss and grads.
Tolerance: max-abs error / max-abs reference <= 1e-5."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu() if torch.is_tensor(a) else torch.from_numpy(np.asarray(a, np.float64))
    b = b.detach().double().cpu() if torch.is_tensor(b) else torch.from_numpy(np.asarray(b, np.float64))
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLDEN / "fusion_mlp.npz"))


def _model(pkg, gold, cuda):
    m = pkg.fusion.FusionMLP(384, 512, 128, 256)
    sd = {k[4:]: torch.from_numpy(v) for k, v in gold.items() if k.startswith("sd__")}
    assert sorted(sd) == sorted(m.state_dict())
    m.load_state_dict(sd)
    return m.to(cuda)


def test_seeded_construction_matches_reference(pkg, gold):
    torch.manual_seed(11)
    m = pkg.fusion.FusionMLP(384, 512, 128, 256)
    for k, v in m.state_dict().items():
        assert torch.equal(v, torch.from_numpy(gold["sd__" + k])), k


def test_fused_kernel_vs_reference_golden(pkg, gold, cuda):
    m = _model(pkg, gold, cuda).eval()
    txt, img = torch.from_numpy(gold["txt"]).to(cuda), torch.from_numpy(gold["img"]).to(cuda)
    with torch.no_grad():
        fused = m(txt, img)
    assert rel(fused, gold["fused"]) <= 1e-5
    idx = torch.arange(300, dtype=torch.int32, device=cuda)
    out = pkg.fusion.fusion_forward(txt, img, m.mlp[0].weight, m.mlp[0].bias, m.mlp[3].weight, m.mlp[3].bias,
                                    normalize=True, img_index=idx, img_fallback=img.mean(0))
    assert rel(out, gold["fused_norm"]) <= 1e-5


def test_infer_all_items_with_fallback_vs_fp64(pkg, oracle, gold, cuda):
    m = _model(pkg, gold, cuda)
    rng = np.random.default_rng(5)
    n_items, n_img = 5000, 3100
    txt = rng.standard_normal((n_items, 384)).astype(np.float32)
    img_indices = np.sort(rng.choice(n_items, n_img, replace=False))       # items that have an image
    img_aligned = rng.standard_normal((n_img, 512)).astype(np.float32)
    idx = pkg.fusion.image_index_for_items(n_items, img_indices)
    out = pkg.fusion.infer_fused_embeddings(m, torch.from_numpy(txt).to(cuda), torch.from_numpy(img_aligned).to(cuda),
                                            torch.from_numpy(idx).to(cuda), chunk=1777)
    mean_img = img_aligned.astype(np.float64).mean(0)
    img_rows = np.where(idx[:, None] >= 0, img_aligned.astype(np.float64)[np.maximum(idx, 0)], mean_img)
    P = {k: v.detach().double().cpu() for k, v in m.state_dict().items()}
    ref = oracle.fusion_mlp(torch.from_numpy(txt).double(), torch.from_numpy(img_rows), P["mlp.0.weight"],
                            P["mlp.0.bias"], P["mlp.3.weight"], P["mlp.3.bias"])
    assert rel(out, ref) <= 1e-5
    assert torch.allclose(out.norm(dim=-1).cpu(), torch.ones(n_items), atol=1e-5)


def test_training_step_loss_and_grads_vs_reference(pkg, gold, cuda):
    m = _model(pkg, gold, cuda).train()
    m.mlp[2].p = 0.0
    t = torch.from_numpy(gold["txt"][:256]).to(cuda)
    im = torch.from_numpy(gold["img"][:256]).to(cuda)
    f = m(t, im)
    loss, lt, li = pkg.fusion.contrastive_fusion_loss(f, m.txt_proj(t), m.img_proj(im))
    loss.backward()
    assert abs(loss.item() - float(gold["loss"])) <= 1e-5 * float(gold["loss"])
    for k, p in m.named_parameters():
        assert rel(p.grad, gold["grad__" + k]) <= 1e-4, k


def _golden_params(gold, cuda):
    return {k[4:]: torch.from_numpy(v).to(cuda) for k, v in gold.items() if k.startswith("sd__")}


def test_native_training_step_vs_reference_golden(pkg, gold, cuda):
    """fusion_train_step (matrix-core GEMMs + ppgat_relu_dropout + ppgat_infonce) at dropout 0
    on the golden batch: loss and every gradient vs the reference's own (fuse_modal.py:39-72
    imported by make_golden.py).  Loss 1e-5 relative, gradients 1e-4 (fp32 sums over B)."""
    m = _model(pkg, gold, cuda).train()
    m.mlp[2].p = 0.0
    t = torch.from_numpy(gold["txt"][:256]).to(cuda)
    im = torch.from_numpy(gold["img"][:256]).to(cuda)
    loss = pkg.fusion.fusion_train_step(m, t, im).cpu()
    assert abs(float(loss[0]) - float(gold["loss"])) <= 1e-5 * float(gold["loss"])
    assert abs(float(loss[1]) - float(gold["loss_txt"])) <= 1e-5 * float(gold["loss_txt"])
    assert abs(float(loss[2]) - float(gold["loss_img"])) <= 1e-5 * float(gold["loss_img"])
    for k, p in m.named_parameters():
        assert rel(p.grad, gold["grad__" + k]) <= 1e-4, (k, rel(p.grad, gold["grad__" + k]))


@pytest.mark.parametrize("B,p", [(512, 0.1), (44, 0.1), (1, 0.0), (1000, 0.3)])
def test_native_training_step_vs_fp64_oracle(pkg, oracle, gold, cuda, B, p):
    """Reference batch size 512, the ragged tail batch (300 = 256 + 44), a single row and a
    larger batch, with dropout: vs the fp64 restatement given the kernel's own mask (the mask
    itself is checked bit-exact against the numpy hash restatement)."""
    m = _model(pkg, gold, cuda).train()
    m.mlp[2].p = p
    g = torch.Generator().manual_seed(B)
    t = torch.randn(B, 384, generator=g)
    im = torch.randn(B, 512, generator=g)
    seed = 0xABCDEF + B
    loss = pkg.fusion.fusion_train_step(m, t.to(cuda), im.to(cuda), seed=seed).detach().cpu()
    ones = torch.ones(B, 256, device=cuda)
    mask_dev = pkg.fusion.relu_dropout(ones, p, seed).cpu()
    mask = oracle.mlp_dropout_scale(seed, B * 256, p).reshape(B, 256)
    assert np.array_equal(mask_dev.numpy(), mask)
    if p > 0:
        assert abs(float((mask == 0).mean()) - p) < 0.02 + 3.0 / np.sqrt(B * 256)
    P = {k: v.detach().double().cpu().requires_grad_(True) for k, v in m.named_parameters()}
    ref, rt, ri = oracle.fusion_train_loss(P, t.double(), im.double(), 0.07, torch.from_numpy(mask).double())
    ref.backward()
    assert abs(float(loss[0]) - float(ref.detach())) <= 1e-5 * max(float(ref.detach()), 1e-3)
    assert abs(float(loss[1]) - float(rt)) <= 1e-5 * max(float(rt), 1e-3)
    assert abs(float(loss[2]) - float(ri)) <= 1e-5 * max(float(ri), 1e-3)
    for k, prm in m.named_parameters():
        assert rel(prm.grad, P[k].grad) <= 1e-4, (k, rel(prm.grad, P[k].grad))


def test_native_train_loop_matches_autograd_loop(pkg, gold, cuda):
    """train_fusion native (device loss accumulation, device kernels) vs the torch-autograd loop
    at dropout 0 from the same weights: per-epoch losses agree (1e-4), and so does the loss of
    the two trained models on the training data.  (Weights are not compared entry by entry:
    Adam's g / sqrt(v) turns last-bit gradient differences on near-zero entries into lr-sized
    steps, so individual weights drift apart while the function they compute does not.)"""
    g = torch.Generator().manual_seed(3)
    txt = torch.randn(1300, 384, generator=g).to(cuda)
    img = torch.randn(1300, 512, generator=g).to(cuda)
    ms = []
    for native in (True, False):
        m = _model(pkg, gold, cuda)
        m.mlp[2].p = 0.0
        ms.append((m, pkg.fusion.train_fusion(m, txt, img, epochs=3, batch_size=512, native=native)))
    (m1, h1), (m2, h2) = ms
    for a, b in zip(h1, h2):
        assert np.allclose(a, b, rtol=1e-4, atol=1e-5), (h1, h2)
    with torch.no_grad():
        l1 = [float(pkg.fusion.contrastive_fusion_loss(m.train()(txt[:512], img[:512]), m.txt_proj(txt[:512]),
                                                       m.img_proj(img[:512]))[0]) for m in (m1, m2)]
    assert abs(l1[0] - l1[1]) <= 1e-3 * abs(l1[1]), l1


def test_autograd_loop_ragged_last_batch(pkg, gold, cuda):
    """train_fusion(native=False) with a last batch of 45 rows (301 = 2 x 128 + 45): the
    autograd InfoNCE backward takes dW = g^T x of the [45, 45] logit gradient through
    hip_ops.gemm_tn, whose rows are not 16-byte aligned (padded there, not refused); the
    per-epoch losses agree with the native loop's."""
    g = torch.Generator().manual_seed(5)
    txt = torch.randn(301, 384, generator=g).to(cuda)
    img = torch.randn(301, 512, generator=g).to(cuda)
    hs = []
    for native in (True, False):
        m = _model(pkg, gold, cuda)
        m.mlp[2].p = 0.0
        hs.append(pkg.fusion.train_fusion(m, txt, img, epochs=2, batch_size=128, native=native))
    for a, b in zip(*hs):
        assert np.allclose(a, b, rtol=1e-4, atol=1e-5), hs
