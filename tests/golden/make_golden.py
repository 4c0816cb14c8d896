#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REAL reference code.

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py

It imports /root/reference/scripts/train_gat_custom.py (the importable custom-GAT
trainer); ``google.cloud.storage`` (imported at module top, :20,
used only by gcs_download/gcs_upload :120-136) is replaced by an inert stub module.
Nothing else of the reference is touched.  Outputs are data only (inputs and the
reference's outputs), written as .npz / .json next to this script:

  layer_<name>.npz   SimpleGATLayer (train_gat_custom.py:63-93) forward in eval mode and
                     the gradients of sum(out * G) for a fixed upstream G.
  knn_small.npz      graphs/build_ii_knn.py main() (k=20, min_sim 0.3) on clustered
                     synthetic embeddings, GCS replaced by local files.
  plumbing_cfg1.npz  config-1 synthetic interactions -> build_splits (:148-162),
                     build_edge_index (:166-175), sample_bpr_epoch (:213-224, seed 42),
                     CustomGAT (:96-115) init at seed 42, eval forward Z, one BPR+Adam
                     step with attn dropout 0, eval_sampled (:184-210) metrics.
"""
from __future__ import annotations

import importlib.util
import json
import random
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path("/root/reference")


def _stub_gcs():
    google = sys.modules.setdefault("google", types.ModuleType("google"))
    cloud = types.ModuleType("google.cloud")
    storage = types.ModuleType("google.cloud.storage")

    class Client:  # never used by the math
        def __init__(self, *a, **k):
            raise RuntimeError("GCS disabled in fixture generation")

    storage.Client = Client
    cloud.storage = storage
    aiplatform = types.ModuleType("google.cloud.aiplatform")  # imported by fuse_modal.py:14, unused by the math
    cloud.aiplatform = aiplatform
    google.cloud = cloud
    sys.modules["google.cloud"] = cloud
    sys.modules["google.cloud.storage"] = storage
    sys.modules["google.cloud.aiplatform"] = aiplatform


def load_reference_custom():
    _stub_gcs()
    sys.path.insert(0, str(REF))
    spec = importlib.util.spec_from_file_location("ref_train_gat_custom",
                                                  REF / "scripts" / "train_gat_custom.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _pkg():
    sys.path.insert(0, str(REPO))
    import importlib
    return importlib.import_module("plotpointe-gat-recommendation_amd.data")


def make_graph(rng, n, e, kind):
    if kind == "uniform":
        src = rng.integers(0, n, e)
        dst = rng.integers(0, n, e)
    elif kind == "skewed":
        # heavy-tailed destinations incl. one hub with > 2 * 1024 in-edges, isolated
        # nodes (no in- and no out-edges), duplicates and self loops
        w = (np.arange(1, n + 1, dtype=np.float64)) ** -1.1
        w[n - 50:] = 0.0          # last 50 nodes: zero in-degree
        w /= w.sum()
        dst = rng.choice(n, e, p=w)
        src = rng.integers(0, n - 80, e)  # last 80 nodes: zero out-degree
        src[:40] = dst[:40]               # self loops
        src[40:80] = src[80:120]; dst[40:80] = dst[80:120]   # duplicates
    else:
        raise ValueError(kind)
    return np.stack([src, dst]).astype(np.int64)


def layer_case(ref, name, seed, n, e, c, kind, x_scale=1.0):
    torch.manual_seed(seed)
    rng = np.random.default_rng(1000 + seed)
    layer = ref.SimpleGATLayer(c, c)            # default attn_dropout=0.1, eval() disables it
    layer.eval()
    ei = make_graph(rng, n, e, kind)
    x = (rng.standard_normal((n, c)) * x_scale).astype(np.float32)
    g = rng.standard_normal((n, c)).astype(np.float32)
    xt = torch.from_numpy(x).requires_grad_(True)
    out = layer(xt, torch.from_numpy(ei))
    (out * torch.from_numpy(g)).sum().backward()
    # max |e| of the pre-clamp logits, to tell the clamp regime apart
    with torch.no_grad():
        h = layer.lin(xt)
        z = (h[ei[0]] * layer.a_src).sum(-1) + (h[ei[1]] * layer.a_dst).sum(-1)
        emax = float(torch.nn.functional.leaky_relu(z, 0.2).abs().max())
    np.savez_compressed(
        HERE / f"layer_{name}.npz",
        x=x, edge_index=ei, G=g,
        lin_weight=layer.lin.weight.detach().numpy(),
        a_src=layer.a_src.detach().numpy(), a_dst=layer.a_dst.detach().numpy(),
        out=out.detach().numpy(),
        dx=xt.grad.numpy(), dW=layer.lin.weight.grad.numpy(),
        da_src=layer.a_src.grad.numpy(), da_dst=layer.a_dst.grad.numpy(),
        emax=np.float32(emax), seed=np.int64(seed),
    )
    print(f"layer_{name}: N={n} E={e} C={c} max|e|={emax:.2f}")


def plumbing_case(ref):
    data = _pkg()
    inter = data.synthetic_interactions_small(seed=0)
    maps = data.node_maps_from_interactions(inter)
    user_to_idx = {k: int(v) for k, v in maps["user_to_idx"].items()}
    item_to_idx = {k: int(v) for k, v in maps["item_to_idx"].items()}
    train_raw, val_raw, test_raw = ref.build_splits(inter)
    # index mapping as in train_gat_custom.py:278-297
    train_idx, val_idx, test_idx = {}, {}, {}
    for u_raw, items in train_raw.items():
        u = user_to_idx.get(str(u_raw), user_to_idx.get(u_raw, None))
        if u is None:
            continue
        ii = [item_to_idx.get(str(it), item_to_idx.get(it, None)) for it in items]
        ii = [t for t in ii if t is not None]
        if ii:
            train_idx[int(u)] = np.array(ii, dtype=np.int64)
    for d_raw, d_idx in ((val_raw, val_idx), (test_raw, test_idx)):
        for u_raw, it in d_raw.items():
            u = user_to_idx.get(str(u_raw)); t = item_to_idx.get(str(it))
            if u is not None and t is not None:
                d_idx[int(u)] = int(t)
    n_users, n_items = maps["n_users"], maps["n_items"]
    ei = ref.build_edge_index(n_users, n_items, train_idx)
    random.seed(42)
    bu, bi, bj = ref.sample_bpr_epoch(train_idx, n_items, 5000)
    feats = np.random.RandomState(0).standard_normal((n_items, 384)).astype(np.float32)

    ref.set_seed(42)
    model = ref.CustomGAT(n_users, n_items, item_feat_dim=384, hidden=128, layers=2)
    sd0 = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    model.eval()
    itf = torch.from_numpy(feats)
    with torch.no_grad():
        Z0 = model(itf, ei).numpy()
    # one training step, attn dropout 0 (GPU/CPU dropout streams cannot match)
    model.train()
    for layer in model.layers:
        layer.drop.p = 0.0
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)
    u = torch.from_numpy(bu).long(); i = torch.from_numpy(bi).long(); j = torch.from_numpy(bj).long()
    Z = model(itf, ei)
    U, I = Z[:n_users], Z[n_users:]
    pos = (U[u] * I[i]).sum(-1); neg = (U[u] * I[j]).sum(-1)
    loss = -torch.log(torch.sigmoid(pos - neg) + 1e-8).mean()
    opt.zero_grad(); loss.backward(); opt.step()
    model.eval()
    with torch.no_grad():
        Z1 = model(itf, ei).numpy()
    # sampled eval (np.random stream, eval_neg_k=100 as SURVEY 8(d) cfg 1)
    cfg = types.SimpleNamespace(eval_neg_k=100)
    np.random.seed(7)
    val_metrics = ref.eval_sampled(model, cfg, itf, ei, train_idx, val_idx)

    order_users = np.array(list(train_idx.keys()), dtype=np.int64)
    np.savez_compressed(
        HERE / "plumbing_cfg1.npz",
        user_id=inter["user_id"].to_numpy().astype("U7"), asin=inter["asin"].to_numpy().astype("U10"),
        ts=inter["ts"].to_numpy(), rating=inter["rating"].to_numpy(),
        n_users=np.int64(n_users), n_items=np.int64(n_items),
        train_users=order_users,
        train_lens=np.array([len(train_idx[k]) for k in order_users], np.int64),
        train_items=np.concatenate([train_idx[k] for k in order_users]),
        val_u=np.array(list(val_idx.keys()), np.int64), val_i=np.array(list(val_idx.values()), np.int64),
        test_u=np.array(list(test_idx.keys()), np.int64), test_i=np.array(list(test_idx.values()), np.int64),
        edge_index=ei.numpy(), bpr_u=bu, bpr_i=bi, bpr_j=bj,
        item_feats=feats,
        **{"sd0__" + k: v for k, v in sd0.items()},
        Z0_items=Z0[n_users:], Z0_users=Z0[:n_users], loss1=np.float32(loss.item()), Z1_items=Z1[n_users:],
    )
    with open(HERE / "plumbing_cfg1_eval.json", "w") as f:
        json.dump({"val_metrics_seed7_negk100": val_metrics}, f, indent=2)
    print(f"plumbing: n_users={n_users} n_items={n_items} E={ei.shape[1]} loss1={loss.item():.6f} val={val_metrics}")


def fusion_case():
    """FusionMLP (embeddings/fuse_modal.py:18-36), InfoNCE (:39-72) and the inference
    normalisation (:239-241) of the real reference, imported with inert GCS/Vertex stubs."""
    _stub_gcs()
    spec = importlib.util.spec_from_file_location("ref_fuse_modal", REF / "embeddings" / "fuse_modal.py")
    fm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fm)
    torch.manual_seed(11)
    model = fm.FusionMLP(384, 512, 128, 256)
    rng = np.random.default_rng(11)
    txt = rng.standard_normal((300, 384)).astype(np.float32)
    img = rng.standard_normal((300, 512)).astype(np.float32)
    model.eval()
    with torch.no_grad():
        fused = model(torch.from_numpy(txt), torch.from_numpy(img))
        fused_n = fused / (fused.norm(dim=-1, keepdim=True) + 1e-8)
    # one training-mode loss/grad evaluation with dropout off (RNG streams cannot match)
    model.train()
    model.mlp[2].p = 0.0
    t, im = torch.from_numpy(txt[:256]), torch.from_numpy(img[:256])
    f = model(t, im)
    loss, lt, li = fm.contrastive_fusion_loss(f, model.txt_proj(t), model.img_proj(im))
    loss.backward()
    np.savez_compressed(
        HERE / "fusion_mlp.npz", txt=txt, img=img,
        **{"sd__" + k: v.detach().numpy() for k, v in model.state_dict().items()},
        fused=fused.numpy(), fused_norm=fused_n.numpy(), loss=np.float32(loss.item()), loss_txt=np.float32(lt),
        loss_img=np.float32(li), **{"grad__" + k: p.grad.numpy() for k, p in model.named_parameters()})
    print(f"fusion: loss={loss.item():.6f} keys={list(model.state_dict().keys())}")


def knn_case():
    """graphs/build_ii_knn.py main() on clustered synthetic embeddings, GCS replaced by local
    files (download copies our .npy, uploads are no-ops); the reference's own output npz
    (scipy COO: rows = item, cols = neighbour, data = cosine) becomes the fixture."""
    import os
    import shutil
    import tempfile
    from scipy.sparse import load_npz

    rng = np.random.default_rng(11)
    n, d, n_cl = 2000, 64, 40
    centers = rng.standard_normal((n_cl, d)).astype(np.float32)
    lab = rng.integers(0, n_cl, n)
    emb = (centers[lab] + 0.9 * rng.standard_normal((n, d))).astype(np.float32)
    noisy = rng.random(n) < 0.15  # weakly clustered rows: some of their top-20 fall below 0.3
    emb[noisy] = (0.35 * centers[lab[noisy]] + rng.standard_normal((int(noisy.sum()), d))).astype(np.float32)
    emb[7] = 0.0  # a zero row (norm 0): the reference's +1e-8 guard
    _stub_gcs()
    storage = sys.modules["google.cloud.storage"]

    class _Blob:
        def __init__(self, src):
            self.src = src

        def download_to_filename(self, path):
            shutil.copy(self.src, path)

        def upload_from_filename(self, path):
            pass

    class _Bucket:
        def __init__(self, src):
            self.src = src

        def blob(self, name):
            return _Blob(self.src)

    work = Path(tempfile.mkdtemp())
    np.save(work / "emb.npy", emb)

    class _Client:
        def __init__(self, *a, **k):
            pass

        def bucket(self, name):
            return _Bucket(str(work / "emb.npy"))

    old_client = storage.Client
    storage.Client = _Client
    spec = importlib.util.spec_from_file_location("ref_build_ii_knn", REF / "graphs" / "build_ii_knn.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    argv, cwd = sys.argv, os.getcwd()
    try:
        os.chdir(work)
        sys.argv = ["build_ii_knn.py", "--project-id", "x", "--embeddings-path", "gs://b/emb.npy",
                    "--output-prefix", "gs://b/out", "--output-name", "ii", "--k", "20", "--min-similarity", "0.3",
                    "--batch-size", "300"]
        mod.main()
        m = load_npz(work / "tmp" / "ii.npz").tocoo()
    finally:
        sys.argv = argv
        os.chdir(cwd)
        storage.Client = old_client
        shutil.rmtree(work, ignore_errors=True)
    np.savez_compressed(HERE / "knn_small.npz", emb=emb, rows=m.row.astype(np.int32), cols=m.col.astype(np.int32),
                        sims=m.data.astype(np.float32), k=20, min_sim=0.3)
    print(f"knn: {m.nnz} edges over {n} items")


def main():
    knn_case()
    fusion_case()
    ref = load_reference_custom()
    layer_case(ref, "small_c8", 0, 300, 3000, 8, "uniform")
    layer_case(ref, "uniform_c128", 1, 1200, 12000, 128, "uniform")
    layer_case(ref, "skewed_c128", 2, 1000, 9000, 128, "skewed")
    layer_case(ref, "clamp_c128", 3, 500, 4000, 128, "uniform", x_scale=6.0)
    plumbing_case(ref)


if __name__ == "__main__":
    main()
