"""The north_star's end-to-end parity claim: final item embeddings after a whole training run.

Golden: ``tests/golden/trajectory_cfg1.{npz,json}``, written by ``make_golden.py trajectory``
from the reference trainer's OWN ``main()`` (scripts/train_gat_custom.py:227-400: 20 epochs
of one 200k-triple BPR batch + Adam(1e-3, wd 1e-4), eval_sampled each epoch with
``--eval-neg-k 100``, best-val checkpoint, reload, test eval, metrics JSON) on the config-1
inputs with the attention dropout at 0, and the export forward of its best checkpoint
(tools/export_item_embeddings.py:136-142).

Here the same run goes through OUR trainer (train.py, ``--model-family gat_custom``, the
host samplers that replay the reference's ``random`` / ``np.random`` streams) and OUR export
tool (export.py), everything on the HIP kernels.  Checked:

1. identical state -> identical embeddings: the reference's best checkpoint through our
   export forward, per item row ``|dZ_i| / |Z_i| <= 1e-5``;
2. the trajectory: per-epoch loss, the best epoch, every epoch's val metrics and the test
   metrics, and the final exported item rows (per row) and every user's top-20.

The trajectory bound is set by the reference itself: its CPU reductions (``index_add_``,
``scatter_add_``, the GEMMs) change order with the thread count and are not even repeatable
at a fixed count, and Adam turns the sign noise of near-zero gradients into lr-sized steps,
so runs of the REFERENCE end apart per item row after 20 epochs.  The fixture holds four
reference runs (torch threads 8, 1, 2, 4): the largest pairwise final item-row spread is the
envelope our run is held to (no multiplier), and every user whose top-20 differs must differ
by less than that envelope in score.  The count of users whose top-20 differ beyond SURVEY.md
8(d)'s 1e-6 near-tie rule is reported next to the same count between reference runs (up to 1
of 1,500 there) and asserted with a slack of 2 users, a tripwire only: it follows the chaotic
final drift; tests/test_gpu_onestep.py is the chaos-free check.  Per-epoch drift (ours and each reference run against the primary run) and
both top-20 rules go to ``gpurun_out/parity/trajectory_cfg1<tag>.json`` (committed under
profiles/); ``PPGAT_REPORT_TAG`` names a variant run (e.g. ``PPGAT_GEMM=fp32``).
"""
import importlib
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT, row_rel, write_report

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _inputs(pkg, root):
    inter = pkg.data.synthetic_interactions_small(seed=0)
    maps = pkg.data.node_maps_from_interactions(inter)
    for d in ("staging", "graphs", "emb"):
        (root / d).mkdir()
    inter.to_parquet(root / "staging" / "interactions.parquet")
    with open(root / "graphs" / "node_maps.json", "w") as f:
        json.dump({k: v for k, v in maps.items() if not k.startswith("idx_to")}, f)
    feats = np.random.RandomState(0).standard_normal((maps["n_items"], 384)).astype(np.float32)
    np.save(root / "emb" / "txt_interacted.npy", feats)
    return maps, feats


def _top20_compare(oracle, Ia, Ua, Ib, Ub, tau):
    """Every user's top-20 by argsort(I @ U[u]) (serving's rule without the
    history mask), fp64 scores from each side's fp32 rows, ties by item index.  A user whose
    lists differ is a near-tie when every differing position's two items are within
    ``tau * max|score|`` on the reference's scores, else a mismatch."""
    Sa = Ua.astype(np.float64) @ Ia.astype(np.float64).T
    Sb = Ub.astype(np.float64) @ Ib.astype(np.float64).T
    exact = near = mism = 0
    worst = 0.0
    for u in range(Sa.shape[0]):
        a, b = oracle.topk_stable(Sa[u], 20), oracle.topk_stable(Sb[u], 20)
        if np.array_equal(a, b):
            exact += 1
            continue
        d = a != b
        gap = float(np.abs(Sb[u, a[d]] - Sb[u, b[d]]).max() / np.abs(Sb[u]).max())
        worst = max(worst, gap)
        if gap < tau:
            near += 1
        else:
            mism += 1
    return exact, near, mism, worst


NEAR_TIE = 1e-6


def test_reference_trajectory_cfg1(pkg, oracle, cuda, tmp_path, capsys, monkeypatch):
    g = dict(np.load(GOLDEN / "trajectory_cfg1.npz"))
    meta = json.loads((GOLDEN / "trajectory_cfg1.json").read_text())
    env = meta["reference_self_spread"]
    spread = env["item_row_rel"]
    envelope = env["envelope_item_row_rel"]
    ref_beyond = max(v["beyond_near_tie_1e-6"] for v in env["pairwise_top20"].values())
    train = importlib.import_module("plotpointe-gat-recommendation_amd.train")
    export = importlib.import_module("plotpointe-gat-recommendation_amd.export")
    maps, feats = _inputs(pkg, tmp_path)
    nu, ni = int(maps["n_users"]), int(maps["n_items"])
    common = ["--staging-prefix", str(tmp_path / "staging"), "--graphs-prefix", str(tmp_path / "graphs"),
              "--embeddings-prefix", str(tmp_path / "emb")]
    rep = {"epochs": 20, "variant": {k: v for k, v in os.environ.items() if k.startswith("PPGAT_")},
           "reference_self_spread_item_row_rel": spread, "reference_envelope_item_row_rel": envelope,
           "reference_pairwise_item_row_rel": env["pairwise_item_row_rel"],
           "reference_pairwise_top20": env["pairwise_top20"]}

    # 1. the reference's best checkpoint through our export forward (identical state)
    ck = tmp_path / "ref_best.pt"
    sd = {k[len("best__"):]: torch.from_numpy(v) for k, v in g.items() if k.startswith("best__")}
    torch.save({"state_dict": sd, "config": meta["config"]}, ck)
    I_fwd = export.main(["--model-family", "gat_custom", "--checkpoint", str(ck), "--item-features", "txt",
                         "--out-local", str(tmp_path / "ref_items.npy")] + common)
    r_fwd, row_fwd, z_fwd = row_rel(I_fwd, g["item_embeddings"])
    rep["forward_same_state"] = {"item_row_rel_max": r_fwd, "worst_row": row_fwd, "zero_rows_max_abs": z_fwd}

    # 2. the whole run through our trainer; the training forward's item rows of every epoch
    # are captured where the loss reads them (the reference fixture records the same rows)
    epoch_items = []
    base_loss = train.model_mod.bpr_loss

    def _loss(Z, n_users, *a, **k):
        epoch_items.append(Z[n_users:].detach().float().cpu().numpy().copy())
        return base_loss(Z, n_users, *a, **k)

    monkeypatch.setattr(train.model_mod, "bpr_loss", _loss)
    capsys.readouterr()
    out = train.main(common + ["--models-prefix", str(tmp_path / "models"), "--model-family", "gat_custom",
                               "--attn-dropout", "0", "--epochs", "20", "--samples-per-epoch", "200000",
                               "--eval-neg-k", "100", "--item-features", "txt", "--seed", "42",
                               "--structured-logs"])
    ev = [json.loads(ln) for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    ours_val = [e["val"] for e in ev if e.get("event") == "epoch_end"]
    ours_loss = np.array([e["loss"] for e in ev if e.get("event") == "epoch_end"])
    ckpt = sorted((tmp_path / "models" / "checkpoints").glob("*.pt"))[-1]
    I = export.main(["--model-family", "gat_custom", "--checkpoint", str(ckpt), "--item-features", "txt",
                     "--out-local", str(tmp_path / "items.npy")] + common)
    m = export.model_from_checkpoint("gat_custom", torch.load(ckpt, weights_only=True), nu, ni, 384).to(cuda).eval()
    d = pkg.data
    u2i, i2i = d.index_maps(maps)
    inter = d.synthetic_interactions_small(seed=0)
    ei = d.build_edge_index(nu, ni, d.map_splits_to_index(*d.build_splits(inter), u2i, i2i)[0]).to(cuda)
    with torch.no_grad():
        U = m(torch.from_numpy(feats).to(cuda), ei)[:nu].cpu().numpy()

    ref_val = meta["val_per_epoch"]
    loss_rel = np.abs(ours_loss - g["loss"]) / np.abs(g["loss"])
    r_items, row_items, z_items = row_rel(I, g["item_embeddings"])
    r_users, _, _ = row_rel(U, g["user_embeddings"])
    ours_best = 1 + int(np.argmax([v["ndcg@20"] for v in ours_val]))
    val_equal = [ours_val[k] == ref_val[k] for k in range(20)]
    val_maxdiff = max(abs(ours_val[k][q] - ref_val[k][q]) for k in range(20) for q in ref_val[k])
    test_maxdiff = max(abs(out["test"][q] - meta["test"][q]) for q in meta["test"])
    kept = env["epochs_kept"]
    drift = {e: row_rel(epoch_items[e - 1], g["epoch_items"][k])[0] for k, e in enumerate(kept)}
    ref_drift = {n: {e: c[e - 1] for e in kept} for n, c in env["per_epoch_item_row_rel_vs_primary"].items()}
    exact, near, beyond, worst_gap = _top20_compare(oracle, I, U, g["item_embeddings"], g["user_embeddings"],
                                                    NEAR_TIE)
    tau = envelope
    _, near_env, mism_env, _ = _top20_compare(oracle, I, U, g["item_embeddings"], g["user_embeddings"], tau)
    rep.update({
        "loss_rel_max": float(loss_rel.max()), "loss_rel_epoch1": float(loss_rel[0]),
        "best_epoch": {"ours": ours_best, "reference": meta["best_epoch"]},
        "val_epochs_equal": int(sum(val_equal)), "val_max_abs_diff": val_maxdiff,
        "test": {"ours": out["test"], "reference": meta["test"], "max_abs_diff": test_maxdiff},
        "item_row_rel_max": r_items, "item_worst_row": row_items, "item_zero_rows_max_abs": z_items,
        "item_row_rel_over_reference_spread": r_items / spread,
        "item_row_rel_over_reference_envelope": r_items / envelope, "user_row_rel_max": r_users,
        "per_epoch_item_row_rel_vs_reference": {"ours": drift, **ref_drift},
        "top20": {"users": nu, "exact": exact, "worst_gap_rel": worst_gap,
                  "rule_1e-6": {"near_tie": near, "beyond": beyond,
                                "reference_pairs_max_beyond": ref_beyond},
                  "rule_envelope": {"tau": tau, "near_tie": near_env, "mismatched": mism_env}},
    })
    # our top-20 against every reference run (same 1e-6 rule): is our run one more draw from
    # the reference's own run-to-run distribution?
    rep["top20"]["rule_1e-6"]["vs_each_reference_run"] = {
        n: _top20_compare(oracle, I, U, g[f"{n}__item_embeddings"], g[f"{n}__user_embeddings"], NEAR_TIE)[2]
        for n in env["threads"][1:]}
    rep["item_row_rel_vs_each_reference_run"] = {
        n: row_rel(I, g[f"{n}__item_embeddings"])[0] for n in env["threads"][1:]}
    tag = os.environ.get("PPGAT_REPORT_TAG", "")
    name = "trajectory_cfg1" + (f"_{tag}" if tag else "")
    write_report(name, rep)
    np.savez_compressed(ROOT / "gpurun_out" / "parity" / f"{name}_rows.npz", items=I, users=U,
                        epoch_items=np.stack(epoch_items))
    assert r_fwd <= 1e-5 and z_fwd == 0.0, rep["forward_same_state"]
    assert loss_rel[0] <= 1e-6, loss_rel[0]          # identical initial state
    assert loss_rel.max() <= 1e-5, loss_rel
    assert ours_best == meta["best_epoch"]
    # one rank flip of one of the 1,500 validation users moves recall@K by 1/1500 and ndcg by less
    assert val_maxdiff <= 1.0 / 1500 + 1e-12 and test_maxdiff <= 1.0 / 1500 + 1e-12, rep
    assert z_items == 0.0
    assert r_items <= envelope, (r_items, envelope)
    # every user whose top-20 differs does so by less than the reference's own run-to-run
    # spread
    assert mism_env == 0, rep["top20"]
    # SURVEY 8(d)'s 1e-6 rule: after 20 chaotic Adam epochs the reference runs themselves
    # differ beyond it (up to ref_beyond users between two of them), so our run -- one more
    # draw -- is held to that count plus a stated slack of 2 users (measured: 2 against the
    # primary run on the default path, 0 with PPGAT_FUSED_DXW=0, profiles/r04/parity).  This
    # is a regression tripwire; the precise training-step check is test_gpu_onestep.py, which
    # starts from the reference's own saved states and has no chaotic amplification.
    assert beyond <= ref_beyond + 2, rep["top20"]["rule_1e-6"]
