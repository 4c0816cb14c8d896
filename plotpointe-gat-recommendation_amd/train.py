"""Trainer counterpart of scripts/train_gat_pyg.py / scripts/train_gat_custom.py main().

Same flags, seeds, split/edge-index/sampler code paths, epoch structure (one large BPR
batch per epoch, eval each epoch, best-val checkpoint, reload, test), metrics-JSON schema
``{"best_val_ndcg@20", "val", "test", "config", "notes"}`` and optional JSONL events
(``run_start`` / ``epoch_end`` / ``run_complete``, plotpointe/utils/structured_log.py:19-38).
GCS is out of scope: the ``--*-prefix`` flags name LOCAL directories holding the same file
names (interactions.parquet, node_maps.json, {fused,txt}_interacted.npy); outputs go to
``{models_prefix}/checkpoints/{run_id}.pt`` and ``{models_prefix}/metrics_{run_id}.json``.
``--synthetic cfg1|cfg2`` builds the SURVEY.md 8(d) stand-in inputs instead.

    python -m plotpointe_gat_amd.train ...   (or: python plotpointe-gat-recommendation_amd/train.py ...)
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Optional

import numpy as np
import torch

if __package__ in (None, ""):  # executed as a file
    import importlib
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    _pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
    data, evaluation, model_mod = _pkg.data, importlib.import_module(_pkg.__name__ + ".evaluation"), _pkg.model
    sampler_mod = _pkg.sampler
else:
    from . import data, evaluation
    from . import model as model_mod
    from . import sampler as sampler_mod


def set_seed(seed: int):
    """train_gat_pyg.py:39-43."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


def enable_determinism(seed: Optional[int] = None):
    """plotpointe/utils/random.py:23-44 (our kernels are deterministic regardless)."""
    if seed is not None:
        set_seed(seed)
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":16:8")
    try:
        torch.use_deterministic_algorithms(True, warn_only=True)
    except Exception:
        pass


def log_event(event: str, run_id: Optional[str] = None, **fields: Any) -> Dict[str, Any]:
    """plotpointe/utils/structured_log.py:19-38."""
    rec: Dict[str, Any] = {"ts": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "event": event}
    if run_id:
        rec["run_id"] = run_id
    rec.update(fields)
    try:
        sys.stdout.write(json.dumps(rec) + os.linesep)
        sys.stdout.flush()
    except Exception:
        pass
    return rec


@dataclass
class Config:
    """train_gat_pyg.py:46-65 (+ model_family, attn_dropout exposed)."""
    project_id: str
    region: str
    staging_prefix: str
    graphs_prefix: str
    embeddings_prefix: str
    models_prefix: str
    hidden_dim: int = 128
    layers: int = 2
    heads: int = 1
    attn_dropout: float = 0.1
    lr: float = 1e-3
    l2: float = 1e-4
    epochs: int = 20
    samples_per_epoch: int = 200_000
    seed: int = 42
    eval_neg_k: int = 1000
    item_features: str = "fused"
    loss: str = "bpr"
    model_family: str = "gat_pyg"


def _local(prefix: str) -> Path:
    if prefix.startswith("gs://"):
        raise ValueError(f"{prefix}: GCS is out of scope here; pass a local directory")
    return Path(prefix)


def load_inputs(cfg: Config, synthetic: Optional[str]):
    """-> (train_pos_idx, val_pos_idx, test_pos_idx, n_users, n_items, item_feats np)"""
    if synthetic:
        if synthetic == "cfg1":
            inter = data.synthetic_interactions_small(seed=0)
        elif synthetic == "cfg2":
            g = data.synthetic_ui_graph(seed=42)
            val = {u: int(v) for u, v in enumerate(g.val_item.tolist()) if v >= 0}
            test = {u: int(v) for u, v in enumerate(g.test_item.tolist()) if v >= 0}
            dim = 128 if cfg.item_features == "fused" else 384
            return g.train_pos_idx(), val, test, g.n_users, g.n_items, data.synthetic_item_features(g.n_items, dim)
        else:
            raise ValueError(synthetic)
        maps = data.node_maps_from_interactions(inter)
        feats = np.random.RandomState(0).standard_normal((maps["n_items"], 384)).astype(np.float32)
    else:
        import pandas as pd
        inter = pd.read_parquet(_local(cfg.staging_prefix) / "interactions.parquet")
        with open(_local(cfg.graphs_prefix) / "node_maps.json") as f:
            maps = json.load(f)
        feat_name = "fused_interacted.npy" if cfg.item_features == "fused" else "txt_interacted.npy"
        feats = np.load(_local(cfg.embeddings_prefix) / feat_name)
    u2i, i2i = data.index_maps(maps)
    tr, va, te = data.map_splits_to_index(*data.build_splits(inter), u2i, i2i)
    return tr, va, te, int(maps["n_users"]), int(maps["n_items"]), feats


def build_model(cfg: Config, n_users: int, n_items: int, feat_dim: int):
    if cfg.model_family == "gat_pyg":
        return model_mod.PyGGAT(n_users, n_items, item_feat_dim=feat_dim, hidden=cfg.hidden_dim, layers=cfg.layers,
                                heads=cfg.heads, attn_dropout=cfg.attn_dropout)
    m = model_mod.CustomGAT(n_users, n_items, item_feat_dim=feat_dim, hidden=cfg.hidden_dim, layers=cfg.layers)
    for layer in m.layers:
        layer.drop.p = cfg.attn_dropout
    return m


def epoch_step(model, opt, item_feats, edge_index, n_users: int, u, i, j, loss: str = "bpr"):
    """One epoch's optimisation step on one GPU (train_gat_custom.py:349-362, identical
    train_gat_pyg.py:307-323): the training forward over the whole graph, the BPR/BCE loss of
    the epoch's sampled triples, zero_grad, backward, ``opt.step()``.  Returns the loss.
    ``PPGAT_BPR_OVERLAP=1`` starts the loss backward's triple sort (it needs the triples only)
    on a side stream before the forward (hip_ops.bpr_prepare; measured no faster at config 2,
    DESIGN.md section 4)."""
    prep = None
    if os.environ.get("PPGAT_BPR_OVERLAP", "0") == "1":
        C = model.user_emb.weight.size(1)
        prep = model_mod.hip_ops.bpr_prepare(n_users + model.n_items, n_users, model.n_items, C, u, i, j)
    Z = model(item_feats, edge_index)
    lo = model_mod.bpr_loss(Z, n_users, u, i, j, loss, prepared=prep)
    opt.zero_grad()
    lo.backward()
    opt.step()
    return lo


class _GlobalRows(torch.nn.Module):
    """A row-sharded model seen as the single-GPU one by eval_sampled / export: forward returns
    every node's rows on every rank (an all_gather; evaluation only, not the training path)."""

    def __init__(self, sharded, to_global):
        super().__init__()
        self.sharded, self.to_global = sharded, to_global
        self.n_users, self.n_items = sharded.n_users, sharded.n_items

    def forward(self, item_feats, edge_index=None):
        return self.to_global(self.sharded(item_feats), self.sharded.dg, self.sharded.comm)


def _init_distributed(args):
    """torch.distributed from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*): one
    process per GPU; several ranks may share a GPU (gloo tests)."""
    import torch.distributed as tdist
    world = int(os.environ.get("WORLD_SIZE", args.world_size))
    if world != args.world_size:
        raise RuntimeError(f"--world-size {args.world_size} but WORLD_SIZE={world} (launch with torchrun)")
    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", rank))
    device = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(device)
    kw = {"device_id": device} if args.backend == "nccl" else {}
    tdist.init_process_group(args.backend, rank=rank, world_size=world, **kw)
    return rank, world, device


def main(argv=None):
    ap = argparse.ArgumentParser(description="Train GAT (MI355X-native)")
    ap.add_argument("--project-id", default="local")
    ap.add_argument("--region", default="us-central1")
    ap.add_argument("--staging-prefix", default="data/staging")
    ap.add_argument("--graphs-prefix", default="data/graphs")
    ap.add_argument("--embeddings-prefix", default="data/embeddings")
    ap.add_argument("--models-prefix", default="models/gat")
    ap.add_argument("--model-family", choices=["gat_pyg", "gat_custom"], default="gat_pyg")
    ap.add_argument("--hidden-dim", type=int, default=128)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--heads", type=int, default=1)
    ap.add_argument("--attn-dropout", type=float, default=0.1)
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--samples-per-epoch", type=int, default=200_000)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--eval-neg-k", type=int, default=1000)
    ap.add_argument("--item-features", choices=["fused", "txt"], default="fused")
    ap.add_argument("--loss", choices=["bpr", "bce"], default="bpr")
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--structured-logs", action="store_true")
    ap.add_argument("--fast-eval", action="store_true", help="vectorised negative sampling (same distribution)")
    ap.add_argument("--device-eval", action="store_true",
                    help="eval candidates drawn on the GPU (ppgat_eval_sample: same rule, counter-based stream)")
    ap.add_argument("--fast-sampler", action="store_true",
                    help="BPR triples drawn on the GPU (ppgat_bpr_sample: same rule, counter-based stream)")
    ap.add_argument("--synthetic", choices=["cfg1", "cfg2"], default=None)
    ap.add_argument("--world-size", type=int, default=1,
                    help="ranks (one process per GPU, launched by torchrun); > 1 shards the model (dist.py)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend (nccl = RCCL on ROCm; gloo only for tests)")
    ap.add_argument("--partition", choices=["auto", "replicated", "halo"], default="auto",
                    help="auto: users sharded / items replicated for U-I graphs, halo otherwise")
    args = ap.parse_args(argv)
    cfg = Config(project_id=args.project_id, region=args.region, staging_prefix=args.staging_prefix,
                 graphs_prefix=args.graphs_prefix, embeddings_prefix=args.embeddings_prefix,
                 models_prefix=args.models_prefix, hidden_dim=args.hidden_dim, layers=args.layers, heads=args.heads,
                 attn_dropout=args.attn_dropout, epochs=args.epochs, samples_per_epoch=args.samples_per_epoch,
                 seed=args.seed, eval_neg_k=args.eval_neg_k, item_features=args.item_features, loss=args.loss,
                 model_family=args.model_family)
    if args.deterministic:
        enable_determinism(cfg.seed)
    set_seed(cfg.seed)
    if not torch.cuda.is_available():
        raise RuntimeError("this trainer runs the HIP kernels: a ROCm GPU is required")
    rank, world, device = 0, 1, torch.device("cuda")
    if args.world_size > 1:
        if cfg.model_family != "gat_pyg":
            raise NotImplementedError("--world-size > 1: the sharded model is PyGGAT (--model-family gat_pyg)")
        rank, world, device = _init_distributed(args)
    lead = rank == 0
    tag = "GAT-PYG" if cfg.model_family == "gat_pyg" else "GAT-CUSTOM"
    run_id = f"{cfg.model_family}_d{cfg.hidden_dim}_{int(time.time())}"
    if world > 1:  # one run id (checkpoint / metrics names) for every rank: rank 0's
        import torch.distributed as tdist
        ids = [run_id]
        tdist.broadcast_object_list(ids, src=0)
        run_id = ids[0]
    if args.structured_logs:
        log_event("run_start", run_id=run_id, model_family=cfg.model_family,
                  config={**cfg.__dict__, "device": str(device)})
    tr, va, te, n_users, n_items, feats_np = load_inputs(cfg, args.synthetic)
    print(f"[{tag}] n_users={n_users}, n_items={n_items}")
    edge_index = data.build_edge_index(n_users, n_items, tr).to(device)
    item_feats = torch.tensor(feats_np, dtype=torch.float32).to(device)
    assert item_feats.shape[0] == n_items
    model = build_model(cfg, n_users, n_items, item_feats.size(1)).to(device)
    sharded = None
    if world > 1:
        # every rank built the same full model (same seed); each keeps its shard
        import importlib
        dist_mod = importlib.import_module(model_mod.__name__.rsplit(".", 1)[0] + ".dist")
        comm = dist_mod.Comm()
        part = args.partition
        if part == "auto":
            part = "replicated"
        if part == "replicated":
            dg = dist_mod.build_replicated_graph(edge_index, n_users + n_items, n_users, world, rank)
            sharded = dist_mod.ReplicatedPyGGAT(model, dg, comm)
            loss_fn, to_global = dist_mod.replicated_bpr_loss, dist_mod.replicated_rows_to_global
        else:
            dg = dist_mod.build_halo_graph(edge_index, n_users + n_items, n_users, world, rank)
            sharded = dist_mod.HaloPyGGAT(model, dg, comm)
            loss_fn, to_global = dist_mod.halo_bpr_loss, dist_mod.halo_rows_to_global
        eval_model = _GlobalRows(sharded, to_global)
        opt = torch.optim.Adam(sharded.parameters(), lr=cfg.lr, weight_decay=cfg.l2)
    else:
        eval_model = model
        opt = torch.optim.Adam(model.parameters(), lr=cfg.lr, weight_decay=cfg.l2)
    out_dir = _local(cfg.models_prefix)
    (out_dir / "checkpoints").mkdir(parents=True, exist_ok=True)
    best_path = out_dir / "checkpoints" / f"{run_id}.pt"
    metrics_path = out_dir / f"metrics_{run_id}.json"
    best = -1.0
    val_metrics: Dict[str, float] = {}
    dev_sampler = None
    if args.fast_sampler or args.device_eval:
        lens = np.array([len(tr.get(uu, ())) for uu in range(n_users)], dtype=np.int64)
        ptr = np.concatenate([[0], np.cumsum(lens)])
        flat = np.concatenate([np.asarray(tr[uu], dtype=np.int64) for uu in range(n_users) if lens[uu]] or
                              [np.zeros(0, dtype=np.int64)])
        dev_sampler = sampler_mod.BPRSampler(ptr, flat, n_items, device=device)
    for epoch in range(1, cfg.epochs + 1):
        model.train()
        if args.fast_sampler:
            u, i, j = dev_sampler.sample(cfg.samples_per_epoch, seed=cfg.seed,
                                         offset=(epoch - 1) * cfg.samples_per_epoch)
        else:
            u_arr, i_arr, j_arr = data.sample_bpr_epoch(tr, n_items, cfg.samples_per_epoch)
            u = torch.from_numpy(u_arr).long().to(device)
            i = torch.from_numpy(i_arr).long().to(device)
            j = torch.from_numpy(j_arr).long().to(device)
        if sharded is None:
            loss_val = float(epoch_step(model, opt, item_feats, edge_index, n_users, u, i, j, cfg.loss).item())
        else:
            # each rank: its own users' triples (the sum over ranks is the reference's mean),
            # dense gradients all-reduced, user rows updated by their owner
            sharded.train()
            Zl = sharded(item_feats)
            loss = loss_fn(Zl, sharded.dg, sharded.comm, u, i, j, n_users, n_items, loss=cfg.loss,
                           plan_key=epoch)  # one triple draw per epoch, the same epoch on every rank
            opt.zero_grad()
            loss.backward()
            sharded.allreduce_grads()
            opt.step()
            tot = loss.detach().clone()
            sharded.comm.all_reduce_(tot)
            loss_val = float(tot.item())
        if lead:
            print(f"[{tag}][Epoch {epoch}] loss={loss_val:.4f} ({cfg.loss})")
        eval_model.eval()
        val_metrics = evaluation.eval_sampled(eval_model, cfg, item_feats, edge_index, tr, va, fast=args.fast_eval,
                                              sampler=dev_sampler if args.device_eval else None,
                                              seed=cfg.seed + epoch)
        if lead:
            print(f"[{tag}][Epoch {epoch}] val: {val_metrics}")
        if args.structured_logs and lead:
            log_event("epoch_end", run_id=run_id, epoch=epoch, loss=loss_val, val=val_metrics)
        if val_metrics.get("ndcg@20", 0.0) > best:
            best = val_metrics.get("ndcg@20", 0.0)
            sd = model.state_dict() if sharded is None else sharded.full_state_dict()  # collective when sharded
            if lead:
                torch.save({"state_dict": sd, "config": cfg.__dict__}, best_path)
                print(f"[{tag}] Saved new best checkpoint")
    if world > 1:
        import torch.distributed as tdist
        tdist.barrier()  # rank 0's checkpoint is on disk
    ckpt = torch.load(best_path, map_location=device, weights_only=True)
    model.load_state_dict(ckpt["state_dict"])
    if sharded is not None:
        with torch.no_grad():
            ids = torch.as_tensor(sharded.dg.own_user_ids(), dtype=torch.int64, device=model.user_emb.weight.device)
            sharded.user_emb_local.copy_(model.user_emb.weight.index_select(0, ids))
    eval_model.eval()
    test_metrics = evaluation.eval_sampled(eval_model, cfg, item_feats, edge_index, tr, te, fast=args.fast_eval,
                                           sampler=dev_sampler if args.device_eval else None, seed=cfg.seed)
    if lead:
        print(f"[{tag}] test: {test_metrics}")
    out = {"best_val_ndcg@20": float(best), "val": val_metrics, "test": test_metrics, "config": cfg.__dict__,
           "notes": f"One-backward-per-epoch with S sampled BPR triples; features={cfg.item_features}; "
                    f"loss={cfg.loss}"}
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()
        if not lead:
            return out
    with open(metrics_path, "w") as f:
        json.dump(out, f, indent=2)
    print(f"[{tag}] Complete. Wrote {best_path} and {metrics_path}")
    if args.structured_logs:
        log_event("run_complete", run_id=run_id, best_val_ndcg20=float(best), test=test_metrics,
                  artifacts={"checkpoint": str(best_path), "metrics": str(metrics_path)})
    return out


if __name__ == "__main__":
    main()
