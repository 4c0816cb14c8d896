#!/usr/bin/env python3
"""Device-memory budget of one config-5 training step (bench.py's step, eager, one GPU) at a
given scale of the 200M-edge synthetic: torch.cuda.memory_allocated at the phase boundaries of
the multi-head layers (wrapping hip_ops' xgat forward / backward pieces), the live tensors by
role, and the step's peak -- the per-tensor budget behind DESIGN.md section 7's N = 1 figure.

    python tools/mem_probe.py --scale 0.125
"""
import argparse
import importlib
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def gb(x):
    return round(x / 1e9, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.125)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
    O = pkg.hip_ops
    data = pkg.data
    dev = torch.device("cuda", 0)
    log = []

    def mark(what):
        torch.cuda.synchronize()
        log.append((what, gb(torch.cuda.memory_allocated(dev)), gb(torch.cuda.max_memory_allocated(dev))))
        print(f"[mem] {what:48s} alloc {log[-1][1]:8.2f} GB  peak {log[-1][2]:8.2f} GB", flush=True)

    def wrap(mod, name):
        f = getattr(mod, name)

        def w(*a, **k):
            mark(f"> {name}")
            r = f(*a, **k)
            mark(f"< {name}")
            return r
        setattr(mod, name, w)

    for n in ("xgat_forward", "xgat_backward", "_xgat_weight_grads", "gemm_tn_big", "colmax_abs"):
        wrap(O, n)
    g = data.synthetic_scaling_graph(args.scale, seed=42)
    feats_np = data.synthetic_item_features(g.n_items, 256, seed=42)
    ei_np = g.edge_index_numpy()
    E, N = ei_np.shape[1], g.n_nodes
    u, i, j = data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, 200_000, seed=42)
    mark("start")
    ei = torch.from_numpy(ei_np).to(dev)
    feats = torch.from_numpy(feats_np).to(dev)
    tu, ti, tj = (torch.from_numpy(a).to(dev) for a in (u, i, j))
    mark("inputs on device (edge_index int64, features, triples)")
    torch.manual_seed(42)
    model = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=256, hidden=256, layers=2, heads=4, attn_dropout=0.1).to(dev)
    mark("model parameters")
    pkg.graph_cache.get(ei, N)
    mark("CSR / CSC / schedules built")
    opt = pkg.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)
    for s in range(args.steps):
        model.train()
        Z = model(feats, ei)
        mark(f"step {s}: forward done")
        loss = pkg.bpr_loss(Z, g.n_users, tu, ti, tj)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        mark(f"step {s}: backward done")
        opt.step()
        del Z, loss
        mark(f"step {s}: Adam done")
    rec = {"scale": args.scale, "nodes": N, "edges": E, "xgat_agg": os.environ.get("PPGAT_XGAT_AGG", "auto"),
           "peak_gb": gb(torch.cuda.max_memory_allocated(dev)),
           "device_gb": gb(torch.cuda.get_device_properties(dev).total_memory), "marks": log}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
