#!/usr/bin/env python3
"""eval_sampled at config 2 (scripts/train_gat_pyg.py:150-176): the reference's host loop
(its np.random rejection draw per user, evaluation.sample_eval_candidates) timed on a
bounded sample of users and scaled, against the device path (ppgat_eval_sample +
ppgat_sampled_rank) over every evaluated user, 1000 negatives each."""
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")


def main():
    d = pkg.data
    dev = torch.device("cuda", 0)
    g = d.synthetic_ui_graph(seed=42)
    users = np.flatnonzero(g.val_item >= 0)
    pos = g.val_item[users]
    Z = torch.randn(g.n_nodes, 128, device=dev)
    s = pkg.sampler.BPRSampler(g.user_ptr, g.user_items, g.n_items, device=dev)
    tu, tp = torch.from_numpy(users).to(dev), torch.from_numpy(pos).to(dev)
    for _ in range(2):
        c = s.eval_candidates(tu, tp, 1000, seed=1)
        r = pkg.evaluation.sampled_rank(Z, g.n_users, tu, c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for k in range(reps):
        c = s.eval_candidates(tu, tp, 1000, seed=k, check=False)
        r = pkg.evaluation.sampled_rank(Z, g.n_users, tu, c)
    torch.cuda.synchronize()
    t_dev = (time.perf_counter() - t0) / reps
    # host: the reference's draw for a sample of users, scaled to all of them
    sample = 2000
    tr = {int(u): g.user_items[g.user_ptr[u]:g.user_ptr[u + 1]] for u in users[:sample]}
    ev = {int(u): int(p) for u, p in zip(users[:sample], pos[:sample])}
    np.random.seed(0)
    t0 = time.perf_counter()
    pkg.evaluation.sample_eval_candidates(tr, ev, g.n_items, 1000)
    t_host = (time.perf_counter() - t0) * len(users) / sample
    print(json.dumps({"users": int(len(users)), "negatives": 1000, "device_s": t_dev,
                      "host_reference_draw_s_scaled": t_host, "host_sample_users": sample,
                      "speedup": t_host / t_dev}), flush=True)


if __name__ == "__main__":
    main()
