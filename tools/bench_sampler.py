#!/usr/bin/env python3
"""BPR sampler at config 2 (scripts/train_gat_pyg.py:179-190: 200k triples per epoch over the
192,403-user train lists): device time of ppgat_bpr_sample (kernel events through libppgat's
profiler, one-time prepare reported apart) vs the reference's Python loop
(data.sample_bpr_epoch, the same code path as the reference) on the host."""
import importlib
import json
import random
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")


def main():
    S = 200_000
    g = pkg.data.synthetic_ui_graph()
    dev = torch.device("cuda", 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    smp = pkg.sampler.BPRSampler(g.user_ptr, g.user_items, g.n_items, device=dev)
    torch.cuda.synchronize()
    prep_s = time.perf_counter() - t0
    for _ in range(3):
        smp.sample(S, seed=1, check=False)
    torch.cuda.synchronize()
    pkg._lib.profile_enable(True)
    pkg._lib.profile_reset()
    reps = 20
    t0 = time.perf_counter()
    for r in range(reps):
        smp.sample(S, seed=42, offset=r * S, check=False)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ms, n = pkg._lib.profile_read("sample")
    pkg._lib.profile_enable(False)
    tr = {u: g.user_items[g.user_ptr[u]:g.user_ptr[u + 1]] for u in range(g.n_users)}
    random.seed(42)
    t0 = time.perf_counter()
    pkg.data.sample_bpr_epoch(tr, g.n_items, S)
    cpu_s = time.perf_counter() - t0
    print(json.dumps({"triples": S, "users": g.n_users, "items": g.n_items, "train_interactions": int(g.user_ptr[-1]),
                      "gpu_kernel_us": 1e3 * ms / max(n, 1), "gpu_wall_us_per_epoch": 1e6 * wall,
                      "prepare_ms_once": 1e3 * prep_s, "cpu_reference_loop_s": cpu_s,
                      "speedup_kernel_vs_cpu": cpu_s / (ms / max(n, 1) / 1e3)}))


if __name__ == "__main__":
    main()
