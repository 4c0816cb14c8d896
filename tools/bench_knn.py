#!/usr/bin/env python3
"""I-I kNN build at config-3 size (graphs/build_ii_knn.py on 63,001 items x 128-d fused
embeddings, k=20, min_similarity 0.3): GPU time of ppgat_amd.knn.build_ii_knn vs the CPU
oracle (the reference's own numpy/sklearn loop, oracle/knn_oracle.py) timed on a sample of
query rows and scaled to all rows.  The reference's published CPU time for this step is
78-100 s (docs/PHASE0_REPORT.md:183,193)."""
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
    n, d, k = 63_001, 128, 20
    rng = np.random.default_rng(42)
    centers = rng.standard_normal((2000, d)).astype(np.float32)
    emb = (centers[rng.integers(0, 2000, n)] + 1.2 * rng.standard_normal((n, d))).astype(np.float32)
    dev = torch.device("cuda", 0)
    e = torch.from_numpy(emb).to(dev)
    for _ in range(2):
        pkg.knn.build_ii_knn(e, k=k, min_similarity=0.3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        rows, cols, sims = pkg.knn.build_ii_knn(e, k=k, min_similarity=0.3)
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / reps
    from oracle import knn_oracle
    sample = 2000
    t0 = time.perf_counter()
    knn_oracle.ii_knn(emb[:sample], k, 0.3)  # note: sample x sample, scaled by n^2 below
    cpu_small = time.perf_counter() - t0
    cpu_est = cpu_small * (n / sample) ** 2
    print(json.dumps({"items": n, "dim": d, "k": k, "edges": int(rows.numel()), "gpu_s": gpu_s,
                      "gpu_tflops_sim_gemm": 2.0 * n * n * d / gpu_s / 1e12,
                      "cpu_oracle_s_scaled_from_2000x2000": cpu_est, "reference_published_cpu_s": "78-100"}))


if __name__ == "__main__":
    main()
