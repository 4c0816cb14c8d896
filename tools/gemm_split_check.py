#!/usr/bin/env python3
"""Projection GEMMs at config-2 shapes (N = 255,404, 128 x 128): accuracy against fp64 and
per-call time (HIP events) of whichever kernel family PPGAT_GEMM selects (default: the split
bf16 matrix-core kernels; PPGAT_GEMM=fp32: the fp32 MFMA kernels).  Run it once per setting.
Error = max |y - y64| / max |y64| over the output (the tests' max-abs/max-abs measure)."""
import argparse
import importlib
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
ops = pkg.hip_ops
lib = pkg._lib.load()


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def rel(a, b):
    return float((a.double() - b).abs().max() / b.abs().max())


def cfg5(dev, iters):
    """Config-5 share shapes (M = 1.875M rows): out = agg W_t ([M, 1024] x [1024, 256]) and
    gt = g W_g ([M, 256] x [256, 1024]) through ppgat_gemm_nn (both B layouts), and the weight
    gradient G = g^T agg ([M, 256]^T [M, 1024], ppgat_gemm_tn_big); errors vs fp64 on 4096
    sampled rows (NN) and on the whole product (TN)."""
    M = 1_875_000
    g = torch.Generator(device=dev).manual_seed(0)
    out = {"mode": os.environ.get("PPGAT_GEMM", "split"), "cfg": 5}
    rows = torch.randint(0, M, (4096,), device=dev, generator=g)
    for name, K, Nc in (("out_1024x256", 1024, 256), ("gt_256x1024", 256, 1024)):
        X = torch.randn(M, K, device=dev, generator=g)
        B0 = torch.randn(K, Nc, device=dev, generator=g) * 0.05
        B1 = B0.t().contiguous()
        y0 = ops.gemm_nn(X, B0, 0, Nc)
        y1 = ops.gemm_nn(X, B1, 1, Nc)
        out[f"{name}_layouts_equal"] = bool(torch.equal(y0, y1))
        out[f"{name}_err"] = rel(y0[rows], X[rows].double() @ B0.double())
        for lay, B in ((0, B0), (1, B1)):
            us = timeit(lambda: ops.gemm_nn(X, B, lay, Nc, out=y0), iters)
            out[f"{name}_layout{lay}_us"] = us
            out[f"{name}_layout{lay}_tflops"] = 2.0 * M * K * Nc / us / 1e6
        del X, y0, y1
    A = torch.randn(M, 256, device=dev, generator=g)
    Bt = torch.randn(M, 1024, device=dev, generator=g)
    G = ops.gemm_tn_big(A, Bt)
    out["tn_big_err"] = rel(G, A.double().t() @ Bt.double())
    us = timeit(lambda: ops.gemm_tn_big(A, Bt), iters)
    out["tn_big_us"] = us
    out["tn_big_tflops"] = 2.0 * M * 256 * 1024 / us / 1e6
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=255_404)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfg5", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.cfg5:
        return cfg5(dev, max(3, args.iters // 4))
    N, K = args.n, args.k
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, K, device=dev, generator=g)
    W = torch.randn(128, K, device=dev, generator=g) * 0.1
    b = torch.randn(128, device=dev, generator=g)
    a_s = torch.randn(128, device=dev, generator=g)
    a_d = torch.randn(128, device=dev, generator=g)
    D = torch.randn(N, 128, device=dev, generator=g)
    S = torch.randn(N, 2, device=dev, generator=g)
    Wd = torch.randn(128, 128, device=dev, generator=g) * 0.1
    dx = torch.empty(N, 128, device=dev)
    st = pkg._lib.stream_handle(dev)
    out = {"mode": os.environ.get("PPGAT_GEMM", "split"), "n": N, "k": K}

    y, s1, s2 = ops.project(x, W, att_src=a_s, att_dst=a_d)
    y64 = x.double() @ W.double().t()
    out["fwd_err"] = rel(y, y64)
    out["s_src_err"] = rel(s1, y64 @ a_s.double())
    out["s_dst_err"] = rel(s2, y64 @ a_d.double())
    yb = ops.project(x, W, bias=b)
    out["fwd_bias_err"] = rel(yb, y64 + b.double())

    def run_dx():
        pkg._lib.check(lib.ppgat_project_bwd_input(D.data_ptr(), 128, N, 128, Wd.data_ptr(), 128, 128, a_s.data_ptr(),
                                                   a_d.data_ptr(), S.data_ptr(), 2, dx.data_ptr(), 128, st), "dx")
    run_dx()
    torch.cuda.synchronize()
    A_s = a_s.double() @ Wd.double()
    A_d = a_d.double() @ Wd.double()
    dx64 = D.double() @ Wd.double() + S[:, :1].double() * A_s + S[:, 1:].double() * A_d
    out["dx_err"] = rel(dx, dx64)
    # bitwise repeatability
    y2, _, _ = ops.project(x, W, att_src=a_s, att_dst=a_d)
    out["fwd_bitwise_repeat"] = bool(torch.equal(y, y2))

    # weight gradient D^T x (+ V^T x, colsum D), full 128 x 128 and a masked shape
    G, cs, GV = ops.gemm_tn(D, x, want_colsum=True, V=S)
    out["tn_err"] = rel(G, D.double().t() @ x.double())
    out["tn_v_err"] = rel(GV, S.double().t() @ x.double())
    out["tn_colsum_err"] = rel(cs, D.double().sum(0))
    Gm, _, _ = ops.gemm_tn(D[:, :64], x[:, :96])
    out["tn_masked_err"] = rel(Gm, D[:, :64].double().t() @ x[:, :96].double())
    Gs, _, _ = ops.gemm_tn(D[:1001], x[:1001])
    out["tn_small_err"] = rel(Gs, D[:1001].double().t() @ x[:1001].double())

    out["us_fwd_scores"] = timeit(lambda: ops.project(x, W, att_src=a_s, att_dst=a_d), args.iters)
    out["us_dx"] = timeit(run_dx, args.iters)
    out["us_tn_V"] = timeit(lambda: ops.gemm_tn(D, x, V=S), args.iters)
    flop = 2 * N * 128 * K
    out["tflops_fwd_fp32_equiv"] = flop / out["us_fwd_scores"] / 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()
