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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=255_404)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
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
