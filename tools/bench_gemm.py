#!/usr/bin/env python3
"""Micro-benchmark of the projection / weight-gradient GEMMs at config-2 shapes
(N = 255,404 rows, 128 x 128), each launched `--iters` times; prints per-call
microseconds (HIP events) next to the library GEMM (torch / hipBLASLt) on the same shape."""
import argparse
import importlib
import json
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=255_404)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--cfg5", action="store_true", help="config-5 share shapes of ppgat_gemm_nn, both B layouts")
    ap.add_argument("--tn5", action="store_true", help="config-5 weight gradient G = g^T agg (ppgat_gemm_tn_big)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.cfg5:
        return cfg5(dev, args.iters)
    if args.tn5:
        M = 1_875_000
        g = torch.Generator(device=dev).manual_seed(0)
        A = torch.randn(M, 256, device=dev, generator=g)
        B = torch.randn(M, 1024, device=dev, generator=g)
        us = timeit(lambda: ops.gemm_tn_big(A, B), args.iters)
        print(json.dumps({"tn_big_us": us, "tflops": 2.0 * M * 256 * 1024 / us / 1e6}))
        return
    N = args.n
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, 128, device=dev, generator=g)
    W = torch.randn(128, 128, device=dev, generator=g)
    a_s = torch.randn(128, device=dev, generator=g)
    a_d = torch.randn(128, device=dev, generator=g)
    D = torch.randn(N, 128, device=dev, generator=g)
    S = torch.randn(N, 2, device=dev, generator=g)
    dx = torch.empty(N, 128, device=dev)
    st = pkg._lib.stream_handle(dev)
    res = {}
    import ctypes
    nb = ctypes.c_size_t(0)
    pkg._lib.check(lib.ppgat_project_bwd_fused_workspace_bytes(N, ctypes.byref(nb)), "ws")
    ws = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
    G = torch.empty(128, 128, device=dev)
    GV = torch.empty(2, 128, device=dev)

    def fused_dxw():  # dx + D^T x + S^T x in one pass (ppgat_project_bwd_fused)
        pkg._lib.check(lib.ppgat_project_bwd_fused(D.data_ptr(), 128, S.data_ptr(), 2, x.data_ptr(), 128, None, 128, N,
                                                   N, 128, W.data_ptr(), 128, a_s.data_ptr(), a_d.data_ptr(),
                                                   dx.data_ptr(), 128, G.data_ptr(), GV.data_ptr(), ws.data_ptr(),
                                                   nb.value, st), "fused")
    cases = {
        "proj_fwd_scores": lambda: ops.project(x, W, att_src=a_s, att_dst=a_d),
        "proj_dx": lambda: pkg._lib.check(lib.ppgat_project_bwd_input(D.data_ptr(), 128, N, 128, W.data_ptr(), 128, 128,
                                                                      a_s.data_ptr(), a_d.data_ptr(), S.data_ptr(), 2,
                                                                      dx.data_ptr(), 128, st), "dx"),
        "fused_dxw": lambda: fused_dxw(),
        "nn_fwd": lambda: ops.gemm_nn(x, W, 1, 128),
        "nn_dx": lambda: ops.gemm_nn(D, W, 0, 128),
        "tn_dW_V": lambda: ops.gemm_tn(D, x, V=S),
        "tn_plain": lambda: ops.gemm_tn(D, x),
        "blas_fwd": lambda: torch.nn.functional.linear(x, W),
        "blas_dx": lambda: D @ torch.randn(128, 128, device=dev),
    }
    for k, fn in cases.items():
        if args.only and k not in args.only.split(","):
            continue
        res[k] = timeit(fn, args.iters)
    flop = 2 * N * 128 * 128
    out = {k: {"us": v, "tflops": flop / v / 1e6} for k, v in res.items()}
    if hasattr(lib, "ppgat_debug_clock_mhz"):  # diagnostic build (-DPPGAT_CLOCK_PROBE=1)
        import ctypes
        lib.ppgat_debug_clock_mhz.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        for slot, name in ((0, "proj16"), (1, "tn128")):
            mhz = ctypes.c_double(0.0)
            if lib.ppgat_debug_clock_mhz(slot, 4096, ctypes.byref(mhz)) == 0:
                out[f"clock_mhz_{name}"] = mhz.value
    print(json.dumps(out, indent=1))


def cfg5(dev, iters):
    """out = agg W_t / H ([1.875M, 1024] x [1024, 256]) and gt = g W_g ([1.875M, 256] x [256, 1024]),
    B given as [K][N] (layout 0) or as its transpose [N][K] (layout 1)."""
    M = 1_875_000
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, K, Nc in (("out_1024x256", 1024, 256), ("gt_256x1024", 256, 1024)):
        X = torch.randn(M, K, device=dev, generator=g)
        B0 = torch.randn(K, Nc, device=dev, generator=g)
        B1 = B0.t().contiguous()
        y0 = ops.gemm_nn(X, B0, 0, Nc)
        y1 = ops.gemm_nn(X, B1, 1, Nc)
        import os
        if not os.environ.get("PPGAT_NNH2_LAB"):  # the lab variants' outputs are not the product
            assert torch.equal(y0, y1), name  # same products, same order
        # fingerprint of the exact bits (compare runs with PPGAT_GEMM_NNP=0 / 1) and the fp64 error
        import hashlib
        res[f"{name}_sha1"] = hashlib.sha1(y0.cpu().numpy().tobytes()).hexdigest()
        rows = torch.arange(0, M, 997, device=dev)
        ref = X[rows].double() @ B0.double()
        res[f"{name}_rel_err_sampled_rows"] = float((y0[rows].double() - ref).abs().max() / ref.abs().max())
        flop = 2.0 * M * K * Nc
        for lay, B in ((0, B0), (1, B1)):
            us = timeit(lambda: ops.gemm_nn(X, B, lay, Nc, out=y0), iters)
            res[f"{name}_layout{lay}"] = {"us": us, "tflops": flop / us / 1e6}
        del X, y0, y1
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
