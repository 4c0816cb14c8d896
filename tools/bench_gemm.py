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
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
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
    cases = {
        "proj_fwd_scores": lambda: ops.project(x, W, att_src=a_s, att_dst=a_d),
        "proj_dx": lambda: pkg._lib.check(lib.ppgat_project_bwd_input(D.data_ptr(), 128, N, 128, W.data_ptr(), 128, 128,
                                                                      a_s.data_ptr(), a_d.data_ptr(), S.data_ptr(), 2,
                                                                      dx.data_ptr(), 128, st), "dx"),
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


if __name__ == "__main__":
    main()
