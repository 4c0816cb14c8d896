#!/usr/bin/env python3
"""Where the edge kernels spend their time at config 2: ppgat_fwd and ppgat_bwd_edges timed
on the whole work schedule, on the long items only (degree > --short) and on the short-item
suffix only (items are ordered by descending degree), with synthetic row values."""
import argparse
import ctypes
import importlib
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
ops = pkg.hip_ops
_lib = pkg._lib


def sub(s, lo, hi):
    """Schedule struct over items [lo, hi) (hub pieces only if lo == 0)."""
    e = 4
    nh, hubs = (s.n_hub_items, s.n_hubs) if lo == 0 else (0, 0)
    cs = _lib.Schedule(s.item_row.data_ptr() + lo * e, s.item_beg.data_ptr() + lo * e, s.item_end.data_ptr() + lo * e,
                       hi - lo, nh, s.hub_row.data_ptr(), s.hub_ptr.data_ptr(), hubs,
                       min(max(s.n_long_items - lo, nh), hi - lo))
    return cs, (hi - lo) - nh + hubs  # the node count the validation expects for this subset


def timeit(fn, iters=20):
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
    ap.add_argument("--short", type=int, default=16)
    args = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    g = pkg.data.synthetic_ui_graph()
    ei = torch.from_numpy(g.edge_index_numpy()).to(dev)
    G = ops.csr_build(ei, g.n_nodes)
    N, E, C = G.n_nodes, G.n_edges, 128
    gen = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(N, C, device=dev, generator=gen)
    s_src = torch.randn(N, device=dev, generator=gen)
    s_dst = torch.randn(N, device=dev, generator=gen)
    go = torch.randn(N, C, device=dev, generator=gen)
    nstate = torch.stack([s_dst, torch.full_like(s_dst, 3.0), torch.full_like(s_dst, 0.1), s_src], 1).contiguous()
    out = torch.empty(N, C, device=dev)
    m = torch.empty(N, device=dev)
    invl = torch.empty(N, device=dev)
    D = torch.empty(N, C, device=dev)
    S = torch.empty(N, 2, device=dev)
    dz = torch.empty(E, device=dev)
    st = _lib.stream_handle(dev)
    res = {}
    for name, sched in (("fwd", G.fwd_sched), ("bwd_src", G.bwd_sched)):
        beg = sched.item_beg[:sched.n_items].cpu()
        end = sched.item_end[:sched.n_items].cpu()
        deg = (end - beg)
        k = int((deg > args.short).sum())  # descending-degree order after the hub pieces
        nb = ctypes.c_size_t(0)
        _lib.check(lib.ppgat_fwd_workspace_bytes(sched.n_hub_items, 1, C, ctypes.byref(nb)), "ws")
        ws = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
        for part, (lo, hi) in (("all", (0, sched.n_items)), ("long", (0, k)), ("short", (k, sched.n_items))):
            cs, Ns = sub(sched, lo, hi)
            if name == "fwd":
                fn = lambda cs=cs, Ns=Ns: _lib.check(lib.ppgat_fwd(ctypes.byref(cs), G.col.data_ptr(), G.csr_eid.data_ptr(), Ns,
                                                            E, 1, C, h.data_ptr(), s_src.data_ptr(), s_dst.data_ptr(),
                                                            None, 0, 0.2, 0.1, 7, None, out.data_ptr(), m.data_ptr(),
                                                            invl.data_ptr(), None, ws.data_ptr(), nb.value, st), "fwd")
            else:
                fn = lambda cs=cs, Ns=Ns: _lib.check(lib.ppgat_bwd_edges(ctypes.byref(cs), G.row.data_ptr(),
                                                                  G.csc_eid.data_ptr(), G.csc2csr.data_ptr(), E, 1, C,
                                                                  h.data_ptr(), s_src.data_ptr(), nstate.data_ptr(),
                                                                  go.data_ptr(), 0, 0.2, 0.1, 7, None, D.data_ptr(), C,
                                                                  S.data_ptr(), 2, dz.data_ptr(), ws.data_ptr(),
                                                                  nb.value, st), "bwd")
            res[f"{name}_{part}"] = {"us": timeit(fn), "items": hi - lo, "edges": int(deg[lo:hi].sum())}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
