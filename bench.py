#!/usr/bin/env python3
"""Headline benchmark: edges/sec of the GAT fwd+bwd training step, d=128, on the
1.69M-interaction U-I graph (BASELINE.json metric, config 2: PyG-semantics GAT,
fused features, BPR, 2 layers, heads=1, d=128).

One "step" = the reference's training step (scripts/train_gat_pyg.py:312-323):
  Z = PyGGAT(item_feats, edge_index) (train mode, attn dropout 0.1)
  BPR loss over S=200k pre-sampled triples; loss.backward(); Adam step.
value = E * L * K / t over K timed steps (E = edge_index columns, L = 2 layers).
Inputs (graph, features, triples) are resident in HBM before the timed region.

Usage: python bench.py [--gpus N --steps K --warmup W]
N>1: launched by torch.distributed.run, one rank per GPU.
"""
from __future__ import annotations

import argparse
import gc
import importlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
data = pkg.data
_lib = pkg._lib

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--heads", type=int, default=1)
    ap.add_argument("--samples", type=int, default=200_000)
    ap.add_argument("--attn-dropout", type=float, default=0.1)
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=2,
                    help="2: U-I graph (headline); 3: U-I + I-I kNN k=20 edges (SURVEY.md 8(d) cfg 3); "
                         "4: config 2 row-sharded with the all_to_all halo (N>1); "
                         "5: 10M x 5M x 200M-edge synthetic, d=256, heads=4 (roofline / scaling run)")
    ap.add_argument("--scale", type=float, default=None,
                    help="config 5 size multiplier (default world/8: one GPU's share of the 8-GPU run, "
                         "so the per-GPU work is the same at every N)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0,
                    help="approximate CPU time budget of the oracle baseline leg (0 disables)")
    ap.add_argument("--traffic-json", default=None,
                    help="committed PMC summary (default: profiles/r06/cfg2_pmc_traffic.json for config 2, "
                         "profiles/r03/cfg5_pmc_traffic.json for config 5 at its default scale)")
    ap.add_argument("--partition", choices=["auto", "replicated", "halo"], default="auto",
                    help="N>1: 'replicated' = users sharded, item rows on every rank (dist.build_replicated_graph); "
                         "'halo' = users and items row-sharded, RCCL all_to_all of the halo rows per layer "
                         "(dist.build_halo_graph); auto = replicated for configs 2/3, halo for configs 4/5")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="capture the training step once in a hipGraph and replay it (auto: on for N>1 over RCCL, "
                         "where the per-rank step is short enough for host launch overhead to dominate)")
    ap.add_argument("--dist-at-1", action="store_true",
                    help="rehearsal: run the N>1 code path (process group, partition, collectives) with one rank")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) for real runs; gloo only to rehearse the N>1 flow with "
                         "several ranks on one GPU (tests/test_gpu_dist.py)")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# algorithmic bytes per launch (DESIGN.md "Kernels and their rooflines")
# ---------------------------------------------------------------------------
def algo_bytes(kernel: str, N: int, E: int, H: int, C: int, dropout: bool, xform_k: int = 0,
               dz_slot: bool = False, gather_g=False) -> float:
    """Algorithmic bytes per launch.  xform_k > 0: the aggregate-then-
    transform kernels (heads > 1, x rows of xform_k floats gathered instead of h rows).
    dz_slot: pass B reads each edge's dz position (the sharded layouts); otherwise dz is stored
    at the edge's own CSC position (no index read).  gather_g: the multi-head pass B gathers
    g_i (C floats) per edge and reads hs_j / writes acc_j (H * C floats) per source
    (ppgat_xgat_bwd_edges_g) instead of gathering gt_i (H * xform_k floats); "gd" (deferred D,
    ppgat_xgat_bwd_edges_gd) writes dalpha and beta dalpha per edge and no ds_src."""
    d = 4 if dropout else 0
    sl = 4 if dz_slot else 0
    if xform_k:
        K = xform_k
        if kernel == "fwd":    # k_fwd_x: col, s_src[H], x_j | sched, s_dst[H], agg[H, K], m, inv_l
            return E * (4 + 4 * H + 4 * K + d) + N * (12 + 4 * H + 4 * H * K + 8 * H)
        if kernel == "bwd_src" and gather_g == "gd":  # deferred D: dalpha and beta dalpha out, no S
            return E * (4 + sl + 16 * H + 4 * C + 8 * H + d) + N * (12 + 4 * H * C + 4 * H + 4 * H * C)
        if kernel == "bwd_src" and gather_g:  # k_bwd_g: row, (slot), nstate[H], g_i[C], dz[H] | sched, hs, s_src, acc, S
            return E * (4 + sl + 16 * H + 4 * C + 4 * H + d) + N * (12 + 4 * H * C + 4 * H + 4 * H * C + 4 * H)
        if kernel == "bwd_src":  # k_bwd_x: row, (slot), nstate[H], gt_i[H, K], dz[H] | sched, x, s_src, dx, S
            return E * (4 + sl + 16 * H + 4 * H * K + 4 * H + d) + N * (12 + 4 * K + 4 * H + 4 * K + 4 * H)
        if kernel == "bwd_pro":  # gt, agg in; s_dst, m, inv_l in; nstate out
            return N * (8 * H * K + 12 * H + 16 * H)
        if kernel == "scores":
            return N * (4 * K + 8 * H)
        return 0.0
    if kernel == "fwd":
        per_e = 4 + 4 * H + 4 * H * C + d * H / max(H, 1)
        per_n = 8 + 4 * H + 4 * C + 8 * H
        return E * per_e + N * per_n
    if kernel == "bwd_src":
        per_e = 4 + sl + 4 * H * 4 + 4 * C + 4 * H + d  # row, (slot), nstate, g_i, dz
        per_n = 8 + 4 * H + 4 * H * C * 2 + 4 * H
        return E * per_e + N * per_n
    if kernel == "bwd_epi":  # (+ the csr2csc index per edge when dz is in CSC order)
        return E * (4 * H + (0 if dz_slot else 4)) + N * (8 + 4 * H + 4 * H * C * 3)
    if kernel == "bwd_pro":
        return N * (4 * C + 4 * C + 4 * H)
    if kernel == "scores":
        return N * (4 * H * C + 8 * H)
    return 0.0


def host_cores() -> int:
    """CPU cores this process may run on: the affinity mask, further capped by a cgroup CPU
    quota when one is set (a GPU box's share of its host is smaller than os.cpu_count())."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except Exception:
        pass
    return max(1, n)


def measured_copy_gbs(dev, nbytes: int = 1 << 30, reps: int = 10) -> dict:
    """Achievable-HBM yardstick on this box, beside the spec peak: a 1 GiB
    buffer copied `reps` times (read + write bytes / time, HIP events on the current stream) by
    libppgat's float4 streaming copy (ppgat_stream_copy; the guide measures 6.29 TB/s for a
    float4 copy) and, for comparison, by torch's copy kernel (what earlier rounds reported)."""
    lib = _lib.load()
    n = nbytes // 4
    src = torch.ones(n, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    st = _lib.stream_handle(dev)
    out = {}
    for name, run in (("f4", lambda: _lib.check(lib.ppgat_stream_copy(src.data_ptr(), dst.data_ptr(), 4 * n, st),
                                                "stream_copy")),
                      ("torch", lambda: dst.copy_(src))):
        run()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            run()
        b.record()
        torch.cuda.synchronize(dev)
        out[name] = 2.0 * n * 4 * reps / (a.elapsed_time(b) / 1e3) / 1e9
    del src, dst
    return out


def cpu_baseline(g: data.UIGraph, feats: np.ndarray, hidden: int, layers: int, budget_s: float):
    """Oracle (torch CPU restatement of PyG GATConv, oracle/gat_oracle.py) fwd+bwd of the
    L GAT layers, on a bounded prefix sample of the same graph: median of 5 timed
    iterations after one warm-up, on every core the process may use."""
    from oracle import gat_oracle
    threads = host_cores()
    torch.set_num_threads(threads)
    # sample: the first n_u users (all their train edges) -> ~400k directed edges
    target_e = 400_000
    ucum = np.cumsum(np.diff(g.user_ptr)) * 2
    n_u = int(np.searchsorted(ucum, target_e)) + 1
    n_u = min(n_u, g.n_users)
    ptr = g.user_ptr[:n_u + 1]
    users = np.repeat(np.arange(n_u), np.diff(ptr))
    ei = torch.from_numpy(data.edge_index_numpy(g.n_users, users, g.user_items[:ptr[-1]]))
    E = ei.size(1)
    N = g.n_nodes
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.standard_normal((N, hidden)).astype(np.float32))
    torch.manual_seed(0)
    params = []
    for _ in range(layers):
        W = (torch.rand(hidden, hidden) * 2 - 1) * (6 / (2 * hidden)) ** 0.5
        a_s = (torch.rand(1, 1, hidden) * 2 - 1) * (6 / (1 + hidden)) ** 0.5
        a_d = (torch.rand(1, 1, hidden) * 2 - 1) * (6 / (1 + hidden)) ** 0.5
        params.append([t.requires_grad_(True) for t in (W, a_s, a_d, torch.zeros(hidden))])

    def once():
        h = x
        for W, a_s, a_d, b in params:
            h = gat_oracle.pyg_gat_conv(h, ei, W, a_s, a_d, b, 1)
        h.square().mean().backward()

    once()  # warm-up
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        once()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": E * layers / med, "unit": "edges/sec", "cores": threads, "kind": "port",
            "host_cpu_count": os.cpu_count(),
            "sample": f"oracle pyg_gat_conv x{layers} layers fwd+bwd (no lin/loss/Adam), first {n_u} users' "
                      f"train edges = {E} of {2 * len(g.user_items)} directed edges over all {N} nodes, d={hidden}, "
                      f"median of 5 iterations ({min(times):.2f}-{max(times):.2f} s each) after 1 warm-up, "
                      f"{threads} threads (affinity/cgroup share of {os.cpu_count()} host CPUs), "
                      f"torch {torch.__version__} CPU"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_path = world > 1 or args.dist_at_1
    if args.dist_at_1:
        os.environ.setdefault("PPGAT_COMM_ALWAYS", "1")
        for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29517")):
            os.environ.setdefault(k, v)
    if dist_path:
        import torch.distributed as dist
        local = local if args.dist_backend == "nccl" else 0  # gloo rehearsal: ranks share GPU 0
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    def note(msg):  # progress on stderr (the large config-5 setup takes minutes before the first step)
        if rank == 0 and args.config == 5:
            print(f"bench: {msg} ({time.perf_counter() - t_start:.0f} s)", file=sys.stderr, flush=True)
    t_start = time.perf_counter()

    # ---- synthetic inputs; identical on every rank ----
    if args.config == 5:
        scale = args.scale if args.scale is not None else world / 8.0
        args.hidden, args.heads = 256, 4
        g = data.synthetic_scaling_graph(scale, seed=42)
        feats_np = data.synthetic_item_features(g.n_items, 256, seed=42)
    else:
        scale = None
        g = data.synthetic_ui_graph(seed=42)
        feats_np = data.synthetic_item_features(g.n_items, 128, seed=42)
    ei_np = g.edge_index_numpy()
    if args.config == 3:  # I-I kNN relation appended to the homogeneous edge_index (A10, "extension")
        rows, cols, _ = data.synthetic_ii_edges(g, k=20, seed=42)
        ei_np = np.concatenate([ei_np, data.ii_edge_columns(g.n_users, rows, cols)], 1)
    E, N = ei_np.shape[1], g.n_nodes
    note(f"graph generated: {N:,} nodes, {E:,} edge_index columns")
    u, i, j = data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, args.samples, seed=42)
    ei = torch.from_numpy(ei_np).to(dev)
    feats = torch.from_numpy(feats_np).to(dev)
    tu, ti, tj = (torch.from_numpy(a).to(dev) for a in (u, i, j))
    torch.manual_seed(42)
    full = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=feats_np.shape[1], hidden=args.hidden, layers=args.layers,
                      heads=args.heads, attn_dropout=args.attn_dropout).to(dev)
    part = args.partition if args.partition != "auto" else ("halo" if args.config in (4, 5) else "replicated")
    if dist_path and part == "replicated":
        # strong scaling of the fixed config-2 job: users sharded, the 63k item rows on every
        # rank, every edge homed with its user; item rows merged by all_reduce (dist.py)
        comm = pkg.dist.Comm()
        dg = pkg.dist.build_replicated_graph(ei, N, g.n_users, world, rank)
        model = pkg.dist.ReplicatedPyGGAT(full, dg, comm)
    elif dist_path:
        # users and items row-sharded, edges homed at their destination's rank, one RCCL
        # all_to_all of the halo rows per layer and direction (dist.py)
        comm = pkg.dist.Comm()
        dg = pkg.dist.build_halo_graph(ei, N, g.n_users, world, rank)
        model = pkg.dist.HaloPyGGAT(full, dg, comm)
    else:
        model = full
        pkg.graph_cache.get(ei, N)  # one-time CSR/CSC build (not timed)
    note("model and graph views on the device")
    # same Adam update as train_gat_pyg.py:299 (lr 1e-3, L2 1e-4): libppgat's device Adam (optim.py)
    # hipGraph replay by default (one captured step: ~150 launches enqueued once), except the
    # gloo rehearsal whose collectives run on the host
    use_graph = args.graph == "on" or (args.graph == "auto" and not (dist_path and args.dist_backend == "gloo"))
    if args.config == 5 and scale > 0.5 and args.graph == "auto":
        # the whole 200M-edge graph on one GPU: a capture holds the step's buffers in a private
        # pool beside the persistent ~150 GB and does not fit 288 GB (profiles/r06/
        # x11_bench_cfg5_full_graph_oom.log); the eager step enqueues in 9 ms of a 558-ms step
        use_graph = False
    opt = pkg.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4, capturable=use_graph)
    # the loss backward's sort on a side stream beside the forward: off by default, measured no
    # faster inside the captured step (1.890 vs 1.881 ms, profiles/r05/w1_bench.log)
    bpr_overlap = os.environ.get("PPGAT_BPR_OVERLAP", "0") == "1"
    one = torch.ones((), dtype=torch.float32, device=dev)  # loss.backward()'s seed, made once (no fill per step)

    def step():
        model.train()
        if use_graph:
            _lib.dropout_advance(dev)  # fresh dropout masks on every replay
        if dist_path:
            Z = model(feats)
            loss_fn = pkg.dist.replicated_bpr_loss if part == "replicated" else pkg.dist.halo_bpr_loss
            loss = loss_fn(Z, dg, comm, tu, ti, tj, g.n_users, g.n_items, plan_key="bench")  # fixed triples
            opt.zero_grad(set_to_none=True)
            loss.backward(one)
            model.allreduce_grads()
        else:
            prep = pkg.hip_ops.bpr_prepare(N, g.n_users, g.n_items, args.hidden, tu, ti, tj) if bpr_overlap else None
            Z = model(feats, ei)
            loss = pkg.bpr_loss(Z, g.n_users, tu, ti, tj, prepared=prep)
            opt.zero_grad(set_to_none=True)
            loss.backward(one)
        opt.step()
        return loss

    graph = None
    note("warming up")
    if use_graph:
        # warm up on a side stream (allocator pools, RCCL communicators, lazy inits), then
        # capture one whole step -- forward, loss, backward, collectives, Adam -- and replay it
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(args.warmup, 2)):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        # the warm-up's cached blocks back to the device: the capture allocates the step's
        # buffers in a private pool of its own, and at the whole 200M-edge graph (229 GB peak)
        # two copies of the working set do not fit in 288 GB
        gc.collect()
        torch.cuda.empty_cache()
        ok = 1
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                # keep only the value: the captured autograd graph (and its AccumulateGrad
                # nodes, tied to the capture stream) must not outlive the capture
                loss_static = step().detach()
        except Exception as exc:  # capture refused (driver / RCCL): time the same step eagerly instead
            print(f"bench: hipGraph capture failed ({type(exc).__name__}: {exc})", file=sys.stderr, flush=True)
            graph, ok = None, 0
        if graph is None:
            # (outside the handler: the exception's frames hold the failed capture's tensors)
            gc.collect()
            torch.cuda.empty_cache()  # the failed capture's private pool, before the eager steps
        torch.cuda.synchronize()
        if dist_path:
            # one shared decision: replay only if every rank captured (a rank running eagerly
            # beside replaying ranks would pair its collectives with different calls)
            flag = torch.tensor([ok], dtype=torch.int32, device=dev if args.dist_backend == "nccl" else "cpu")
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
            if int(flag.item()) == 0:
                graph = None
        if graph is not None:
            graph.replay()  # the capture itself ran nothing: one replay so every rank starts from a replayed step
        else:
            print("bench: running the step eagerly", file=sys.stderr, flush=True)
            for _ in range(max(args.warmup, 1)):
                step()
        torch.cuda.synchronize()
    else:
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    note("warm; timing")
    _lib.profile_reset()
    _lib.profile_enable(graph is None)  # per-kernel events in eager mode only (not capturable)
    if dist_path:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if graph is not None:
            graph.replay()
        else:
            loss = step()
    t_host = time.perf_counter() - t0  # host time to enqueue the K steps (launch overhead check)
    torch.cuda.synchronize()
    if dist_path:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    _lib.profile_enable(False)
    kern_src = "HIP events on the launch stream inside the timed region"
    if graph is not None:
        loss = loss_static
        # graph replays carry no per-kernel events: time the same step eagerly for the
        # kernel breakdown and the roofline (after the timed region; not part of value)
        torch.cuda.synchronize()
        _lib.profile_reset()
        _lib.profile_enable(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        _lib.profile_enable(False)
        kern_src = "HIP events, eager replay of the same step after the timed graph replays"
    if dist_path:
        tt = torch.tensor([el], dtype=torch.float64)
        tt = tt.to(dev) if args.dist_backend == "nccl" else tt
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = float(tt.item())
    loss_val = loss.detach().clone()
    if dist_path:  # each rank's loss covers its own users' triples: the job's loss is their sum
        comm.all_reduce_(loss_val)
    K = args.steps
    H, C = args.heads, args.hidden
    # the multi-head layers run aggregate-then-transform when H*C exceeds the input width
    xform_k = C if (H > 1 and H * C > C and pkg.hip_ops.xgat_supported(C, H, C)) else 0
    # the backward formulation hip_ops.xgat_backward picks for these layer sizes
    src_homed = dist_path and part == "halo" and xform_k and pkg.dist.source_homed_backward(dg)
    if src_homed:  # the source-homed backward (dist._halo_xgat_backward): deferred D unless PPGAT_XGAT_GATHER=g
        gather_mode = "g" if os.environ.get("PPGAT_XGAT_GATHER") == "g" else "gd"
    elif xform_k and dist_path and part == "halo":  # the formulation the local layer sizes select
        gather_mode = pkg.hip_ops._xgat_gather_mode(C, H, dg.R, dg.n_own, dg.bwd_view.n_bwd_edges, C)
    else:
        gather_mode = pkg.hip_ops._xgat_gather_mode(C, H) if xform_k else None
    gather_g = gather_mode in ("g", "gd")
    kern = {k: _lib.profile_read(k) for k in ("scores", "fwd", "bwd_pro", "bwd_src", "bwd_epi", "bwd_red",
                                               "proj", "proj_bwd", "gemm_tn", "adam")}
    fused_ms = sum(ms for k, (ms, _) in kern.items() if k not in ("proj", "proj_bwd", "gemm_tn", "adam"))
    value = E * args.layers * K / el  # the whole job: every edge of the global graph, once per layer
    dom = max(("fwd", "bwd_src", "bwd_epi"), key=lambda k: kern[k][0])
    dom_ms, dom_n = kern[dom]
    # one layer pass may be several launches (the sharded backward runs halo / item sources
    # first and the rest after the exchange): average per layer pass, K steps x L layers
    passes = args.steps * args.layers
    avg_s = dom_ms / max(passes, 1) / 1e3
    if dist_path:
        # rank 0's kernels run over its local graph: price them on its own rows and edges
        if part == "replicated":
            v = dg.view
        else:
            v = dg.fwd_view if dom == "fwd" else dg.bwd_view
        if src_homed and dom != "fwd":  # the backward passes run over the own sources' out-edges
            ab = algo_bytes(dom, dg.n_own, dg.src_views.n_edges, H, C, args.attn_dropout > 0, xform_k,
                            dz_slot=False, gather_g=gather_mode)
        else:
            ab = algo_bytes(dom, v.n_rows, v.n_fwd_edges if dom == "fwd" else v.n_bwd_edges, H, C,
                            args.attn_dropout > 0, xform_k, dz_slot=part != "replicated",
                            gather_g=gather_mode if gather_g else False)
    else:
        ab = algo_bytes(dom, N, E, H, C, args.attn_dropout > 0, xform_k, gather_g=gather_mode if gather_g else False)
    achieved = ab / avg_s / 1e9
    traffic = traffic_src = traffic_dram = None
    try:
        if dist_path:
            raise LookupError("the committed PMC summary is for the unsharded graph")
        tj_path = args.traffic_json or str(ROOT / "profiles" / ("r03/cfg5_pmc_traffic.json" if args.config == 5
                                                                 else "r06/cfg2_pmc_traffic.json"))
        tj_ = json.loads(Path(tj_path).read_text())
        # PMC summaries are per workload (config, scale) and per multi-head backward formulation
        if tj_.get("config", 2) == args.config and tj_.get("scale", scale if args.config == 5 else None) == (
                scale if args.config == 5 else None) and (
                not xform_k or tj_.get("bwd_gather", "gt") == (gather_mode if gather_g else "gt")):
            traffic = tj_.get("per_launch_bytes", {}).get(dom)
            traffic_src = os.path.relpath(tj_path, ROOT)
            traffic_dram = tj_.get("per_launch_dram_bytes", {}).get(dom)
    except Exception:
        pass
    copies = measured_copy_gbs(dev) if rank == 0 else None
    copy_gbs = copies["f4"] if copies else None
    if args.config == 5:
        metric = "edges/sec GAT fwd+bwd, d=256 heads=4, 200M-edge synthetic (config 5)"
        workload = (f"cfg5 x{scale:g}: PyGGAT train step (fwd+BPR+bwd+Adam), {g.n_users:,} users + {g.n_items:,} "
                    f"items, {g.n_interactions:,} interactions (Zipf items), d=256, heads=4")
        data_desc = "synthetic (config-5 scaling graph, Poisson users / Zipf items, random-init weights)"
    else:
        metric = "edges/sec GAT fwd+bwd, d=128, 1.69M-edge U-I graph"
        workload = (("cfg2: PyGGAT train step (fwd+BPR+bwd+Adam), 1,689,116 interactions, "
                     "192,403 users + 63,001 items") if args.config == 2 else
                    ("cfg4: the cfg2 train step, users and items row-sharded (all_to_all halo)")
                    if args.config == 4 else
                    "cfg3: cfg2 + I-I kNN (k=20, sim>=0.3) edges, PyGGAT train step")
        data_desc = "synthetic (config-2 statistics-matched U-I graph, random-init weights)"
    result = {
        "metric": metric,
        "value": value,
        "unit": "edges/sec",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": el / K * 1e3,
        "host_enqueue_ms_per_step": t_host / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if (world == 1 or args.config == 5) else "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": data_desc,
        "config": {"workload": workload,
                   "edges": E, "nodes": N, "layers": args.layers, "heads": H, "hidden": C,
                   "bpr_samples": args.samples, "attn_dropout": args.attn_dropout,
                   "parallelism": ("single" if not dist_path else
                                   f"user-sharded x{world}, item rows replicated (RCCL all_reduce)"
                                   if part == "replicated" else
                                   f"row-sharded x{world}, RCCL all_to_all halo + grad all_reduce")},
        "hip_graph": graph is not None,
        "device_mem_peak_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
        "formulation": ("aggregate-then-transform (x_j gathered once per edge for all heads)" if xform_k else
                        "transform-then-aggregate (h_j gathered per edge)"),
        "gemm": ("fp32 MFMA, exact fp32 FMA chains (PPGAT_GEMM=fp32)" if os.environ.get("PPGAT_GEMM") == "fp32" else
                 "fp32 operands and results on the matrix cores through operand splits (DESIGN.md 4.3): "
                 "fp16 two-term split with power-of-two row/column scales, 3 MFMAs per product, <= 2^-21 "
                 "relative per product, for the large-M NN and TN products (k_gemm_nnh3, k_gemm_tnh); bf16 "
                 "three-term split, 6 MFMAs, <= 2^-24, for the rest"
                 if args.config == 5 and os.environ.get("PPGAT_GEMM_F16", "1") != "0" else
                 "fp32 operands and results on the matrix cores through the bf16 three-term split (6 MFMAs "
                 "per product, <= 2^-24 relative per product: k_projx, k_dxw; DESIGN.md 4.3), fp32 MFMA "
                 "for the small weight-gradient products"),
        "kernel_timing": kern_src,
        "fused_kernel_edges_per_sec": E * args.layers * K / (fused_ms / 1e3) if fused_ms else None,
        "kernel_ms_per_step": {k: ms / K for k, (ms, n) in kern.items()},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     # the L2's fabric requests destined for DRAM (TCC_EA0_*REQ_DRAM / *REQ): the
                     # memory-side Infinity Cache sits behind them, so its hits are not split off
                     "traffic_dram_destined": traffic_dram,
                     "algo_bytes_per_launch": ab, "avg_launch_ms": avg_s * 1e3, "launches": dom_n,
                     "launches_per_layer_pass": dom_n / max(passes, 1),
                     "measured_copy_gbs": copy_gbs,
                     "frac_of_copy": achieved / copy_gbs if copy_gbs else None,
                     "torch_copy_gbs": copies["torch"] if copies else None},
        "loss": float(loss_val.item()),
        "optimizer": "Adam (libppgat device kernel, torch.optim.Adam semantics)",
    }
    if rank == 0 and world == 1 and args.cpu_baseline_seconds > 0 and args.config != 5:
        result["cpu_baseline"] = cpu_baseline(g, feats_np, C, args.layers, args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist_path:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
