#!/usr/bin/env python3
"""One rank's share of an N-GPU config-2 step, on one GPU, collectives stubbed out.

    python tools/scale_probe.py --world 8 --rank 0 [--partition replicated|halo]

Builds the same per-rank graph and model as `bench.py --gpus N` and times the step with
every collective replaced by a no-op (results are NOT the job's; only the compute and the
host enqueue time of one rank are measured).  Shows what is left per rank once the
exchange is overlapped or free: the floor under N-GPU ms/step."""
import argparse
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
from importlib import import_module  # noqa: E402

_lib = import_module("plotpointe-gat-recommendation_amd._lib")
data = pkg.data


class NullComm:
    def __init__(self, world, rank):
        self.world, self.rank, self.backend, self.group, self.active = world, rank, "null", None, True

    def all_gather_rows(self, t):
        return t.contiguous().repeat((self.world,) + (1,) * (t.dim() - 1))

    def reduce_scatter_rows(self, t):
        return t.contiguous()[: t.size(0) // self.world].contiguous()

    def all_reduce_(self, t, op=None):
        return t

    own_id = 0  # a node id this rank owns (set after the graph is built): the stubbed id exchange

    def all_to_all_rows(self, t, send_counts, recv_counts, out=None):
        # stub: received rows are zeros, received ids are an id this rank owns (so the loss
        # plan's requests resolve to local rows); timing only
        n = int(sum(recv_counts))
        if out is None:
            fill = self.own_id if not t.is_floating_point() else 0
            out = torch.full((n,) + tuple(t.shape[1:]), fill, dtype=t.dtype, device=t.device)
        return out

    def all_to_all_counts(self, counts):
        return [int(c) for c in counts]

    def broadcast_int(self, value, src=0):
        return int(value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--partition", choices=["replicated", "halo"], default="replicated")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph", action="store_true", help="capture the step in a hipGraph (as bench.py for N>1)")
    ap.add_argument("--streams", action="store_true",
                    help="report the stub as RCCL so the comm-stream overlaps (fwd_split / bwd_split) run as at N>1")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = data.synthetic_ui_graph(seed=42)
    feats = torch.from_numpy(data.synthetic_item_features(g.n_items, 128, seed=42)).to(dev)
    ei = torch.from_numpy(g.edge_index_numpy()).to(dev)
    u, i, j = data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, 200_000, seed=42)
    tu, ti, tj = (torch.from_numpy(a).to(dev) for a in (u, i, j))
    torch.manual_seed(42)
    full = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=128, hidden=128, layers=2, heads=1,
                      attn_dropout=0.1).to(dev)
    comm = NullComm(args.world, args.rank)
    if args.streams:
        comm.backend = "nccl"
    D = pkg.dist
    if args.partition == "replicated":
        dg = D.build_replicated_graph(ei, g.n_nodes, g.n_users, args.world, args.rank)
        model = D.ReplicatedPyGGAT(full, dg, comm)
        loss_fn = D.replicated_bpr_loss
        n_edges = dg.view.n_fwd_edges
    else:
        dg = D.build_halo_graph(ei, g.n_nodes, g.n_users, args.world, args.rank)
        comm.own_id = int(dg.owned()[1][0])  # first own item
        model = D.HaloPyGGAT(full, dg, comm)
        loss_fn = D.halo_bpr_loss
        n_edges = dg.fwd_view.n_fwd_edges
    opt = pkg.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4, capturable=args.graph)

    def step():
        model.train()
        if args.graph:
            _lib.dropout_advance(dev)
        Z = model(feats)
        loss = loss_fn(Z, dg, comm, tu, ti, tj, g.n_users, g.n_items)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        model.allreduce_grads()
        opt.step()

    run = step
    if args.graph:
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(args.warmup, 2)):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        run = graph.replay
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(not args.graph)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    _lib.profile_enable(False)
    kern = {k: _lib.profile_read(k)[0] / args.steps for k in ("fwd", "bwd_pro", "bwd_src", "bwd_epi", "proj",
                                                               "gemm_tn", "adam")}
    print(json.dumps({"partition": args.partition, "graph": args.graph, "world": args.world, "rank": args.rank,
                      "rows": int(dg.R), "local_edges": int(n_edges), "global_edges": int(ei.size(1)),
                      "ms_per_step": el / args.steps * 1e3, "host_enqueue_ms_per_step": th / args.steps * 1e3,
                      "kernel_ms_per_step": kern}), flush=True)


if __name__ == "__main__":
    main()
