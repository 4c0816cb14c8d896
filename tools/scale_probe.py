#!/usr/bin/env python3
"""One rank's share of an N-GPU step, on one GPU, collectives stubbed out.

    python tools/scale_probe.py --world 8 --rank 0 [--partition replicated|halo]
    python tools/scale_probe.py --config 5 --world 8 --rank 7 --streams --a2a-gbs 640

Builds the same per-rank graph and model as `bench.py --gpus N` (config 2, or --config 5: the
200M-edge synthetic, d=256, heads=4, halo partition) and times the step with every collective
replaced by a stub (results are NOT the job's; only the compute and the host enqueue time of
one rank are measured).  Without --a2a-gbs the stub is free: the floor under N-GPU ms/step.
With --a2a-gbs B the stub holds the stream it runs on for this rank's exchange time at B GB/s
(max(bytes sent, bytes received) / B per all_to_all, 2 (N-1)/N x bytes / B per all_reduce;
a GPU-side sleep of one wave, calibrated at start): with --streams the exchanges run on the
communication stream as RCCL's would, so the step time shows how much of the modelled
exchange the overlaps hide.  A model, not a measurement of RCCL over xGMI: the real
all_to_all also reads and writes HBM beside the compute."""
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
    def __init__(self, world, rank, gbs=0.0, cycles_per_ms=0.0):
        self.world, self.rank, self.backend, self.group, self.active = world, rank, "null", None, True
        self.gbs, self.cycles_per_ms = gbs, cycles_per_ms
        self.modelled_ms = 0.0   # exchange time modelled per step (host-side tally)

    def _hold(self, nbytes):
        """Hold the current stream for nbytes at self.gbs (the modelled exchange)."""
        if self.gbs <= 0 or nbytes <= 0:
            return
        ms = nbytes / (self.gbs * 1e9) * 1e3
        self.modelled_ms += ms
        torch.cuda._sleep(int(ms * self.cycles_per_ms))

    def all_gather_rows(self, t):
        return t.contiguous().repeat((self.world,) + (1,) * (t.dim() - 1))

    def reduce_scatter_rows(self, t):
        return t.contiguous()[: t.size(0) // self.world].contiguous()

    def all_reduce_(self, t, op=None):
        self._hold(2 * (self.world - 1) / self.world * t.numel() * t.element_size())
        return t

    own_ids = None  # node ids of this rank's own items (set after the graph is built): the stubbed id exchange

    def all_to_all_rows(self, t, send_counts, recv_counts, out=None):
        # stub: received rows are zeros; received ids (the loss plan's requests from the peers)
        # are this rank's own items in turn -- each own item then gets about as many returned
        # copies as at world 8 (at most a few), not all of them one row; timing only
        n = int(sum(recv_counts))
        row = t[0].numel() * t.element_size() if t.dim() and t.size(0) else 0
        row = row or (int(np.prod(t.shape[1:])) * t.element_size() if t.dim() > 1 else t.element_size())
        self._hold(max(int(sum(send_counts)), n) * row)
        if out is None:
            if not t.is_floating_point() and self.own_ids is not None and len(self.own_ids):
                ids = self.own_ids.to(t.device)
                out = ids[torch.arange(n, device=t.device) % len(ids)].to(t.dtype)
            else:
                out = torch.zeros((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        return out

    def exchange(self, plan, src, out, part=None):
        """Comm.exchange stub: the plan's rows are not moved (timing only); holds the stream for
        max(rows sent, rows received) x row bytes (of the part's runs when ``part`` is given)."""
        row = (src[0].numel() if src.dim() and src.size(0) else int(np.prod(src.shape[1:]))) * src.element_size()
        if part is None:
            ns, nr = plan.n_send, plan.n_recv
        else:
            sp, rp = plan.parts[part]
            ns = sum(n for runs in sp for _, n in runs)
            nr = sum(n for runs in rp for _, n in runs)
        self._hold(max(ns, nr) * row)
        return out

    def exchange_back(self, plan, halo, out=None):
        row = (int(np.prod(halo.shape[1:])) if halo.dim() > 1 else 1) * halo.element_size()
        self._hold(max(plan.n_send, plan.n_recv) * row)
        if out is None:
            out = torch.zeros((plan.n_send,) + tuple(halo.shape[1:]), dtype=halo.dtype, device=halo.device)
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
    ap.add_argument("--config", type=int, choices=[2, 5], default=2)
    ap.add_argument("--a2a-gbs", type=float, default=0.0,
                    help="model each exchange as this rank's bytes at this rate (GB/s); 0: free")
    ap.add_argument("--host-profile", action="store_true", help="cProfile one eager step after the timed ones")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.config == 5:
        args.partition = "halo"
        g = data.synthetic_scaling_graph(1.0, seed=42)
        fdim, hidden, heads = 256, 256, 4
    else:
        g = data.synthetic_ui_graph(seed=42)
        fdim, hidden, heads = 128, 128, 1
    feats = torch.from_numpy(data.synthetic_item_features(g.n_items, fdim, seed=42)).to(dev)
    ei = torch.from_numpy(g.edge_index_numpy()).to(dev)
    u, i, j = data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, 200_000, seed=42)
    tu, ti, tj = (torch.from_numpy(a).to(dev) for a in (u, i, j))
    torch.manual_seed(42)
    full = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=fdim, hidden=hidden, layers=2, heads=heads,
                      attn_dropout=0.1).to(dev)
    cyc = 0.0
    cal = []
    if args.a2a_gbs > 0:  # calibrate the GPU sleep: cycles per millisecond (median of 6 timings)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1_000_000)
        for n in (20_000_000, 40_000_000) * 3:
            a.record()
            torch.cuda._sleep(n)
            b.record()
            torch.cuda.synchronize()
            cal.append(n / a.elapsed_time(b))
        cyc = float(np.median(cal))
    comm = NullComm(args.world, args.rank, args.a2a_gbs, cyc)
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
        del ei
        ei = None
        torch.cuda.empty_cache()
        comm.own_ids = torch.from_numpy(dg.own_node_ids()[dg.n_own_u:].astype(np.int64))  # own items
        model = D.HaloPyGGAT(full, dg, comm)
        loss_fn = D.halo_bpr_loss
        n_edges = dg.fwd_view.n_fwd_edges
    opt = pkg.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4, capturable=args.graph)

    def step():
        model.train()
        if args.graph:
            _lib.dropout_advance(dev)
        Z = model(feats)
        loss = loss_fn(Z, dg, comm, tu, ti, tj, g.n_users, g.n_items, plan_key="probe")  # fixed triples
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
    comm.modelled_ms = 0.0
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
    if args.host_profile:
        import cProfile
        import io
        import pstats
        prof = cProfile.Profile()
        prof.enable()
        step()
        torch.cuda.synchronize()
        prof.disable()
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(30)
        print(buf.getvalue(), flush=True)
    sleep_check = None
    if cyc > 0:  # the calibration re-checked after the run: one sleep of the modelled per-step exchange
        want = comm.modelled_ms / args.steps
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda._sleep(int(want * cyc))
        b.record()
        torch.cuda.synchronize()
        sleep_check = {"intended_ms": want, "measured_ms": a.elapsed_time(b)}
    print(json.dumps({"config": args.config, "partition": args.partition, "graph": args.graph, "world": args.world,
                      "rank": args.rank, "streams": args.streams, "a2a_gbs": args.a2a_gbs,
                      "sleep_cycles_per_ms": cyc, "sleep_calibration": cal, "sleep_check": sleep_check,
                      "modelled_exchange_ms_per_step": comm.modelled_ms / args.steps if not args.graph else None,
                      "rows": int(dg.R), "local_edges": int(n_edges), "global_edges": int(2 * g.n_interactions),
                      "ms_per_step": el / args.steps * 1e3, "host_enqueue_ms_per_step": th / args.steps * 1e3,
                      "kernel_ms_per_step": kern}), flush=True)


if __name__ == "__main__":
    main()
