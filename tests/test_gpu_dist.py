"""Row-sharded path with the real HIP stages (GPU): world_size 1 over RCCL, and world_size
2 as two processes sharing the box's single GPU with gloo (device tensors staged through
the host) -- both must equal the unsharded single-GPU model (fp32 tolerance 1e-5)."""
import importlib
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(dev, heads=1):
    pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
    g = pkg.data.synthetic_ui_graph(n_users=3000, n_items=800, n_interactions=40_000, seed=5)
    ei = torch.from_numpy(g.edge_index_numpy()).to(dev)
    feats = torch.from_numpy(pkg.data.synthetic_item_features(g.n_items, 64, seed=5)).to(dev)
    torch.manual_seed(0)
    full = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=64, hidden=128, layers=2, heads=heads, attn_dropout=0.2)
    with torch.no_grad():
        for conv in full.convs:
            conv.bias.uniform_(-0.1, 0.1)
    full = full.to(dev).train()
    u, i, j = pkg.data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, 20_000, seed=1)
    return pkg, g, ei, feats, full, [torch.from_numpy(a).to(dev) for a in (u, i, j)]


def _sharded(rank, world, out_dir, heads, segmented=True):
    dev = torch.device("cuda", 0)
    pkg, g, ei, feats, full, (u, i, j) = _setup(dev, heads)
    D = pkg.dist
    comm = D.Comm()
    if str(segmented).startswith("replicated"):
        return _replicated(rank, world, out_dir, dev, pkg, g, ei, feats, full, (u, i, j), comm,
                           staged=segmented == "replicated-staged")
    segs = [(0, g.n_users), (g.n_users, g.n_nodes)] if segmented else None
    dg = D.build_dist_graph(ei, g.n_nodes, world, rank, segments=segs)
    model = D.ShardedPyGGAT(full, dg, comm).train()
    torch.manual_seed(123)
    Z = model(feats)
    loss = D.sharded_bpr_loss(Z, dg, comm, u, i, j, g.n_users, g.n_items)
    loss.backward()
    model.allreduce_grads()
    tot = loss.detach().clone()
    comm.all_reduce_(tot)
    Zg = D.gather_rows_to_global(Z.detach(), dg, comm)
    grads = {n: p.grad.detach().cpu() for n, p in model.named_parameters() if n != "user_emb_local"}
    C = model.user_emb_local.size(1)
    blk = torch.zeros(dg.R, C, device=dev)
    blk[:model.u1 - model.u0] = model.user_emb_local.grad
    ug = comm.all_gather_rows(blk).cpu()
    rows = [ug[r * dg.R: r * dg.R + (min(int(dg.bounds[r + 1]), g.n_users) - min(int(dg.bounds[r]), g.n_users))]
            for r in range(world)]
    if rank == 0:
        torch.save({"Z": Zg.cpu(), "loss": tot.cpu(), "grads": grads, "user_grad": torch.cat(rows)},
                   os.path.join(out_dir, f"sharded_{world}.pt"))


def _replicated(rank, world, out_dir, dev, pkg, g, ei, feats, full, uij, comm, staged=False):
    """Users sharded, item rows on every rank (dist.build_replicated_graph); the fused
    layer with RepHooks, or (staged) the stage-by-stage path the CPU tests also run."""
    D = pkg.dist
    u, i, j = uij
    rg = D.build_replicated_graph(ei, g.n_nodes, g.n_users, world, rank)
    model = D.ReplicatedPyGGAT(full, rg, comm, stages=pkg.hip_ops.HipStages() if staged else None).train()
    torch.manual_seed(123)
    Z = model(feats)
    loss = D.replicated_bpr_loss(Z, rg, comm, u, i, j, g.n_users, g.n_items)
    loss.backward()
    model.allreduce_grads()
    tot = loss.detach().clone()
    comm.all_reduce_(tot)
    Zg = D.replicated_rows_to_global(Z.detach(), rg, comm)
    items = comm.all_gather_rows(Z.detach()[rg.RU:].contiguous()).view(world, g.n_items, -1)
    grads = {n: p.grad.detach().cpu() for n, p in model.named_parameters() if n != "user_emb_local"}
    blk = torch.zeros(rg.RU_max, model.user_emb_local.size(1), device=dev)
    blk[:model.u1 - model.u0] = model.user_emb_local.grad
    ug = comm.all_gather_rows(blk).cpu()
    ub = rg.user_bounds
    rows = [ug[r * rg.RU_max: r * rg.RU_max + int(ub[r + 1] - ub[r])] for r in range(world)]
    if rank == 0:
        assert all(torch.equal(items[r], items[0]) for r in range(world)), "item replicas differ"
        torch.save({"Z": Zg.cpu(), "loss": tot.cpu(), "grads": grads, "user_grad": torch.cat(rows)},
                   os.path.join(out_dir, f"sharded_{world}.pt"))


def _worker(rank, world, port, out_dir, heads, segmented=True):
    sys.path.insert(0, str(ROOT))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _sharded(rank, world, out_dir, heads, segmented)
    finally:
        dist.destroy_process_group()


def _unsharded(dev, heads):
    pkg, g, ei, feats, full, (u, i, j) = _setup(dev, heads)
    torch.manual_seed(123)
    Z = full(feats, ei)
    loss = pkg.bpr_loss(Z, g.n_users, u, i, j)
    loss.backward()
    return Z.detach().cpu(), loss.detach().cpu(), {n: p.grad.detach().cpu() for n, p in full.named_parameters()}


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _check(res, ref):
    Z, loss, grads = ref
    assert _rel(res["Z"], Z) <= 1e-5
    assert abs(float(res["loss"]) - float(loss)) <= 1e-5 * abs(float(loss))
    assert _rel(res["user_grad"], grads["user_emb.weight"]) <= 1e-5
    # vector-valued grads (att_*, bias, item_proj.bias) are sums over every node with
    # cancellation, and the two sides sum in different orders: same 1e-4 bound as the
    # attention-vector grads of test_gpu_parity.py against the oracle.  Here BOTH sides are
    # fp32 sums in different orders, so their errors vs the exact value can add: 2x that
    # bound for the attention vectors (measured 1.2e-4 on convs.1.att_dst once the
    # destination-sum reductions changed order; each side stays within 1e-4 of the oracle)
    for k, v in res["grads"].items():
        tol = 1e-5 if v.dim() == 2 and "att" not in k else (2e-4 if "att" in k else 1e-4)
        assert _rel(v, grads[k]) <= tol, k


@pytest.mark.parametrize("heads,segmented", [(1, True), (2, False), (1, "replicated"), (2, "replicated"),
                                             (1, "replicated-staged")])
def test_sharded_world1_rccl(cuda, tmp_path, heads, segmented):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda)
    try:
        _sharded(0, 1, str(tmp_path), heads, segmented)
    finally:
        dist.destroy_process_group()
    _check(torch.load(tmp_path / "sharded_1.pt", weights_only=False), _unsharded(cuda, heads))


@pytest.mark.parametrize("segmented", [True, False, "replicated", "replicated-staged"])
def test_sharded_world2_shared_gpu(cuda, tmp_path, segmented):
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), 1, segmented), nprocs=2, join=True,
                       start_method="spawn")
    _check(torch.load(tmp_path / "sharded_2.pt", weights_only=False), _unsharded(cuda, 1))


def test_bench_two_ranks_rehearsal(cuda, tmp_path):
    """The N>1 flow of bench.py (torch.distributed.run launch, row-sharded model, sharded
    loss, grad all-reduce, Adam, max-over-ranks timing, one JSON line from rank 0), two
    ranks sharing this box's GPU over gloo -- the driver's 2/4/8-GPU runs use RCCL."""
    import json
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--dist-backend", "gloo"]
    p = subprocess.run(cmd, cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["scaling"] == "strong" and res["value"] > 0
    assert res["config"]["parallelism"].startswith("user-sharded x2")
