"""Multi-GPU paths with the real HIP stages (GPU), checked against the fp64 CPU oracle.

* world_size 1 over RCCL with PPGAT_COMM_ALWAYS=1, so every collective (all_to_all halo,
  all_reduce merges) actually runs through RCCL on the device;
* world_size 2 as two processes sharing the box's single GPU over gloo (device tensors staged
  through the host) -- the N>1 orchestration with the HIP kernels.

Partitions: halo (users and items row-sharded, all_to_all of h at heads 1 and of the
pre-projection x at heads 2), replicated items (fused layer with the ppgat_rep_merge
kernels, heads 1 and 2), and the replicated staged path.  Reference: the unsharded oracle
model (oracle/gat_oracle.py) on the same parameters and dropout masks (dist.SharedSeeds).
Tolerances as tests/test_gpu_parity.py: 1e-5 (outputs, matrices), 1e-4 (vector grads).

Sizes: a 3,800-node toy for the partition / heads matrix, and config 4 itself -- the whole
config-2 graph (255,404 nodes, 2,608,620 columns, its real hubs, halo and plan sizes) at
world 2, against the fp64 oracle run on the device.

Rendezvous: the parent process opens the TCPStore on port 0 (the OS picks a free port at
bind time, so no other process can take it between choosing and binding) and the ranks
join it as clients; torchrun launches use the c10d rendezvous on 127.0.0.1:0, which does
the same.
"""
import importlib
import os
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import assert_kink_ties, check_att_dst, dx_rows, kink_report, kink_sides, row_rel, write_report

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _master_store():
    """A TCPStore server bound to a free port chosen at bind time (held by this process)."""
    return dist.TCPStore("127.0.0.1", 0, None, is_master=True, wait_for_workers=False)


def _setup(dev, heads=1, size="toy"):
    """heads 1, 2: hidden 128; heads 4: hidden 256 (config 5's layer shape: the halo path
    exchanges x and runs the aggregate-then-transform kernels).  size "cfg4": the full
    config-2 graph, features and 200k triples of bench.py (attention dropout 0.1)."""
    pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
    if size == "cfg4":
        g = pkg.data.synthetic_ui_graph(seed=42)
        fdim, p, S, tseed = 128, 0.1, 200_000, 42
        feats = torch.from_numpy(pkg.data.synthetic_item_features(g.n_items, 128, seed=42)).to(dev)
    else:
        g = pkg.data.synthetic_ui_graph(n_users=3000, n_items=800, n_interactions=40_000, seed=5)
        fdim, p, S, tseed = 64, 0.2, 20_000, 1
        feats = torch.from_numpy(pkg.data.synthetic_item_features(g.n_items, 64, seed=5)).to(dev)
    ei = torch.from_numpy(g.edge_index_numpy()).to(dev)
    torch.manual_seed(0)
    hidden = 256 if heads == 4 else 128
    full = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=fdim, hidden=hidden, layers=2, heads=heads,
                      attn_dropout=p)
    with torch.no_grad():
        for conv in full.convs:
            conv.bias.uniform_(-0.1, 0.1)
    full = full.to(dev).train()
    u, i, j = pkg.data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, S, seed=tseed)
    return pkg, g, ei, feats, full, [torch.from_numpy(a).to(dev) for a in (u, i, j)]


def _run(rank, world, out_dir, heads, part, size="toy", dev_index=0):
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)
    if part.endswith("fsplit"):  # the forward split by destination class (read at first use)
        os.environ["PPGAT_FWD_SPLIT"] = "1"
    if part == "halo-dstbwd":  # the round-3 multi-head halo backward (edges at the destination's owner)
        os.environ["PPGAT_HALO_BWD"] = "dst"
        part = "halo"
    elif part == "halo-srcg":  # the source-homed backward with D from the gt GEMM's prologue
        os.environ["PPGAT_XGAT_GATHER"] = "g"
        part = "halo"
    pkg, g, ei, feats, full, (u, i, j) = _setup(dev, heads, size)
    D = pkg.dist
    if part == "halo-g2":
        # the gradient reaching the lower layer is a NEW tensor (2 g, as if a hook sat between the
        # layers) while the layer above has already started that layer's halo exchange from its
        # own dx: the backward must redo the exchange from the real g (dist.py)
        orig = D._halo_xgat_backward_deferred_d

        def _two_g(saved, g_, hg, comm_, stages, want_bias_grad, pre=None, link_in=None):
            return orig(saved, g_ * 2 if pre is not None else g_, hg, comm_, stages, want_bias_grad, pre, link_in)
        D._halo_xgat_backward_deferred_d = _two_g
        part = "halo"
    comm = D.Comm()
    if part == "halo":
        dg = D.build_halo_graph(ei, g.n_nodes, g.n_users, world, rank)
        model = D.HaloPyGGAT(full, dg, comm).train()
        loss_fn, to_global = D.halo_bpr_loss, D.halo_rows_to_global
    else:
        dg = D.build_replicated_graph(ei, g.n_nodes, g.n_users, world, rank)
        st = pkg.hip_ops.HipStages() if part == "replicated-staged" else None
        model = D.ReplicatedPyGGAT(full, dg, comm, stages=st).train()
        loss_fn, to_global = D.replicated_bpr_loss, D.replicated_rows_to_global
    torch.manual_seed(123 + 1000 * rank)
    if size == "cfg4":
        pkg.hip_ops.KINK_TAP = []  # the LeakyReLU side of every local logit (for the oracle)
    Z = model(feats)
    if size == "cfg4":
        torch.save([(e.cpu(), p_.cpu()) for e, p_ in pkg.hip_ops.KINK_TAP[:2]], os.path.join(out_dir, f"kinks_{rank}.pt"))
        pkg.hip_ops.KINK_TAP = None
    loss = loss_fn(Z, dg, comm, u, i, j, g.n_users, g.n_items)
    loss.backward()
    model.allreduce_grads()
    tot = loss.detach().clone()
    comm.all_reduce_(tot)
    Zg = to_global(Z.detach(), dg, comm)
    grads = {n: p.grad.detach().cpu() for n, p in model.named_parameters() if n != "user_emb_local"}
    ug = model._user_rows_global(model.user_emb_local.grad, g.n_users).cpu()
    if part != "halo":
        items = comm.all_gather_rows(Z.detach()[dg.RU:].contiguous()).view(world, g.n_items, -1)
        assert all(torch.equal(items[r], items[0]) for r in range(world)), "item replicas differ"
    if rank == 0:
        torch.save({"Z": Zg.cpu(), "loss": tot.cpu(), "grads": grads, "user_grad": ug},
                   os.path.join(out_dir, f"sharded_{world}.pt"))


def _worker(rank, world, port, out_dir, heads, part, size="toy", backend="gloo"):
    sys.path.insert(0, str(ROOT))
    store = dist.TCPStore("127.0.0.1", port, None, is_master=False)  # the parent holds the server
    if backend == "nccl":  # one GPU per rank (RCCL): the comm-stream overlap paths run for real
        dev = torch.device("cuda", rank)
        dist.init_process_group("nccl", store=store, rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
    try:
        _run(rank, world, out_dir, heads, part, size, dev_index=rank if backend == "nccl" else 0)
    finally:
        dist.destroy_process_group()


def _oracle(heads, size="toy", on_device=False, kink_pos=None, kink_stats=None):
    """The unsharded fp64 oracle model + BPR loss and its gradients (on the CPU, or with the
    oracle's torch ops on the device for the full-size graph); ``kink_pos``: the LeakyReLU side
    per layer and edge the kernels took (tests/test_gpu_fullsize.py KINK_TIE)."""
    from oracle import gat_oracle as O
    dev = torch.device("cuda", 0)
    pkg, g, ei, feats, full, (u, i, j) = _setup(dev, heads, size)
    at = dev if on_device else torch.device("cpu")
    P = {k: v.detach().double().to(at).requires_grad_(True) for k, v in full.named_parameters()}
    torch.manual_seed(123)
    base = pkg.dist._dropout_seed()
    seeds = [pkg.dist.derive_seed(base, k) for k in range(2)]
    p = full.convs[0].dropout
    Z = O.pyg_gat_model(P, feats.double().to(at), ei.to(at), 2, heads, dropout_p=p, seeds=seeds, kink_pos=kink_pos,
                        kink_stats=kink_stats)
    loss = O.bpr_loss(Z, g.n_users, u.to(at), i.to(at), j.to(at))
    loss.backward()
    return Z.detach().cpu(), loss.detach().cpu(), {k: v.grad.cpu() for k, v in P.items()}


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _check(res, ref, n_users=None, name=None):
    Z, loss, grads = ref
    if name is not None:
        write_report(name, {
            "Z_rel": _rel(res["Z"], Z), "item_row_rel_max": row_rel(res["Z"][n_users:], Z[n_users:])[0],
            "user_row_rel_max": row_rel(res["Z"][:n_users], Z[:n_users])[0],
            "loss_rel": abs(float(res["loss"]) - float(loss)) / abs(float(loss)),
            "user_grad_rel": _rel(res["user_grad"], grads["user_emb.weight"]),
            "grad_rel": {k: _rel(v, grads[k]) for k, v in res["grads"].items()}})
    assert _rel(res["Z"], Z) <= 1e-5
    assert abs(float(res["loss"]) - float(loss)) <= 1e-5 * abs(float(loss))
    assert _rel(res["user_grad"], grads["user_emb.weight"]) <= 1e-5
    for k, v in res["grads"].items():
        tol = 1e-5 if v.dim() == 2 else 1e-4  # vector grads: sums over every node, with cancellation
        assert _rel(v, grads[k]) <= tol, (k, _rel(v, grads[k]))


@pytest.mark.parametrize("heads,part", [(1, "halo"), (2, "halo"), (4, "halo"), (1, "replicated"), (2, "replicated"),
                                        (1, "replicated-staged"), (1, "replicated-fsplit"),
                                        (2, "replicated-fsplit")])
def test_sharded_world1_rccl(cuda, tmp_path, monkeypatch, heads, part):
    monkeypatch.setenv("PPGAT_COMM_ALWAYS", "1")  # run every collective through RCCL at world 1
    # fsplit: the forward split by destination class, the item-row merge on the comm stream
    monkeypatch.setenv("PPGAT_FWD_SPLIT", "1" if part.endswith("fsplit") else "0")
    store = _master_store()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=cuda)
    try:
        _run(0, 1, str(tmp_path), heads, part)
    finally:
        dist.destroy_process_group()
    _check(torch.load(tmp_path / "sharded_1.pt", weights_only=False), _oracle(heads))


@pytest.mark.parametrize("heads,part", [(1, "halo"), (2, "halo"), (4, "halo"), (4, "halo-dstbwd"), (4, "halo-srcg"),
                                        (4, "halo-g2"), (1, "replicated"),
                                        (2, "replicated"), (1, "replicated-staged")])
def test_sharded_world2_shared_gpu(cuda, tmp_path, heads, part):
    store = _master_store()
    mp.start_processes(_worker, args=(2, store.port, str(tmp_path), heads, part), nprocs=2, join=True,
                       start_method="spawn")
    del store
    Z, loss, grads = _oracle(heads)
    if part == "halo-g2":  # the lower layer saw 2 g: its parameters' and its inputs' gradients double
        grads = {k: v * 2 if k.startswith(("convs.0.", "item_proj.", "user_emb.")) else v for k, v in grads.items()}
    _check(torch.load(tmp_path / "sharded_2.pt", weights_only=False), (Z, loss, grads))


@pytest.mark.parametrize("world,heads,part", [(3, 4, "halo"), (4, 4, "halo"), (4, 1, "halo"), (4, 1, "replicated")])
def test_sharded_world34_shared_gpu(cuda, tmp_path, world, heads, part):
    """Three and four ranks on this GPU over gloo: the halo plans' runs and halves, the
    touched-rows gradient exchange and the link order with more than one peer per rank (the
    8-GPU node's paths at a size that fits here), against the unsharded fp64 oracle."""
    store = _master_store()
    mp.start_processes(_worker, args=(world, store.port, str(tmp_path), heads, part), nprocs=world, join=True,
                       start_method="spawn")
    del store
    _check(torch.load(tmp_path / f"sharded_{world}.pt", weights_only=False), _oracle(heads))


@pytest.mark.parametrize("heads,part", [(4, "halo"), (4, "halo-g2"), (1, "halo"), (1, "replicated"),
                                        (2, "replicated-fsplit")])
def test_sharded_world2_rccl(cuda, tmp_path, heads, part):
    """World 2 over RCCL, one process per GPU: the communication-stream paths (HaloRows.start's
    overlapped all_to_alls, the backward's early start of the layer below, the Dtab exchange
    beside the main-stream partial exchanges and the column-bound all_reduce; the replicated
    partition's item-row merges on the comm stream) with real cross-rank ordering -- gloo takes
    the synchronous branch.  Needs two visible GPUs: skipped on a one-GPU box."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (one process per GPU over RCCL)")
    store = _master_store()
    mp.start_processes(_worker, args=(2, store.port, str(tmp_path), heads, part, "toy", "nccl"), nprocs=2,
                       join=True, start_method="spawn")
    del store
    Z, loss, grads = _oracle(heads)
    if part == "halo-g2":
        grads = {k: v * 2 if k.startswith(("convs.0.", "item_proj.", "user_emb.")) else v for k, v in grads.items()}
    _check(torch.load(tmp_path / "sharded_2.pt", weights_only=False), (Z, loss, grads))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("part", ["halo", "replicated"])
def test_cfg4_full_graph_world2(cuda, tmp_path, part):
    """Config 4 (BASELINE.json: the config-2 graph row-sharded, all_to_all halo + gradient
    all-reduce) at its real size: the whole 2.6M-column graph, 200k triples, attention dropout
    0.1, two ranks on this GPU over gloo (RCCL on the driver's 8-GPU node).  Z (per row too),
    loss, every dense gradient and the user-row gradient against the unsharded fp64 oracle.
    "replicated" is the partition configs 2/3 use at N > 1."""
    store = _master_store()
    mp.start_processes(_worker, args=(2, store.port, str(tmp_path), 1, part, "cfg4"), nprocs=2, join=True,
                       start_method="spawn")
    del store
    res = torch.load(tmp_path / "sharded_2.pt", weights_only=False)
    n_users, E = 192_403, 2_608_620
    sides = kink_sides([torch.load(tmp_path / f"kinks_{r}.pt", weights_only=False) for r in range(2)], E, 1, 2)
    kst = []
    Z, loss, grads = _oracle(1, "cfg4", on_device=True, kink_pos=[s_.to(cuda) for s_ in sides], kink_stats=kst)
    err = {k: _rel(v, grads[k]) for k, v in res["grads"].items()}
    err["user_emb.weight"] = _rel(res["user_grad"], grads["user_emb.weight"])
    r_items = row_rel(res["Z"][n_users:], Z[n_users:])[0]
    write_report(f"cfg4_world2_{part}", {
        "Z_rel": _rel(res["Z"], Z), "item_row_rel_max": r_items,
        "user_row_rel_max": row_rel(res["Z"][:n_users], Z[:n_users])[0],
        "loss_rel": abs(float(res["loss"]) - float(loss)) / abs(float(loss)), "grad_rel": err,
        "kink_ties_per_layer": kink_report(kst),
        "oracle": "unsharded fp64 oracle on the device, LeakyReLU sides as the kernels took them"})
    assert_kink_ties(kst)  # the kernels' side differs from the fp64 sign only at fp32 ties
    assert _rel(res["Z"], Z) <= 1e-5 and r_items <= 1e-5
    assert abs(float(res["loss"]) - float(loss)) <= 1e-5 * abs(float(loss))
    for k, e in err.items():
        tol = 1e-5 if grads[k].dim() == 2 else 1e-4
        if k.endswith("att_dst"):  # a possibly cancelling sum (conftest.check_att_dst)
            check_att_dst(e * float(grads[k].abs().max()), grads[k], grads[k.replace("att_dst", "att_src")], tol)
            continue
        assert e <= tol, (k, e)


# ---------------------------------------------------------------------------
# config 5's layer on the halo partition at size: one GPU's 25M-edge share of the 200M-edge
# synthetic, GATConv(256, 256, heads=4) (train_gat_pyg.py:77), two ranks
# ---------------------------------------------------------------------------
def _cfg5_setup():
    """The inputs of tests/test_gpu_fullsize.py::test_cfg5_share_layer_full_gradients."""
    import numpy as np
    pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
    g = pkg.data.synthetic_scaling_graph(1 / 8, seed=42)
    N, C, H = g.n_nodes, 256, 4
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.standard_normal((N, C), dtype=np.float32))
    G = torch.from_numpy(rng.standard_normal((N, C), dtype=np.float32))
    torch.manual_seed(9)
    conv = pkg.GATConv(C, C, heads=H, dropout=0.1, add_self_loops=False, concat=False)
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    return pkg, g, g.edge_index_numpy(), x, G, conv


CFG5_SEED = 424242


def _run_cfg5(rank, world, out_dir):
    """One config-5 layer in train mode through dist._HaloLayerX (the non-first layer: user and
    item halo rows of x both exchanged by all_to_all, the halo sources' input gradients returned
    to their owners and added in peer order); the rank's own rows of out and dx, its partial
    dense gradients, the kink sides of its edges and the plan sizes go to ``out_dir``."""
    import numpy as np
    dev = torch.device("cuda", 0)
    pkg, g, ei_np, x, G, conv = _cfg5_setup()
    D = pkg.dist
    comm = D.Comm()
    conv = conv.to(dev).train()
    hg = D.build_halo_graph(torch.from_numpy(ei_np).to(dev), g.n_nodes, g.n_users, world, rank)
    own = torch.from_numpy(hg.own_node_ids())
    x_own = x[own].to(dev).requires_grad_(True)
    pkg.hip_ops.KINK_TAP = []
    try:
        out = D._HaloLayerX.apply(x_own, None, conv.lin.weight, conv.att_src, conv.att_dst, conv.bias, hg, comm,
                                  pkg.hip_ops.HipStages(), conv.heads, conv.out_channels, float(conv.negative_slope),
                                  float(conv.dropout), CFG5_SEED)
        kinks = [(e.cpu(), p_.cpu()) for e, p_ in pkg.hip_ops.KINK_TAP]
    finally:
        pkg.hip_ops.KINK_TAP = None
    (out * G[own].to(dev)).sum().backward()
    torch.cuda.synchronize()
    plans = {"n_own": hg.n_own, "n_halo_users": hg.plan_u.n_recv, "n_halo_items": hg.plan_i.n_recv,
             "send_users": hg.plan_u.n_send, "send_items": hg.plan_i.n_send,
             "local_edges": hg.fwd_view.n_fwd_edges, "row_bytes": 4 * x.size(1)}
    torch.save({"own": own, "out": out.detach().cpu(), "dx": x_own.grad.cpu(), "kinks": kinks, "plans": plans,
                "grads": {n: p_.grad.detach().cpu() for n, p_ in conv.named_parameters()}},
               os.path.join(out_dir, f"cfg5_{rank}.pt"))


def _worker_cfg5(rank, world, port, out_dir):
    sys.path.insert(0, str(ROOT))
    store = dist.TCPStore("127.0.0.1", port, None, is_master=False)
    dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
    try:
        _run_cfg5(rank, world, out_dir)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_cfg5_share_halo_world2(cuda, tmp_path):
    """Config 5's layer (GATConv(256, 256, heads=4), 25M edges, 1.875M rows, attention dropout
    0.1) on the halo partition at world 2 -- two ranks on this GPU over gloo (RCCL on the
    driver's 8-GPU node): the aggregate-then-transform layer with the x halo exchange and the
    gradient return (dist._HaloLayerX) at config-5 plan sizes, hub distribution and exchange
    volumes.  out and dx of every row, dW, datt_src, datt_dst, dbias (summed over the ranks)
    against the exact chunked fp64 oracle (the single-GPU share test's inputs and seed)."""
    from oracle import gat_oracle as O
    store = _master_store()
    mp.start_processes(_worker_cfg5, args=(2, store.port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    del store
    res = [torch.load(tmp_path / f"cfg5_{r}.pt", weights_only=False) for r in range(2)]
    pkg, g, ei_np, x, G, conv = _cfg5_setup()
    N, E, H = g.n_nodes, ei_np.shape[1], conv.heads
    out = torch.empty(N, conv.out_channels)
    dx = torch.empty(N, x.size(1))
    for r in res:
        out[r["own"]] = r["out"]
        dx[r["own"]] = r["dx"]
    grads = {k: res[0]["grads"][k] + res[1]["grads"][k] for k in res[0]["grads"]}  # the 2-rank all-reduce
    sides = kink_sides([r["kinks"] for r in res], E, H, 1)
    del res[0]["out"], res[0]["dx"], res[1]["out"], res[1]["dx"]
    P = {k: v.detach().to(cuda) for k, v in conv.named_parameters()}
    kst = []
    ei = torch.from_numpy(ei_np).to(cuda)
    out_r, dx_r, gr, dxm_r = O.pyg_gat_conv_chunked(P, x.to(cuda), ei, G.to(cuda), H, float(conv.dropout), CFG5_SEED,
                                                    kink_pos=sides[0].to(cuda), kink_stats=kst, dx_message=True)
    U = O.pyg_dx_attention_scale(P, x.to(cuda), ei, G.to(cuda), H, float(conv.dropout), CFG5_SEED)
    cond_dx, dx_rep = dx_rows(dx, dx_r, dxm_r, U, ei)
    del U
    del ei, dxm_r
    names = ("lin.weight", "att_src", "att_dst", "bias")
    err = {"out": _rel(out, out_r.cpu()), "dx": _rel(dx, dx_r.cpu())}
    err.update({k: _rel(grads[k], gr[k].cpu()) for k in names})
    plans = [r["plans"] for r in res]
    rb = plans[0]["row_bytes"]
    write_report("cfg5_share_halo_world2", {
        "edges": E, "nodes": N, "heads": H, "world": 2, "rel": err,
        "row_rel_max": {"out": row_rel(out, out_r.cpu())[0], "dx": row_rel(dx, dx_r.cpu())[0], "dx_cond": cond_dx},
        "dx_rows": dx_rep,
        "kink_ties": kink_report(kst), "plans": plans,
        "exchange_bytes_per_direction": [
            {"recv": (p_["n_halo_users"] + p_["n_halo_items"]) * rb, "send": (p_["send_users"] + p_["send_items"]) * rb}
            for p_ in plans],
        "oracle": "chunked fp64 pyg_gat_conv on the device (unsharded), LeakyReLU sides as the kernels took them"})
    assert_kink_ties(kst)
    assert sum(p_["local_edges"] for p_ in plans) == E
    assert err["out"] <= 1e-5 and err["dx"] <= 1e-5 and err["lin.weight"] <= 1e-5 and err["bias"] <= 1e-5, err
    assert err["att_src"] <= 1e-4, err
    check_att_dst(err["att_dst"] * float(gr["att_dst"].abs().max()), gr["att_dst"].cpu(), gr["att_src"].cpu(), 1e-4)
    # every row of dx within 1e-5 of the scale of its terms (conftest.dx_rows), as single-GPU
    assert cond_dx <= 1e-5, dx_rep


class _StubComm:
    """A one-rank communicator that behaves like RCCL where stream ordering can be seen: the
    collectives run on the CURRENT stream behind a ~1 ms spin kernel and then change the data
    (SUM: +1, MAX: +0.5), so a reader not ordered after the collective reads stale values.
    ``backend`` "nccl" takes the overlapped (comm-stream) paths, anything else the inline ones."""

    def __init__(self, backend):
        self.world, self.rank, self.group, self.active, self.backend = 1, 0, None, True, backend

    def all_reduce_(self, t, op=dist.ReduceOp.SUM):
        torch.cuda._sleep(2_000_000)
        if t.dtype.is_floating_point:
            t.add_(1.0 if op == dist.ReduceOp.SUM else 0.5)
        # integer MAX (the weight-gradient column bound's IEEE bits): one rank's maximum is itself
        return t

    def all_gather_rows(self, t):
        return t.contiguous()

    def reduce_scatter_rows(self, t):
        return t.contiguous()

    def all_to_all_rows(self, t, send_counts, recv_counts, out=None):
        n = int(sum(recv_counts))
        out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device) if out is None else out
        torch.cuda._sleep(2_000_000)
        if n:
            out.copy_(t[:n] * 2.0)
        return out

    def broadcast_int(self, value, src=0):
        return int(value)

    def all_to_all_counts(self, counts):
        return [int(c) for c in counts]


@pytest.mark.parametrize("fsplit", ["0", "1"])
def test_comm_stream_overlap_ordering(cuda, monkeypatch, fsplit):
    """The replicated partition's comm-stream overlaps -- the backward item-row all_reduce
    beside the item sources' edge pass (on by default) and, with PPGAT_FWD_SPLIT=1, the forward
    item-row merge beside the user destinations -- give bitwise the results of the inline
    path when the collective is slow and changes the data (at world 1 over RCCL
    all_reduce is the identity, so an ordering bug would not show there)."""
    monkeypatch.setenv("PPGAT_FWD_SPLIT", fsplit)
    res = {}
    for backend in ("nccl", "inline"):
        pkg, g, ei, feats, full, (u, i, j) = _setup(cuda, 1)
        D = pkg.dist
        comm = _StubComm(backend)
        rg = D.build_replicated_graph(ei, g.n_nodes, g.n_users, 1, 0)
        model = D.ReplicatedPyGGAT(full, rg, comm).train()
        torch.manual_seed(123)
        Z = model(feats)
        loss = D.replicated_bpr_loss(Z, rg, comm, u, i, j, g.n_users, g.n_items)
        loss.backward()
        model.allreduce_grads()
        torch.cuda.synchronize()
        res[backend] = [Z.detach().clone(), loss.detach().clone()] + [
            p.grad.detach().clone() for _, p in sorted(model.named_parameters()) if p.grad is not None]
    assert len(res["nccl"]) == len(res["inline"])
    for a, b in zip(res["nccl"], res["inline"]):
        assert torch.equal(a, b)


class _StubComm2(_StubComm):
    """World 2 as seen from rank 0, in one process: the all_to_all runs on the CURRENT stream
    behind a ~1 ms spin kernel and fills the received rows from the sent ones (row k of the
    result = 2 x sent row k mod n_sent), so a reader not ordered after it reads stale rows."""

    def __init__(self, backend):
        super().__init__(backend)
        self.world = 2

    def all_to_all_rows(self, t, send_counts, recv_counts, out=None):
        n = int(sum(recv_counts))
        out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device) if out is None else out
        torch.cuda._sleep(2_000_000)
        if n:
            if t.size(0):
                out.copy_(t[torch.arange(n, device=t.device) % t.size(0)] * 2.0)
            else:
                out.fill_(0.25)
        return out

    # the halo plans' run exchanges (dist.Comm.exchange / exchange_back): the rows the runs send,
    # then the same slow, data-changing stand-in
    def exchange(self, plan, src, out, part=None):  # (a part rewrites the whole slice the same way)
        return self.all_to_all_rows(src[plan.send_idx], plan.send_counts, plan.recv_counts, out=out)

    def exchange_back(self, plan, halo, out=None):
        return self.all_to_all_rows(halo, plan.recv_counts, plan.send_counts, out=out)


def test_halo_forward_overlap_ordering(cuda):
    """The halo partition's multi-head layers (dist._HaloLayerX, heads 4) with the exchanges on
    the communication stream -- the first layer's halo user rows sent before the item
    projections, the next layer's halo rows sent as each destination-class phase finishes, the
    gradient return beside the own sources' pass -- give bitwise the results of the inline
    path when every all_to_all is slow and produces data only its readers may see."""
    res = {}
    for backend in ("nccl", "inline"):
        pkg, g, ei, feats, full, _ = _setup(cuda, 4)
        D = pkg.dist
        comm = _StubComm2(backend)
        hg = D.build_halo_graph(ei, g.n_nodes, g.n_users, 2, 0)
        assert hg.bipartite and hg.n_halo_u > 0 and hg.plan_i.n_recv > 0
        model = D.HaloPyGGAT(full, hg, comm).train()
        torch.manual_seed(123)
        Z = model(feats)
        G = torch.randn(Z.shape, generator=torch.Generator().manual_seed(7)).to(cuda)
        (Z * G).sum().backward()
        torch.cuda.synchronize()
        res[backend] = [Z.detach().clone()] + [p.grad.detach().clone() for _, p in sorted(model.named_parameters())
                                               if p.grad is not None]
    assert len(res["nccl"]) == len(res["inline"]) > 4
    for a, b in zip(res["nccl"], res["inline"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("cols", [4, 12, 16, 130, 256, 512])
def test_rows_gather_and_return_add_bitwise(cuda, cols):
    """ppgat_rows_gather (the narrow and the one-wave-per-row kernels) equals
    torch indexing, and ppgat_rows_return_add equals the same adds done in peer (k) order --
    bitwise, with rows getting 0 to 11 copies (more than one 8-load batch) and a ragged tail."""
    pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
    st = pkg.hip_ops.HipStages()
    g = torch.Generator(device=cuda).manual_seed(cols)
    n_src, n = 5003, 4097
    src = torch.randn(n_src, cols, device=cuda, generator=g)
    idx = torch.randint(0, n_src, (n,), device=cuda, generator=g)
    assert torch.equal(st.gather_rows(src, idx), src[idx])
    cnt = torch.randint(0, 12, (n,), device=cuda, generator=g)
    ptr = torch.zeros(n + 1, dtype=torch.int32, device=cuda)
    ptr[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    tot = int(ptr[-1])
    ret = torch.randn(tot + 7, cols, device=cuda, generator=g)
    pos = torch.randperm(tot + 7, device=cuda, generator=g)[:tot].to(torch.int32)
    dst = torch.randn(n, cols, device=cuda, generator=g)
    ref = dst.clone()
    for j in range(int(cnt.max())):  # the j-th copy of every row that has one, in k order
        rows = torch.nonzero(cnt > j).squeeze(1)
        ref[rows] += ret[pos[(ptr[rows] + j).long()].long()]
    st.return_add(dst, ret, ptr, pos)
    assert torch.equal(dst, ref)
