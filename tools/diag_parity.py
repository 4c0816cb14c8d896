#!/usr/bin/env python3
"""Diagnose a full-size parity gap: which rows, and which side (our kernels, the device fp64
oracle, or the CPU fp64 oracle) is off.

  python tools/diag_parity.py cfg5   # GATConv(256,256,H=4) on the config-5 share: worst dx rows,
                                     # re-checked by the exact CPU subgraph oracle
  python tools/diag_parity.py cfg4   # the config-2 step: single-GPU model vs device / CPU oracles
"""
import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")
from oracle import gat_oracle as O  # noqa: E402


def rowrel(a, b):
    a, b = a.double().cpu().numpy(), b.double().cpu().numpy()
    nb = np.linalg.norm(b, axis=1)
    r = np.linalg.norm(a - b, axis=1) / np.maximum(nb, 1e-300)
    return r, nb


def cfg5():
    cuda = torch.device("cuda:0")
    H, C = 4, 256
    g = pkg.data.synthetic_scaling_graph(1 / 8, seed=42)
    ei_np = g.edge_index_numpy()
    N = g.n_nodes
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.standard_normal((N, C), dtype=np.float32))
    Gup = torch.from_numpy(rng.standard_normal((N, C), dtype=np.float32))
    torch.manual_seed(9)
    conv = pkg.GATConv(C, C, heads=H, dropout=0.1, add_self_loops=False, concat=False)
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    conv = conv.to(cuda).train()
    cm = importlib.import_module("plotpointe-gat-recommendation_amd.conv")
    cm._dropout_seed = lambda: 424242
    ei = torch.from_numpy(ei_np).to(cuda)
    xd = x.to(cuda).requires_grad_(True)
    Gd = Gup.to(cuda)
    out = conv(xd, ei)
    (out * Gd).sum().backward()
    dx = xd.grad.detach().cpu()
    P = {k: v.detach() for k, v in conv.named_parameters()}
    _, dx_r, _ = O.pyg_gat_conv_chunked(P, x.to(cuda), ei, Gd, H, 0.1, 424242)
    r, nb = rowrel(dx, dx_r)
    worst = np.argsort(-r)[:12]
    indeg = np.bincount(ei_np[1], minlength=N)
    outdeg = np.bincount(ei_np[0], minlength=N)
    print("rows with rel > 1e-5:", int((r > 1e-5).sum()), "of", N, " > 1e-3:", int((r > 1e-3).sum()))
    print("rel quantiles 50/99/99.9/max:", np.quantile(r, [.5, .99, .999]).tolist(), float(r.max()))
    bad = r > 1e-5
    print("bad rows: users", int((bad[:g.n_users]).sum()), "items", int((bad[g.n_users:]).sum()))
    print("bad rows outdeg quantiles:", np.quantile(outdeg[bad], [0, .5, 1]).tolist() if bad.any() else None,
          "all rows outdeg max", int(outdeg.max()))
    # CPU exact subgraph oracle for the worst rows
    csr = O.csr_from_edge_index(ei_np, N)
    rowptr, csr_eid, colptr, row = csr[0], csr[2], csr[3], csr[4]
    Pc = {k: v.double().cpu() for k, v in P.items()}
    res = []
    for s in worst[:6]:
        T = np.unique(np.concatenate([[s], row[colptr[s]:colptr[s + 1]]]))
        cols = np.concatenate([csr_eid[rowptr[t]:rowptr[t + 1]] for t in T])
        sub = ei_np[:, cols]
        nodes = np.union1d(np.unique(sub.reshape(-1)), [s])
        inv = np.searchsorted(nodes, sub.reshape(-1)).reshape(2, -1)
        xs = x[nodes].double().requires_grad_(True)
        o = O.pyg_gat_conv(xs, torch.from_numpy(inv), Pc["lin.weight"], Pc["att_src"], Pc["att_dst"], Pc["bias"], H,
                           dropout_p=0.1, seed=424242, eid=cols)
        Gm = torch.zeros(len(nodes), C, dtype=torch.float64)
        tl = np.searchsorted(nodes, T)
        Gm[tl] = Gup[T].double()
        (o * Gm).sum().backward()
        gcpu = xs.grad[np.searchsorted(nodes, [s])][0]
        # the same subgraph in fp32 (what an fp32 CPU implementation of the reference computes)
        xs32 = x[nodes].float().requires_grad_(True)
        P32 = {k: v.float() for k, v in Pc.items()}
        o32 = O.pyg_gat_conv(xs32, torch.from_numpy(inv), P32["lin.weight"], P32["att_src"], P32["att_dst"],
                             P32["bias"], H, dropout_p=0.1, seed=424242, eid=cols)
        (o32 * Gm.float()).sum().backward()
        g32 = xs32.grad[np.searchsorted(nodes, [s])][0].double()
        e_ours = float((dx[s].double() - gcpu).norm() / gcpu.norm())
        e_dev = float((dx_r[s].cpu() - gcpu).norm() / gcpu.norm())
        e_32 = float((g32 - gcpu).norm() / gcpu.norm())
        # in-degrees of the destinations of s's out-edges (alpha ~ 1 where that is 1)
        dd = indeg[row[colptr[s]:colptr[s + 1]]]
        res.append({"row": int(s), "user": bool(s < g.n_users), "outdeg": int(outdeg[s]), "indeg": int(indeg[s]),
                    "rel_ours_vs_device": float(r[s]), "rel_ours_vs_cpu": e_ours, "rel_device_vs_cpu": e_dev,
                    "rel_fp32_oracle_vs_cpu": e_32, "out_dst_indeg_min": int(dd.min()) if len(dd) else -1,
                    "dx_norm": float(gcpu.norm()), "dx_norm_max_all": float(nb.max())})
        print(res[-1], flush=True)
    return res


def cfg4():
    cuda = torch.device("cuda:0")
    g = pkg.data.synthetic_ui_graph(seed=42)
    feats = torch.from_numpy(pkg.data.synthetic_item_features(g.n_items, 128, seed=42))
    ei = torch.from_numpy(g.edge_index_numpy())
    torch.manual_seed(0)
    full = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=128, hidden=128, layers=2, heads=1, attn_dropout=0.1)
    with torch.no_grad():
        for conv in full.convs:
            conv.bias.uniform_(-0.1, 0.1)
    full = full.to(cuda).train()
    u, i, j = (torch.from_numpy(a) for a in pkg.data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, 200_000,
                                                                     seed=42))
    torch.manual_seed(123)
    base = pkg.dist._dropout_seed()
    seeds = [pkg.dist.derive_seed(base, k) for k in range(2)]
    # ours, single GPU, with exactly these seeds
    cm = importlib.import_module("plotpointe-gat-recommendation_amd.conv")
    it = iter(seeds)
    cm._dropout_seed = lambda: next(it)
    Z = full(feats.to(cuda), ei.to(cuda))
    pkg.bpr_loss(Z, g.n_users, u.to(cuda), i.to(cuda), j.to(cuda)).backward()
    ours = {k: v.grad.detach().double().cpu() for k, v in full.named_parameters()}
    out = {}
    for where, dt in (("cuda", torch.float64), ("cpu", torch.float64), ("cpu32", torch.float32)):
        dev = torch.device(where[:3] if where != "cuda" else "cuda")
        P = {k: v.detach().to(dev, dt).requires_grad_(True) for k, v in full.named_parameters()}
        Zr = O.pyg_gat_model(P, feats.to(dev, dt), ei.to(dev), 2, 1, dropout_p=0.1, seeds=seeds)
        O.bpr_loss(Zr, g.n_users, u.to(dev), i.to(dev), j.to(dev)).backward()
        out[where] = {k: v.grad.detach().double().cpu() for k, v in P.items()}
    rep = {}
    for k in ours:
        a, b, c = ours[k], out["cuda"][k], out["cpu"][k]
        sc = float(c.abs().max())
        rep[k] = {"ours_vs_cpu": float((a - c).abs().max()) / sc, "device_vs_cpu": float((b - c).abs().max()) / sc,
                  "ours_vs_device": float((a - b).abs().max()) / sc,
                  "fp32_oracle_vs_cpu": float((out["cpu32"][k] - c).abs().max()) / sc}
        if k == "user_emb.weight":
            rr, nb = rowrel(a, c)
            r32, _ = rowrel(out["cpu32"][k], c)
            w = np.argsort(-rr)[:5]
            rep[k]["worst_rows"] = [{"row": int(q), "rel_ours": float(rr[q]), "rel_fp32_oracle": float(r32[q]),
                                     "norm": float(nb[q]), "norm_max": float(nb.max())} for q in w]
        print(k, rep[k], flush=True)
    return rep


def cfg4b():
    """Layer 0 of the config-2 step: every intermediate of our backward (h, grad_out, D_i,
    ds_src, ds_dst, dh, dz) against its fp64 value, on the worst user rows."""
    cuda = torch.device("cuda:0")
    ops = importlib.import_module("plotpointe-gat-recommendation_amd.hip_ops")
    g = pkg.data.synthetic_ui_graph(seed=42)
    feats = torch.from_numpy(pkg.data.synthetic_item_features(g.n_items, 128, seed=42))
    ei_np = g.edge_index_numpy()
    ei = torch.from_numpy(ei_np)
    torch.manual_seed(0)
    full = pkg.PyGGAT(g.n_users, g.n_items, item_feat_dim=128, hidden=128, layers=2, heads=1, attn_dropout=0.1)
    with torch.no_grad():
        for conv in full.convs:
            conv.bias.uniform_(-0.1, 0.1)
    full = full.to(cuda).train()
    u, i, j = (torch.from_numpy(a) for a in pkg.data.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, 200_000,
                                                                     seed=42))
    torch.manual_seed(123)
    base = pkg.dist._dropout_seed()
    seeds = [pkg.dist.derive_seed(base, k) for k in range(2)]
    cm = importlib.import_module("plotpointe-gat-recommendation_amd.conv")
    it = iter(seeds)
    cm._dropout_seed = lambda: next(it)
    cap = []
    orig = ops._bwd_edges_dst

    def spy(gr, h, s_src, nstate, grad_out, D, S, heads, channels, mode, slope, p, seed, seed_buf=None):
        dzb = torch.empty(max(gr.n_edges, 1) * heads, dtype=torch.float32, device=h.device)
        ops._bwd_edges_src(gr, gr.bwd_sched, 0, h, s_src, nstate, grad_out, D, S, dzb, heads, channels, mode, slope,
                           p, seed, seed_buf)
        ops._bwd_dst_sum(gr, dzb, S, heads)
        cap.append(dict(h=h.detach().clone(), s_src=s_src.detach().clone(), nstate=nstate.detach().clone(),
                        g=grad_out.detach().clone(), D=D.detach().clone(), S=S.detach().clone(), dz=dzb.clone(),
                        csc_eid=gr.csc_eid.detach().long().clone(), row=gr.row.detach().long().clone(),
                        seed=int(seed_buf.item()) if seed_buf is not None else None))
    ops._bwd_edges_dst = spy
    Z = full(feats.to(cuda), ei.to(cuda))
    pkg.bpr_loss(Z, g.n_users, u.to(cuda), i.to(cuda), j.to(cuda)).backward()
    torch.cuda.synchronize()
    ours_ug = full.user_emb.weight.grad.detach().double().cpu()
    L0 = cap[-1]  # backward runs layer 1 first: the last capture is layer 0
    # fp64 reference with the intermediates of layer 0
    dev = cuda
    P = {k: v.detach().to(dev, torch.float64).requires_grad_(True) for k, v in full.named_parameters()}
    f64 = feats.to(dev, torch.float64)
    eid = ei.to(dev)
    x0 = torch.cat([P["user_emb.weight"], f64 @ P["item_proj.weight"].t() + P["item_proj.bias"]], 0)
    out0 = O.pyg_gat_conv(x0, eid, P["convs.0.lin.weight"], P["convs.0.att_src"], P["convs.0.att_dst"],
                          P["convs.0.bias"], 1, dropout_p=0.1, seed=seeds[0])
    out0.retain_grad()
    Zr = O.pyg_gat_conv(out0, eid, P["convs.1.lin.weight"], P["convs.1.att_src"], P["convs.1.att_dst"],
                        P["convs.1.bias"], 1, dropout_p=0.1, seed=seeds[1])
    O.bpr_loss(Zr, g.n_users, u.to(dev), i.to(dev), j.to(dev)).backward()
    with torch.no_grad():
        W = P["convs.0.lin.weight"]
        h = x0 @ W.t()
        ss = h @ P["convs.0.att_src"].view(-1)
        sd = h @ P["convs.0.att_dst"].view(-1)
        src, dst = eid[0], eid[1]
        z = ss[src] + sd[dst]
        e = torch.where(z > 0, z, 0.2 * z)
        N = h.size(0)
        emax = torch.full((N,), -np.inf, dtype=torch.float64, device=dev).scatter_reduce(0, dst, e, "amax")
        ex = (e - emax[dst]).exp()
        s = torch.zeros(N, dtype=torch.float64, device=dev).scatter_add_(0, dst, ex) + 1e-16
        al = ex / s[dst]
        d = torch.from_numpy(O.dropout_scale(seeds[0], np.arange(ei.size(1)), 0, 0.1)).to(dev, torch.float64)
        go = out0.grad
        da = d * (go[dst] * h[src]).sum(1)
        Dref = torch.zeros(N, dtype=torch.float64, device=dev).index_add_(0, dst, al * da)
        dz = al * (da - Dref[dst]) * torch.where(z > 0, 1.0, 0.2)
        ds_src = torch.zeros(N, dtype=torch.float64, device=dev).index_add_(0, src, dz)
        ds_dst = torch.zeros(N, dtype=torch.float64, device=dev).index_add_(0, dst, dz)
        dh = torch.zeros(N, 128, dtype=torch.float64, device=dev).index_add_(0, src, (al * d)[:, None] * go[dst])
    ref_ug = P["user_emb.weight"].grad.detach().cpu()
    rr, nb = rowrel(ours_ug, ref_ug)
    worst = np.argsort(-rr)[:4]
    rep = []

    def r(a, b):
        a, b = a.double().cpu(), b.double().cpu()
        return float((a - b).norm() / max(float(b.norm()), 1e-300))
    for q in worst:
        q = int(q)
        ine = np.flatnonzero(ei_np[1] == q)
        oute = np.flatnonzero(ei_np[0] == q)
        rec = {"row": q, "rel_user_grad": float(rr[q]), "in_deg": len(ine), "out_deg": len(oute),
               "h": r(L0["h"][q], h[q]), "grad_out": r(L0["g"][q], go[q]),
               "D_i": [float(L0["nstate"][q, 0, 3]), float(Dref[q])],
               "ds_src": [float(L0["S"][q, 0]), float(ds_src[q])], "ds_dst": [float(L0["S"][q, 1]), float(ds_dst[q])],
               "dh": r(L0["D"][q], dh[q]),
               "in_edges": [{"src": int(ei_np[0, k]), "alpha": float(al[k]), "drop": float(d[k]), "dz": float(dz[k]),
                             "D_src_ours": float(L0["nstate"][int(ei_np[0, k]), 0, 3]),
                             "D_src_ref": float(Dref[int(ei_np[0, k])])} for k in ine[:16]],
               "out_edges": [{"dst": int(ei_np[1, k]), "alpha": float(al[k]), "drop": float(d[k]), "dz": float(dz[k]),
                              "indeg_dst": int((ei_np[1] == ei_np[1, k]).sum()),
                              "D_dst_ours": float(L0["nstate"][int(ei_np[1, k]), 0, 3]),
                              "D_dst_ref": float(Dref[int(ei_np[1, k])]),
                              "g_dst_rel": r(L0["g"][int(ei_np[1, k])], go[int(ei_np[1, k])])} for k in oute[:16]]}
        rep.append(rec)
        print(json.dumps(rec), flush=True)
    # global view of each intermediate
    glob = {"grad_out": float((L0["g"].double() - go).abs().max() / go.abs().max()),
            "D_i": float((L0["nstate"][:, 0, 3].double() - Dref).abs().max() / Dref.abs().max()),
            "ds_src": float((L0["S"][:, 0].double() - ds_src).abs().max() / ds_src.abs().max()),
            "ds_dst": float((L0["S"][:, 1].double() - ds_dst).abs().max() / ds_dst.abs().max()),
            "dh": float((L0["D"].double() - dh).abs().max() / dh.abs().max()),
            "h": float((L0["h"].double() - h).abs().max() / h.abs().max())}
    # per-edge logit gradients, CSC order
    E = ei.size(1)
    ceid = L0["csc_eid"][:E]
    dz_o = L0["dz"][:E].double()
    dz_r = dz[ceid]
    err = (dz_o - dz_r).abs()
    glob["dz"] = float(err.max() / dz_r.abs().max())
    glob["seed_used"] = L0["seed"]
    glob["seed_passed"] = seeds[0]
    top = torch.argsort(err, descending=True)[:12]
    ed = []
    for k in top.tolist():
        e_ = int(ceid[k])
        ed.append({"csc_pos": k, "eid": e_, "src": int(ei_np[0, e_]), "dst": int(ei_np[1, e_]),
                   "row_in_csc": int(L0["row"][k]), "dz_ours": float(dz_o[k]), "dz_ref": float(dz_r[k]),
                   "alpha": float(al[e_]), "drop": float(d[e_]), "z": float(z[e_]),
                   "alpha_d_da": float(al[e_] * da[e_]), "alpha_D": float(al[e_] * Dref[int(ei_np[1, e_])])})
        print(json.dumps(ed[-1]), flush=True)
    nbad = int((err > 1e-3 * dz_r.abs().max()).sum())
    glob["edges_dz_err_gt_1e-3"] = nbad
    print("global", json.dumps(glob), flush=True)
    rep.append({"global": glob, "worst_edges": ed})
    return rep


if __name__ == "__main__":
    what = sys.argv[1]
    res = {"cfg5": cfg5, "cfg4": cfg4, "cfg4b": cfg4b}[what]()
    outp = ROOT / "gpurun_out" / f"diag_{what}.json"
    outp.parent.mkdir(exist_ok=True)
    outp.write_text(json.dumps(res, indent=2))
