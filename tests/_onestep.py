"""Shared pieces of the one-step training parity tests (fixture ``tests/golden/onestep_cfg1.*``,
written by ``make_golden.py onestep`` from the reference trainer's own main() run: its full
state after 0, 1, 2, 5, 8, 12, 16, 19 optimizer steps and the reference's one-epoch replays
of each state at four thread counts and in float64).

* ``load_state(s)``   -- the saved state: params, Adam moments and step count, both RNG states.
* ``inputs(pkg)``     -- the config-1 inputs exactly as main() builds them (our data module's
  restatements, bit-exact against the reference: tests/test_data_plumbing.py).
* ``f64_step``        -- the epoch in float64 on the CPU: oracle.custom_gat_model (the restated
  SimpleGATLayer stack), oracle.bpr_loss, torch autograd, torch.optim.Adam in float64.  Pinned
  to the reference's own float64 replay by the fixture's checksums
  (tests/test_onestep_oracle.py).
* ``grad_stats``      -- a gradient against the float64 one: max|g - g64| / max|g64| per tensor
  and the entries whose sign differs (an early Adam step is ~lr * sign(g)).
"""
from __future__ import annotations

import json
import random

import numpy as np
import torch

from conftest import GOLDEN

FIX = GOLDEN / "onestep_cfg1"
SAMPLES = 200_000
LR, WD = 1e-3, 1e-4          # train_gat_custom.py Config.lr / l2 (:53-54)


def load():
    arrays = np.load(str(FIX) + ".npz")
    meta = json.loads((GOLDEN / "onestep_cfg1.json").read_text())
    return arrays, meta


def load_state(arrays, meta, s: int):
    p = f"s{s}__"
    keys = [k[len(p + "param__"):] for k in arrays.files if k.startswith(p + "param__")]
    params = {k: torch.from_numpy(arrays[p + "param__" + k].copy()) for k in keys}
    step = float(arrays[p + "step"])
    moments = None
    if step > 0:
        moments = {k: (torch.from_numpy(arrays[p + "exp_avg__" + k].copy()),
                       torch.from_numpy(arrays[p + "exp_avg_sq__" + k].copy())) for k in keys}
    ms = meta["states"][str(s)]
    ver, gauss = ms["py_random_version_gauss"]
    py_random = (ver, tuple(int(v) for v in arrays[p + "py_random"]), gauss)
    kind, pos, has_g, cg = ms["np_random"]
    np_random = (kind, arrays[p + "np_random_key"].copy(), pos, has_g, cg)
    return dict(params=params, step=step, moments=moments, py_random=py_random, np_random=np_random)


def inputs(pkg):
    d = pkg.data
    inter = d.synthetic_interactions_small(seed=0)
    maps = d.node_maps_from_interactions(inter)
    u2i, i2i = d.index_maps(maps)
    tr, va, _ = d.map_splits_to_index(*d.build_splits(inter), u2i, i2i)
    n_users, n_items = int(maps["n_users"]), int(maps["n_items"])
    feats = np.random.RandomState(0).standard_normal((n_items, 384)).astype(np.float32)
    ei = d.build_edge_index(n_users, n_items, tr)
    return dict(tr=tr, va=va, n_users=n_users, n_items=n_items, feats=feats, ei=ei)


def make_adam(params, st, device=None):
    """torch.optim.Adam(lr=1e-3, weight_decay=1e-4) over ``params`` (named order) carrying the
    saved moments and step count, as main()'s optimizer held them."""
    opt = torch.optim.Adam(list(params.values()), lr=LR, weight_decay=WD)
    if st["moments"] is not None:
        for k, p in params.items():
            m, v = st["moments"][k]
            opt.state[p] = {"step": torch.tensor(st["step"]), "exp_avg": m.to(p.device, p.dtype).clone(),
                            "exp_avg_sq": v.to(p.device, p.dtype).clone()}
    return opt


def sample_triples(pkg, st, inp):
    random.setstate(st["py_random"])
    return pkg.data.sample_bpr_epoch(inp["tr"], inp["n_items"], SAMPLES)


def f64_step(pkg, oracle, st, inp):
    """The epoch in float64 on the CPU (loss, gradients, next params, next eval item rows)."""
    u, i, j = (torch.from_numpy(a).long() for a in sample_triples(pkg, st, inp))
    P = {k: v.double().clone().requires_grad_(True) for k, v in st["params"].items()}
    feats = torch.from_numpy(inp["feats"]).double()
    Z = oracle.custom_gat_model(P, feats, inp["ei"], 2)
    loss = oracle.bpr_loss(Z, inp["n_users"], u, i, j)
    opt = make_adam(P, st)
    opt.zero_grad()
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in P.items()}
    opt.step()
    with torch.no_grad():
        Zn = oracle.custom_gat_model(P, feats, inp["ei"], 2)
    return dict(loss=float(loss.detach()), grads=grads, params={k: p.detach().clone() for k, p in P.items()},
                items=Zn[inp["n_users"]:].numpy(), triples=(u, i, j))


def grad_stats(g, g64):
    out = {}
    for k, ref in g64.items():
        a = np.asarray(g[k].detach().double().cpu() if torch.is_tensor(g[k]) else g[k], np.float64)
        b = np.asarray(ref.double() if torch.is_tensor(ref) else ref, np.float64)
        out[k] = {"maxabs_rel": float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)),
                  "sign_flips": int(((np.sign(a) != np.sign(b)) & (b != 0)).sum())}
    return out


def lr_flips(params, params64):
    """Parameters whose step differs from the float64 step by more than lr / 2."""
    return int(sum(int((p.detach().double().cpu() - params64[k]).abs().gt(0.5 * LR).sum())
                   for k, p in params.items()))
