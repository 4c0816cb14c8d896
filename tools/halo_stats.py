#!/usr/bin/env python3
"""Halo exchange volume of the row-sharded partition (dist.build_halo_graph) for a config,
computed on the host with the partition code itself (no GPU):

    python tools/halo_stats.py --config 5 --world 8      # 200M-edge synthetic, d=256, heads=4
    python tools/halo_stats.py --config 2 --world 8      # config 4 (config-2 graph)
    python tools/halo_stats.py --config 5 --item-partition contiguous   # the round-3 ownership

Per rank: own rows, halo rows received, rows sent, local (destination-owned) edges; bytes per
layer and direction for the exchanged operand (x: C_in floats when H*C > C_in, else h)."""
import argparse
import importlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
pkg = importlib.import_module("plotpointe-gat-recommendation_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--item-partition", choices=["dealt", "contiguous"], default="dealt")
    ap.add_argument("--runs", action="store_true",
                    help="also the send runs per rank and peer (dist.peer_masks / send_order_key: Comm.exchange "
                         "sends each run straight from the row table)")
    ap.add_argument("--touched", action="store_true",
                    help="also the halo rows the loss's 200k triples touch (bench / scale_probe draw): the rows "
                         "the top layer's g exchange carries (dist._touch_plans)")
    args = ap.parse_args()
    d = pkg.data
    if args.config == 5:
        g = d.synthetic_scaling_graph(1.0, seed=42)
        row_bytes = 256 * 4  # x rows (H*C = 1024 > C_in = 256)
    else:
        g = d.synthetic_ui_graph(seed=42)
        row_bytes = 128 * 4  # h rows (H*C = C_in)
    N, nu, W = g.n_nodes, g.n_users, args.world
    users = np.repeat(np.arange(nu, dtype=np.int64), np.diff(g.user_ptr))
    items = g.user_items.astype(np.int64) + nu
    # the U-I columns come in (u -> i, i -> u) pairs: each interaction is a message both ways
    deg = np.bincount(users, minlength=N) * 2 + np.bincount(items, minlength=N) * 2 + 4.0
    owner, _ = pkg.dist.halo_owner(deg.astype(np.float64), nu, W, args.item_partition)  # the partition code itself
    ou, oi = owner[users], owner[items]
    if args.runs:
        D = pkg.dist
        src = np.concatenate([users, items])
        dst = np.concatenate([items, users])
        mask = D.peer_masks(src, owner[dst], owner, W)
        del src, dst
        key = D.send_order_key(mask, owner, W)
        ids = np.arange(N)
        for r in range(W):
            row = {"rank": r}
            for name, sel in (("users", ids[:nu]), ("items", ids[nu:])):
                mine = sel[owner[sel] == r]
                mine = mine[np.lexsort((mine, key[mine]))]
                m = mask[mine]
                runs = [int(D._runs(((m >> np.uint32(q)) & np.uint32(1)).astype(bool))[0].size) for q in range(W)]
                row[name] = {"rows": int(len(mine)), "runs_per_peer": runs, "runs": int(sum(runs)),
                             "classes": int(np.unique(m).size)}
            print(json.dumps(row), flush=True)
    if args.touched:
        D = pkg.dist
        src = np.concatenate([users, items])
        dst = np.concatenate([items, users])
        mask = D.peer_masks(src, owner[dst], owner, W)
        del src, dst
        tu, ti, tj = d.sample_bpr_numpy(g.user_ptr, g.user_items, g.n_items, 200_000, seed=42)
        T = np.zeros(N, bool)
        T[np.concatenate([tu, ti + nu, tj + nu])] = True
        pc = np.zeros(N, np.int64)  # peers holding each row
        for q in range(W):
            pc += ((mask >> np.uint32(q)) & np.uint32(1)).astype(np.int64)
        print(json.dumps({"touched_rows": int(T.sum()), "touched_users": int(T[:nu].sum()),
                          "touched_items": int(T[nu:].sum())}), flush=True)
        for r in range(W):
            held = ((mask >> np.uint32(r)) & np.uint32(1)).astype(bool)
            own = owner == r
            print(json.dumps({"rank": r, "halo_rows": int(held.sum()), "halo_rows_touched": int((held & T).sum()),
                              "sent_rows": int(pc[own].sum()), "sent_rows_touched": int(pc[own & T].sum()),
                              "recv_GB_dense": held.sum() * row_bytes / 1e9,
                              "recv_GB_touched": (held & T).sum() * row_bytes / 1e9}), flush=True)
    out = []
    for r in range(W):
        own = int((owner == r).sum())
        # edges homed at r: u -> i with owner(i) == r (sources: users), i -> u with owner(u) == r (sources: items)
        m1 = oi == r
        m2 = ou == r
        halo_u = np.unique(users[m1 & (ou != r)])
        halo_i = np.unique(items[m2 & (oi != r)])
        # rows r sends: its users with an item elsewhere, its items with a user elsewhere (unique per peer)
        s_u = np.unique(oi[(ou == r) & (oi != r)].astype(np.int64) * N + users[(ou == r) & (oi != r)]).size
        s_i = np.unique(ou[(oi == r) & (ou != r)].astype(np.int64) * N + items[(oi == r) & (ou != r)]).size
        n_halo = len(halo_u) + len(halo_i)
        out.append({"rank": r, "own_rows": own, "halo_rows": n_halo, "halo_users": len(halo_u),
                    "halo_items": len(halo_i), "sent_rows": s_u + s_i, "sent_users": s_u, "sent_items": s_i,
                    "local_edges": int(m1.sum() + m2.sum()),
                    "recv_GB_per_layer_dir": n_halo * row_bytes / 1e9, "send_GB_per_layer_dir": (s_u + s_i) * row_bytes / 1e9})
        print(json.dumps(out[-1]), flush=True)
    # per training step: layer 1 exchanges the user rows only (the halo items' input rows come
    # from the replicated item features), layer 2 every halo row; each backward mirrors its
    # forward.  An all_to_all ends with its busiest rank: max over ranks of max(send, recv).
    l1 = max(max(o["halo_users"], o["sent_users"]) for o in out) * row_bytes / 1e9
    l2 = max(max(o["halo_rows"], o["sent_rows"]) for o in out) * row_bytes / 1e9
    print(json.dumps({"layer1_GB_busiest_rank": l1, "layer2_GB_busiest_rank": l2, "step_GB_busiest_rank": 2 * (l1 + l2)}))
    sends = [o["send_GB_per_layer_dir"] for o in out]
    print(json.dumps({"config": args.config, "world": W, "item_partition": args.item_partition, "nodes": N,
                      "edges": 2 * len(users), "row_bytes": row_bytes,
                      "max_send_over_mean": max(sends) / (sum(sends) / W),
                      "max_recv_GB": max(o["recv_GB_per_layer_dir"] for o in out),
                      "max_send_GB": max(o["send_GB_per_layer_dir"] for o in out),
                      "max_local_edges": max(o["local_edges"] for o in out)}))


if __name__ == "__main__":
    main()
