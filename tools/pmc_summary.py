#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT_JSON [CONFIG [key=value ...]]

(key=value pairs are copied into the JSON, e.g. scale=0.125 bwd_gather=g for config 5: bench.py
uses a summary only for the workload it was collected on.)

gfx950 corrections (MI355X_MICROARCH.md "HBM"): counters are in KiB (x1024); FETCH_SIZE
reports 1/2 of the bytes of a wide (16 B/lane) coalesced read -- all of our kernels read
with 16-byte float4 accesses, so FETCH is doubled; WRITE_SIZE is exact for 16-B stores.
The correction is cross-checked on k_scores, whose algorithmic bytes are exact
(reads h once: N*H*C*4, writes 2*N*H*4).
"""
import csv
import glob
import json
import sys
from collections import defaultdict

KERNELS = {"k_fwd<": "fwd_long", "k_fwd_short<": "fwd_short", "k_bwd_src<": "bwd_src_long",
           "k_bwd_src_short<": "bwd_src_short", "k_bwd_epi<": "bwd_epi", "k_bwd_pro<": "bwd_pro",
           "k_scores<": "scores", "k_gemm_tn": "gemm_tn", "k_bpr_chunks<": "bpr_chunks", "k_bpr_fwd<": "bpr_fwd",
           "k_proj16<0>": "proj_fwd", "k_proj16<1>": "proj_dx", "k_tn128<": "tn128", "k_adam": "adam",
           # the multi-head (aggregate-then-transform) edge passes: one kernel each
           "k_fwd_x<": "fwd", "k_bwd_x<": "bwd_src", "k_bwd_g<": "bwd_src"}
# one edge pass = its one-item-per-wave kernel + its four-items-per-wave short-item kernel
PASSES = {"fwd": ("fwd_long", "fwd_short"), "bwd_src": ("bwd_src_long", "bwd_src_short")}


def load(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            for pat, key in KERNELS.items():
                if pat in name:
                    vals[key].append(float(r["Counter_Value"]))
    return vals


def main():
    fd, wd, out = sys.argv[1:4]
    config = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    dram_dir = None
    extra = []
    for kv in sys.argv[5:]:
        if kv.startswith("dram_dir="):
            dram_dir = kv.split("=", 1)[1]
        else:
            extra.append(kv)
    sys.argv[5:] = extra
    fetch = load(fd, "FETCH_SIZE")
    write = load(wd, "WRITE_SIZE")
    res = {"note": "per-launch HBM-side bytes (L2 fabric requests, Infinity-Cache hits included); "
                   "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->bytes",
           "config": config, "per_launch_bytes": {}, "raw_kib": {}}
    for kv in sys.argv[5:]:
        key, val = kv.split("=", 1)
        try:
            res[key] = float(val)
        except ValueError:
            res[key] = val
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(len(fetch.get(k, [])), 1)
        w = sum(write.get(k, [0])) / max(len(write.get(k, [])), 1)
        res["raw_kib"][k] = {"fetch": f, "write": w, "launches": len(fetch.get(k, []))}
        res["per_launch_bytes"][k] = (2 * f + w) * 1024
    for k, parts in PASSES.items():
        if any(q in res["per_launch_bytes"] for q in parts):
            res["per_launch_bytes"][k] = sum(res["per_launch_bytes"].get(q, 0.0) for q in parts)
    if dram_dir:
        # a third pass: the L2's fabric requests split by destination (TCC_EA0_{RD,WR}REQ vs their
        # _DRAM parts, "destined for DRAM (MC)").  The memory-side Infinity Cache sits behind the
        # MC, so _DRAM requests still include MALL hits: this splits off GMI/IO traffic, not the
        # on-die cache (rocprofv3 exposes no MALL hit counter on gfx950)
        cnt = {c: load(dram_dir, c) for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_WRREQ_sum",
                                              "TCC_EA0_WRREQ_DRAM_sum")}
        mean = lambda c, k: sum(cnt[c].get(k, [0])) / max(len(cnt[c].get(k, [])), 1)  # noqa: E731
        res["dram_destined"] = {}
        res["per_launch_dram_bytes"] = {}
        for k in res["raw_kib"]:
            rd, rdd, wr, wrd = (mean(c, k) for c in cnt)
            frd = rdd / rd if rd else 0.0
            fwr = wrd / wr if wr else 0.0
            f, w = res["raw_kib"][k]["fetch"], res["raw_kib"][k]["write"]
            res["dram_destined"][k] = {"rdreq": rd, "rdreq_dram": rdd, "wrreq": wr, "wrreq_dram": wrd,
                                       "read_frac": frd, "write_frac": fwr}
            res["per_launch_dram_bytes"][k] = (2 * f * frd + w * fwr) * 1024
        for k, parts in PASSES.items():
            if any(q in res["per_launch_dram_bytes"] for q in parts):
                res["per_launch_dram_bytes"][k] = sum(res["per_launch_dram_bytes"].get(q, 0.0) for q in parts)
    json.dump(res, open(out, "w"), indent=2)
    print(json.dumps(res, indent=2))


if __name__ == "__main__":
    main()
