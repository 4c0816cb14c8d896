#!/usr/bin/env python3
"""Where a scale_probe step waits on the modelled exchange: reads a rocprofv3 kernel trace of
`tools/scale_probe.py --streams --a2a-gbs G` (the exchange stand-in is torch's spin kernel on
the communication stream) and prints, for the last full step (between the last two Adam kernels),
the compute-stream idle gaps longer than a threshold with the kernels around them and the sleeps
in flight -- i.e. the exposed exchange and what it blocks.

    python tools/probe_timeline.py TRACE_CSV [--min-gap-us 200]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-gap-us", type=float, default=200.0)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    for r in rows:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["t0"])
    adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    a, b = adam[-2] + 1, adam[-1] + 1
    step = rows[a:b]
    is_sleep = lambda r: "sleep" in r["Kernel_Name"].lower() or "spin_kernel" in r["Kernel_Name"]
    sleeps = [r for r in step if is_sleep(r)]
    comp = [r for r in step if not is_sleep(r)]
    per_q = defaultdict(float)
    for r in comp:
        per_q[r["Queue_Id"]] += (r["t1"] - r["t0"]) / 1e3
    t_start, t_end = step[0]["t0"], step[-1]["t1"]
    print(f"step span {(t_end - t_start) / 1e6:.2f} ms; compute kernels {sum(per_q.values()) / 1e3:.2f} ms "
          f"(by queue: {dict((q, round(v / 1e3, 2)) for q, v in per_q.items())}); "
          f"sleeps {sum(r['t1'] - r['t0'] for r in sleeps) / 1e6:.2f} ms in {len(sleeps)}")
    # compute-idle intervals: no compute kernel running on any queue
    iv = sorted((r["t0"], r["t1"], r) for r in comp)
    gaps, cur_end, prev = [], iv[0][1], iv[0][2]
    for t0, t1, r in iv[1:]:
        if t0 > cur_end:
            gaps.append((cur_end, t0, prev, r))
        if t1 > cur_end:
            cur_end, prev = t1, r
    total = sum(g[1] - g[0] for g in gaps) / 1e6
    print(f"compute idle: {total:.2f} ms in {len(gaps)} gaps")
    for g0, g1, before, after in gaps:
        d = (g1 - g0) / 1e3
        if d < args.min_gap_us:
            continue
        fly = [s for s in sleeps if s["t0"] < g1 and s["t1"] > g0]
        print(f"  {(g0 - t_start) / 1e6:7.2f} ms +{d / 1e3:6.2f} ms  after {before['Kernel_Name'][:48]:48s}  "
              f"before {after['Kernel_Name'][:48]:48s}  sleeps in flight: {len(fly)}")


if __name__ == "__main__":
    main()
