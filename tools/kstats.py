#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv per training step: python tools/kstats.py FILE STEPS"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs'])/steps/1e3:8.1f} us/step  calls/step={int(r['Calls'])/steps:5.1f}  "
          f"avg={float(r['AverageNs'])/1e3:7.1f} us  {r['Name'][:100]}")
print(f"total {tot/steps/1e6:.3f} ms/step")
