#!/usr/bin/env python3
"""Mean per-dispatch value of every counter collected for the kernels whose name contains
PATTERN, over one or more rocprofv3 --pmc output directories:

    python tools/pmc_kernel.py PATTERN DIR [DIR ...]

Prints one JSON object: {counter: mean value per dispatch, "dispatches": n, "avg_us": mean
duration from the trace timestamps}."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    pat, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(list)
    durs = {}
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if pat not in r["Kernel_Name"]:
                    continue
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs[(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    out["dispatches"] = max((len(v) for v in vals.values()), default=0)
    out["avg_us"] = sum(durs.values()) / max(len(durs), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
