#!/usr/bin/env python3
"""Average each PMC counter per dispatch, per kernel, over a rocprofv3
counter_collection.csv (the last dispatches of every kernel: steady state)."""
import collections
import csv
import sys


def main(path, last=3):
    rows = list(csv.DictReader(open(path)))
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gw::", "")
        by[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = []
    for k, cs in by.items():
        vals = {}
        for c, lst in cs.items():
            # sum over per-XCD/instance rows of one dispatch, then average the last dispatches
            per = collections.defaultdict(float)
            for d, v in lst:
                per[d] += v
            ds = sorted(per)[-last:]
            vals[c] = sum(per[d] for d in ds) / len(ds)
        out.append((k, vals))
    out.sort(key=lambda kv: -max(kv[1].values()))
    for k, vals in out[:14]:
        print(f"{k[:40]:40s} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))


if __name__ == "__main__":
    main(sys.argv[1])
