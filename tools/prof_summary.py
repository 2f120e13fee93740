#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV per bench step.

A step starts at a k_ops1 dispatch (gw_tick) and runs until the next one, so
the collect (sync kernels) belongs to the step before it.  Reports, over the
last N steps: per-kernel average duration per step, calls per step, VGPRs,
LDS, scratch, and the step's GPU-busy vs wall span."""
import collections
import csv
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("gw::", "")


def main(path, last=5):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).split("<")[0] == "k_ops1"]
    if not starts:
        print("no ticks found")
        return
    steps = []
    for j, s in enumerate(starts):
        e = starts[j + 1] if j + 1 < len(starts) else len(rows)
        steps.append(rows[s:e])
    steps = steps[-last:]
    agg = collections.defaultdict(lambda: [0.0, 0, None])
    busy = wall = 0.0
    for st in steps:
        t0 = int(st[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in st)
        wall += (t1 - t0) / 1e3
        for r in st:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            busy += d
            a = agg[short(r["Kernel_Name"])]
            a[0] += d; a[1] += 1
            a[2] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
    n = len(steps)
    print(f"steps={n}  gpu-busy/step={busy/n:.1f} us  wall-span/step={wall/n:.1f} us")
    print(f"{'kernel':40s} {'us/step':>9s} {'calls':>6s} {'%':>6s}  vgpr/agpr/sgpr/lds/scratch")
    for k, (t, c, meta) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{k:40s} {t/n:9.1f} {c/n:6.1f} {100*t/busy:6.2f}  {'/'.join(meta)}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
