#!/usr/bin/env python3
"""GPU idle gaps of a bench step from a rocprofv3 --runtime-trace --kernel-trace run.

A step starts at a k_ops1 dispatch.  For the last N steps: the GPU-busy time,
the wall span, and every idle gap > 2 us between consecutive kernels (copies
included) with the kernels on either side and the HIP API calls the host made
while the GPU idled (what the host was doing on the critical path).

usage: python tools/rt_gaps.py <rocprofv3 output dir> [N]"""
import csv
import glob
import os
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("gw::", "")


def load(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main(d, last=5):
    ks = load(d, "*kernel_trace.csv")
    api = load(d, "*hip_api_trace.csv")
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(ks) if short(r["Kernel_Name"]).split("<")[0] == "k_ops1"]
    steps = [(starts[j], starts[j + 1] if j + 1 < len(starts) else len(ks)) for j in range(len(starts))][-last - 1:-1]
    tot_idle = tot_span = 0.0
    for s, e in steps:
        rows = ks[s:e + 1] if e < len(ks) else ks[s:e]
        t0 = int(rows[0]["Start_Timestamp"])
        t1 = int(rows[-1]["Start_Timestamp"])          # up to the next step's first kernel
        busy = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[:-1])
        gaps = []
        for a, b in zip(rows, rows[1:]):
            g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
            if g > 2.0:
                lo, hi = int(a["End_Timestamp"]), int(b["Start_Timestamp"])
                calls = [(r["Function"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                         for r in api if int(r["Start_Timestamp"]) < hi and int(r["End_Timestamp"]) > lo]
                gaps.append((g, short(a["Kernel_Name"]), short(b["Kernel_Name"]), calls))
        span = (t1 - t0) / 1e3
        tot_idle += span - busy
        tot_span += span
        print(f"step: span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us")
        for g, a, b, calls in sorted(gaps, reverse=True)[:8]:
            agg = {}
            for f, dur in calls:
                v = agg.setdefault(f, [0, 0.0])
                v[0] += 1
                v[1] += dur
            top = ", ".join(f"{f} x{n} ({t:.0f} us)" for f, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:5])
            print(f"  gap {g:6.1f} us  {a} -> {b}   host: {top}")
        if gaps and "--seq" in sys.argv:                 # the host calls inside the largest gap, in order
            g, a, b, _ = max(gaps)
            i = next(k for k, (x, y) in enumerate(zip(rows, rows[1:]))
                     if short(x["Kernel_Name"]) == a and short(y["Kernel_Name"]) == b)
            lo, hi = int(rows[i]["End_Timestamp"]), int(rows[i + 1]["Start_Timestamp"])
            for r in api:
                st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                if en > lo and st < hi:
                    print(f"      {(st - lo) / 1e3:8.1f} .. {(en - lo) / 1e3:8.1f} us  {r['Function']}")
    if steps:
        print(f"mean: span {tot_span / len(steps):.1f} us, idle {tot_idle / len(steps):.1f} us")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0], int(args[1]) if len(args) > 1 else 5)
