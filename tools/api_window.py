#!/usr/bin/env python3
"""Merged host/device timeline of the last client-path repetition in a
rocprofv3 --runtime-trace --kernel-trace run of tools/probe_msgs.py: HIP API
calls (host) and kernels (device) between the last gw_client_events' first
kernel (minus a margin for its host prologue) and the last fan-out kernel,
each with its start offset and duration in us.

usage: python tools/api_window.py <rocprofv3 output dir>"""
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


def main(d):
    ks = load(d, "*kernel_trace.csv")
    api = load(d, "*hip_api_trace.csv")
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [r for r in ks if short(r["Kernel_Name"]).startswith("k_event_client_compact")]
    fo = [r for r in ks if short(r["Kernel_Name"]).startswith("k_fanout_final")]
    if len(ev) < 2 or not fo:
        print("no client-path kernels in the trace")
        return
    t0 = int(ev[-2]["Start_Timestamp"]) - 300_000
    t1 = int(fo[-1]["End_Timestamp"]) + 100_000
    rows = []
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s <= t1:
            rows.append((s, e, "host", r["Function"]))
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s <= t1:
            rows.append((s, e, "gpu ", short(r["Kernel_Name"])))
    rows.sort()
    base = rows[0][0] if rows else t0
    for s, e, who, name in rows:
        print(f"{(s - base) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {who}  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
