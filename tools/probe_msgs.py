#!/usr/bin/env python3
"""Host wall time of the SURVEY 8(f) client paths at config #3, call by call:
gw_client_events and gw_fanout repeated on the same tick (steady state: no
buffer growth), and the per-client collect (GW_SYNC_BY_CLIENT) against the
plain one on the following ticks.  Run under `rocprofv3 --runtime-trace
--kernel-trace` to see the HIP API calls inside each.

usage: python tools/probe_msgs.py [--entities 1000000] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from goworld_amd import gpuaoi, traces  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entities", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    tr = traces.config3(ticks=6, seed=3, n=a.entities)
    g = gpuaoi.GpuAOI(0)
    gpuaoi.load_space(g, tr, chunk=1 << 18)
    g.sync_collect(copy=False)
    out = {"entities": a.entities}
    for t in range(2):
        g.submit(tr.ticks[t])
        g.tick(copy=False)
        g.sync_collect(copy=False)
    g.synchronize()
    calls = np.ascontiguousarray(tr.ticks[1]["slot"], np.uint32)
    ev, fo = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        cr, de = g.client_events(copy=False)
        t1 = time.perf_counter()
        f = g.fanout(calls, copy=False)
        t2 = time.perf_counter()
        ev.append((t1 - t0) * 1e6)
        fo.append((t2 - t1) * 1e6)
    out["client_events_us"] = [round(v, 1) for v in ev]
    out["client_events_device_us"] = round(cr.device_us, 1)
    out["fanout_us"] = [round(v, 1) for v in fo]
    out["fanout_device_us"] = round(f.device_us, 1)
    out["creates"], out["destroys"], out["deliveries"] = cr.n_rec, de.n_rec, f.n_rec
    plain, bycl = [], []
    for t in range(2, 6):
        g.submit(tr.ticks[t])
        g.tick(copy=False)
        g.synchronize()
        t0 = time.perf_counter()
        s = g.sync_collect(copy=False, by_client=(t % 2 == 1))
        g.synchronize()
        (bycl if t % 2 == 1 else plain).append((time.perf_counter() - t0) * 1e6)
    out["collect_plain_us"] = [round(v, 1) for v in plain]
    out["collect_by_client_us"] = [round(v, 1) for v in bycl]
    out["records"] = s.n_rec
    print(json.dumps(out), flush=True)
    g.close()


if __name__ == "__main__":
    main()
