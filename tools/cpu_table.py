#!/usr/bin/env python3
"""CPU baselines per BASELINE config, bounded samples.

Test/measurement infrastructure: runs the oracle (oracle/, the C restatement
of go-aoi's XZList + InterestedIn/By glue, and oracle/gridmt.c) on the host
cores, never the product path.  Per config:
  st  one thread, XZList restatement, ops applied one by one (the reference's
      single game goroutine), time-bounded: per-op cost, updates/s, raw events/s
  mt  oracle/gridmt.c (OpenMP uniform grid, batched tick + collect) on THREADS
      cores, full ticks: updates/s, events/s, records/s, ms per tick
Config #4 (10k spaces): st over a sample of spaces, mt = THREADS processes of
st over disjoint spaces.  Config #5 (16M world): st and mt on a 2M-entity
world of the same density (L = 46341), stated as such.
usage: python tools/cpu_table.py [--threads 16] [--budget 20] [--configs 1,2,3,4,5] > out.json
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from goworld_amd import traces as T   # noqa: E402
from oracle import pyorc              # noqa: E402


def st_run(tr, budget, tick=0, chunk=500):
    sp = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.XZLIST)
    t0 = time.perf_counter()
    pyorc.load_trace(sp, tr)
    build = time.perf_counter() - t0
    ops = tr.ticks[tick]
    done, spent, raw, net = 0, 0.0, 0, 0
    while done < len(ops) and spent < budget:
        part = ops[done:done + chunk]
        t = time.perf_counter()
        assert sp.tick(part) == 0
        spent += time.perf_counter() - t
        re_, rl_, _, _ = sp.raw_counts()
        e, l = sp.events()
        raw += re_ + rl_
        net += len(e) + len(l)
        done += len(part)
    sp.close()
    return dict(ops=done, seconds=spent, per_op_us=spent / max(done, 1) * 1e6, updates_per_sec=done / spent,
                raw_events_per_sec=raw / spent, net_events_per_sec=net / spent, full_tick=done == len(ops),
                build_s=build)


def mt_run(tr, threads, budget):
    m = pyorc.GridMT(tr.capacity, tr.d, tr.bounds, threads=threads)
    m.load(tr)
    m.collect()
    done = ev = rec = steps = 0
    spent = 0.0
    for ops in tr.ticks:
        t = time.perf_counter()
        assert m.tick(ops) == 0
        e, l = m.events()
        r = m.collect()
        spent += time.perf_counter() - t
        done += len(ops); ev += len(e) + len(l); rec += len(r); steps += 1
        if spent > budget:
            break
    m.close()
    return dict(threads=threads, ticks=steps, updates_per_sec=done / spent, events_per_sec=ev / spent,
                records_per_sec=rec / spent, ms_per_tick=spent / steps * 1e3)


def _c4_worker(args):
    spaces, budget = args
    ops = sec = raw = 0.0
    t_end = time.perf_counter() + budget
    n_sp = 0
    for s in spaces:
        r = st_run(T.config4_space(s, ticks=1), 1e9)
        ops += r["ops"]; sec += r["seconds"]; raw += r["raw_events_per_sec"] * r["seconds"]
        n_sp += 1
        if time.perf_counter() > t_end:
            break
    return ops, sec, raw, n_sp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--budget", type=float, default=20.0)
    ap.add_argument("--configs", default="1,2,3,4,5")
    a = ap.parse_args()
    cfgs = [int(x) for x in a.configs.split(",")]
    out = {"threads": a.threads, "budget_s": a.budget}
    try:
        out["cpu_model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        out["cpu_model"] = None
    out["nproc"] = os.cpu_count()
    out["GOMAXPROCS"] = "n/a (no Go toolchain; the C restatement of go-aoi runs instead)"
    if 1 in cfgs:
        tr = T.config1(ticks=3)
        out["config1"] = {"st": st_run(tr, a.budget), "mt": mt_run(tr, a.threads, a.budget)}
    if 2 in cfgs:
        tr = T.config2(ticks=4)
        out["config2"] = {"st": st_run(tr, a.budget), "mt": mt_run(tr, a.threads, a.budget)}
    if 3 in cfgs:
        tr = T.config3(ticks=4)
        out["config3"] = {"st": st_run(tr, a.budget), "mt": mt_run(tr, a.threads, a.budget)}
    if 4 in cfgs:
        st = _c4_worker((range(0, 10_000, 50), a.budget))
        per = [list(range(k, 10_000, a.threads)) for k in range(a.threads)]
        t0 = time.perf_counter()
        with mp.Pool(a.threads) as pool:
            rs = pool.map(_c4_worker, [(p, a.budget) for p in per])
        wall = time.perf_counter() - t0
        ops = sum(r[0] for r in rs)
        out["config4"] = {"st": {"spaces": st[3], "ops": st[0], "per_op_us": st[1] / st[0] * 1e6,
                                 "updates_per_sec": st[0] / st[1], "raw_events_per_sec": st[2] / st[1],
                                 "tick_s_extrapolated": 1e6 * st[1] / st[0]},
                          "mt": {"processes": a.threads, "spaces": sum(r[3] for r in rs), "ops": ops,
                                 "updates_per_sec": ops / max(r[1] for r in rs),
                                 "what": "THREADS processes, each the single-thread restatement over its own spaces "
                                         "(1 tick each); rate = ops / the slowest process's apply time"}}
    if 5 in cfgs:
        n, side = 2_000_000, 46341.0       # config #5 density (16M / 131072^2)
        tr = T.dyadic_walk_trace(5, n, side, 100.0, 3, 0.10, 512)
        out["config5"] = {"what": f"{n} entities at config #5 density (L = {side:g}); per-op cost grows "
                                  f"with N/L for XZList", "st": st_run(tr, a.budget),
                          "mt": mt_run(tr, a.threads, a.budget)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
