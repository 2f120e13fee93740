#!/usr/bin/env python3
"""Benchmark of the MI355X AOI + entity-sync hot path (BASELINE.json metric).

A step = one game tick of the hot path over one batch of synthetic input:
gw_tick (apply the tick's 100k Moved ops, update every neighbour list, emit the
canonical enter/leave streams) + gw_sync_collect (CollectEntitySyncInfos:
per-watcher position/yaw records).  Workload at N=1 is BASELINE config #3,
the 1M-entity clustered-hotspot single space the metric is quoted on.  With
--gpus N each rank owns an independent 1M-entity space on its own GPU (spaces
never span processes in the reference, SpaceManager.go:11-31): weak scaling,
no data-path collective.  Inputs (ops of every tick) are resident in HBM
before the timed region; outputs stay in HBM (device-resident boundary).

Run:  python bench.py [--gpus N --steps K --warmup W]
N>1:  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from goworld_amd import gpuaoi, traces  # noqa: E402

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak (MI355X_MICROARCH.md: 8.0 TB/s spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--entities", type=int, default=1_000_000)
    ap.add_argument("--side", type=float, default=32768.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--profile-stages", type=int, default=1, help="HIP-event stage timing in the timed region")
    return ap.parse_args()


def dist_setup(n_gpus):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=ws)   # control plane only (barrier, max)
        pg = dist
    return rank, local, ws, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allreduce(pg, vals, op):
    if pg is None:
        return vals
    import torch
    t = torch.tensor(vals, dtype=torch.float64)
    pg.all_reduce(t, op=op)
    return t.tolist()


STAGE_KERNEL = {"diff": "k_mover<2, 1>"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass
    (tools/gpu/pmc.sh: FETCH_SIZE*2 + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md); PMC counters cannot be read inside the timed run."""
    try:
        import json as _j
        d = _j.load(open(PMC_FILE))
        return d[kernel]["hbm_bytes"], os.path.relpath(PMC_FILE, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_baseline(tr, seconds):
    """Oracle XZList restatement (go-aoi algorithm + goworld glue), one thread,
    replaying tick 0's ops one by one until the time budget is spent."""
    from oracle import pyorc
    sp = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.XZLIST)
    t0 = time.perf_counter()
    pyorc.load_trace(sp, tr)
    build_s = time.perf_counter() - t0
    ops = tr.ticks[0]
    done, spent, chunk = 0, 0.0, 200
    while spent < seconds and done < len(ops):
        part = ops[done:done + chunk]
        t = time.perf_counter()
        rc = sp.tick(part)
        spent += time.perf_counter() - t
        assert rc == 0
        done += len(part)
    sp.close()
    return {"value": done / spent, "unit": "updates/s", "cores": 1, "kind": "port",
            "sample": f"{done} Moved ops of tick 0 of config #3 (1M entities), applied one by one through the "
                      f"XZList restatement incl. InterestedIn/By glue and raw->net event reduction, "
                      f"{spent:.1f}s timed; initial population bulk-built untimed ({build_s:.1f}s)",
            "per_op_us": spent / done * 1e6}


def main():
    a = parse()
    rank, local, ws, pg = dist_setup(a.gpus)
    ticks = a.warmup + a.steps
    tr = traces.config3(ticks=ticks, seed=3 + rank, n=a.entities, side=a.side)
    g = gpuaoi.GpuAOI(local)
    t_load = time.perf_counter()
    sid, base = gpuaoi.load_space(g, tr, chunk=1 << 18)
    g.sync_collect(copy=False)                      # clear the Enter flags (untimed)
    t_load = time.perf_counter() - t_load
    # all ticks' ops resident in HBM before timing
    m = len(tr.ticks[0])
    ops_all = np.concatenate(tr.ticks)
    dev_ops = g.dev_alloc(ops_all.nbytes)
    g.h2d(dev_ops, ops_all)
    nbytes_tick = m * traces.OP_DTYPE.itemsize

    stage_us, stage_bytes, stage_n = {}, {}, {}

    def acc_stages():
        for name, us, b in g.stage_times():
            stage_us[name] = stage_us.get(name, 0.0) + us
            stage_bytes[name] = stage_bytes.get(name, 0) + b
            stage_n[name] = stage_n.get(name, 0) + 1

    def step(t, prof):
        g.submit_device(dev_ops + t * nbytes_tick, m)
        r = g.tick(copy=False)
        s = g.sync_collect(copy=False)
        if prof:
            acc_stages()          # tick + collect stages; the collect already synced the stream
        return r, s

    for t in range(a.warmup):
        step(t, False)
    g.set_profiling(bool(a.profile_stages))
    tot = dict(ops=0, events=0, records=0, bytes_alg=0, pairs=0, a_old=0, a_new=0)
    barrier(pg)
    g.synchronize()
    t0 = time.perf_counter()
    for t in range(a.warmup, ticks):
        r, s = step(t, bool(a.profile_stages))
        tot["ops"] += r.movers
        tot["events"] += r.n_enter + r.n_leave
        tot["records"] += s.n_rec
        tot["bytes_alg"] += r.bytes_alg + s.bytes_alg
        tot["pairs"] += r.pairs_tested
        tot["a_old"] += r.nbr_old
        tot["a_new"] += r.nbr_new
    g.synchronize()
    t1 = time.perf_counter()
    barrier(pg)
    elapsed = t1 - t0
    if pg is not None:
        mx = allreduce(pg, [elapsed], pg.ReduceOp.MAX)[0]
        sums = allreduce(pg, [tot["ops"], tot["events"], tot["records"]], pg.ReduceOp.SUM)
    else:
        mx = elapsed
        sums = [tot["ops"], tot["events"], tot["records"]]
    if rank != 0:
        return
    K = a.steps
    line = {
        "metric": "entity AOI updates/sec + enter/leave events/sec, 1M-entity space, 1/2/4/8 GPU",
        "value": sums[0] / mx,
        "unit": "updates/s",
        "n_gpus": ws,
        "steps": K,
        "warmup": a.warmup,
        "ms_per_step": mx / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded SplitMix64 traces, SURVEY 8(d) config #3)",
        "config": {"workload": "config #3: single AOI space per GPU, 1M entities, 70% uniform + 30% in 64 "
                               "Gaussian hotspots (sigma 200), 10% movers per tick (+-4 / hotspot +-16), "
                               "AOI distance 100, world 32768^2; step = gw_tick + gw_sync_collect",
                   "entities_per_gpu": a.entities, "movers_per_tick": m, "aoi_dist": 100.0,
                   "world_side": a.side, "gates": 1, "parallelism": f"independent spaces x{ws} (no comm)"},
        "events_per_sec": sums[1] / mx,
        "records_per_sec": sums[2] / mx,
        "device_us_per_step": (sum(stage_us.values()) / K) if stage_us else None,
        "bytes_alg_per_step": tot["bytes_alg"] / K,
        "tick_hbm_frac": (tot["bytes_alg"] / K) / (mx / K) / (HBM_PEAK_GBS * 1e9),
        "load_s": t_load,
    }
    if stage_us:
        stages = {n: {"avg_us": stage_us[n] / stage_n[n], "bytes_alg": stage_bytes[n] / stage_n[n]}
                  for n in stage_us}
        # the dominant kernel: k_mover, alone in stage "diff" (16 B per candidate tested + 4 B per
        # own event), timed by HIP events on the library's stream
        dom = "diff"
        ach = stages[dom]["bytes_alg"] / (stages[dom]["avg_us"] * 1e-6) / 1e9
        traffic, src = pmc_traffic(STAGE_KERNEL[dom])
        line["roofline"] = {"bound": "hbm", "kernel": STAGE_KERNEL[dom], "achieved": ach, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                            "traffic_unit": "bytes/launch", "traffic_source": src,
                            "bytes_alg_per_launch": stages[dom]["bytes_alg"], "avg_us": stages[dom]["avg_us"]}
        line["stages"] = {n: {"avg_us": round(v["avg_us"], 2), "GBps_alg": round(
            v["bytes_alg"] / max(v["avg_us"], 1e-9) / 1e3, 1)} for n, v in stages.items()}
    else:
        line["roofline"] = None
    if not a.no_cpu_baseline and ws == 1:
        cb = cpu_baseline(traces.config3(ticks=1, seed=3, n=a.entities, side=a.side), a.cpu_seconds)
        line["cpu_baseline"] = cb
    print(json.dumps(line), flush=True)
    g.dev_free(dev_ops)
    g.close()


if __name__ == "__main__":
    main()
