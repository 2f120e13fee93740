#!/usr/bin/env python3
"""Per-rank cost of a decomposed world at R ranks, measured on ONE GPU.

The driver runs the real N-GPU bench (one process per GPU, halo rows over RCCL
inside the library).  This tool rehearses it on a single MI355X: R world
contexts (gw_world_create, one X-strip each) live in one process on the same
device, the halo rows move between them by pointer (rank r+1's send buffer is
rank r's receive buffer: gw_world_route -> gw_world_submit, no copy), and every
rank's step is run ALONE on the GPU and timed with a device sync on both
sides:

    step_r = gw_world_route (4 routing kernels + its host sync)
           + gw_tick + gw_sync_collect (one host sync)

so step_r is what rank r costs on its own GPU, minus the RCCL transfer (two
grouped send/recv rounds with <= 2 peers; its bytes are reported).  Ranks
meet at every exchange, so the projected N-GPU step is the mean over steps of
max_r step_r (+ the exchange); projected throughput = all ranks' updates /
that.  The same world at R = 1 gives the baseline of the
projected speedup.  Workloads: config #5 (16M uniform world, L = 131072) and
the metric's 1M clustered space (config #3 as one world).

usage: python tools/sim_ranks.py [--which c5|c3] [--ranks 1,2,4,8] [--warmup 20] [--steps 10]
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

from goworld_amd import dworld, gpuaoi, traces  # noqa: E402


def world_ticks(which, ticks, n):
    """(n, side, max_step, x0, z0, yaw0, [(ops, x_before)] per tick)."""
    if which == "c5":
        side, max_step = 131072.0, 4.0
        walk = traces.WorldWalk(seed=5, n=n, side=side)
        x0, z0, yaw0 = walk.x(), walk.z(), walk.yaw.copy()
        tk = [walk.next_tick() for _ in range(ticks)]
    else:
        side, max_step = 32768.0, 16.0
        tr = traces.config3(ticks=ticks, seed=3, n=n, side=side)
        x0, z0, yaw0 = tr.init_x, tr.init_z, tr.init_yaw
        xcur = tr.init_x.copy()
        tk = []
        for ops in tr.ticks:
            xb = xcur[ops["slot"]].copy()
            xcur[ops["slot"]] = ops["x"]
            tk.append((ops, xb))
    return side, max_step, x0, z0, yaw0, tk


class SimWorld(dworld.LocalWorld):
    """dworld.LocalWorld with per-rank step timing."""

    def __init__(self, R, n, side, max_step, x0, z0, yaw0, tk, device=0):
        super().__init__(R, n, side, max_step, x0, z0, yaw0, device=device)
        self.ticks = []                           # per tick: [(dev_ptr, m)] per rank, resident in HBM
        for ops, xb in tk:
            self.ticks.append([(self.upload(r, o), len(o)) for r, o in enumerate(self.split(ops, xb))])

    def step(self, t, phases=None):
        """One tick of every rank; returns (per-rank seconds, updates, events, records, halo rows).
        phases: dict accumulating host seconds per phase (route / tick call / collect call) over ranks."""
        times = [0.0] * self.R
        ptrs = [p for p, _ in self.ticks[t]]
        ms = [m for _, m in self.ticks[t]]
        rows = self.route_submit(ptrs, ms, times)
        if phases is not None:
            phases["route"] += sum(times)
            for r in range(self.R):
                phases["per_rank"][r][0] += times[r]
        upd = ev = rec = 0
        for r, g in enumerate(self.g):
            g.synchronize()
            t0 = time.perf_counter()
            g.tick(copy=False, defer=True)
            t1 = time.perf_counter()
            s = g.sync_collect(copy=False)
            t2 = time.perf_counter()
            times[r] += t2 - t0
            if phases is not None:
                phases["tick_call"] += t1 - t0
                phases["collect_call"] += t2 - t1
                phases["per_rank"][r][1] += t1 - t0
                phases["per_rank"][r][2] += t2 - t1
            res = g.tick_result()
            upd += ms[r]
            ev += res.n_enter + res.n_leave
            rec += s.n_rec
        return times, upd, ev, rec, rows

    def close(self):
        self.check()
        super().close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", choices=["c5", "c3"], default="c5")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--entities", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = a.entities or (16_000_000 if a.which == "c5" else 1_000_000)
    ticks = a.warmup + a.steps
    t0 = time.perf_counter()
    side, max_step, x0, z0, yaw0, tk = world_ticks(a.which, ticks, n)
    print(f"# {a.which}: {n} entities, {ticks} ticks generated in {time.perf_counter() - t0:.1f}s", flush=True)
    out = []
    base = None
    for R in [int(v) for v in a.ranks.split(",")]:
        t0 = time.perf_counter()
        w = SimWorld(R, n, side, max_step, x0, z0, yaw0, tk)
        load = time.perf_counter() - t0
        stages = None
        for t in range(a.warmup):
            if t == a.warmup - 3:                  # the last 3 warm-up steps: device time per stage of rank 0
                w.g[0].set_profiling(1)
            w.step(t)
        if a.warmup >= 3:
            acc = {}
            for name, us, _, calls in w.g[0].stage_times():
                v = acc.setdefault(name, [0.0, 0])
                v[0] += us
                v[1] += calls
            w.g[0].set_profiling(0)
            stages = {k: round(v[0] / 3, 1) for k, v in acc.items()}
        per = np.zeros(R)
        smax = 0.0
        upd = ev = rec = rows = 0
        phases = {"route": 0.0, "tick_call": 0.0, "collect_call": 0.0, "per_rank": [[0.0, 0.0, 0.0] for _ in range(R)]}
        for t in range(a.warmup, ticks):
            ts, u, e, rc, rw = w.step(t, phases)
            per += np.array(ts)
            smax += max(ts)                        # ranks meet at every exchange: a step costs its slowest rank
            upd += u; ev += e; rec += rc; rows += rw
        w.close()
        per_ms = per / a.steps * 1e3
        step_ms = smax / a.steps * 1e3
        row_bytes = rows / a.steps * 32            # gw_halo_row = 32 B
        line = {"which": a.which, "ranks": R, "entities": n, "steps": a.steps,
                "rank_ms": [round(v, 4) for v in per_ms.tolist()], "step_ms": step_ms,
                "max_rank_ms": float(per_ms.max()), "mean_rank_ms": float(per_ms.mean()),
                "updates_per_step": upd / a.steps, "events_per_step": ev / a.steps,
                "records_per_step": rec / a.steps, "halo_bytes_per_step_all_ranks": row_bytes,
                "projected_updates_per_sec_excl_exchange": upd / a.steps / (step_ms * 1e-3),
                "projected_events_per_sec_excl_exchange": ev / a.steps / (step_ms * 1e-3),
                "load_s": round(load, 1),
                "host_us_per_rank_step": {k: round(v / a.steps / R * 1e6, 1) for k, v in phases.items()
                                          if k != "per_rank"},
                "route_tick_collect_us_by_rank": [[round(v / a.steps * 1e6, 1) for v in pr]
                                                  for pr in phases["per_rank"]]}
        if stages:
            line["rank0_device_us_per_stage"] = stages
        if base is None and R == 1:
            base = line
        if base is not None:
            line["projected_speedup_vs_1_excl_exchange"] = base["step_ms"] / step_ms
        print(json.dumps(line), flush=True)
        out.append(line)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
