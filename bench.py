#!/usr/bin/env python3
"""Benchmark of the MI355X AOI + entity-sync hot path (BASELINE.json metric).

A step = one game tick of the hot path over one batch of synthetic input:
gw_tick (apply the tick's 100k Moved ops, update every neighbour list, emit the
canonical enter/leave streams) + gw_sync_collect (CollectEntitySyncInfos:
per-watcher position/yaw records).  Workload at N=1 is BASELINE config #3,
the 1M-entity clustered-hotspot single space the metric is quoted on.

N>1, --mode world (default): one world space decomposed into N X-strips, one
per GPU (BASELINE config #5, goworld_amd/dworld.py): each strip has config
#3's statistics (1M entities per strip by default, --entities 2000000 gives
config #5's 16M at N=8), and each tick every rank routes its ops, exchanges
its halo rows with both neighbours over RCCL (xGMI) and ticks its strip.
Weak scaling.  Bench strips reflect their walkers at the strip borders
(migration is covered by the parity tests, tests/test_dworld.py); the halo
traffic of the border bands is real.
N>1, --mode spaces: an independent 1M-entity space per GPU (spaces never span
processes in the reference, SpaceManager.go:11-31): no data-path collective.

Inputs (ops of every tick) are resident in HBM before the timed region;
outputs stay in HBM (device-resident boundary).

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
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="multi-threaded CPU baseline time budget")
    ap.add_argument("--cpu-st-max-seconds", type=float, default=240.0,
                    help="guard on the single-thread baseline (it replays one full tick)")
    ap.add_argument("--e2e-steps", type=int, default=3, help="untimed end-to-end steps (host in/out)")
    ap.add_argument("--profile-stages", type=int, default=1,
                    help="1: HIP events around the dominant kernel's stage in the timed region (roofline) and "
                         "a per-stage breakdown over extra untimed steps; 0: none")
    ap.add_argument("--mode", choices=["world", "spaces"], default="world", help="N>1 regime")
    ap.add_argument("--config", type=int, choices=[3, 4, 5], default=3,
                    help="3: config #3 per GPU (weak); 4: config #4, 10k independent 1k-entity spaces, space s on "
                         "GPU s mod N (strong); 5: the 16M uniform world of config #5 over N strips (strong)")
    ap.add_argument("--spaces", type=int, default=10_000, help="config #4: number of spaces")
    ap.add_argument("--comm", choices=["nccl", "gloo"], default="nccl",
                    help="halo exchange backend (gloo: rehearsal of several ranks on one GPU)")
    ap.add_argument("--halo-cap", type=int, default=4096, help="halo entities per neighbour per tick")
    ap.add_argument("--halo-cap-load", type=int, default=16384, help="the same, for the ticks that load the world")
    ap.add_argument("--device", type=int, default=None, help="force a device (rehearsals on one GPU)")
    ap.add_argument("--sync-by-client", action="store_true",
                    help="collect grouped per client (GW_SYNC_BY_CLIENT, the gate's regroup on the GPU)")
    ap.add_argument("--client-msgs", type=int, default=5,
                    help="extra untimed ticks measuring gw_client_events + gw_fanout (N=1 config #3; 0 = off)")
    ap.add_argument("--capacity", type=int, default=None,
                    help="slot capacity of the space (N=1: cost of a strip's id range at N ranks)")
    return ap.parse_args()


class Ctl:
    """Control plane (barrier, max/sum of scalars) on a gloo group; the data
    path (halo rows) uses the default group (RCCL) in world mode."""

    def __init__(self, a):
        self.ws = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0")) if a.device is None else a.device
        self.group = None
        if self.ws > 1:
            import torch
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if a.mode == "world" and a.comm == "nccl":
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl", rank=self.rank, world_size=self.ws,
                                        device_id=torch.device("cuda", self.local))
                self.group = dist.new_group(backend="gloo")
                t = torch.ones(1, device=torch.device("cuda", self.local))
                dist.all_reduce(t)            # bring up the RCCL communicator on all ranks
                torch.cuda.synchronize()
            else:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.ws)
                self.group = dist.group.WORLD
            self.dist = dist

    def barrier(self):
        if self.group is not None:
            self.dist.barrier(group=self.group)

    def reduce(self, vals, op):
        if self.group is None:
            return vals
        import torch
        t = torch.tensor(vals, dtype=torch.float64)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op), group=self.group)
        return t.tolist()


STAGE_KERNEL = {"diff": "k_mover<2, 1>"}
PMC_DIR = os.path.join(ROOT, "profiles")


def src_hash():
    """Hash of the kernel sources (the PMC pass must come from this HEAD)."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, "goworld_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".hpp", ".cpp")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def pmc_traffic(config):
    """HBM bytes per launch per kernel from the committed rocprofv3 PMC pass of
    this config (tools/gpu/pmc.sh: FETCH_SIZE*2 + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md), only if it was taken on these kernel
    sources (src_hash); PMC counters cannot be read inside the timed run."""
    path = os.path.join(PMC_DIR, f"pmc_config{config}.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None, "missing"
    if d.get("src_hash") != src_hash():
        return None, os.path.relpath(path, ROOT), "stale (taken on other kernel sources)"
    return d.get("kernels", {}), os.path.relpath(path, ROOT), d.get("src_hash")


def cpu_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "cpus_allowed": allowed,
            "GOMAXPROCS": "n/a (no Go toolchain: the go-aoi algorithm runs as its C restatement)"}


def cpu_baseline(tr, max_seconds):
    """Oracle XZList restatement (go-aoi v0.2.0 algorithm + goworld glue:
    InterestedIn/By sets, create/destroy message counts), ONE thread, replaying
    all of tick 0's ops one by one (the reference's single game goroutine,
    GameService.go:77-190); max_seconds only guards against a pathological host."""
    from oracle import pyorc
    sp = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.XZLIST)
    t0 = time.perf_counter()
    pyorc.load_trace(sp, tr)
    build_s = time.perf_counter() - t0
    ops = tr.ticks[0]
    done, spent, chunk = 0, 0.0, 1000
    raw_e = raw_l = net = 0
    while done < len(ops) and spent < max_seconds:
        part = ops[done:done + chunk]
        t = time.perf_counter()
        rc = sp.tick(part)
        spent += time.perf_counter() - t
        assert rc == 0
        re_, rl_, _, _ = sp.raw_counts()
        e, l = sp.events()
        raw_e += re_; raw_l += rl_; net += len(e) + len(l)
        done += len(part)
    sp.close()
    full = done == len(ops)
    return {"value": done / spent, "unit": "updates/s", "cores": 1, "kind": "port",
            "sample": (f"{'all' if full else 'first'} {done} Moved ops of tick 0 of config #3 (1M entities; "
                       f"{'one full tick' if full else 'time guard hit'}), applied one by one through the C "
                       f"restatement of go-aoi's XZList incl. InterestedIn/By glue, {spent:.1f}s on one core; "
                       f"initial population bulk-built untimed ({build_s:.1f}s)"),
            "per_op_us": spent / done * 1e6, "full_tick": full,
            "raw_events_per_sec": (raw_e + raw_l) / spent, "net_events_per_sec": net / spent,
            **cpu_info()}


def cpu_baseline_mt(seconds, entities, side):
    """Fairness point: oracle/gridmt.c, a multi-threaded (OpenMP)
    uniform-grid CPU implementation of the same batched tick + collect, on the
    host cores this job may use (OMP_NUM_THREADS; 16 per GPU on the box), over
    config #3 ticks until the time budget is spent."""
    from oracle import pyorc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = min(threads, 16)
    tr = traces.config3(ticks=8, seed=3, n=entities, side=side)
    m = pyorc.GridMT(tr.capacity, tr.d, tr.bounds, threads=threads)
    m.load(tr)
    m.collect()                                       # the Enter flags (untimed)
    done = ev = rec = 0
    spent = 0.0
    for ops in tr.ticks:
        t = time.perf_counter()
        assert m.tick(ops) == 0
        e, l = m.events()
        r = m.collect()
        spent += time.perf_counter() - t
        done += len(ops)
        ev += len(e) + len(l)
        rec += len(r)
        if spent > seconds:
            break
    m.close()
    steps = done // len(tr.ticks[0])
    return {"value": done / spent, "unit": "updates/s", "cores": threads, "kind": "port",
            "events_per_sec": ev / spent, "records_per_sec": rec / spent, "ms_per_step": spent / steps * 1e3,
            "sample": f"{steps} full ticks of config #3 (tick + collect, canonical events and records) through "
                      f"oracle/gridmt.c: OpenMP uniform grid, {threads} threads, the batched contract "
                      f"(checked bit-exact against the oracle in tests/test_oracle.py)"}


class SpaceRun:
    """N=1 (config #3) and --mode spaces: one independent space per GPU."""

    def __init__(self, a, ctl, ticks):
        self.tr = traces.config3(ticks=ticks, seed=3 + ctl.rank, n=a.entities, side=a.side)
        if a.capacity:
            self.tr.capacity = max(a.capacity, a.entities)
            self.tr.gates = np.concatenate([self.tr.gates, np.zeros(self.tr.capacity - a.entities, np.uint16)])
        self.g = g = gpuaoi.GpuAOI(ctl.local)
        gpuaoi.load_space(g, self.tr, chunk=1 << 18)
        g.sync_collect(copy=False)                      # clear the Enter flags (untimed)
        # all ticks' ops resident in HBM before timing
        self.m = len(self.tr.ticks[0])
        self.host_ticks = self.tr.ticks
        ops_all = np.concatenate(self.tr.ticks)
        self.dev_ops = g.dev_alloc(ops_all.nbytes)
        g.h2d(self.dev_ops, ops_all)
        self.nbytes_tick = self.m * traces.OP_DTYPE.itemsize
        self.by_client = a.sync_by_client
        self.parallelism = f"independent spaces x{ctl.ws} (no comm)" if ctl.ws > 1 else "single GPU"
        self.n_world = a.entities * (ctl.ws if ctl.ws > 1 else 1)

    def step(self, t):
        g = self.g
        g.submit_device(self.dev_ops + t * self.nbytes_tick, self.m)
        g.tick(copy=False, defer=True)       # no host sync: the collect's sync settles it
        s = g.sync_collect(copy=False, by_client=self.by_client)
        r = g.tick_result()
        return r.movers, r, s

    def step_e2e(self, t):
        """The Go caller's game tick: host ops in (gw_submit: pageable host
        memory, copied to the device), the canonical events and the sync
        records out to pinned host buffers (GW_TICK_COPY_TO_HOST /
        GW_SYNC_COPY_TO_HOST), i.e. PCIe both ways."""
        g = self.g
        g.submit(self.host_ticks[t])
        r = g.tick(copy=True)
        s = g.sync_collect(copy=True, by_client=self.by_client)
        return r.movers, r, s

    def close(self):
        self.g.dev_free(self.dev_ops)
        self.g.close()


class ManySpacesRun(SpaceRun):
    """--config 4 (BASELINE config #4): `spaces` independent spaces of 1k entities (L = 1024, d = 100,
    K ~ 38), space s on GPU s mod N (SpaceManager.go:11-31: a space never spans processes), no
    collective; every space of a GPU is ticked and collected by the same launches.  The population
    and the walk (10% movers per space per tick, +-4 on the 1/128 grid, reflected) are drawn per
    rank with the seeded generators of goworld_amd/traces.py, vectorised over spaces."""

    def __init__(self, a, ctl, ticks):
        T = traces
        mine = np.arange(ctl.rank, a.spaces, ctl.ws)
        S, per, L, Q = len(mine), 1000, 1024.0, int(T.Q)
        seed = 4_000_000 + ctl.rank
        self.g = g = gpuaoi.GpuAOI(ctl.local)
        bases = np.zeros(S, np.int64)
        sids = []
        for i in range(S):
            sid, bases[i] = g.create_space(100.0, per, bounds=(-L / 2, -L / 2, L / 2, L / 2))
            sids.append(sid)
        n = S * per
        lo, hi = -int(L / 2 * Q), int(L / 2 * Q)
        kx = T.rand_int(T.stream_key(seed, 1), n, lo, hi)
        kz = T.rand_int(T.stream_key(seed, 2), n, lo, hi)
        yaw = (T.rand_f32(T.stream_key(seed, 3), n) * np.float32(2 * np.pi)).astype(np.float32)
        slots = (bases[:, None] + np.arange(per)[None, :]).reshape(-1).astype(np.uint32)
        for i in range(S):
            sl = slice(i * per, (i + 1) * per)
            g.restore(sids[i], slots[sl], kx[sl] / Q, np.zeros(per, np.float32), kz[sl] / Q, yaw[sl])
        g.set_clients(slots, np.ones(n, np.uint16))          # every entity has a client, 1 gate
        g.sync_collect(copy=False)                            # clear the Enter flags (untimed)
        m = per // 10
        coprime = np.array([1, 3, 7, 9, 11, 13, 17, 19, 21, 23], np.int64)
        ops_all = []
        for t in range(ticks):
            o = T.rand_int(T.stream_key(seed, 100, t), S, 0, per)
            p = coprime[T.rand_int(T.stream_key(seed, 101, t), S, 0, len(coprime))]
            local = (o[:, None] + np.arange(m)[None, :] * p[:, None]) % per     # distinct within a space
            idx = (np.arange(S)[:, None] * per + local).reshape(-1)
            q = (T.rand_unit(T.stream_key(seed, 102, t), 2 * len(idx)) * 1025).astype(np.int64) - 512
            kx[idx] = T._reflect_q(kx[idx] + q[:len(idx)], lo, hi)
            kz[idx] = T._reflect_q(kz[idx] + q[len(idx):], lo, hi)
            ops = T.make_ops(len(idx))
            ops["kind"] = T.OP_MOVED
            ops["sync_flags"] = T.SIF_NEIGHBOR | T.SIF_OWN
            ops["slot"] = slots[idx]
            ops["x"] = (kx[idx] / Q).astype(np.float32)
            ops["z"] = (kz[idx] / Q).astype(np.float32)
            ops["yaw"] = yaw[idx]
            ops_all.append(ops)
        self.m = len(ops_all[0])
        self.host_ticks = ops_all
        ops_all = np.concatenate(ops_all)
        self.dev_ops = g.dev_alloc(ops_all.nbytes)
        g.h2d(self.dev_ops, ops_all)
        self.nbytes_tick = self.m * T.OP_DTYPE.itemsize
        self.by_client = a.sync_by_client
        self.parallelism = f"{a.spaces} independent spaces, s -> GPU s mod {ctl.ws} ({S} on this GPU, no comm)"
        self.n_world = a.spaces * per
        self.tr = None


class WorldRun:
    """--mode world, N>1 (or --config 5): one world of N strips (dworld.StripRank per rank)."""

    def __init__(self, a, ctl, ticks):
        import torch
        from goworld_amd import dworld
        self.torch = torch
        dev = torch.device("cuda", ctl.local)
        torch.cuda.set_device(dev)
        ws, r = ctl.ws, ctl.rank
        if a.config == 5:
            # config #5: 16M uniform, L = 131072, strips of L / N, step +-4
            tr = traces.config5_strip(r, ws, ticks=ticks)
            n, side, side_z, max_step = tr.n, 131072.0 / ws, 131072.0, 4.0
        else:
            n, side = a.entities, a.side
            tr = traces.config3(ticks=ticks, seed=3 + r, n=n, side=side)
            side_z, max_step = side, 16.0                       # config #3 steps: +-4, hotspots +-16
        x0 = -ws * side / 2
        geom = dworld.Strips(x0, side, ws, tr.d, max_step)
        off = np.float32(x0 + (r + 0.5) * side)                 # strip r's centre (exact in f32)
        lo, hi = geom.ext(r)
        bounds = (max(lo, x0), -side_z / 2, min(hi, x0 + ws * side), side_z / 2)
        self.n_world = n * ws
        self.g = gpuaoi.GpuAOI(ctl.local)
        eng = dworld.HipStrip(self.g)
        pg = None if a.comm == "nccl" else ctl.group
        cdev = dev if a.comm == "nccl" else torch.device("cpu")
        self.sr = sr = dworld.StripRank(eng, geom, r, n * ws, bounds, dev, pg=pg, comm_device=cdev,
                                        halo_cap=a.halo_cap, halo_cap_max=a.halo_cap_load)
        eng.set_clients(np.arange(n * ws, dtype=np.uint32), np.ones(n * ws, np.uint16))  # config #3: 1 gate, all clients

        def words(ops):
            o = ops.copy()
            o["slot"] += np.uint32(r * n)
            o["x"] += off
            return torch.from_numpy(dworld.ops_to_words(o).copy()).to(dev)
        enter = traces.enter_ops(tr.init_slots, tr.init_x, tr.init_y, tr.init_z, tr.init_yaw)
        for i in range(0, n, 1 << 18):
            sr.step(words(enter[i:i + (1 << 18)]), copy=False, cap=a.halo_cap_load, no_events=True)
        sr.collect(copy=False)
        self.m = len(tr.ticks[0])
        self.words = [words(t) for t in tr.ticks]              # resident in HBM
        torch.cuda.synchronize()
        self.parallelism = (f"decomposed world, {ws} X-strips, halo rows over {a.comm.upper()}" if ws > 1
                            else "single GPU, one-strip world")
        self.tr = tr

    def step(self, t):
        self.sr.step(self.words[t], copy=False, defer=True)
        s = self.sr.collect(copy=False)
        return self.m, self.sr.e.tick_result(), s

    def close(self):
        self.sr.check()
        self.g.close()


def client_msgs(run, t0, n):
    """SURVEY 8(f) ranks 2-3, outside the headline step: after each of n more
    ticks, gw_client_events (create/destroy messages of the tick's events) and
    gw_fanout of one AllClients call per mover (e.g. an attribute change),
    outputs left on the device; wall time per call (each ends in a host sync)."""
    g = run.g
    t_ev = t_fo = 0.0
    n_cr = n_de = n_fo = n_calls = b_ev = b_fo = 0
    for t in range(t0, t0 + n):
        run.step(t)
        calls = run.tr.ticks[t]["slot"]
        g.synchronize()
        c0 = time.perf_counter()
        cr, de = g.client_events(copy=False)
        c1 = time.perf_counter()
        fo = g.fanout(calls, copy=False)
        c2 = time.perf_counter()
        t_ev += c1 - c0
        t_fo += c2 - c1
        n_cr += cr.n_rec; n_de += de.n_rec; n_fo += fo.n_rec; n_calls += len(calls)
        b_ev += cr.bytes_alg + de.bytes_alg; b_fo += fo.bytes_alg
    return {"ticks": n,
            "client_events": {"avg_us": t_ev / n * 1e6, "creates_per_tick": n_cr / n, "destroys_per_tick": n_de / n,
                              "msgs_per_sec": (n_cr + n_de) / t_ev, "GBps_alg": b_ev / t_ev / 1e9},
            "fanout": {"avg_us": t_fo / n * 1e6, "calls_per_tick": n_calls / n, "deliveries_per_tick": n_fo / n,
                       "deliveries_per_sec": n_fo / t_fo, "GBps_alg": b_fo / t_fo / 1e9},
            "timing": "host wall clock around each call (one host sync inside each); not part of ms_per_step"}


def main():
    a = parse()
    ctl = Ctl(a)
    ws, rank = ctl.ws, ctl.rank
    extra = 5 if a.profile_stages else 0         # untimed steps for the per-stage breakdown
    cm = a.client_msgs if (ws == 1 and a.config == 3) else 0
    world = (ws > 1 and a.mode == "world") or a.config == 5
    n_e2e = 0 if world else a.e2e_steps
    ticks = a.warmup + a.steps + extra + cm + n_e2e
    t_load = time.perf_counter()
    if a.config == 4:
        run = ManySpacesRun(a, ctl, ticks)
    else:
        run = WorldRun(a, ctl, ticks) if world else SpaceRun(a, ctl, ticks)
    t_load = time.perf_counter() - t_load
    g = run.g

    stage_us, stage_bytes, stage_n = {}, {}, {}

    def acc_stages():
        for name, us, b, calls in g.stage_times():
            stage_us[name] = stage_us.get(name, 0.0) + us
            stage_bytes[name] = stage_bytes.get(name, 0) + b
            stage_n[name] = stage_n.get(name, 0) + calls

    for t in range(a.warmup):
        run.step(t)
    g.set_profiling(2 if a.profile_stages else 0)    # the dominant kernel's stage only
    tot = dict(ops=0, events=0, records=0, bytes_alg=0, mover_alg=0, a_nbr=0, cand=0, own_copy_alg=0,
               sync_write_alg=0)
    ctl.barrier()
    g.synchronize()
    t0 = time.perf_counter()
    for t in range(a.warmup, a.warmup + a.steps):
        upd, r, s = run.step(t)
        tot["ops"] += upd
        tot["events"] += r.n_enter + r.n_leave
        tot["records"] += s.n_rec
        tot["bytes_alg"] += r.bytes_alg + s.bytes_alg
        ev = r.n_enter + r.n_leave
        # SURVEY 8(d) terms per kernel: k_mover produces the neighbour-list
        # terms and the net events, 4*(A_old+A_new) + 8*E; k_own_copy reads and
        # writes the events (8*E each way); k_sync_write writes the records
        tot["mover_alg"] += 4 * (r.nbr_old + r.nbr_new) + 8 * ev
        tot["own_copy_alg"] += 16 * ev
        tot["sync_write_alg"] += 24 * s.n_rec
        tot["a_nbr"] += r.nbr_old + r.nbr_new
        tot["cand"] += r.pairs_tested
    g.synchronize()
    t1 = time.perf_counter()
    ctl.barrier()
    elapsed = t1 - t0
    dom_us = dom_bytes = None
    if a.profile_stages:
        # HIP events recorded live around the dominant kernel in the timed region, read back here
        for name, us, b, calls in g.stage_times():
            if name == "diff":
                dom_us, dom_bytes = us / calls, b / calls
        # per-stage breakdown: every stage timed over a few more (untimed) steps
        g.set_profiling(1)
        for t in range(a.warmup + a.steps, a.warmup + a.steps + extra):
            run.step(t)
        acc_stages()
        g.set_profiling(0)
    client = client_msgs(run, a.warmup + a.steps + extra, cm) if cm else None
    e2e = None
    if n_e2e:
        # end-to-end game ticks (host ops in, events + records out over PCIe),
        # after the timed region; wall clock per step
        t_e, e_ops = 0.0, 0
        for t in range(a.warmup + a.steps + extra + cm, a.warmup + a.steps + extra + cm + n_e2e):
            g.synchronize()
            c0 = time.perf_counter()
            upd, r, s_ = run.step_e2e(t)
            t_e += time.perf_counter() - c0
            e_ops += upd
        e2e = {"ms_per_step": t_e / n_e2e * 1e3, "updates_per_sec": e_ops / t_e, "steps": n_e2e,
               "what": "gw_submit(host ops) + gw_tick(COPY_TO_HOST) + gw_sync_collect(COPY_TO_HOST): the Go "
                       "caller's tick, events and compact records copied to pinned host memory (PCIe); "
                       "wall clock, untimed by the headline"}
    mx = ctl.reduce([elapsed], "MAX")[0]
    sums = ctl.reduce([tot["ops"], tot["events"], tot["records"]], "SUM")
    if rank != 0:
        run.close()
        return
    K = a.steps
    if a.config == 4:
        workload = (f"config #4: {a.spaces} independent AOI spaces x 1000 entities (uniform, L = 1024, AOI "
                    f"distance 100), 10% movers per space per tick (step +-4), space s on GPU s mod {ws}, every "
                    f"space of a GPU in one tick; step = gw_tick + gw_sync_collect")
    elif a.config == 5:
        workload = (f"config #5: one 16M-entity uniform world space, L = 131072, AOI distance 100, 10% movers "
                    f"per tick (step +-4), decomposed into {ws} X-strip(s) of {131072 // ws} x 131072 (walkers "
                    f"reflect at strip borders); step = route + halo exchange + gw_tick + gw_sync_collect")
    elif world:
        workload = (f"config #5 shape: one world space of {ws} x {a.entities} entities decomposed into {ws} "
                    f"X-strips of {a.side:g} x {a.side:g}, each with config #3 statistics (70% uniform + 30% in "
                    f"64 Gaussian hotspots, 10% movers per tick), AOI distance 100; step = route + halo "
                    f"exchange + gw_tick + gw_sync_collect on every rank")
    else:
        workload = ("config #3: single AOI space per GPU, 1M entities, 70% uniform + 30% in 64 "
                    "Gaussian hotspots (sigma 200), 10% movers per tick (+-4 / hotspot +-16), "
                    "AOI distance 100, world 32768^2; step = gw_tick + gw_sync_collect")
    line = {
        "metric": "entity AOI updates/sec + enter/leave events/sec, 1M-entity space, 1/2/4/8 GPU",
        "value": sums[0] / mx,
        "unit": "updates/s",
        "n_gpus": ws,
        "steps": K,
        "warmup": a.warmup,
        "ms_per_step": mx / K * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if a.config in (4, 5) else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": (f"synthetic (seeded SplitMix64 traces, SURVEY 8(d) config #{a.config})" if a.config in (4, 5) else
                 "synthetic (seeded SplitMix64 traces, SURVEY 8(d) config #3" + (" per strip)" if world else ")")),
        "config": {"workload": workload,
                   "entities_per_gpu": run.n_world // ws, "world_entities": run.n_world,
                   "movers_per_tick_per_gpu": run.m, "aoi_dist": 100.0,
                   "world_side": {4: 1024.0, 5: 131072.0}.get(a.config, a.side), "gates": 1,
                   "parallelism": run.parallelism},
        "events_per_sec": sums[1] / mx,
        "records_per_sec": sums[2] / mx,
        "device_us_per_step": (sum(stage_us.values()) / extra) if stage_us else None,
        "bytes_alg_per_step": tot["bytes_alg"] / K,
        "tick_hbm_frac": (tot["bytes_alg"] / K) / (mx / K) / (HBM_PEAK_GBS * 1e9),
        "load_s": t_load,
    }
    if stage_us or dom_us:
        # the dominant kernel: k_mover, alone in stage "diff", timed live by HIP
        # events on the library's stream in every timed step.  achieved = its
        # SURVEY 8(d) bytes per launch (4*(A_old+A_new) + 8*E: the neighbour-list
        # and event terms it produces; A and E from gw_tick_out) / that duration
        mover_alg = tot["mover_alg"] / K
        ach = mover_alg / (dom_us * 1e-6) / 1e9
        kern, psrc, pstamp = pmc_traffic(a.config if a.config != 5 or ws == 1 else None)
        def traffic(k):
            return (kern or {}).get(k, {}).get("hbm_bytes") if kern else None
        mv = STAGE_KERNEL["diff"]
        line["roofline"] = {"bound": "hbm", "kernel": mv, "achieved": ach, "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic(mv),
                            "traffic_unit": "bytes/launch", "traffic_source": psrc, "traffic_src_hash": pstamp,
                            "bytes_alg_per_launch": mover_alg, "avg_us": dom_us,
                            "bytes_alg_def": "SURVEY 8(d): 4*(A_old+A_new) + 8*(n_enter+n_leave) per tick",
                            "impl_bytes_per_launch": 16 * tot["cand"] / K + 4 * tot["events"] / K,
                            "impl_bytes_def": "16 B per candidate pair tested + 4 B per own event (what the "
                                              "kernel actually reads; not the roofline numerator)",
                            "timing": "HIP events around the kernel on its stream, every timed step"}
        kt = {}
        for k, alg in ((mv, mover_alg), ("k_own_copy", tot["own_copy_alg"] / K),
                       ("k_sync_write<4>", tot["sync_write_alg"] / K)):
            tr_ = traffic(k)
            kt[k] = {"bytes_alg": alg, "traffic": tr_, "traffic_over_alg": (tr_ / alg) if (tr_ and alg) else None}
        line["kernels"] = kt
    if stage_us:
        stages = {n: {"avg_us": stage_us[n] / stage_n[n], "bytes_alg": stage_bytes[n] / stage_n[n]}
                  for n in stage_us}
        line["stages"] = {n: {"avg_us": round(v["avg_us"], 2), "GBps_impl": round(
            v["bytes_alg"] / max(v["avg_us"], 1e-9) / 1e3, 1)} for n, v in stages.items()}
    if not (stage_us or dom_us):
        line["roofline"] = None
    if e2e:
        line["t_e2e"] = e2e
        line["t_device_ms_per_step"] = mx / K * 1e3
    if client:
        line["client_msgs"] = client
    if not a.no_cpu_baseline and ws == 1 and a.config == 3:
        cb = cpu_baseline(traces.config3(ticks=1, seed=3, n=a.entities, side=a.side), a.cpu_st_max_seconds)
        line["cpu_baseline"] = cb
        line["cpu_baseline_mt"] = cpu_baseline_mt(a.cpu_seconds, a.entities, a.side)
    print(json.dumps(line), flush=True)
    run.close()


if __name__ == "__main__":
    main()
