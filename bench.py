#!/usr/bin/env python3
"""Benchmark of the MI355X AOI + entity-sync hot path (BASELINE.json metric:
entity AOI updates/s + enter/leave events/s, 1M-entity space, 1/2/4/8 GPU).

A step = one game tick of the hot path over one batch of synthetic input:
gw_tick (apply the tick's Moved ops, update every relation, emit the canonical
enter/leave streams) + gw_sync_collect (CollectEntitySyncInfos: per-watcher
position/yaw records).

N=1 (default): BASELINE config #3, the 1M-entity clustered-hotspot space the
metric is quoted on, on one GPU.
N>1 (default --mode world): the SAME 1M-entity space decomposed into N
X-strips, one per GPU (strong scaling; goworld_amd/dworld.py over the
library's gw_world_* path): each tick every rank routes its owned ops,
exchanges halo rows with both neighbours (and far rows of long moves) over
RCCL inside the library (xGMI) and ticks its strip; walkers cross borders.
Two legs ride along in every N>1 line:
  "spaces": an independent 1M-entity config #3 space per GPU (seed 3 + rank),
  no data-path collective (weak scaling: a space never spans processes in the
  reference, engine/entity/SpaceManager.go:11-31, so that is how it shards);
  "config5": the north star's 16M-entity world decomposed over the same N GPUs
  (also measured at N=1).  --no-spaces-leg / --no-config5 skip them.
--mode spaces: the weak line as the headline ("c3world" rides along).
--config 4 / 5: BASELINE config #4 (10k spaces x 1k) / #5 as the headline.
--comm loopback --gpus N: the world's N ranks as N threads of ONE process on
one device (the library's loopback transport, the RCCL path's exact call
sequence): a rehearsal of the multi-rank path, not a scaling number.

Inputs (ops of every tick) are resident in HBM before the timed region;
outputs stay in HBM (device-resident boundary); t_e2e reports the host-in /
host-out tick separately.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N>1 without torchrun: this process spawns the N rank processes itself,
      one per GPU, and never touches a GPU; rank 0 prints the line)
N>1:  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
      (WORLD_SIZE must equal --gpus)
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

PCIE_GBS = 57.1          # device->host copy rate into pinned memory on the box (tools/micro/pcie.hip, profiles/r03f_pcie.txt)
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
    ap.add_argument("--e2e-steps", type=int, default=8, help="untimed end-to-end steps (host in/out), split over "
                                                                 "the two caller paths; the first of each is a warm-up")
    ap.add_argument("--e2e-wire", type=int, default=1,
                    help="1: half the end-to-end steps take the Go shim's path instead: the 48-B game->gate wire "
                         "records (gw_sync_encode_wire) to the host, the compact records left on the device")
    ap.add_argument("--profile-stages", type=int, default=1,
                    help="1: HIP events around the dominant kernel's stage in the timed region (roofline) and "
                         "a per-stage breakdown over extra untimed steps; 0: none")
    ap.add_argument("--mode", choices=["world", "spaces"], default="world",
                    help="N>1 with config 3: world = the metric's 1M space decomposed over the N GPUs (strong; "
                         "default); spaces = an independent 1M space per GPU, no comm (weak)")
    ap.add_argument("--no-c3world", dest="c3world", action="store_false",
                    help="N>1, --mode spaces: skip the extra strong-scaling leg of the 1M space decomposed over N GPUs")
    ap.add_argument("--no-spaces-leg", dest="spaces_leg", action="store_false",
                    help="N>1, --mode world: skip the weak-scaling leg (an independent 1M space per GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / control-plane rehearsal: ranks, barriers and the max-over-ranks timing with no "
                         "GPU work (CPU tests)")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=3,
                    help="3: the metric's 1M clustered space (N=1: one GPU; N>1: decomposed over the N GPUs); "
                         "4: config #4, 10k independent 1k-entity spaces, space s on GPU s mod N (strong); "
                         "5: the 16M uniform world of config #5 over N strips (strong)")
    ap.add_argument("--spaces", type=int, default=10_000, help="config #4: number of spaces")
    ap.add_argument("--comm", choices=["rccl", "gloo", "loopback"], default="rccl",
                    help="halo exchange: RCCL inside the library (gw_world_step, one process per GPU); gloo "
                         "(rank processes sharing one GPU, rows through the host); loopback (ONE process, --gpus N "
                         "rank threads on --device, gw_world_step over the library's loopback transport: the "
                         "multi-rank call sequence on one GPU, not a scaling number)")
    ap.add_argument("--world-entities", type=int, default=16_000_000, help="config #5 world population")
    ap.add_argument("--no-config5", dest="config5", action="store_false",
                    help="skip the extra config #5 (16M decomposed world) measurement")
    ap.add_argument("--warmup5", type=int, default=5)
    ap.add_argument("--steps5", type=int, default=10, help="config #5 timed ticks (SURVEY 8(d): 10)")
    ap.add_argument("--device", type=int, default=None, help="force a device (rehearsals on one GPU)")
    ap.add_argument("--gates", type=int, default=1,
                    help="config #2/#3: gate processes the clients are spread over (SURVEY 8(d): G = 1 by default, "
                         "optionally G = 4; goworld_actions.ini deploys 3); the collect then partitions its records "
                         "by gate (Entity.go:1208-1219)")
    ap.add_argument("--sync-by-client", action="store_true",
                    help="collect grouped per client (GW_SYNC_BY_CLIENT, the gate's regroup on the GPU)")
    ap.add_argument("--client-msgs", type=int, default=5,
                    help="extra untimed ticks measuring gw_client_events + gw_fanout (N=1 config #3; 0 = off)")
    ap.add_argument("--capacity", type=int, default=None,
                    help="slot capacity of the space (N=1: cost of a strip's id range at N ranks)")
    return ap.parse_args()


class Ctl:
    """Control plane (barrier, max/sum of scalars, the RCCL id broadcast) on a
    gloo group; the data path (halo rows) runs inside the library over its
    own RCCL communicator."""

    def __init__(self, a):
        self.ws = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0")) if a.device is None else a.device
        self.group = None
        if self.ws > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.ws)
            self.group = dist.group.WORLD
            self.dist = dist

    def close(self, ok=True):
        """Leave the group together (a rank process that exits while its
        peers' gloo threads still talk to it can abort them)."""
        if self.group is None:
            return
        if ok:
            self.dist.barrier(group=self.group)
        self.dist.destroy_process_group()
        self.group = None

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

    def bcast_bytes(self, b: bytes) -> bytes:
        if self.group is None:
            return b
        import torch
        t = torch.tensor(list(b), dtype=torch.uint8)
        self.dist.broadcast(t, src=0, group=self.group)
        return bytes(t.tolist())


def launch(a):
    """--gpus N is the number of rank processes, one per GPU.  Under torchrun
    (WORLD_SIZE set) this process is one of them and WORLD_SIZE must equal N.
    Otherwise, for N > 1, this process is only the launcher: it never touches
    a GPU, starts N copies of this script with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set (rank r on GPU r, or on --device for one-GPU rehearsals),
    lets rank 0 print the line, stops the others when one fails and returns
    the exit code.  Returns None when this process should run as a rank."""
    env_ws = os.environ.get("WORLD_SIZE")
    if a.gpus < 1:
        print(f"bench.py: --gpus {a.gpus} must be >= 1", file=sys.stderr)
        return 2
    if env_ws is not None:
        if int(env_ws) != a.gpus:
            print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_ws} (launch N ranks for --gpus N)",
                  file=sys.stderr)
            return 2
        return None
    if a.gpus == 1 or a.comm == "loopback":        # loopback: the N ranks are threads of this process
        return None
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc, live = 0, set(range(a.gpus))
    try:
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                    for q in live:
                        procs[q].send_signal(signal.SIGTERM)
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def dry_run(a, ctl):
    """Control-plane rehearsal (no GPU): W + K empty steps between barriers,
    the max-over-ranks time and the sum of the ranks' unit counts, as measure()."""
    for _ in range(a.warmup):
        ctl.barrier()
    ctl.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctl.barrier()
    el = time.perf_counter() - t0
    ctl.barrier()
    mx = ctl.reduce([el], "MAX")[0]
    ranks = ctl.reduce([1.0], "SUM")[0]
    if ctl.rank == 0:
        print(json.dumps({"metric": "entity AOI updates/sec + enter/leave events/sec, 1M-entity space, 1/2/4/8 GPU",
                          "value": None, "unit": "updates/s", "n_gpus": ctl.ws, "steps": a.steps,
                          "warmup": a.warmup, "ms_per_step": mx / max(a.steps, 1) * 1e3, "dry_run": True,
                          "ranks_reporting": int(ranks), "higher_is_better": True}), flush=True)


# the diff stage's kernel: k_mover_c (one wave per primary mover entry), k_mover (one wave per
# mover-grid entry, GW_MOVER_COMPACT=0), or k_mover_pair when GW_PAIR_MAX > 0
# (k_mover_c<2, false, 0>: the variant without the group-teleport paths, launched unless the context is a
# world of >= 2 strips, and without the per-gate split of a context with 3-16 gate ids;
# k_mover_small<2, true>: the half-wave walk)
STAGE_KERNEL = {"diff": "k_mover_pair<2>" if int(os.environ.get("GW_PAIR_MAX", "0") or 0) > 0
                else "k_mover<2, 1>" if os.environ.get("GW_MOVER_COMPACT", "1") == "0" else "k_mover_c<2, false, 0>"}
# the stage's kernel differs in small-space mode (config #4: many spaces whose grids fit LDS)
STAGE_KERNEL_C4 = {"diff": "k_mover_small<2, true>", "sync_write": "k_sync_write_small2"}
PMC_DIR = os.path.join(ROOT, "profiles")


def src_hash():
    """Hash of the device-code sources (kernels, their launchers and device
    headers): the PMC pass must come from these exact kernels."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, "goworld_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith(".hip") or f in ("dev_common.hpp", "prim.hpp", "gw_internal.hpp"):
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


def cpu_quota():
    """CPU cores the cgroup grants this job (cpu.max quota / period), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def cpu_baseline_mt(seconds, entities, side, threads=None):
    """Fairness point: oracle/gridmt.c, a multi-threaded (OpenMP)
    uniform-grid CPU implementation of the same batched tick + collect, over
    config #3 ticks until the time budget is spent.  threads: by default the
    job's share (OMP_NUM_THREADS, 16 per GPU on the box); main() also runs it
    on every core the process may use (sched_getaffinity)."""
    from oracle import pyorc
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
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
        if a.config == 2:                               # BASELINE config #2: 100k uniform, L = 10240
            self.tr = traces.config2(ticks=ticks, seed=2 + ctl.rank)
        else:
            self.tr = traces.config3(ticks=ticks, seed=3 + ctl.rank, n=a.entities, side=a.side)
        if a.gates > 1:                                 # clients spread round-robin over the gates
            self.tr.gates = np.where(self.tr.gates > 0, 1 + np.arange(len(self.tr.gates)) % a.gates,
                                     0).astype(np.uint16)
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
        self.n_world = self.tr.n * (ctl.ws if ctl.ws > 1 else 1)

    def step(self, t):
        # gw_step: submit + deferred tick + collect in one call (the collect's
        # sync settles the tick); the library's output structs are read back
        r, s = self.g.step_device(self.dev_ops + t * self.nbytes_tick, self.m, by_client=self.by_client)
        return r.movers, r, s

    def replay(self, t0, k):
        """gw_replay: steps t0 .. t0+k-1 (each one gw_step) in one call, the
        tick loop in C as the Go caller runs it (no per-step Python)."""
        return self.g.replay_device(self.dev_ops + t0 * self.nbytes_tick, self.m, self.m, k, by_client=self.by_client)

    def step_e2e(self, t, wire=False):
        """The Go caller's game tick: host ops in (gw_submit: pageable host
        memory, copied to the device), the canonical events out to pinned host
        buffers (GW_TICK_COPY_TO_HOST), then either the compact 24-B sync
        records (GW_SYNC_COPY_TO_HOST; wire=False) or, as the Go shim's Collect
        does, the 48-B game->gate wire packets (gw_sync_encode_wire with
        COPY_TO_HOST; the compact records stay on the device; wire=True)."""
        g = self.g
        c0 = time.perf_counter()
        g.submit(self.host_ticks[t])
        c1 = time.perf_counter()
        r = g.tick(copy=True, view=True)
        c2 = time.perf_counter()
        s = g.sync_collect(copy=not wire, by_client=self.by_client, view=True)
        c3 = time.perf_counter()
        self.e2e_parts = {"submit": c1 - c0, "tick": c2 - c1, "collect": c3 - c2,
                          "tick_device_us": r.device_us, "collect_device_us": s.device_us,
                          "ops_bytes": len(self.host_ticks[t]) * traces.OP_DTYPE.itemsize,
                          "event_bytes": 8 * (r.n_enter + r.n_leave), "record_bytes": 0 if wire else 24 * s.n_rec}
        if wire:
            data, pk, nb, dev_us = g.encode_wire(copy=True, view=True)
            self.e2e_parts.update(wire=time.perf_counter() - c3, wire_bytes=nb, wire_device_us=dev_us)
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


def world_workload(a, ticks, which):
    """The world legs' population and walk: which = "c3", the metric's 1M
    clustered space as one world (steps +-4, hotspots +-16); "c5", config #5's
    16M uniform world (L = 131072, +-4).  Returns (n, side, max_step, x0, z0,
    yaw0, ticks) with ticks a generator of (ops, x before the tick): every rank
    regenerates the same walk and keeps the ops of the entities it owns at the
    start of each tick."""
    if which == "c5":
        n, side, max_step = a.world_entities, 131072.0, 4.0
        walk = traces.WorldWalk(seed=5, n=n, side=side)
        return n, side, max_step, walk.x(), walk.z(), walk.yaw.copy(), (walk.next_tick() for _ in range(ticks))
    n, side, max_step = a.entities, a.side, 16.0
    tr = traces.config3(ticks=ticks, seed=3, n=n, side=side)
    xcur = tr.init_x.copy()

    def gen3():
        for ops in tr.ticks:
            xb = xcur[ops["slot"]].copy()
            xcur[ops["slot"]] = ops["x"]
            yield ops, xb
    return n, side, max_step, tr.init_x, tr.init_z, tr.init_yaw, gen3()


class WorldRun:
    """One world decomposed into N X-strips, one per GPU (dworld.StripRank over
    the library's gw_world_* path; halo rows over RCCL inside the library).
    which = "c3": the metric's 1M-entity clustered space (config #3) as one
    world over N strips; "c5": config #5, the 16M uniform world (L = 131072).
    Both walks are global: entities cross strip borders and migrate between
    ranks (world_workload)."""

    def __init__(self, a, ctl, ticks, which):
        import torch
        from goworld_amd import dworld
        self.torch = torch
        dev = torch.device("cuda", ctl.local)
        torch.cuda.set_device(dev)
        ws, r = ctl.ws, ctl.rank
        n, side, max_step, x0_all, z0_all, yaw0, gen = world_workload(a, ticks, which)
        geom = dworld.Strips(-side / 2, side / ws, ws, 100.0, max_step)
        lo, hi = geom.ext(r)
        bounds = (max(lo, -side / 2), -side / 2, min(hi, side / 2), side / 2)
        self.n_world = n
        self.g = g = gpuaoi.GpuAOI(ctl.local)
        eng = dworld.HipStrip(g)
        comm = "rccl" if (ws > 1 and a.comm == "rccl") else "torch"
        if comm == "rccl":
            g.comm_init(ctl.bcast_bytes(gpuaoi.comm_unique_id() if r == 0 else bytes(gpuaoi.COMM_ID_BYTES)), ws, r)
        self.sr = sr = dworld.StripRank(eng, geom, r, n, bounds, dev, pg=ctl.group, comm=comm,
                                        comm_device=torch.device("cpu"))
        eng.set_clients(np.arange(n, dtype=np.uint32), np.ones(n, np.uint16))   # 1 gate, every entity a client

        def words(ops):
            return torch.from_numpy(dworld.ops_to_words(ops).copy()).to(dev)
        # load: every rank enters the entities it owns (routed to its neighbours
        # as ghosts), in id order, in the same number of chunks on every rank
        owner0 = geom.owner(x0_all)
        mine = np.nonzero(owner0 == r)[0].astype(np.uint32)
        chunk = 1 << 21
        n_chunks = max(1, -(-int(np.bincount(owner0, minlength=ws).max()) // chunk))
        enter = traces.enter_ops(mine, x0_all[mine], np.zeros(len(mine), np.float32), z0_all[mine], yaw0[mine])
        for k in range(n_chunks):
            sr.step(words(enter[k * chunk:(k + 1) * chunk]), copy=False, no_events=True)
        sr.collect(copy=False)
        self.words, self.m_ticks, self.slots = [], [], []
        for ops, xb in gen:
            own = ops[geom.owner(xb) == r]
            self.words.append(words(own))                    # resident in HBM
            self.m_ticks.append(len(own))
            self.slots.append(own["slot"])
        self.m = int(np.mean(self.m_ticks))
        self.one_call = comm == "rccl" or ws == 1        # the exchange runs inside the library
        torch.cuda.synchronize()
        self.parallelism = (f"decomposed world, {ws} X-strips of {side / ws:g} x {side:g}, halo rows over "
                            f"{'RCCL (gw_world_step)' if comm == 'rccl' else 'gloo'}" if ws > 1
                            else "single GPU, one-strip world")
        self.ranks = ws
        self.tr = None

    def step(self, t):
        if self.one_call:                    # gw_step: gw_world_step + tick + collect in one call
            w = self.words[t]
            r, s = self.g.step_device(w.data_ptr(), w.shape[0])
            return self.m_ticks[t], r, s
        self.sr.step(self.words[t], copy=False, defer=True)
        s = self.sr.collect(copy=False)
        return self.m_ticks[t], self.sr.e.tick_result(), s

    def close(self):
        self.sr.check()
        self.g.close()


class _Sum:
    """Counters of one step summed over the loopback ranks (TickOut / SyncOut fields measure() reads)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class _RanksG:
    """measure()'s view of the loopback ranks' contexts: every call on all of
    them (stage times: per stage the slowest rank)."""

    def __init__(self, lw):
        self.lw = lw

    def synchronize(self):
        for g in self.lw.g:
            g.synchronize()

    def set_profiling(self, mode):
        for g in self.lw.g:
            g.set_profiling(mode)

    def stage_times(self):
        best = {}
        for g in self.lw.g:
            for name, us, b, calls in g.stage_times():
                if name not in best or us / max(calls, 1) > best[name][0] / max(best[name][2], 1):
                    best[name] = (us, b, calls)
        return [(k, *v) for k, v in best.items()]


class LoopbackWorldRun:
    """--comm loopback: the world of world_workload decomposed into --gpus R
    X-strips whose R contexts live in THIS process on one device, each rank
    driven by its own thread through gw_step (gw_world_step over the library's
    loopback transport: the count round, host read, far all-gather and exact
    rows of the RCCL path, bytes copied between the contexts; dworld.
    LoopbackWorld).  The R ranks share one GPU, so the time is not a scaling
    number; the line shows the multi-rank path running end to end."""

    def __init__(self, a, ticks, which):
        from goworld_amd import dworld
        R = a.gpus
        n, side, max_step, x0_all, z0_all, yaw0, gen = world_workload(a, ticks, which)
        geom = dworld.Strips(-side / 2, side / R, R, 100.0, max_step)
        dev = a.device if a.device is not None else 0
        self.lw = lw = dworld.LoopbackWorld(geom, n, (-side / 2, -side / 2, side / 2, side / 2), device=dev)
        lw.load(x0_all, z0_all, yaw0)
        self.ptrs, self.m_ticks = [], []
        for ops, xb in gen:
            own = geom.owner(xb)
            mine = [ops[own == r] for r in range(R)]
            self.ptrs.append([(lw.upload(r, mine[r]), len(mine[r])) for r in range(R)])
            self.m_ticks.append(sum(len(x) for x in mine))
        self.g = _RanksG(lw)
        self.n_world, self.ranks = n, R
        self.m = int(np.mean(self.m_ticks) / R)          # per rank
        self.parallelism = (f"decomposed world, {R} X-strips of {side / R:g} x {side:g}, {R} rank threads on "
                            f"device {dev}, halo rows over the loopback transport (gw_world_step); the ranks share "
                            f"one GPU: not a scaling number")
        self.tr = None

    def step(self, t):
        ptrs = self.ptrs[t]

        def one(r, g):
            to, so = g.step_device(*ptrs[r])
            return (to.n_enter, to.n_leave, to.bytes_alg, to.nbr_old, to.nbr_new, to.pairs_tested, so.n_rec,
                    so.bytes_alg)
        v = np.array(self.lw.run(one), np.float64).sum(axis=0)
        r = _Sum(n_enter=int(v[0]), n_leave=int(v[1]), bytes_alg=int(v[2]), nbr_old=int(v[3]), nbr_new=int(v[4]),
                 pairs_tested=int(v[5]))
        return self.m_ticks[t], r, _Sum(n_rec=int(v[6]), bytes_alg=int(v[7]))

    def close(self):
        self.lw.check()
        self.lw.close()


def client_msgs(run, t0, n):
    """SURVEY 8(f) ranks 2-3, outside the headline step: after each of n more
    ticks, gw_client_events (create/destroy messages of the tick's events) and
    gw_fanout of one AllClients call per mover (e.g. an attribute change),
    outputs left on the device; wall time per call (each ends in a host sync)."""
    g = run.g
    t_ev = t_fo = 0.0
    n_cr = n_de = n_fo = n_calls = b_ev = b_fo = 0
    # one untimed call of each on the last tick first: the first call's buffer
    # allocations (hipMalloc of the message and sort buffers, ~0.8 / 1.2 ms)
    # stay out of the per-tick averages
    g.synchronize()
    g.client_events(copy=False)
    g.fanout(run.tr.ticks[max(t0 - 1, 0)]["slot"], copy=False)
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
            "timing": "host wall clock around each call (one host sync inside each), after one untimed call "
                      "of each; not part of ms_per_step"}


def measure(run, a, ctl, warmup, steps, profile, extra):
    """W untimed steps, then exactly K steps bracketed by a barrier and a device
    sync on both sides; HIP events around the dominant kernel's stage in every
    timed step; a per-stage breakdown over `extra` more untimed steps."""
    g = run.g
    for t in range(warmup):
        run.step(t)
    g.set_profiling(2 if profile else 0)    # the dominant kernel's stage only
    tot = dict(ops=0, events=0, records=0, bytes_alg=0, mover_alg=0, cand=0, events_alg=0, sync_write_alg=0)
    ctl.barrier()
    g.synchronize()
    t0 = time.perf_counter()
    if hasattr(run, "replay"):                  # the K steps as one gw_replay call
        sm = run.replay(warmup, steps)
        ev = sm["n_enter"] + sm["n_leave"]
        tot.update(ops=sm["movers"], events=ev, records=sm["n_rec"], bytes_alg=sm["bytes_alg"],
                   mover_alg=4 * (sm["nbr_old"] + sm["nbr_new"]) + 8 * ev, events_alg=8 * ev,
                   sync_write_alg=24 * sm["n_rec"], cand=sm["pairs_tested"])
    for t in range(warmup, warmup + steps) if not hasattr(run, "replay") else ():
        upd, r, s = run.step(t)
        ev = r.n_enter + r.n_leave
        tot["ops"] += upd
        tot["events"] += ev
        tot["records"] += s.n_rec
        tot["bytes_alg"] += r.bytes_alg + s.bytes_alg
        # SURVEY 8(d) terms per kernel: k_mover produces the neighbour-list
        # terms and the net events, 4*(A_old+A_new) + 8*E; k_bucket_sort writes
        # the canonical event arrays (8*E); k_sync_write writes the records
        tot["mover_alg"] += 4 * (r.nbr_old + r.nbr_new) + 8 * ev
        tot["events_alg"] += 8 * ev
        tot["sync_write_alg"] += 24 * s.n_rec
        tot["cand"] += r.pairs_tested
    g.synchronize()
    t1 = time.perf_counter()
    ctl.barrier()
    res = {"elapsed": t1 - t0, "tot": tot, "dom_us": None, "stages": {}}
    if profile:
        for name, us, b, calls in g.stage_times():       # HIP events read back here, after the timed region
            if name == "diff":
                res["dom_us"] = us / calls
        g.set_profiling(1)
        for t in range(warmup + steps, warmup + steps + extra):
            run.step(t)
        acc = {}
        for name, us, b, calls in g.stage_times():
            v = acc.setdefault(name, [0.0, 0, 0])
            v[0] += us; v[1] += b; v[2] += calls
        res["stages"] = {n: {"avg_us": v[0] / v[2], "bytes_impl": v[1] / v[2]} for n, v in acc.items()}
        g.set_profiling(0)
    mx = ctl.reduce([res["elapsed"]], "MAX")[0]
    sums = ctl.reduce([tot["ops"], tot["events"], tot["records"]], "SUM")
    res.update(max_elapsed=mx, sum_ops=sums[0], sum_events=sums[1], sum_records=sums[2])
    return res


def roofline_fields(res, K, config, ws):
    """The dominant kernel (k_mover, alone in stage "diff", timed live by HIP
    events on the library's stream in every timed step): achieved = its SURVEY
    8(d) bytes per launch (4*(A_old+A_new) + 8*E, the neighbour-list and event
    terms it produces, from gw_tick_out) / that duration."""
    tot, dom_us = res["tot"], res["dom_us"]
    out = {}
    if dom_us:
        mover_alg = tot["mover_alg"] / K
        ach = mover_alg / (dom_us * 1e-6) / 1e9
        kern, psrc, pstamp = pmc_traffic(config) if ws == 1 else (None, None, "n/a (N>1)")

        def traffic(k):
            if not kern:
                return None
            if k not in kern:                   # a template's other instantiation, if only one was profiled
                alt = [n for n in kern if n.split("<")[0] == k.split("<")[0]]
                k = alt[0] if len(alt) == 1 else k
            return kern.get(k, {}).get("hbm_bytes")
        names = STAGE_KERNEL_C4 if config == 4 else STAGE_KERNEL
        mv = names["diff"]
        sw = names.get("sync_write", "k_sync_write<4, false>")
        out["roofline"] = {"bound": "hbm", "kernel": mv, "achieved": ach, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic(mv),
                           "traffic_unit": "bytes/launch", "traffic_source": psrc, "traffic_src_hash": pstamp,
                           "bytes_alg_per_launch": mover_alg, "avg_us": dom_us,
                           "bytes_alg_def": "SURVEY 8(d): 4*(A_old+A_new) + 8*(n_enter+n_leave) per tick",
                           "impl_bytes_per_launch": 16 * tot["cand"] / K + 4 * tot["events"] / K,
                           "impl_bytes_def": "16 B per candidate pair tested + 4 B per own event (what the "
                                             "kernel reads; not the roofline numerator)",
                           "timing": "HIP events around the kernel on its stream, every timed step"}
        kt = {}
        for k, alg in ((mv, mover_alg), ("k_bucket_sort", tot["events_alg"] / K),
                       (sw, tot["sync_write_alg"] / K)):
            tr_ = traffic(k)
            kt[k] = {"bytes_alg": alg, "traffic": tr_, "traffic_over_alg": (tr_ / alg) if (tr_ and alg) else None}
        out["kernels"] = kt
    else:
        out["roofline"] = None
    if res["stages"]:
        out["stages"] = {n: {"avg_us": round(v["avg_us"], 2),
                             "GBps_impl": round(v["bytes_impl"] / max(v["avg_us"], 1e-9) / 1e3, 1)}
                         for n, v in res["stages"].items()}
    return out


def main():
    a = parse()
    rc = launch(a)
    if rc is not None:                              # the launcher of N ranks (or a bad --gpus)
        sys.exit(rc)
    ctl = Ctl(a)
    ok = False
    try:
        if a.dry_run:
            dry_run(a, ctl)
        else:
            run(a, ctl)
        ok = True
    finally:
        ctl.close(ok)


def run(a, ctl):
    ws, rank = ctl.ws, ctl.rank
    loop = a.comm == "loopback" and a.gpus > 1   # the N ranks are threads of this process on one device
    R = a.gpus if loop else ws                    # ranks of the run
    extra = 5 if a.profile_stages else 0         # untimed steps for the per-stage breakdown
    if a.config == 2:
        kind = "c2"                                 # config #2 (100k uniform), one space per GPU
    elif a.config == 4:
        kind = "c4"
    elif a.config == 5:
        kind = "c5"
    elif R > 1 and (a.mode == "world" or loop):
        kind = "c3world"                            # the metric's 1M space decomposed over the N GPUs (default)
    else:
        kind = "c3"                                 # N=1: the 1M space on one GPU
    if loop and kind not in ("c3world", "c5"):
        print("bench.py: --comm loopback runs a decomposed world (config 3 --mode world, or --config 5)",
              file=sys.stderr)
        sys.exit(2)
    c3world_leg = a.c3world and R > 1 and kind == "c3"   # --mode spaces: the 1M space decomposed, beside it
    spaces_leg = a.spaces_leg and R > 1 and kind == "c3world" and not loop   # the weak line, beside the world
    c5_leg = a.config5 and kind in ("c3", "c3world") and not loop
    if not loop and (kind in ("c5", "c3world") or c5_leg or c3world_leg):
        # torch (decomposed-world runs) brings its own HIP runtime: it must
        # initialise before the library's runtime does, in this process
        import torch
        torch.cuda.set_device(ctl.local)
        torch.zeros(1, device=torch.device("cuda", ctl.local))
    cm = a.client_msgs if (ws == 1 and kind == "c3") else 0
    n_e2e = a.e2e_steps if kind in ("c2", "c3", "c4") else 0
    W, K = a.warmup, a.steps
    ticks = W + K + extra + cm + n_e2e
    t_load = time.perf_counter()
    if kind == "c4":
        run = ManySpacesRun(a, ctl, ticks)
    elif kind in ("c5", "c3world"):
        which = "c5" if kind == "c5" else "c3"
        run = LoopbackWorldRun(a, ticks, which) if loop else WorldRun(a, ctl, ticks, which)
    else:
        run = SpaceRun(a, ctl, ticks)
    t_load = time.perf_counter() - t_load
    g = run.g
    res = measure(run, a, ctl, W, K, a.profile_stages, extra)
    client = client_msgs(run, W + K + extra, cm) if cm else None
    e2e = {}
    if n_e2e >= 2:
        # end-to-end game ticks (host ops in, events + records / wire packets out
        # over PCIe), after the timed region; wall clock per step, the first of
        # each path (which allocates the pinned host buffers) untimed
        t_next = W + K + extra + cm
        for key, wire in (("t_e2e", False), ("t_e2e_wire", True)):
            if wire and not a.e2e_wire:
                continue
            t_e, e_ops, parts = 0.0, 0, {}
            n2 = n_e2e // 2 - 1 if a.e2e_wire else n_e2e - 1
            if n2 < 1:
                continue
            run.step_e2e(t_next, wire)
            t_next += 1
            for _ in range(n2):
                g.synchronize()
                c0 = time.perf_counter()
                upd, r, s_ = run.step_e2e(t_next, wire)
                t_e += time.perf_counter() - c0
                t_next += 1
                e_ops += upd
                for k, v in run.e2e_parts.items():
                    parts[k] = parts.get(k, 0.0) + v
            pa = {k: v / n2 for k, v in parts.items()}
            h2d = pa["ops_bytes"]
            d2h = pa["event_bytes"] + pa["record_bytes"] + pa.get("wire_bytes", 0)
            ms = t_e / n2 * 1e3
            # PCIe roofline of the step: its host<->device bytes at the copy rate
            # tools/micro/pcie.hip measures on the box (pinned, one stream)
            floor_ms = (h2d + d2h) / (PCIE_GBS * 1e9) * 1e3
            e2e[key] = {
                "ms_per_step": ms, "updates_per_sec": e_ops / t_e, "steps": n2,
                "breakdown_ms": {k: round(pa[k] * 1e3, 3) for k in ("submit", "tick", "collect", "wire") if k in pa},
                "device_ms": {"tick": round(pa["tick_device_us"] / 1e3, 3),
                              "collect": round(pa["collect_device_us"] / 1e3, 3),
                              **({"wire": round(pa["wire_device_us"] / 1e3, 3)} if wire else {})},
                "bytes_per_step": {"ops_h2d": h2d, "events_d2h": pa["event_bytes"],
                                   **({"wire_d2h": pa["wire_bytes"]} if wire else {"records_d2h": pa["record_bytes"]})},
                "pcie_GBps": {"tick": round(pa["event_bytes"] / pa["tick"] / 1e9, 2),
                              **({"wire": round(pa["wire_bytes"] / pa["wire"] / 1e9, 2)} if wire else
                                 {"collect": round(pa["record_bytes"] / pa["collect"] / 1e9, 2)})},
                "pcie_roofline": {"bound": "pcie", "peak_GBps": PCIE_GBS, "floor_ms": round(floor_ms, 3),
                                  "frac": round(floor_ms / ms, 3)},
                "what": ("gw_submit(host ops) + gw_tick(COPY_TO_HOST) + gw_sync_collect() + "
                         "gw_sync_encode_wire(COPY_TO_HOST): the Go shim's tick (INTEGRATION.md), events and "
                         "48-B wire packets to pinned host memory" if wire else
                         "gw_submit(host ops) + gw_tick(COPY_TO_HOST) + gw_sync_collect(COPY_TO_HOST): events "
                         "and compact 24-B records to pinned host memory") +
                        "; wall clock per call (device_ms: HIP events of the same calls, copies included); "
                        "untimed by the headline"}
    parallelism, n_world, m_rank = run.parallelism, run.n_world, run.m
    run.close()
    def world_leg(which, warmup, steps, workload):
        runw = WorldRun(a, ctl, warmup + steps + (extra if a.profile_stages else 0), which)
        rw = measure(runw, a, ctl, warmup, steps, a.profile_stages, extra)
        leg = {"workload": workload, "value": rw["sum_ops"] / rw["max_elapsed"], "unit": "updates/s",
               "events_per_sec": rw["sum_events"] / rw["max_elapsed"],
               "records_per_sec": rw["sum_records"] / rw["max_elapsed"],
               "ms_per_step": rw["max_elapsed"] / steps * 1e3, "steps": steps, "warmup": warmup,
               "scaling": "strong", "n_gpus": ws, "parallelism": runw.parallelism,
               "roofline_frac": (roofline_fields(rw, steps, 5 if which == "c5" else 3, ws).get("roofline")
                                 or {}).get("frac")}
        runw.close()
        return leg
    # --mode spaces: the metric's 1M space decomposed over the same N GPUs (strong), beside the weak headline
    c3w = None
    if c3world_leg:
        c3w = world_leg("c3", W, K, (
            f"config #3 as one world: the 1M-entity clustered space decomposed into {ws} X-strips of "
            f"{a.side / ws:g}, one per GPU (walkers cross strip borders); step = route + RCCL halo exchange + "
            f"gw_tick + gw_sync_collect on every rank"))
    # --mode world (default): an independent 1M config #3 space per GPU (weak, no collective), beside it
    spc = None
    if spaces_leg:
        runs = SpaceRun(a, ctl, W + K)
        rs = measure(runs, a, ctl, W, K, False, 0)
        spc = {"workload": (f"config #3: an independent 1M-entity space per GPU (seed 3 + rank), {ws} GPUs, no "
                            f"collective; step = gw_tick + gw_sync_collect"),
               "value": rs["sum_ops"] / rs["max_elapsed"], "unit": "updates/s",
               "events_per_sec": rs["sum_events"] / rs["max_elapsed"],
               "records_per_sec": rs["sum_records"] / rs["max_elapsed"],
               "ms_per_step": rs["max_elapsed"] / K * 1e3, "steps": K, "warmup": W, "scaling": "weak",
               "n_gpus": ws, "parallelism": runs.parallelism}
        runs.close()
    # the north star's 16M decomposed world (config #5) at the same N, strong scaling
    c5 = None
    if c5_leg:
        c5 = world_leg("c5", a.warmup5, a.steps5, (
            "config #5: one 16M-entity uniform world space, L = 131072, AOI distance 100, 10% movers "
            f"per tick (+-4; walkers cross strip borders), decomposed into {ws} X-strip(s); step = "
            "route + RCCL halo exchange + gw_tick + gw_sync_collect on every rank"))
    if rank != 0:
        return
    mx = res["max_elapsed"]
    if kind == "c4":
        workload = (f"config #4: {a.spaces} independent AOI spaces x 1000 entities (uniform, L = 1024, AOI "
                    f"distance 100), 10% movers per space per tick (step +-4), space s on GPU s mod {ws}, every "
                    f"space of a GPU in one tick; step = gw_tick + gw_sync_collect")
    elif kind == "c5":
        workload = c5 and c5["workload"] or (
            f"config #5: one 16M-entity uniform world space, L = 131072, AOI distance 100, 10% movers per tick "
            f"(+-4; walkers cross strip borders), decomposed into {ws} X-strip(s); step = route + RCCL halo "
            f"exchange + gw_tick + gw_sync_collect on every rank")
    elif kind == "c2":
        workload = ("config #2: single AOI space per GPU, 100k uniform-random entities, L = 10240, AOI distance "
                    "100, 10% movers per tick (+-4); step = gw_tick + gw_sync_collect")
    elif kind == "c3world":
        workload = (f"config #3 as one world: the 1M-entity clustered space (70% uniform + 30% in 64 Gaussian "
                    f"hotspots, sigma 200; 10% movers per tick, +-4 / hotspot +-16; AOI distance 100; world "
                    f"32768^2) decomposed into {R} X-strips of {a.side / R:g}, "
                    + (f"{R} rank threads on one GPU (loopback transport)" if loop else "one per GPU")
                    + " (walkers cross strip borders); step = route + "
                    + ("loopback" if loop else "RCCL") + " halo exchange + gw_tick + gw_sync_collect on every rank")
    else:
        workload = ("config #3: single AOI space per GPU, 1M entities, 70% uniform + 30% in 64 "
                    "Gaussian hotspots (sigma 200), 10% movers per tick (+-4 / hotspot +-16), "
                    "AOI distance 100, world 32768^2; step = gw_tick + gw_sync_collect"
                    + (f"; {ws} independent spaces (seed 3 + rank), one per GPU, no collective" if ws > 1 else ""))
    cfg_no = {"c2": 2, "c3": 3, "c3world": 3, "c4": 4, "c5": 5}[kind]
    line = {
        "metric": "entity AOI updates/sec + enter/leave events/sec, 1M-entity space, 1/2/4/8 GPU",
        "value": res["sum_ops"] / mx,
        "unit": "updates/s",
        "n_gpus": ws,
        "ranks": R,
        "steps": K,
        "warmup": W,
        "ms_per_step": mx / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if (ws > 1 and kind in ("c2", "c3")) else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (seeded SplitMix64 traces, SURVEY 8(d) config #{cfg_no})",
        "config": {"workload": workload, "world_entities": n_world, "entities_per_gpu": n_world // R,
                   "movers_per_tick_per_gpu": m_rank, "aoi_dist": 100.0,
                   "world_side": {2: 10240.0, 4: 1024.0, 5: 131072.0}.get(cfg_no, a.side),
                   "gates": a.gates if kind in ("c2", "c3") else 1,
                   "parallelism": parallelism},
        "events_per_sec": res["sum_events"] / mx,
        "records_per_sec": res["sum_records"] / mx,
        "device_us_per_step": (sum(v["avg_us"] for v in res["stages"].values())) if res["stages"] else None,
        "bytes_alg_per_step": res["tot"]["bytes_alg"] / K,
        "step_hbm_frac": (res["tot"]["bytes_alg"] / K) / (mx / K) / (HBM_PEAK_GBS * 1e9),
        "load_s": t_load,
    }
    line.update(roofline_fields(res, K, cfg_no, ws))
    line.update(e2e)
    if e2e:
        line["t_device_ms_per_step"] = mx / K * 1e3
    if client:
        line["client_msgs"] = client
    if loop:
        line["comm"] = "loopback"
    if c3w:
        line["c3world"] = c3w
    if spc:
        line["spaces"] = spc
    if c5:
        line["config5"] = c5
    if not a.no_cpu_baseline and ws == 1 and kind == "c3":
        cb = cpu_baseline(traces.config3(ticks=1, seed=3, n=a.entities, side=a.side), a.cpu_st_max_seconds)
        line["cpu_baseline"] = cb
        line["cpu_baseline_mt"] = cpu_baseline_mt(a.cpu_seconds, a.entities, a.side)
        allowed = cpu_info()["cpus_allowed"] or 1
        if allowed != line["cpu_baseline_mt"]["cores"]:
            # every core the process may use (the cgroup quota, if any, is stated: it may throttle them)
            mt = cpu_baseline_mt(a.cpu_seconds, a.entities, a.side, threads=allowed)
            mt["cgroup_cpu_quota_cores"] = cpu_quota()
            line["cpu_baseline_mt_all_cores"] = mt
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
