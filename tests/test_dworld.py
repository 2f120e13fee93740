"""Decomposed world (SURVEY.md 8(e) regime 2): the union of what the strip
ranks emit for the entities they own equals, tick by tick, what one global
oracle space emits for the whole world — events and sync records — on a
strip trace with migration across borders, churn, Leave + re-Enter inside a
tick, repeated moves and Sync ops.

CPU tests run the halo protocol over gloo with world_size 2 and 3 and an
oracle space per rank; the GPU test runs the same ranks on the HIP engine
(two processes on the one GPU, gloo between them)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from goworld_amd import dworld, traces as T

import torch_router
from oracle import pyorc

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

TRACE = dict(seed=7, n=800, strip_w=300.0, height=600.0, d=50.0, max_step=8.0, ticks=12)
COLLECT_EVERY = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(world, engine, tmp_path, timeout=240, args=None, collect_every=COLLECT_EVERY):
    port = _free_port()
    procs, outs = [], []
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for r in range(world):
        out = str(tmp_path / f"rank{r}.npz")
        outs.append(out)
        cmd = [sys.executable, os.path.join(HERE, "dworld_worker.py"), "--rank", str(r), "--world", str(world),
               "--port", str(port), "--out", out, "--engine", engine,
               "--collect-every", str(collect_every)]
        for k, v in (TRACE if args is None else args).items():
            cmd += [f"--{k.replace('_', '-')}", str(v)]
        procs.append(subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            logs.append(o.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    bad = [r for r, p in enumerate(procs) if p.returncode != 0]
    # the rank that failed first is usually not rank 0 (the others then lose their peer)
    assert not bad, "\n".join(f"rank {r} failed (rc {procs[r].returncode}):\n{logs[r][-2500:]}" for r in bad)
    return [np.load(o) for o in outs]


def _sort_ev(e):
    return e[np.lexsort((e["target"], e["watcher"]))]


def _sort_rec(r):
    return r[np.lexsort((r["watcher"], r["entity"]))]


TELEPORT = dict(TRACE, teleports=3)


def _check(world, results, trace=TRACE):
    tr = T.strip_world_trace(trace["seed"], trace["n"], world, trace["strip_w"], trace["height"],
                             trace["d"], trace["ticks"], trace["max_step"], teleports=trace.get("teleports", 0),
                             groups=trace.get("groups", 0))
    o = pyorc.OracleSpace(tr.n, tr.d, pyorc.SEQRULE)
    o.set_clients(tr.gates)
    n_ev = n_rec = 0
    for t in range(len(tr.ticks)):
        assert o.tick(tr.global_ops(t)) == 0
        e, l = o.events()
        for name, exp in (("enter", e), ("leave", l)):
            got = np.concatenate([res[f"{name}_{t}"] for res in results])
            assert len(got) == len(exp), (t, name, len(got), len(exp))
            assert _sort_ev(got).tobytes() == _sort_ev(exp).tobytes(), f"tick {t}: {name} events differ"
            n_ev += len(exp)
        if f"rec_{t}" in results[0]:
            exp = o.collect()
            got = np.concatenate([res[f"rec_{t}"] for res in results])
            assert len(got) == len(exp), (t, len(got), len(exp))
            assert _sort_rec(got).tobytes() == _sort_rec(exp).tobytes(), f"tick {t}: records differ"
            n_rec += len(exp)
    assert n_ev > 1000 and n_rec > 1000       # the trace exercises the protocol


def test_strip_geometry():
    g = dworld.Strips(0.0, 300.0, 3, 50.0, 8.0)
    assert g.h > g.d + 2 * g.max_step
    assert g.ext(1) == (300.0 - g.h, 600.0 + g.h)
    assert list(g.owner([-5.0, 0.0, 299.99, 300.0, 900.0])) == [0, 0, 0, 1, 2]
    lo, hi = g.own_range_f32(1)
    assert (lo, hi) == (300.0, 600.0)
    assert g.own_range_f32(0)[0] < -1e38 and g.own_range_f32(2)[1] > 1e38
    with pytest.raises(ValueError):
        dworld.Strips(0.0, 60.0, 3, 50.0, 8.0)      # strips narrower than the halo


def test_strip_trace_migrates():
    tr = T.strip_world_trace(TRACE["seed"], TRACE["n"], 2, TRACE["strip_w"], TRACE["height"],
                             TRACE["d"], TRACE["ticks"], TRACE["max_step"])
    # owners are strips of the start-of-tick positions; entities cross borders
    x = np.zeros(tr.n, np.float32)
    crossings = 0
    for t, (ops, own) in enumerate(tr.ticks):
        for op, r in zip(ops, own):
            if op["kind"] in (T.OP_ENTER, T.OP_MOVED):
                if t and op["kind"] == T.OP_MOVED:
                    crossings += int((x[op["slot"]] >= 300.0) != (op["x"] >= 300.0))
                x[op["slot"]] = op["x"]
    assert crossings > 5


@pytest.mark.parametrize("world", [2, 3])
def test_dworld_gloo_oracle_ranks(world, tmp_path):
    _check(world, _run_ranks(world, "oracle", tmp_path))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_dworld_gpu_ranks(world, tmp_path):
    """The HIP engine per rank (HipRouter + gw_route_halo), ranks sharing the GPU."""
    _check(world, _run_ranks(world, "hip", tmp_path, timeout=100))


def _teleports_cross_two_strips(world):
    tr = T.strip_world_trace(TELEPORT["seed"], TELEPORT["n"], world, TELEPORT["strip_w"], TELEPORT["height"],
                             TELEPORT["d"], TELEPORT["ticks"], TELEPORT["max_step"], teleports=TELEPORT["teleports"])
    far = 0
    for t in range(1, len(tr.ticks)):
        ops, own = tr.ticks[t]
        dst = np.clip(np.floor(ops["x"] / tr.strip_w).astype(np.int64), 0, world - 1)
        far += int(np.sum((ops["kind"] == T.OP_MOVED) & (np.abs(dst - own) >= 2)))
    return far


@pytest.mark.parametrize("world", [2, 3, 4])
def test_dworld_gloo_oracle_teleports(world, tmp_path):
    """Long moves (Entity.SetPosition has no step bound, Entity.go:1185-1187):
    entities jump anywhere, across two or more strips, every tick; their rows
    reach every rank holding either end, their pairs are emitted by the other
    member's owner, and the union still equals one global oracle space."""
    assert world == 2 or _teleports_cross_two_strips(world) >= 5
    _check(world, _run_ranks(world, "oracle", tmp_path, args=TELEPORT), trace=TELEPORT)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_dworld_gpu_teleports(world, tmp_path):
    """The same with the HIP engine per rank (gw_world_route / gw_world_far /
    gw_world_submit_far over gloo), ranks sharing the GPU."""
    _check(world, _run_ranks(world, "hip", tmp_path, timeout=100, args=TELEPORT), trace=TELEPORT)


GROUPS = dict(TRACE, teleports=2, groups=6)


def _long_pairs(world, trace):
    """Pairs of entities that both jump (long moves) in one tick and are related
    before or after it (by the oracle's relation), over the trace."""
    tr = T.strip_world_trace(trace["seed"], trace["n"], world, trace["strip_w"], trace["height"], trace["d"],
                             trace["ticks"], trace["max_step"], teleports=trace["teleports"], groups=trace["groups"])
    o = pyorc.OracleSpace(tr.n, tr.d, pyorc.SEQRULE)
    x = np.zeros(tr.n, np.float32)
    pres = np.zeros(tr.n, bool)
    both = 0
    for t in range(len(tr.ticks)):
        ops = tr.global_ops(t)
        before = {s: set(o.neighbors(s).tolist()) for s in range(tr.n) if pres[s]}
        mv = ops[(ops["kind"] == T.OP_MOVED)]
        far = set(int(op["slot"]) for op in mv if pres[op["slot"]] and abs(float(op["x"]) - float(x[op["slot"]])) >
                  tr.max_step)
        assert o.tick(ops) == 0
        for op in ops:
            if op["kind"] in (T.OP_ENTER, T.OP_MOVED):
                x[op["slot"]], pres[op["slot"]] = op["x"], True
            elif op["kind"] == T.OP_LEAVE:
                pres[op["slot"]] = False
        for a in far:
            after = set(o.neighbors(a).tolist())
            both += len((before.get(a, set()) | after) & far)
    o.close()
    return both // 2


@pytest.mark.parametrize("world", [2, 3, 4])
def test_dworld_gloo_oracle_group_teleports(world, tmp_path):
    """Group teleports (related entities jumping in one tick: together,
    apart, or next to each other) across strips: the long-mover lists carry
    every long mover's state before and after the tick to every rank, and
    the union of the ranks' outputs still equals one global oracle space."""
    assert _long_pairs(world, GROUPS) >= 20            # the trace has related long-mover pairs
    _check(world, _run_ranks(world, "oracle", tmp_path, args=GROUPS), trace=GROUPS)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_dworld_gpu_group_teleports(world, tmp_path):
    """The same with the HIP engine per rank (gw_world_route / gw_world_far /
    gw_world_longs / gw_world_submit_longs over gloo), ranks sharing the GPU."""
    _check(world, _run_ranks(world, "hip", tmp_path, timeout=100, args=GROUPS), trace=GROUPS)


WALK_SMALL = dict(trace="walk", seed=9, n=20000, side=6144.0, ticks=5)


@pytest.mark.parametrize("world", [2, 3])
def test_dworld_gloo_oracle_walk(world, tmp_path):
    """Config #5 shape at test scale: a uniform walk whose entities cross strip
    borders every tick; the union of the ranks' outputs equals one global
    oracle space (dyadic positions: the windows are symmetric)."""
    res = _run_ranks(world, "oracle", tmp_path, args=WALK_SMALL, collect_every=1)
    tr = T.walk_strip_trace(WALK_SMALL["seed"], WALK_SMALL["n"], WALK_SMALL["side"], world, WALK_SMALL["ticks"])
    o = pyorc.OracleSpace(tr.n, tr.d, pyorc.SEQRULE)
    o.set_clients(tr.gates)
    assert o.tick(tr.global_ops(0)) == 0
    o.collect()
    n_ev = 0
    for t in range(1, len(tr.ticks)):
        assert o.tick(tr.global_ops(t)) == 0
        e, l = o.events()
        for name, exp in (("enter", e), ("leave", l)):
            got = np.concatenate([r[f"{name}_{t}"] for r in res])
            assert _sort_ev(got).tobytes() == _sort_ev(exp).tobytes(), f"tick {t}: {name} events differ"
            n_ev += len(exp)
        exp = o.collect()
        got = np.concatenate([r[f"rec_{t}"] for r in res])
        assert _sort_rec(got).tobytes() == _sort_rec(exp).tobytes(), f"tick {t}: records differ"
    assert n_ev > 1000


@pytest.mark.gpu
def test_dworld_gpu_walk_1m_equals_single_context(tmp_path):
    """SURVEY 4 item 4 at config #5 density: a 1M-entity world decomposed into
    3 strips (3 HIP-engine processes on the one GPU, rows over gloo through
    the library's gw_world_route / gw_world_submit) equals a single-context
    HIP run of the same world, tick by tick: the union of the ranks' owned
    events and records (entities migrate across borders every tick)."""
    from goworld_amd import gpuaoi
    args = dict(trace="walk", seed=11, n=1_000_000, side=32768.0, ticks=4)
    res = _run_ranks(3, "hip", tmp_path, timeout=110, args=args, collect_every=1)
    tr = T.walk_strip_trace(args["seed"], args["n"], args["side"], 3, args["ticks"])
    with gpuaoi.GpuAOI(0) as g:
        sid, base = g.create_space(tr.d, tr.n, tr.bounds)
        g.set_clients(np.arange(tr.n, dtype=np.uint32), tr.gates)
        g.submit(tr.global_ops(0))
        g.tick(copy=False, no_events=True)
        g.sync_collect(copy=False)
        n_ev = n_rec = 0
        for t in range(1, len(tr.ticks)):
            g.submit(tr.global_ops(t))
            r = g.tick()
            for name, exp in (("enter", r.enter), ("leave", r.leave)):
                got = np.concatenate([x[f"{name}_{t}"] for x in res])
                assert len(got) == len(exp), (t, name, len(got), len(exp))
                assert _sort_ev(got).tobytes() == _sort_ev(exp).tobytes(), f"tick {t}: {name} events differ"
                n_ev += len(exp)
            exp = g.sync_collect().records
            got = np.concatenate([x[f"rec_{t}"] for x in res])
            assert len(got) == len(exp), (t, len(got), len(exp))
            assert _sort_rec(got).tobytes() == _sort_rec(exp).tobytes(), f"tick {t}: records differ"
            n_rec += len(exp)
    assert n_ev > 100_000 and n_rec > 1_000_000


@pytest.mark.gpu
def test_rccl_self_exchange_and_allreduce():
    """The library's RCCL communicator on the one GPU (a 1-rank communicator):
    a grouped send/recv to itself moves the bytes, the all-reduce of one rank
    is the identity, and a one-strip world ticked by gw_world_step (its RCCL
    path with no neighbours) equals the plain space."""
    import torch
    from goworld_amd import gpuaoi
    with gpuaoi.GpuAOI(0) as g:
        g.comm_init(gpuaoi.comm_unique_id(), 1, 0)
        assert g.comm_info() == (1, 0)
        src = np.arange(1 << 16, dtype=np.uint32)
        a, b = g.dev_alloc(src.nbytes), g.dev_alloc(src.nbytes)
        g.h2d(a, src)
        g.comm_exchange([(0, a, src.nbytes, b, src.nbytes)])
        back = np.zeros_like(src)
        g.d2h(back, b)
        assert np.array_equal(back, src)
        v = np.array([5, 7, 1 << 40], np.uint64)
        g.h2d(a, v)
        g.comm_allreduce_u64(a, 3, gpuaoi.RED_MAX)
        g.synchronize()
        w = np.zeros(3, np.uint64)
        g.d2h(w, a)
        assert np.array_equal(w, v)
        g.dev_free(a)
        g.dev_free(b)
    tr = T.walk_strip_trace(13, 30000, 8192.0, 1, 4)
    outs = []
    for path in ("world", "plain"):
        with gpuaoi.GpuAOI(0) as g:
            if path == "world":
                g.comm_init(gpuaoi.comm_unique_id(), 1, 0)
                g.world_create(0.0, 8192.0, tr.d, tr.max_step, 1, 0, tr.n, tr.bounds)
            else:
                g.create_space(tr.d, tr.n, tr.bounds)
            g.set_clients(np.arange(tr.n, dtype=np.uint32), tr.gates)
            seq = []
            for t in range(len(tr.ticks)):
                ops = tr.global_ops(t)
                if path == "world":
                    dev = torch.from_numpy(ops.view(np.uint8).copy()).to("cuda:0")
                    torch.cuda.synchronize()               # the copy ran on torch's stream
                    g.world_step(dev.data_ptr(), len(ops))
                    r = g.tick()
                    del dev
                else:
                    g.submit(ops)
                    r = g.tick()
                seq.append((r.enter.tobytes(), r.leave.tobytes(), g.sync_collect().records.tobytes()))
            outs.append(seq)
    assert outs[0] == outs[1]


@pytest.mark.gpu
def test_world_step_host_ops():
    """gw_world_step_host (the Go caller's host ops, staged by the library):
    a one-strip world fed host ops equals the plain space, tick by tick; the
    host checks reject a bad kind / an id outside the world / non-finite
    coordinates before anything is queued, and a second stage before the tick
    is refused.  Then a 2-strip world on the one GPU (two contexts, rows handed
    over by pointer) driven by gw_world_stage_ops + gw_world_route equals the
    plain space's events and records."""
    from goworld_amd import gpuaoi
    tr = T.walk_strip_trace(17, 20000, 8192.0, 1, 4)
    outs = []
    for path in ("world", "plain"):
        with gpuaoi.GpuAOI(0) as g:
            if path == "world":
                g.world_create(0.0, 8192.0, tr.d, tr.max_step, 1, 0, tr.n, tr.bounds)
            else:
                g.create_space(tr.d, tr.n, tr.bounds)
            g.set_clients(np.arange(tr.n, dtype=np.uint32), tr.gates)
            seq = []
            for t in range(len(tr.ticks)):
                ops = tr.global_ops(t)
                if path == "world":
                    bad = ops[:4].copy()
                    bad["slot"][2] = tr.n
                    with pytest.raises(gpuaoi.GwError):
                        g.world_step_host(bad)
                    bad = ops[:4].copy()
                    bad["kind"][1] = 9
                    with pytest.raises(gpuaoi.GwError):
                        g.world_step_host(bad)
                    if len(ops) and ops["kind"][0] in (T.OP_ENTER, T.OP_MOVED):
                        bad = ops[:1].copy()
                        bad["x"][0] = np.inf
                        with pytest.raises(gpuaoi.GwError):
                            g.world_step_host(bad)
                    g.world_step_host(ops)
                    with pytest.raises(gpuaoi.GwError):
                        g.world_stage_ops(ops[:1])             # the queued tick still reads the staged ops
                else:
                    g.submit(ops)
                r = g.tick()
                seq.append((r.enter.tobytes(), r.leave.tobytes(), g.sync_collect().records.tobytes()))
            outs.append(seq)
    assert outs[0] == outs[1]
    # two strips on the one GPU, host ops staged per rank
    tr2 = T.walk_strip_trace(19, 20000, 8192.0, 2, 4)
    geom = dworld.Strips(0.0, tr2.strip_w, 2, tr2.d, tr2.max_step)
    gs = [gpuaoi.GpuAOI(0) for _ in range(2)]
    try:
        for r, g in enumerate(gs):
            lo, hi = geom.ext(r)
            g.world_create(geom.x0, geom.w, geom.d, geom.max_step, 2, r, tr2.n,
                           (max(lo, tr2.bounds[0]), tr2.bounds[1], min(hi, tr2.bounds[2]), tr2.bounds[3]))
            g.set_clients(np.arange(tr2.n, dtype=np.uint32), tr2.gates)
        with gpuaoi.GpuAOI(0) as ref:
            ref.create_space(tr2.d, tr2.n, tr2.bounds)
            ref.set_clients(np.arange(tr2.n, dtype=np.uint32), tr2.gates)
            for t in range(len(tr2.ticks)):
                sends = []
                for r, g in enumerate(gs):
                    dev = g.world_stage_ops(tr2.rank_ops(t, r))
                    sends.append(g.world_route(dev, len(tr2.rank_ops(t, r))))
                gs[0].world_submit([(0, 0), sends[1][0]])
                gs[1].world_submit([sends[0][1], (0, 0)])
                res = [g.tick() for g in gs]
                ref.submit(tr2.global_ops(t))
                e = ref.tick()
                if t == 0:
                    for g in gs:
                        g.sync_collect()
                    ref.sync_collect()
                    continue
                for name, exp in (("enter", e.enter), ("leave", e.leave)):
                    got = np.concatenate([getattr(x, name) for x in res])
                    assert _sort_ev(got).tobytes() == _sort_ev(exp).tobytes(), f"tick {t}: {name} events differ"
                got = np.concatenate([g.sync_collect().records for g in gs])
                assert _sort_rec(got).tobytes() == _sort_rec(ref.sync_collect().records).tobytes()
    finally:
        for g in gs:
            g.close()


def _canon_rows(buf):
    rows = buf.reshape(-1, 3, 8).cpu().numpy()
    used = rows[np.any(rows[:, :, 0] & 0xFF, axis=1)]
    assert len(used) == len(rows), "exact-size rows must not carry NOP padding"
    slot = used[:, :, 1].max(axis=1)
    return used[np.argsort(slot, kind="stable")]


@pytest.mark.gpu
def test_hip_router_rows_match_torch_router():
    """gw_world_route (gw_route_halo rows, exact size) writes, per neighbour,
    the same entity rows as the torch statement of the protocol
    (tests/torch_router.py), tick by tick, for the middle rank of a 3-strip
    world (order of entities aside)."""
    import torch
    from goworld_amd import gpuaoi
    tr = T.strip_world_trace(TRACE["seed"], TRACE["n"], 3, TRACE["strip_w"], TRACE["height"],
                             TRACE["d"], TRACE["ticks"], TRACE["max_step"])
    geom = dworld.Strips(0.0, tr.strip_w, 3, tr.d, tr.max_step)
    dev = torch.device("cuda:0")
    with gpuaoi.GpuAOI(0) as g:
        eng = dworld.HipStrip(g)
        eng.create_world(geom, 1, tr.n, tr.bounds)
        ref = torch_router.Router(geom, 1, tr.n, dev, tr.n)
        n_rows = n_long = 0
        for t in range(len(tr.ticks)):
            w = torch.from_numpy(dworld.ops_to_words(tr.rank_ops(t, 1)).copy()).to(dev)
            st = dworld.stamps_for(t, 1, 3, w.shape[0], dev)
            for side, (a, b) in enumerate(zip(eng.route(w, st), ref.route_exact(w, st))):
                ca, cb = _canon_rows(a), _canon_rows(b)
                assert ca.shape == cb.shape, (t, side, ca.shape, cb.shape)
                assert ca.tobytes() == cb.tobytes(), f"tick {t} side {side}: halo rows differ"
                n_rows += len(ca)
            # the long-mover list (group teleports) equals the torch statement's
            la, lb = eng.longs(), ref.longs_exact()
            assert np.array_equal(np.sort(la, order="slot"), np.sort(lb, order="slot")), f"tick {t}: long lists"
            n_long += len(la)
            eng.submit(w, st, [None, None])
            eng.tick(copy=False)
            if t % 3 == 2:
                eng.collect(copy=False)
                ref.collected()
        assert n_rows > 300
        # no overflow; the same long moves (entities that come back after ticks
        # owned elsewhere, whose ghost rows this lone rank never got)
        ov, n_long_moves, bad = eng.g.halo_status()
        assert ov == 0 and bad == 0 and n_long_moves == ref.long_count() > 0 and n_long > 0
        # invalid slots are counted, never followed
        bad = w.clone()
        bad[:, 1] = tr.n + 5
        eng.route(bad)
        assert eng.status()[2] == bad.shape[0]
        torch.cuda.synchronize()
