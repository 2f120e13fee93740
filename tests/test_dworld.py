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


def _run_ranks(world, engine, tmp_path, timeout=240):
    port = _free_port()
    procs, outs = [], []
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for r in range(world):
        out = str(tmp_path / f"rank{r}.npz")
        outs.append(out)
        cmd = [sys.executable, os.path.join(HERE, "dworld_worker.py"), "--rank", str(r), "--world", str(world),
               "--port", str(port), "--out", out, "--engine", engine,
               "--collect-every", str(COLLECT_EVERY)]
        for k, v in TRACE.items():
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
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-3000:]}"
    return [np.load(o) for o in outs]


def _sort_ev(e):
    return e[np.lexsort((e["target"], e["watcher"]))]


def _sort_rec(r):
    return r[np.lexsort((r["watcher"], r["entity"]))]


def _check(world, results):
    tr = T.strip_world_trace(TRACE["seed"], TRACE["n"], world, TRACE["strip_w"], TRACE["height"],
                             TRACE["d"], TRACE["ticks"], TRACE["max_step"])
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


def _canon_rows(buf, K):
    rows = buf.view(K, 3, 8).cpu().numpy()
    used = rows[np.any(rows[:, :, 0] & 0xFF, axis=1)]
    slot = used[:, :, 1].max(axis=1)
    return used[np.argsort(slot, kind="stable")]


@pytest.mark.gpu
def test_hip_router_rows_match_torch_router():
    """gw_route_halo (halo.hip) writes, per neighbour, the same entity rows
    as the torch statement of the protocol (tests/torch_router.py), tick by tick, for
    the middle rank of a 3-strip world (order of entities aside)."""
    import torch
    from goworld_amd import gpuaoi
    tr = T.strip_world_trace(TRACE["seed"], TRACE["n"], 3, TRACE["strip_w"], TRACE["height"],
                             TRACE["d"], TRACE["ticks"], TRACE["max_step"])
    geom = dworld.Strips(0.0, tr.strip_w, 3, tr.d, tr.max_step)
    dev = torch.device("cuda:0")
    K = 512
    with gpuaoi.GpuAOI(0) as g:
        eng = dworld.HipStrip(g)
        eng.create_space(tr.d, tr.n, tr.bounds)
        hip = eng.make_router(geom, 1, tr.n, dev, K)
        ref = torch_router.Router(geom, 1, tr.n, dev, K)
        n_rows = 0
        for t in range(len(tr.ticks)):
            w = torch.from_numpy(dworld.ops_to_words(tr.rank_ops(t, 1)).copy()).to(dev)
            st = dworld.stamps_for(t, 1, 3, w.shape[0], dev)
            for side, (a, b) in enumerate(zip(hip.route(w, st), ref.route(w, st))):
                ca, cb = _canon_rows(a, K), _canon_rows(b, K)
                assert ca.shape == cb.shape, (t, side, ca.shape, cb.shape)
                assert ca.tobytes() == cb.tobytes(), f"tick {t} side {side}: halo rows differ"
                n_rows += len(ca)
            eng.submit(w, st)
            eng.tick(copy=False)
            if t % 3 == 2:
                eng.collect(copy=False)
                ref.collected()
        assert n_rows > 300
        # no overflow; the same move-bound violations (entities that come back
        # after ticks owned elsewhere, whose ghost rows this lone rank never got)
        assert hip.status() == ref.status()
        # invalid slots are counted, never followed
        bad = w.clone()
        bad[:, 1] = tr.n + 5
        hip.route(bad, st)
        assert hip.status()[2] == bad.shape[0]
        torch.cuda.synchronize()
