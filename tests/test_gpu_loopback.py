"""GPU: the decomposed world's multi-rank call sequence inside the library
(gw_world_step: route, count round, host read of the counts, far-count
all-gather at >= 3 ranks, far settle, exact-size neighbour rows and far rows,
queue) run by R ranks on the one MI355X over the loopback transport
(gw_comm_init_local): R contexts of this process, each driven by its own host
thread as a rank process drives its own, collectives as copies between the
contexts with RCCL's matching semantics (goworld_amd/csrc/xport.cpp).

* the transport alone: a ring exchange and the u64 all-reduce of 3 ranks;
* 3 and 4 strips of the teleport strip trace (long moves across two or more
  strips every tick: the far all-gather and far rows run every tick) against
  one global oracle space (test_dworld._check: events per tick, records per
  collect);
* the 1M-entity walk world at 8 strips (config #5 density, walkers cross
  borders every tick) through gw_step (world step + deferred tick + collect in
  one call, as bench.py's world legs run it) against ONE context fed the same
  ops in the world's stamp order."""
import os

import numpy as np
import pytest

from goworld_amd import dworld, gpuaoi
from goworld_amd import traces as T

from test_dworld import GROUPS, TELEPORT, _check, _sort_ev, _sort_rec

pytestmark = pytest.mark.gpu

os.environ.setdefault("GW_LOOPBACK_TIMEOUT_S", "30")   # a failing rank must not hang its peers past the test limit


def test_loopback_ring_exchange_and_allreduce():
    R = 3
    gs = [gpuaoi.GpuAOI(0) for _ in range(R)]
    try:
        gpuaoi.comm_init_local(gs)
        assert [g.comm_info() for g in gs] == [(R, r) for r in range(R)]
        n = 1 << 14
        src, dst = [], []
        for r, g in enumerate(gs):
            a, b = g.dev_alloc(4 * n), g.dev_alloc(4 * n)
            g.h2d(a, (np.arange(n, dtype=np.uint32) * 7 + r).astype(np.uint32))
            src.append(a)
            dst.append(b)
        w = LoopbackRuns(gs)
        # ring: rank r sends to r+1 and receives from r-1 in one group
        w.run(lambda r, g: g.comm_exchange([((r + 1) % R, src[r], 4 * n, 0, 0), ((r - 1) % R, 0, 0, dst[r], 4 * n)]))
        for r, g in enumerate(gs):
            back = np.zeros(n, np.uint32)
            g.d2h(back, dst[r])
            assert np.array_equal(back, np.arange(n, dtype=np.uint32) * 7 + (r - 1) % R)
        for op, fold in ((gpuaoi.RED_SUM, sum), (gpuaoi.RED_MAX, max)):
            vals = [np.array([r + 1, 10 * (R - r), 1 << (40 + r)], np.uint64) for r in range(R)]
            for r, g in enumerate(gs):
                g.h2d(src[r], vals[r])
            w.run(lambda r, g: (g.comm_allreduce_u64(src[r], 3, op), g.synchronize()))
            exp = np.array([fold(int(v[i]) for v in vals) for i in range(3)], np.uint64)
            for r, g in enumerate(gs):
                got = np.zeros(3, np.uint64)
                g.d2h(got, src[r])
                assert np.array_equal(got, exp), (op, r, got, exp)
        # a count mismatch is an error on both sides, not a hang or a silent short copy
        with pytest.raises(gpuaoi.GwError):
            w.run(lambda r, g: g.comm_exchange([((r + 1) % R, src[r], 4 * n if r else 8, 0, 0),
                                                ((r - 1) % R, 0, 0, dst[r], 4 * n)]))
        w.close()
    finally:
        for g in gs:
            g.close()


class LoopbackRuns:
    """Persistent rank threads over existing contexts (the transport test)."""

    def __init__(self, gs):
        self.g = gs
        self.th = [dworld._RankThread(r) for r in range(len(gs))]

    run = dworld.LoopbackWorld.run

    def close(self):
        for th in self.th:
            th.stop()


@pytest.mark.parametrize("world,trace", [(3, "teleports"), (4, "teleports"), (2, "groups"), (3, "groups"),
                                         (4, "groups")])
def test_loopback_world_teleports_vs_oracle(world, trace):
    """Strip trace with churn, Leave + re-Enter inside a tick, Sync ops and long
    moves per tick across two or more strips (groups: related entities jumping
    together, apart or next to each other, whose pairs come from the long-mover
    lists), through gw_world_step on every rank thread; the union of the
    ranks' owned events and records equals one global oracle space."""
    TR = TELEPORT if trace == "teleports" else GROUPS
    tr = T.strip_world_trace(TR["seed"], TR["n"], world, TR["strip_w"], TR["height"], TR["d"], TR["ticks"],
                             TR["max_step"], teleports=TR["teleports"], groups=TR.get("groups", 0))
    geom = dworld.Strips(0.0, tr.strip_w, world, tr.d, tr.max_step)
    lw = dworld.LoopbackWorld(geom, tr.n, tr.bounds, gates=tr.gates)
    try:
        ptrs = [[lw.upload(r, tr.rank_ops(t, r)) for r in range(world)] for t in range(len(tr.ticks))]
        collect_every = 3

        def rank(r, g):
            out = {"far": 0}
            for t in range(len(tr.ticks)):
                g.world_step(ptrs[t][r], len(tr.rank_ops(t, r)))
                out["far"] += sum(rows for q, (_, rows) in g.world_far().items() if q != r)   # rows sent far
                res = g.tick()
                out[f"enter_{t}"], out[f"leave_{t}"] = res.enter, res.leave
                if (t + 1) % collect_every == 0 or t == len(tr.ticks) - 1:
                    out[f"rec_{t}"] = g.sync_collect().records
            return out
        results = lw.run(rank)
        lw.check()
    finally:
        lw.close()
    far = sum(x.pop("far") for x in results)
    assert world < 3 or far > 0                            # the far round moved rows
    _check(world, results, trace=TR)


def test_loopback_world_1m_8_strips_equals_single_context():
    """The 1M-entity walk world over 8 strips through gw_step (the bench's
    world step) equals one context, tick by tick: union of the owned events
    byte for byte after a (watcher, target) sort, union of the records as a
    sorted multiset."""
    R, n, side, ticks = 8, 1_000_000, 32768.0, 4
    tr = T.walk_strip_trace(11, n, side, R, ticks)
    geom = dworld.Strips(0.0, tr.strip_w, R, tr.d, tr.max_step)
    lw = dworld.LoopbackWorld(geom, tr.n, tr.bounds, gates=tr.gates)
    try:
        ptrs = [[lw.upload(r, tr.rank_ops(t, r)) for r in range(R)] for t in range(ticks)]

        def rank(r, g):
            out = []
            for t in range(ticks):
                if t == 0:                                 # the load: no events, records discarded
                    g.world_step(ptrs[t][r], len(tr.rank_ops(t, r)))
                    g.tick(copy=False, no_events=True)
                    g.sync_collect(copy=False)
                    continue
                tres, sres = g.step_device(ptrs[t][r], len(tr.rank_ops(t, r)))
                e = np.zeros(tres.n_enter, np.uint64)
                l_ = np.zeros(tres.n_leave, np.uint64)
                if len(e):
                    g.d2h(e, tres.enter_dev)
                if len(l_):
                    g.d2h(l_, tres.leave_dev)
                rec = np.zeros(sres.n_rec * 6, np.uint32)
                if len(rec):
                    g.d2h(rec, sres.rec_dev)
                out.append((e, l_, rec))
            return out
        results = lw.run(rank)
        lw.check()
    finally:
        lw.close()
    n_ev = n_rec = 0
    with gpuaoi.GpuAOI(0) as g:
        g.create_space(tr.d, tr.n, tr.bounds)
        g.set_clients(np.arange(tr.n, dtype=np.uint32), tr.gates)
        g.submit(tr.global_ops(0))
        g.tick(copy=False, no_events=True)
        g.sync_collect(copy=False)
        for t in range(1, ticks):
            g.submit(tr.global_ops(t))
            r = g.tick()
            for k, (name, exp) in enumerate((("enter", r.enter), ("leave", r.leave))):
                got = np.concatenate([x[t - 1][k] for x in results]).view(exp.dtype)
                assert len(got) == len(exp), (t, name, len(got), len(exp))
                assert _sort_ev(got).tobytes() == _sort_ev(exp).tobytes(), f"tick {t}: {name} events differ"
                n_ev += len(exp)
            exp = g.sync_collect().records
            got = np.concatenate([x[t - 1][2] for x in results]).view(exp.dtype)
            assert len(got) == len(exp), (t, len(got), len(exp))
            assert _sort_rec(got).tobytes() == _sort_rec(exp).tobytes(), f"tick {t}: records differ"
            n_rec += len(exp)
    assert n_ev > 100_000 and n_rec > 1_000_000


def test_world_missing_long_lists_are_reported_as_conflicts():
    """Group teleports need every rank's long-mover list (gw_world_submit_longs):
    a long mover's pairs with the other long movers are emitted only from the
    lists.  Two strip contexts driven by pointer (gw_world_route -> world_far ->
    world_longs -> gw_world_submit / submit_far / submit_longs, as a caller's
    own transport would); rank 1 never gets the lists, so the pairs of the long
    movers landing in its strip are lost, and gw_world_status must say so
    (conflicts > 0 there, 0 on rank 0, which got them)."""
    from goworld_amd.traces import LONG_DTYPE
    R, TR, skip = 2, GROUPS, 1
    tr = T.strip_world_trace(TR["seed"], TR["n"], R, TR["strip_w"], TR["height"], TR["d"], TR["ticks"],
                             TR["max_step"], teleports=TR["teleports"], groups=TR["groups"])
    geom = dworld.Strips(0.0, tr.strip_w, R, tr.d, tr.max_step)
    gs, bufs = [], []
    try:
        for r in range(R):
            g = gpuaoi.GpuAOI(0)
            gs.append(g)
            lo, hi = geom.ext(r)
            b = (max(lo, tr.bounds[0]), tr.bounds[1], min(hi, tr.bounds[2]), tr.bounds[3])
            g.world_create(geom.x0, geom.w, geom.d, geom.max_step, R, r, tr.n, b)
            g.set_clients(np.arange(tr.n, dtype=np.uint32), tr.gates)
        conflicts = [0] * R
        n_long = 0
        for t in range(len(tr.ticks)):
            ptrs = []
            for r, g in enumerate(gs):
                ops = np.ascontiguousarray(tr.rank_ops(t, r))
                p = g.dev_alloc(max(ops.nbytes, 64))
                bufs.append((g, p))
                if len(ops):
                    g.h2d(p, ops)
                ptrs.append((p, len(ops)))
            sends = []
            for g, (p, m) in zip(gs, ptrs):
                g.synchronize()
                sends.append(g.world_route(p, m))
            fars = [g.world_far() for g in gs]
            parts = []
            for g in gs:
                lp, ln_ = g.world_longs()
                if ln_:
                    a = np.zeros(ln_, LONG_DTYPE)
                    g.d2h(a, lp)
                    parts.append(a)
            longs = np.concatenate(parts) if parts else np.zeros(0, LONG_DTYPE)
            n_long += len(longs)
            lptr = 0
            if len(longs):
                lptr = gs[0].dev_alloc(longs.nbytes)
                bufs.append((gs[0], lptr))
                gs[0].h2d(lptr, longs)
            for r, g in enumerate(gs):
                left = sends[r - 1][1] if r > 0 else (0, 0)
                right = sends[r + 1][0] if r + 1 < R else (0, 0)
                g.world_submit([left, right])
                for q in range(R):
                    if r in fars[q]:
                        g.world_submit_far(*fars[q][r])
                if len(longs) and r != skip:
                    g.world_submit_longs(lptr, len(longs))
            for g in gs:
                g.tick(copy=False)
                g.sync_collect(copy=False)
            for r, g in enumerate(gs):
                conflicts[r] += g.world_status()[1]        # local counters (no communicator)
    finally:
        for g, p in bufs:
            g.synchronize()
            g.dev_free(p)
        for g in gs:
            g.close()
    assert n_long > 0
    assert conflicts[skip] > 0 and conflicts[1 - skip] == 0, conflicts
