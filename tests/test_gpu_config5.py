"""GPU: BASELINE config #5 at its workload — the 16M-entity world (L = 131072,
d = 100, 10 % movers per tick, +-4 on the 1/128 grid, walkers cross strip
borders) decomposed into 8 X-strips equals ONE 16M-entity context, tick by
tick (SURVEY.md §4 item 4, §8(e) regime 2).

The 8 strips are 8 world contexts (gw_world_create) in this process on the
one GPU, halo rows handed over by pointer (gw_world_route -> gw_world_submit,
dworld.LocalWorld); a multi-GPU run moves the same rows over RCCL.  The single
context takes the same ops in the same global order (rank-major, as the world
stamps order them).  Per tick: the union of the strips' owned enter / leave
events equals the single context's, byte for byte after a (watcher, target)
sort; the union of their sync records equals the single context's as a
multiset (count + two independent order-free 64-bit digests: each strip emits
its entities' records in its own grid order).  The single context is in turn
checked against the CPU oracle: oracle/gridmt.c (equal to ORC_SEQRULE on every
oracle test trace) ran the same op stream, and tests/golden/digests.json keeps
its per-tick event SHA-256s and record digests (make_golden.py config5_16m)."""
import numpy as np
import pytest

import golden_data as G
from goworld_amd import dworld, gpuaoi
from goworld_amd import traces as T

pytestmark = pytest.mark.gpu

N, SIDE, R, TICKS = 16_000_000, 131072.0, 8, 3
M1 = np.uint64(0x9E3779B97F4A7C15)
M2 = np.uint64(0xBF58476D1CE4E5B9)


def _mix(z):
    z = z.copy()
    z ^= z >> np.uint64(30)
    z *= M2
    z ^= z >> np.uint64(27)
    z *= np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return z


def rec_digest(recs: np.ndarray):
    """Order-free digest of a record multiset: (count, sum of h1, sum of h2) mod 2^64."""
    w = np.ascontiguousarray(recs).view(np.uint64).reshape(-1, 3)
    with np.errstate(over="ignore"):
        h1 = _mix(w[:, 0] ^ _mix(w[:, 1] + M1) ^ _mix(w[:, 2] * M2 + np.uint64(7)))
        h2 = _mix((w[:, 0] * M1) ^ _mix(w[:, 1] ^ M2) ^ _mix(w[:, 2] + np.uint64(0x632BE59BD9B4E019)))
        return len(recs), int(h1.sum(dtype=np.uint64)), int(h2.sum(dtype=np.uint64))


def _dev_records(g, s):
    out = np.zeros(s.n_rec, gpuaoi.REC_DTYPE)
    if s.n_rec:
        g.d2h(out, s.rec_dev)
    return out


def _dev_events(g, ptr, n):
    out = np.zeros(n, gpuaoi.EVENT_DTYPE)
    if n:
        g.d2h(out, ptr)
    return out


def _key(e):
    return np.sort((e["watcher"].astype(np.uint64) << np.uint64(32)) | e["target"].astype(np.uint64))


def test_config5_16m_world_8_strips_equals_single_context():
    walk = T.WorldWalk(seed=5, n=N, side=SIDE)
    x0, z0, yaw0 = walk.x(), walk.z(), walk.yaw.copy()
    tk = [walk.next_tick() for _ in range(TICKS)]
    lw = dworld.LocalWorld(R, N, SIDE, 4.0, x0, z0, yaw0)
    single = gpuaoi.GpuAOI(0)
    try:
        sid, base = single.create_space(100.0, N, (-SIDE / 2, -SIDE / 2, SIDE / 2, SIDE / 2))
        assert base == 0
        single.restore(sid, np.arange(N, dtype=np.uint32), x0, np.zeros(N, np.float32), z0, yaw0)
        single.set_clients(np.arange(N, dtype=np.uint32), np.ones(N, np.uint16))
        single.sync_collect(copy=False)
        n_ev = n_rec = 0
        oracle = G.digests()["config5_16m"]
        single_out, single_ops = [], []
        for t, (ops, xb) in enumerate(tk):
            parts = lw.split(ops, xb)
            lw.route_submit([lw.upload(r, p) for r, p in enumerate(parts)], [len(p) for p in parts])
            got_e, got_l, got_r = [], [], []
            for g in lw.g:
                res = g.tick(copy=False)
                got_e.append(_dev_events(g, res.enter_dev, res.n_enter))
                got_l.append(_dev_events(g, res.leave_dev, res.n_leave))
                s = g.sync_collect(copy=False)
                g.synchronize()
                got_r.append(rec_digest(_dev_records(g, s)))
            single_ops.append(np.concatenate(parts))
            single.submit(single_ops[-1])                 # the world's stamp order: rank-major
            res = single.tick(copy=False)
            exp_e = _dev_events(single, res.enter_dev, res.n_enter)
            exp_l = _dev_events(single, res.leave_dev, res.n_leave)
            s = single.sync_collect(copy=False)
            single.synchronize()
            exp_r = rec_digest(_dev_records(single, s))
            single_out.append(dict(n_enter=len(exp_e), n_leave=len(exp_l), enter_sha=G.sha(exp_e),
                                   leave_sha=G.sha(exp_l), rec_digest=list(exp_r)))
            for name, got, exp in (("enter", got_e, exp_e), ("leave", got_l, exp_l)):
                g_all = np.concatenate(got)
                assert len(g_all) == len(exp), (t, name, len(g_all), len(exp))
                assert np.array_equal(_key(g_all), _key(exp)), f"tick {t}: {name} events differ"
                n_ev += len(exp)
            cnt = sum(d[0] for d in got_r)
            h1 = sum(d[1] for d in got_r) % (1 << 64)
            h2 = sum(d[2] for d in got_r) % (1 << 64)
            assert (cnt, h1, h2) == exp_r, f"tick {t}: sync records differ"
            n_rec += cnt
        lw.check()
        assert n_ev > TICKS * 3_000_000 and n_rec > TICKS * 50_000_000    # config #5 density
        # the single context against the oracle's run of the same stream
        tr = T.SpaceTrace(n=N, capacity=N, d=100.0, bounds=(-SIDE / 2, -SIDE / 2, SIDE / 2, SIDE / 2),
                          init_slots=np.arange(N, dtype=np.uint32), init_x=x0, init_y=np.zeros(N, np.float32),
                          init_z=z0, init_yaw=yaw0, ticks=single_ops, gates=np.ones(N, np.uint16))
        assert G.trace_input_sha(tr) == oracle["input_sha"], "trace generator changed (not a parity failure)"
        for t, (got, exp) in enumerate(zip(single_out, oracle["ticks"])):
            assert got["n_enter"] == exp["n_enter"] and got["n_leave"] == exp["n_leave"], t
            assert got["enter_sha"] == exp["enter_sha"] and got["leave_sha"] == exp["leave_sha"], f"tick {t}: events"
            assert got["rec_digest"] == exp["rec_digest"], f"tick {t}: records"
    finally:
        single.close()
        lw.close()
