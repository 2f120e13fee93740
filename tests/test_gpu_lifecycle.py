"""GPU: the space lifecycle through the C ABI.

The reference creates and destroys spaces at run time (goworld.go:52-60
CreateSpaceLocally / CreateSpaceAnywhere; SpaceManager.putSpace / delSpace,
engine/entity/SpaceManager.go:21-27; Space.OnDestroy destroys its entities
first, Space.go:143-151) and a space takes any number of entities
(Space.enter, Space.go:179-217).  Here:

* gw_space_grow past the initial capacity mid-trace — the space's state moves
  to a new slot range (another space sits behind it) and every later tick
  stays bit-exact against the oracle (XZList restatement), for the grown space
  and for its neighbour in slot order;
* 1,000 create / load / tick / leave / destroy cycles keep the slot and cell
  ranges bounded (ranges and space ids are reused), and a long-lived space
  ticks correctly throughout;
* destroying a space that still holds an entity is refused, also after
  device-resident submits (the check runs on the device)."""
import numpy as np
import pytest

import golden_data as G
from goworld_amd import gpuaoi
from goworld_amd import traces as T
from oracle import pyorc

pytestmark = pytest.mark.gpu


def _canon(recs, gates):
    return G.canonical_records(recs, gates)


def _local(ev, base):
    out = ev.copy()
    out["watcher"] -= base
    out["target"] -= base
    return out


def _check_tick(g_res, o, base, lo, hi, what):
    """Events of slots [lo, hi) of the GPU result (global) == the oracle's (local)."""
    e, l = o.events()
    for name, got, exp in (("enter", g_res.enter, e), ("leave", g_res.leave, l)):
        mine = got[(got["watcher"] >= lo) & (got["watcher"] < hi)]
        assert _local(mine, base).tobytes() == exp.tobytes(), f"{what}: {name} events"


def _check_records(recs, o, base, lo, hi, gates, what):
    mine = recs[(recs["entity"] >= lo) & (recs["entity"] < hi)].copy()
    mine["watcher"] -= base
    mine["entity"] -= base
    assert _canon(mine, gates).tobytes() == _canon(o.collect(), gates).tobytes(), f"{what}: records"


def test_grow_moves_space_mid_trace_bit_exact():
    n, n0, t_grow = 600, 400, 3
    tr = T.dyadic_walk_trace(51, n, 1024.0, 100.0, 8, move_frac=0.3, hot_frac=0.3, n_hot=3, gate_count=2,
                             client_frac=0.8)
    tb = T.dyadic_walk_trace(52, 50, 512.0, 100.0, 8, move_frac=0.4, gate_count=1, client_frac=1.0)
    oa = pyorc.OracleSpace(n, tr.d, pyorc.XZLIST)
    ob = pyorc.OracleSpace(tb.capacity, tb.d, pyorc.XZLIST)
    g = gpuaoi.GpuAOI(0)
    try:
        sa, base = g.create_space(tr.d, n0, tr.bounds)
        sb, base_b = g.create_space(tb.d, tb.capacity, tb.bounds)      # right behind A
        assert base_b == base + n0
        first = np.arange(n0, dtype=np.uint32)
        g.restore(sa, first + base, tr.init_x[:n0], tr.init_y[:n0], tr.init_z[:n0], tr.init_yaw[:n0])
        oa.bulk_enter(first, tr.init_x[:n0], tr.init_y[:n0], tr.init_z[:n0], tr.init_yaw[:n0])
        for s in range(n0):
            if tr.gates[s]:
                oa.set_client(s, int(tr.gates[s]))
        g.set_clients(first + base, tr.gates[:n0])
        g.restore(sb, np.arange(tb.capacity, dtype=np.uint32) + base_b, tb.init_x, tb.init_y, tb.init_z,
                  tb.init_yaw)
        g.set_clients(np.arange(tb.capacity, dtype=np.uint32) + base_b, tb.gates)
        pyorc.load_trace(ob, tb)
        g.sync_collect()
        oa.collect()
        ob.collect()
        cx, cz, cyaw = tr.init_x.copy(), tr.init_z.copy(), tr.init_yaw.copy()
        for t in range(len(tr.ticks)):
            ops = tr.ticks[t]
            if t < t_grow:
                ops = ops[ops["slot"] < n0]
            elif t == t_grow:
                nb = g.grow_space(sa, n)
                assert nb != base and nb >= base_b + tb.capacity     # moved past B
                info = g.context_info()
                assert info["live_slots"] == n + tb.capacity and info["live_spaces"] == 2
                base = nb
                late = np.arange(n0, n, dtype=np.uint32)
                g.set_clients(late + base, tr.gates[n0:])
                for s in late:
                    if tr.gates[s]:
                        oa.set_client(int(s), int(tr.gates[s]))
                ops = np.concatenate([T.enter_ops(late, cx[late], np.zeros(len(late), np.float32), cz[late],
                                                  cyaw[late]), ops])
            cx[tr.ticks[t]["slot"]] = tr.ticks[t]["x"]
            cz[tr.ticks[t]["slot"]] = tr.ticks[t]["z"]
            cyaw[tr.ticks[t]["slot"]] = tr.ticks[t]["yaw"]
            ga = T.with_global_slots(ops, base)
            gb = T.with_global_slots(tb.ticks[t], base_b)
            g.submit(np.concatenate([gb, ga]) if t % 2 else np.concatenate([ga, gb]))
            r = g.tick()
            assert oa.tick(ops) == 0 and ob.tick(tb.ticks[t]) == 0
            hi_a = base + (n if t >= t_grow else n0)      # A's slot range (B sits right behind it before the grow)
            _check_tick(r, oa, base, base, hi_a, f"A tick {t}")
            _check_tick(r, ob, base_b, base_b, base_b + tb.capacity, f"B tick {t}")
            recs = g.sync_collect().records
            _check_records(recs, oa, base, base, hi_a, tr.gates, f"A tick {t}")
            _check_records(recs, ob, base_b, base_b, base_b + tb.capacity, tb.gates, f"B tick {t}")
        for s in range(0, n, 7):
            assert np.array_equal(g.neighbors(base + s) - base, oa.neighbors(s)), s
    finally:
        g.close()
        oa.close()
        ob.close()


def test_create_destroy_cycles_reuse_ranges():
    keep = T.dyadic_walk_trace(53, 300, 512.0, 100.0, 1, move_frac=0.3, gate_count=1, client_frac=1.0)
    o = pyorc.OracleSpace(keep.capacity, keep.d, pyorc.SEQRULE)
    pyorc.load_trace(o, keep)
    g = gpuaoi.GpuAOI(0)
    try:
        sk, bk = gpuaoi.load_space(g, keep)
        g.sync_collect()
        o.collect()
        rng = np.random.default_rng(7)
        peak = 0
        sids = set()
        walk = keep.ticks[0]
        for cyc in range(1000):
            cap = int(rng.integers(200, 1500))
            sid, base = g.create_space(100.0, cap, (-256, -256, 256, 256))
            sids.add(sid)
            k = min(cap, 120)
            sl = np.arange(k, dtype=np.uint32) + base
            x = (rng.integers(-256 * 128, 256 * 128, k) / 128).astype(np.float32)
            z = (rng.integers(-256 * 128, 256 * 128, k) / 128).astype(np.float32)
            g.restore(sid, sl, x, np.zeros(k, np.float32), z, np.zeros(k, np.float32))
            if cyc % 100 == 0:                 # the long-lived space ticks alongside
                ops = walk.copy()
                ops["x"] = ops["x"] + np.float32(cyc % 3)
                mv = T.with_global_slots(ops, bk)
                g.submit(mv)
                r = g.tick()
                assert o.tick(ops) == 0
                _check_tick(r, o, bk, bk, bk + keep.capacity, f"cycle {cyc}")
            lv = T.make_ops(k)
            lv["kind"] = T.OP_LEAVE
            lv["slot"] = sl
            g.submit(lv)
            g.tick()
            g.destroy_space(sid)
            info = g.context_info()
            peak = max(peak, info["total_slots"])
            assert info["live_spaces"] == 1 and info["live_slots"] == keep.capacity
        assert peak <= keep.capacity + 1500            # one space's range at a time, reused
        assert len({v & 0xFFFFF for v in sids}) == 1   # the space index is reused,
        assert len(sids) == 1000                       # each time under a new generation
        info = g.context_info()
        assert info["total_slots"] == keep.capacity and info["total_cells"] == info["live_cells"]
        _check_records(g.sync_collect().records, o, bk, bk, bk + keep.capacity, keep.gates, "after the cycles")
    finally:
        g.close()
        o.close()


def test_destroy_refuses_a_non_empty_space_after_device_submits():
    g = gpuaoi.GpuAOI(0)
    try:
        sid, base = g.create_space(100.0, 64)
        ops = T.enter_ops(np.array([base + 5], np.uint32), np.array([1.0], np.float32), np.zeros(1, np.float32),
                          np.array([2.0], np.float32), np.zeros(1, np.float32))
        dev = g.dev_alloc(ops.nbytes)
        g.h2d(dev, ops)
        g.submit_device(dev, 1)                      # trusted: the host mirror is no longer used
        g.tick()
        with pytest.raises(gpuaoi.GwError) as e:
            g.destroy_space(sid)
        assert e.value.code == -2
        lv = T.make_ops(1)
        lv["kind"], lv["slot"] = T.OP_LEAVE, base + 5
        g.h2d(dev, lv)
        g.submit_device(dev, 1)
        g.tick()
        g.destroy_space(sid)
        with pytest.raises(gpuaoi.GwError):
            g.destroy_space(sid)                     # gone
        # the index is reused by the next space; the old id stays refused for
        # every call that takes a space id and leaves the new space alone
        sid2, base2 = g.create_space(100.0, 64)
        assert sid2 & 0xFFFFF == sid & 0xFFFFF and sid2 != sid
        for call in (lambda: g.destroy_space(sid), lambda: g.grow_space(sid, 128),
                     lambda: g.set_ownership(sid, 0.0, 1.0),
                     lambda: g.restore(sid, np.array([base2], np.uint32), np.ones(1, np.float32),
                                       np.zeros(1, np.float32), np.ones(1, np.float32), np.zeros(1, np.float32))):
            with pytest.raises(gpuaoi.GwError) as e:
                call()
            assert e.value.code == -5 and "stale" in str(e.value)
        assert g.context_info()["live_spaces"] == 1 and g.grow_space(sid2, 64) == base2
        g.destroy_space(sid2)
        g.dev_free(dev)
    finally:
        g.close()
