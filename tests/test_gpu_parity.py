"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same seeded traces — bit-exact events, sync records and neighbour lists.

Event and sync-record streams are compared byte for byte as the GPU emits them:
events in the canonical (watcher, target) order; records in the documented
order (gate, entity, own record first, then the watchers in the window walk's
grid order), predicted here from the oracle's records and the grid geometry,
or (gate, watcher, entity) with GW_SYNC_BY_CLIENT (the reference's own order is
Go map order, i.e. random).

The oracle engines are equal to each other on every trace (test_oracle.py), so
the GPU is checked against ORC_SEQRULE for speed and against ORC_XZLIST (the
go-aoi restatement) on the small and adversarial traces.  Parity at the go-aoi
boundary itself is unpinned (see oracle/orc.h).
"""
import numpy as np
import pytest

from goworld_amd import gpuaoi, traces as T
from oracle import pyorc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx_factory():
    made = []

    def make():
        g = gpuaoi.GpuAOI(0)
        made.append(g)
        return g
    yield make
    for g in made:
        g.close()


def _sorted_records(recs, gates_of):
    if len(recs) == 0:
        return recs
    g = gates_of[recs["watcher"]]
    order = np.lexsort((recs["watcher"], recs["entity"], g))
    return recs[order]


def grid_cells(tr, x, z, cells_per_d=2):
    """The library's uniform-grid cell of positions (x, z) of one space, as
    gw_space_create / dev_common.hpp cell_of compute it (float32)."""
    b = [float(v) for v in tr.bounds]
    d = float(tr.d)
    ex, ez = b[2] - b[0], b[3] - b[1]
    maxabs = max(abs(b[0]), abs(b[2]), abs(b[1]), abs(b[3]))
    span = 2.0 * d + 4e-6 * (maxabs + d) + 1e-3
    cs = max(max(d / cells_per_d, max(ex, ez) / 4096.0), span / 9.0)
    inv = np.float32(1.0 / cs)
    W, H = max(1, int(np.ceil(ex / cs))), max(1, int(np.ceil(ez / cs)))

    def cellc(v, o, lim):
        f = np.floor((np.asarray(v, np.float32) - np.float32(o)) * inv)
        return np.clip(f, 0, lim - 1).astype(np.int64)
    return cellc(z, b[1], H) * W + cellc(x, b[0], W)


class Harness:
    """One GPU context with several spaces, each mirrored by an oracle space.
    Positions are tracked from the ops to predict the record stream's exact
    order (the walk's grid order)."""

    def __init__(self, g, trs, mode=pyorc.SEQRULE):
        self.g, self.trs = g, trs
        self.orcs, self.bases = [], []
        cap_total = 0
        self.x, self.z = [], []
        for tr in trs:
            sid, base = gpuaoi.load_space(g, tr)
            o = pyorc.OracleSpace(tr.capacity, tr.d, mode)
            pyorc.load_trace(o, tr)
            self.orcs.append(o)
            self.bases.append(base)
            cap_total = base + tr.capacity
            x = np.zeros(tr.capacity, np.float32)
            z = np.zeros(tr.capacity, np.float32)
            x[tr.init_slots], z[tr.init_slots] = tr.init_x, tr.init_z
            self.x.append(x)
            self.z.append(z)
        self.gates = np.zeros(cap_total, np.uint16)
        for tr, b in zip(trs, self.bases):
            if tr.gates is not None:
                self.gates[b:b + tr.capacity] = tr.gates

    def track(self, i, ops):
        aoi = np.isin(ops["kind"], [T.OP_ENTER, T.OP_MOVED])
        self.x[i][ops["slot"][aoi]] = ops["x"][aoi]
        self.z[i][ops["slot"][aoi]] = ops["z"][aoi]

    def check_collect(self):
        r = self.g.sync_collect()
        exp, keys = [], []
        for i, (o, b, tr) in enumerate(zip(self.orcs, self.bases, self.trs)):
            e = o.collect()
            cell = grid_cells(tr, self.x[i][e["watcher"]], self.z[i][e["watcher"]])
            own = e["watcher"] == e["entity"]
            e["watcher"] += b
            e["entity"] += b
            exp.append(e)
            keys.append(np.where(own, -1, cell))
        exp = np.concatenate(exp) if exp else np.zeros(0, pyorc.REC_DTYPE)
        cell = np.concatenate(keys) if keys else np.zeros(0, np.int64)
        # the documented stream order: (gate, entity, own record first, then the
        # watchers' (grid cell, slot)) - compared raw, no host re-sort of the GPU output
        exp = exp[np.lexsort((exp["watcher"], cell, exp["entity"], self.gates[exp["watcher"]]))]
        assert r.n_rec == len(exp)
        assert r.records.tobytes() == exp.tobytes(), "sync records differ"
        assert r.gate_off[0] == 0 and r.gate_off[-1] == len(exp)
        for gid in range(len(r.gate_off) - 1):
            assert np.all(self.gates[r.records["watcher"][r.gate_off[gid]:r.gate_off[gid + 1]]] == gid)
        return r

    def step(self, t):
        ops = [T.with_global_slots(tr.ticks[t], b) for tr, b in zip(self.trs, self.bases)]
        self.g.submit(np.concatenate(ops))
        res = self.g.tick()
        ee, ll = [], []
        for i, (tr, o, b) in enumerate(zip(self.trs, self.orcs, self.bases)):
            assert o.tick(tr.ticks[t]) == 0
            self.track(i, tr.ticks[t])
            e, l = o.events()
            e = e.copy(); l = l.copy()
            for a in (e, l):
                a["watcher"] += b
                a["target"] += b
            ee.append(e); ll.append(l)
        ee, ll = np.concatenate(ee), np.concatenate(ll)
        assert res.n_enter == len(ee) and res.n_leave == len(ll), (res.n_enter, len(ee), res.n_leave, len(ll))
        assert res.enter.tobytes() == ee.tobytes(), "enter events differ"
        assert res.leave.tobytes() == ll.tobytes(), "leave events differ"
        return res

    def check_lists(self, sample=None):
        for tr, o, b in zip(self.trs, self.orcs, self.bases):
            slots = range(tr.capacity) if sample is None else sample
            for s in slots:
                got = self.g.neighbors(b + s)
                exp = o.neighbors(s).astype(np.uint32) + b
                assert np.array_equal(got, exp), f"neighbour list of slot {s} differs"


def test_tiny_hand_made(ctx_factory):
    g = ctx_factory()
    sid, base = g.create_space(100.0, 8)
    o = pyorc.OracleSpace(8, 100.0, pyorc.XZLIST)
    ops = T.make_ops(4)
    ops["kind"] = 1
    ops["sync_flags"] = 3
    ops["slot"] = [0, 1, 2, 3]
    ops["x"] = [0, 50, 100, 400]
    ops["z"] = [0, 0, 100, 0]
    g.set_clients(np.arange(4, dtype=np.uint32) + base, np.ones(4, np.uint16))
    for s in range(4):
        o.set_client(s, 1)
    g.submit(T.with_global_slots(ops, base))
    r = g.tick()
    assert o.tick(ops) == 0
    e, l = o.events()
    assert r.enter.tobytes() == e.tobytes() and r.n_leave == 0 == len(l)
    assert list(g.neighbors(base + 0)) == [base + 1, base + 2]
    rec = g.sync_collect().records
    gates = np.zeros(base + 8, np.uint16)
    gates[base:base + 4] = 1
    assert _sorted_records(rec, gates).tobytes() == _sorted_records(o.collect(), gates[base:]).tobytes()


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_adversarial_rounding_and_churn_vs_xzlist(ctx_factory, seed):
    tr = T.adversarial_trace(seed, n=300, ticks=12, leave_masks=seed == 13)   # 13: Leave keep-masks
    h = Harness(ctx_factory(), [tr], mode=pyorc.XZLIST)
    h.check_collect()
    for t in range(len(tr.ticks)):
        h.step(t)
        h.check_collect()
    h.check_lists()


def test_config1_float_walk_vs_xzlist(ctx_factory):
    tr = T.config1(ticks=30, n=1000, big_steps=True)
    h = Harness(ctx_factory(), [tr], mode=pyorc.XZLIST)
    h.check_collect()
    for t in range(len(tr.ticks)):
        h.step(t)
        h.check_collect()
    h.check_lists()


def test_config2_uniform_100k(ctx_factory):
    tr = T.config2(ticks=3)
    h = Harness(ctx_factory(), [tr])
    h.check_collect()
    for t in range(len(tr.ticks)):
        h.step(t)
        h.check_collect()
    h.check_lists(sample=range(0, tr.capacity, 97))


@pytest.mark.parametrize("flat", ["0", "1"])
def test_bucket_items_made_by_count_pass(ctx_factory, flat, monkeypatch):
    """The bucket path's items (own runs + mirror events) are made either by
    k_flat_items ahead of the count pass or by the count pass itself (the
    default from 128 tiles of items up); GW_BK_FLAT forces either on a 100k
    space of a few tiles and on the 200k hotspot space (tens of tiles):
    events and records stay exact against the oracle."""
    monkeypatch.setenv("GW_BK_FLAT", flat)
    for tr in (T.config2(ticks=2), T.config3(ticks=1, n=200_000, side=14654.0)):
        h = Harness(ctx_factory(), [tr])
        h.check_collect()
        for t in range(len(tr.ticks)):
            h.step(t)
            h.check_collect()


def test_unmerged_launches(ctx_factory, monkeypatch):
    """The launch merges of round 5 each keep their separate-launch path for
    comparison (GW_POST_SPLIT: k_mover_post apart from k_bits_list;
    GW_PLACE_SPLIT: k_place and k_grid_copy apart; GW_DIRTY_SPLIT: k_grid_dirty
    apart from k_bounds): with all three set, events, records and neighbour
    lists of the 200k hotspot space stay exact against the oracle."""
    for k in ("GW_POST_SPLIT", "GW_PLACE_SPLIT", "GW_DIRTY_SPLIT"):
        monkeypatch.setenv(k, "1")
    tr = T.config3(ticks=2, n=200_000, side=14654.0)
    h = Harness(ctx_factory(), [tr])                    # gw_init reads the knobs
    h.check_collect()
    for t in range(len(tr.ticks)):
        h.step(t)
        h.check_collect()
    h.check_lists(sample=range(0, tr.capacity, 401))


def test_hotspot_clustered_200k(ctx_factory):
    tr = T.config3(ticks=2, n=200_000, side=14654.0)   # 1M-config density, smaller world
    h = Harness(ctx_factory(), [tr])
    h.check_collect()
    for t in range(len(tr.ticks)):
        r = h.step(t)
        assert r.n_enter > 0
        h.check_collect()
    h.check_lists(sample=range(0, tr.capacity, 211))


def test_many_spaces_one_launch(ctx_factory):
    trs = [T.config4_space(s, ticks=3, n=300) for s in range(40)]
    for i, tr in enumerate(trs):
        tr.gates = np.where(tr.gates > 0, 1 + (i % 3), 0).astype(np.uint16)   # 3 gates
    h = Harness(ctx_factory(), trs)
    h.check_collect()
    for t in range(3):
        h.step(t)
        h.check_collect()
    h.check_lists()


@pytest.mark.parametrize("n", [3000, 9000])
def test_everyone_at_one_point(ctx_factory, n):
    """Maximum skew: every entity in one cell, K = N-1 (hotspot stress; n=9000
    exceeds the LDS tiers and exercises the global-scratch paths)."""
    tr = T.SpaceTrace(n=n, capacity=n, d=100.0, bounds=(-1000, -1000, 1000, 1000),
                      init_slots=np.arange(n, dtype=np.uint32), init_x=np.full(n, 5.0, np.float32),
                      init_y=np.zeros(n, np.float32), init_z=np.full(n, -5.0, np.float32),
                      init_yaw=np.zeros(n, np.float32), ticks=[], gates=np.ones(n, np.uint16))
    ops = T.make_ops(n // 2)
    ops["kind"] = T.OP_MOVED
    ops["sync_flags"] = 2
    ops["slot"] = np.arange(0, n, 2)
    ops["x"] = np.where(np.arange(n // 2) % 3 == 0, 500.0, 5.0)
    ops["z"] = -5.0
    tr.ticks = [ops]
    h = Harness(ctx_factory(), [tr])
    h.check_collect()
    h.step(0)
    h.check_collect()
    h.check_lists(sample=range(0, n, 37))


def test_outside_bounds_and_large_coordinates(ctx_factory):
    """Entities outside the grid bounds land in clamped edge cells: still exact."""
    tr = T.adversarial_trace(21, n=200, ticks=6)
    for a in (tr.init_x, tr.init_z):
        a *= np.float32(40.0)          # +-12000, far outside the +-500 bounds
    for ops in tr.ticks:
        ops["x"] *= np.float32(40.0)
        ops["z"] *= np.float32(40.0)
    h = Harness(ctx_factory(), [tr], mode=pyorc.XZLIST)
    for t in range(len(tr.ticks)):
        h.step(t)
        h.check_collect()
    h.check_lists()


def test_empty_and_sync_only_ticks(ctx_factory):
    g = ctx_factory()
    tr = T.dyadic_walk_trace(9, 500, 1024.0, 100.0, 1)
    h = Harness(g, [tr])
    h.check_collect()
    r = g.tick()                       # nothing submitted
    assert r.n_enter == r.n_leave == 0
    ops = T.make_ops(5)
    ops["kind"] = T.OP_SYNC
    ops["sync_flags"] = 3
    ops["slot"] = np.arange(5)
    ops["yaw"] = 1.25
    ops["x"] = tr.init_x[:5]
    ops["z"] = tr.init_z[:5]
    tr.ticks = [ops]
    r = h.step(0)
    assert r.n_enter == r.n_leave == 0
    h.check_collect()


def test_invalid_ops_raise(ctx_factory):
    g = ctx_factory()
    sid, base = g.create_space(100.0, 4)
    bad = T.make_ops(1)
    bad["kind"] = T.OP_MOVED
    bad["slot"] = base
    with pytest.raises(gpuaoi.GwError):
        g.submit(bad)                  # Moved before Enter (reference: nil implData panic)
    bad["kind"] = T.OP_ENTER
    bad["slot"] = base + 99
    with pytest.raises(gpuaoi.GwError):
        g.submit(bad)
    with pytest.raises(gpuaoi.GwError):
        g.create_space(0.0, 4)         # EnableAOI(0) panics (Space.go:92-94)


def test_repeat_runs_are_deterministic(ctx_factory):
    tr = T.adversarial_trace(31, n=300, ticks=5)
    outs = []
    for _ in range(2):
        g = ctx_factory()
        gpuaoi.load_space(g, tr)
        seq = []
        for ops in tr.ticks:
            g.submit(ops)
            r = g.tick()
            seq.append((r.enter.tobytes(), r.leave.tobytes(), g.sync_collect().records.tobytes()))
        outs.append(seq)
    assert outs[0] == outs[1]


def test_long_dense_run(ctx_factory):
    """Dense world, many ticks, SetYaw ops on entities that do not move (sync
    records without an AOI op), neighbour queries between ticks and the total
    neighbour count against the oracle."""
    n, ticks = 1500, 40
    tr = T.dyadic_walk_trace(77, n, 640.0, 100.0, ticks, move_frac=0.12, step_q=4096)
    for t, ops in enumerate(tr.ticks):          # add SetYaw ops on entities that do not move
        moving = set(ops["slot"].tolist())
        extra = [s for s in range(t, n, 97) if s not in moving][:5]
        if extra:
            yo = T.make_ops(len(extra))
            yo["kind"] = T.OP_SYNC
            yo["sync_flags"] = 3
            yo["slot"] = extra
            yo["yaw"] = np.float32(t)
            # SetYaw carries the entity's current position (Entity.go:1284-1290)
            yo["x"], yo["z"] = 0, 0
            tr.ticks[t] = np.concatenate([ops, yo])
    # positions carried by the SYNC ops must be the entities' real positions
    x, z = tr.init_x.copy(), tr.init_z.copy()
    for ops in tr.ticks:
        mv = ops["kind"] == T.OP_MOVED
        x[ops["slot"][mv]] = ops["x"][mv]
        z[ops["slot"][mv]] = ops["z"][mv]
        sy = ops["kind"] == T.OP_SYNC
        ops["x"][sy] = x[ops["slot"][sy]]
        ops["z"][sy] = z[ops["slot"][sy]]
    h = Harness(ctx_factory(), [tr])
    h.check_collect()
    for t in range(ticks):
        h.step(t)
        h.check_collect()
        if t % 13 == 12:
            h.check_lists(sample=range(0, n, 7))
    h.check_lists()
    assert h.g.total_neighbors() == h.orcs[0].total_neighbors()


def _oracle_events(o, ops):
    assert o.tick(ops) == 0
    e, l = o.events()
    return e.copy(), l.copy()


@pytest.mark.parametrize("dense", [False, True])
def test_deferred_tick_with_collect(ctx_factory, dense):
    """GW_TICK_DEFER: device ops, the tick returns without a host sync, the
    collect's one sync settles it (records checked), then gw_tick_result gives
    the tick's events.  dense: every mover sees thousands of candidates, so the
    first tick overflows the own-event regions and the redo runs in the settle."""
    if dense:
        n = 6000
        tr = T.SpaceTrace(n=n, capacity=n, d=100.0, bounds=(-1000, -1000, 1000, 1000),
                          init_slots=np.arange(n, dtype=np.uint32),
                          init_x=(np.arange(n) % 40).astype(np.float32), init_y=np.zeros(n, np.float32),
                          init_z=(np.arange(n) // 40 % 40).astype(np.float32),
                          init_yaw=np.zeros(n, np.float32), ticks=[], gates=np.ones(n, np.uint16))
        for t in range(3):
            ops = T.make_ops(n // 3)
            ops["kind"] = T.OP_MOVED
            ops["sync_flags"] = 3
            ops["slot"] = np.arange(t, n, 3)[: n // 3]
            ops["x"] = np.where(np.arange(n // 3) % 2 == 0, 150.0 + t, 10.0 + t)
            ops["z"] = 7.0
            tr.ticks.append(ops)
    else:
        tr = T.config2(ticks=4, n=30_000)
    g = ctx_factory()
    gpuaoi.load_space(g, tr)
    o = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.SEQRULE)
    pyorc.load_trace(o, tr)
    g.sync_collect(copy=False)
    o.collect()
    gates = tr.gates
    for t in range(len(tr.ticks)):
        ops = tr.ticks[t]
        dev = g.dev_alloc(max(ops.nbytes, 1))
        g.h2d(dev, ops)
        g.submit_device(dev, len(ops))
        r0 = g.tick(copy=False, defer=True)
        assert r0.ops == len(ops) and r0.n_enter == 0          # nothing read back yet
        rec = g.sync_collect()                                  # settles the tick
        ee, ll = _oracle_events(o, ops)
        exp = _sorted_records(o.collect(), gates)
        assert rec.n_rec == len(exp)
        assert _sorted_records(rec.records, gates).tobytes() == exp.tobytes()
        r = g.tick_result()
        assert (r.n_enter, r.n_leave) == (len(ee), len(ll))
        e = np.zeros(r.n_enter, gpuaoi.EVENT_DTYPE)
        l = np.zeros(r.n_leave, gpuaoi.EVENT_DTYPE)
        if r.n_enter:
            g.d2h(e, r.enter_dev)
        if r.n_leave:
            g.d2h(l, r.leave_dev)
        assert e.tobytes() == ee.tobytes() and l.tobytes() == ll.tobytes()
        g.synchronize()
        g.dev_free(dev)
    # a deferred tick followed by another tick (no collect) settles in order
    if not dense:
        for t in range(2):
            ops = tr.ticks[t]
            dev = g.dev_alloc(ops.nbytes)
            g.h2d(dev, ops)
            g.submit_device(dev, len(ops))
            g.tick(copy=False, defer=True)
            g.synchronize()
            g.dev_free(dev)
        g.tick_result()


def test_sync_by_client_matches_gate_dispatch(ctx_factory):
    """GW_SYNC_BY_CLIENT: records grouped per client inside each gate, order
    (gate, watcher, entity), with the client segment table; the per-client
    packets built from them equal the gate's dispatch (GateService.go:350-375,
    restated in oracle/pyorc.gate_dispatch) of the oracle's game->gate packets."""
    import struct
    tr = T.config2(ticks=3, n=20_000)
    tr.gates = np.where(np.arange(tr.capacity) % 7 == 6, 0, 1 + np.arange(tr.capacity) % 3).astype(np.uint16)
    g = ctx_factory()
    gpuaoi.load_space(g, tr)
    o = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.SEQRULE)
    pyorc.load_trace(o, tr)
    eid = [pyorc.fixed_uuid(i) for i in range(tr.capacity)]
    cid = [pyorc.fixed_uuid(i | 0x80000000) for i in range(tr.capacity)]
    for t in range(-1, len(tr.ticks)):
        if t >= 0:
            g.submit(tr.ticks[t])
            g.tick(copy=False)
            assert o.tick(tr.ticks[t]) == 0
        r = g.sync_collect(by_client=True)
        exp = o.collect()
        exp = exp[np.lexsort((exp["entity"], exp["watcher"], tr.gates[exp["watcher"]]))]
        assert r.records.tobytes() == exp.tobytes(), f"tick {t}: per-client records differ"
        # client table: one segment per watcher, in stream order
        w = r.records["watcher"]
        heads = np.nonzero(np.r_[True, w[1:] != w[:-1]])[0] if len(w) else np.zeros(0, np.int64)
        assert np.array_equal(r.client_off, np.r_[heads, len(w)].astype(np.uint64))
        assert np.array_equal(r.client_slot, w[heads])
        # gate_off still partitions the stream by gate
        gsel = tr.gates[w]
        for gid in range(len(r.gate_off) - 1):
            assert np.all(gsel[r.gate_off[gid]:r.gate_off[gid + 1]] == gid)
        if t == len(tr.ticks) - 1:
            got = {}
            for k in range(len(r.client_slot)):
                seg = r.records[r.client_off[k]:r.client_off[k + 1]]
                got[cid[int(r.client_slot[k])]] = struct.pack("<H", 1502) + b"".join(
                    eid[int(e["entity"])] + struct.pack("<4f", e["x"], e["y"], e["z"], e["yaw"]) for e in seg)
            want = {}
            for pkt in pyorc.split_wire(o.wire()):
                want.update(pyorc.gate_dispatch(pkt))
            assert len(want) > 1000 and got == want


def test_clients_change_between_tick_and_collect(ctx_factory):
    """The collect takes a mover's count of neighbours with a client from the
    diff's cache only while it is current: attaching / detaching clients after
    the tick (GameClient set or cleared, GameClient.go:14-27) must be seen by
    the next collect; flags accumulate over two ticks without a collect."""
    tr = T.config2(ticks=4, n=20_000)
    g = ctx_factory()
    h = Harness(g, [tr])
    h.check_collect()
    rng = np.random.default_rng(5)
    for t in range(len(tr.ticks)):
        h.step(t)
        if t % 2 == 0:
            continue                          # two ticks' flags per collect
        sel = rng.choice(tr.capacity, 3000, replace=False).astype(np.uint32)
        newg = np.where(rng.random(3000) < 0.5, 0, 1 + rng.integers(0, 3, 3000)).astype(np.uint16)
        g.set_clients(sel, newg)              # after the tick, before the collect
        h.gates[sel] = newg
        for s, gg in zip(sel.tolist(), newg.tolist()):
            h.orcs[0].set_client(s, gg)
        h.check_collect()


@pytest.mark.parametrize("which,ng,lane_max", [("config2", 3, None), ("config3", 3, None), ("config3", 15, None),
                                                ("config3", 5, 1)])
def test_gate_counts_from_diff(ctx_factory, monkeypatch, which, ng, lane_max):
    """Several gates (2 < G <= 16): a collect right after the tick takes each
    mover's record count per gate from the diff's split (World.nbg) instead of
    walking its window; records and gate partitions must equal the oracle's,
    hotspot cells included (config #3 shape at a reduced population).  With
    GW_GATE_LANE_MAX=1 every mover with more than one client candidate on a
    lane is left without a split (as past 255 per lane), so one collect mixes
    split and walked entries."""
    if lane_max is not None:
        monkeypatch.setenv("GW_GATE_LANE_MAX", str(lane_max))
    tr = (T.config2(ticks=3, n=20_000) if which == "config2"
          else T.config3(ticks=3, n=60_000, side=32768.0 * (0.06 ** 0.5)))
    i = np.arange(tr.capacity)
    tr.gates = np.where(i % 5 == 4, 0, 1 + i % ng).astype(np.uint16)
    h = Harness(ctx_factory(), [tr])
    h.check_collect()
    for t in range(len(tr.ticks)):
        h.step(t)
        h.check_collect()


def test_restore_equals_enter_ticks(ctx_factory):
    """gw_space_restore (freeze/restore bulk path) leaves the
    same state as the Enter ops flushed with TICK_NO_EVENTS: identical events,
    records and neighbour lists over the following ticks; bad restores raise."""
    tr = T.adversarial_trace(41, n=600, ticks=4)
    outs = []
    for via in (False, True):
        g = ctx_factory()
        sid, base = gpuaoi.load_space(g, tr, via_ticks=via)
        seq = [g.sync_collect().records.tobytes()]
        for ops in tr.ticks:
            g.submit(ops)
            r = g.tick()
            seq.append((r.enter.tobytes(), r.leave.tobytes(), g.sync_collect().records.tobytes()))
        seq.append([g.neighbors(s).tobytes() for s in range(0, tr.capacity, 7)])
        outs.append(seq)
        if not via:
            with pytest.raises(gpuaoi.GwError):      # already present
                g.restore(sid, [base], [0.0], [0.0], [0.0], [0.0])
    assert outs[0] == outs[1]
    g = ctx_factory()
    sid, base = g.create_space(100.0, 8)
    with pytest.raises(gpuaoi.GwError):              # duplicate slot in one restore
        g.restore(sid, [base, base], [0.0, 1.0], [0.0, 0.0], [0.0, 0.0], [0.0, 0.0])
    with pytest.raises(gpuaoi.GwError):              # outside the space
        g.restore(sid, [base + 8], [0.0], [0.0], [0.0], [0.0])


@pytest.mark.parametrize("which", ["config2_3gates", "adversarial_1gate"])
def test_client_events_and_fanout_match_oracle(ctx_factory, which):
    """SURVEY 8(f) ranks 2-3 on the device: the create/destroy client messages
    of each tick's events (Entity.go:236-246, GameClient.go:37-59; creates carry
    the target's position and yaw) and the AllClients fan-out of calls
    (Entity.go:743-749), both bit-exact with the oracle's restatement, order
    (gate, watcher, target / call), gate_off partitioning each stream."""
    if which == "config2_3gates":
        tr = T.config2(ticks=3, n=20_000)
        tr.gates = np.where(np.arange(tr.capacity) % 7 == 6, 0, 1 + np.arange(tr.capacity) % 3).astype(np.uint16)
    else:
        tr = T.adversarial_trace(9, n=400, ticks=10)
        tr.gates = (np.arange(tr.capacity) % 3 != 0).astype(np.uint16)
    g = ctx_factory()
    gpuaoi.load_space(g, tr)
    o = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.SEQRULE)
    pyorc.load_trace(o, tr)
    rng = np.random.default_rng(7)
    n_cr = n_de = n_fo = 0
    for t, ops in enumerate(tr.ticks):
        g.submit(ops)
        g.tick(copy=False)
        assert o.tick(ops) == 0
        cr, de = g.client_events()
        ocr, ode = o.client_events()
        assert cr.records.tobytes() == ocr.tobytes(), f"tick {t}: create messages differ"
        assert de.records.tobytes() == ode.tobytes(), f"tick {t}: destroy messages differ"
        calls = rng.integers(0, tr.capacity, 3000).astype(np.uint32)
        f = g.fanout(calls)
        assert f.records.tobytes() == o.fanout(calls).tobytes(), f"tick {t}: fan-out differs"
        for res in (cr, de, f):
            gsel = tr.gates[res.records["watcher"]]
            assert res.gate_off[-1] == len(res.records)
            for gid in range(len(res.gate_off) - 1):
                assert np.all(gsel[res.gate_off[gid]:res.gate_off[gid + 1]] == gid)
        n_cr += len(cr.records); n_de += len(de.records); n_fo += len(f.records)
        if t % 3 == 2:
            g.sync_collect(copy=False)
            o.collect()
    assert n_cr > 0 and n_de > 0 and n_fo > 1000
    assert len(g.fanout(np.zeros(0, np.uint32)).records) == 0
    with pytest.raises(gpuaoi.GwError):
        g.fanout([tr.capacity + 5])


def test_tick_statistics_match_oracle(ctx_factory):
    """gw_tick_out.movers / nbr_old / nbr_new (the A_old, A_new terms of the
    SURVEY 8(d) algorithmic bytes) equal the oracle's list sizes: distinct
    slots with an AOI op, and the sums of their neighbour-list lengths before
    and after the tick."""
    tr = T.adversarial_trace(31, n=300, ticks=6)
    g = ctx_factory()
    gpuaoi.load_space(g, tr)
    o = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.SEQRULE)
    pyorc.load_trace(o, tr)
    for ops in tr.ticks:
        aoi = np.unique(ops["slot"][np.isin(ops["kind"], [T.OP_ENTER, T.OP_MOVED, T.OP_LEAVE])])
        a_old = sum(len(o.neighbors(int(s))) for s in aoi)
        assert o.tick(ops) == 0
        a_new = sum(len(o.neighbors(int(s))) for s in aoi)
        g.submit(ops)
        r = g.tick()
        assert (r.movers, r.nbr_old, r.nbr_new) == (len(aoi), a_old, a_new)


@pytest.mark.parametrize("pad", [150_000, 1_600_000])
def test_client_paths_wide_slot_keys(ctx_factory, pad):
    """The client paths' stable sorts by watcher slot at wider keys: an empty
    first space of `pad` slots puts the traced space's slots past 2^17 (18-bit
    keys) or 2^20 (21-bit keys), three 8-bit onesweep passes instead of the two
    of a 16-bit key (the last pass's digit then spans fewer bits).  Client
    messages, fan-out and the per-client collect equal the oracle's, slots
    shifted by the space's base."""
    tr = T.config2(ticks=3, n=20_000)
    tr.gates = np.where(np.arange(tr.capacity) % 7 == 6, 0, 1 + np.arange(tr.capacity) % 3).astype(np.uint16)
    g = ctx_factory()
    g.create_space(100.0, pad, (-1000.0, -1000.0, 1000.0, 1000.0))
    sid, base = gpuaoi.load_space(g, tr)
    assert base >= pad
    gates = np.zeros(base + tr.capacity, np.uint16)
    gates[base:] = tr.gates
    o = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.SEQRULE)
    pyorc.load_trace(o, tr)
    rng = np.random.default_rng(11)

    def shifted(a, fields):
        a = a.copy()
        for f in fields:
            a[f] += np.uint32(base)
        return a
    n_fo = n_rec = 0
    for t, ops in enumerate(tr.ticks):
        g.submit(T.with_global_slots(ops, base))
        g.tick(copy=False)
        assert o.tick(ops) == 0
        cr, de = g.client_events()
        ocr, ode = o.client_events()
        assert cr.records.tobytes() == shifted(ocr, ("watcher", "entity")).tobytes(), f"tick {t}: creates differ"
        assert de.records.tobytes() == shifted(ode, ("watcher", "target")).tobytes(), f"tick {t}: destroys differ"
        calls = rng.integers(0, tr.capacity, 3000).astype(np.uint32)
        f = g.fanout(calls + np.uint32(base))
        assert f.records.tobytes() == shifted(o.fanout(calls), ("watcher", "entity")).tobytes(), \
            f"tick {t}: fan-out differs"
        r = g.sync_collect(by_client=True)
        exp = shifted(o.collect(), ("watcher", "entity"))
        exp = exp[np.lexsort((exp["entity"], exp["watcher"], gates[exp["watcher"]]))]
        assert r.records.tobytes() == exp.tobytes(), f"tick {t}: per-client records differ"
        n_fo += len(f.records)
        n_rec += len(r.records)
    assert n_fo > 1000 and n_rec > 10_000


@pytest.mark.parametrize("ngates", [3, 15, 20])
def test_multi_gate_partitions(ctx_factory, ngates):
    """Clients spread over several gates (Entity.go:1208-1219 sends one packet
    per gate): the records come grouped by gate, inside a gate in the one-gate
    stream's order, with gate_off partitioning them.  Up to GATE_DIRECT_MAX gate
    ids (3 and 15 gates + "no client") the count and write passes place every
    record straight into its gate's partition; 20 gates take the stable sort by
    gate.  Exact stream order against the oracle."""
    tr = T.config2(ticks=3, n=20_000)
    cap = tr.capacity
    tr.gates = np.where(np.arange(cap) % 11 == 10, 0, 1 + np.arange(cap) % ngates).astype(np.uint16)
    h = Harness(ctx_factory(), [tr])
    r = h.check_collect()
    assert len(r.gate_off) == ngates + 2
    for t in range(len(tr.ticks)):
        h.step(t)
        r = h.check_collect()
        assert int(r.gate_off[1]) == 0                   # gate 0 (no client) holds no record
        assert np.all(np.diff(r.gate_off[1:].astype(np.int64)) > 0)   # every gate has records


@pytest.mark.parametrize("half_rows", [0, 4])
def test_half_wave_walk_fallbacks(ctx_factory, half_rows, monkeypatch):
    """Small-space mode walks movers two per wave (a half-wave each) when both
    windows fit a half's row lanes; other pairs go to k_mover_list (one wave
    per entry from the global grids).  GW_HALF_ROWS lowers the row limit so
    that every pair (0) or the pairs with windows of more than 4 rows take the
    fallback: events, records and neighbour lists stay exact against the
    oracle over 40 small spaces with 3 gates."""
    monkeypatch.setenv("GW_HALF_ROWS", str(half_rows))
    g = ctx_factory()                                   # gw_init reads GW_HALF_ROWS
    monkeypatch.delenv("GW_HALF_ROWS")
    trs = [T.config4_space(s, ticks=3, n=300) for s in range(40)]
    for i, tr in enumerate(trs):
        tr.gates = np.where(tr.gates > 0, 1 + (i % 3), 0).astype(np.uint16)
    h = Harness(g, trs)
    h.check_collect()
    for t in range(3):
        h.step(t)
        h.check_collect()
    h.check_lists()


def test_small_space_redo_with_fallbacks(ctx_factory, monkeypatch):
    """Small-space mode with every pair on the fallback list (GW_HALF_ROWS=0)
    and dense spaces whose first tick overflows the own-event regions and the
    event buffers, so the tick's diff + events are redone: the redo must start
    the fallback list (DevStats.n_fall) afresh instead of appending the first
    attempt's entries again.  Events, records and neighbour lists
    against the oracle over 6 dense spaces with 2 gates."""
    monkeypatch.setenv("GW_HALF_ROWS", "0")
    g = ctx_factory()                                   # gw_init reads GW_HALF_ROWS
    monkeypatch.delenv("GW_HALF_ROWS")
    trs = []
    for s in range(6):
        n = 480
        rng = np.random.default_rng(900 + s)
        x = (rng.integers(0, 240, n) * 0.5).astype(np.float32)
        z = (rng.integers(0, 240, n) * 0.5).astype(np.float32)
        tr = T.SpaceTrace(n=n, capacity=n, d=100.0, bounds=(-200, -200, 320, 320),
                          init_slots=np.arange(n, dtype=np.uint32), init_x=x, init_y=np.zeros(n, np.float32),
                          init_z=z, init_yaw=np.zeros(n, np.float32), ticks=[],
                          gates=np.where(np.arange(n) % 3 == 0, 0, 1 + (np.arange(n) + s) % 2).astype(np.uint16))
        for t in range(3):
            m = n // 3
            ops = T.make_ops(m)
            ops["kind"] = T.OP_MOVED
            ops["sync_flags"] = 3
            ops["slot"] = np.arange(t, n, 3)[:m]
            ops["x"] = np.where(np.arange(m) % 2 == 0, 150.0 + 4 * t, 10.0 + t).astype(np.float32)
            ops["z"] = (rng.integers(0, 240, m) * 0.5).astype(np.float32)
            ops["yaw"] = np.float32(t)
            tr.ticks.append(ops)
        trs.append(tr)
    h = Harness(g, trs)
    h.check_collect()
    for t in range(3):
        h.step(t)
        h.check_collect()
    h.check_lists()
