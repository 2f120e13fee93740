"""Generate the committed golden fixtures of the AOI + sync path (tests/golden/).

Run from the repo root:  python tests/golden/make_golden.py   (≈3 min, 8 cores)

Why generated here: the reference holds no AOI/sync tests, fixtures or golden
vectors, and the module that does the AOI arithmetic (github.com/xiaonanln/
go-aoi v0.2.0, reference go.mod:25) is neither vendored nor runnable without Go
(SURVEY.md 8(c)).  Parity at the go-aoi boundary is therefore UNPINNED; these
vectors pin the restatement instead, so that the oracle, the GPU path and any
later refactor of either are held to the same bytes:

* every fixture is produced only after the three oracle engines agree on it —
  ORC_XZLIST (go-aoi's linked-list algorithm + the InterestedIn/By glue of
  Entity.go:227-246, per call), ORC_BRUTE (O(N) window test per call) and
  ORC_SEQRULE (the batched per-tick contract the GPU implements) — and, for
  the large digests, oracle/gridmt.c agrees with ORC_SEQRULE too;
* inputs are stored as data (the ops of every tick, the initial population,
  the client table), not as generator calls: a fixture stays valid if
  goworld_amd/traces.py changes;
* outputs are the canonical net events of every tick (full arrays), the
  CollectEntitySyncInfos records (full for the first tick, SHA-256 of the
  canonical bytes for every tick), the XZList raw callback / client message
  counts, the SHA-256 of the game->gate wire bytes (Entity.go:1210-1254,
  netutil LE) and a digest of the final InterestedIn sets.

Large configs (#2 100k, #3 1M) are kept as digests only (digests.json): the
trace is regenerated from its seed and its input ops are hashed first, so a
generator change is reported as such and not as a parity failure.

Files (numpy .npz, no pickles: load with allow_pickle=False):
  <name>.npz   see FIELDS below
  digests.json per config: input hash, per tick counts + SHA-256 of the
               canonical enter / leave / record bytes
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from goworld_amd import traces as T   # noqa: E402  (input generator only)
from oracle import pyorc              # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

FIELDS = """
  capacity, d            space size and AOI distance (Space.EnableAOI(d))
  bounds                 grid sizing hint (minx, minz, maxx, maxz); no effect on results
  init_slots/x/y/z/yaw   initial population, bulk-entered in index order with
                         sync flags 3 (Space.enter, Space.go:196)
  gates                  u16 per slot, 0 = no client
  ops, tick_off          all ticks' gw_op records (24 B, include/gpuaoi.h),
                         tick t = ops[tick_off[t]:tick_off[t+1]]
  enter, enter_off       canonical net enter events (watcher, target) per tick
  leave, leave_off       same for leave
  rec0                   sync records of tick 0's collect, canonical
                         (gate(watcher), entity, watcher) order
  n_rec, rec_sha         per tick: record count, SHA-256 of canonical bytes
  wire_sha               per tick: SHA-256 of the game->gate packets
  raw                    per tick: XZList raw OnEnterAOI, OnLeaveAOI calls,
                         create / destroy client messages (u64 x4)
  nbr_total, nbr_sha     after the last tick: sum |InterestedIn|, SHA-256 of
                         the ascending lists of slots 0..capacity-1, each
                         prefixed by its u32 length
"""


def sha(b) -> str:
    return hashlib.sha256(b if isinstance(b, (bytes, bytearray)) else np.ascontiguousarray(b).tobytes()).hexdigest()


def neighbour_digest(o: pyorc.OracleSpace, capacity: int) -> str:
    h = hashlib.sha256()
    for s in range(capacity):
        nb = o.neighbors(s).astype(np.uint32)
        h.update(np.uint32(len(nb)).tobytes())
        h.update(nb.tobytes())
    return h.hexdigest()


def run_small(tr, with_brute: bool = True) -> dict:
    """Replay tr through every oracle engine; assert they agree; return the
    fixture arrays."""
    modes = [pyorc.XZLIST, pyorc.SEQRULE] + ([pyorc.BRUTE] if with_brute else [])
    spaces = {}
    for m in modes:
        o = pyorc.OracleSpace(tr.capacity, tr.d, m)
        pyorc.load_trace(o, tr)
        spaces[m] = o
    enter, leave, enter_off, leave_off = [], [], [0], [0]
    n_rec, rec_sha, wire_sha, raw = [], [], [], []
    rec0 = None
    for t, ops in enumerate(tr.ticks):
        outs = {}
        for m, o in spaces.items():
            assert o.tick(ops) == 0, f"oracle mode {m} rejected tick {t}"
            e, l = o.events()
            r = o.collect()
            outs[m] = (e.tobytes(), l.tobytes(), r.tobytes())
            if m == pyorc.XZLIST:
                wire = o.wire()
                ev, lv, rv = e, l, r
                raw.append(o.raw_counts())
        ref = outs[pyorc.XZLIST]
        for m, v in outs.items():
            assert v == ref, f"oracle engines disagree at tick {t} (mode {m})"
        enter.append(ev); leave.append(lv)
        enter_off.append(enter_off[-1] + len(ev)); leave_off.append(leave_off[-1] + len(lv))
        n_rec.append(len(rv)); rec_sha.append(sha(rv)); wire_sha.append(sha(wire))
        if t == 0:
            rec0 = rv
    o = spaces[pyorc.XZLIST]
    for m, s in spaces.items():
        assert s.total_neighbors() == o.total_neighbors()
    nd = neighbour_digest(o, tr.capacity)
    if pyorc.BRUTE in spaces:
        assert neighbour_digest(spaces[pyorc.BRUTE], tr.capacity) == nd
    assert neighbour_digest(spaces[pyorc.SEQRULE], tr.capacity) == nd
    ops_all = np.concatenate(tr.ticks) if tr.ticks else T.make_ops(0)
    tick_off = np.cumsum([0] + [len(x) for x in tr.ticks]).astype(np.uint64)
    gates = tr.gates if tr.gates is not None else np.zeros(tr.capacity, np.uint16)
    return dict(
        capacity=np.uint32(tr.capacity), d=np.float32(tr.d), bounds=np.array(tr.bounds, np.float32),
        init_slots=tr.init_slots.astype(np.uint32), init_x=tr.init_x.astype(np.float32),
        init_y=tr.init_y.astype(np.float32), init_z=tr.init_z.astype(np.float32),
        init_yaw=tr.init_yaw.astype(np.float32), gates=gates.astype(np.uint16),
        ops=ops_all, tick_off=tick_off,
        enter=np.concatenate(enter), enter_off=np.array(enter_off, np.uint64),
        leave=np.concatenate(leave), leave_off=np.array(leave_off, np.uint64),
        rec0=rec0, n_rec=np.array(n_rec, np.uint64),
        rec_sha=np.array(rec_sha, dtype="S64"), wire_sha=np.array(wire_sha, dtype="S64"),
        raw=np.array(raw, np.uint64).reshape(-1, 4),
        nbr_total=np.uint64(o.total_neighbors()), nbr_sha=np.bytes_(nd),
    )


def small_fixtures():
    """(name, trace, run brute force too) of the committed fixtures."""
    return [
        # BASELINE config #1: examples/test_game, 1k float32 random walkers (non-dyadic)
        ("cfg1_walk", T.config1(ticks=30), True),
        # #1b: same with +-4 steps (events every tick)
        ("cfg1b_steps", T.config1(ticks=30, big_steps=True), True),
        # rounding-edge positions (asymmetric rounded windows) + Leave/re-Enter/Sync churn
        ("adversarial_s11", T.adversarial_trace(11, n=300, ticks=20), True),
        ("adversarial_s12", T.adversarial_trace(12, n=300, ticks=20), True),
        # the same churn with non-zero Position.Y and yaw on every entity and
        # op, server-side moves (OWN | NEIGHBOR) beside client ones, Leave
        # keep-masks: the sync payload is (x, y, z, yaw) of the last op
        ("server_y_s13", T.adversarial_trace(13, n=300, ticks=20, leave_masks=True, with_y=True), True),
        # dyadic walk (configs #2-#5 shape) with hotspots, 3 gates, 80% clients
        ("dyadic_hot_2k", T.dyadic_walk_trace(21, 2000, 2048.0, 100.0, 20, move_frac=0.25,
                                              hot_frac=0.4, n_hot=4, gate_count=3,
                                              client_frac=0.8), False),
    ]


def digest_configs():
    return [
        ("config2_100k", lambda: T.config2(ticks=3), 3),
        ("config3_1m", lambda: T.config3(ticks=2), 2),
    ]


def trace_input_sha(tr) -> str:
    h = hashlib.sha256()
    for a in (tr.init_slots, tr.init_x, tr.init_y, tr.init_z, tr.init_yaw, tr.gates):
        h.update(np.ascontiguousarray(a).tobytes())
    for ops in tr.ticks:
        h.update(ops.tobytes())
    return h.hexdigest()


def run_digest(tr) -> dict:
    """ORC_SEQRULE and gridmt (independent implementations of the batched
    contract) must agree; the digests are taken from the oracle."""
    o = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.SEQRULE)
    pyorc.load_trace(o, tr)
    g = pyorc.GridMT(tr.capacity, tr.d, tr.bounds)
    g.load(tr)
    ticks = []
    for t, ops in enumerate(tr.ticks):
        assert o.tick(ops) == 0 and g.tick(ops) == 0
        e, l = o.events()
        r = o.collect()
        ge, gl = g.events()
        gr = g.collect()
        assert ge.tobytes() == e.tobytes() and gl.tobytes() == l.tobytes(), f"gridmt events differ at {t}"
        gates = tr.gates
        def canon(x):   # gridmt's order inside an entity differs: compare canonically
            return x[np.lexsort((x["watcher"], x["entity"], gates[x["watcher"]]))].tobytes()
        assert canon(gr) == canon(r) == r.tobytes(), f"gridmt records differ at {t}"
        ticks.append(dict(n_enter=len(e), n_leave=len(l), n_rec=len(r),
                          enter_sha=sha(e), leave_sha=sha(l), rec_sha=sha(r)))
        print(f"  tick {t}: {len(e)} enter, {len(l)} leave, {len(r)} records", flush=True)
    return dict(input_sha=trace_input_sha(tr), ticks=ticks,
                nbr_total=int(o.total_neighbors()))


def config5_world_trace(ticks: int = 3):
    """Config #5 (the 16M world) as the single-context op stream
    of tests/test_gpu_config5.py: the world walk's ops of each tick split by
    the strip that owns each mover before the tick (8 strips) and concatenated
    rank-major, the order the world's stamps give them; the population
    entered in slot order (the test's restore), one gate for every entity."""
    from goworld_amd.dworld import Strips
    n, side, ranks = 16_000_000, 131072.0, 8
    walk = T.WorldWalk(seed=5, n=n, side=side)
    x0, z0, yaw0 = walk.x(), walk.z(), walk.yaw.copy()
    geom = Strips(-side / 2, side / ranks, ranks, 100.0, 4.0)
    ops_t = []
    for _ in range(ticks):
        ops, xb = walk.next_tick()
        own = geom.owner(xb)
        ops_t.append(np.concatenate([ops[own == r] for r in range(ranks)]))
    return T.SpaceTrace(n=n, capacity=n, d=100.0, bounds=(-side / 2, -side / 2, side / 2, side / 2),
                        init_slots=np.arange(n, dtype=np.uint32), init_x=x0, init_y=np.zeros(n, np.float32),
                        init_z=z0, init_yaw=yaw0, ticks=ops_t, gates=np.ones(n, np.uint16))


def rec_digest(recs: np.ndarray):
    """Order-free digest of a record multiset, (count, sum h1, sum h2) mod 2^64:
    the one tests/test_gpu_config5.py takes of the GPU's records."""
    m1, m2 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xBF58476D1CE4E5B9)

    def mix(z):
        z = z.copy()
        z ^= z >> np.uint64(30)
        z *= m2
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
        return z
    w = np.ascontiguousarray(recs).view(np.uint64).reshape(-1, 3)
    with np.errstate(over="ignore"):
        h1 = mix(w[:, 0] ^ mix(w[:, 1] + m1) ^ mix(w[:, 2] * m2 + np.uint64(7)))
        h2 = mix((w[:, 0] * m1) ^ mix(w[:, 1] ^ m2) ^ mix(w[:, 2] + np.uint64(0x632BE59BD9B4E019)))
        return [len(recs), int(h1.sum(dtype=np.uint64)), int(h2.sum(dtype=np.uint64))]


def run_config5_digest(tr) -> dict:
    """gridmt (oracle/gridmt.c, equal to ORC_SEQRULE on every trace of
    tests/test_oracle.py and on the #2 / #3 / #4 digests above) over the 16M
    world as one space: per tick the canonical events' SHA-256 and the
    records' order-free digest.  The load's own collect is not digested."""
    g = pyorc.GridMT(tr.capacity, tr.d, tr.bounds)
    g.load(tr)
    g.collect()
    ticks = []
    for t, ops in enumerate(tr.ticks):
        assert g.tick(ops) == 0
        e, l = g.events()
        r = g.collect()
        ticks.append(dict(n_enter=len(e), n_leave=len(l), n_rec=len(r), enter_sha=sha(e), leave_sha=sha(l),
                          rec_digest=rec_digest(r)))
        print(f"  tick {t}: {len(e)} enter, {len(l)} leave, {len(r)} records", flush=True)
        del r
    return dict(input_sha=trace_input_sha(tr), ticks=ticks, engine="gridmt")


def multi_digest_configs():
    return [("config4_10k", lambda: [T.config4_space(s, ticks=2) for s in range(10_000)])]


def run_multi_digest(trs) -> dict:
    """Independent spaces in one context, loaded and collected once (that
    collect is not digested: 3.5e8 records), then ticked: each space through
    ORC_SEQRULE and gridmt (must agree), outputs shifted to global slots (space i's slots
    start at the sum of the earlier capacities) and merged in the canonical
    orders: events by (watcher, target) = the spaces' arrays back to back;
    records by (gate(watcher), entity, watcher)."""
    bases = np.cumsum([0] + [tr.capacity for tr in trs])
    gates = np.concatenate([tr.gates for tr in trs])
    n_ticks = len(trs[0].ticks)
    acc = [dict(e=[], l=[], r=[]) for _ in range(n_ticks)]
    nbr = 0
    for i, tr in enumerate(trs):
        o = pyorc.OracleSpace(tr.capacity, tr.d, pyorc.SEQRULE)
        pyorc.load_trace(o, tr)
        g = pyorc.GridMT(tr.capacity, tr.d, tr.bounds)
        g.load(tr)
        o.collect()                      # the load's own collect is not part of the digest
        g.collect()
        b = np.uint32(bases[i])
        for t, ops in enumerate(tr.ticks):
            assert o.tick(ops) == 0 and g.tick(ops) == 0
            e, l = o.events()
            ge, gl = g.events()
            assert ge.tobytes() == e.tobytes() and gl.tobytes() == l.tobytes(), f"space {i} tick {t}"
            r = o.collect()
            g.collect()
            for a, k in ((e, "e"), (l, "l")):
                a = a.copy()
                a["watcher"] += b
                a["target"] += b
                acc[t][k].append(a)
            r = r.copy()
            r["watcher"] += b
            r["entity"] += b
            acc[t]["r"].append(r)
        nbr += int(o.total_neighbors())
        if i % 1000 == 0:
            print(f"  space {i}", flush=True)
    ticks = []
    for t in range(n_ticks):
        e = np.concatenate(acc[t]["e"])
        l = np.concatenate(acc[t]["l"])
        r = np.concatenate(acc[t]["r"])
        r = r[np.lexsort((r["watcher"], r["entity"], gates[r["watcher"]]))]
        ticks.append(dict(n_enter=len(e), n_leave=len(l), n_rec=len(r),
                          enter_sha=sha(e), leave_sha=sha(l), rec_sha=sha(r)))
        print(f"  tick {t}: {len(e)} enter, {len(l)} leave, {len(r)} records", flush=True)
    h = hashlib.sha256()
    for tr in trs:
        h.update(bytes.fromhex(trace_input_sha(tr)))
    return dict(input_sha=h.hexdigest(), ticks=ticks, nbr_total=nbr, spaces=len(trs))


def main(argv):
    only = set(argv[1:])
    for name, tr, brute in small_fixtures():
        if only and name not in only:
            continue
        print(f"{name}: N={tr.n}, {len(tr.ticks)} ticks", flush=True)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **run_small(tr, brute))
    digest_names = [n for n, _, _ in digest_configs()] + [n for n, _ in multi_digest_configs()] + ["config5_16m"]
    if only and not any(n in only for n in digest_names):
        return
    out = {"_note": "SHA-256 of canonical outputs (tests/golden/make_golden.py); "
                    "records in (gate(watcher), entity, watcher) order"}
    for name, make, _ in digest_configs():
        if only and name not in only:
            continue
        print(f"{name}", flush=True)
        out[name] = run_digest(make())
    for name, make in multi_digest_configs():
        if only and name not in only:
            continue
        print(f"{name}", flush=True)
        out[name] = run_multi_digest(make())
    if "config5_16m" in only:                  # (on request only: ~16 GB, minutes on 8 cores)
        print("config5_16m", flush=True)
        out["config5_16m"] = run_config5_digest(config5_world_trace())
    path = os.path.join(HERE, "digests.json")
    if only and os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
        old.update(out)
        out = old
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv)
