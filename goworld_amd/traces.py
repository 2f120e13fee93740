"""Seeded synthetic movement traces for the AOI + sync path.

Workload generator shared by tests/ and bench.py.  It is not oracle code: it
only produces inputs.  Every random number comes from a counter-based
SplitMix64 (value = mix64(key + (i+1)*golden)), so any (seed, stream, index)
can be regenerated independently and the traces are identical on every host.

Positions of the perf configs live on a dyadic grid of step 1/128 with
|x| < 2**17, so x +- d is exact in float32 and the reference window test is
symmetric.  Config #1 and the adversarial traces are
deliberately non-dyadic float32 to exercise the rounded-bounds / seq rule.

Sources of the workload shapes (reference paths):
  #1 examples/test_game/Avatar.go:124-131 (integer positions in [-400,400)),
     examples/test_client/ClientBot.go:214-223 (p=0.5 per 100 ms, dx~U(-.01,.01),
     dz~U(-.01,0), yaw~U(0,3.14)), examples/test_game/MySpace.go:28 (EnableAOI(100)).
  #2-#5 BASELINE.json configs, parameters from SURVEY.md 8(d).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# gw_op layout of include/gpuaoi.h (24 bytes, little-endian)
OP_DTYPE = np.dtype([("kind", "u1"), ("sync_flags", "u1"), ("reserved", "<u2"),
                     ("slot", "<u4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4"),
                     ("yaw", "<f4")])
assert OP_DTYPE.itemsize == 24
# gw_long_move (include/gpuaoi.h): a long mover's state before and after a tick
LONG_DTYPE = np.dtype([("slot", "<u4"), ("reserved", "<u4", (3,)), ("old_x", "<f4"), ("old_z", "<f4"),
                       ("new_x", "<f4"), ("new_z", "<f4"), ("old_stamp", "<u8"), ("new_stamp", "<u8")])

OP_ENTER, OP_MOVED, OP_LEAVE, OP_SYNC = 1, 2, 3, 4
SIF_OWN, SIF_NEIGHBOR = 1, 2
Q = 128.0  # dyadic quantum denominator


def mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def stream_key(seed: int, *stream: int) -> np.uint64:
    k = mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF))
    for s in stream:
        with np.errstate(over="ignore"):
            k = mix64(k ^ mix64(np.uint64(s & 0xFFFFFFFFFFFFFFFF) + GOLDEN))
    return np.uint64(k)


def rand_u64(key, n: int, offset: int = 0) -> np.ndarray:
    idx = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(np.uint64(key) + idx * GOLDEN)


def rand_unit(key, n: int) -> np.ndarray:
    """Uniform float64 in [0, 1)."""
    return (rand_u64(key, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def rand_f32(key, n: int) -> np.ndarray:
    """Uniform float32 in [0, 1) with 24 random bits (like Go rand.Float32)."""
    return ((rand_u64(key, n) >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0))


def rand_int(key, n: int, lo: int, hi: int) -> np.ndarray:
    """Uniform integers in [lo, hi)."""
    span = hi - lo
    return (lo + (rand_unit(key, n) * span).astype(np.int64)).clip(lo, hi - 1)


def make_ops(n: int) -> np.ndarray:
    return np.zeros(n, dtype=OP_DTYPE)


@dataclasses.dataclass
class SpaceTrace:
    """One space: initial population + per-tick ops (local slots)."""
    n: int                     # entities (== capacity unless extra headroom)
    capacity: int
    d: float
    bounds: tuple              # (minx, minz, maxx, maxz)
    init_slots: np.ndarray     # u32, bulk-enter order
    init_x: np.ndarray
    init_y: np.ndarray
    init_z: np.ndarray
    init_yaw: np.ndarray
    ticks: list                # list of OP_DTYPE arrays
    gates: np.ndarray | None = None  # u16 per slot (0 = no client)


def _reflect_q(k: np.ndarray, lo_q: int, hi_q: int) -> np.ndarray:
    """Reflect integer 1/128 units into [lo_q, hi_q)."""
    k = np.where(k < lo_q, 2 * lo_q - k, k)
    k = np.where(k >= hi_q, 2 * (hi_q - 1) - k, k)
    return np.clip(k, lo_q, hi_q - 1)


def _choose_movers(key, n: int, m: int) -> np.ndarray:
    """m distinct slots, in random order (the op order of the tick)."""
    r = rand_u64(key, n)
    if m >= n:
        return np.argsort(r, kind="stable").astype(np.uint32)
    part = np.argpartition(r, m - 1)[:m]
    return part[np.argsort(r[part], kind="stable")].astype(np.uint32)


def dyadic_walk_trace(seed: int, n: int, side: float, d: float, ticks: int,
                      move_frac: float = 0.10, step_q: int = 512,
                      hot_frac: float = 0.0, n_hot: int = 64, sigma: float = 200.0,
                      hot_step_q: int = 2048, gate_count: int = 1,
                      client_frac: float = 1.0, capacity: int | None = None,
                      side_z: float | None = None) -> SpaceTrace:
    """Configs #2/#3/#4/#5: uniform (+ optional Gaussian hotspots) on the 1/128
    grid, in [-side/2, side/2) x [-side_z/2, side_z/2) (side_z = side)."""
    side_z = side if side_z is None else side_z
    assert max(side, side_z) / 2 * Q <= 2 ** 24, "dyadic exactness needs |x| <= 2**17"
    half_q = int(side / 2 * Q)
    lo_q, hi_q = -half_q, half_q
    zlo_q, zhi_q = -int(side_z / 2 * Q), int(side_z / 2 * Q)
    n_hot_ent = int(round(n * hot_frac))
    n_bg = n - n_hot_ent
    kx = rand_int(stream_key(seed, 1), n, lo_q, hi_q)
    kz = rand_int(stream_key(seed, 2), n, zlo_q, zhi_q)
    if n_hot_ent:
        cx = rand_unit(stream_key(seed, 3), n_hot) * side - side / 2
        cz = rand_unit(stream_key(seed, 4), n_hot) * side - side / 2
        which = rand_int(stream_key(seed, 5), n_hot_ent, 0, n_hot)
        u1 = 1.0 - rand_unit(stream_key(seed, 6), n_hot_ent)   # (0,1]
        u2 = rand_unit(stream_key(seed, 7), n_hot_ent)
        u3 = 1.0 - rand_unit(stream_key(seed, 8), n_hot_ent)
        u4 = rand_unit(stream_key(seed, 9), n_hot_ent)
        gx = np.sqrt(-2.0 * np.log(u1)) * np.cos(2 * math.pi * u2)
        gz = np.sqrt(-2.0 * np.log(u3)) * np.cos(2 * math.pi * u4)
        hx = np.round((cx[which] + sigma * gx) * Q).astype(np.int64)
        hz = np.round((cz[which] + sigma * gz) * Q).astype(np.int64)
        kx[n_bg:] = np.clip(hx, lo_q, hi_q - 1)
        kz[n_bg:] = np.clip(hz, zlo_q, zhi_q - 1)
    is_hot = np.zeros(n, dtype=bool)
    is_hot[n_bg:] = True
    yaw = (rand_f32(stream_key(seed, 10), n) * np.float32(2 * math.pi)).astype(np.float32)
    cap = capacity or n
    slots = np.arange(n, dtype=np.uint32)
    init_x = (kx / Q).astype(np.float32)
    init_z = (kz / Q).astype(np.float32)
    tr = SpaceTrace(n=n, capacity=cap, d=float(d),
                    bounds=(-side / 2, -side_z / 2, side / 2, side_z / 2),
                    init_slots=slots, init_x=init_x, init_y=np.zeros(n, np.float32),
                    init_z=init_z, init_yaw=yaw, ticks=[])
    gates = np.zeros(cap, dtype=np.uint16)
    has_client = rand_unit(stream_key(seed, 11), n) < client_frac
    gsel = rand_int(stream_key(seed, 12), n, 1, gate_count + 1).astype(np.uint16)
    gates[:n] = np.where(has_client, gsel, 0)
    tr.gates = gates
    m = int(round(n * move_frac))
    for t in range(ticks):
        movers = _choose_movers(stream_key(seed, 100, t), n, m)
        sq = np.where(is_hot[movers], hot_step_q, step_q)
        dx = (rand_unit(stream_key(seed, 101, t), m) * (2 * sq + 1)).astype(np.int64) - sq
        dz = (rand_unit(stream_key(seed, 102, t), m) * (2 * sq + 1)).astype(np.int64) - sq
        kx[movers] = _reflect_q(kx[movers] + dx, lo_q, hi_q)
        kz[movers] = _reflect_q(kz[movers] + dz, zlo_q, zhi_q)
        yaw[movers] = rand_f32(stream_key(seed, 103, t), m) * np.float32(2 * math.pi)
        from_client = rand_unit(stream_key(seed, 104, t), m) < 0.5
        ops = make_ops(m)
        ops["kind"] = OP_MOVED
        # setPositionYaw: neighbours always, own client unless the move came
        # from the client (Entity.go:1199-1204)
        ops["sync_flags"] = np.where(from_client, SIF_NEIGHBOR, SIF_NEIGHBOR | SIF_OWN)
        ops["slot"] = movers
        ops["x"] = (kx[movers] / Q).astype(np.float32)
        ops["z"] = (kz[movers] / Q).astype(np.float32)
        ops["yaw"] = yaw[movers]
        tr.ticks.append(ops)
    return tr


def config2(ticks: int = 100, seed: int = 2, n: int = 100_000) -> SpaceTrace:
    """#2: 100k uniform, L=10240, 10% movers, step +-4."""
    return dyadic_walk_trace(seed, n, 10240.0, 100.0, ticks, 0.10, 512)


def config3(ticks: int = 20, seed: int = 3, n: int = 1_000_000, side: float = 32768.0) -> SpaceTrace:
    """#3: 1M clustered hotspots: 70% uniform, 30% in 64 Gaussians (sigma 200);
    hotspot movers step +-16, others +-4; 10% movers."""
    return dyadic_walk_trace(seed, n, side, 100.0, ticks, 0.10, 512,
                             hot_frac=0.30, n_hot=64, sigma=200.0, hot_step_q=2048)


def config5_strip(rank: int, ranks: int, ticks: int = 20, seed: int = 5,
                  n_world: int = 16_000_000, side: float = 131072.0) -> SpaceTrace:
    """#5: the 16M uniform world (L = 131072, d = 100, 10% movers, step +-4)
    cut into `ranks` X-strips; strip `rank`'s population (n_world / ranks
    entities, uniform in the strip, centred at x = 0: shift by the strip's
    centre).  Walkers reflect at the strip borders."""
    return dyadic_walk_trace(seed * 1000 + rank, n_world // ranks, side / ranks, 100.0, ticks, 0.10, 512,
                             side_z=side)


class WorldWalk:
    """Config #5 as ONE world: n entities uniform on the 1/128
    grid in [-side/2, side/2)^2, each tick `move_frac` of them (a fixed random
    permutation walked in windows, so movers are distinct within a tick) step
    +-step on both axes, reflected at the WORLD borders only, so entities
    cross strip borders and migrate between ranks.  Every rank regenerates the
    same walk and keeps the ops of the entities it owns at the start of the
    tick (the strip of their x then), in the world's op order."""

    def __init__(self, seed: int = 5, n: int = 16_000_000, side: float = 131072.0, d: float = 100.0,
                 move_frac: float = 0.10, step: float = 4.0):
        self.n, self.side, self.d = n, side, d
        self.half_q = int(side / 2 * Q)
        self.seed = seed
        self.kx = rand_int(stream_key(seed, 1), n, -self.half_q, self.half_q)
        self.kz = rand_int(stream_key(seed, 2), n, -self.half_q, self.half_q)
        self.yaw = (rand_f32(stream_key(seed, 10), n) * np.float32(2 * math.pi)).astype(np.float32)
        self.perm = np.argsort(rand_u64(stream_key(seed, 3), n), kind="stable").astype(np.uint32)
        self.m = int(round(n * move_frac))
        self.step_q = int(step * Q)
        self.t = 0

    def x(self) -> np.ndarray:
        return (self.kx / Q).astype(np.float32)

    def z(self) -> np.ndarray:
        return (self.kz / Q).astype(np.float32)

    def next_tick(self):
        """(ops of the whole world in call order, x of every mover before the tick)."""
        t, n, m = self.t, self.n, self.m
        start = (t * m) % n
        idx = np.arange(start, start + m) % n
        movers = self.perm[idx]
        x_before = (self.kx[movers] / Q).astype(np.float32)
        sq = self.step_q
        dx = (rand_unit(stream_key(self.seed, 101, t), m) * (2 * sq + 1)).astype(np.int64) - sq
        dz = (rand_unit(stream_key(self.seed, 102, t), m) * (2 * sq + 1)).astype(np.int64) - sq
        self.kx[movers] = _reflect_q(self.kx[movers] + dx, -self.half_q, self.half_q)
        self.kz[movers] = _reflect_q(self.kz[movers] + dz, -self.half_q, self.half_q)
        self.yaw[movers] = rand_f32(stream_key(self.seed, 103, t), m) * np.float32(2 * math.pi)
        from_client = rand_unit(stream_key(self.seed, 104, t), m) < 0.5
        ops = make_ops(m)
        ops["kind"] = OP_MOVED
        ops["sync_flags"] = np.where(from_client, SIF_NEIGHBOR, SIF_NEIGHBOR | SIF_OWN)
        ops["slot"] = movers
        ops["x"] = (self.kx[movers] / Q).astype(np.float32)
        ops["z"] = (self.kz[movers] / Q).astype(np.float32)
        ops["yaw"] = self.yaw[movers]
        self.t += 1
        return ops, x_before


def config4_space(space: int, ticks: int = 20, seed: int = 4, n: int = 1000) -> SpaceTrace:
    """#4: one of the 10k independent spaces (1k entities, L=1024, d=100)."""
    return dyadic_walk_trace(seed * 1_000_003 + space, n, 1024.0, 100.0, ticks, 0.10, 512)


def config1(ticks: int = 1000, seed: int = 1, n: int = 1000, big_steps: bool = False) -> SpaceTrace:
    """#1: examples/test_game single space, float32 random walk (non-dyadic).

    Positions start on integers in [-400,400) (Avatar.go:124-131).  Each tick
    every bot moves with p=0.5: X += -0.01 + 0.02*r, Z += -0.01 + 0.01*r,
    yaw = r*3.14, all float32 (ClientBot.go:214-223).  Variant #1b
    (big_steps) scales the step to +-4 to produce events."""
    k = stream_key(seed, 1)
    x = rand_int(k, n, -400, 400).astype(np.float32)
    z = rand_int(stream_key(seed, 2), n, -400, 400).astype(np.float32)
    yaw = np.zeros(n, np.float32)
    tr = SpaceTrace(n=n, capacity=n, d=100.0, bounds=(-1000.0, -1000.0, 1000.0, 1000.0),
                    init_slots=np.arange(n, dtype=np.uint32), init_x=x.copy(),
                    init_y=np.zeros(n, np.float32), init_z=z.copy(), init_yaw=yaw.copy(), ticks=[])
    tr.gates = np.ones(n, dtype=np.uint16)
    mr = np.float32(4.0 if big_steps else 0.01)
    for t in range(ticks):
        mv = rand_unit(stream_key(seed, 100, t), n) < 0.5
        order = np.argsort(rand_u64(stream_key(seed, 105, t), n), kind="stable")
        movers = order[mv[order]].astype(np.uint32)
        m = len(movers)
        r1 = rand_f32(stream_key(seed, 101, t), m)
        r2 = rand_f32(stream_key(seed, 102, t), m)
        r3 = rand_f32(stream_key(seed, 103, t), m)
        x[movers] = x[movers] + (-mr + (mr * np.float32(2)) * r1)
        z[movers] = z[movers] + (-mr + mr * r2)
        yaw[movers] = r3 * np.float32(3.14)
        ops = make_ops(m)
        ops["kind"] = OP_MOVED
        ops["sync_flags"] = SIF_NEIGHBOR          # syncPositionYawFromClient: fromClient
        ops["slot"] = movers
        ops["x"] = x[movers]
        ops["z"] = z[movers]
        ops["yaw"] = yaw[movers]
        tr.ticks.append(ops)
    return tr


def adversarial_trace(seed: int, n: int = 400, ticks: int = 30, d: float = 100.0,
                      churn: bool = True, leave_masks: bool = False, with_y: bool = False) -> SpaceTrace:
    """Non-dyadic float32 positions placed on the rounding edge of each other's
    windows (other.x == fl(c.x +- d) +- 1 ulp), so the rounded-bounds test is
    asymmetric and the seq rule decides.  With churn, ticks also contain
    Leave / re-Enter / Sync ops and repeated ops on one slot.  leave_masks:
    Leave ops carry a random keep-mask of pending sync bits (0..3; the entity
    stays in the game in the nil space, Space.go:219-242) instead of 0.
    with_y: every entity has a non-zero Position.Y and yaw, and every Enter /
    Moved gives it a new Y and yaw (setPositionYaw sets both around
    Space.move, Entity.go:1189-1205; SetYaw only the yaw): the sync payload
    then differs from (x, 0, z, yaw) in every record."""
    d32 = np.float32(d)
    base_x = (rand_unit(stream_key(seed, 1), n) * 600 - 300).astype(np.float32)
    base_z = (rand_unit(stream_key(seed, 2), n) * 600 - 300).astype(np.float32)
    # pull half of the entities onto the window edge of a random partner
    partner = rand_int(stream_key(seed, 3), n, 0, n)
    sel = rand_unit(stream_key(seed, 4), n) < 0.5
    sgn = np.where(rand_unit(stream_key(seed, 5), n) < 0.5, -1, 1)
    ulps = rand_int(stream_key(seed, 6), n, -1, 2)
    for i in np.nonzero(sel)[0]:
        p = partner[i]
        edge = np.float32(base_x[p] + d32) if sgn[i] > 0 else np.float32(base_x[p] - d32)
        for _ in range(abs(int(ulps[i]))):
            edge = np.nextafter(edge, np.float32(np.inf if ulps[i] > 0 else -np.inf), dtype=np.float32)
        base_x[i] = edge
        base_z[i] = base_z[p] + np.float32(rand_unit(stream_key(seed, 7, int(i)), 1)[0] * 50)
    x, z = base_x.copy(), base_z.copy()
    yaw = np.zeros(n, np.float32)
    y = np.zeros(n, np.float32)
    if with_y:
        y = (rand_unit(stream_key(seed, 8), n) * 97 - 40).astype(np.float32)
        yaw = (rand_unit(stream_key(seed, 9), n) * 360 - 180).astype(np.float32)
    present = np.ones(n, dtype=bool)
    tr = SpaceTrace(n=n, capacity=n, d=float(d), bounds=(-500.0, -500.0, 500.0, 500.0),
                    init_slots=np.arange(n, dtype=np.uint32), init_x=x.copy(),
                    init_y=y.copy(), init_z=z.copy(), init_yaw=yaw.copy(), ticks=[])
    tr.gates = np.where(np.arange(n) % 5 == 4, 0, 1 + np.arange(n) % 3).astype(np.uint16)
    for t in range(ticks):
        k = stream_key(seed, 200, t)
        cnt = int(n * 0.3)
        picks = rand_int(k, cnt, 0, n)          # repeats allowed: several ops per slot
        kinds_r = rand_unit(stream_key(seed, 201, t), cnt)
        tgt = rand_int(stream_key(seed, 202, t), cnt, 0, n)
        edge_sgn = rand_unit(stream_key(seed, 203, t), cnt) < 0.5
        ny = (rand_unit(stream_key(seed, 204, t), cnt) * 211 - 100).astype(np.float32)
        nyaw = (rand_unit(stream_key(seed, 205, t), cnt) * 360 - 180).astype(np.float32)
        rows = []
        for j in range(cnt):
            a = int(picks[j])
            if not present[a]:
                if churn and kinds_r[j] < 0.7:
                    b = int(tgt[j])
                    nx = np.float32(x[b] + d32) if edge_sgn[j] else np.float32(x[b] - d32)
                    x[a], z[a] = nx, np.float32(z[b] + np.float32(kinds_r[j] * 30))
                    if with_y:
                        y[a], yaw[a] = ny[j], nyaw[j]
                    present[a] = True
                    rows.append((OP_ENTER, 3, a, x[a], y[a], z[a], yaw[a]))
                continue
            if churn and kinds_r[j] < 0.05:
                present[a] = False
                mask = int(kinds_r[j] * 80) & 3 if leave_masks else 0
                rows.append((OP_LEAVE, mask, a, x[a], y[a], z[a], yaw[a]))
            elif churn and kinds_r[j] < 0.10:
                yaw[a] = nyaw[j] if with_y else np.float32(kinds_r[j] * 31)
                rows.append((OP_SYNC, 3, a, x[a], y[a], z[a], yaw[a]))
            else:
                b = int(tgt[j])
                nx = np.float32(x[b] + d32) if edge_sgn[j] else np.float32(x[b] - d32)
                if kinds_r[j] < 0.55:
                    nx = np.nextafter(nx, np.float32(np.inf), dtype=np.float32)
                x[a] = nx
                z[a] = np.float32(z[b] + np.float32((kinds_r[j] - 0.5) * 120))
                if with_y:
                    y[a], yaw[a] = ny[j], nyaw[j]
                rows.append((OP_MOVED, 2 if kinds_r[j] < 0.5 else 3, a, x[a], y[a], z[a], yaw[a]))
        ops = make_ops(len(rows))
        if rows:
            arr = np.array(rows, dtype=object)
            ops["kind"] = arr[:, 0].astype(np.uint8)
            ops["sync_flags"] = arr[:, 1].astype(np.uint8)
            ops["slot"] = arr[:, 2].astype(np.uint32)
            ops["x"] = arr[:, 3].astype(np.float32)
            ops["y"] = arr[:, 4].astype(np.float32)
            ops["z"] = arr[:, 5].astype(np.float32)
            ops["yaw"] = arr[:, 6].astype(np.float32)
        tr.ticks.append(ops)
    return tr


def with_global_slots(ops: np.ndarray, base: int) -> np.ndarray:
    out = ops.copy()
    out["slot"] = ops["slot"] + np.uint32(base)
    return out


def enter_ops(slots, x, y, z, yaw, flags: int = SIF_OWN | SIF_NEIGHBOR) -> np.ndarray:
    """Enter ops for an initial population (Space.enter sets Own|Neighbor,
    Space.go:196)."""
    ops = make_ops(len(slots))
    ops["kind"] = OP_ENTER
    ops["sync_flags"] = flags
    ops["slot"] = slots
    ops["x"], ops["y"], ops["z"], ops["yaw"] = x, y, z, yaw
    return ops


@dataclasses.dataclass
class StripTrace:
    """A decomposed world (config #5 shape): global ops per tick, each tagged
    with the rank that owns it (the strip of the entity's x at the start of
    the tick, or of the Enter position).  Tick 0 enters the population."""
    n: int
    d: float
    ranks: int
    strip_w: float
    max_step: float
    bounds: tuple
    gates: np.ndarray
    ticks: list                # list of (ops OP_DTYPE, owner int64) per tick

    def rank_ops(self, t: int, r: int) -> np.ndarray:
        ops, own = self.ticks[t]
        return ops[own == r]

    def global_ops(self, t: int) -> np.ndarray:
        """The reference call order: rank-major, each rank's ops in order
        (the order of the global stamps)."""
        ops, own = self.ticks[t]
        return ops[np.argsort(own, kind="stable")]


def strip_world_trace(seed: int, n: int, ranks: int, strip_w: float, height: float, d: float,
                      ticks: int, max_step: float, move_frac: float = 0.5,
                      churn: bool = True, edge_frac: float = 0.2, teleports: int = 0,
                      groups: int = 0) -> StripTrace:
    """Random walk across strips (entities migrate between ranks) with churn:
    Leave, re-Enter anywhere, Leave + re-Enter nearby inside one tick, two
    moves of one entity in one tick, Sync ops.  Positions are dyadic except
    an `edge_frac` share placed on strip borders and on the window edge of a
    border entity (x = border +- d, +-1 ulp).  `teleports` > 0: up to that
    many present entities per tick jump anywhere in the world (a Moved op far
    beyond max_step: Entity.SetPosition has no step bound, Entity.go:1185-1187),
    chosen so that no two of them are related before or after the tick.
    `groups` > 0: that many group teleports per tick besides (Entity.SetPosition
    of several related entities in one tick; enterLocalSpace moves entities
    together, Entity.go:975-998), by turns: an entity and up to two neighbours
    within d jump by the same far offset (related before and after), jump to
    separate far places (related before only), or two entities far apart jump
    next to each other (related after only)."""
    W = ranks * strip_w
    step_q = int(max_step * Q) // 2          # half a step per move, <= 2 moves per tick
    lo_q, hi_q = 0, int(W * Q)
    zlo_q, zhi_q = 0, int(height * Q)
    kx = rand_int(stream_key(seed, 1), n, lo_q, hi_q)
    kz = rand_int(stream_key(seed, 2), n, zlo_q, zhi_q)
    x = (kx / Q).astype(np.float32)
    z = (kz / Q).astype(np.float32)
    # edge cases: entities on the borders and on window edges across them
    sel = np.nonzero(rand_unit(stream_key(seed, 3), n) < edge_frac)[0]
    border = (rand_int(stream_key(seed, 4), len(sel), 1, max(2, ranks)) * strip_w).astype(np.float32)
    kind = rand_int(stream_key(seed, 5), len(sel), 0, 5)
    d32 = np.float32(d)
    for j, i in enumerate(sel):
        b = border[j]
        v = [b, np.float32(b + d32), np.float32(b - d32),
             np.nextafter(np.float32(b + d32), np.float32(np.inf), dtype=np.float32),
             np.nextafter(b, np.float32(-np.inf), dtype=np.float32)][int(kind[j])]
        x[i] = np.float32(min(max(v, 0.0), W - 1.0))
    yaw = np.zeros(n, np.float32)
    present = np.ones(n, dtype=bool)
    gates = np.where(np.arange(n) % 5 == 4, 0, 1 + np.arange(n) % 3).astype(np.uint16)

    def owner(xs):
        return np.clip(np.floor(np.asarray(xs, np.float64) / strip_w).astype(np.int64), 0, ranks - 1)

    def walk(xv, zv, key, cnt):
        dx = rand_int(stream_key(seed, *key, 0), cnt, -step_q, step_q + 1)
        dz = rand_int(stream_key(seed, *key, 1), cnt, -step_q, step_q + 1)
        nx = np.clip(xv.astype(np.float64) + dx / Q, 0.0, W - 1.0).astype(np.float32)
        nz = np.clip(zv.astype(np.float64) + dz / Q, 0.0, height - 1.0).astype(np.float32)
        return nx, nz

    tr = StripTrace(n=n, d=float(d), ranks=ranks, strip_w=float(strip_w), max_step=float(max_step),
                    bounds=(0.0, 0.0, float(W), float(height)), gates=gates, ticks=[])
    ops = make_ops(n)
    ops["kind"] = OP_ENTER
    ops["sync_flags"] = SIF_OWN | SIF_NEIGHBOR
    ops["slot"] = np.arange(n, dtype=np.uint32)
    ops["x"], ops["z"], ops["yaw"] = x, z, yaw
    order = np.argsort(rand_u64(stream_key(seed, 6), n), kind="stable")
    tr.ticks.append((ops[order], owner(x[order])))
    for t in range(1, ticks):
        u = rand_unit(stream_key(seed, 100, t), n)
        v = rand_unit(stream_key(seed, 101, t), n)
        own0 = owner(x)
        rows1, rows2 = [], []                 # first / second op of an entity

        def emit(rows, k, f, ids, xs, zs, ys):
            o = make_ops(len(ids))
            o["kind"], o["sync_flags"], o["slot"] = k, f, ids
            o["x"], o["z"], o["yaw"] = xs, zs, ys
            rows.append(o)
        ids = np.arange(n)
        pres = present.copy()
        # plain moves (one or two per tick, half a step each)
        mv = ids[pres & (u < move_frac)]
        nx, nz = walk(x[mv], z[mv], (102, t), len(mv))
        x[mv], z[mv] = nx, nz
        emit(rows1, OP_MOVED, np.where(v[mv] < 0.5, SIF_NEIGHBOR, SIF_NEIGHBOR | SIF_OWN), mv, nx, nz, yaw[mv])
        two = mv[v[mv] < 0.15]
        nx, nz = walk(x[two], z[two], (103, t), len(two))
        x[two], z[two] = nx, nz
        emit(rows2, OP_MOVED, 0, two, nx, nz, yaw[two])
        # sync-only ops (SetYaw)
        sy = ids[pres & (u >= move_frac) & (u < move_frac + 0.1)]
        yaw[sy] = (v[sy] * 6.25).astype(np.float32)
        emit(rows1, OP_SYNC, np.where(v[sy] < 0.3, SIF_OWN, SIF_NEIGHBOR | SIF_OWN), sy, x[sy], z[sy], yaw[sy])
        if teleports:
            # candidates: present, no other op this tick; far jumps; no two
            # jumpers within 2d + 2 max_step of each other (old or new position)
            cand = ids[pres & (u >= move_frac + 0.1) & (u < 0.97)]
            cand = cand[np.argsort(rand_u64(stream_key(seed, 109, t), len(cand)), kind="stable")]
            tx = (rand_int(stream_key(seed, 110, t), len(cand), lo_q, hi_q) / Q).astype(np.float32)
            tz = (rand_int(stream_key(seed, 111, t), len(cand), zlo_q, zhi_q) / Q).astype(np.float32)
            sep = 2 * d + 2 * max_step + 1
            taken_x, taken_z, jumps = [], [], []
            for j, i in enumerate(cand.tolist()):
                if len(jumps) == teleports:
                    break
                if abs(float(tx[j]) - float(x[i])) <= 2 * d + 4 * max_step:
                    continue                                   # a short jump: not a teleport
                pts = [(float(x[i]), float(z[i])), (float(tx[j]), float(tz[j]))]
                if any(abs(px - qx) <= sep and abs(pz - qz) <= sep
                       for px, pz in pts for qx, qz in zip(taken_x, taken_z)):
                    continue
                taken_x += [p[0] for p in pts]
                taken_z += [p[1] for p in pts]
                jumps.append(j)
            jumps = np.array(jumps, np.int64)
            tp = cand[jumps]
            x[tp], z[tp] = tx[jumps], tz[jumps]
            emit(rows1, OP_MOVED, SIF_NEIGHBOR | SIF_OWN, tp, x[tp], z[tp], yaw[tp])
        if groups:
            taken = set(tp.tolist()) if teleports else set()
            cand = [i for i in ids[pres & (u >= move_frac + 0.1) & (u < 0.97)].tolist() if i not in taken]
            perm = np.argsort(rand_u64(stream_key(seed, 112, t), len(cand)), kind="stable")
            cand = [cand[k] for k in perm.tolist()]
            far = 2 * d + 4 * max_step
            rx = rand_int(stream_key(seed, 113, t), 64 * groups, lo_q, hi_q) / Q
            rz = rand_int(stream_key(seed, 114, t), 64 * groups, zlo_q, zhi_q) / Q
            ro = (rand_int(stream_key(seed, 115, t), 64 * groups, -int(d / 2 * Q), int(d / 2 * Q) + 1) / Q)
            draw = iter(range(64 * groups))
            used, gids, gx, gz = set(), [], [], []

            def far_spot(i):                       # a random place a teleport away from entity i
                for k in draw:
                    if abs(rx[k] - float(x[i])) > far:
                        return float(rx[k]), float(rz[k]), k
                return None
            for gi in range(groups):
                s0 = next((i for i in cand if i not in used), None)
                if s0 is None:
                    break
                mode = gi % 3
                if mode < 2:
                    mem = [s0] + [i for i in cand if i not in used and i != s0 and abs(float(x[i] - x[s0])) <= d
                                  and abs(float(z[i] - z[s0])) <= d][:2]
                else:
                    mem = [s0] + [i for i in cand if i not in used and i != s0 and
                                  abs(float(x[i] - x[s0])) > far + d][:1]
                spot = far_spot(s0)
                if spot is None or len(mem) < 2:
                    used.add(s0)
                    continue
                tx0, tz0, k0 = spot
                for j, i in enumerate(mem):
                    if mode == 0:                      # together: the same offset
                        nx_, nz_ = float(x[i]) + tx0 - float(x[s0]), float(z[i]) + tz0 - float(z[s0])
                    elif mode == 1 and j:              # split: a separate far place each
                        sp = far_spot(i)
                        if sp is None:
                            continue
                        nx_, nz_ = sp[0], sp[1]
                    elif mode == 2 and j:              # merge: next to the first one's destination
                        nx_, nz_ = tx0 + float(ro[k0]), tz0 + float(ro[(k0 + 1) % len(ro)])
                    else:
                        nx_, nz_ = tx0, tz0
                    nx_ = float(np.float32(min(max(nx_, 0.0), W - 1.0)))
                    nz_ = float(np.float32(min(max(nz_, 0.0), height - 1.0)))
                    if abs(nx_ - float(x[i])) <= far:     # clipped back near: not a teleport
                        continue
                    used.add(i)
                    gids.append(i); gx.append(nx_); gz.append(nz_)
                used.add(s0)
            if gids:
                gi_ = np.array(gids, np.int64)
                x[gi_] = np.array(gx, np.float32)
                z[gi_] = np.array(gz, np.float32)
                emit(rows1, OP_MOVED, SIF_NEIGHBOR | SIF_OWN, gi_, x[gi_], z[gi_], yaw[gi_])
        enter_owner = {}
        if churn:
            lv = ids[pres & (u >= 0.97) & (u < 0.985)]            # leave for a while
            emit(rows1, OP_LEAVE, 0, lv, x[lv], z[lv], yaw[lv])
            present[lv] = False
            rl = ids[pres & (u >= 0.985)]                        # leave + re-enter nearby
            emit(rows1, OP_LEAVE, 0, rl, x[rl], z[rl], yaw[rl])
            nx, nz = walk(x[rl], z[rl], (104, t), len(rl))
            x[rl], z[rl] = nx, nz
            emit(rows2, OP_ENTER, SIF_OWN | SIF_NEIGHBOR, rl, nx, nz, yaw[rl])
            back = ids[~pres & (u < 0.4)]                         # re-enter anywhere
            bx = (rand_int(stream_key(seed, 105, t), len(back), lo_q, hi_q) / Q).astype(np.float32)
            bz = (rand_int(stream_key(seed, 106, t), len(back), zlo_q, zhi_q) / Q).astype(np.float32)
            x[back], z[back] = bx, bz
            present[back] = True
            emit(rows1, OP_ENTER, SIF_OWN | SIF_NEIGHBOR, back, bx, bz, yaw[back])
            enter_owner = dict(zip(back.tolist(), owner(bx).tolist()))
        r1 = np.concatenate(rows1)
        r1 = r1[np.argsort(rand_u64(stream_key(seed, 107, t), len(r1)), kind="stable")]
        r2 = np.concatenate(rows2)
        r2 = r2[np.argsort(rand_u64(stream_key(seed, 108, t), len(r2)), kind="stable")]
        allops = np.concatenate([r1, r2])
        own = own0[allops["slot"]].copy()
        for k, i in enumerate(allops["slot"].tolist()):
            if i in enter_owner:
                own[k] = enter_owner[i]
        tr.ticks.append((allops, own))
    return tr


def walk_strip_trace(seed: int, n: int, side: float, ranks: int, ticks: int) -> StripTrace:
    """A config #5-shaped decomposed world at test scale: WorldWalk (uniform,
    dyadic, 10% movers per tick stepping +-4, reflected at the world border)
    shifted to [0, side)^2 and cut into `ranks` strips of side / ranks; tick 0
    enters everyone (id order), later ticks are the walk; each op tagged with
    the strip of the entity's x at the start of the tick."""
    w = WorldWalk(seed=seed, n=n, side=side)
    half = np.float32(side / 2)
    strip_w = side / ranks

    def owner(xs):
        return np.clip(np.floor(np.asarray(xs, np.float64) / strip_w).astype(np.int64), 0, ranks - 1)
    gates = np.where(np.arange(n) % 5 == 4, 0, 1 + np.arange(n) % 3).astype(np.uint16)
    tr = StripTrace(n=n, d=w.d, ranks=ranks, strip_w=float(strip_w), max_step=4.0,
                    bounds=(0.0, 0.0, float(side), float(side)), gates=gates, ticks=[])
    x0 = w.x() + half
    ops = enter_ops(np.arange(n, dtype=np.uint32), x0, np.zeros(n, np.float32), w.z() + half, w.yaw.copy())
    tr.ticks.append((ops, owner(x0)))
    for _ in range(1, ticks):
        ops, xb = w.next_tick()
        ops["x"] += half
        ops["z"] += half
        tr.ticks.append((ops, owner(xb + half)))
    return tr

