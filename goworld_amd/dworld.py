"""Decomposed world: one AOI space split into X-strips, one strip per process
(SURVEY.md 8(e) regime 2, BASELINE config #5).

The reference never splits a space across processes (one Space lives in one
game process, engine/entity/SpaceManager.go:11-31); this is the scale-out of
the same contract.  go-aoi's relation is a pure function of the two positions
and of which member made the later AOI call, so a strip needs
no neighbour lists from its neighbours, only the current state of the
entities near its borders:

* rank r OWNS the entities whose x lies in [lo_r, hi_r) and HOLDS, in one
  local space, every entity whose x lies in its extended range
  [lo_r - h, hi_r + h) (owned + ghosts), h = d + 2*max_step + margin;
* the owner (at the start of the tick) applies an entity's ops and forwards
  their NET effect to each neighbour whose extended range the entity is in
  before or after the tick, as up to three rows per entity, in order:
    LEAVE  (the entity left the space and came back inside the tick),
    ENTER / MOVED / LEAVE  (the net AOI change relative to that range; the
           payload and global stamp of the entity's last AOI op),
    SYNC   (the payload of its last non-Leave op and every sync flag still
           pending since the last collect);
  which reproduces exactly the state the engine keeps per entity (Space.go:
  196-250 via gw_op semantics: pos = last non-Leave op, AOI state and stamp =
  last AOI op, flags = OR since the last Leave);
* every op carries a global stamp (tick-major, then rank-major, then the op's
  index), so all ranks order the ops of all ranks the same way;
* after the tick a rank emits events only for watchers, and sync records only
  for entities, that it owns (gw_space_set_ownership).  An entity that
  crosses a border is a ghost of the new owner already, so its old relations
  are known where its events are computed.

Requirements (checked): a present entity moves at most max_step in x per tick;
strips are wider than h + max_step, so an entity is only ever held by its
owner and the owner's two neighbours.

On the GPU the routing is the engine's (gw_route_halo, halo.hip: the entity
state before the tick is the routing state; four light passes over the owned
ops, rows placed by wave-aggregated atomics into fixed-size NOP-padded
buffers, no host sync).  tests/torch_router.py restates the same protocol in
torch for the CPU tests' mock engine and as the row-for-row reference of the
HIP rows.  The halo exchange is torch.distributed point-to-point (RCCL over
xGMI with the nccl backend, gloo for the CPU tests); all AOI work is the HIP
engine's, on torch's stream (gw_set_stream).  Local slots are the global
entity ids (the local space's capacity is the world population).
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch

OP_NOP, OP_ENTER, OP_MOVED, OP_LEAVE, OP_SYNC = 0, 1, 2, 3, 4
SIF_MASK = 3            # GW_SIF_OWN_CLIENT | GW_SIF_NEIGHBOR_CLIENTS (include/gpuaoi.h)
OP_WORDS = 6            # gw_op as 6 int32 words: kind | flags<<8, slot, x, y, z, yaw
ROW_WORDS = 8           # + the u64 stamp
ROWS_PER_ENTITY = 3
STAMP_STRIDE = 1 << 26  # stamp = 1 + (tick * ranks + rank) * STAMP_STRIDE + op index


@dataclasses.dataclass
class Strips:
    """Geometry: strip r = [x0 + r*w, x0 + (r+1)*w); the outer strips extend
    to infinity."""
    x0: float
    w: float
    ranks: int
    d: float
    max_step: float

    def __post_init__(self):
        if self.ranks > 2 and not self.w > self.h + self.max_step:
            raise ValueError(f"strip width {self.w} must exceed halo {self.h} + max_step {self.max_step}")

    @property
    def h(self) -> float:
        # a relation needs |dx| <= d (+ float32 rounding of c +- d); an entity
        # that crossed a border moved <= max_step, so its old neighbours lie
        # within d + max_step of the strip; one more max_step for their moves
        return float(self.d + 2 * self.max_step + 1.0 + 1e-5 * (abs(self.x0) + self.ranks * self.w))

    def lo(self, r: int) -> float:
        return -np.inf if r == 0 else self.x0 + r * self.w

    def hi(self, r: int) -> float:
        return np.inf if r == self.ranks - 1 else self.x0 + (r + 1) * self.w

    def ext(self, r: int) -> tuple[float, float]:
        return self.lo(r) - self.h, self.hi(r) + self.h

    def owner(self, x) -> np.ndarray:
        r = np.floor((np.asarray(x, np.float64) - self.x0) / self.w).astype(np.int64)
        return np.clip(r, 0, self.ranks - 1)

    def own_range_f32(self, r: int) -> tuple[float, float]:
        """[lo, hi) as float32 bounds with the same membership for float32 x."""
        def f(v, side):
            if not np.isfinite(v):
                return float(np.float32(-3.0e38 if side < 0 else 3.0e38))
            v32 = np.float32(v)
            # smallest float32 >= v (x >= lo  <=>  x >= that float32)
            if float(v32) < v:
                v32 = np.nextafter(v32, np.float32(np.inf), dtype=np.float32)
            return float(v32)
        return f(self.lo(r), -1), f(self.hi(r), 1)


def stamps_for(tick: int, rank: int, ranks: int, n: int, device) -> torch.Tensor:
    if n >= STAMP_STRIDE:
        raise ValueError("too many ops in one tick for the stamp layout")
    base = 1 + (tick * ranks + rank) * STAMP_STRIDE
    return torch.arange(base, base + n, dtype=torch.int64, device=device)


def ops_to_words(ops: np.ndarray) -> np.ndarray:
    """gw_op structured array -> (n, 6) int32 words (same bytes)."""
    return np.ascontiguousarray(ops).view(np.int32).reshape(-1, OP_WORDS)


def words_to_ops(words: np.ndarray) -> np.ndarray:
    from .traces import OP_DTYPE
    return np.ascontiguousarray(words, dtype=np.int32).reshape(-1).view(OP_DTYPE)


class HipRouter:
    """The routing on the GPU: gw_route_halo of the rank's engine context
    writes the rows of both neighbours into persistent torch buffers."""

    def __init__(self, g, geom: Strips, rank: int, device, halo_cap: int):
        self.g, self.geom, self.r, self.K = g, geom, rank, halo_cap
        self.bufs, self.dsts = [], []
        for nb in (rank - 1, rank + 1):
            if 0 <= nb < geom.ranks:
                b = torch.zeros((halo_cap * ROWS_PER_ENTITY, ROW_WORDS), dtype=torch.int32, device=device)
                lo, hi = geom.ext(nb)
                self.bufs.append(b)
                self.dsts.append((float(np.float32(lo)), float(np.float32(hi)), b.data_ptr(), halo_cap))
            else:
                self.bufs.append(None)

    def route(self, words: torch.Tensor, stamps: torch.Tensor, cap: int | None = None):
        if not self.dsts:
            return None, None            # a one-strip world has no neighbours
        cap = self.K if cap is None else min(cap, self.K)
        self.g.route_halo(words.data_ptr(), stamps.data_ptr(), words.shape[0], float(self.geom.max_step),
                          [(lo, hi, p, cap) for lo, hi, p, _ in self.dsts])
        return tuple(None if b is None else b[:cap * ROWS_PER_ENTITY] for b in self.bufs)

    def receive(self, buf):
        pass                        # the engine's own state is the routing state

    def collected(self):
        pass

    def status(self):
        return self.g.halo_status()


def exchange(pg, rank: int, ranks: int, send_left, send_right, nrows: int, device, comm_device):
    """Halo exchange with both neighbours (point-to-point, one round)."""
    import torch.distributed as dist
    shape = (nrows, ROW_WORDS)
    mv = (lambda t: t) if comm_device == device else (lambda t: t.to(comm_device))
    recv = {}
    ops = []
    for nb, send in ((rank - 1, send_left), (rank + 1, send_right)):
        if 0 <= nb < ranks:
            recv[nb] = torch.empty(shape, dtype=torch.int32, device=comm_device)
            ops.append(dist.P2POp(dist.isend, mv(send).contiguous(), nb, group=pg))
            ops.append(dist.P2POp(dist.irecv, recv[nb], nb, group=pg))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    back = (lambda t: t) if comm_device == device else (lambda t: t.to(device))
    return [back(recv[nb]) for nb in (rank - 1, rank + 1) if nb in recv]


class HipStrip:
    """Engine adapter: a gpuaoi.GpuAOI context sharing one stream with torch
    (made torch's current stream), so routing kernels, collectives and AOI
    kernels are ordered without host syncs.  Routing: HipRouter."""

    def __init__(self, g):
        self.g = g
        self._keep = []
        self.stream = torch.cuda.Stream()
        torch.cuda.set_stream(self.stream)
        g.set_stream(self.stream.cuda_stream)

    def create_space(self, d, cap, bounds):
        return self.g.create_space(d, cap, bounds)

    def set_ownership(self, sid, lo, hi):
        self.g.set_ownership(sid, lo, hi)

    def set_clients(self, slots, gates):
        self.g.set_clients(slots, gates)

    def make_router(self, geom, rank, n_global, device, halo_cap):
        return HipRouter(self.g, geom, rank, device, halo_cap)

    def submit(self, words: torch.Tensor, stamps: torch.Tensor):
        words, stamps = words.contiguous(), stamps.contiguous()
        self._keep += [words, stamps]        # alive until the tick has consumed them
        self.g.submit_device_stamped(words.data_ptr(), stamps.data_ptr(), words.shape[0])

    def submit_rows(self, rows: torch.Tensor):
        rows = rows.contiguous()
        self._keep.append(rows)
        self.g.submit_device_rows(rows.data_ptr(), rows.shape[0])

    def tick(self, copy=True, no_events=False, defer=False):
        res = self.g.tick(copy=copy, no_events=no_events, defer=defer)
        if not defer or copy:
            self._keep = []          # consumed (a deferred tick keeps them until its collect)
        return res

    def tick_result(self):
        return self.g.tick_result()

    def collect(self, copy=True):
        res = self.g.sync_collect(copy=copy)     # settles a deferred tick
        self._keep = []
        return res


class StripRank:
    """One rank of a decomposed world.  `engine` follows HipStrip's interface
    (make_router / create_space / set_ownership / set_clients / submit /
    submit_rows / tick / collect)."""

    def __init__(self, engine, geom: Strips, rank: int, n_global: int, bounds, device,
                 pg=None, comm_device=None, halo_cap: int = 1 << 14, halo_cap_max: int | None = None):
        """halo_cap: entities per neighbour per tick (steady state); a call may
        ask for up to halo_cap_max (e.g. the ticks that load the population)."""
        self.e, self.g, self.r = engine, geom, rank
        self.dev = device
        self.pg = pg
        self.cdev = comm_device if comm_device is not None else device
        self.cap = halo_cap
        self.router = engine.make_router(geom, rank, n_global, device, max(halo_cap, halo_cap_max or 0))
        self.sid, base = engine.create_space(geom.d, n_global, bounds)
        if base != 0:
            raise ValueError("a strip rank holds one space per context (local slot = global id)")
        engine.set_ownership(self.sid, *geom.own_range_f32(rank))
        self.tick_no = 0

    def submit(self, words: torch.Tensor, cap: int | None = None):
        """Queue this rank's owned ops of one tick (int32 (m, 6) gw_op words on
        the device, in call order), route and exchange the halo rows (cap:
        entities per neighbour for this tick; every rank must pass the same)."""
        m = words.shape[0]
        cap = min(self.cap if cap is None else cap, self.router.K)
        st = stamps_for(self.tick_no, self.r, self.g.ranks, m, self.dev)
        sl, sr = self.router.route(words, st, cap)
        nrows = cap * ROWS_PER_ENTITY
        if self.g.ranks > 1:
            recvd = exchange(self.pg, self.r, self.g.ranks, sl, sr, nrows, self.dev, self.cdev)
        else:
            recvd = []
        self.e.submit(words, st)
        for buf in recvd:
            self.router.receive(buf)
            self.e.submit_rows(buf)
        self.tick_no += 1

    def tick(self, copy=True, **kw):
        return self.e.tick(copy=copy, **kw)

    def step(self, words: torch.Tensor, copy=True, cap: int | None = None, **kw):
        self.submit(words, cap)
        return self.tick(copy=copy, **kw)

    def collect(self, copy=True):
        res = self.e.collect(copy=copy)
        self.router.collected()
        return res

    def check(self):
        """Host check of the contract counters (one sync; call outside timed loops)."""
        ov, bad, bad_ops = self.router.status()
        if ov > 0:
            raise RuntimeError(f"halo buffers overflowed by {ov} entities (raise halo_cap)")
        if bad:
            raise RuntimeError(f"{bad} owned entities moved more than max_step in one tick")
        if bad_ops:
            raise RuntimeError(f"{bad_ops} ops with an invalid slot or kind")
