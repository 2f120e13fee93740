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
HIP rows.  The halo exchange runs inside the library over its RCCL
communicator (gw_comm_init + gw_world_step: row counts, one host sync, then
exactly the used rows, grouped ncclSend/ncclRecv with both neighbours on the
context's stream over xGMI), or over a torch.distributed group for the CPU
tests and one-GPU rehearsals (gloo, exchange_rows).  All AOI work is the HIP
engine's.  Local slots are the global entity ids (the local space's capacity
is the world population).
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
RES_LONG = 1            # gw_op.reserved bit of a halo row: the entity moved more than max_step this tick


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


def exchange_rows(pg, rank: int, ranks: int, sends, device, comm_device):
    """Host-transport halo exchange with both neighbours (torch.distributed
    point-to-point; gloo for the CPU tests and the one-GPU rehearsals): the
    row counts first, then exactly the used rows.  sends: [to_left, to_right]
    int32 (rows, 8) tensors (None where there is no neighbour).  Returns the
    received [from_left, from_right] on `device`."""
    import torch.distributed as dist
    mv = (lambda t: t) if comm_device == device else (lambda t: t.to(comm_device))
    nbs = [(0, rank - 1), (1, rank + 1)]
    nbs = [(side, nb) for side, nb in nbs if 0 <= nb < ranks]
    cnt_in = {side: torch.zeros(1, dtype=torch.int64) for side, _ in nbs}
    ops = []
    for side, nb in nbs:
        rows = 0 if sends[side] is None else int(sends[side].shape[0])
        ops.append(dist.P2POp(dist.isend, torch.tensor([rows], dtype=torch.int64), nb, group=pg))
        ops.append(dist.P2POp(dist.irecv, cnt_in[side], nb, group=pg))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    recv = [None, None]
    ops = []
    for side, nb in nbs:
        n_in = int(cnt_in[side].item())
        if sends[side] is not None and sends[side].shape[0]:
            ops.append(dist.P2POp(dist.isend, mv(sends[side]).contiguous(), nb, group=pg))
        if n_in:
            recv[side] = torch.empty((n_in, ROW_WORDS), dtype=torch.int32, device=comm_device)
            ops.append(dist.P2POp(dist.irecv, recv[side], nb, group=pg))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    back = (lambda t: t) if comm_device == device else (lambda t: t.to(device))
    return [None if r is None else back(r) for r in recv]


def exchange_far(pg, rank: int, ranks: int, far: dict, device, comm_device):
    """Host-transport exchange of the rows of long moves (teleports) with every
    rank (gloo for the CPU tests and one-GPU rehearsals): the (ranks x ranks)
    matrix of row counts first (all_gather), then exactly the used rows.
    far: {dest rank: (rows, 8) int32} (dest == rank: rows for this rank
    itself).  Returns the received row tensors on `device`, by source rank."""
    import torch.distributed as dist
    cnt = torch.zeros(ranks, dtype=torch.int64)
    for q, rows in far.items():
        cnt[q] = int(rows.shape[0])
    allc = [torch.zeros(ranks, dtype=torch.int64) for _ in range(ranks)]
    dist.all_gather(allc, cnt, group=pg)
    mv = (lambda t: t) if comm_device == device else (lambda t: t.to(comm_device))
    back = (lambda t: t) if comm_device == device else (lambda t: t.to(device))
    out, ops = [], []
    for p in range(ranks):
        n_in = int(allc[p][rank].item())
        if p == rank:
            if n_in:
                out.append(far[rank])
            continue
        if int(cnt[p].item()):
            ops.append(dist.P2POp(dist.isend, mv(far[p]).contiguous(), p, group=pg))
        if n_in:
            buf = torch.empty((n_in, ROW_WORDS), dtype=torch.int32, device=comm_device)
            ops.append(dist.P2POp(dist.irecv, buf, p, group=pg))
            out.append(buf)
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return [back(t) for t in out]


def exchange_longs(pg, rank: int, ranks: int, mine: np.ndarray) -> np.ndarray:
    """Host-transport all-gather of the long-mover lists (gw_long_move rows,
    group teleports; gloo for the CPU tests and one-GPU rehearsals): every
    rank's list, concatenated in rank order."""
    import torch.distributed as dist
    from .traces import LONG_DTYPE
    raw = torch.from_numpy(np.ascontiguousarray(mine, LONG_DTYPE).view(np.uint8).copy())
    cnt = torch.tensor([raw.numel()], dtype=torch.int64)
    allc = [torch.zeros(1, dtype=torch.int64) for _ in range(ranks)]
    dist.all_gather(allc, cnt, group=pg)
    mx = max(int(c.item()) for c in allc)
    if mx == 0:
        return np.zeros(0, LONG_DTYPE)
    pad = torch.zeros(mx, dtype=torch.uint8)
    pad[:raw.numel()] = raw
    bufs = [torch.zeros(mx, dtype=torch.uint8) for _ in range(ranks)]
    dist.all_gather(bufs, pad, group=pg)
    return np.concatenate([b[:int(c.item())].numpy() for b, c in zip(bufs, allc)]).view(LONG_DTYPE)


class HipStrip:
    """Engine adapter over the library's decomposed world (gw_world_*): a
    gpuaoi.GpuAOI context sharing one stream with torch (made torch's current
    stream), so routing kernels, exchanges and AOI kernels are ordered without
    host syncs beyond the library's own.  comm="rccl": the exchange runs inside
    the library over its RCCL communicator (gw_world_step); otherwise the rows
    travel over the caller's torch.distributed group (gw_world_route ->
    exchange_rows -> gw_world_submit)."""

    def __init__(self, g):
        self.g = g
        self._keep = []
        self.stream = torch.cuda.Stream()
        torch.cuda.set_stream(self.stream)
        g.set_stream(self.stream.cuda_stream)

    def create_world(self, geom: Strips, rank: int, n_global: int, bounds):
        return self.g.world_create(geom.x0, geom.w, geom.d, geom.max_step, geom.ranks, rank, n_global, bounds)

    def set_clients(self, slots, gates):
        self.g.set_clients(slots, gates)

    def step(self, words: torch.Tensor):
        words = words.contiguous()
        self._keep.append(words)                # alive until the tick has consumed it
        self.g.world_step(words.data_ptr(), words.shape[0])

    def route(self, words: torch.Tensor, stamps=None):
        words = words.contiguous()
        self._keep.append(words)
        out = []
        for ptr, rows in self.g.world_route(words.data_ptr(), words.shape[0]):
            if not ptr:
                out.append(None)
                continue
            buf = np.zeros((rows, ROW_WORDS), np.int32)
            if rows:
                self.g.d2h(buf, ptr)
            out.append(torch.from_numpy(buf))
        return out

    def far(self) -> dict:
        """Rows of the last route for ranks that are not neighbours (long
        moves), {rank: (rows, 8) int32 host tensor}."""
        out = {}
        for q, (ptr, rows) in self.g.world_far().items():
            buf = np.zeros((rows, ROW_WORDS), np.int32)
            self.g.d2h(buf, ptr)
            out[q] = torch.from_numpy(buf)
        return out

    def longs(self) -> np.ndarray:
        """This rank's long-mover list of the last route (gw_long_move rows, host copy)."""
        from .traces import LONG_DTYPE
        ptr, n = self.g.world_longs()
        out = np.zeros(n, LONG_DTYPE)
        if n:
            self.g.d2h(out, ptr)
        return out

    def submit(self, words: torch.Tensor, stamps, recvd, far_in=(), longs=None):
        rows = []
        dev = torch.device("cuda", torch.cuda.current_device())
        for r in recvd:
            if r is None or r.shape[0] == 0:
                rows.append((0, 0))
                continue
            r = r.to(device=dev, dtype=torch.int32).contiguous()
            self._keep.append(r)
            rows.append((r.data_ptr(), r.shape[0]))
        self.g.world_submit(rows)
        for r in far_in:
            if r is None or r.shape[0] == 0:
                continue
            r = r.to(device=dev, dtype=torch.int32).contiguous()
            self._keep.append(r)
            self.g.world_submit_far(r.data_ptr(), r.shape[0])
        if longs is not None and len(longs):           # every rank's long-mover list for the tick
            t = torch.from_numpy(np.ascontiguousarray(longs).view(np.uint8).copy()).to(dev)
            self._keep.append(t)
            self.g.world_submit_longs(t.data_ptr(), len(longs))

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

    def collected(self):
        pass

    def status(self):
        return self.g.world_status()


class StripRank:
    """One rank of a decomposed world.  `engine` follows HipStrip's interface
    (create_world / set_clients / route / submit / [step] / tick / collect /
    status); comm = "rccl" (HIP engine: exchange inside the library) or
    "torch" (exchange_rows over the process group `pg`)."""

    def __init__(self, engine, geom: Strips, rank: int, n_global: int, bounds, device,
                 pg=None, comm: str = "torch", comm_device=None):
        self.e, self.g, self.r = engine, geom, rank
        self.dev = device
        self.pg = pg
        self.comm = comm
        self.cdev = comm_device if comm_device is not None else device
        self.sid = engine.create_world(geom, rank, n_global, bounds)
        self.tick_no = 0

    def submit(self, words: torch.Tensor):
        """Queue this rank's owned ops of one tick (int32 (m, 6) gw_op words on
        the device, in call order): route, exchange the halo rows with both
        neighbours, queue own ops + received rows."""
        m = words.shape[0]
        if self.comm == "rccl":
            self.e.step(words)
        else:
            st = stamps_for(self.tick_no, self.r, self.g.ranks, m, self.dev)
            sends = self.e.route(words, st)
            far = self.e.far()
            lg = self.e.longs()
            if self.g.ranks > 1:
                recvd = exchange_rows(self.pg, self.r, self.g.ranks, sends, self.dev, self.cdev)
                far_in = exchange_far(self.pg, self.r, self.g.ranks, far, self.dev, self.cdev)
                lg = exchange_longs(self.pg, self.r, self.g.ranks, lg)
            else:
                recvd = [None, None]
                far_in = [far[self.r]] if self.r in far else []
            self.e.submit(words, st, recvd, far_in, longs=lg)
        self.tick_no += 1

    def tick(self, copy=True, **kw):
        return self.e.tick(copy=copy, **kw)

    def step(self, words: torch.Tensor, copy=True, **kw):
        self.submit(words)
        return self.tick(copy=copy, **kw)

    def collect(self, copy=True):
        res = self.e.collect(copy=copy)
        self.e.collected()
        return res

    def check(self):
        """Host check of the contract counters (one sync; call outside timed loops)."""
        ov, conflicts, bad_ops = self.e.status()
        if ov > 0:
            raise RuntimeError(f"halo buffers overflowed by {ov} entities")
        if conflicts:
            raise RuntimeError(f"{conflicts} long-move conflicts (pairs of related entities that both moved more "
                               f"than max_step in one tick)")
        if bad_ops:
            raise RuntimeError(f"{bad_ops} ops with an invalid slot or kind")


class LocalWorld:
    """R strip contexts of one decomposed world in ONE process on one device
    (gw_world_create each), the halo rows handed from rank to rank by pointer:
    rank r+1's send buffer is rank r's receive buffer (gw_world_route ->
    gw_world_submit, no copy).  Used to rehearse the N-GPU world on the one
    MI355X (tools/sim_ranks.py) and to check config #5 at its full size
    against a single context (tests/test_gpu_golden.py).  x0/z0/yaw0: the
    world's initial population; each rank enters the entities it owns, routed
    to its neighbours as ghosts, in the same number of chunks everywhere."""

    def __init__(self, R, n, side, max_step, x0, z0, yaw0, device=0, gates=None, d=100.0):
        from . import gpuaoi, traces
        self.R = R
        self.geom = geom = Strips(-side / 2, side / R, R, d, max_step)
        self.g = []
        gates = np.ones(n, np.uint16) if gates is None else gates
        for r in range(R):
            g = gpuaoi.GpuAOI(device)
            lo, hi = geom.ext(r)
            bounds = (max(lo, -side / 2), -side / 2, min(hi, side / 2), side / 2)
            g.world_create(geom.x0, geom.w, geom.d, geom.max_step, R, r, n, bounds)
            g.set_clients(np.arange(n, dtype=np.uint32), gates)
            self.g.append(g)
        self.bufs = []
        owner0 = geom.owner(x0)
        chunk = 1 << 21
        n_chunks = max(1, -(-int(np.bincount(owner0, minlength=R).max()) // chunk))
        enters = []
        for r in range(R):
            mine = np.nonzero(owner0 == r)[0].astype(np.uint32)
            enters.append(traces.enter_ops(mine, x0[mine], np.zeros(len(mine), np.float32), z0[mine], yaw0[mine]))
        for k in range(n_chunks):
            parts = [e[k * chunk:(k + 1) * chunk] for e in enters]
            ptrs = [self.upload(r, p) for r, p in enumerate(parts)]
            self.route_submit(ptrs, [len(p) for p in parts])
            for g in self.g:
                g.tick(copy=False, no_events=True)
        for g in self.g:
            g.sync_collect(copy=False)

    def upload(self, r, ops):
        """ops of rank r into device memory (kept until close)."""
        ops = np.ascontiguousarray(ops)
        p = self.g[r].dev_alloc(max(ops.nbytes, 64))
        if ops.nbytes:
            self.g[r].h2d(p, ops)
        self.bufs.append((r, p))
        return p

    def split(self, ops, x_before):
        """A tick's world ops -> per-rank owned ops (the strip of x before the tick), in call order."""
        own = self.geom.owner(x_before)
        return [ops[own == r] for r in range(self.R)]

    def route_submit(self, ptrs, ms, times=None):
        """Route every rank's owned ops and queue them with its neighbours' rows;
        returns the halo rows moved.  times[r] += rank r's routing wall time."""
        import time
        if self.R == 1:                           # one strip: gw_world_step stamps and queues, no routing
            t0 = time.perf_counter()
            self.g[0].world_step(ptrs[0], ms[0])
            if times is not None:
                times[0] += time.perf_counter() - t0
            return 0
        sends = []
        for r, g in enumerate(self.g):
            g.synchronize()
            t0 = time.perf_counter()
            sends.append(g.world_route(ptrs[r], ms[r]))
            if times is not None:
                times[r] += time.perf_counter() - t0
        fars = [g.world_far() for g in self.g]                   # long moves: {dest: (ptr, rows)}
        lptr = self._longs_all()                                   # every rank's long-mover list
        rows = 0
        for r, g in enumerate(self.g):
            left = sends[r - 1][1] if r > 0 else (0, 0)           # left neighbour's rows to its right
            right = sends[r + 1][0] if r + 1 < self.R else (0, 0)
            rows += left[1] + right[1]
            g.world_submit([left, right])
            for p in range(self.R):
                if r in fars[p]:
                    ptr, n = fars[p][r]
                    g.world_submit_far(ptr, n)
                    rows += n
            if lptr[1]:
                g.world_submit_longs(*lptr)
        return rows

    def _longs_all(self):
        """The ranks' long-mover lists of the last route concatenated into one
        device buffer (all contexts share the device): (ptr, n)."""
        from .traces import LONG_DTYPE
        parts = []
        for g in self.g:
            ptr, n = g.world_longs()
            if n:
                a = np.zeros(n, LONG_DTYPE)
                g.d2h(a, ptr)
                parts.append(a)
        if not parts:
            return 0, 0
        allv = np.concatenate(parts)
        cap, ptr = getattr(self, "_lbuf", (0, 0))
        if allv.nbytes > cap:
            if ptr:
                self.g[0].dev_free(ptr)
            cap = 2 * allv.nbytes
            ptr = self.g[0].dev_alloc(cap)
            self._lbuf = (cap, ptr)
        self.g[0].h2d(ptr, allv)
        return ptr, len(allv)

    def check(self):
        for r, g in enumerate(self.g):
            ov, bad, bad_ops = g.world_status()
            if ov or bad or bad_ops:
                raise RuntimeError(f"rank {r}: contract counters {ov} {bad} {bad_ops}")

    def close(self):
        for r, p in self.bufs:
            self.g[r].dev_free(p)
        self.bufs = []
        if getattr(self, "_lbuf", (0, 0))[1]:
            self.g[0].dev_free(self._lbuf[1])
            self._lbuf = (0, 0)
        for g in self.g:
            g.close()


class _RankThread:
    """A persistent host thread driving one rank's context (a rank process
    drives its context from one thread; the library's calls on it are
    blocking and release the GIL, so the R threads run their calls
    concurrently)."""

    def __init__(self, r):
        import queue
        import threading
        self.q_in, self.q_out = queue.Queue(), queue.Queue()
        self.t = threading.Thread(target=self._loop, name=f"gw-rank-{r}", daemon=True)
        self.t.start()

    def _loop(self):
        while True:
            job = self.q_in.get()
            if job is None:
                return
            fn, args = job
            try:
                self.q_out.put((True, fn(*args)))
            except BaseException as e:            # handed to the caller of run()
                self.q_out.put((False, e))

    def stop(self):
        self.q_in.put(None)
        self.t.join(timeout=30)


class LoopbackWorld:
    """R strip contexts of one decomposed world in ONE process, each driven by
    its own host thread through gw_world_step over the library's loopback
    transport (gw_comm_init_local): the exact call sequence R rank processes
    run over RCCL (route, count round, host read of the counts, far-count
    all-gather at R >= 3, exact-size rows and far rows, queue), with the bytes
    moved by copies between the contexts on the one device.  run(fn) calls
    fn(r, g) on every rank's thread at once and returns the R results."""

    def __init__(self, geom: Strips, n_global: int, bounds, device: int = 0, gates=None):
        from . import gpuaoi
        self.R, self.geom, self.n = geom.ranks, geom, n_global
        self.g = [gpuaoi.GpuAOI(device) for _ in range(self.R)]
        self.th = []
        try:
            for r, g in enumerate(self.g):
                lo, hi = geom.ext(r)
                b = (max(lo, bounds[0]), bounds[1], min(hi, bounds[2]), bounds[3])
                g.world_create(geom.x0, geom.w, geom.d, geom.max_step, self.R, r, n_global, b)
                g.set_clients(np.arange(n_global, dtype=np.uint32),
                              np.ones(n_global, np.uint16) if gates is None else gates)
            gpuaoi.comm_init_local(self.g)
            self.th = [_RankThread(r) for r in range(self.R)]
        except BaseException:
            self.close()
            raise
        self.bufs = []

    def run(self, fn, *args):
        for r, th in enumerate(self.th):
            th.q_in.put((fn, (r, self.g[r]) + args))
        out, err = [], None
        for th in self.th:                          # every rank's result, then the first error
            ok, v = th.q_out.get()
            out.append(v if ok else None)
            if not ok and err is None:
                err = v
        if err is not None:
            raise err
        return out

    def upload(self, r, ops) -> int:
        """ops (gw_op array) of rank r into device memory (kept until close); returns the pointer."""
        ops = np.ascontiguousarray(ops)
        p = self.g[r].dev_alloc(max(ops.nbytes, 64))
        if ops.nbytes:
            self.g[r].h2d(p, ops)
        self.bufs.append((r, p))
        return p

    def load(self, x0, z0, yaw0, chunk: int = 1 << 21):
        """Every rank enters the entities it owns (routed to its neighbours as
        ghosts) through gw_world_step, no events, in the same number of chunks."""
        from . import traces
        owner0 = self.geom.owner(x0)
        n_chunks = max(1, -(-int(np.bincount(owner0, minlength=self.R).max()) // chunk))
        ptrs = []
        for r in range(self.R):
            mine = np.nonzero(owner0 == r)[0].astype(np.uint32)
            ops = traces.enter_ops(mine, x0[mine], np.zeros(len(mine), np.float32), z0[mine], yaw0[mine])
            ptrs.append([(self.upload(r, ops[k * chunk:(k + 1) * chunk]), len(ops[k * chunk:(k + 1) * chunk]))
                         for k in range(n_chunks)])

        def one(r, g):
            for p, m in ptrs[r]:
                g.world_step(p, m)
                g.tick(copy=False, no_events=True)
            g.sync_collect(copy=False)
        self.run(one)

    def check(self):
        """Contract counters summed over the ranks (gw_world_status is a collective)."""
        st = self.run(lambda r, g: g.world_status())
        ov, conflicts, bad_ops = st[0]
        if ov or conflicts or bad_ops:
            raise RuntimeError(f"world contract counters: overflow {ov}, conflicts {conflicts}, bad ops {bad_ops}")

    def close(self):
        for th in self.th:
            th.stop()
        self.th = []
        for r, p in getattr(self, "bufs", []):
            self.g[r].dev_free(p)
        self.bufs = []
        for g in self.g:
            g.close()
        self.g = []
