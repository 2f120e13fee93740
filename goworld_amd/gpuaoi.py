"""ctypes binding of the C ABI in include/gpuaoi.h (libgpuaoi.so).

This is the Python-side host of the drop-in boundary, used by tests/ and
bench.py.  It mirrors the reference's calls one to one:

  GpuAOI.create_space(d, ...)   <- Space.EnableAOI(d)          (engine/entity/Space.go:91-106)
  GpuAOI.submit(ops)            <- aoiMgr.Enter/Moved/Leave    (Space.go:201-203, 233-235, 250)
  GpuAOI.tick()                 <- OnEnterAOI/OnLeaveAOI fan-out (Entity.go:227-246), batched
  GpuAOI.sync_collect()         <- CollectEntitySyncInfos       (Entity.go:1221-1267)
  GpuAOI.neighbors(slot)        <- Entity.InterestedIn / InterestedBy (Entity.go:53-54)

There is no CPU fallback: if the HIP library is missing or a call fails, an
exception is raised (errors map to the reference's gwlog.Panicf on misuse).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os

import numpy as np

from .traces import LONG_DTYPE, OP_DTYPE

_HERE = os.path.dirname(os.path.abspath(__file__))
# GW_LIB_PATH selects another build of the same library (A/B experiments)
LIB_PATH = os.environ.get("GW_LIB_PATH") or os.path.join(_HERE, "lib", "libgpuaoi.so")

EVENT_DTYPE = np.dtype([("watcher", "<u4"), ("target", "<u4")])
REC_DTYPE = np.dtype([("watcher", "<u4"), ("entity", "<u4"), ("x", "<f4"), ("y", "<f4"),
                      ("z", "<f4"), ("yaw", "<f4")])

FANOUT_DTYPE = np.dtype([("watcher", "<u4"), ("entity", "<u4"), ("item", "<u4")])

TICK_COPY_TO_HOST, TICK_NO_EVENTS, TICK_DEFER = 1, 2, 4
MSG_COPY_TO_HOST = 1
SYNC_COPY_TO_HOST, SYNC_BY_CLIENT = 1, 2
MAX_STAGES = 32

_u64, _u32, _f64 = C.c_uint64, C.c_uint32, C.c_double


class ReplaySum(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("ops", "movers", "n_enter", "n_leave", "n_rec", "pairs_tested",
                                          "nbr_old", "nbr_new", "bytes_alg")]


class TickOut(C.Structure):
    _fields_ = [("enter", C.c_void_p), ("leave", C.c_void_p), ("enter_dev", C.c_void_p),
                ("leave_dev", C.c_void_p), ("n_enter", _u64), ("n_leave", _u64), ("ops", _u64),
                ("movers", _u64), ("pairs_tested", _u64), ("nbr_old", _u64), ("nbr_new", _u64),
                ("bytes_alg", _u64), ("device_us", _f64)]


class SyncOut(C.Structure):
    _fields_ = [("rec", C.c_void_p), ("rec_dev", C.c_void_p), ("n_rec", _u64),
                ("gate_off", C.POINTER(_u64)), ("n_gates", _u32), ("flagged", _u64),
                ("bytes_alg", _u64), ("device_us", _f64), ("n_clients", _u32),
                ("client_slot", C.POINTER(_u32)), ("client_off", C.POINTER(_u64)),
                ("client_slot_dev", C.c_void_p), ("client_off_dev", C.c_void_p)]


class MsgOut(C.Structure):
    _fields_ = [("rec", C.c_void_p), ("rec_dev", C.c_void_p), ("n_rec", _u64), ("gate_off", C.POINTER(_u64)),
                ("n_gates", _u32), ("bytes_alg", _u64), ("device_us", _f64)]


class StageTimes(C.Structure):
    _fields_ = [("n", _u32), ("name", C.c_char_p * MAX_STAGES), ("us", _f64 * MAX_STAGES),
                ("bytes_alg", _u64 * MAX_STAGES), ("calls", _u32 * MAX_STAGES)]


class HaloDst(C.Structure):
    _fields_ = [("x_lo", C.c_float), ("x_hi", C.c_float), ("rows", C.c_void_p), ("cap_entities", _u32),
                ("reserved", _u32)]


class Xfer(C.Structure):
    _fields_ = [("peer", C.c_int32), ("reserved", _u32), ("send", C.c_void_p), ("send_bytes", _u64),
                ("recv", C.c_void_p), ("recv_bytes", _u64)]


class WorldGeom(C.Structure):
    _fields_ = [("x0", C.c_float), ("strip_w", C.c_float), ("aoi_dist", C.c_float), ("max_step", C.c_float),
                ("ranks", _u32), ("rank", _u32)]


class CtxInfo(C.Structure):
    _fields_ = [("total_slots", _u32), ("live_slots", _u32), ("total_cells", _u32), ("live_cells", _u32),
                ("live_spaces", _u32), ("reserved", _u32)]


COMM_ID_BYTES = 128
RED_SUM, RED_MAX = 0, 1


class WireOut(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("bytes_dev", C.c_void_p), ("n_bytes", _u64), ("n_packets", _u32),
                ("gate", C.POINTER(C.c_uint16)), ("off", C.POINTER(_u64)), ("device_us", _f64)]


class GwError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gpuaoi error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load libgpuaoi.so; raises if it was not built (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make` (HIP/gfx950); "
                               "there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.gw_abi_version.restype = C.c_int
        L.gw_init.argtypes = [C.c_int, C.POINTER(vp)]
        L.gw_shutdown.argtypes = [vp]
        L.gw_shutdown.restype = None
        L.gw_last_error.argtypes = [vp]
        L.gw_last_error.restype = C.c_char_p
        L.gw_space_create.argtypes = [vp, C.c_float, _u32, vp, C.POINTER(_u32), C.POINTER(_u32)]
        L.gw_space_destroy.argtypes = [vp, _u32]
        L.gw_space_grow.argtypes = [vp, _u32, _u32, C.POINTER(_u32)]
        L.gw_context_info.argtypes = [vp, C.POINTER(CtxInfo)]
        L.gw_submit.argtypes = [vp, vp, _u32]
        L.gw_submit_device.argtypes = [vp, vp, _u32]
        L.gw_set_clients.argtypes = [vp, vp, vp, _u32]
        L.gw_tick.argtypes = [vp, _u32, C.POINTER(TickOut)]
        L.gw_tick_result.argtypes = [vp, C.POINTER(TickOut)]
        L.gw_space_restore.argtypes = [vp, _u32, vp, vp, vp, vp, vp, _u32, C.c_uint8]
        L.gw_sync_collect.argtypes = [vp, _u32, C.POINTER(SyncOut)]
        L.gw_step.argtypes = [vp, vp, _u32, C.c_int, _u32, _u32, C.POINTER(TickOut), C.POINTER(SyncOut)]
        L.gw_replay.argtypes = [vp, vp, _u32, C.c_uint64, _u32, _u32, C.POINTER(ReplaySum)]
        L.gw_neighbors.argtypes = [vp, _u32, vp, _u32, C.POINTER(_u32)]
        L.gw_set_profiling.argtypes = [vp, C.c_int]
        L.gw_get_stage_times.argtypes = [vp, C.POINTER(StageTimes)]
        L.gw_total_neighbors.argtypes = [vp, C.POINTER(_u64)]
        L.gw_device_alloc.argtypes = [vp, C.c_size_t, C.POINTER(vp)]
        L.gw_device_free.argtypes = [vp, vp]
        L.gw_memcpy_h2d.argtypes = [vp, vp, vp, C.c_size_t]
        L.gw_memcpy_d2h.argtypes = [vp, vp, vp, C.c_size_t]
        L.gw_synchronize.argtypes = [vp]
        L.gw_submit_device_stamped.argtypes = [vp, vp, vp, _u32]
        L.gw_space_set_ownership.argtypes = [vp, _u32, C.c_float, C.c_float]
        L.gw_set_stream.argtypes = [vp, vp]
        L.gw_route_halo.argtypes = [vp, vp, vp, _u32, C.c_float, C.POINTER(HaloDst), _u32]
        L.gw_submit_device_rows.argtypes = [vp, vp, _u32]
        L.gw_halo_status.argtypes = [vp, C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u64)]
        L.gw_client_events.argtypes = [vp, _u32, C.POINTER(MsgOut), C.POINTER(MsgOut)]
        L.gw_fanout.argtypes = [vp, vp, _u32, _u32, C.POINTER(MsgOut)]
        L.gw_comm_unique_id.argtypes = [vp]
        L.gw_comm_init.argtypes = [vp, vp, C.c_int, C.c_int]
        L.gw_comm_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.gw_comm_init_local.argtypes = [C.POINTER(vp), C.c_int]
        L.gw_comm_exchange.argtypes = [vp, C.POINTER(Xfer), _u32]
        L.gw_comm_allreduce_u64.argtypes = [vp, vp, _u32, C.c_int]
        L.gw_world_create.argtypes = [vp, C.POINTER(WorldGeom), _u32, vp, C.POINTER(_u32)]
        L.gw_world_step.argtypes = [vp, vp, _u32]
        L.gw_world_route.argtypes = [vp, vp, _u32, C.POINTER(vp * 2), C.POINTER(_u32 * 2)]
        L.gw_world_submit.argtypes = [vp, C.POINTER(vp * 2), C.POINTER(_u32 * 2)]
        L.gw_world_status.argtypes = [vp, C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u64)]
        L.gw_world_far.argtypes = [vp, C.POINTER(vp), C.POINTER(C.POINTER(_u32))]
        L.gw_world_submit_far.argtypes = [vp, vp, _u32]
        L.gw_world_longs.argtypes = [vp, C.POINTER(vp), C.POINTER(_u32)]
        L.gw_world_submit_longs.argtypes = [vp, vp, _u32]
        L.gw_world_stage_ops.argtypes = [vp, vp, _u32, C.POINTER(vp)]
        L.gw_world_step_host.argtypes = [vp, vp, _u32]
        L.gw_set_entity_ids.argtypes = [vp, vp, vp, _u32]
        L.gw_clear_entity_ids.argtypes = [vp, vp, _u32]
        L.gw_set_client_ids.argtypes = [vp, vp, vp, _u32]
        L.gw_set_client_syncing.argtypes = [vp, vp, vp, _u32]
        L.gw_submit_client_sync.argtypes = [vp, vp, _u32, C.POINTER(_u32), C.POINTER(_u32)]
        L.gw_sync_encode_wire.argtypes = [vp, _u32, C.POINTER(WireOut)]
        _lib = L
    return _lib


EXPORTED = ["gw_abi_version", "gw_init", "gw_shutdown", "gw_last_error", "gw_space_create",
            "gw_space_destroy", "gw_submit", "gw_submit_device", "gw_set_clients", "gw_tick",
            "gw_sync_collect", "gw_step", "gw_replay", "gw_neighbors", "gw_set_profiling", "gw_get_stage_times",
            "gw_total_neighbors", "gw_device_alloc", "gw_device_free", "gw_memcpy_h2d",
            "gw_memcpy_d2h", "gw_synchronize", "gw_submit_device_stamped", "gw_space_set_ownership",
            "gw_set_stream", "gw_route_halo", "gw_submit_device_rows", "gw_halo_status", "gw_tick_result", "gw_space_restore",
            "gw_client_events", "gw_fanout", "gw_comm_unique_id", "gw_comm_init", "gw_comm_info",
            "gw_comm_exchange", "gw_comm_allreduce_u64", "gw_world_create", "gw_world_step", "gw_world_route",
            "gw_world_submit", "gw_world_status", "gw_set_entity_ids", "gw_clear_entity_ids", "gw_set_client_ids",
            "gw_set_client_syncing", "gw_submit_client_sync", "gw_sync_encode_wire", "gw_space_grow",
            "gw_context_info", "gw_world_far", "gw_world_submit_far", "gw_world_stage_ops",
            "gw_world_step_host", "gw_comm_init_local", "gw_world_longs", "gw_world_submit_longs"]


def comm_init_local(ctxs) -> None:
    """gw_comm_init_local: the GpuAOI contexts of this process become ranks 0..n-1
    of a loopback group (each then driven by its own thread, as a rank process)."""
    arr = (C.c_void_p * len(ctxs))(*[g._h.value for g in ctxs])
    rc = lib().gw_comm_init_local(arr, len(ctxs))
    if rc:
        raise GwError(rc, lib().gw_last_error(ctxs[0]._h).decode(errors="replace") if ctxs else "")


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (rank 0); distribute the bytes to every rank (any channel)."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    rc = lib().gw_comm_unique_id(C.cast(buf, C.c_void_p))
    if rc:
        raise GwError(rc, "gw_comm_unique_id failed")
    return buf.raw


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _host_view(ptr, n: int, dtype) -> np.ndarray:
    """A numpy view (no copy) of n records at a library-owned host pointer."""
    if not n or not ptr:
        return np.zeros(0, dtype)
    return np.frombuffer((C.c_uint8 * (n * dtype.itemsize)).from_address(ptr), dtype=dtype)


@dataclasses.dataclass
class TickResult:
    enter: np.ndarray | None
    leave: np.ndarray | None
    n_enter: int
    n_leave: int
    ops: int
    movers: int
    pairs_tested: int
    nbr_old: int
    nbr_new: int
    bytes_alg: int
    device_us: float
    enter_dev: int = 0
    leave_dev: int = 0


@dataclasses.dataclass
class SyncResult:
    records: np.ndarray | None
    n_rec: int
    gate_off: np.ndarray
    flagged: int
    bytes_alg: int
    device_us: float
    rec_dev: int = 0
    client_slot: np.ndarray | None = None     # by_client: watcher slot of each client segment
    client_off: np.ndarray | None = None      # by_client: n_clients + 1 offsets into records


@dataclasses.dataclass
class MsgResult:
    records: np.ndarray
    gate_off: np.ndarray
    bytes_alg: int
    device_us: float
    n_rec: int = 0
    rec_dev: int = 0


class GpuAOI:
    """One gw_ctx on one HIP device (one process per GPU)."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        rc = lib().gw_init(device, C.byref(self._h))
        if rc:
            raise GwError(rc, "gw_init failed (no HIP device?)")
        self.spaces: list[tuple[int, int, int]] = []   # (id, base, capacity)

    def _chk(self, rc: int):
        if rc:
            raise GwError(rc, lib().gw_last_error(self._h).decode())

    def close(self):
        if self._h:
            lib().gw_shutdown(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # Space.EnableAOI(d)
    def create_space(self, d: float, capacity: int, bounds=None) -> tuple[int, int]:
        sid, base = _u32(), _u32()
        b = None
        if bounds is not None:
            barr = (C.c_float * 4)(*[float(v) for v in bounds])
            b = C.cast(barr, C.c_void_p)
        self._chk(lib().gw_space_create(self._h, float(d), int(capacity), b, C.byref(sid), C.byref(base)))
        self.spaces.append((sid.value, base.value, capacity))
        return sid.value, base.value

    def destroy_space(self, sid: int):
        """SpaceManager.delSpace after Space.OnDestroy (the space must be empty)."""
        self._chk(lib().gw_space_destroy(self._h, sid))
        self.spaces = [t for t in self.spaces if t[0] != sid]

    def grow_space(self, sid: int, capacity: int) -> int:
        """Grow space sid to `capacity` slots; returns its (possibly new) first slot."""
        nb = _u32()
        self._chk(lib().gw_space_grow(self._h, sid, int(capacity), C.byref(nb)))
        self.spaces = [(i, nb.value, capacity) if i == sid else (i, b, cp) for i, b, cp in self.spaces]
        return nb.value

    def context_info(self) -> dict:
        o = CtxInfo()
        self._chk(lib().gw_context_info(self._h, C.byref(o)))
        return {k: getattr(o, k) for k, _ in CtxInfo._fields_ if k != "reserved"}

    def restore(self, sid: int, slots, x, y, z, yaw, flags: int = 3):
        """Bulk Enter in index order without events (restore path, Space.go:209-214)."""
        a = [np.ascontiguousarray(v, dtype=t) for v, t in
             ((slots, np.uint32), (x, np.float32), (y, np.float32), (z, np.float32), (yaw, np.float32))]
        self._chk(lib().gw_space_restore(self._h, sid, *[_p(v) for v in a], len(a[0]), flags))

    def submit(self, ops: np.ndarray):
        ops = np.ascontiguousarray(ops, dtype=OP_DTYPE)
        self._chk(lib().gw_submit(self._h, _p(ops), len(ops)))

    def submit_device(self, dev_ptr: int, n: int):
        self._chk(lib().gw_submit_device(self._h, C.c_void_p(dev_ptr), n))

    def submit_device_stamped(self, dev_ops: int, dev_stamps: int, n: int):
        """Device ops with explicit global stamps (decomposed world)."""
        self._chk(lib().gw_submit_device_stamped(self._h, C.c_void_p(dev_ops), C.c_void_p(dev_stamps), n))

    def set_ownership(self, sid: int, x_lo: float, x_hi: float):
        """Emit events / records only for entities with x in [x_lo, x_hi) (Space strip)."""
        self._chk(lib().gw_space_set_ownership(self._h, sid, x_lo, x_hi))

    def set_stream(self, hip_stream: int | None):
        """Run on a caller's stream (e.g. torch.cuda.current_stream().cuda_stream)."""
        self._chk(lib().gw_set_stream(self._h, hip_stream or None))

    def route_halo(self, dev_ops: int, dev_stamps: int, n: int, max_step: float, dsts):
        """dsts: list of (x_lo, x_hi, dev_rows_ptr, cap_entities) (decomposed world, owner side)."""
        arr = (HaloDst * max(1, len(dsts)))(*[HaloDst(lo, hi, C.c_void_p(p), cap, 0) for lo, hi, p, cap in dsts])
        self._chk(lib().gw_route_halo(self._h, C.c_void_p(dev_ops), C.c_void_p(dev_stamps), n, max_step, arr,
                                      len(dsts)))

    def submit_device_rows(self, dev_rows: int, n: int):
        self._chk(lib().gw_submit_device_rows(self._h, C.c_void_p(dev_rows), n))

    def halo_status(self) -> tuple[int, int, int]:
        v = [_u64() for _ in range(3)]
        self._chk(lib().gw_halo_status(self._h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def set_clients(self, slots, gates):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        g = np.ascontiguousarray(gates, dtype=np.uint16)
        self._chk(lib().gw_set_clients(self._h, _p(s), _p(g), len(s)))

    def tick(self, copy: bool = True, no_events: bool = False, defer: bool = False, view: bool = False) -> TickResult:
        """defer (device-resident ops, copy=False): launch without a host sync;
        the result holds only `ops` until tick_result() (or the next collect).
        view (with copy): the event arrays are views of the library's pinned
        host buffers (valid until the next tick), as a Go caller reads them."""
        o = TickOut()
        fl = (TICK_COPY_TO_HOST if copy else 0) | (TICK_NO_EVENTS if no_events else 0) | \
            (TICK_DEFER if defer and not copy else 0)
        self._chk(lib().gw_tick(self._h, fl, C.byref(o)))
        if view and copy and not no_events:
            return TickResult(_host_view(o.enter, o.n_enter, EVENT_DTYPE), _host_view(o.leave, o.n_leave, EVENT_DTYPE),
                              o.n_enter, o.n_leave, o.ops, o.movers, o.pairs_tested, o.nbr_old, o.nbr_new,
                              o.bytes_alg, o.device_us, o.enter_dev or 0, o.leave_dev or 0)
        return self._tick_result(o, copy, no_events)

    def step_device(self, dev_ptr: int, n: int, by_client: bool = False):
        """gw_step with device-resident ops: submit + deferred tick + collect in
        one call, outputs left on the device.  Returns the library's TickOut and
        SyncOut structures (reused between calls: read them before the next
        step) -- the bench's hot loop, with no per-step Python objects."""
        if not hasattr(self, "_step_outs"):
            self._step_outs = (TickOut(), SyncOut())
        to, so = self._step_outs
        self._chk(lib().gw_step(self._h, C.c_void_p(dev_ptr), n, 1, 0, SYNC_BY_CLIENT if by_client else 0,
                                C.byref(to), C.byref(so)))
        return to, so

    def replay_device(self, dev_ptr: int, n: int, stride_ops: int, ticks: int, by_client: bool = False) -> dict:
        """gw_replay: `ticks` gw_step calls over a device-resident op log (tick t
        at dev_ptr + t * stride_ops ops); returns the summed counters."""
        r = ReplaySum()
        self._chk(lib().gw_replay(self._h, C.c_void_p(dev_ptr), n, stride_ops, ticks,
                                  SYNC_BY_CLIENT if by_client else 0, C.byref(r)))
        return {f: getattr(r, f) for f, _ in ReplaySum._fields_}

    def tick_result(self) -> TickResult:
        """Outputs of the last tick (settles a deferred tick)."""
        o = TickOut()
        self._chk(lib().gw_tick_result(self._h, C.byref(o)))
        return self._tick_result(o, False, False)

    def _tick_result(self, o, copy, no_events) -> TickResult:
        e = l = None
        if copy and not no_events:
            e = np.zeros(o.n_enter, EVENT_DTYPE)
            l = np.zeros(o.n_leave, EVENT_DTYPE)
            if o.n_enter:
                C.memmove(_p(e), o.enter, o.n_enter * 8)
            if o.n_leave:
                C.memmove(_p(l), o.leave, o.n_leave * 8)
        return TickResult(e, l, o.n_enter, o.n_leave, o.ops, o.movers, o.pairs_tested, o.nbr_old,
                          o.nbr_new, o.bytes_alg, o.device_us, o.enter_dev or 0, o.leave_dev or 0)

    def sync_collect(self, copy: bool = True, by_client: bool = False, view: bool = False) -> SyncResult:
        """by_client: records grouped per client inside each gate (the gate's
        regroup, GateService.go:350-375), with the client segment table.
        view (with copy): records are a view of the pinned host buffer."""
        o = SyncOut()
        fl = (SYNC_COPY_TO_HOST if copy else 0) | (SYNC_BY_CLIENT if by_client else 0)
        self._chk(lib().gw_sync_collect(self._h, fl, C.byref(o)))
        r = None
        if copy and view:
            r = _host_view(o.rec, o.n_rec, REC_DTYPE)
        elif copy:
            r = np.zeros(o.n_rec, REC_DTYPE)
            if o.n_rec:
                C.memmove(_p(r), o.rec, o.n_rec * 24)
        goff = np.array([o.gate_off[i] for i in range(o.n_gates + 1)], dtype=np.uint64)
        res = SyncResult(r, o.n_rec, goff, o.flagged, o.bytes_alg, o.device_us, o.rec_dev or 0)
        if by_client and copy:
            n = o.n_clients
            res.client_slot = np.ctypeslib.as_array(o.client_slot, (max(n, 1),))[:n].copy()
            res.client_off = np.ctypeslib.as_array(o.client_off, (n + 1,)).copy()
        return res

    @staticmethod
    def _msgs(o: MsgOut, dtype) -> MsgResult:
        r = np.zeros(o.n_rec if o.rec else 0, dtype)
        if o.n_rec and o.rec:
            C.memmove(_p(r), o.rec, o.n_rec * dtype.itemsize)
        goff = np.array([o.gate_off[i] for i in range(o.n_gates + 1)], dtype=np.uint64)
        return MsgResult(r, goff, o.bytes_alg, o.device_us, o.n_rec, o.rec_dev or 0)

    def client_events(self, copy: bool = True) -> tuple[MsgResult, MsgResult]:
        """Client messages of the last tick's events (Entity.interest/uninterest,
        Entity.go:236-246): creates (REC_DTYPE: watcher, target, target's x,y,z,yaw)
        and destroys (EVENT_DTYPE), each grouped (gate, watcher, target)."""
        cr, de = MsgOut(), MsgOut()
        fl = MSG_COPY_TO_HOST if copy else 0
        self._chk(lib().gw_client_events(self._h, fl, C.byref(cr), C.byref(de)))
        return self._msgs(cr, REC_DTYPE), self._msgs(de, EVENT_DTYPE)

    def fanout(self, slots, copy: bool = True) -> MsgResult:
        """AllClients fan-out of calls on slots[k] (Entity.CallAllClients,
        Entity.go:743-749): FANOUT_DTYPE records grouped (gate, watcher, call)."""
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        o = MsgOut()
        self._chk(lib().gw_fanout(self._h, _p(s), len(s), MSG_COPY_TO_HOST if copy else 0, C.byref(o)))
        return self._msgs(o, FANOUT_DTYPE)

    def neighbors(self, slot: int) -> np.ndarray:
        n = _u32()
        self._chk(lib().gw_neighbors(self._h, slot, None, 0, C.byref(n)))
        buf = np.zeros(n.value, np.uint32)
        if n.value:
            self._chk(lib().gw_neighbors(self._h, slot, _p(buf), n.value, C.byref(n)))
        return buf

    def total_neighbors(self) -> int:
        v = _u64()
        self._chk(lib().gw_total_neighbors(self._h, C.byref(v)))
        return v.value

    def set_profiling(self, mode):
        """0 / False off, 1 / True every stage, 2 only the dominant kernel's stage ("diff")."""
        self._chk(lib().gw_set_profiling(self._h, int(mode)))

    def stage_times(self) -> list[tuple[str, float, int, int]]:
        """(stage, total us, total algorithmic bytes, calls) over every stage
        recorded since the last call (one host sync, here)."""
        t = StageTimes()
        self._chk(lib().gw_get_stage_times(self._h, C.byref(t)))
        return [(t.name[i].decode(), t.us[i], t.bytes_alg[i], t.calls[i]) for i in range(t.n)]

    # device memory helpers (bench: inputs resident in HBM)
    def dev_alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        self._chk(lib().gw_device_alloc(self._h, nbytes, C.byref(p)))
        return p.value

    def dev_free(self, ptr: int):
        self._chk(lib().gw_device_free(self._h, C.c_void_p(ptr)))

    def h2d(self, dev_ptr: int, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        self._chk(lib().gw_memcpy_h2d(self._h, C.c_void_p(dev_ptr), _p(arr), arr.nbytes))

    def d2h(self, arr: np.ndarray, dev_ptr: int):
        self._chk(lib().gw_memcpy_d2h(self._h, _p(arr), C.c_void_p(dev_ptr), arr.nbytes))

    def synchronize(self):
        self._chk(lib().gw_synchronize(self._h))

    # ---- ids, client-sync decode, wire encode -------
    def set_entity_ids(self, slots, ids: bytes):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        b = np.frombuffer(bytes(ids), np.uint8)
        assert len(b) == 16 * len(s)
        self._chk(lib().gw_set_entity_ids(self._h, _p(s), _p(b), len(s)))

    def clear_entity_ids(self, slots):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        self._chk(lib().gw_clear_entity_ids(self._h, _p(s), len(s)))

    def set_client_ids(self, slots, ids: bytes):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        b = np.frombuffer(bytes(ids), np.uint8)
        assert len(b) == 16 * len(s)
        self._chk(lib().gw_set_client_ids(self._h, _p(s), _p(b), len(s)))

    def set_client_syncing(self, slots, on):
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        o = np.ascontiguousarray(on, dtype=np.uint8)
        self._chk(lib().gw_set_client_syncing(self._h, _p(s), _p(o), len(s)))

    def submit_client_sync(self, payload: bytes) -> tuple[int, int]:
        """MT_SYNC_POSITION_YAW_FROM_CLIENT payload (32-B records) -> (applied, left to the caller)."""
        b = np.frombuffer(bytes(payload), np.uint8)
        assert len(b) % 32 == 0
        ap, tc = _u32(), _u32()
        self._chk(lib().gw_submit_client_sync(self._h, _p(b), len(b) // 32, C.byref(ap), C.byref(tc)))
        return ap.value, tc.value

    def encode_wire(self, copy: bool = True, view: bool = False):
        """-> (bytes or None, [(gate, offset, length)], n_bytes, device_us) of the last collect's packets.
        view (with copy): the packets are a u8 view of the library's pinned host buffer (valid until
        the next encode), as a Go caller would read them in place."""
        o = WireOut()
        self._chk(lib().gw_sync_encode_wire(self._h, 1 if copy else 0, C.byref(o)))
        pk = [(o.gate[k], o.off[k], o.off[k + 1] - o.off[k]) for k in range(o.n_packets)]
        if copy and view:
            return _host_view(o.bytes, o.n_bytes, np.dtype(np.uint8)), pk, o.n_bytes, o.device_us
        data = C.string_at(o.bytes, o.n_bytes) if (copy and o.n_bytes) else (b"" if copy else None)
        return data, pk, o.n_bytes, o.device_us

    # ---- RCCL communicator (library-internal data-path collectives) -------
    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = C.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        self._chk(lib().gw_comm_init(self._h, C.cast(buf, C.c_void_p), nranks, rank))

    def comm_info(self) -> tuple[int, int]:
        n, r = C.c_int(), C.c_int()
        self._chk(lib().gw_comm_info(self._h, C.byref(n), C.byref(r)))
        return n.value, r.value

    def comm_exchange(self, xfers):
        """xfers: list of (peer, send_ptr, send_bytes, recv_ptr, recv_bytes) (device memory)."""
        arr = (Xfer * max(1, len(xfers)))(*[Xfer(p, 0, C.c_void_p(sp), sb, C.c_void_p(rp), rb)
                                             for p, sp, sb, rp, rb in xfers])
        self._chk(lib().gw_comm_exchange(self._h, arr, len(xfers)))

    def comm_allreduce_u64(self, dev_ptr: int, n: int, op: int = RED_SUM):
        self._chk(lib().gw_comm_allreduce_u64(self._h, C.c_void_p(dev_ptr), n, op))

    # ---- decomposed world ----------------------------------------------------
    def world_create(self, x0, strip_w, d, max_step, ranks, rank, capacity, bounds) -> int:
        geom = WorldGeom(x0, strip_w, d, max_step, ranks, rank)
        barr = (C.c_float * 4)(*[float(v) for v in bounds])
        sid = _u32()
        self._chk(lib().gw_world_create(self._h, C.byref(geom), capacity, C.cast(barr, C.c_void_p), C.byref(sid)))
        self._ranks = int(ranks)
        self.spaces.append((sid.value, 0, capacity))
        return sid.value

    def world_step(self, dev_ops: int, n: int):
        """Route + RCCL exchange + queue this rank's tick (then tick / sync_collect)."""
        self._chk(lib().gw_world_step(self._h, C.c_void_p(dev_ops), n))

    def world_step_host(self, ops: np.ndarray):
        """gw_world_step_host: this rank's owned ops from host memory (staged by the library)."""
        ops = np.ascontiguousarray(ops, dtype=OP_DTYPE)
        self._chk(lib().gw_world_step_host(self._h, _p(ops), len(ops)))

    def world_stage_ops(self, ops: np.ndarray) -> int:
        """gw_world_stage_ops: host ops -> a library-owned device copy (valid until the tick)."""
        ops = np.ascontiguousarray(ops, dtype=OP_DTYPE)
        p = C.c_void_p()
        self._chk(lib().gw_world_stage_ops(self._h, _p(ops), len(ops), C.byref(p)))
        return p.value or 0

    def world_route(self, dev_ops: int, n: int):
        """-> ((left_ptr, left_rows), (right_ptr, right_rows)) device rows to send (ptr 0 = no neighbour)."""
        ptrs, rows = (C.c_void_p * 2)(), (_u32 * 2)()
        self._chk(lib().gw_world_route(self._h, C.c_void_p(dev_ops), n, C.byref(ptrs), C.byref(rows)))
        return [(ptrs[i] or 0, rows[i]) for i in range(2)]

    def world_submit(self, recv):
        """recv: [(left_ptr, left_rows), (right_ptr, right_rows)] received rows (device)."""
        ptrs = (C.c_void_p * 2)(*[C.c_void_p(p or None) for p, _ in recv])
        rows = (_u32 * 2)(*[n for _, n in recv])
        self._chk(lib().gw_world_submit(self._h, C.byref(ptrs), C.byref(rows)))

    def world_far(self) -> dict:
        """After world_route: {dest rank: (device ptr, rows)} of the long moves' rows
        (this rank's own LEAVE rows under its own rank)."""
        rows, cnt = C.c_void_p(), C.POINTER(_u32)()
        self._chk(lib().gw_world_far(self._h, C.byref(rows), C.byref(cnt)))
        out, off = {}, 0
        nranks = self._ranks
        for q in range(nranks):
            k = cnt[q]
            if k:
                out[q] = (rows.value + off * 3 * 32, k * 3)
            off += k
        return out

    def world_submit_far(self, dev_rows: int, n_rows: int):
        """Queue far rows received for this tick (after world_submit)."""
        self._chk(lib().gw_world_submit_far(self._h, C.c_void_p(dev_rows), n_rows))

    def world_longs(self) -> tuple[int, int]:
        """After world_route: (device ptr, n) of this rank's long-mover list (gw_long_move)."""
        p, n = C.c_void_p(), _u32()
        self._chk(lib().gw_world_longs(self._h, C.byref(p), C.byref(n)))
        return p.value or 0, n.value

    def world_submit_longs(self, dev_ptr: int, n: int):
        """Queue every rank's long-mover lists for this tick (after world_submit; device memory)."""
        self._chk(lib().gw_world_submit_longs(self._h, C.c_void_p(dev_ptr or None), n))

    def world_status(self) -> tuple[int, int, int]:
        """(halo overflows, long-move conflicts, bad ops), summed over ranks."""
        v = [_u64() for _ in range(3)]
        self._chk(lib().gw_world_status(self._h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)


def load_space(g: GpuAOI, tr, bounds=None, chunk: int = 1 << 21, via_ticks: bool = False) -> tuple[int, int]:
    """Create a space for a SpaceTrace and bulk-load its initial population
    (the restore path, Space.go:209-214): gw_space_restore, or (via_ticks)
    Enter ops in trace order flushed in chunks with TICK_NO_EVENTS; both equal
    one sequential Enter stream."""
    from .traces import enter_ops, with_global_slots
    sid, base = g.create_space(tr.d, tr.capacity, bounds if bounds is not None else tr.bounds)
    if via_ticks:
        ops = with_global_slots(enter_ops(tr.init_slots, tr.init_x, tr.init_y, tr.init_z, tr.init_yaw), base)
        for i in range(0, len(ops), chunk):
            g.submit(ops[i:i + chunk])
            g.tick(copy=False, no_events=True)
    else:
        g.restore(sid, np.asarray(tr.init_slots, np.uint32) + np.uint32(base), tr.init_x, tr.init_y, tr.init_z,
                  tr.init_yaw)
    if tr.gates is not None:
        nz = np.nonzero(tr.gates)[0]
        g.set_clients(nz.astype(np.uint32) + base, tr.gates[nz])
    return sid, base
