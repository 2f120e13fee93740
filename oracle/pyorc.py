"""ctypes binding of the CPU oracle (oracle/orc.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by goworld_amd/.  Parity at the go-aoi
boundary is UNPINNED (see orc.h): go-aoi v0.2.0 and a Go toolchain are absent.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liborc.so")

XZLIST, BRUTE, SEQRULE = 0, 1, 2

EVENT_DTYPE = np.dtype([("watcher", "<u4"), ("target", "<u4")])
REC_DTYPE = np.dtype([("watcher", "<u4"), ("entity", "<u4"), ("x", "<f4"), ("y", "<f4"),
                      ("z", "<f4"), ("yaw", "<f4")])

FANOUT_DTYPE = np.dtype([("watcher", "<u4"), ("entity", "<u4"), ("item", "<u4")])

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp, u32, u64, f32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_float
        L.orc_new.restype = vp
        L.orc_new.argtypes = [u32, f32, C.c_int]
        L.orc_free.argtypes = [vp]
        L.orc_bulk_enter.argtypes = [vp, u32, vp, vp, vp, vp, vp, C.c_uint8]
        L.orc_tick.argtypes = [vp, vp, u32]
        L.orc_event_counts.argtypes = [vp, C.POINTER(u64), C.POINTER(u64)]
        L.orc_events_copy.argtypes = [vp, vp, vp]
        L.orc_raw_counts.argtypes = [vp] + [C.POINTER(u64)] * 4
        L.orc_set_client.argtypes = [vp, u32, C.c_uint16]
        L.orc_collect.restype = u64
        L.orc_collect.argtypes = [vp]
        L.orc_records_copy.argtypes = [vp, vp]
        L.orc_encode_wire.restype = u64
        L.orc_encode_wire.argtypes = [vp, vp]
        L.orc_fixed_uuid_u32.argtypes = [u32, C.c_char_p]
        L.orc_neighbors.restype = u32
        L.orc_neighbors.argtypes = [vp, u32, vp, u32]
        L.orc_interested_by.restype = u32
        L.orc_interested_by.argtypes = [vp, u32, vp, u32]
        L.orc_total_neighbors.restype = u64
        L.orc_total_neighbors.argtypes = [vp]
        L.orc_present.argtypes = [vp, u32]
        L.orc_in_window.argtypes = [f32, f32, f32, f32, f32]
        L.orc_client_creates.restype = u64
        L.orc_client_creates.argtypes = [vp, vp]
        L.orc_client_destroys.restype = u64
        L.orc_client_destroys.argtypes = [vp, vp]
        L.orc_fanout.restype = u64
        L.orc_fanout.argtypes = [vp, vp, u32, vp]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class OracleSpace:
    """One reference space on the CPU (see orc.h for the three modes)."""

    def __init__(self, capacity: int, d: float, mode: int = XZLIST):
        self._h = lib().orc_new(capacity, d, mode)
        if not self._h:
            raise ValueError("orc_new failed")
        self.capacity, self.d, self.mode = capacity, d, mode

    def close(self):
        if self._h:
            lib().orc_free(self._h)
            self._h = None

    __del__ = close

    def bulk_enter(self, slots, x, y, z, yaw, flags: int = 3):
        a = [np.ascontiguousarray(v, dtype=t) for v, t in
             ((slots, np.uint32), (x, np.float32), (y, np.float32), (z, np.float32), (yaw, np.float32))]
        rc = lib().orc_bulk_enter(self._h, len(a[0]), *[_ptr(v) for v in a], flags)
        if rc:
            raise RuntimeError(f"orc_bulk_enter rc={rc}")

    def tick(self, ops: np.ndarray) -> int:
        ops = np.ascontiguousarray(ops)
        return lib().orc_tick(self._h, _ptr(ops), len(ops))

    def events(self):
        ne, nl = C.c_uint64(), C.c_uint64()
        lib().orc_event_counts(self._h, C.byref(ne), C.byref(nl))
        e = np.zeros(ne.value, EVENT_DTYPE)
        l = np.zeros(nl.value, EVENT_DTYPE)
        lib().orc_events_copy(self._h, _ptr(e), _ptr(l))
        return e, l

    def raw_counts(self):
        v = [C.c_uint64() for _ in range(4)]
        lib().orc_raw_counts(self._h, *[C.byref(x) for x in v])
        return tuple(x.value for x in v)

    def set_clients(self, gates: np.ndarray):
        for i, g in enumerate(np.asarray(gates)):
            if g:
                lib().orc_set_client(self._h, i, int(g))

    def set_client(self, slot: int, gate: int):
        lib().orc_set_client(self._h, slot, gate)

    def collect(self) -> np.ndarray:
        n = lib().orc_collect(self._h)
        r = np.zeros(n, REC_DTYPE)
        lib().orc_records_copy(self._h, _ptr(r))
        return r

    def wire(self) -> bytes:
        n = lib().orc_encode_wire(self._h, None)
        buf = np.zeros(n, np.uint8)
        lib().orc_encode_wire(self._h, _ptr(buf))
        return buf.tobytes()

    def neighbors(self, slot: int) -> np.ndarray:
        n = lib().orc_neighbors(self._h, slot, None, 0)
        b = np.zeros(n, np.uint32)
        lib().orc_neighbors(self._h, slot, _ptr(b), n)
        return b

    def interested_by(self, slot: int) -> np.ndarray:
        n = lib().orc_interested_by(self._h, slot, None, 0)
        b = np.zeros(n, np.uint32)
        lib().orc_interested_by(self._h, slot, _ptr(b), n)
        return b

    def total_neighbors(self) -> int:
        return lib().orc_total_neighbors(self._h)

    def client_events(self):
        """(creates, destroys) of the last tick: the sendCreateEntity /
        sendDestroyEntity messages (GameClient.go:37-59), order (gate, watcher, target)."""
        n = lib().orc_client_creates(self._h, None)
        cr = np.zeros(n, REC_DTYPE)
        lib().orc_client_creates(self._h, _ptr(cr))
        n = lib().orc_client_destroys(self._h, None)
        de = np.zeros(n, EVENT_DTYPE)
        lib().orc_client_destroys(self._h, _ptr(de))
        return cr, de

    def fanout(self, slots) -> np.ndarray:
        """CallAllClients deliveries (Entity.go:743-749), order (gate, watcher, call)."""
        sl = np.ascontiguousarray(slots, dtype=np.uint32)
        n = lib().orc_fanout(self._h, _ptr(sl), len(sl), None)
        out = np.zeros(n, FANOUT_DTYPE)
        lib().orc_fanout(self._h, _ptr(sl), len(sl), _ptr(out))
        return out

    def present(self, slot: int) -> bool:
        return bool(lib().orc_present(self._h, slot))

    def relation(self):
        """All neighbour lists as a dict slot -> sorted array (small N only)."""
        return {i: self.neighbors(i) for i in range(self.capacity)}


def fixed_uuid(v: int) -> bytes:
    buf = C.create_string_buffer(16)
    lib().orc_fixed_uuid_u32(v, buf)
    return buf.raw[:16]


def in_window(cx, cz, d, ox, oz) -> bool:
    return bool(lib().orc_in_window(cx, cz, d, ox, oz))


def load_trace(sp: OracleSpace, tr, flags: int = 3):
    sp.bulk_enter(tr.init_slots, tr.init_x, tr.init_y, tr.init_z, tr.init_yaw, flags)
    if tr.gates is not None:
        sp.set_clients(tr.gates)


MT_SYNC_POSITION_YAW_ON_CLIENTS = 1502   # proto.go:107-109 (the value orc_encode_wire writes)
_WIRE_REC = np.dtype([("cid", "S16"), ("data", "V32")])   # clientid[16] + eid[16] + x,y,z,yaw


def split_wire(buf: bytes) -> list:
    """The game->gate packets concatenated by OracleSpace.wire() (one per gate:
    u16 msgtype, u16 gateid, 48-B records).  Records start with an ASCII
    clientid, so a 0xDE byte (low byte of msgtype 1502) only starts a header."""
    out, i = [], 0
    while i < len(buf):
        assert buf[i] == MT_SYNC_POSITION_YAW_ON_CLIENTS & 0xFF
        j = i + 4
        while j < len(buf) and buf[j] != MT_SYNC_POSITION_YAW_ON_CLIENTS & 0xFF:
            j += 48
        out.append(buf[i:j])
        i = j
    return out


def gate_dispatch(packet: bytes) -> dict:
    """GateService.handleSyncPositionYawOnClients (GateService.go:350-375)
    restated on one game->gate packet: records split by clientid; a client's
    data (eid + x,y,z,yaw, 32 B per record) is appended in packet order and
    sent as one packet u16 MT_SYNC_POSITION_YAW_ON_CLIENTS + data.  Returns
    {clientid: packet bytes} (the reference visits clients in Go map order, so
    the client order is not part of the result)."""
    mt = int(np.frombuffer(packet, "<u2", 1, 0)[0])
    assert mt == MT_SYNC_POSITION_YAW_ON_CLIENTS
    out = {}
    for r in np.frombuffer(packet[4:], _WIRE_REC):       # skip msgtype and the useless gateid
        out.setdefault(bytes(r["cid"]), [np.uint16(MT_SYNC_POSITION_YAW_ON_CLIENTS).tobytes()]).append(
            bytes(r["data"]))
    return {k: b"".join(v) for k, v in out.items()}


# ---------------------------------------------------------------------------
# gridmt.c: multi-threaded uniform-grid CPU fairness baseline
_GMT_PATH = os.path.join(_HERE, "build", "libgridmt.so")
_gmt = None


def gmt_lib():
    global _gmt
    if _gmt is None:
        if not os.path.exists(_GMT_PATH):
            build()
        L = C.CDLL(_GMT_PATH)
        vp, u32, u64, f32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_float
        L.gmt_new.restype = vp
        L.gmt_new.argtypes = [u32, f32, f32, f32, f32, f32, C.c_int]
        L.gmt_free.argtypes = [vp]
        L.gmt_set_clients.argtypes = [vp, vp]
        L.gmt_load.argtypes = [vp, u32, vp, vp, vp, vp, vp]
        L.gmt_tick.argtypes = [vp, vp, u32]
        L.gmt_event_counts.argtypes = [vp, C.POINTER(u64), C.POINTER(u64)]
        L.gmt_events_copy.argtypes = [vp, vp, vp]
        L.gmt_collect.argtypes = [vp]
        L.gmt_collect.restype = u64
        L.gmt_records_copy.argtypes = [vp, vp]
        L.gmt_threads.argtypes = [vp]
        _gmt = L
    return _gmt


class GridMT:
    """Multi-threaded (OpenMP) uniform-grid CPU implementation of the batched
    tick + collect; threads = 0 uses OMP_NUM_THREADS / all cores."""

    def __init__(self, capacity: int, d: float, bounds, threads: int = 0):
        self._h = gmt_lib().gmt_new(capacity, d, *[float(b) for b in bounds], threads)
        self.capacity = capacity

    def close(self):
        if self._h:
            gmt_lib().gmt_free(self._h)
            self._h = None

    __del__ = close

    @property
    def threads(self) -> int:
        return gmt_lib().gmt_threads(self._h)

    def load(self, tr):
        a = [np.ascontiguousarray(v, dtype=t) for v, t in
             ((tr.init_slots, np.uint32), (tr.init_x, np.float32), (tr.init_y, np.float32),
              (tr.init_z, np.float32), (tr.init_yaw, np.float32))]
        assert gmt_lib().gmt_load(self._h, len(a[0]), *[_ptr(v) for v in a]) == 0
        if tr.gates is not None:
            gates = np.zeros(self.capacity, np.uint16)
            gates[:len(tr.gates)] = tr.gates
            gmt_lib().gmt_set_clients(self._h, _ptr(gates))

    def tick(self, ops: np.ndarray) -> int:
        ops = np.ascontiguousarray(ops)
        return gmt_lib().gmt_tick(self._h, _ptr(ops), len(ops))

    def events(self):
        ne, nl = C.c_uint64(), C.c_uint64()
        gmt_lib().gmt_event_counts(self._h, C.byref(ne), C.byref(nl))
        e = np.zeros(ne.value, EVENT_DTYPE)
        l = np.zeros(nl.value, EVENT_DTYPE)
        gmt_lib().gmt_events_copy(self._h, _ptr(e), _ptr(l))
        return e, l

    def collect(self) -> np.ndarray:
        n = gmt_lib().gmt_collect(self._h)
        r = np.zeros(n, REC_DTYPE)
        gmt_lib().gmt_records_copy(self._h, _ptr(r))
        return r
