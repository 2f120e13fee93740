"""Readers of the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py).  Shared by the CPU oracle tests and the GPU
parity tests; data only, nothing here computes an expected result."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

from goworld_amd import traces as T

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SMALL = ["cfg1_walk", "cfg1b_steps", "adversarial_s11", "adversarial_s12", "dyadic_hot_2k", "server_y_s13"]

EVENT_DTYPE = np.dtype([("watcher", "<u4"), ("target", "<u4")])
REC_DTYPE = np.dtype([("watcher", "<u4"), ("entity", "<u4"), ("x", "<f4"), ("y", "<f4"),
                      ("z", "<f4"), ("yaw", "<f4")])


class Fixture:
    """One small fixture: the trace (as T.SpaceTrace) and the expected outputs."""

    def __init__(self, name: str):
        self.name = name
        with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
            f = {k: z[k] for k in z.files}
        self.f = f
        ops = f["ops"].view(T.OP_DTYPE) if f["ops"].dtype != T.OP_DTYPE else f["ops"]
        off = f["tick_off"].astype(np.int64)
        self.trace = T.SpaceTrace(
            n=len(f["init_slots"]), capacity=int(f["capacity"]), d=float(f["d"]),
            bounds=tuple(float(b) for b in f["bounds"]),
            init_slots=f["init_slots"], init_x=f["init_x"], init_y=f["init_y"], init_z=f["init_z"],
            init_yaw=f["init_yaw"], ticks=[ops[off[t]:off[t + 1]] for t in range(len(off) - 1)],
            gates=f["gates"])

    @property
    def ticks(self) -> int:
        return len(self.trace.ticks)

    def events(self, t: int):
        eo, lo = self.f["enter_off"].astype(np.int64), self.f["leave_off"].astype(np.int64)
        e = self.f["enter"][eo[t]:eo[t + 1]].view(EVENT_DTYPE)
        l = self.f["leave"][lo[t]:lo[t + 1]].view(EVENT_DTYPE)
        return e, l

    def n_rec(self, t: int) -> int:
        return int(self.f["n_rec"][t])

    def rec_sha(self, t: int) -> str:
        return self.f["rec_sha"][t].decode()

    def wire_sha(self, t: int) -> str:
        return self.f["wire_sha"][t].decode()

    def raw(self, t: int) -> tuple:
        return tuple(int(v) for v in self.f["raw"][t])

    @property
    def rec0(self) -> np.ndarray:
        return self.f["rec0"].view(REC_DTYPE)

    @property
    def nbr_total(self) -> int:
        return int(self.f["nbr_total"])

    @property
    def nbr_sha(self) -> str:
        return bytes(self.f["nbr_sha"]).decode()


def sha(a) -> str:
    return hashlib.sha256(a if isinstance(a, (bytes, bytearray)) else np.ascontiguousarray(a).tobytes()).hexdigest()


def canonical_records(recs: np.ndarray, gates: np.ndarray) -> np.ndarray:
    """(gate(watcher), entity, watcher) order: the fixtures' record order."""
    if len(recs) == 0:
        return recs
    return recs[np.lexsort((recs["watcher"], recs["entity"], gates[recs["watcher"]]))]


def neighbour_sha(lists) -> str:
    h = hashlib.sha256()
    for nb in lists:
        nb = np.asarray(nb, np.uint32)
        h.update(np.uint32(len(nb)).tobytes())
        h.update(nb.tobytes())
    return h.hexdigest()


def digests() -> dict:
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


def trace_input_sha(tr) -> str:
    h = hashlib.sha256()
    for a in (tr.init_slots, tr.init_x, tr.init_y, tr.init_z, tr.init_yaw, tr.gates):
        h.update(np.ascontiguousarray(a).tobytes())
    for ops in tr.ticks:
        h.update(ops.tobytes())
    return h.hexdigest()


DIGEST_TRACES = {
    "config2_100k": lambda: T.config2(ticks=3),
    "config3_1m": lambda: T.config3(ticks=2),
}


# config #4: 10k independent spaces of 1k entities in ONE context (slots of
# space i at [1000 i, 1000 (i + 1))); digests over the whole context's outputs
MULTI_DIGEST_TRACES = {
    "config4_10k": lambda: [T.config4_space(s, ticks=2) for s in range(10_000)],
}


def multi_input_sha(trs) -> str:
    h = hashlib.sha256()
    for tr in trs:
        h.update(bytes.fromhex(trace_input_sha(tr)))
    return h.hexdigest()
