"""Host-side timing of one bench step's calls (config #3, N=1): where the time
between the collect's sync and the next tick's first kernel goes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from goworld_amd import gpuaoi, traces  # noqa: E402

tr = traces.config3(ticks=40)
g = gpuaoi.GpuAOI(0)
gpuaoi.load_space(g, tr, chunk=1 << 18)
g.sync_collect(copy=False)
m = len(tr.ticks[0])
ops_all = np.concatenate(tr.ticks)
dev = g.dev_alloc(ops_all.nbytes)
g.h2d(dev, ops_all)
nb = m * traces.OP_DTYPE.itemsize
T = {k: 0.0 for k in ("submit", "tick", "collect", "result", "loop")}
K = 0
for t in range(40):
    a = time.perf_counter()
    g.submit_device(dev + t * nb, m)
    b = time.perf_counter()
    g.tick(copy=False, defer=True)
    c = time.perf_counter()
    g.sync_collect(copy=False)
    d = time.perf_counter()
    g.tick_result()
    e = time.perf_counter()
    if t >= 20:
        K += 1
        for k, v in (("submit", b - a), ("tick", c - b), ("collect", d - c), ("result", e - d), ("loop", e - a)):
            T[k] += v
print({k: round(v / K * 1e6, 1) for k, v in T.items()}, "us per step")
g.close()
