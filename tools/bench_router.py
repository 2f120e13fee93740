"""Per-tick cost of the decomposed-world routing on one GPU: 100k owned Moved
ops of a config #3 strip (rank min(3, N-1) of an N-strip world); HipRouter
(gw_route_halo) and the torch statement (tests/torch_router.py).
usage: python tools/bench_router.py [N]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from goworld_amd import dworld, gpuaoi, traces as T  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch_router  # noqa: E402

ws = int(sys.argv[1]) if len(sys.argv) > 1 else 8
r, n, side, K = min(3, ws - 1), 1_000_000, 32768.0, 16384
dev = torch.device("cuda", 0)
tr = T.config3(ticks=12, seed=3, n=n, side=side)
x0 = -ws * side / 2
geom = dworld.Strips(x0, side, ws, tr.d, 16.0)
off = np.float32(x0 + (r + 0.5) * side)


def words(ops):
    o = ops.copy()
    o["slot"] += np.uint32(r * n)
    o["x"] += off
    return torch.from_numpy(dworld.ops_to_words(o).copy()).to(dev)


g = gpuaoi.GpuAOI(0)
eng = dworld.HipStrip(g)
lo, hi = geom.ext(r)
eng.create_space(tr.d, n * ws, (max(lo, x0), -side / 2, min(hi, x0 + ws * side), side / 2))
routers = {"hip": eng.make_router(geom, r, n * ws, dev, K), "torch": torch_router.Router(geom, r, n * ws, dev, K)}
enter = T.enter_ops(tr.init_slots, tr.init_x, tr.init_y, tr.init_z, tr.init_yaw)
tick = 0
for i in range(0, n, 1 << 18):
    w = words(enter[i:i + (1 << 18)])
    st = dworld.stamps_for(tick, r, ws, len(w), dev)
    for rt in routers.values():
        rt.route(w, st)
    eng.submit(w, st)
    eng.tick(copy=False, no_events=True)
    tick += 1
W = [words(t) for t in tr.ticks]
torch.cuda.synchronize()

def timed(fn, reps=12):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for t in range(reps):
        fn(t)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


# gw_route_halo leaves the engine state alone: route tick 0's ops repeatedly
st0 = dworld.stamps_for(tick, r, ws, len(W[0]), dev)
print(f"hip: route {timed(lambda t: routers['hip'].route(W[0], st0)):.1f} us/tick", flush=True)
# torch router: one timed pass over 12 ticks (its state advances)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for t in range(12):
    routers["torch"].route(W[t], dworld.stamps_for(tick + t, r, ws, len(W[t]), dev))
e1.record()
torch.cuda.synchronize()
print(f"torch: route {e0.elapsed_time(e1) / 12 * 1e3:.1f} us/tick")
print("hip status", routers["hip"].status(), "torch status", routers["torch"].status())
g.close()
