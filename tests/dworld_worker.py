"""One rank of a decomposed-world parity run (launched by tests/test_dworld.py
as a subprocess; gloo over 127.0.0.1).

--engine oracle : the rank's local space is a CPU oracle space (test
                  infrastructure: checks the routing / halo protocol alone);
--engine hip    : the rank's local space is the HIP engine on cuda:0 (the
                  product path; several ranks share the one GPU).

Writes the rank's owned events per tick and records per collect to --out.
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from goworld_amd import dworld, traces as T  # noqa: E402
import torch_router  # noqa: E402  (tests/, on sys.path as the script's dir)


class OracleStrip:
    """Mock engine (test only): an oracle space fed the rank's local op rows
    in global-stamp order, with the engine's ownership filters."""

    def __init__(self):
        from oracle import pyorc
        self.pyorc = pyorc
        self.words, self.stamps = [], []

    def create_world(self, geom, rank, n_global, bounds):
        self.max_step = np.float32(geom.max_step)
        self.router = torch_router.Router(geom, rank, n_global, torch.device("cpu"), n_global)
        self.o = self.pyorc.OracleSpace(n_global, geom.d, self.pyorc.SEQRULE)
        self.o_d = geom.d
        self.x = np.zeros(n_global, np.float32)
        self.present = np.zeros(n_global, bool)
        self.lo, self.hi = (np.float32(v) for v in geom.own_range_f32(rank))
        return 0

    def route(self, words, stamps):
        return self.router.route_exact(words, stamps)

    def far(self):
        return self.router.far_exact()

    def longs(self):
        return self.router.longs_exact()

    def submit(self, words, stamps, recvd=(), far_in=(), longs=None):
        self.tick_longs = longs
        self.words.append(words.cpu().numpy())
        self.stamps.append(stamps.cpu().numpy())
        for rows in list(recvd) + list(far_in):
            if rows is None:
                continue
            self.router.receive(rows)
            w, s = torch_router.split_rows(rows)
            self.words.append(w.cpu().numpy())
            self.stamps.append(s.cpu().numpy())

    def collected(self):
        self.router.collected()

    def status(self):
        return self.router.status()

    def set_clients(self, slots, gates):
        for s, g in zip(np.asarray(slots).tolist(), np.asarray(gates).tolist()):
            if g:
                self.o.set_client(int(s), int(g))

    def _owned(self, xs):
        return (xs >= self.lo) & (xs < self.hi)

    def tick(self, copy=True, no_events=False):
        w = np.concatenate(self.words)
        s = np.concatenate(self.stamps)
        self.words, self.stamps = [], []
        keep = (w[:, 0] & 0xFF) != 0
        w, s = w[keep], s[keep]
        # long movers: a row says so (RES_LONG), or an owned op moved one
        # further than max_step; their pairs are emitted by the other member's owner
        lng = np.zeros(len(self.x), bool)
        lng[w[((w[:, 0] >> 16) & dworld.RES_LONG) != 0][:, 1]] = True
        ops = dworld.words_to_ops(w[np.argsort(s, kind="stable")])
        x0, p0 = self.x.copy(), self.present.copy()
        for op in ops:
            k, sl = int(op["kind"]), int(op["slot"])
            if k in (T.OP_ENTER, T.OP_MOVED):
                self.x[sl], self.present[sl] = op["x"], True
            elif k == T.OP_LEAVE:
                self.present[sl] = False
        assert self.o.tick(ops) == 0
        e, l = self.o.events()
        lng |= p0 & self.present & (np.abs(self.x - x0) > self.max_step)
        xr = np.where(self.present, self.x, x0)
        own = self._owned(xr)

        def mine(ev):
            wt, tg = ev["watcher"], ev["target"]
            return ev[(own[wt] & ~lng[wt]) | (lng[wt] & own[tg] & ~lng[tg])].copy()
        enter, leave = mine(e), mine(l)
        # pairs of two long movers (group teleports): from every rank's long
        # list, by the owner of the watcher's new position (the engine's rule)
        L = getattr(self, "tick_longs", None)
        self.tick_longs = None
        if L is not None and len(L):
            d = np.float32(self.o_d)

            def rel(ax, az, as_, bx, bz, bs):
                cx, cz, ox, oz = (ax, az, bx, bz) if as_ > bs else (bx, bz, ax, az)
                return (ox >= np.float32(cx - d)) and (ox <= np.float32(cx + d)) and \
                       (oz >= np.float32(cz - d)) and (oz <= np.float32(cz + d))
            ee, ll = [], []
            for a in L:
                if not self._owned(np.float32(a["new_x"])):
                    continue
                for b in L:
                    if b["slot"] == a["slot"]:
                        continue
                    ro = rel(a["old_x"], a["old_z"], int(a["old_stamp"]), b["old_x"], b["old_z"], int(b["old_stamp"]))
                    rn = rel(a["new_x"], a["new_z"], int(a["new_stamp"]), b["new_x"], b["new_z"], int(b["new_stamp"]))
                    if ro != rn:
                        (ll if ro else ee).append((int(a["slot"]), int(b["slot"])))
            ev_t = enter.dtype
            enter = np.concatenate([enter, np.array(ee, dtype=np.uint32).reshape(-1, 2).view(ev_t).reshape(-1)])
            leave = np.concatenate([leave, np.array(ll, dtype=np.uint32).reshape(-1, 2).view(ev_t).reshape(-1)])
        return _Res(enter=enter, leave=leave)

    def collect(self, copy=True):
        r = self.o.collect()
        ent = r["entity"]
        # own records of leavers that kept their flag (the owner's copy; ghost
        # copies had theirs cleared by the LEAVE row) are emitted too
        keep = self._owned(self.x[ent]) & (self.present[ent] | (r["watcher"] == ent))
        return _Res(records=r[keep].copy())


class _Res:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--engine", choices=["oracle", "hip"], default="oracle")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--n", type=int, default=800)
    ap.add_argument("--strip-w", type=float, default=300.0)
    ap.add_argument("--height", type=float, default=600.0)
    ap.add_argument("--d", type=float, default=50.0)
    ap.add_argument("--max-step", type=float, default=8.0)
    ap.add_argument("--ticks", type=int, default=12)
    ap.add_argument("--collect-every", type=int, default=3)
    ap.add_argument("--trace", choices=["strip", "walk"], default="strip")
    ap.add_argument("--side", type=float, default=36864.0, help="walk: world side")
    ap.add_argument("--teleports", type=int, default=0, help="strip: jumps anywhere per tick")
    ap.add_argument("--groups", type=int, default=0, help="strip: group teleports per tick")
    a = ap.parse_args()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank,
                            world_size=a.world)
    if a.trace == "walk":
        tr = T.walk_strip_trace(a.seed, a.n, a.side, a.world, a.ticks)
    else:
        tr = T.strip_world_trace(a.seed, a.n, a.world, a.strip_w, a.height, a.d, a.ticks, a.max_step,
                                 teleports=a.teleports, groups=a.groups)
    geom = dworld.Strips(0.0, tr.strip_w, a.world, tr.d, tr.max_step)
    if a.engine == "oracle":
        eng, dev = OracleStrip(), torch.device("cpu")
    else:
        from goworld_amd import gpuaoi
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        eng = dworld.HipStrip(gpuaoi.GpuAOI(0))
    sr = dworld.StripRank(eng, geom, a.rank, a.n, tr.bounds, dev, comm="torch", comm_device=torch.device("cpu"))
    eng.set_clients(np.arange(a.n, dtype=np.uint32), tr.gates)
    out = {}
    for t in range(len(tr.ticks)):
        w = torch.from_numpy(dworld.ops_to_words(tr.rank_ops(t, a.rank)).copy()).to(dev)
        if a.trace == "walk" and t == 0:
            sr.step(w, copy=False, no_events=True)      # the load: no events, its records discarded
            sr.collect(copy=False)
            continue
        res = sr.step(w)
        out[f"enter_{t}"], out[f"leave_{t}"] = res.enter, res.leave
        if (t + 1) % a.collect_every == 0 or t == len(tr.ticks) - 1:
            out[f"rec_{t}"] = sr.collect().records
    sr.check()
    np.savez(a.out, **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
