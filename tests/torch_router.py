"""Torch statement of the decomposed-world routing protocol (test
infrastructure).

The product path routes on the GPU with gw_route_halo (goworld_amd/csrc/
halo.hip, driven by goworld_amd/dworld.HipRouter).  This module restates the
same protocol as eager torch ops: it is the mock engine's router of the CPU
multi-rank tests (tests/dworld_worker.py, gloo) and the row-for-row reference
of tests/test_dworld.py::test_hip_router_rows_match_torch_router.
"""
from __future__ import annotations

import torch

from goworld_amd.dworld import (OP_ENTER, OP_LEAVE, OP_MOVED, OP_SYNC, OP_WORDS, RES_LONG, ROW_WORDS,
                                ROWS_PER_ENTITY, SIF_MASK, Strips)


def _f32(words_col: torch.Tensor) -> torch.Tensor:
    return words_col.contiguous().view(torch.float32)


class Router:
    """Torch statement of the routing protocol (the GPU path runs HipRouter).

    State of one rank: position, presence and pending sync flags of every
    entity the rank holds (owned or ghost), indexed by global id (+ one dummy
    row, index n, that absorbs masked-out scatters and invalid slots)."""

    def __init__(self, geom: Strips, rank: int, n_global: int, device, halo_cap: int):
        self.g, self.r, self.n, self.dev, self.K = geom, rank, n_global, device, halo_cap
        n1 = n_global + 1
        self.x = torch.zeros(n1, dtype=torch.float32, device=device)
        self.z = torch.zeros(n1, dtype=torch.float32, device=device)
        self.stamp = torch.zeros(n1, dtype=torch.int64, device=device)    # of the last AOI op
        self.present = torch.zeros(n1, dtype=torch.bool, device=device)
        self.pflags = torch.zeros(n1, dtype=torch.int32, device=device)
        self.scratch = torch.full((n1,), -1, dtype=torch.int64, device=device)
        self.overflow = torch.zeros((), dtype=torch.int64, device=device)
        self.long_moves = torch.zeros((), dtype=torch.int64, device=device)
        self.last_far = {}
        self.last_longs = None
        self.ext_lo, self.ext_hi = geom.ext(rank)
        self.lo, self.hi = geom.lo(rank), geom.hi(rank)

    # -- per-entity reductions over one op list (scratch is left all -1) ----
    def _last(self, slot, idx, mask):
        t = self.scratch
        key = torch.where(mask, idx, torch.full_like(idx, -1))
        t.scatter_reduce_(0, slot, key, reduce="amax", include_self=True)
        out = t[slot]
        t[slot] = -1
        return out

    def _any(self, slot, bit, mask):
        t = self.scratch
        v = torch.where(mask, bit, torch.zeros_like(bit)).to(torch.int64)
        t.scatter_reduce_(0, slot, v, reduce="amax", include_self=True)
        out = t[slot].clamp(min=0).to(bit.dtype)
        t[slot] = -1
        return out

    def route(self, words: torch.Tensor, stamps: torch.Tensor, cap: int | None = None):
        """Owned ops of one tick -> (send to left, send to right): NOP-padded
        int32 row buffers (cap * 3, 8) in gw_halo_row layout (cap <= K
        entities).  Updates the routing state.  No host sync."""
        g, r = self.g, self.r
        cap = self.K if cap is None else min(cap, self.K)
        m = words.shape[0]
        dev = self.dev
        kind = words[:, 0] & 0xFF
        flags = (words[:, 0] >> 8) & SIF_MASK
        raw = words[:, 1].to(torch.int64) & 0xFFFFFFFF
        valid = (kind >= OP_ENTER) & (kind <= OP_SYNC) & (raw < self.n)
        slot = torch.where(valid, raw, torch.full((m,), self.n, dtype=torch.int64, device=dev))
        idx = torch.arange(m, dtype=torch.int64, device=dev)
        aoi = valid & (kind != OP_SYNC)
        lv = kind == OP_LEAVE
        la = self._last(slot, idx, aoi)                       # last AOI op
        ll = self._last(slot, idx, lv)                        # last Leave
        lp = self._last(slot, idx, valid & ~lv)               # last payload op
        lany = self._last(slot, idx, valid)                   # the entity's representative row
        # syncInfoFlag: a Leave's sync_flags is the mask of pending bits kept
        # (Space.leave leaves the flag alone, Space.go:219-242); per bit: the
        # old bit unless a Leave cleared it, OR the bits set after that Leave
        rep = valid & (lany == idx)
        has_aoi, had_leave = la >= 0, ll >= 0
        la_c, lp_c = la.clamp(min=0), lp.clamp(min=0)
        ka = kind[la_c]
        xa = _f32(words[:, 2])[la_c]
        za = _f32(words[:, 4])[la_c]
        old_x, old_p, old_f = self.x[slot], self.present[slot], self.pflags[slot]
        old_z, old_s = self.z[slot], self.stamp[slot]
        new_p = torch.where(has_aoi, ka != OP_LEAVE, old_p)
        new_x = torch.where(has_aoi & new_p, xa, old_x)
        new_z = torch.where(has_aoi & new_p, za, old_z)
        new_s = torch.where(has_aoi, stamps[la_c], old_s)
        new_f = torch.zeros_like(old_f)
        for c in range(2):
            bit = (flags >> c) & 1
            clr = self._last(slot, idx, valid & lv & (bit == 0))
            set_after = self._any(slot, bit, valid & ~lv & (idx > clr))
            keep = torch.where(clr < 0, (old_f >> c) & 1, torch.zeros_like(old_f))
            new_f |= (keep | set_after) << c
        # a long move (present before and after, |dx| > max_step, e.g. a
        # teleport): its AOI rows carry RES_LONG, and every rank whose held
        # range has the old or the new position gets rows, not only the
        # neighbours
        moved = rep & has_aoi & old_p & new_p
        lng = moved & ((new_x - old_x).abs() > g.max_step)
        self.long_moves += lng.sum()
        # the long-mover list (group teleports): state before and after the tick
        from goworld_amd.traces import LONG_DTYPE
        import numpy as np
        li = torch.nonzero(lng).flatten()
        lst = np.zeros(int(li.numel()), LONG_DTYPE)
        if li.numel():
            lst["slot"] = slot[li].cpu().numpy()
            lst["old_x"], lst["old_z"] = old_x[li].cpu().numpy(), old_z[li].cpu().numpy()
            lst["new_x"], lst["new_z"] = new_x[li].cpu().numpy(), new_z[li].cpu().numpy()
            lst["old_stamp"], lst["new_stamp"] = old_s[li].cpu().numpy(), new_s[li].cpu().numpy()
        self.last_longs = lst
        sends = []
        self.last_used = []
        self.last_far = {}
        dests = [(r - 1, True), (r + 1, True)]
        if bool(lng.any()):
            dests += [(q, False) for q in range(g.ranks) if abs(q - r) > 1]
        for nb, is_nb in dests:
            if nb < 0 or nb >= g.ranks:
                sends.append(None)
                continue
            lo, hi = g.ext(nb)
            was = old_p & (old_x >= lo) & (old_x < hi)
            now = new_p & (new_x >= lo) & (new_x < hi)
            nop = torch.zeros_like(kind)
            k0 = torch.where(has_aoi & had_leave & was & now, torch.full_like(kind, OP_LEAVE), nop)
            k1 = torch.where(now & (~was | had_leave), torch.full_like(kind, OP_ENTER),
                             torch.where(was & now, torch.full_like(kind, OP_MOVED),
                                         torch.where(was, torch.full_like(kind, OP_LEAVE), nop)))
            k1 = torch.where(has_aoi, k1, nop)
            k2 = torch.where(now & ((new_f != 0) | (lp > la)), torch.full_like(kind, OP_SYNC), nop)
            sel = rep & ((k0 | k1 | k2) != 0)
            if not is_nb:
                sel = sel & lng                         # far ranks hear only of long moves
            fl = torch.where(lng, torch.full_like(kind, RES_LONG << 16), nop)
            k0 = torch.where(k0 != 0, k0 | fl, k0)
            k1 = torch.where(k1 != 0, k1 | fl, k1)
            buf = self._pack(words, stamps, slot, sel, k0, ll.clamp(min=0), k1, la_c, k2, lp_c, new_f, lany, cap)
            if is_nb:
                sends.append(buf)
            else:
                used = self.last_used.pop()
                if used:
                    self.last_far[nb] = buf[:used * ROWS_PER_ENTITY]
        if bool(lng.any()):
            # this rank's own copy of a long mover that left its held range:
            # a LEAVE row for itself (keep-mask 0) after the tick's own ops,
            # so no rank keeps a copy outside its range
            away = lng & ~((new_x >= self.ext_lo) & (new_x < self.ext_hi))
            if bool(away.any()):
                nop = torch.zeros_like(kind)
                k1 = torch.where(away, torch.full_like(kind, OP_LEAVE | (RES_LONG << 16)), nop)
                buf = self._pack(words, stamps, slot, away, nop, la_c, k1, la_c, nop, lp_c,
                                 torch.zeros_like(new_f), lany, cap)
                self.last_far[r] = buf[:self.last_used.pop() * ROWS_PER_ENTITY]
        # routing state of the rows this rank owns (dummy row n absorbs the rest)
        s = torch.where(rep, slot, torch.full_like(slot, self.n))
        self.x[s] = new_x
        self.z[s] = new_z
        self.stamp[s] = new_s
        self.present[s] = new_p
        self.pflags[s] = new_f
        return sends[0], sends[1]

    def route_exact(self, words: torch.Tensor, stamps: torch.Tensor):
        """route() trimmed to the used rows (the exact-size exchange)."""
        sends = list(self.route(words, stamps))
        used = iter(self.last_used)
        return [None if b is None else b[:next(used) * ROWS_PER_ENTITY] for b in sends]

    def _pack(self, words, stamps, slot, sel, k0, i0, k1, i1, k2, i2, f2, i_last, K):
        """Entity rows (row 0, 1, 2 of each selected entity) compacted into a
        buffer of K entities; unused rows are NOPs (all-zero)."""
        m = words.shape[0]
        pos = torch.cumsum(sel.to(torch.int64), 0) - 1
        self.overflow = torch.maximum(self.overflow, sel.sum() - K)
        dst = torch.where(sel & (pos < K), pos, torch.full_like(pos, K))
        st32 = stamps.contiguous().view(torch.int32).view(-1, 2)
        rows = torch.zeros((m, ROWS_PER_ENTITY, ROW_WORDS), dtype=torch.int32, device=self.dev)
        s32 = slot.to(torch.int32)
        # row 0: LEAVE before a re-Enter inside the tick
        rows[:, 0, 0] = k0
        rows[:, 0, 1] = s32
        rows[:, 0, 6:] = st32[i0]
        # row 1: the net AOI op, with the last AOI op's payload and stamp
        rows[:, 1, 0] = k1
        rows[:, 1, 1] = s32
        rows[:, 1, 2:6] = words[i1, 2:6]
        rows[:, 1, 6:] = st32[i1]
        # row 2: SYNC with the latest payload and the pending flags
        rows[:, 2, 0] = k2 | (f2 << 8)
        rows[:, 2, 1] = s32
        rows[:, 2, 2:6] = words[i2, 2:6]
        rows[:, 2, 6:] = st32[i_last.clamp(min=0)]
        rows = rows * (torch.stack([k0, k1, k2], 1) != 0).to(torch.int32).unsqueeze(2)
        buf = torch.zeros((K + 1, ROWS_PER_ENTITY, ROW_WORDS), dtype=torch.int32, device=self.dev)
        buf.index_copy_(0, dst, rows)   # duplicates only at the trash row K
        self.last_used.append(int(min(int(sel.sum()), K)))
        return buf[:K].reshape(-1, ROW_WORDS)

    def receive(self, buf: torch.Tensor):
        """Ghost rows from a neighbour: updates the routing state."""
        rows = buf.view(-1, ROWS_PER_ENTITY, ROW_WORDS)
        k1 = rows[:, 1, 0] & 0xFF
        k2 = rows[:, 2, 0] & 0xFF
        f2 = (rows[:, 2, 0] >> 8) & SIF_MASK
        kany = (rows[:, 0, 0] | rows[:, 1, 0] | rows[:, 2, 0]) & 0xFF
        slot = torch.maximum(torch.maximum(rows[:, 0, 1], rows[:, 1, 1]), rows[:, 2, 1]).to(torch.int64)
        slot = torch.where(kany != 0, slot, torch.full_like(slot, self.n))
        cur_x, cur_p, cur_z, cur_s = self.x[slot], self.present[slot], self.z[slot], self.stamp[slot]
        p = torch.where(k1 != 0, k1 != OP_LEAVE, cur_p)
        x = torch.where((k1 != 0) & p, _f32(rows[:, 1, 2]), cur_x)
        zz = torch.where((k1 != 0) & p, _f32(rows[:, 1, 4]), cur_z)
        st = torch.where(k1 != 0, rows[:, 1, 6:8].contiguous().view(torch.int64).view(-1), cur_s)
        f = torch.where(k2 != 0, f2, torch.zeros_like(f2))
        self.x[slot] = x
        self.z[slot] = zz
        self.stamp[slot] = st
        self.present[slot] = p
        self.pflags[slot] = f

    def collected(self):
        """Sync flags are cleared everywhere by a collect (Entity.go:1221-1267)."""
        self.pflags.zero_()

    def longs_exact(self):
        """This rank's long-mover list of the last route() (gw_long_move rows)."""
        return self.last_longs

    def far_exact(self) -> dict:
        """Rows of the last route() for ranks that are not neighbours (long
        moves only), exact size: {rank: (rows, 8) int32}."""
        return dict(self.last_far)

    def status(self):
        """(overflow, long-move conflicts (not detected here: 0), bad ops)."""
        ov = int(self.overflow.item())
        self.overflow.zero_()
        return max(ov, 0), 0, 0

    def long_count(self):
        v = int(self.long_moves.item())
        self.long_moves.zero_()
        return v


def split_rows(buf: torch.Tensor):
    """gw_halo_row buffer (rows, 8) int32 -> (op words (rows, 6), stamps (rows,))."""
    return buf[:, :OP_WORDS].contiguous(), buf[:, OP_WORDS:].contiguous().view(torch.int64).view(-1)
