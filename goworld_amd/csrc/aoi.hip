// aoi.hip — gfx950 kernels of one AOI tick.
//
// The relation of a pair is a pure function of the current positions and of
// the global stamps of the members' last AOI ops (gw_internal.hpp, DESIGN.md
// §2), so the tick keeps no neighbour lists.  For one tick:
//   ops      last-op dedupe per slot; movers save their pre-tick position and
//            stamp (PrevEnt), take a new stamp and join the mover list
//   grid     incremental: movers that stay in their cell are patched in
//            place; cells that lose or gain entities are re-sorted by slot (a
//            wave per cell, LDS bitonic), every other cell is shifted by the
//            scan of the new cell counts.  gn stays in (cell, slot) order.
//   gm       mover grid: each mover at its old and its new cell (counting
//            sort whose cursor counts back to zero)
//   diff     one wave per mover (in mover-grid order, i.e. by cell: windows
//            of neighbouring waves overlap in L2) walks the non-movers of gn
//            and the mover grid over its old and new windows, evaluates the
//            old and new relation of every candidate and emits own events,
//            sorted
//   mirror   the relation is symmetric, so an own event (A,B) of a mover with
//            an op-less B is also B's event (B,A): the mover keeps (B, A) in
//            its region (no atomics: device-scope atomics run memory-side on a
//            multi-XCD part, so a count per mirror event cost more than the
//            event itself)
//   events   movers in slot order (bitmap compaction), their own and mirror
//            events flattened into one array (key = leave<<wbits | watcher,
//            value = target), one stable LSD radix sort by key: mirror events
//            enter the sort in mover-slot order and own events target-sorted,
//            so the result is the canonical (watcher, target) order, enters
//            then leaves, written as gw_event by the last pass
// Outputs are placed by scans and sorts; the atomics left are histogram /
// cursor updates of the grid, one bitmap OR per mover and per-shard
// statistics.  No MFMA: compare and gather work bound by L2/HBM latency and
// bandwidth.
#include "dev_common.hpp"

namespace gw {

constexpr uint32_t SORT_LDS = 1024;     // own events sorted in a wave's LDS up to this many
constexpr uint32_t NO_CELL = 0xffffffffu;

// appends v for every lane with pred to list (64-bit counter), one atomic per
// wave; every lane of the wave must call it
__device__ __forceinline__ void wave_append(bool pred, uint32_t v, uint32_t* list, unsigned long long* cnt) {
    const uint64_t bm = wave_ballot(pred);
    if (!bm) return;
    const int leader = __builtin_ctzll(bm);
    unsigned long long base = 0;
    if (lane_id() == leader) base = atomicAdd(cnt, (unsigned long long)popc64(bm));
    base = __shfl(base, leader, 64);
    if (pred) list[base + (uint64_t)popc64(bm & lanemask_lt())] = v;
}

// ---------------------------------------------------------------------------
// ops: last-op dedupe per slot (seq = index in the tick's op stream).  Every
// op stores its tagged index into its slot's words with plain stores (one of
// the racing values lands); k_ops2 then raises each word to the largest index
// with an atomicMax from the ops that find a smaller one, i.e. only where a
// slot has several ops.  (An atomicMax per word and op runs memory-side on a
// multi-XCD part: 2M of them took 90 us at config #4's 1M ops.)
__global__ void __launch_bounds__(NT) k_ops1(TickBufs b) {
    const uint32_t i = b.op0 + blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    if (op.kind == GW_OP_NOP) return;
    if (op.slot >= b.w.cap || op.kind > GW_OP_SYNC) {
        atomicAdd(&b.st->bad_ops, 1ull);
        return;
    }
    const unsigned long long v = ol_put(b.ol_tag, i);
    OpLast& o = b.ol[op.slot];
    if (op.kind != GW_OP_LEAVE) o.pos = v;
    if (op.kind != GW_OP_SYNC) o.aoi = v;
    if (op.kind == GW_OP_LEAVE) {
        o.leave = v;
        for (int c = 0; c < 2; ++c)                     // the last Leave that clears bit c
            if (!((op.sync_flags >> c) & 1)) o.clr[c] = v;
    }
}
__global__ void __launch_bounds__(NT) k_ops2(TickBufs b) {
    const uint32_t i = b.op0 + blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    if (op.kind == GW_OP_NOP || op.slot >= b.w.cap || op.kind > GW_OP_SYNC) return;
    const unsigned long long v = ol_put(b.ol_tag, i);
    OpLast& w = b.ol[op.slot];
    const OpLast o = w;
    const int32_t me = (int32_t)i;
    if (op.kind != GW_OP_LEAVE && ol_get(o.pos, b.ol_tag) < me) atomicMax(&w.pos, v);
    if (op.kind != GW_OP_SYNC && ol_get(o.aoi, b.ol_tag) < me) atomicMax(&w.aoi, v);
    if (op.kind == GW_OP_LEAVE) {
        if (ol_get(o.leave, b.ol_tag) < me) atomicMax(&w.leave, v);
        for (int c = 0; c < 2; ++c)
            if (!((op.sync_flags >> c) & 1) && ol_get(o.clr[c], b.ol_tag) < me) atomicMax(&w.clr[c], v);
    }
}

// syncInfoFlag across a Leave.  Space.leave leaves the flag alone (Space.go:
// 219-242); a Leave's sync_flags is the mask of pending bits the entity keeps
// (all when it stays in the game in the nil space, none when it is destroyed
// or enters another AOI space, whose Enter flags it anew).  In call order the
// ops are f -> (f & mask) and f -> (f | bits); per bit c the result is: the
// old bit unless some Leave cleared c, OR'd with the bits of the ops after the
// last Leave that cleared c.  The slot's last Leave clears in k_ops3, every
// op's bits after it are OR'd in by k_place (a later launch: clear, then OR).
__device__ __forceinline__ uint2 classify_mover(const TickBufs& b, uint32_t i, uint32_t A, const AoiEnt& a,
                                                const PrevEnt& p, bool lng, uint32_t gate, uint32_t gidx);

// Per op: the syncInfoFlag bits, the sync payload of the slot's last
// non-Leave op; the slot's last AOI op saves the pre-tick position and stamp
// (PrevEnt), takes its stamp, updates the AOI state and classifies the mover
// for the incremental grid (state in registers: no second pass re-reading the
// op, the dedupe record and the slot state)
__global__ void __launch_bounds__(NT) k_ops3(TickBufs b) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    bool mv = false, lng = false;
    uint32_t s = 0, fbits = 0;
    AoiEnt a;
    PrevEnt p;
    uint32_t gate = 0;
    uint32_t gidx = 0;
    if (i < b.m) {
        const gw_op op = b.ops[i];
        s = op.slot;
        if (s < b.w.cap && op.kind >= GW_OP_ENTER && op.kind <= GW_OP_SYNC) {
            const OpLast o = b.ol[s];
            // the slot's state, loaded with its dedupe record (used when op i
            // is the slot's last AOI op, nearly always): one round trip less
            const AoiEnt a0 = b.w.rec[s].a;
            const unsigned long long st0 = b.w.rec[s].stamp;
            gidx = b.w.rec[s].gidx;
            gate = b.w.rec[s].gate;
            struct { int32_t pos, aoi, leave, clr[2]; } ol;
            ol.pos = ol_get(o.pos, b.ol_tag);
            ol.aoi = ol_get(o.aoi, b.ol_tag);
            ol.leave = ol_get(o.leave, b.ol_tag);
            ol.clr[0] = ol_get(o.clr[0], b.ol_tag);
            ol.clr[1] = ol_get(o.clr[1], b.ol_tag);
            // syncInfoFlag |= bits of every call after the last Leave that
            // cleared them (Space.go:196, Entity.go:1199-1204, 1286): OR'd in
            // by k_place, after the slot's last Leave cleared its bits here
            if (op.kind != GW_OP_LEAVE && op.sync_flags) {
                for (int c = 0; c < 2; ++c)
                    if (((op.sync_flags >> c) & 1) && (int32_t)i > ol.clr[c]) fbits |= 1u << c;
            } else if (op.kind == GW_OP_LEAVE && ol.leave == (int32_t)i) {
                uint32_t clear = 0;
                for (int c = 0; c < 2; ++c)
                    if (ol.clr[c] >= 0) clear |= 1u << c;
                if (clear) atomicAnd(&b.w.flags[flag_word(s)], ~(clear << flag_sh(s)));
            }
            if (ol.pos == (int32_t)i) b.w.rec[s].p = make_float4(op.x, op.y, op.z, op.yaw);
            if (ol.aoi == (int32_t)i) {                 // the slot's mover entry (never a SYNC op)
                a = a0;
                const bool was = (a.meta & PRESENT_BIT) != 0;
                p.ox = was ? a.x : qnan();
                p.oz = was ? a.z : qnan();
                p.ostamp = st0;
                b.w.rec[s].pv = p;
                b.w.rec[s].stamp = b.stamps ? b.stamps[i] : b.stamp_base + i;
                if (op.kind == GW_OP_LEAVE) a.meta &= ~PRESENT_BIT;
                else { a.x = op.x; a.z = op.z; a.meta |= PRESENT_BIT; }
                b.w.rec[s].a = a;
                mv = true;
                // decomposed world: a long mover (a halo row says so, or an
                // owned op moved it further than max_step)
                lng = (op.reserved & RES_LONG) != 0 ||
                      (was && (a.meta & PRESENT_BIT) && fabsf(a.x - p.ox) > b.long_step);
            }
        }
    }
    // mover count: one add per wave into a private-ish shard (a per-block add
    // to one counter serialised ~4k atomics at 1M ops: ~100 us at config #4)
    const uint32_t nw = (uint32_t)popc64(wave_ballot(mv));
    if (lane_id() == 0 && nw) shard_add(b.st, blockIdx.x * NWAVE + (threadIdx.x >> 6), SH_MOVERS, nw);
    uint2 cc = make_uint2(NO_CELL, NO_CELL);
    if (mv) cc = classify_mover(b, i, s, a, p, lng, gate, gidx);
    if (i < b.m) b.mcell[i] = make_uint4(cc.x, cc.y, s, fbits);   // k_place reads them back coalesced
}

// Restore path (Space.go:209-214, EntityManager.go:556-617): entity i enters
// with stamp base + i, i.e. exactly as n Enter calls in index order; with no
// neighbour lists there is nothing else to build (the grid is rebuilt next).
__global__ void __launch_bounds__(NT) k_restore(World w, const uint32_t* __restrict__ slots,
                                                const float4* __restrict__ xyzw, uint32_t n,
                                                unsigned long long stamp_base, uint32_t flags) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slots[i];
    const float4 p = xyzw[i];
    AoiEnt a = w.rec[s].a;
    a.x = p.x;
    a.z = p.z;
    a.meta |= PRESENT_BIT;
    w.rec[s].a = a;
    w.rec[s].p = p;
    w.rec[s].stamp = stamp_base + i;
    if (flags & 3u) atomicOr(&w.flags[flag_word(s)], (flags & 3u) << flag_sh(s));
}
void launch_restore(const World& w, const uint32_t* slots, const float4* xyzw, uint32_t n,
                    unsigned long long stamp_base, uint32_t flags, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_restore, dim3(nblk(n, NT)), dim3(NT), 0, s, w, slots, xyzw, n, stamp_base, flags);
}

void tick_ops(const TickBufs& b, hipStream_t s) {
    if (b.m > b.op0) {
        hipLaunchKernelGGL(k_ops1, dim3(nblk(b.m - b.op0, NT)), dim3(NT), 0, s, b);
        hipLaunchKernelGGL(k_ops2, dim3(nblk(b.m - b.op0, NT)), dim3(NT), 0, s, b);
    }
    hipLaunchKernelGGL(k_ops3, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// full rebuild: stable LSD radix sort of (cell, slot) pairs (absent slots get
// the sentinel key ncells and sort last), so gn[] is in (cell, slot) order
__global__ void __launch_bounds__(NT) k_grid_keys(World w, uint32_t* k0, uint32_t* v0) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s >= w.cap) return;
    const AoiEnt a = w.rec[s].a;
    uint32_t key = w.ncells;
    if (a.meta & PRESENT_BIT) key = cell_of(w.sp[a.meta & SPACE_MASK], a.x, a.z);
    k0[s] = key;
    v0[s] = s;
}
__global__ void __launch_bounds__(NT) k_grid_fill(World w, const uint32_t* __restrict__ keys,
                                                  const uint32_t* __restrict__ slots) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= w.cap) return;
    const uint32_t key = keys[i];
    if (key < w.ncells) {
        const uint32_t s = slots[i];
        const AoiEnt a = w.rec[s].a;
        GEnt e;
        e.x = a.x; e.z = a.z; e.slot = s;
        e.meta = key | gate_meta(w.rec[s].gate);
        w.gn[i] = e;
    }
}
// gidx = offset of the slot's entry inside its cell (stays valid while the
// cell shifts as a block; rewritten only where the cell is re-merged)
__global__ void __launch_bounds__(NT) k_grid_rel(World w) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= w.gn_start[w.ncells]) return;
    const GEnt e = w.gn[i];
    w.rec[e.slot].gidx = i - w.gn_start[e.meta & CELL_MASK];
}
// gn_start[c] = first index with key >= c (binary search over the sorted keys)
__global__ void __launch_bounds__(NT) k_grid_starts(World w, const uint32_t* __restrict__ keys, DevStats* st) {
    uint32_t c = blockIdx.x * NT + threadIdx.x;
    if (c > w.ncells) return;
    uint32_t lo = 0, hi = w.cap;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (keys[mid] < c) lo = mid + 1; else hi = mid;
    }
    w.gn_start[c] = lo;
    if (c == w.ncells && st) st->n_present = lo;
}

void grid_rebuild(const World& w, DevStats* st, uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1,
                  RadixTmp& rt, int key_bits, hipStream_t s) {
    const uint32_t C = w.cap;
    hipLaunchKernelGGL(k_grid_keys, dim3(nblk1(C, NT)), dim3(NT), 0, s, w, k0, v0);
    int r = radix_sort<uint32_t>(k0, v0, k1, v1, C, nullptr, 0, key_bits, rt, s);
    const uint32_t* keys = r ? k1 : k0;
    const uint32_t* slots = r ? v1 : v0;
    hipLaunchKernelGGL(k_grid_fill, dim3(nblk1(C, NT)), dim3(NT), 0, s, w, keys, slots);
    hipLaunchKernelGGL(k_grid_starts, dim3(nblk1((uint64_t)w.ncells + 1, NT)), dim3(NT), 0, s, w, keys, st);
    hipLaunchKernelGGL(k_grid_rel, dim3(nblk1(C, NT)), dim3(NT), 0, s, w);
}

// ---------------------------------------------------------------------------
// incremental grid.  co / cn: the mover's cell before / after the tick
// (NO_CELL when absent).  co is the cell its pre-tick grid entry sits in.  A
// mover is slot s's last AOI op (no list: a single-address list counter
// serialises across the chip).

// per mover: mover-grid histogram; a mover staying in its cell is patched in
// place, the others count as a departure / an arrival of their cells (called
// by k_ops3, op i, with the slot's state after the tick and before it).  The
// mover's mover-grid entry (tags aside) goes to mtmp[i] and its cells are
// returned for mcell[i], so k_place reads them coalesced.
__device__ __forceinline__ uint2 classify_mover(const TickBufs& b, uint32_t i, uint32_t A, const AoiEnt& a,
                                                const PrevEnt& p, bool lng, uint32_t gate, uint32_t gidx) {
    const SpaceP P = b.w.sp[a.meta & SPACE_MASK];
    uint32_t co = NO_CELL, cn = NO_CELL;
    if (p.ox == p.ox) co = cell_of(P, p.ox, p.oz);
    if (a.meta & PRESENT_BIT) cn = cell_of(P, a.x, a.z);
    if (co != NO_CELL || cn != NO_CELL) {
        const bool pn = cn != NO_CELL;
        MEnt m;
        m.x = pn ? a.x : qnan(); m.z = pn ? a.z : qnan();
        m.ox = p.ox; m.oz = p.oz;
        m.slot = A; m.tags = lng ? TAG_LONG : 0u; m.client = gate; m.space = a.meta & SPACE_MASK;   // client: its gate
        b.mtmp[i] = m;
    }
    const uint32_t at = co != NO_CELL ? b.w.gn_start[co] + gidx : 0u;   // (loaded before the atomics)
    if (co != NO_CELL) atomicAdd(&b.gm_cnt[co], 1u);
    if (cn != NO_CELL && cn != co) atomicAdd(&b.gm_cnt[cn], 1u);
    if (co != NO_CELL && co == cn) {
        GEnt e;
        e.x = a.x; e.z = a.z; e.slot = A;
        e.meta = cn | gate_meta(gate) | b.mbit;
        b.w.gn[at] = e;
    } else {
        if (co != NO_CELL) {
            atomicAdd(&b.dep[co], 1u);
            b.w.gn[at].slot = DEPARTED;
        }
        if (cn != NO_CELL) atomicAdd(&b.arr[cn], 1u);
    }
    return make_uint2(co, cn);
}

// per cell: entries after the tick; cells with departures or arrivals are
// flagged dirty
__global__ void __launch_bounds__(NT) k_cellcnt(TickBufs b) {
    const uint32_t c = blockIdx.x * NT + threadIdx.x;
    const uint32_t NC = b.w.ncells;
    if (c < NC) {
        const uint32_t old = b.w.gn_start[c + 1] - b.w.gn_start[c];
        const uint32_t d = b.dep[c], r = b.arr[c];
        b.cnt_new[c] = old - d + r;
        if (d | r) b.dep[c] = d | CELL_DIRTY;
    } else if (c == NC) {
        b.cnt_new[c] = 0;
    }
}

// per mover: its mover-grid entries (the cursor counts gm_cnt back to zero)
// and, for an arrival, its grid entry behind the kept entries of the new cell
__device__ __forceinline__ void place_one(const TickBufs& b, uint32_t i) {
    if (i >= b.m) return;
    const uint4 cc = b.mcell[i];
    if (cc.w) atomicOr(&b.w.flags[flag_word(cc.z)], cc.w << flag_sh(cc.z));   // op i's syncInfoFlag bits
    const uint32_t co = cc.x, cn = cc.y;
    if (co == NO_CELL && cn == NO_CELL) return;             // not a mover, or absent before and after
    const bool pn = cn != NO_CELL;
    const bool arrive = pn && cn != co;
    // every load, then every cursor atomic, all in flight together (an atomic
    // with a return made the loads after it wait for it)
    MEnt e = b.mtmp[i];
    uint32_t so = 0, sn = 0, g0 = 0, g1 = 0, dp = 0, nx = 0;
    if (co != NO_CELL) so = b.gm_start[co];
    if (arrive) {
        sn = b.gm_start[cn];
        g0 = b.w.gn_start[cn];
        g1 = b.w.gn_start[cn + 1];
        dp = b.dep[cn];
        nx = b.start_nxt[cn];
    }
    uint32_t ro = 0, rn = 0, ra = 0;
    if (co != NO_CELL) ro = atomicSub(&b.gm_cnt[co], 1u);
    if (arrive) {
        rn = atomicSub(&b.gm_cnt[cn], 1u);
        ra = atomicSub(&b.arr[cn], 1u);
    }
    const uint32_t gm_meta = gate_meta(e.client);            // (the mover's gate)
    if (co != NO_CELL) {
        e.tags = (e.tags & TAG_LONG) | TAG_OLD | (cn == co ? TAG_NEW | TAG_PRIMARY : 0u) | (pn ? 0u : TAG_PRIMARY);
        b.gm[so + ro - 1u] = e;
    }
    if (arrive) {
        e.tags = (e.tags & TAG_LONG) | TAG_NEW | TAG_PRIMARY;
        b.gm[sn + rn - 1u] = e;
        const uint32_t kept = (g1 - g0) - (dp & ~CELL_DIRTY);
        GEnt g;
        g.x = e.x; g.z = e.z; g.slot = e.slot;
        g.meta = cn | gm_meta | b.mbit;
        b.gn_nxt[nx + kept + ra - 1u] = g;
    }
}

// clean cells move as a block: new index = start_nxt + offset in the cell
// (grid-stride over the present entries: the grid is sized by the slot
// capacity, a world strip holds a fraction of it)
__device__ __forceinline__ void grid_copy(const TickBufs& b, uint32_t blk, uint32_t nblk) {
    const uint32_t n = b.w.gn_start[b.w.ncells];
    for (uint32_t i = blk * NT + threadIdx.x; i < n; i += nblk * NT) {
        GEnt e = b.w.gn[i];
        if (e.slot == DEPARTED) continue;
        const uint32_t c = e.meta & CELL_MASK;
        if (b.dep[c] & CELL_DIRTY) continue;
        e.meta &= ~b.mstale;                                      // the last tick's mover bit
        b.gn_nxt[b.start_nxt[c] + (i - b.w.gn_start[c])] = e;   // gidx (offset in the cell) unchanged
    }
}
__global__ void __launch_bounds__(NT) k_place(TickBufs b) { place_one(b, blockIdx.x * NT + threadIdx.x); }
__global__ void __launch_bounds__(NT) k_grid_copy(TickBufs b) { grid_copy(b, blockIdx.x, gridDim.x); }
// both in one launch (they touch disjoint cells of the new grid: arrivals
// into dirty cells, clean cells as blocks): blocks [0, np) place, the rest copy
__global__ void __launch_bounds__(NT) k_place_copy(TickBufs b, uint32_t np) {
    if (blockIdx.x < np) place_one(b, blockIdx.x * NT + threadIdx.x);
    else grid_copy(b, blockIdx.x - np, gridDim.x - np);
}

// Dirty cells: the kept entries (already in slot order) merge with the
// arrivals (few, in arrival order at the cell's tail) by rank: a kept entry
// moves up by the arrivals with a smaller slot, an arrival lands after the
// kept entries and arrivals with a smaller slot.  A wave scans the flags of
// dirty_span cells and merges its dirty ones; cells with more than 64
// arrivals are compacted and sorted by the wave (bitonic, in place).
__device__ __forceinline__ void grid_dirty(const TickBufs& b, uint32_t blk) {
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t span = b.dirty_span;
    const uint32_t c0 = (blk * NWAVE + (threadIdx.x >> 6)) * span;
    if (c0 >= b.w.ncells) return;
    const uint32_t cl = c0 + ln;
    uint64_t dm = wave_ballot(ln < (int)span && cl < b.w.ncells && (b.dep[cl] & CELL_DIRTY));
    while (dm) {
        const uint32_t c = c0 + (uint32_t)__builtin_ctzll(dm);
        dm &= dm - 1;
        const uint32_t so = b.w.gn_start[c], old = b.w.gn_start[c + 1] - so;
        const uint32_t sn = b.start_nxt[c], nn = b.start_nxt[c + 1] - sn;
        const uint32_t kept = old - (b.dep[c] & ~CELL_DIRTY);
        const uint32_t narr = nn - kept;
        if (narr > 64) {                          // rare: compact the kept entries, sort the cell
            uint32_t run = 0;
            for (uint32_t base = 0; base < old; base += 64) {
                const uint32_t i = base + ln;
                GEnt e;
                e.slot = DEPARTED;
                if (i < old) e = b.w.gn[so + i];
                e.meta &= ~b.mstale;                  // the last tick's mover bit
                const bool keep = i < old && e.slot != DEPARTED;
                const uint64_t bm = wave_ballot(keep);
                if (keep) b.gn_nxt[sn + run + (uint32_t)popc64(bm & lt)] = e;   // arrivals sit behind `kept`
                run += (uint32_t)popc64(bm);
            }
            wave_sync();
            bitonic_inplace<64>(b.gn_nxt + sn, nn, ln, [](const GEnt& e) { return e.slot; }, [] { wave_sync(); });
            for (uint32_t j = (uint32_t)ln; j < nn; j += 64) b.w.rec[b.gn_nxt[sn + j].slot].gidx = j;
            if (ln == 0) b.dep[c] = 0;
            continue;
        }
        // arrivals: one per lane, read before any write of the cell's new range
        GEnt ar;
        ar.slot = 0xffffffffu;
        if (ln < (int)narr) ar = b.gn_nxt[sn + kept + ln];
        uint32_t arank = 0;                       // arrivals with a smaller slot, then + kept below
        for (uint32_t j = 0; j < narr; ++j) {
            const uint32_t aj = (uint32_t)__builtin_amdgcn_readlane((int)ar.slot, (int)j);
            arank += (ln < (int)narr && aj < ar.slot) ? 1u : 0u;
        }
        uint32_t k0 = 0;                          // kept entries before this chunk
        for (uint32_t base = 0; base < old; base += 64) {
            const uint32_t i = base + ln;
            GEnt e;
            e.slot = DEPARTED;
            if (i < old) e = b.w.gn[so + i];
            e.meta &= ~b.mstale;                  // the last tick's mover bit
            const bool keep = i < old && e.slot != DEPARTED;
            const uint64_t bm = wave_ballot(keep);
            uint32_t below = 0;                   // arrivals below this kept entry
            for (uint32_t j = 0; j < narr; ++j) {
                const uint32_t aj = (uint32_t)__builtin_amdgcn_readlane((int)ar.slot, (int)j);
                below += aj < e.slot ? 1u : 0u;
                const uint32_t kb = (uint32_t)popc64(wave_ballot(keep && e.slot < aj));
                if (ln == (int)j) arank += kb;
            }
            if (keep) {
                const uint32_t at = sn + k0 + (uint32_t)popc64(bm & lt) + below;
                b.gn_nxt[at] = e;
                b.w.rec[e.slot].gidx = at - sn;
            }
            k0 += (uint32_t)popc64(bm);
        }
        if (ln < (int)narr) {
            b.gn_nxt[sn + arank] = ar;
            b.w.rec[ar.slot].gidx = arank;
        }
        if (ln == 0) b.dep[c] = 0;
    }
}
__global__ void __launch_bounds__(NT) k_grid_dirty(TickBufs b) { grid_dirty(b, blockIdx.x); }
static uint32_t dirty_blocks(const TickBufs& b) { return nblk1((uint64_t)b.w.ncells, b.dirty_span * NWAVE); }


void tick_grid(const TickBufs& b, ScanCtx& sc, hipStream_t s, bool dirty) {
    const uint32_t NC = b.w.ncells;
    hipLaunchKernelGGL(k_cellcnt, dim3(nblk1((uint64_t)NC + 1, NT)), dim3(NT), 0, s, b);
    // both cell scans in one launch; totals land in the low words of the
    // (zeroed, little-endian) 64-bit counters.  (Computing the cell counts in
    // the scan's loads instead of k_cellcnt: grid stage +10 us at config #3,
    // +23 us at config #4 -- the tiles post their aggregates later.)
    scan_pair32(b.cnt_new, b.gm_cnt, b.start_nxt, b.gm_start, (uint64_t)NC + 1, sc, (uint32_t*)&b.st->n_present,
                (uint32_t*)&b.st->n_gm, s);
    const uint32_t np = nblk1(b.m, NT), nc = std::min<uint32_t>(nblk1(b.w.cap, NT), 16384);
    if (b.place_split) {                                    // two launches (for comparison)
        hipLaunchKernelGGL(k_place, dim3(np), dim3(NT), 0, s, b);
        hipLaunchKernelGGL(k_grid_copy, dim3(nc), dim3(NT), 0, s, b);
    } else {
        hipLaunchKernelGGL(k_place_copy, dim3(np + nc), dim3(NT), 0, s, b, np);
    }
    if (dirty) hipLaunchKernelGGL(k_grid_dirty, dim3(dirty_blocks(b)), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// The cells a mover scans: the rectangles of its old and new windows, merged
// into their bounding box when they touch (visiting extra cells is harmless:
// every candidate is evaluated exactly, each cell once).
__device__ __forceinline__ Rects mover_rects(const SpaceP& P, bool po, float ox, float oz, bool pn, float x,
                                             float z) {
    Rects m;
    m.n = 0;
    Rect ro = po ? search_rect(P, ox, oz) : empty_rect();
    Rect rn = pn ? search_rect(P, x, z) : empty_rect();
    if (!ro.empty() && !rn.empty()) {
        const bool touch = ro.x0 <= rn.x1 + 1 && rn.x0 <= ro.x1 + 1 && ro.z0 <= rn.z1 + 1 && rn.z0 <= ro.z1 + 1;
        if (touch) {
            Rect u;
            u.x0 = min(ro.x0, rn.x0); u.x1 = max(ro.x1, rn.x1);
            u.z0 = min(ro.z0, rn.z0); u.z1 = max(ro.z1, rn.z1);
            m.r[m.n++] = u;
        } else {
            m.r[m.n++] = ro;
            m.r[m.n++] = rn;
        }
    } else if (!ro.empty()) {
        m.r[m.n++] = ro;
    } else if (!rn.empty()) {
        m.r[m.n++] = rn;
    }
    return m;
}

// candidate bound of each primary mover-grid entry (entries of gn and gm in
// its cells) -> the size of its own-event region.  The index ranges of its
// rows (<= RR_ROWS) go to rowrec for k_mover, whose wave then starts its walk
// one load after its entry instead of three (entry -> space -> row starts).
// (gs: the new grid's row starts -- b.w.gn_start once b.w is the new grid,
// b.start_nxt before)
__device__ __forceinline__ void bounds_one(const TickBufs& b, uint64_t m, const uint32_t* __restrict__ gs) {
    const uint64_t ngm = b.st->n_gm;
    if (m >= ngm && !(b.heavy_min && m - lane_id() < ngm)) return;   // heavy mode: whole waves reach the ballot
    MEnt e;
    e.tags = 0;
    if (m < ngm) e = b.gm[m];
    uint64_t c = 0;
    if (e.tags & TAG_PRIMARY) {
        const SpaceP P = b.w.sp[e.space];
        const Rects R = mover_rects(P, e.ox == e.ox, e.ox, e.oz, e.x == e.x, e.x, e.z);
        uint4* rec = b.rowrec ? b.rowrec + m * RR_ROWS : nullptr;
        uint32_t nr = 0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (q >= R.n) break;
            const Rect rr = q == 0 ? R.r[0] : R.r[1];
            for (int cz = rr.z0; cz <= rr.z1; ++cz, ++nr) {
                const uint32_t row = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
                const uint32_t g0 = gs[row + rr.x0], g1 = gs[row + rr.x1 + 1];
                const uint32_t m0 = b.gm_start[row + rr.x0], m1 = b.gm_start[row + rr.x1 + 1];
                c += (g1 - g0) + (m1 - m0);
                if (rec && nr < RR_ROWS) rec[nr] = make_uint4(g0, g1, m0, m1);
            }
        }
        if (rec) {
            if (nr > RR_ROWS) rec[0] = make_uint4(1u, 0u, 0u, 0u);   // too many rows: k_mover builds its own
            for (uint32_t r = nr; r < RR_ROWS; ++r) rec[r] = make_uint4(0u, 0u, 0u, 0u);
        }
        if (e.tags & TAG_LONG) c += b.n_long;   // its pairs with the other long movers (long_pairs)
    } else if (m < ngm) {         // a secondary entry has no events or statistics (coalesced here)
        b.mstat[m] = 0;
        b.ownc[m] = 0;
        b.mirc[m] = 0;
    }
    // heavy-first mode: the longest walks are listed apart and dispatched first
    const bool hv = (e.tags & TAG_PRIMARY) && b.heavy_min && c >= b.heavy_min;
    const uint64_t hm = wave_ballot(hv);
    if (hm) {
        const int leader = __builtin_ctzll(hm);
        uint32_t base = 0;
        if (lane_id() == leader) base = (uint32_t)atomicAdd(&b.st->n_heavy, (unsigned long long)popc64(hm));
        base = __shfl(base, leader, 64);
        if (hv) b.heavy[base + (uint32_t)popc64(hm & lanemask_lt())] = (uint32_t)m;
    }
    if (m < ngm) b.cand[m] = c | ((e.tags & TAG_PRIMARY) && !hv ? PRIM_ONE : 0ull);
}
__global__ void __launch_bounds__(NT) k_bounds(TickBufs b) {
    bounds_one(b, (uint64_t)blockIdx.x * NT + threadIdx.x, b.w.gn_start);
}
// the dirty cells' merges and the bounds in one launch: the bounds read the
// new grid's row starts and the mover grid, not its entries (b: the buffers
// before the flip to the new grid; blocks [0, nd) merge)
__global__ void __launch_bounds__(NT) k_dirty_bounds(TickBufs b, uint32_t nd) {
    if (blockIdx.x < nd) grid_dirty(b, blockIdx.x);
    else bounds_one(b, (uint64_t)(blockIdx.x - nd) * NT + threadIdx.x, b.start_nxt);
}

// the scan of the tagged bounds lists the primary entries in mover-grid
// (cell) order: pidx[k] = the k-th, k_mover's wave k
struct PrimPost {
    uint32_t* pidx;
    __device__ bool active() const { return pidx != nullptr; }
    __device__ void operator()(uint64_t i, uint64_t excl, uint64_t x) const {
        if (x >> PRIM_SHIFT) pidx[excl >> PRIM_SHIFT] = (uint32_t)i;
    }
};

void tick_movers(const TickBufs& b, ScanCtx& sc, hipStream_t s, const TickBufs* pre) {
    const uint64_t nmax = 2ull * b.m;
    const uint64_t* ngm = (const uint64_t*)&b.st->n_gm;
    if (pre) {
        const uint32_t nd = dirty_blocks(*pre);
        hipLaunchKernelGGL(k_dirty_bounds, dim3(nd + nblk1(nmax, NT)), dim3(NT), 0, s, *pre, nd);
    } else {
        hipLaunchKernelGGL(k_bounds, dim3(nblk1(nmax, NT)), dim3(NT), 0, s, b);
    }
    scan_exclusive<uint64_t, uint64_t>(b.cand, b.reg, nmax, ngm, sc, (uint64_t*)&b.st->cand_total, s,
                                       PrimPost{b.compact && !b.small_ents && !b.pair_max ? b.pidx : nullptr});
}

// ---------------------------------------------------------------------------
// diff: one wave per primary mover-grid entry (mover A).  For every candidate
// B in A's cells the old relation (pre-tick positions and stamps) and the new
// one are evaluated; r_old != r_new is an own event (A,B).  Non-movers come
// from gn (old = new position), movers from the mover grid, where B's entry at
// its old cell stands for the pair when r_old holds and its entry at the new
// cell when only r_new does, so each pair is taken once.  The row ranges of
// both grids are walked flattened (Flat), DIFF_U chunks of 64 candidates with
// their loads in flight together.  Events (B<<1 | leave) go to A's region and
// are sorted there: registers up to 64, LDS up to SORT_LDS, else a block sort
// later.  The count of new neighbours with a client is kept for the collect.

struct Cand {
    float x, z, ox, oz;
    uint32_t slot;
    uint32_t info;       // tags | CAND_CLIENT | CAND_NONMOVER | (GW) gate id & 15 << CAND_GATE
};
constexpr uint32_t CAND_NONMOVER = 1u << 31;
constexpr uint32_t CAND_CLIENT = 1u << 30;
constexpr int CAND_GATE = 24;

// Where a walk reads its candidates: the row starts of both grids (Flat of a
// mover's rectangles) and the entries, in HBM or, in small-space mode, LDS
// copies indexed like HBM.
struct GlobalSrc {
    const GEnt* GN;
    const uint32_t* GS;
    const uint32_t* MS;
    const MEnt* GM;
    __device__ __forceinline__ Flat flat(const SpaceP& P, const Rects& R) const { return flat_build<2>(P, R, GS, MS); }
    __device__ __forceinline__ GEnt gn(uint32_t i) const { return GN[i]; }
    __device__ __forceinline__ MEnt gm(uint32_t i) const { return GM[i]; }
    // entry i of the grid (kind 0) or the mover grid (kind 1) as 16-B words
    __device__ __forceinline__ const uint4* ptr(uint32_t kind, uint32_t i) const {
        return kind ? (const uint4*)(GM + i) : (const uint4*)(GN + i);
    }
};

// The relation of a pair from the two entities' positions and last-AOI-op
// stamps alone: the window of the member with the later op.
__device__ __forceinline__ bool pair_rel(float ax, float az, unsigned long long as, float bx, float bz,
                                         unsigned long long bs, float d) {
    return as > bs ? in_win(ax, az, d, bx, bz) : in_win(bx, bz, d, ax, az);
}

// A long mover's own events with the other long movers (group teleports): the
// lists hold every long mover's state before and after the tick, so the old
// and the new relation of each pair are evaluated here even when no rank holds
// both ends.  Events are appended to A's region before its sort.
// A's entry in the lists of the tick, -1 if not listed (no list queued, or
// its owner's list missing)
__device__ __forceinline__ int32_t long_index(const TickBufs& b, uint32_t A) {
    const uint32_t nl = b.n_long;
    int32_t ia = -1;
    for (uint32_t base = 0; base < nl && ia < 0; base += 64) {
        const uint32_t j = base + (uint32_t)lane_id();
        const uint64_t hit = wave_ballot(j < nl && b.longs[j].slot == A);
        if (hit) ia = (int32_t)(base + (uint32_t)__builtin_ctzll(hit));
    }
    return ia;
}

__device__ __forceinline__ void long_pairs(const TickBufs& b, uint32_t A, int32_t ia, float d, uint32_t* out,
                                        uint64_t cap, uint32_t& n, uint32_t& l_nl) {
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t nl = b.n_long;
    const gw_long_move LA = b.longs[ia];
    for (uint32_t base = 0; base < nl; base += 64) {
        const uint32_t j = base + (uint32_t)ln;
        gw_long_move L;
        L.slot = A;
        if (j < nl) L = b.longs[j];
        bool ev = false, lv = false;
        if (L.slot != A) {
            lv = pair_rel(LA.old_x, LA.old_z, LA.old_stamp, L.old_x, L.old_z, L.old_stamp, d);
            ev = lv != pair_rel(LA.new_x, LA.new_z, LA.new_stamp, L.new_x, L.new_z, L.new_stamp, d);
        }
        const uint64_t be = wave_ballot(ev);
        const uint32_t at = n + (uint32_t)popc64(be & lt);
        if (ev && at < cap) out[at] = (lv ? 0x80000000u : 0u) | L.slot;
        n += (uint32_t)popc64(be);
        l_nl += (ev && lv) ? 1u : 0u;
    }
}

// One mover-grid entry m by one wave, candidates from S; lds: SCAP sort slots
// per wave.
// RR (k_mover): the row ranges k_bounds gathered, loaded with the entry
// itself (the walk then starts one round trip after the wave does).
// LONGS = false: a context without long movers (not a world of >= 2 strips,
// TickBufs::long_step infinite) compiles the group-teleport paths out.
// GW > 0 (2 < G <= 4 * GW gates): the new neighbours with a client are also
// counted per gate (World.nbg), so a multi-gate collect right after the tick
// takes its per-gate record counts from there instead of walking the window
template <int DIFF_U, uint32_t SCAP, class Src, bool RR = false, bool LONGS = true, int GW = 0>
__device__ __forceinline__ void mover_one(const TickBufs& b, uint64_t m, uint32_t* lds, const Src& S) {
    const int ln = lane_id();
    const uint2 rr = (RR && ln < (int)(2 * RR_ROWS)) ? ((const uint2*)b.rowrec)[m * 2 * RR_ROWS + ln]
                                                    : make_uint2(0u, 0u);
    const MEnt me = S.gm(m);
    if (!(me.tags & TAG_PRIMARY)) {
        if (ln == 0) {
            b.mstat[m] = 0;
            b.ownc[m] = 0;
            b.mirc[m] = 0;
        }
        return;
    }
    const uint64_t lt = lanemask_lt();
    const World& w = b.w;
    const uint64_t reg = b.reg[m] & CAND_MASK, cap = b.cand[m] & CAND_MASK;
    if (reg + cap > b.own_cap) {                      // region past the buffers: the host redoes the diff
        if (ln == 0) {
            atomicOr(&b.st->overflow, 1ull);
            b.ownc[m] = 0;
            b.mirc[m] = 0;
            b.mstat[m] = 0;
        }
        return;
    }
    const uint32_t A = me.slot;
    const SpaceP P = w.sp[me.space];
    const float d = P.d;
    const bool pn = me.x == me.x, po = me.ox == me.ox;
    // decomposed world: A's own events only where A is owned (after the tick,
    // before it for a leaver); an op-less B's events only where B is owned
    const bool ownA = owned_x(P, pn ? me.x : me.ox);
    // a long mover's pairs are emitted by the owners of the other members
    // (they hold both ends of every pair that changes)
    const bool longA = LONGS && (me.tags & TAG_LONG) != 0;
    // A's stamps are read only at a boundary tie (rare): loaded up front, the
    // in-order memory counter made every first chunk wait for them too
    Win wo = win_of(me.ox, me.oz, d), wn = win_of(me.x, me.z, d);
    wo.to_vgprs();
    wn.to_vgprs();
    uint32_t* out = b.own + reg;
    uint64_t* mir = b.mir + reg;
    uint32_t n = 0, nm_ = 0;
    // per-lane counts, summed once after the walk (a ballot + popcount per
    // count and chunk was ~10 scalar instructions of every chunk's chain)
    uint32_t l_old = 0, l_new = 0, l_cli = 0, l_nl = 0, l_nml = 0;
    uint32_t l_lc = 0;      // (LONGS) pairs with another long mover related before or after the tick
    // (GW) per-lane counts by gate: 8 bits per gate, gate g in byte g % 8 of
    // l_g[g / 8] (GW VGPRs: 16-bit fields cost k_mover_c a wave of residency;
    // one 64-bit add per candidate); exact while every lane's l_cli <= 255
    // (TickBufs.gate_lane_max), else the split is not published
    constexpr bool GATES = GW > 0;
    unsigned long long l_g[GW > 0 ? GW / 2 : 1] = {};
    Flat f;
    // the row ranges k_bounds gathered (<= RR_ROWS rows x 2 grids: lanes 0..15)
    const bool rr_ok =
        RR && (uint32_t)__builtin_amdgcn_readfirstlane((int)rr.x) <= (uint32_t)__builtin_amdgcn_readfirstlane((int)rr.y);
    if (rr_ok)
        f = flat_from(rr.x, rr.y - rr.x);
    else
        f = S.flat(P, mover_rects(P, po, me.ox, me.oz, pn, me.x, me.z));
    // long ranges (crowded rows): walk the live ranges with readlanes, a chunk
    // overlaps one or two of them; short ones: the shuffle binary search
    const bool walk = f.total >= (uint32_t)popc64(f.live) * b.walk_min;
    for (uint32_t base = 0; base < f.total; base += 64u * DIFF_U) {
        uint32_t idx[DIFF_U], kd[DIFF_U];
        if (walk) flat_map_walk<DIFF_U, 2>(f, base, idx, kd);
        else if (rr_ok) flat_map<DIFF_U, 2, 2 * RR_ROWS>(f, base, idx, kd);
        else flat_map<DIFF_U, 2>(f, base, idx, kd);
        // branch-free candidate loads: every lane reads two 16-B words from its
        // grid's entry (a gn entry twice), lanes past the end read lane 0's, so
        // the loads of all DIFF_U chunks are in flight before the first is used
        // (a divergent gn / gm branch made each chunk wait out its own loads)
        uint4 q0[DIFF_U], q1[DIFF_U];
#pragma unroll
        for (int u = 0; u < DIFF_U; ++u) {
            if (base + 64u * u >= f.total) break;              // wave-uniform
            const uint32_t i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)idx[u]);
            const uint32_t k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)kd[u]);
            const bool valid = idx[u] != ~0u;
            const uint4* p = S.ptr(valid ? kd[u] : k0, valid ? idx[u] : i0);
            q0[u] = p[0];
            q1[u] = p[(valid ? kd[u] : k0) ? 1 : 0];
        }
        Cand cc[DIFF_U];
#pragma unroll
        for (int u = 0; u < DIFF_U; ++u) {
            if (base + 64u * u >= f.total) break;              // wave-uniform
            const bool gm = kd[u] != 0;
            const uint32_t meta = q0[u].w;                     // gn: x z slot meta; gm: x z ox oz | slot tags client space
            cc[u].x = __uint_as_float(q0[u].x);
            cc[u].z = __uint_as_float(q0[u].y);
            cc[u].ox = gm ? __uint_as_float(q0[u].z) : cc[u].x;
            cc[u].oz = gm ? __uint_as_float(q0[u].w) : cc[u].z;
            const uint32_t slot = gm ? q1[u].x : ((meta & b.mbit) ? A : q0[u].z);   // movers come from gm
            const uint32_t info = gm ? (q1[u].y | (q1[u].z ? CAND_CLIENT : 0u))
                                     : (TAG_OLD | TAG_NEW | (meta & CLIENT_BIT ? CAND_CLIENT : 0u) | CAND_NONMOVER);
            const bool valid = idx[u] != ~0u;
            cc[u].slot = valid ? slot : A;                     // invalid: skipped below
            const uint32_t gbits = !GATES ? 0u
                                 : gm   ? (q1[u].z & 15u) << CAND_GATE
                                        : (meta & GATE_MASK) >> (GATE_SHIFT - CAND_GATE);
            cc[u].info = valid ? info | gbits : 0u;
        }
#pragma unroll
        for (int u = 0; u < DIFF_U; ++u) {
            if (base + 64u * u >= f.total) break;              // wave-uniform
            const Cand& e = cc[u];
            // branch-free but for the rounding band (rare): the relation,
            // take / event / count bits as lane values (a branch per test made
            // the compiler keep every bit as an exec mask: scalar ALU work in
            // every chunk)
            // A's tests of B; B's tests of A only in the rounding band (Win::eps)
            bool iao, ian, near_o, near_n;
            wo.test(e.ox, e.oz, iao, near_o);
            wn.test(e.x, e.z, ian, near_n);
            const bool nmv = (e.info & CAND_NONMOVER) != 0;
            bool ro = iao, rn = ian;
            if (near_o | near_n) {
                const bool ibo = in_win(e.ox, e.oz, d, me.ox, me.oz), ibn = in_win(e.x, e.z, d, me.x, me.z);
                if ((iao != ibo) | (ian != ibn)) {
                    const unsigned long long sA = w.rec[A].stamp, soA = w.rec[A].pv.ostamp;
                    const unsigned long long sb = w.rec[e.slot].stamp;
                    const unsigned long long sbo = nmv ? sb : w.rec[e.slot].pv.ostamp;
                    ro = resolve(iao, ibo, soA, sbo);
                    rn = resolve(ian, ibn, sA, sb);
                }
            }
            // the pair is taken at B's old entry when related before, else at its new one
            const bool take = (e.slot != A) & ((((e.info & TAG_OLD) != 0) & ro) |
                                               (((e.info & TAG_NEW) != 0) & rn & !ro));
            const bool t_ro = take & ro, t_rn = take & rn;
            const bool t_cli = t_rn & ((e.info & CAND_CLIENT) != 0);
            bool ev = take & (ro != rn);
            const bool lv = ro;
            const uint32_t key = (lv ? 0x80000000u : 0u) | e.slot;      // own events sort as (leave, target)
            l_old += (uint32_t)t_ro;
            l_new += (uint32_t)t_rn;
            l_cli += (uint32_t)t_cli;
            if (GATES) {
                // bits CAND_GATE - 3 .. CAND_GATE - 1 of info are clear: this
                // is 8 * (gate % 8), the gate's byte in its word
                const uint32_t sh = (e.info >> (CAND_GATE - 3)) & 0x38u;
                const unsigned long long inc = (unsigned long long)(t_cli ? 1u : 0u) << sh;
                if (GW == 2) {
                    l_g[0] += inc;
                } else {
                    const bool hi = ((e.info >> (CAND_GATE + 3)) & 1u) != 0;   // gates 8..15
                    l_g[0] += hi ? 0ull : inc;
                    l_g[GW / 2 - 1] += hi ? inc : 0ull;
                }
            }
            // B has no op: (B,A) is B's event too (kept in A's region; the
            // events stage places it)
            const bool mev = ev & nmv & owned_x(P, e.x);
            // a long mover's pairs: with a short mover B by B's owner (it holds
            // both ends); with another long mover from the long lists (below)
            const bool longB = (e.info & TAG_LONG) != 0;
            ev = ev && (longA ? !longB && owned_x(P, e.x == e.x ? e.x : e.ox) : ownA);
            const uint64_t be = wave_ballot(ev), bm = wave_ballot(mev);
            const uint32_t at = n + (uint32_t)popc64(be & lt);
            if (ev && at < cap) out[at] = key;
            const uint32_t atm = nm_ + (uint32_t)popc64(bm & lt);
            if (mev && atm < cap) mir[atm] = ((uint64_t)e.slot << 32) | (A << 1) | (lv ? 1u : 0u);
            n += (uint32_t)popc64(be);
            nm_ += (uint32_t)popc64(bm);
            l_nl += (ev && lv) ? 1u : 0u;
            l_nml += (mev && lv) ? 1u : 0u;
            if (LONGS) l_lc += (longA && longB && (t_ro || t_rn)) ? 1u : 0u;
        }
    }
    // group teleports: A is a long mover whose new position is owned here (not
    // its old owner, where it left); its pairs with the other long movers come
    // from the lists of every rank
    // If the lists do not cover A (a caller's transport skipped
    // gw_world_submit_longs, or a rank's list is missing), nobody emits those
    // pairs: the related ones are counted into HaloStats.conflicts, which
    // gw_world_status reports
    if (longA && pn && owned_x(P, me.x)) {
        const int32_t ia = long_index(b, A);
        if (ia >= 0) {
            long_pairs(b, A, ia, d, out, cap, n, l_nl);
        } else if (b.conflicts) {
            const uint32_t lc = wave_incl_scan<uint32_t>(l_lc);
            const uint32_t nlc = (uint32_t)__builtin_amdgcn_readlane((int)lc, 63);
            if (ln == 0 && nlc) atomicAdd(b.conflicts, (unsigned long long)nlc);
        }
    }
    // the wave's sums (DPP scans, lane 63): old | new, client | own leaves, mirror leaves
    const unsigned long long s_on = wave_incl_scan<unsigned long long>(l_old | ((unsigned long long)l_new << 32));
    const unsigned long long s_cl = wave_incl_scan<unsigned long long>(l_cli | ((unsigned long long)l_nl << 32));
    const uint32_t s_ml = wave_incl_scan<uint32_t>(l_nml);
    const uint32_t c_old = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s_on, 63);
    const uint32_t c_new = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s_on >> 32), 63);
    const uint32_t c_cli = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s_cl, 63);
    const uint32_t nl = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s_cl >> 32), 63);
    const uint32_t nml = (uint32_t)__builtin_amdgcn_readlane((int)s_ml, 63);
    // sort the own events by (target, kind)
    if (n > 1) {
        if (n <= b.rank_sort) {                    // a few events: place each by its rank
            wave_sync();
            const uint32_t v = ln < (int)n ? out[ln] : 0xffffffffu;
            uint32_t r = 0;
            for (uint32_t j = 0; j < n; ++j) r += (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j) < v ? 1u : 0u;
            wave_sync();
            if (ln < (int)n) out[r] = v;
        } else if (n <= 64) {
            wave_sync();
            uint32_t v = ln < (int)n ? out[ln] : 0xffffffffu;
            v = wave_sort64(v);
            if (ln < (int)n) out[ln] = v;
        } else if (n <= SCAP) {
            uint32_t* L = lds + (threadIdx.x >> 6) * SCAP;
            wave_sync();
            for (uint32_t i = ln; i < n; i += 64) L[i] = out[i];
            wave_sync();
            bitonic_inplace<64>(L, n, ln, [](uint32_t v) { return v; }, [] { wave_sync(); });
            for (uint32_t i = ln; i < n; i += 64) out[i] = L[i];
        } else if (ln == 0) {
            b.big[atomicAdd(&b.st->n_big, 1ull)] = (uint32_t)m;
        }
    }
    const uint32_t so = c_old, sn = c_new, scl = c_cli;
    // (GATES) the split is exact when no lane's byte can have wrapped
    const bool g_ok = GATES && pn && !wave_ballot(l_cli > b.gate_lane_max);
    if (g_ok) {
        // the wave's per-gate sums in 16-bit fields (<= 64 x 255): bytes 0, 2
        // and 1, 3 of each word summed apart, then laid out as World.nbg
        unsigned long long v = 0;
#pragma unroll
        for (int j = 0; j < GW; ++j) {
            const uint32_t lw = (uint32_t)(l_g[j >> 1] >> (32 * (j & 1)));               // gates 4j .. 4j+3
            const uint32_t se = wave_incl_scan<uint32_t>(lw & 0x00ff00ffu);              // gates 4j, 4j+2
            const uint32_t so_ = wave_incl_scan<uint32_t>((lw >> 8) & 0x00ff00ffu);      // gates 4j+1, 4j+3
            const uint32_t te = (uint32_t)__builtin_amdgcn_readlane((int)se, 63);
            const uint32_t to = (uint32_t)__builtin_amdgcn_readlane((int)so_, 63);
            const unsigned long long t = (unsigned long long)(te & 0xffffu) | ((unsigned long long)(to & 0xffffu) << 16) |
                                         ((unsigned long long)(te >> 16) << 32) | ((unsigned long long)(to >> 16) << 48);
            if (ln == j) v = t;
        }
        if (ln < 4) w.nbg[(uint64_t)A * 4 + ln] = v;
    }
    if (ln == 0) {
        b.ownc[m] = (unsigned long long)(n - nl) | ((unsigned long long)nl << 32);
        b.mirc[m] = (unsigned long long)(nm_ - nml) | ((unsigned long long)nml << 32);
        if (n | nm_) {                                     // listed for the events stage (slot order)
            atomicOr(&b.movbit[A >> 5], 1u << (A & 31u));
            b.gmi[A] = (uint32_t)m;
        }
        if (pn) w.nbc[A] = ((unsigned long long)w.epoch << 32) | scl | (g_ok ? NBC_GATES : 0u);
        // per-mover statistics, summed by k_mover_post (no atomics here: 2 per
        // mover into 256 shards cost 25 us at config #3 and 180 us at config #4)
        b.mstat[m] = (unsigned long long)so | ((unsigned long long)sn << 32);
    }
}

// WPB waves per block: a block keeps its LDS until its slowest wave ends, so
// small blocks keep more waves resident when hotspot movers run long
// SGPRs decide k_mover's residency: a SIMD holds floor(800 / (ceil(sgpr/16)*16 + 16))
// waves (MI355X_MICROARCH.md): 106 SGPRs -> 6 waves, <= 80 -> 8 (34 spilled to
// VGPR lanes; config #3 diff 180 -> 172 us).  GW_KMOVER_SGPR=0: no cap
#ifndef GW_KMOVER_SGPR
#define GW_KMOVER_SGPR 80
#endif
#if GW_KMOVER_SGPR
#define KMOVER_SGPR __attribute__((amdgpu_num_sgpr(GW_KMOVER_SGPR)))
#else
#define KMOVER_SGPR
#endif
// 8 waves per SIMD also with the split by gate (GW = 2: 65 VGPRs uncapped, 7
// waves; capped, no spill)
#define KMOVER_OCC __attribute__((amdgpu_waves_per_eu(8, 8)))
// one wave per primary entry (pidx, cell order): no wave is dispatched for
// the secondary entries (half the mover grid), whose zeros k_bounds wrote
template <int DIFF_U, bool LONGS, int GW>
__global__ void __launch_bounds__(64) KMOVER_SGPR KMOVER_OCC k_mover_c(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[SORT_LDS];
    const uint64_t k = blockIdx.x;
    const uint64_t np = b.st->cand_total >> PRIM_SHIFT;
    uint32_t m;
    if (b.heavy_min) {                            // heavy entries first, then the others in cell order
        const uint64_t nh = b.st->n_heavy;
        if (k >= nh + np) return;
        m = k < nh ? b.heavy[k] : b.pidx[k - nh];
    } else {
        m = b.pidx[k];                            // in bounds (k < ops), read with the count
        if (k >= np) return;
    }
    mover_one<DIFF_U, SORT_LDS, GlobalSrc, true, LONGS, GW>(b, m, lds,
                                                               GlobalSrc{b.w.gn, b.w.gn_start, b.gm_start, b.gm});
}

template <int DIFF_U, int WPB>
__global__ void __launch_bounds__(64 * WPB) k_mover(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[WPB * SORT_LDS];
    const uint64_t m = (uint64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    if (m >= b.st->n_gm) return;
    mover_one<DIFF_U, SORT_LDS, GlobalSrc, true>(b, m, lds, GlobalSrc{b.w.gn, b.w.gn_start, b.gm_start, b.gm});
}

// Two mover-grid entries per wave (a half-wave each), small-space mode: with
// ~80 candidates per mover the per-mover setup dominates a wave's VALU.  A
// half holds <= 16 row ranges x 2 grids; the row scan is the wave scan minus
// lane 31's prefix for the upper half; a lane finds its range by a 5-step
// search over its half's prefixes; ballots are masked per half; own events
// (<= 32) are sorted inside the half in registers, more go to the block sort.
// GM: the mover-grid entries (LDS when the block staged them); L: this wave's
// 64 LDS words, the first 32 own events of each half (sorted from there, no
// read-back of HBM).  Returns false (nothing done) when either entry needs
// more rows: the caller then runs both through mover_one.
// RC (k_mover_small with its space's entries staged): region offset | bound
// << 32 of entry m at RC[m - rc0], read from LDS instead of HBM
template <int HU>
__device__ __forceinline__ bool mover_half(const TickBufs& b, uint64_t m0, uint64_t m_end, const SpaceP& P,
                                           const GEnt* GN, const uint32_t* GS, const uint32_t* MS,
                                           const MEnt* GM, uint32_t* L, const uint2* RC = nullptr,
                                           uint32_t rc0 = 0) {
    const int ln = lane_id();
    const uint32_t half = (uint32_t)ln >> 5, hl = (uint32_t)ln & 31u, hb = half << 5;
    const uint64_t hmask = half ? 0xffffffff00000000ull : 0x00000000ffffffffull;
    const uint64_t lt = lanemask_lt();
    const uint64_t m = m0 + half;
    const bool valid = m < m_end;
    MEnt me;
    me.tags = 0;
    me.x = me.z = me.ox = me.oz = qnan();
    me.slot = 0; me.client = 0; me.space = 0;
    if (valid) me = GM[m];
    const bool prim = valid && (me.tags & TAG_PRIMARY);
    const bool pn = me.x == me.x, po = me.ox == me.ox;
    Rects R;
    R.n = 0;
    if (prim) R = mover_rects(P, po, me.ox, me.oz, pn, me.x, me.z);
    // (no loop over R.r[q]: a dynamically indexed Rects lives in scratch)
    const int nr0 = R.n > 0 ? R.r[0].z1 - R.r[0].z0 + 1 : 0;
    const int nr1 = R.n > 1 ? R.r[1].z1 - R.r[1].z0 + 1 : 0;
    if (wave_ballot(nr0 + nr1 > (int)b.half_rows)) return false;   // wave-uniform (<= 16 rows: one half's lanes)
    const World& w = b.w;
    // the HBM reads of this pair (region) are first needed at the first
    // write: the row ranges and candidates (LDS) go first; stamps only at a
    // boundary tie
    uint64_t reg = 0, cap = 0;
    const bool go = prim;
    const uint32_t A = me.slot;
    if (prim) {
        if (RC) {
            const uint2 rc = RC[m - rc0];
            reg = rc.x;
            cap = rc.y;
        } else {
            reg = b.reg[m] & CAND_MASK;
            cap = b.cand[m] & CAND_MASK;
        }
    }
    const uint64_t own_cap = b.own_cap;
    const float d = P.d;
    const bool ownA = owned_x(P, pn ? me.x : me.ox);
    const bool longA = (me.tags & TAG_LONG) != 0;           // (see mover_one)
    const Win wo = win_of(me.ox, me.oz, d), wn = win_of(me.x, me.z, d);
    // this half's row ranges: lane hl = row hl/2 of the rects, grid hl%2
    uint32_t rs = 0, rl = 0;
    if (go) {
        const int row = (int)(hl >> 1), kind = (int)(hl & 1u);
        if (row < nr0 + nr1) {
            const bool first = row < nr0;
            const int x0 = first ? R.r[0].x0 : R.r[1].x0;
            const int x1 = first ? R.r[0].x1 : R.r[1].x1;
            const int cz = first ? R.r[0].z0 + row : R.r[1].z0 + (row - nr0);
            const uint32_t base = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
            const uint32_t* st = kind ? MS : GS;
            rs = st[base + x0];
            rl = st[base + x1 + 1] - rs;
        }
    }
    const uint32_t inc64 = wave_incl_scan<uint32_t>(rl);
    const uint32_t lo31 = (uint32_t)__builtin_amdgcn_readlane((int)inc64, 31);
    const uint32_t inc = half ? inc64 - lo31 : inc64;
    const uint32_t pre = inc - rl;
    const uint32_t tot0 = lo31, tot1 = (uint32_t)__builtin_amdgcn_readlane((int)inc64, 63) - lo31;
    const uint32_t total = half ? tot1 : tot0;
    const uint32_t tmax = max(tot0, tot1);
    uint32_t* out = b.own + reg;
    uint64_t* mir = b.mir + reg;
    uint32_t n = 0, nl = 0, nm_ = 0, nml = 0;
    uint32_t c_old = 0, c_new = 0, c_cli = 0;
    uint64_t l_on = 0, l_cl = 0;      // per lane: old | new << 32, client | own leaves << 32
    uint32_t l_ml = 0;                // per lane: mirror leaves
    // the half's first candidate (its first non-empty range): what a lane past
    // the half's end reads
    const uint32_t f_lane = (uint32_t)__builtin_ctzll((wave_ballot(rl != 0) & hmask) | (1ull << 63));
    const uint32_t f_idx = (uint32_t)__shfl((int)rs, (int)f_lane, 64);
    const uint32_t f_kind = f_lane & 1u;
    for (uint32_t base = 0; base < tmax; base += 32u * HU) {   // wave-uniform
        // candidate loads without a divergent gn / gm branch (see mover_one):
        // a lane past its half's end reads its half's first candidate
        uint4 q0[HU], q1[HU];
        uint32_t kind[HU];
        bool in[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            in[u] = false;
            kind[u] = 0;
            if (base + 32u * u >= tmax) continue;            // wave-uniform
            const uint32_t kk = base + 32u * u + hl;
            uint32_t l2 = 0;
#pragma unroll
            for (int step = 16; step; step >>= 1) {
                const uint32_t c2 = l2 + (uint32_t)step;
                const uint32_t pv = (uint32_t)__shfl((int)pre, (int)(hb + min(c2, 31u)), 64);
                if (c2 < 32u && pv <= kk) l2 = c2;
            }
            const uint32_t ss = (uint32_t)__shfl((int)rs, (int)(hb + l2), 64);
            const uint32_t sp = (uint32_t)__shfl((int)pre, (int)(hb + l2), 64);
            in[u] = kk < total;
            const bool use = in[u];
            kind[u] = use ? (l2 & 1u) : f_kind;
            const uint32_t idx = use ? ss + (kk - sp) : f_idx;
            const uint4* p = kind[u] ? (const uint4*)(GM + idx) : (const uint4*)(GN + idx);
            const bool any = total != 0;                       // a half with no candidates reads nothing
            q0[u] = any ? p[0] : make_uint4(0u, 0u, 0u, 0u);
            q1[u] = any ? p[kind[u]] : make_uint4(0u, 0u, 0u, 0u);
        }
        Cand cc[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            cc[u].info = 0;
            cc[u].slot = A;
            if (base + 32u * u >= tmax) continue;            // wave-uniform
            const bool gmk = kind[u] != 0;
            const uint32_t meta = q0[u].w;
            cc[u].x = __uint_as_float(q0[u].x);
            cc[u].z = __uint_as_float(q0[u].y);
            cc[u].ox = gmk ? __uint_as_float(q0[u].z) : cc[u].x;
            cc[u].oz = gmk ? __uint_as_float(q0[u].w) : cc[u].z;
            const uint32_t slot = gmk ? q1[u].x : ((meta & b.mbit) ? A : q0[u].z);
            const uint32_t info = gmk ? (q1[u].y | (q1[u].z ? CAND_CLIENT : 0u))
                                      : (TAG_OLD | TAG_NEW | (meta & CLIENT_BIT ? CAND_CLIENT : 0u) | CAND_NONMOVER);
            cc[u].slot = in[u] ? slot : A;
            cc[u].info = in[u] ? info : 0u;
        }
#pragma unroll
        for (int u = 0; u < HU; ++u) {
            if (base + 32u * u >= tmax) break;               // wave-uniform
            const Cand& e = cc[u];
            // as mover_one: branch-free but for the rounding band (Win::eps),
            // counts per lane, summed per half after the walk
            bool iao, ian, near_o, near_n;
            wo.test(e.ox, e.oz, iao, near_o);
            wn.test(e.x, e.z, ian, near_n);
            const bool nmv = (e.info & CAND_NONMOVER) != 0;
            bool ro = iao, rn = ian;
            if (near_o | near_n) {
                const bool ibo = in_win(e.ox, e.oz, d, me.ox, me.oz), ibn = in_win(e.x, e.z, d, me.x, me.z);
                if ((iao != ibo) | (ian != ibn)) {
                    const unsigned long long sA = w.rec[A].stamp, soA = w.rec[A].pv.ostamp;
                    const unsigned long long sb = w.rec[e.slot].stamp;
                    const unsigned long long sbo = nmv ? sb : w.rec[e.slot].pv.ostamp;
                    ro = resolve(iao, ibo, soA, sbo);
                    rn = resolve(ian, ibn, sA, sb);
                }
            }
            const bool take = go & (e.slot != A) & ((((e.info & TAG_OLD) != 0) & ro) |
                                                    (((e.info & TAG_NEW) != 0) & rn & !ro));
            const bool t_ro = take & ro, t_rn = take & rn;
            const bool t_cli = t_rn & ((e.info & CAND_CLIENT) != 0);
            bool ev = take & (ro != rn);
            const bool lv = ro;
            const uint32_t key = (lv ? 0x80000000u : 0u) | e.slot;
            l_on += (uint64_t)t_ro | ((uint64_t)t_rn << 32);
            const bool mev = ev & nmv & owned_x(P, e.x);
            const bool longB = (e.info & TAG_LONG) != 0;
            // (long movers never come here: k_mover_pair runs them through mover_one)
            ev = ev && (longA ? !longB && owned_x(P, e.x == e.x ? e.x : e.ox) : ownA);
            l_cl += (uint64_t)t_cli | ((uint64_t)(ev & lv) << 32);
            l_ml += (uint32_t)(mev & lv);
            const uint64_t be = wave_ballot(ev) & hmask;
            const uint64_t bm = wave_ballot(mev) & hmask;
            const uint32_t at = n + (uint32_t)popc64(be & lt);
            if (ev && at < 32u) L[hb + at] = key;
            else if (ev && at < cap && reg + cap <= own_cap) out[at] = key;
            const uint32_t atm = nm_ + (uint32_t)popc64(bm & lt);
            if (mev && atm < cap && reg + cap <= own_cap) mir[atm] = ((uint64_t)e.slot << 32) | (A << 1) | (lv ? 1u : 0u);
            n += (uint32_t)popc64(be);
            nm_ += (uint32_t)popc64(bm);
        }
    }
    // the halves' sums of the per-lane counts: lane 31 (half 0), lane 63 - lane 31 (half 1)
    {
        const uint64_t s_on = wave_incl_scan<unsigned long long>(l_on);
        const uint64_t s_cl = wave_incl_scan<unsigned long long>(l_cl);
        const uint32_t s_ml = wave_incl_scan<uint32_t>(l_ml);
        auto half_sum64 = [&](uint64_t v) {
            const uint64_t lo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), 31) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 31);
            const uint64_t hi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), 63) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
            return half ? hi - lo : lo;
        };
        const uint64_t on = half_sum64(s_on), cl = half_sum64(s_cl);
        const uint32_t ml_lo = (uint32_t)__builtin_amdgcn_readlane((int)s_ml, 31);
        const uint32_t ml_hi = (uint32_t)__builtin_amdgcn_readlane((int)s_ml, 63);
        c_old = (uint32_t)on;
        c_new = (uint32_t)(on >> 32);
        c_cli = (uint32_t)cl;
        nl = (uint32_t)(cl >> 32);
        nml = half ? ml_hi - ml_lo : ml_lo;
    }
    // own events by (leave, target): <= 32 in registers inside the half, more
    // by the block sort (the first 32 written out of L unsorted)
    wave_sync();
    const bool ovf = prim && reg + cap > own_cap;           // region past the buffers: the host redoes the diff
    if (ovf && hl == 0) atomicOr(&b.st->overflow, 1ull);
    const bool fin = prim && !ovf;
    const uint32_t nw = fin ? (uint32_t)min((uint64_t)n, cap) : 0u;   // keys to place (n <= cap but for a bug)
    const bool reg_sort = nw > 1 && n <= 32;
    uint32_t v = hl < nw ? L[hb + hl] : 0xffffffffu;
    if (hl < nw && !reg_sort) out[hl] = v;
    if (wave_ballot(reg_sort)) {
        const uint32_t n2 = reg_sort ? n : 0u;
        const uint32_t nmax = max((uint32_t)__builtin_amdgcn_readlane((int)n2, 0),
                                  (uint32_t)__builtin_amdgcn_readlane((int)n2, 32));
        if (nmax <= b.rank_sort) {                  // a few events per half: place each by its rank
            uint32_t r = 0;
            for (uint32_t j = 0; j < nmax; ++j) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)v, 32 + (int)j);
                r += (half ? hi : lo) < v ? 1u : 0u;
            }
            if (reg_sort && hl < n) out[r] = v;
        } else {
            v = half_sort32(v);
            if (reg_sort && hl < n) out[hl] = v;
        }
    }
    if (fin && n > 32 && hl == 0) b.big[atomicAdd(&b.st->n_big, 1ull)] = (uint32_t)m;
    if (valid && hl == 0) {
        if (!fin) {
            b.mstat[m] = 0;
            b.ownc[m] = 0;
            b.mirc[m] = 0;
        } else {
            b.ownc[m] = (unsigned long long)(n - nl) | ((unsigned long long)nl << 32);
            b.mirc[m] = (unsigned long long)(nm_ - nml) | ((unsigned long long)nml << 32);
            if (n | nm_) {
                atomicOr(&b.movbit[A >> 5], 1u << (A & 31u));
                b.gmi[A] = (uint32_t)m;
            }
            if (pn) w.nbc[A] = ((unsigned long long)w.epoch << 32) | c_cli;
            b.mstat[m] = (unsigned long long)c_old | ((unsigned long long)c_new << 32);
        }
    }
    return true;
}

// General mode, two mover-grid entries per wave: a short candidate list
// (config #3's uniform background, config #5: ~50 candidates) pays the
// per-mover setup (rects, row ranges, scan, sort, writes) for half a wave;
// a pair with a longer list (hotspots: own events sorted in LDS, not by the
// half-wave register sort) or more rows than a half holds, or two spaces, runs
// both entries through mover_one, one after the other.
template <int DIFF_U>
__global__ void __launch_bounds__(64) k_mover_pair(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[SORT_LDS];
    const uint64_t m0 = (uint64_t)blockIdx.x * 2;
    const uint64_t ngm = b.st->n_gm;
    if (m0 >= ngm) return;
    const uint64_t m1 = min(m0 + 2, ngm);
    const GlobalSrc src{b.w.gn, b.w.gn_start, b.gm_start, b.gm};
    const uint64_t c0 = b.cand[m0] & CAND_MASK, c1 = m0 + 1 < m1 ? b.cand[m0 + 1] & CAND_MASK : 0;
    const uint32_t s0 = b.gm[m0].space, s1 = m0 + 1 < m1 ? b.gm[m0 + 1].space : s0;
    const uint32_t tg = b.gm[m0].tags | (m0 + 1 < m1 ? b.gm[m0 + 1].tags : 0u);
    if (max(c0, c1) <= b.pair_max && s0 == s1 && !(tg & TAG_LONG)) {   // wave-uniform; long movers: mover_one
        if (mover_half<2>(b, m0, m1, b.w.sp[s0], src.GN, src.GS, src.MS, src.GM, lds)) return;
    }
    mover_one<DIFF_U, SORT_LDS>(b, m0, lds, src);
    wave_sync();
    if (m0 + 1 < m1) mover_one<DIFF_U, SORT_LDS>(b, m0 + 1, lds, src);
}

// Small-space mode (every space's grid fits in LDS: config #4's 10k spaces of
// 1k): one block per space copies the space's grid entries and the row
// starts of both grids into LDS, then its waves walk the space's mover-grid
// entries with every grid candidate and row start read from LDS (mover-grid
// candidates, ~10 % of them, stay global).
constexpr uint32_t SMALL_SORT = 256;    // own events sorted in LDS up to this many (more: block sort)
constexpr uint32_t SMALL_GM = 256;      // mover-grid entries of a space staged in LDS (more: read from HBM)
// half-wave mode: a wave's own-event words (2 halves x 32), then (from word
// NWAVE * SMALL_HL of the sort space) the staged entries' regions and bounds
constexpr uint32_t SMALL_HL = 64;
static_assert(NWAVE * SMALL_HL + 2 * SMALL_GM <= NWAVE * SMALL_SORT, "staged regions fit the sort space");

template <int DIFF_U, bool HALVES>
__device__ __forceinline__ void small_walk(const TickBufs& b, uint32_t m0, uint32_t m1, const SpaceP& P,
                                           const GlobalSrc& src, uint32_t* lds, const uint2* RC = nullptr) {
    if (HALVES) {
        // a pair the half-wave walk cannot take (a window of more rows than a
        // half holds) goes to k_mover_list, one wave per entry from the global
        // grids: with no mover_one inlined here the kernel fits 96 VGPRs, 5
        // waves per SIMD instead of 4 (128 VGPRs)
        uint32_t* L = lds + (threadIdx.x >> 6) * SMALL_HL;
        for (uint32_t m = m0 + (threadIdx.x >> 6) * 2; m < m1; m += NWAVE * 2) {
            if (!mover_half<2>(b, m, m1, P, src.GN, src.GS, src.MS, src.GM, L, RC, m0) && lane_id() == 0) {
                const uint32_t k = m + 1 < m1 ? 2u : 1u;
                const uint32_t at = (uint32_t)atomicAdd(&b.st->n_fall, (unsigned long long)k);
                b.fall[at] = m;
                if (k == 2) b.fall[at + 1] = m + 1;
            }
            wave_sync();
        }
        return;
    }
    for (uint32_t m = m0 + (threadIdx.x >> 6); m < m1; m += NWAVE) {
        mover_one<DIFF_U, SMALL_SORT>(b, m, lds, src);
        wave_sync();
    }
}

// (GW_MS_MINB: blocks per CU the register allocation must allow; 4 caps the
// VGPRs at 128: 4 waves per SIMD instead of 3 at 129, as LDS allows 5 blocks;
// config #4 diff 854 -> 711 us.  The half-wave kernel without mover_one fits
// 96 at 5.)
#ifndef GW_MS_MINB
#define GW_MS_MINB 4
#endif
#ifndef GW_MSH_MINB
#define GW_MSH_MINB 5
#endif
template <int DIFF_U, bool HALVES>
__global__ void __launch_bounds__(NT, HALVES ? GW_MSH_MINB : GW_MS_MINB) k_mover_small(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[NWAVE * SMALL_SORT];
    extern __shared__ uint4 dyn_lds[];
    const uint32_t s = blockIdx.x;
    const SpaceP P = b.w.sp[s];
    const uint32_t cb = P.cell_base, nc = (uint32_t)(P.W * P.H);
    const uint32_t m0 = b.gm_start[cb], m1 = b.gm_start[cb + nc];
    if (m0 >= m1) return;                                   // block-uniform: no movers here
    const uint32_t g0 = b.w.gn_start[cb], g1 = b.w.gn_start[cb + nc];
    GEnt* G = (GEnt*)dyn_lds;
    uint32_t* S = (uint32_t*)(G + b.small_ents);
    uint32_t* MS = S + nc + 1;
    MEnt* GL = (MEnt*)(dyn_lds + (b.small_ents + (2 * ((size_t)b.small_cells + 1) + 3) / 4));
    const uint32_t ng = min(g1 - g0, b.small_ents);        // (host guarantee: g1 - g0 <= small_ents)
    const bool stage = m1 - m0 <= SMALL_GM;                 // block-uniform
    lds_fill16<NT>((uint4*)G, (const uint4*)(b.w.gn + g0), ng);
    for (uint32_t i = threadIdx.x; i <= nc; i += NT) {
        S[i] = b.w.gn_start[cb + i];
        MS[i] = b.gm_start[cb + i];
    }
    // half-wave mode: the entries' regions and bounds too (no HBM read in the
    // walk loop but the rare boundary-tie stamps: the pairs' event stores are
    // not drained by the next pair's region loads), while offsets fit 32 bits
    uint2* RC = (HALVES && stage && b.own_cap <= 0xffffffffull) ? (uint2*)(lds + NWAVE * SMALL_HL) : nullptr;
    if (stage)
        for (uint32_t i = threadIdx.x; i < m1 - m0; i += NT) {
            GL[i] = b.gm[m0 + i];
            if (RC) RC[i] = make_uint2((uint32_t)(b.reg[m0 + i] & CAND_MASK), (uint32_t)(b.cand[m0 + i] & CAND_MASK));
        }
    __syncthreads();
    // every mover's own entry and its mover-grid candidates from LDS when staged
    if (stage) small_walk<DIFF_U, HALVES>(b, m0, m1, P, GlobalSrc{G - g0, S - cb, MS - cb, GL - m0}, lds, RC);
    else small_walk<DIFF_U, HALVES>(b, m0, m1, P, GlobalSrc{G - g0, S - cb, MS - cb, b.gm}, lds);
}

// the entries k_mover_small's half-wave walk left (fall[], n_fall on the
// device): one wave each, candidates from the global grids
template <int DIFF_U>
__global__ void __launch_bounds__(64) k_mover_list(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[SORT_LDS];
    const uint64_t nf = b.st->n_fall;
    for (uint64_t k = blockIdx.x; k < nf; k += gridDim.x) {
        mover_one<DIFF_U, SORT_LDS>(b, b.fall[k], lds, GlobalSrc{b.w.gn, b.w.gn_start, b.gm_start, b.gm});
        wave_sync();
    }
}

// A_old | A_new << 32 of every mover-grid entry, one shard per
// block (STAT_SHARDS blocks, so no two blocks add to the same words)
// Blocks [0, STAT_SHARDS) sum the statistics; the others block-sort the own
// events of movers with too many for LDS (k_mover listed them in big[]): one
// launch for both small jobs.
// (role index r < STAT_SHARDS: a shard of the sums; above: the block sorts)
__device__ __forceinline__ void mover_post(const TickBufs& b, uint32_t r, uint32_t nr) {
    if (r >= (uint32_t)STAT_SHARDS) {                       // block-uniform role
        const uint64_t nb = b.st->n_big;
        for (uint64_t k = r - STAT_SHARDS; k < nb; k += nr - STAT_SHARDS) {
            const uint32_t m = b.big[k];
            const uint64_t c = b.ownc[m];
            const uint32_t n = (uint32_t)(lo32(c) + hi32(c));
            bitonic_inplace<NT>(b.own + (b.reg[m] & CAND_MASK), n, (int)threadIdx.x, [](uint32_t v) { return v; },
                                [] { __syncthreads(); });
            __syncthreads();
        }
        return;
    }
    // A_old | A_new << 32 into this block's shard; the tick's enters | leaves
    // << 32 (own + mirror events of every entry) into ev_pk, one add per block
    __shared__ unsigned long long red[2][NWAVE];
    const uint64_t n = b.st->n_gm;
    unsigned long long a = 0, e = 0;
    for (uint64_t m = (uint64_t)r * NT + threadIdx.x; m < n; m += (uint64_t)STAT_SHARDS * NT) {
        a += b.mstat[m];
        e += b.ownc[m] + b.mirc[m];
    }
    a = wave_sum<unsigned long long>(a);
    e = wave_sum<unsigned long long>(e);
    if (lane_id() == 0) { red[0][threadIdx.x >> 6] = a; red[1][threadIdx.x >> 6] = e; }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = e = 0;
        for (int i = 0; i < NWAVE; ++i) { a += red[0][i]; e += red[1][i]; }
        shard_add(b.st, r, SH_AOLD, a);
        if (e) atomicAdd(&b.st->ev_pk, e);
    }
}
__global__ void __launch_bounds__(NT) k_mover_post(TickBufs b) { mover_post(b, blockIdx.x, gridDim.x); }


// ---------------------------------------------------------------------------
// events stage.  (1) movers with events in slot order: compaction of the
// mover bitmap (one 32-slot word per thread, striped tiles, decoupled
// look-back; words are cleared as they are read).
// Blocks [nt, gridDim) do k_mover_post's work (the statistics sums and the
// block sorts; neither waits on anything), so the two small jobs share one
// launch; the tiles take tickets among themselves only.
template <int IPT>
__global__ void __launch_bounds__(NT) k_bits_list(uint32_t* __restrict__ bits, uint64_t nwords,
                                                  uint32_t* __restrict__ list, unsigned long long* __restrict__ status,
                                                  unsigned long long* __restrict__ ticket, unsigned long long tbase,
                                                  uint32_t tag, unsigned long long* total, TickBufs pb, uint32_t nt) {
    if (blockIdx.x >= nt) {                                 // block-uniform role
        mover_post(pb, blockIdx.x - nt, gridDim.x - nt);
        return;
    }
    __shared__ uint32_t lds[IPT * NWAVE];
    __shared__ uint32_t s_tile, s_prefix;
    if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tbase);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t t0 = (uint64_t)tile * (IPT * NT);
    uint32_t wv[IPT], c[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        wv[j] = i < nwords ? bits[i] : 0u;
        c[j] = (uint32_t)__popc(wv[j]);
    }
    uint32_t tot;
    tile_excl_scan_striped<uint32_t, IPT>(c, lds, tot);
    if (threadIdx.x < 64) {
        const uint32_t excl = scan_lookback<uint32_t>(status, tile, tag, tot);
        if (threadIdx.x == 0) s_prefix = excl;
    }
    __syncthreads();
    const uint32_t pre = s_prefix;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (!wv[j]) continue;
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        uint32_t v = wv[j], at = pre + c[j];
        while (v) {
            const uint32_t bit = (uint32_t)__builtin_ctz(v);
            v &= v - 1;
            list[at++] = (uint32_t)(i * 32 + bit);
        }
        bits[i] = 0;
    }
    if (tile == nt - 1 && threadIdx.x == 0) *total = pre + tot;
}

// (2) per listed mover: all its events (own + mirror), packed enters | leaves<<32,
// and what the flatten needs of it in one 16-B record + its region offset
__global__ void __launch_bounds__(NT) k_mover_counts(TickBufs b) {
    const uint64_t k = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (k >= b.st->n_mlist) return;
    const uint32_t A = b.mlist[k];
    const uint32_t m = b.gmi[A];
    const uint64_t oc = b.ownc[m], mc = b.mirc[m];
    b.mcnt[k] = oc + mc;
    const uint32_t nm = (uint32_t)(lo32(mc) + hi32(mc));
    b.minfo[k] = make_uint4(A, (uint32_t)lo32(oc), (uint32_t)hi32(oc), nm);
    b.mreg[k] = b.reg[m] & CAND_MASK;
    // bucket path: items = one per nonempty own run (enters, leaves) + one per mirror event
    b.icnt[k] = (lo32(oc) ? 1u : 0u) + (hi32(oc) ? 1u : 0u) + nm;
}
// bucket path: the event totals (the general path takes them from the scan of mcnt)

// (3) the listed movers' events flattened at their scanned offsets, in list
// (slot) order: own events (watcher A, target-sorted), then the mirror events
// (watcher W, target A).  Keys carry the leave bit above the slot bits.  One
// wave per 64 output positions (every wave independent): chunk_first[c] is
// the mover whose events hold position 64c; lane i loads mover first + i, and
// lane p finds its mover by a binary search over those movers' ends (7
// shuffles), so loads and stores are runs of consecutive addresses whatever
// the per-mover counts.
__global__ void __launch_bounds__(NT) k_chunk_first(TickBufs b) {
    const uint64_t k = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (k >= b.st->n_mlist) return;
    if (lo32(b.st->ev_pk) + hi32(b.st->ev_pk) > b.ev_cap) return;   // overflow: nothing is flattened (redo)
    const uint64_t off = b.moff[k];
    const uint64_t at = lo32(off) + hi32(off);
    const uint4 mi = b.minfo[k];
    const uint64_t end = at + mi.y + mi.z + mi.w;
    for (uint64_t c = (at + 63) >> 6; (c << 6) < end; ++c) b.chunk_first[c] = (uint32_t)k;
}
// bucket path: chunk_first from the items scan's store phase (its offsets
// are at hand there), nothing when the tick overflowed (the host redoes it)
struct ItemsPost {
    uint32_t* chunk_first;
    const unsigned long long* ev_pk;
    uint64_t ev_cap;
    __device__ bool active() const {
        const unsigned long long e = *ev_pk;
        return lo32(e) + hi32(e) <= ev_cap;
    }
    __device__ void operator()(uint64_t k, uint32_t at, uint32_t cnt) const {
        const uint64_t end = (uint64_t)at + cnt;
        for (uint64_t c = ((uint64_t)at + 63) >> 6; (c << 6) < end; ++c) chunk_first[c] = (uint32_t)k;
    }
};
// element p = 64c + lane of the flat list (wave-uniform c; every lane runs
// the shuffles); false past E
__device__ __forceinline__ bool flat_elem(const TickBufs& b, uint64_t c, uint64_t E, uint32_t& key, uint32_t& val) {
    const uint64_t nl_ = b.st->n_mlist;
    const int ln = lane_id();
    const uint32_t q0 = b.chunk_first[c];
    const uint64_t k = (uint64_t)q0 + ln;
    uint64_t at = ~0ull, end = ~0ull, reg = 0;
    uint4 mi = make_uint4(0, 0, 0, 0);
    if (k < nl_) {
        const uint64_t off = b.moff[k];
        mi = b.minfo[k];
        reg = b.mreg[k];
        at = lo32(off) + hi32(off);
        end = at + mi.y + mi.z + mi.w;
    }
    const uint64_t p = (c << 6) + ln;
    // first lane q whose mover ends after p (ends ascend with the lane)
    uint32_t lo = 0, hi = 64;
#pragma unroll
    for (int s = 0; s < 7; ++s) {                           // [lo, hi) of 64 closes in 7 halvings
        const uint32_t mid = min((lo + hi) >> 1, 63u);
        const uint64_t e = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(end >> 32), (int)mid, 64) << 32) |
                           (uint32_t)__shfl((int)(uint32_t)end, (int)mid, 64);
        if (lo < hi) {
            if (e <= p) lo = mid + 1; else hi = mid;
        }
    }
    const int q = (int)min(lo, 63u);
    const uint64_t qat = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(at >> 32), q, 64) << 32) |
                         (uint32_t)__shfl((int)(uint32_t)at, q, 64);
    const uint64_t qreg = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(reg >> 32), q, 64) << 32) |
                          (uint32_t)__shfl((int)(uint32_t)reg, q, 64);
    const uint32_t qA = (uint32_t)__shfl((int)mi.x, q, 64), qn = (uint32_t)__shfl((int)(mi.y + mi.z), q, 64);
    if (p >= E) return false;
    const uint32_t j = (uint32_t)(p - qat);                 // index inside mover q's events
    const uint32_t lvb = 1u << b.wbits;
    if (j < qn) {
        const uint32_t e = b.own[qreg + j];
        key = ((e >> 31) ? lvb : 0u) | qA;
        val = e & 0x7fffffffu;
    } else {
        const uint64_t e = b.mir[qreg + (j - qn)];
        key = ((e & 1u) ? lvb : 0u) | (uint32_t)hi32(e);
        val = (uint32_t)(lo32(e) >> 1);
    }
    return true;
}

// flat list: (key, value) arrays for the general sort, or one u64
// (leave<<wbits | watcher) << wbits | target per event for the bucket path
__global__ void __launch_bounds__(NT) k_flatten(TickBufs b) {
    const uint64_t E = lo32(b.st->ev_pk) + hi32(b.st->ev_pk);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (E > b.ev_cap) atomicOr(&b.st->overflow, 1ull);
        b.st->n_sort = E > b.ev_cap ? 0 : E;              // nothing is sorted on overflow (the host redoes)
    }
    if (E > b.ev_cap) return;
    const uint64_t c = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if ((c << 6) >= E) return;
    uint32_t key, val;
    if (!flat_elem(b, c, E, key, val)) return;
    const uint64_t p = (c << 6) + lane_id();
    b.fk0[p] = key;
    b.fv0[p] = val;
}

// Bucket path items (u64): a mirror event (leave, watcher W, target A) is
// (leave<<wbits | W) << wbits | A; an own run of mover A (all its enters, or
// all its leaves; a mover's own events are sorted by (leave, target)) is
// BK_RUN | (leave<<wbits | A) << wbits | k (k: its listed-mover index).  A
// (leave, watcher) key holds one run (the watcher moved) or mirror events
// only (it did not), so items sort by their masked key and runs expand to
// their events at output time.
constexpr int BK_RUN_BIT = BK_KEY_BITS;               // just above the (leave, watcher, target) bits
constexpr uint64_t BK_RUN = 1ull << BK_RUN_BIT;
// item of flat position p = 64c + ln (wave-uniform c; every lane runs the
// shuffles) and the events it stands for (bk_weight); false past NI
__device__ __forceinline__ bool flat_item(const TickBufs& b, uint64_t c, uint64_t NI, uint64_t nl_, int ln,
                                          uint64_t& item, uint32_t& wt) {
    const uint32_t q0 = b.chunk_first[c];
    const uint64_t k = (uint64_t)q0 + ln;
    uint32_t at = 0xffffffffu, end = 0xffffffffu;
    uint4 mi = make_uint4(0, 0, 0, 0);
    uint64_t reg = 0;
    if (k < nl_) {
        at = b.ioff[k];
        end = at + b.icnt[k];
        mi = b.minfo[k];
        reg = b.mreg[k];
    }
    const uint32_t p = (uint32_t)((c << 6) + ln);
    uint32_t lo = 0, hi = 64;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
        const uint32_t mid = min((lo + hi) >> 1, 63u);
        const uint32_t e = (uint32_t)__shfl((int)end, (int)mid, 64);
        if (lo < hi) {
            if (e <= p) lo = mid + 1; else hi = mid;
        }
    }
    const int q = (int)min(lo, 63u);
    const uint32_t qat = (uint32_t)__shfl((int)at, q, 64);
    const uint64_t qreg = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(reg >> 32), q, 64) << 32) |
                          (uint32_t)__shfl((int)(uint32_t)reg, q, 64);
    const uint32_t qA = (uint32_t)__shfl((int)mi.x, q, 64);
    const uint32_t qe = (uint32_t)__shfl((int)mi.y, q, 64), ql = (uint32_t)__shfl((int)mi.z, q, 64);
    if (p >= NI) return false;
    const uint32_t W = (uint32_t)b.wbits;
    const uint32_t lvb = 1u << W;
    const uint32_t j = p - qat;
    const uint32_t nr = (qe ? 1u : 0u) + (ql ? 1u : 0u);
    if (j < nr) {
        const bool leave = (j == 1) || !qe;
        item = BK_RUN | ((uint64_t)((leave ? lvb : 0u) | qA) << W) | (q0 + (uint32_t)q);
        wt = leave ? ql : qe;
    } else {
        const uint64_t e = b.mir[qreg + (j - nr)];
        item = ((uint64_t)(((e & 1u) ? lvb : 0u) | (uint32_t)hi32(e)) << W) | (uint32_t)(lo32(e) >> 1);
        wt = 1u;
    }
    return true;
}
__device__ __forceinline__ void flat_chunk(const TickBufs& b, uint64_t c, uint64_t NI, uint64_t nl_, int ln) {
    uint64_t item;
    uint32_t wt;
    if (flat_item(b, c, NI, nl_, ln, item, wt)) b.bk_a[(c << 6) + ln] = item;
}

__global__ void __launch_bounds__(NT) k_flat_items(TickBufs b) {
    const uint64_t E = lo32(b.st->ev_pk) + hi32(b.st->ev_pk);
    const uint64_t NI = b.st->n_items;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (E > b.ev_cap) atomicOr(&b.st->overflow, 1ull);
        const uint64_t n = E > b.ev_cap ? 0 : NI;
        b.st->n_sort = n;
        const uint64_t T = (n + BK_TILE - 1) / BK_TILE;      // tiles in use: the count table's stride
        b.st->bk_tiles = T;
        b.st->bk_cells = T << b.bk_bits;
    }
    if (E > b.ev_cap) return;
    const int ln = lane_id();
    const uint64_t nl_ = b.st->n_mlist;
    // grid-stride over the 64-position chunks: the grid is sized by the last
    // tick's item count, not by the event capacity (750k mostly idle waves
    // cost 60 us of dispatch at config #4)
    for (uint64_t c = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6); (c << 6) < NI;
         c += (uint64_t)gridDim.x * NWAVE)
        flat_chunk(b, c, NI, nl_, ln);
}

// (4) bucket path.  Events are keyed by the full (leave, watcher, target) —
// unique within a tick — so no pass needs to be stable: the flat list is
// cut into tiles; each tile counts its events per bucket (a range of
// (leave, watcher)); one exclusive scan of the bucket-major count table gives
// every (bucket, tile) its offset; each tile stages its events by bucket in
// LDS and writes runs; each bucket (a few thousand events) is then sorted in
// LDS and written as gw_event.  Two passes over the events instead of three
// stable radix passes with look-back.  A bucket larger than the LDS sort is
// reported (overflow + bk_max) and the host redoes the tick on the general
// sort.
//
// Bucket bounds are quantiles of the previous tick's (leave, watcher) keys
// (bk_split_next), so skewed slot ranges (hotspot entities in adjacent slots)
// still give buckets of about the mean size; bucket(k) = #{bounds <= k},
// found through a 2^12-cell table of bound counts (A[x] = #{bounds < x <<
// lsh}) and a binary search inside the cell (usually empty).
// Flat entries: bucket << 54 | (leave<<wbits | watcher) << wbits | target
// (wbits <= 26, or the host takes the general sort).
constexpr int BK_LUT_BITS = 12;
// staged keys carry their bucket above the run bit (the scatter strips it)
constexpr int BK_KEY_SHIFT = 64 - BK_MAXBITS;
static_assert(BK_RUN_BIT < BK_KEY_SHIFT, "run bit below the staged bucket bits");

struct BkLut {
    uint32_t sp[1 << BK_MAXBITS];
    uint16_t a[(1 << BK_LUT_BITS) + 1];
};
__device__ __forceinline__ void bk_lut_build(const TickBufs& b, BkLut& L, uint32_t NB, int& lsh) {
    const uint32_t stride = BK_NSPLIT / NB;
    for (uint32_t i = threadIdx.x; i + 1 < NB; i += blockDim.x) L.sp[i] = b.bk_split[(i + 1) * stride];
    const int kb = b.wbits + 1;
    const int lb = min(kb, BK_LUT_BITS);
    lsh = kb - lb;
    __syncthreads();
    for (uint32_t x = threadIdx.x; x <= (1u << lb); x += blockDim.x) {
        const uint64_t v = (uint64_t)x << lsh;                 // count bounds < v
        uint32_t lo = 0, hi = NB - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint64_t)L.sp[mid] < v) lo = mid + 1; else hi = mid;
        }
        L.a[x] = (uint16_t)lo;
    }
    __syncthreads();
}
__device__ __forceinline__ uint32_t bk_bucket(const BkLut& L, int lsh, uint32_t key) {
    const uint32_t x = key >> lsh;
    uint32_t lo = L.a[x], hi = L.a[x + 1];
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.sp[mid] <= key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// events an item stands for (a run: its mover's enters or leaves)
__device__ __forceinline__ uint32_t bk_weight(const TickBufs& b, uint64_t item) {
    if (!(item & BK_RUN)) return 1u;
    const uint32_t W = (uint32_t)b.wbits;
    const uint4 mi = b.minfo[(uint32_t)item & ((1u << W) - 1u)];
    return ((item >> (2 * W)) & 1u) ? mi.z : mi.y;
}

// per (bucket, tile): items | events << 32
// FLAT: the items are made here (flat_item) and stored for the scatter, in
// place of a k_flat_items launch before this one: the run weights come with
// the item, and the sizes k_flat_items published are computed by every block
// (block 0 publishes them)
template <bool FLAT>
__global__ void __launch_bounds__(BK_NT) k_bk_count(TickBufs b) {
    __shared__ uint32_t h[1 << BK_MAXBITS], hw[1 << BK_MAXBITS];
    __shared__ BkLut lut;
    const int t = threadIdx.x;
    const uint32_t NB = 1u << b.bk_bits;
    uint64_t n, T, nl_ = 0;
    if (FLAT) {
        const uint64_t E = lo32(b.st->ev_pk) + hi32(b.st->ev_pk);
        n = E > b.ev_cap ? 0 : b.st->n_items;               // nothing is sorted on overflow (the host redoes)
        T = (n + BK_TILE - 1) / BK_TILE;
        nl_ = b.st->n_mlist;
        if (blockIdx.x == 0 && t == 0) {
            if (E > b.ev_cap) atomicOr(&b.st->overflow, 1ull);
            b.st->n_sort = n;
            b.st->bk_tiles = T;
            b.st->bk_cells = T << b.bk_bits;
        }
    } else {
        n = b.st->n_sort;
        T = b.st->bk_tiles;
    }
    if (blockIdx.x >= T) return;                            // block-uniform
    const int W = b.wbits;
    const uint64_t km = (1ull << (2 * W + 1)) - 1;
    constexpr int IPT = BK_TILE / BK_NT;
    // the first tile's items and their weights are loaded before the bucket
    // table is built (its bound loads and searches overlap them); a strip's
    // tick has a few tiles, so this pass is one load chain long
    uint64_t k[IPT];
    uint32_t wt[IPT];
    auto load = [&](uint64_t tile) {
        const uint64_t base = tile * BK_TILE;
        if (FLAT) {
            // flat_item's chain for the IPT chunks of this wave, stage by
            // stage, so each stage's loads of all chunks are in flight together
            const int ln = lane_id();
            const uint64_t c0 = (base >> 6) + (uint64_t)(t >> 6);
            uint32_t q0[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint64_t c = c0 + (uint64_t)j * (BK_NT / 64);
                q0[j] = (c << 6) < n ? b.chunk_first[c] : 0u;
            }
            uint32_t at[IPT], end[IPT], ma[IPT], me[IPT], ml[IPT];
            uint64_t reg[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint64_t c = c0 + (uint64_t)j * (BK_NT / 64);
                const uint64_t kk = (uint64_t)q0[j] + ln;
                at[j] = end[j] = 0xffffffffu;
                ma[j] = me[j] = ml[j] = 0;
                reg[j] = 0;
                if ((c << 6) < n && kk < nl_) {
                    at[j] = b.ioff[kk];
                    end[j] = b.icnt[kk];
                    const uint4 mi = b.minfo[kk];
                    ma[j] = mi.x;
                    me[j] = mi.y;
                    ml[j] = mi.z;
                    reg[j] = b.mreg[kk];
                }
            }
            const uint32_t W = (uint32_t)b.wbits;
            const uint32_t lvb = 1u << W;
            uint64_t mj[IPT];                                       // mirror event index, ~0: a run or nothing
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint64_t c = c0 + (uint64_t)j * (BK_NT / 64);
                k[j] = 0;
                wt[j] = 0;
                mj[j] = ~0ull;
                if ((c << 6) >= n) continue;                        // wave-uniform
                if (end[j] != 0xffffffffu) end[j] += at[j];
                const uint32_t p = (uint32_t)((c << 6) + ln);
                uint32_t lo = 0, hi = 64;
#pragma unroll
                for (int s = 0; s < 7; ++s) {
                    const uint32_t mid = min((lo + hi) >> 1, 63u);
                    const uint32_t e = (uint32_t)__shfl((int)end[j], (int)mid, 64);
                    if (lo < hi) {
                        if (e <= p) lo = mid + 1; else hi = mid;
                    }
                }
                const int q = (int)min(lo, 63u);
                const uint32_t qat = (uint32_t)__shfl((int)at[j], q, 64);
                const uint64_t qreg = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(reg[j] >> 32), q, 64) << 32) |
                                      (uint32_t)__shfl((int)(uint32_t)reg[j], q, 64);
                const uint32_t qA = (uint32_t)__shfl((int)ma[j], q, 64);
                const uint32_t qe = (uint32_t)__shfl((int)me[j], q, 64), ql = (uint32_t)__shfl((int)ml[j], q, 64);
                if (p >= n) continue;
                const uint32_t jj = p - qat;
                const uint32_t nr = (qe ? 1u : 0u) + (ql ? 1u : 0u);
                if (jj < nr) {
                    const bool leave = (jj == 1) || !qe;
                    k[j] = BK_RUN | ((uint64_t)((leave ? lvb : 0u) | qA) << W) | (q0[j] + (uint32_t)q);
                    wt[j] = leave ? ql : qe;
                } else {
                    mj[j] = qreg + (jj - nr);
                }
            }
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if (mj[j] == ~0ull) continue;
                const uint64_t e = b.mir[mj[j]];
                k[j] = ((uint64_t)(((e & 1u) ? lvb : 0u) | (uint32_t)hi32(e)) << W) | (uint32_t)(lo32(e) >> 1);
                wt[j] = 1u;
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t i = base + (uint64_t)j * BK_NT + t;
            k[j] = i < n ? b.bk_a[i] : 0ull;
        }
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t i = base + (uint64_t)j * BK_NT + t;
            wt[j] = i < n ? bk_weight(b, k[j]) : 0u;
        }
    };
    load(blockIdx.x);
    int lsh;
    bk_lut_build(b, lut, NB, lsh);                          // (syncs)
    // grid-stride over the tiles: the grid is sized by the last tick's items,
    // not the event capacity (idle 57-KB-LDS blocks queued behind each other)
    for (uint64_t tile = blockIdx.x; tile < T; tile += gridDim.x) {
    for (uint32_t i = t; i < NB; i += BK_NT) h[i] = hw[i] = 0;
    __syncthreads();
    const uint64_t base = tile * BK_TILE;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = base + (uint64_t)j * BK_NT + t;
        if (i < n) {
            const uint32_t q = bk_bucket(lut, lsh, (uint32_t)((k[j] & km) >> W));
            b.bk_id[i] = (uint16_t)q;
            if (FLAT) b.bk_a[i] = k[j];
            atomicAdd(&h[q], 1u);
            atomicAdd(&hw[q], wt[j]);
        }
    }
    if (tile + gridDim.x < T) load(tile + gridDim.x);      // the next tile's loads under the count writes
    __syncthreads();
    for (uint32_t i = t; i < NB; i += BK_NT)
        b.bk_cnt[(uint64_t)i * T + tile] = (unsigned long long)h[i] | ((unsigned long long)hw[i] << 32);
    __syncthreads();                                        // before the next tile zeroes h / hw
    }
}

// exclusive scan of one value per thread over a block of NTH threads
template <int NTH>
__device__ __forceinline__ uint32_t bk_block_excl(uint32_t v, uint32_t* red) {
    const int t = threadIdx.x, w = t >> 6, ln = lane_id();
    const uint32_t inc = wave_incl_scan<uint32_t>(v);
    if (ln == 63) red[w] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int k = 0; k < NTH / 64; ++k) pre += (k < w) ? red[k] : 0u;
    return pre + inc - v;
}

__global__ void __launch_bounds__(BK_NT) k_bucket_scatter(TickBufs b) {
    __shared__ uint64_t stg[BK_TILE];
    __shared__ uint32_t h[1 << BK_MAXBITS], go[1 << BK_MAXBITS];
    __shared__ uint32_t red[BK_NT / 64];
    const int t = threadIdx.x;
    const uint64_t n = b.st->n_sort;
    const uint32_t NB = 1u << b.bk_bits;
    for (uint64_t tile = blockIdx.x; tile * BK_TILE < n; tile += gridDim.x) {   // grid-stride (k_bk_count)
    const uint64_t base = tile * BK_TILE;
    for (uint32_t i = t; i < NB; i += BK_NT) h[i] = 0;
    __syncthreads();
    constexpr int IPT = BK_TILE / BK_NT;
    uint64_t k[IPT];
    uint32_t r[IPT], q[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = base + (uint64_t)j * BK_NT + t;
        k[j] = i < n ? b.bk_a[i] : 0ull;
        q[j] = i < n ? b.bk_id[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = base + (uint64_t)j * BK_NT + t;
        k[j] |= (uint64_t)q[j] << BK_KEY_SHIFT;             // the bucket rides in the staged key
        r[j] = i < n ? atomicAdd(&h[q[j]], 1u) : 0u;
    }
    __syncthreads();
    // thread t: buckets [t*BPT, (t+1)*BPT)
    constexpr int BPT = (1 << BK_MAXBITS) / BK_NT;
    uint32_t cb[BPT], csum = 0;
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
        const uint32_t i = (uint32_t)t * BPT + u;
        cb[u] = i < NB ? h[i] : 0u;
        csum += cb[u];
    }
    uint32_t toff = bk_block_excl<BK_NT>(csum, red);
    const uint64_t T = b.st->bk_tiles;
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
        const uint32_t i = (uint32_t)t * BPT + u;
        if (i < NB) {
            h[i] = toff;
            go[i] = (uint32_t)b.bk_cnt[(uint64_t)i * T + tile] - toff;   // mod 2^32: dst = go + staged index
        }
        toff += cb[u];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = base + (uint64_t)j * BK_NT + t;
        if (i < n) stg[h[q[j]] + r[j]] = k[j];
    }
    __syncthreads();
    const uint32_t tn = (uint32_t)min<uint64_t>((uint64_t)BK_TILE, n - base);
    for (uint32_t i = t; i < tn; i += BK_NT) {              // each bucket's run of the tile is contiguous
        const uint64_t v = stg[i];
        const uint32_t dst = go[(uint32_t)(v >> BK_KEY_SHIFT)] + i;
        if (dst < n) b.bk_b[dst] = v & ((1ull << BK_KEY_SHIFT) - 1);
        else atomicOr(&b.st->overflow, 2ull);              // (inconsistent counts: never by construction)
    }
    __syncthreads();                                        // before the next tile reuses h / go / stg
    }
}

// One bucket per block.  Its items are counting-sorted by bin = (leave,
// watcher - floor) >> bsh (at most BK_HBINS bins; bsh = 0 unless the bucket
// spans a wide, sparse key range) and each bin is sorted in place by the
// masked key (a thread for <= BK_SHORT items, else a wave); the items' event
// counts are then prefix-summed in that order (the bucket's base comes from
// the scanned count table), mirror events are written by their lane and own
// runs are copied from the mover's own-event region by a wave.
__global__ void __launch_bounds__(BK_SNT) k_bucket_sort(TickBufs b) {
    __shared__ uint64_t L[BK_LCAP];
    __shared__ uint32_t hb[BK_HBINS];
    __shared__ uint32_t red[BK_SNT / 64];
    __shared__ uint16_t longs[BK_LCAP / (BK_SHORT + 1) + 1];   // bins sorted by a wave
    __shared__ uint4 runs[BK_RUNS];                            // (dst, src, len, watcher)
    __shared__ uint32_t n_long, n_runs;
    constexpr int NWV = BK_SNT / 64;
    constexpr int CH = BK_LCAP / BK_SNT;                    // max items per thread
    constexpr int WCH = BK_LCAP / BK_SNT;                   // max chunks of 64 per wave
    const uint32_t bk = blockIdx.x;
    const uint32_t NB = 1u << b.bk_bits;
    const uint64_t T = b.st->bk_tiles;
    const uint64_t n_all = b.st->n_sort;
    if (n_all == 0) return;
    const unsigned long long c0 = b.bk_cnt[(uint64_t)bk * T];
    const uint64_t s = lo32(c0);
    const uint64_t e = bk + 1 < NB ? lo32(b.bk_cnt[(uint64_t)(bk + 1) * T]) : n_all;
    if (e <= s) return;
    const uint32_t wbase = (uint32_t)hi32(c0);              // events of the earlier buckets
    const uint32_t n = (uint32_t)(e - s);
    const int t = threadIdx.x, w = t >> 6, ln = lane_id();
    if (n > BK_LCAP) {                                      // too large for LDS: the host redoes on the general sort
        if (t == 0) {
            atomicOr(&b.st->overflow, 1ull);
            atomicMax(&b.st->bk_max, (unsigned long long)n);
        }
        return;
    }
    const uint32_t stride = BK_NSPLIT / NB;
    const uint32_t W = (uint32_t)b.wbits;
    const uint32_t lo = bk ? b.bk_split[bk * stride] : 0u;
    const uint32_t hi_max = bk + 1 < NB ? b.bk_split[(bk + 1) * stride] : (2u << W);
    const uint32_t span = hi_max - lo;
    int bsh = 0;
    while (((span - 1) >> bsh) >= (uint32_t)BK_HBINS) ++bsh;
    const uint32_t nbins = ((span - 1) >> bsh) + 1;
    const uint64_t km = (1ull << (2 * W + 1)) - 1;          // (leave, watcher, target) bits
    for (uint32_t i = t; i < nbins; i += BK_SNT) hb[i] = 0;
    if (t == 0) n_long = n_runs = 0;
    __syncthreads();
    uint64_t key[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const uint32_t i = (uint32_t)t + (uint32_t)k * BK_SNT;
        key[k] = i < n ? b.bk_b[s + i] : 0ull;
    }
#define BK_BIN(v) ((uint32_t)((((v) & km) >> W) - lo) >> bsh)
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const uint32_t i = (uint32_t)t + (uint32_t)k * BK_SNT;
        if (i < n) atomicAdd(&hb[BK_BIN(key[k])], 1u);
    }
    __syncthreads();
    constexpr int PER = BK_HBINS / BK_SNT;                  // consecutive bins per thread
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = (uint32_t)t * PER + q;
        c[q] = i < nbins ? hb[i] : 0u;
        sum += c[q];
    }
    uint32_t run = bk_block_excl<BK_SNT>(sum, red);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = (uint32_t)t * PER + q;
        if (i < nbins) hb[i] = run;
        if (c[q] > (uint32_t)BK_SHORT) longs[atomicAdd(&n_long, 1u)] = (uint16_t)i;
        run += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        const uint32_t i = (uint32_t)t + (uint32_t)k * BK_SNT;
        if (i < n) L[atomicAdd(&hb[BK_BIN(key[k])], 1u)] = key[k];
    }
#undef BK_BIN
    __syncthreads();
    // each bin in place by the masked key.  Short bins: an item's place = the
    // bin start + the bin's items with a smaller key (keys are unique), all
    // read before any is written back
    uint32_t pos[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        pos[k] = 0xffffffffu;
        const uint32_t i = (uint32_t)t + (uint32_t)k * BK_SNT;
        if (i >= n) continue;
        const uint32_t x = (uint32_t)((((key[k]) & km) >> W) - lo) >> bsh;
        const uint32_t r0 = x ? hb[x - 1] : 0u, r1 = hb[x];
        if (r1 - r0 > (uint32_t)BK_SHORT) continue;        // a wave sorts the long bins
        const uint64_t kk = key[k] & km;
        uint32_t r = r0, j = r0;
        for (; j + 4 <= r1; j += 4)
            r += (uint32_t)((L[j] & km) < kk) + (uint32_t)((L[j + 1] & km) < kk) +
                 (uint32_t)((L[j + 2] & km) < kk) + (uint32_t)((L[j + 3] & km) < kk);
        for (; j < r1; ++j) r += (uint32_t)((L[j] & km) < kk);
        pos[k] = r;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CH; ++k)
        if (pos[k] != 0xffffffffu) L[pos[k]] = key[k];
    const uint32_t nl = n_long;
    for (uint32_t q = (uint32_t)w; q < nl; q += NWV) {
        const uint32_t x = longs[q];
        const uint32_t g0 = x ? hb[x - 1] : 0u, gn = hb[x] - g0;
        uint64_t* R = L + g0;
        if (gn <= 64) {                                     // in registers
            uint64_t v = ln < (int)gn ? R[ln] : ~0ull;
            const uint64_t sk = ln < (int)gn ? ((v & km) << 10) | (uint64_t)ln : ~0ull;   // masked key, then lane
            const uint64_t o = wave_sort64_u64(sk);
            const int from = (int)(o & 1023u);
            const uint64_t moved = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), from & 63, 64) << 32) |
                                   (uint32_t)__shfl((int)(uint32_t)v, from & 63, 64);
            wave_sync();
            if (ln < (int)gn) R[ln] = moved;
        } else {
            bitonic_inplace<64>(R, gn, ln, [km](uint64_t v) { return v & km; }, [] { wave_sync(); });
        }
        wave_sync();
    }
    __syncthreads();
    // event offsets: the items' weights prefix-summed in sorted order (wave w
    // takes [w*seg, (w+1)*seg) in chunks of 64); the runs' mover records are
    // loaded for all chunks at once
    const uint32_t seg = (((n + NWV - 1) / NWV) + 63) & ~63u;
    const uint32_t w0 = (uint32_t)w * seg;
    const uint32_t wm = (1u << W) - 1u;
    uint64_t v[WCH];
    uint32_t off[WCH], aux[WCH];
#pragma unroll
    for (int cc = 0; cc < WCH; ++cc) {
        const uint32_t i = w0 + (uint32_t)cc * 64 + ln;
        v[cc] = (cc * 64 < (int)seg && i < n) ? L[i] : 0ull;
    }
    uint4 mi[WCH];
#pragma unroll
    for (int cc = 0; cc < WCH; ++cc) {
        mi[cc] = make_uint4(0, 0, 0, 0);
        aux[cc] = 0;
        if (v[cc] & BK_RUN) {
            const uint32_t k = (uint32_t)v[cc] & wm;
            mi[cc] = b.minfo[k];
            aux[cc] = (uint32_t)b.mreg[k];
        }
    }
    uint32_t carry = 0;
#pragma unroll
    for (int cc = 0; cc < WCH; ++cc) {
        off[cc] = 0;
        if (cc * 64 >= (int)seg) continue;                  // wave-uniform
        const uint32_t i = w0 + (uint32_t)cc * 64 + ln;
        const bool leave = ((v[cc] >> (2 * W)) & 1u) != 0;
        const uint32_t wt = i >= n ? 0u : !(v[cc] & BK_RUN) ? 1u : (leave ? mi[cc].z : mi[cc].y);
        const uint32_t inc = wave_incl_scan<uint32_t>(wt);
        off[cc] = carry + inc - wt;
        carry += (uint32_t)__shfl((int)inc, 63, 64);
    }
    if (ln == 63) red[w] = carry;
    __syncthreads();
    uint32_t wpre = wbase;
    for (int k = 0; k < w; ++k) wpre += red[k];
#pragma unroll
    for (int cc = 0; cc < WCH; ++cc) {
        if (cc * 64 >= (int)seg) continue;
        const uint32_t i = w0 + (uint32_t)cc * 64 + ln;
        if (i >= n) continue;
        const uint32_t dst = wpre + off[cc];
        if (dst >= b.ev_cap) {                              // (never by construction; no wild writes)
            atomicOr(&b.st->overflow, 2ull);
            continue;
        }
        if (!(v[cc] & BK_RUN)) {
            gw_event ev;
            ev.watcher = (uint32_t)(v[cc] >> W) & wm;
            ev.target = (uint32_t)v[cc] & wm;
            b.ev[dst] = ev;
        } else {
            const bool leave = ((v[cc] >> (2 * W)) & 1u) != 0;
            const uint32_t len = leave ? mi[cc].z : mi[cc].y;
            const uint32_t src = aux[cc] + (leave ? mi[cc].y : 0u);
            if (dst + len > b.ev_cap) {
                atomicOr(&b.st->overflow, 2ull);
                continue;
            }
            const uint32_t q = atomicAdd(&n_runs, 1u);
            if (q < (uint32_t)BK_RUNS) {
                runs[q] = make_uint4(dst, src, len, mi[cc].x);
            } else {                                        // list full: this lane copies
                for (uint32_t j = 0; j < len; ++j) {
                    gw_event ev;
                    ev.watcher = mi[cc].x;
                    ev.target = b.own[src + j] & 0x7fffffffu;
                    b.ev[dst + j] = ev;
                }
            }
        }
    }
    __syncthreads();
    // own runs, flattened over the block: run prefix sums in hb (free now),
    // each thread copies every 512th event (binary search for its run)
    const uint32_t nr = min(n_runs, (uint32_t)BK_RUNS);
    const uint32_t rl = (uint32_t)t < nr ? runs[t].z : 0u;  // BK_RUNS == BK_SNT: one run per thread
    const uint32_t rpre = bk_block_excl<BK_SNT>(rl, red);
    if ((uint32_t)t < nr) hb[t] = rpre;
    if (t == BK_SNT - 1) hb[BK_RUNS] = rpre + rl;
    __syncthreads();
    const uint32_t tot = hb[BK_RUNS];
    constexpr int CU = 4;
    for (uint32_t e0 = (uint32_t)t; e0 < tot; e0 += CU * BK_SNT) {
        uint32_t tg[CU], dd[CU], ww[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            const uint32_t e1 = e0 + (uint32_t)u * BK_SNT;
            dd[u] = 0xffffffffu;
            if (e1 >= tot) continue;
            uint32_t lo_ = 0, hi_ = nr;                     // last run with prefix <= e1
            while (hi_ - lo_ > 1) {
                const uint32_t mid = (lo_ + hi_) >> 1;
                if (hb[mid] <= e1) lo_ = mid; else hi_ = mid;
            }
            const uint4 r = runs[lo_];
            const uint32_t j = e1 - hb[lo_];
            tg[u] = b.own[r.y + j];
            dd[u] = r.x + j;
            ww[u] = r.w;
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            if (dd[u] == 0xffffffffu) continue;
            gw_event ev;
            ev.watcher = ww[u];
            ev.target = tg[u] & 0x7fffffffu;
            b.ev[dd[u]] = ev;
        }
    }
}

// quantiles of this tick's sorted (leave, watcher) keys: the next tick's
// bucket bounds (BK_NSPLIT of them; a tick with fewer buckets takes every
// (BK_NSPLIT / NB)-th).  Kept when the tick overflowed or had no events.
constexpr uint32_t SPLIT_PT = BK_NSPLIT / RESET_NT;      // splits per reset thread
// the loads: every split's event in flight together (registers), stored by
// bk_split_store after the statistics copy has been issued
__device__ __forceinline__ bool bk_split_load(const TickBufs& b, unsigned long long ev_pk, unsigned long long overflow,
                                              uint32_t (&v)[SPLIT_PT]) {
    const uint64_t E = lo32(ev_pk) + hi32(ev_pk), ne = lo32(ev_pk);
    if (E == 0 || E > b.ev_cap || overflow) return false;
    const uint32_t lvb = 1u << b.wbits;
#pragma unroll
    for (uint32_t q = 0; q < SPLIT_PT; ++q) {
        const uint32_t j = q * RESET_NT + threadIdx.x;
        const uint64_t p = (uint64_t)j * E / BK_NSPLIT;
        v[q] = (p >= ne ? lvb : 0u) | b.ev[p].watcher;
    }
    return true;
}
__device__ __forceinline__ void bk_split_store(const TickBufs& b, const uint32_t (&v)[SPLIT_PT]) {
#pragma unroll
    for (uint32_t q = 0; q < SPLIT_PT; ++q) {
        const uint32_t j = q * RESET_NT + threadIdx.x;
        if (j) b.bk_split[j] = v[q];
    }
}
// uniform bounds over the key range [0, 2^(wbits+1))
__global__ void __launch_bounds__(NT) k_bk_split_init(uint32_t* sp, int wbits) {
    for (uint32_t j = threadIdx.x; j < BK_NSPLIT; j += NT)
        sp[j] = (uint32_t)(((uint64_t)j << (wbits + 1)) / BK_NSPLIT);
}
void launch_bk_split_init(uint32_t* sp, int wbits, hipStream_t s) {
    hipLaunchKernelGGL(k_bk_split_init, dim3(1), dim3(NT), 0, s, sp, wbits);
}

void tick_diff(const TickBufs& b, hipStream_t s) {
    const uint64_t nmax = 2ull * b.m;
    if (b.small_ents) {                    // small-space mode: a block per space
        const size_t lds = ((size_t)b.small_ents + (2 * ((size_t)b.small_cells + 1) + 3) / 4) * 16 +
                           (size_t)SMALL_GM * sizeof(MEnt);
        if (b.small_halves) {
            hipLaunchKernelGGL((k_mover_small<2, true>), dim3(b.n_spaces), dim3(NT), lds, s, b);
            hipLaunchKernelGGL((k_mover_list<2>), dim3(std::min<uint32_t>(nblk1(nmax, 1), 1024)), dim3(64), 0, s, b);
        } else {
            hipLaunchKernelGGL((k_mover_small<2, false>), dim3(b.n_spaces), dim3(NT), lds, s, b);
        }
        return;
    }
    if (b.pair_max) {                      // two short-list movers per wave (GW_PAIR_MAX, 0 = off)
        hipLaunchKernelGGL((k_mover_pair<2>), dim3(nblk1(nmax, 2)), dim3(64), 0, s, b);
        return;
    }
    if (b.compact) {                       // one wave per primary entry (<= one per op)
        const dim3 g(nblk1(b.m, 1));
        // gate words: 0, or 2 (<= 8 gate ids) / 4 per lane for the split by gate
        const int gw = b.gate_counts ? (b.gate_counts <= 8 ? 2 : 4) : 0;
        if (std::isinf(b.long_step)) {     // no long movers: the group-teleport paths compiled out
            if (gw == 2) hipLaunchKernelGGL((k_mover_c<2, false, 2>), g, dim3(64), 0, s, b);
            else if (gw == 4) hipLaunchKernelGGL((k_mover_c<2, false, 4>), g, dim3(64), 0, s, b);
            else hipLaunchKernelGGL((k_mover_c<2, false, 0>), g, dim3(64), 0, s, b);
        } else {
            if (gw == 2) hipLaunchKernelGGL((k_mover_c<2, true, 2>), g, dim3(64), 0, s, b);
            else if (gw == 4) hipLaunchKernelGGL((k_mover_c<2, true, 4>), g, dim3(64), 0, s, b);
            else hipLaunchKernelGGL((k_mover_c<2, true, 0>), g, dim3(64), 0, s, b);
        }
        return;
    }
    switch (b.diff_u) {                    // GW_MOVER_WPB: waves per k_mover block
    case 2: hipLaunchKernelGGL((k_mover<2, 2>), dim3(nblk1(nmax, 2)), dim3(128), 0, s, b); break;
    case 4: hipLaunchKernelGGL((k_mover<2, 4>), dim3(nblk1(nmax, 4)), dim3(256), 0, s, b); break;
    default: hipLaunchKernelGGL((k_mover<2, 1>), dim3(nblk1(nmax, 1)), dim3(64), 0, s, b); break;
    }
}
void tick_events(const TickBufs& b, ScanCtx& sc, hipStream_t s) {
    const uint64_t nmax = 2ull * b.m;
    // movers in slot order, and k_mover_post's work in the same launch
    // (GW_POST_SPLIT=1: a launch of its own first)
    const uint64_t nwords = (uint64_t)b.w.cap / 32 + 1;
    const uint64_t tile = (uint64_t)SCAN_IPT * NT;
    const uint32_t nb = nblk1(nwords, (uint32_t)tile);
    const bool split = b.post_split != 0;
    if (split) hipLaunchKernelGGL(k_mover_post, dim3(STAT_SHARDS + 64), dim3(NT), 0, s, b);
    if (sc.tag >= SCAN_TAG_MAX) {
        (void)hipMemsetAsync(sc.status, 0, sc.max_tiles * SCAN_WORDS * 8, s);
        sc.tag = 0;
    }
    ++sc.tag;
    hipLaunchKernelGGL(k_bits_list<SCAN_IPT>, dim3(nb + (split ? 0 : STAT_SHARDS + 64)), dim3(NT), 0, s, b.movbit,
                       nwords, b.mlist, sc.status, sc.ticket, sc.tbase, sc.tag, &b.st->n_mlist, b, nb);
    sc.tbase += nb;
    const uint64_t* nml = (const uint64_t*)&b.st->n_mlist;
    hipLaunchKernelGGL(k_mover_counts, dim3(nblk1(b.m, NT)), dim3(NT), 0, s, b);
    if (!b.ev_full) {
        const uint32_t NB = 1u << b.bk_bits;
        scan_exclusive<uint32_t, uint32_t>(b.icnt, b.ioff, b.m, nml, sc, (uint32_t*)&b.st->n_items, s,
                                           ItemsPost{b.chunk_first, &b.st->ev_pk, b.ev_cap});
        const uint64_t fw = std::min<uint64_t>((b.ev_cap + 63) / 64,
                                               std::max<uint64_t>(8192, (2 * b.it_hint + 63) / 64));
        uint32_t fb = nblk1(fw, NWAVE);
        if (b.grid_cap) fb = std::min(fb, b.grid_cap);
        // tile passes: grid-stride over a grid sized by the last tick's items
        uint32_t bt = (uint32_t)std::min<uint64_t>(
            b.bk_tiles, std::max<uint64_t>(256, (2 * b.it_hint + BK_TILE - 1) / BK_TILE));
        if (b.grid_cap) bt = std::min(bt, b.grid_cap);
        // the items made by the count pass when there are many tiles (config #3
        // events 134 -> 131 us, #4 217 -> 214 us); with fewer (config #2, world
        // strips: tens of tiles) those blocks would walk every item's chain
        // alone (+5 us at #2, +5-6 us on #3 / #5 strips), so small ticks keep
        // k_flat_items, which spreads the chains over the chip first
        // (GW_BK_FLAT=0 / 1 forces either)
        const bool flat_in_count = b.bk_flat >= 0 ? b.bk_flat != 0 : b.it_hint >= 128ull * BK_TILE;
        if (flat_in_count) {
            hipLaunchKernelGGL(k_bk_count<true>, dim3(bt), dim3(BK_NT), 0, s, b);
        } else {
            hipLaunchKernelGGL(k_flat_items, dim3(fb), dim3(NT), 0, s, b);
            hipLaunchKernelGGL(k_bk_count<false>, dim3(bt), dim3(BK_NT), 0, s, b);
        }
        scan_exclusive<uint64_t, uint64_t>((const uint64_t*)b.bk_cnt, (uint64_t*)b.bk_cnt,
                                           (uint64_t)NB * b.bk_tiles, (const uint64_t*)&b.st->bk_cells, sc,
                                           (uint64_t*)nullptr, s);
        hipLaunchKernelGGL(k_bucket_scatter, dim3(bt), dim3(BK_NT), 0, s, b);
        hipLaunchKernelGGL(k_bucket_sort, dim3(NB), dim3(BK_SNT), 0, s, b);
    } else {
        scan_exclusive<uint64_t, uint64_t>((const uint64_t*)b.mcnt, (uint64_t*)b.moff, b.m, nml, sc,
                                           (uint64_t*)&b.st->ev_pk, s);
        hipLaunchKernelGGL(k_chunk_first, dim3(nblk1(b.m, NT)), dim3(NT), 0, s, b);
        hipLaunchKernelGGL(k_flatten, dim3(nblk1((b.ev_cap + 63) / 64, NWAVE)), dim3(NT), 0, s, b);
        // one stable sort by (leave, watcher); the last pass writes gw_event
        radix_sort2(b.fk0, b.fv0, b.fk1, b.fv1, b.ev_cap, (const uint64_t*)&b.st->n_sort, 0, b.wbits + 1,
                    b.rtable, s, b.ev, (1u << b.wbits) - 1u);
    }
    (void)nmax;
}

// ---------------------------------------------------------------------------
// after the tick: the next tick's bucket bounds, and the device statistics
// zeroed, so no reset copy runs at the next tick's start.  Nothing per op or
// per mover: the dedupe words age out with their session tag, the mover bits
// with the rebuild parity.  One block: the tick's event totals and overflow
// flag are read from the device statistics before the block zeroes them, so
// the pass needs nothing from the host and a collect queues it behind its
// statistics copy, before its host sync (off the path between the collect and
// the next tick).  The host reads the published words only after a stream
// sync, which makes a kernel's writes to pinned host memory visible: no
// system-scope fence (an L2 write-back of the tick's dirty lines) here
// (GW_PUB_FENCE=1 puts it back, for comparison).
#if defined(GW_PUB_FENCE) && GW_PUB_FENCE
#define PUB_FENCE() __threadfence_system()
#else
#define PUB_FENCE() ((void)0)
#endif
__global__ void __launch_bounds__(RESET_NT) k_tick_reset(TickBufs b, const unsigned long long* __restrict__ pub_src,
                                                        unsigned long long* pub_dst, uint32_t pub_words) {
    // the statistics (at most two DevStats: the tick's and the collect's) are
    // loaded first, every word in flight together, then the next tick's
    // bucket bounds (their event loads depend on the tick's event totals)
    constexpr uint32_t HDR = (uint32_t)(offsetof(DevStats, shard) / 8), DSW = (uint32_t)(sizeof(DevStats) / 8);
    static_assert(STAT_SHARDS * SH_FIELDS == RESET_NT, "one shard word per thread");
    static_assert(SH_FIELDS <= 4 && (SH_FIELDS & (SH_FIELDS - 1)) == 0, "fields per lane group");
    constexpr int QMAX = 2, NWR = RESET_NT / 64;
    const uint32_t nq = min(pub_words / DSW, (uint32_t)QMAX);
    unsigned long long hv[QMAX], sv[QMAX];
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
        hv[q] = sv[q] = 0;
        if ((uint32_t)q < nq) {
            const unsigned long long* src = pub_src + (size_t)q * DSW;
            if (threadIdx.x < HDR) hv[q] = src[threadIdx.x];
            sv[q] = src[HDR + threadIdx.x];               // shard t / SH_FIELDS, field t % SH_FIELDS
        }
    }
    uint32_t v[SPLIT_PT];
    const bool split = b.st && bk_split_load(b, b.st->ev_pk, b.st->overflow, v);
    // written straight into the host's (coherent, pinned) buffer: each DevStats
    // as its header words and, per field, the sum of its shards in shard[0]
    // (20 PCIe stores instead of 1040: the host reads shard[0] only).  The sums:
    // lane xor-shuffles over the shards a wave holds, then the waves' partials
    __shared__ unsigned long long red[QMAX][NWR * SH_FIELDS];
    const int ln = lane_id(), wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
        if ((uint32_t)q >= nq) break;
        unsigned long long x = sv[q];
        for (int o = SH_FIELDS; o < 64; o <<= 1) {
            const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)x, o, 64);
            const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)(x >> 32), o, 64);
            x += ((unsigned long long)hi << 32) | lo;
        }
        if (ln < SH_FIELDS) red[q][wv * SH_FIELDS + ln] = x;
        if (threadIdx.x < HDR) pub_dst[(size_t)q * DSW + threadIdx.x] = hv[q];
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)(QMAX * SH_FIELDS)) {
        const uint32_t q = threadIdx.x / SH_FIELDS, f = threadIdx.x % SH_FIELDS;
        if (q < nq) {
            unsigned long long x = 0;
#pragma unroll
            for (int k = 0; k < NWR; ++k) x += red[q][k * SH_FIELDS + f];
            pub_dst[(size_t)q * DSW + HDR + f] = x;
        }
    }
    if (!b.st) {
        PUB_FENCE();
        return;
    }
    if (split) bk_split_store(b, v);
    __syncthreads();                                        // every read of the statistics done
    unsigned long long* z = (unsigned long long*)b.st;
    for (uint32_t k = threadIdx.x; k < sizeof(DevStats) / 8; k += RESET_NT) z[k] = 0;
    PUB_FENCE();
}

void tick_reset(const TickBufs& b, hipStream_t s) {
    hipLaunchKernelGGL(k_tick_reset, dim3(1), dim3(RESET_NT), 0, s, b, nullptr, nullptr, 0u);
}
struct PubTab {
    PubSeg s[4];
    int n;
};
__global__ void __launch_bounds__(RESET_NT) k_publish_words(PubTab t) {
    for (int q = 0; q < t.n; ++q)
        for (uint32_t k = threadIdx.x; k < t.s[q].words; k += RESET_NT) t.s[q].dst[k] = t.s[q].src[k];
    PUB_FENCE();
}
void publish_words(const PubSeg* segs, int n, hipStream_t s) {
    PubTab t{};
    for (int q = 0; q < n && q < 4; ++q) t.s[t.n++] = segs[q];
    hipLaunchKernelGGL(k_publish_words, dim3(1), dim3(RESET_NT), 0, s, t);
}
void publish_stats(const TickBufs* b, const void* src, void* host_dst, size_t bytes, hipStream_t s) {
    TickBufs t{};
    if (b) t = *b;                                   // with the tick's reset, else the copy alone (t.st null)
    hipLaunchKernelGGL(k_tick_reset, dim3(1), dim3(RESET_NT), 0, s, t, (const unsigned long long*)src,
                       (unsigned long long*)host_dst, (uint32_t)(bytes / 8));
}

}  // namespace gw
