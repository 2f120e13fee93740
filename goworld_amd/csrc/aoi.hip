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
//   diff     one wave per mover (in mover-grid order, i.e. by cell) walks
//            the non-movers of gn and the mover grid over its old and new
//            windows, evaluates the old and new relation of every candidate
//            and emits its own events, sorted (no atomics)
//   opless   the events of op-less watchers (pairs with a mover) come from
//            the watcher side: 64 consecutive grid entries per wave, the
//            movers of their search rectangles staged once, sorted by slot
//            and broadcast to every lane -- counted in one pass, written at
//            the scanned offsets in a second (no atomics, no scatter, no
//            per-watcher sort)
//   events   scan of the per-watcher counts -> canonical offsets; movers copy
//            their sorted own events, op-less watchers write theirs
// Outputs are placed by scans; the atomics left are per-cell histogram /
// cursor updates of the grid and per-shard statistics.  No MFMA: compare and
// gather work bound by L2/HBM latency and bandwidth.
#include <climits>

#include "dev_common.hpp"

namespace gw {

constexpr uint32_t SORT_LDS = 1024;     // own events sorted in a wave's LDS up to this many
constexpr uint32_t NO_CELL = 0xffffffffu;

// ---------------------------------------------------------------------------
// ops: last-op dedupe per slot (seq = index in the tick's op stream)
__global__ void __launch_bounds__(NT) k_ops1(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    if (op.slot >= b.w.cap || op.kind < GW_OP_ENTER || op.kind > GW_OP_SYNC) {
        atomicAdd(&b.st->bad_ops, 1ull);
        return;
    }
    if (op.kind != GW_OP_LEAVE) atomicMax(&b.last_pos[op.slot], (int32_t)i);
    if (op.kind != GW_OP_SYNC) atomicMax(&b.last_aoi[op.slot], (int32_t)i);
    if (op.kind == GW_OP_LEAVE) atomicMax(&b.last_leave[op.slot], (int32_t)i);
}

// a Leave clears syncInfoFlag (the entity leaves this space's sync set)
__global__ void __launch_bounds__(NT) k_ops2(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    if (op.slot >= b.w.cap || op.kind != GW_OP_LEAVE) return;
    if (b.last_leave[op.slot] == (int32_t)i) b.w.flags[op.slot] = 0;
}

__global__ void __launch_bounds__(NT) k_ops3(TickBufs b) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i < b.m) {
        const gw_op op = b.ops[i];
        const uint32_t s = op.slot;
        if (s < b.w.cap && op.kind >= GW_OP_ENTER && op.kind <= GW_OP_SYNC) {
            // syncInfoFlag |= bits of every call after the last Leave (Space.go:196,
            // Entity.go:1199-1204, 1286)
            if ((int32_t)i > b.last_leave[s] && op.sync_flags) atomicOr(&b.w.flags[s], (uint32_t)op.sync_flags);
            if (b.last_pos[s] == (int32_t)i) b.w.pos[s] = make_float4(op.x, op.y, op.z, op.yaw);
            if (b.last_aoi[s] == (int32_t)i) {
                AoiEnt a = b.w.aoi[s];
                PrevEnt p;
                const bool was = (a.meta & PRESENT_BIT) != 0;
                p.ox = was ? a.x : qnan();
                p.oz = was ? a.z : qnan();
                p.ostamp = b.w.stamp[s];
                b.w.prev[s] = p;
                b.w.stamp[s] = b.stamp_base + i;
                if (op.kind == GW_OP_LEAVE) a.meta &= ~PRESENT_BIT;
                else { a.x = op.x; a.z = op.z; a.meta |= PRESENT_BIT; }
                b.w.aoi[s] = a;
            }
        }
    }
}

void tick_ops(const TickBufs& b, hipStream_t s) {
    hipLaunchKernelGGL(k_ops1, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_ops2, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_ops3, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// full rebuild: stable LSD radix sort of (cell, slot) pairs (absent slots get
// the sentinel key ncells and sort last), so gn[] is in (cell, slot) order
__global__ void __launch_bounds__(NT) k_grid_keys(World w, uint32_t* k0, uint32_t* v0) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s >= w.cap) return;
    const AoiEnt a = w.aoi[s];
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
        const AoiEnt a = w.aoi[s];
        GEnt e;
        e.x = a.x; e.z = a.z; e.slot = s;
        e.meta = key | (w.gate[s] ? CLIENT_BIT : 0u);
        w.gn[i] = e;
        w.gidx[s] = i;
    }
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
}

// ---------------------------------------------------------------------------
// incremental grid.  co / cn: the mover's cell before / after the tick
// (NO_CELL when absent).  co is the cell its pre-tick grid entry sits in.
struct MoverCells {
    uint32_t A, co, cn;
    AoiEnt a;
    PrevEnt p;
};
__device__ __forceinline__ MoverCells mover_cells(const World& w, uint32_t A) {
    MoverCells m;
    m.A = A;
    m.a = w.aoi[A];
    m.p = w.prev[A];
    const SpaceP P = w.sp[m.a.meta & SPACE_MASK];
    m.co = m.cn = NO_CELL;
    if (m.p.ox == m.p.ox) m.co = cell_of(P, m.p.ox, m.p.oz);
    if (m.a.meta & PRESENT_BIT) m.cn = cell_of(P, m.a.x, m.a.z);
    return m;
}

// op i is slot s's mover entry when it is s's last AOI op (no list: a
// single-address list counter serialises across the chip)
__device__ __forceinline__ bool op_mover(const TickBufs& b, uint32_t i, uint32_t& s) {
    const gw_op op = b.ops[i];
    s = op.slot;
    return s < b.w.cap && op.kind >= GW_OP_ENTER && op.kind <= GW_OP_LEAVE && b.last_aoi[s] == (int32_t)i;
}

// per mover: mover-grid histogram; a mover staying in its cell is patched in
// place, the others count as a departure / an arrival of their cells
__global__ void __launch_bounds__(NT) k_classify(TickBufs b) {
    __shared__ uint32_t lds[NWAVE];
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    uint32_t A = 0;
    const bool mv = i < b.m && op_mover(b, i, A);
    uint32_t tot;
    (void)block_excl_scan<uint32_t>(mv ? 1u : 0u, lds, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(&b.st->n_movers, (unsigned long long)tot);
    if (mv) {
        const MoverCells mc = mover_cells(b.w, A);
        if (mc.co != NO_CELL) atomicAdd(&b.gm_cnt[mc.co], 1u);
        if (mc.cn != NO_CELL && mc.cn != mc.co) atomicAdd(&b.gm_cnt[mc.cn], 1u);
        if (mc.co != NO_CELL && mc.co == mc.cn) {
            GEnt e;
            e.x = mc.a.x; e.z = mc.a.z; e.slot = mc.A;
            e.meta = mc.cn | (b.w.gate[mc.A] ? CLIENT_BIT : 0u) | MOVER_BIT;
            b.w.gn[b.w.gidx[mc.A]] = e;
        } else {
            if (mc.co != NO_CELL) {
                atomicAdd(&b.dep[mc.co], 1u);
                b.w.gn[b.w.gidx[mc.A]].slot = DEPARTED;
            }
            if (mc.cn != NO_CELL) atomicAdd(&b.arr[mc.cn], 1u);
        }
    }
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
__global__ void __launch_bounds__(NT) k_place(TickBufs b) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    uint32_t A = 0;
    if (i < b.m && op_mover(b, i, A)) {
        const MoverCells mc = mover_cells(b.w, A);
        const bool cl = b.w.gate[mc.A] != 0;
        const bool pn = mc.cn != NO_CELL;
        MEnt e;
        e.x = pn ? mc.a.x : qnan(); e.z = pn ? mc.a.z : qnan();
        e.ox = mc.p.ox; e.oz = mc.p.oz;
        e.slot = mc.A; e.client = cl ? 1u : 0u; e.space = mc.a.meta & SPACE_MASK;
        if (mc.co != NO_CELL) {
            e.tags = TAG_OLD | (mc.cn == mc.co ? TAG_NEW | TAG_PRIMARY : 0u) | (pn ? 0u : TAG_PRIMARY);
            b.gm[b.gm_start[mc.co] + atomicSub(&b.gm_cnt[mc.co], 1u) - 1u] = e;
        }
        if (pn && mc.cn != mc.co) {
            e.tags = TAG_NEW | TAG_PRIMARY;
            b.gm[b.gm_start[mc.cn] + atomicSub(&b.gm_cnt[mc.cn], 1u) - 1u] = e;
            const uint32_t kept = (b.w.gn_start[mc.cn + 1] - b.w.gn_start[mc.cn]) - (b.dep[mc.cn] & ~CELL_DIRTY);
            const uint32_t at = b.start_nxt[mc.cn] + kept + atomicSub(&b.arr[mc.cn], 1u) - 1u;
            GEnt g;
            g.x = mc.a.x; g.z = mc.a.z; g.slot = mc.A;
            g.meta = mc.cn | (cl ? CLIENT_BIT : 0u) | MOVER_BIT;
            b.gn_nxt[at] = g;
        }
    }
}

// clean cells move as a block: new index = start_nxt + offset in the cell
__global__ void __launch_bounds__(NT) k_grid_copy(TickBufs b) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.w.gn_start[b.w.ncells]) return;
    const GEnt e = b.w.gn[i];
    if (e.slot == DEPARTED) return;
    const uint32_t c = e.meta & CELL_MASK;
    if (b.dep[c] & CELL_DIRTY) return;
    const uint32_t at = b.start_nxt[c] + (i - b.w.gn_start[c]);
    b.gn_nxt[at] = e;
    b.w.gidx[e.slot] = at;
}

// Dirty cells: the kept entries (already in slot order) merge with the
// arrivals (few, in arrival order at the cell's tail) by rank: a kept entry
// moves up by the arrivals with a smaller slot, an arrival lands after the
// kept entries and arrivals with a smaller slot.  A wave scans the flags of
// DIRTY_SPAN cells and merges its dirty ones; cells with more than 64
// arrivals go to the block path.
constexpr uint32_t DIRTY_SPAN = 16;
__global__ void __launch_bounds__(NT) k_grid_dirty(TickBufs b) {
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t c0 = (blockIdx.x * NWAVE + (threadIdx.x >> 6)) * DIRTY_SPAN;
    if (c0 >= b.w.ncells) return;
    const uint32_t cl = c0 + ln;
    uint64_t dm = wave_ballot(ln < (int)DIRTY_SPAN && cl < b.w.ncells && (b.dep[cl] & CELL_DIRTY));
    while (dm) {
        const uint32_t c = c0 + (uint32_t)__builtin_ctzll(dm);
        dm &= dm - 1;
        const uint32_t so = b.w.gn_start[c], old = b.w.gn_start[c + 1] - so;
        const uint32_t sn = b.start_nxt[c], nn = b.start_nxt[c + 1] - sn;
        const uint32_t kept = old - (b.dep[c] & ~CELL_DIRTY);
        const uint32_t narr = nn - kept;
        if (narr > 64) {
            if (ln == 0) b.bigcell[atomicAdd(&b.st->n_bigcell, 1ull)] = c;   // rare
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
                b.w.gidx[e.slot] = at;
            }
            k0 += (uint32_t)popc64(bm);
        }
        if (ln < (int)narr) {
            b.gn_nxt[sn + arank] = ar;
            b.w.gidx[ar.slot] = sn + arank;
        }
        if (ln == 0) b.dep[c] = 0;
    }
}

// dirty cells with more than 64 arrivals: block compaction + bitonic in place
__global__ void __launch_bounds__(NT) k_grid_bigcell(TickBufs b) {
    __shared__ uint32_t lds[NWAVE];
    const uint64_t nb = b.st->n_bigcell;
    for (uint64_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const uint32_t c = b.bigcell[k];
        const uint32_t so = b.w.gn_start[c], old = b.w.gn_start[c + 1] - so;
        const uint32_t sn = b.start_nxt[c], nn = b.start_nxt[c + 1] - sn;
        uint32_t run = 0;
        for (uint32_t base = 0; base < old; base += NT) {
            const uint32_t i = base + threadIdx.x;
            GEnt e;
            e.slot = DEPARTED;
            if (i < old) e = b.w.gn[so + i];
            const uint32_t keep = (i < old && e.slot != DEPARTED) ? 1u : 0u;
            uint32_t tot;
            const uint32_t pre = block_excl_scan<uint32_t>(keep, lds, tot);
            if (keep) b.gn_nxt[sn + run + pre] = e;
            run += tot;
        }
        __syncthreads();
        bitonic_inplace<NT>(b.gn_nxt + sn, nn, (int)threadIdx.x, [](const GEnt& e) { return e.slot; },
                            [] { __syncthreads(); });
        for (uint32_t j = threadIdx.x; j < nn; j += NT) b.w.gidx[b.gn_nxt[sn + j].slot] = sn + j;
        if (threadIdx.x == 0) b.dep[c] = 0;
        __syncthreads();
    }
}

void tick_grid(const TickBufs& b, ScanCtx& sc, hipStream_t s) {
    const uint32_t NC = b.w.ncells;
    hipLaunchKernelGGL(k_classify, dim3(nblk1(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_cellcnt, dim3(nblk1((uint64_t)NC + 1, NT)), dim3(NT), 0, s, b);
    // totals land in the low words of the (zeroed, little-endian) 64-bit counters
    scan_exclusive<uint32_t, uint32_t>(b.cnt_new, b.start_nxt, (uint64_t)NC + 1, nullptr, sc,
                                       (uint32_t*)&b.st->n_present, s);
    scan_exclusive<uint32_t, uint32_t>(b.gm_cnt, b.gm_start, (uint64_t)NC + 1, nullptr, sc,
                                       (uint32_t*)&b.st->n_gm, s);
    hipLaunchKernelGGL(k_place, dim3(nblk1(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_grid_copy, dim3(nblk1(b.w.cap, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_grid_dirty, dim3(nblk1((uint64_t)NC, DIRTY_SPAN * NWAVE)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_grid_bigcell, dim3(64), dim3(NT), 0, s, b);
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
// its cells) -> the size of its own-event region
__global__ void __launch_bounds__(NT) k_bounds(TickBufs b) {
    const uint64_t m = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (m >= b.st->n_gm) return;
    const MEnt e = b.gm[m];
    uint64_t c = 0;
    if (e.tags & TAG_PRIMARY) {
        const SpaceP P = b.w.sp[e.space];
        const Rects R = mover_rects(P, e.ox == e.ox, e.ox, e.oz, e.x == e.x, e.x, e.z);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (q >= R.n) break;
            const Rect rr = q == 0 ? R.r[0] : R.r[1];
            for (int cz = rr.z0; cz <= rr.z1; ++cz) {
                const uint32_t row = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
                c += b.w.gn_start[row + rr.x1 + 1] - b.w.gn_start[row + rr.x0];
                c += b.gm_start[row + rr.x1 + 1] - b.gm_start[row + rr.x0];
            }
        }
    }
    b.cand[m] = c;
}

void tick_movers(const TickBufs& b, ScanCtx& sc, hipStream_t s) {
    const uint64_t nmax = 2ull * b.m;
    const uint64_t* ngm = (const uint64_t*)&b.st->n_gm;
    hipLaunchKernelGGL(k_bounds, dim3(nblk1(nmax, NT)), dim3(NT), 0, s, b);
    scan_exclusive<uint64_t, uint64_t>(b.cand, b.reg, nmax, ngm, sc, (uint64_t*)&b.st->cand_total, s);
}

// ---------------------------------------------------------------------------
// diff: one wave per primary mover-grid entry (mover A): its own events.  For
// every candidate B in A's cells the old relation (pre-tick positions and
// stamps) and the new one are evaluated; r_old != r_new is an own event (A,B).
// Non-movers come from gn (old = new position), movers from the mover grid,
// where B's entry at its old cell stands for the pair when r_old holds and its
// entry at the new cell when only r_new does, so each pair is taken once.  The
// row ranges of both grids are walked flattened (Flat), DIFF_U chunks of 64
// candidates with their loads in flight together.  Events (B<<1 | leave) go to
// A's region and are sorted there: registers up to 64, LDS up to SORT_LDS,
// else a block sort later.  The events of the op-less B of such pairs come
// from k_opless (watcher side, the same float expressions evaluated from B),
// so this pass has no atomics.  The count of new
// neighbours with a client is kept for the collect.
struct Cand {
    float x, z, ox, oz;
    uint32_t slot;
    uint32_t info;       // tags | CAND_CLIENT | CAND_NONMOVER
};
constexpr uint32_t CAND_NONMOVER = 1u << 31;
constexpr uint32_t CAND_CLIENT = 1u << 30;

// WPB waves per block: a block keeps its LDS until its slowest wave ends, so
// small blocks keep more waves resident when hotspot movers run long
template <int DIFF_U, int WPB>
__global__ void __launch_bounds__(64 * WPB) k_mover(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[WPB * SORT_LDS];
    const uint64_t m = (uint64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    if (m >= b.st->n_gm) return;
    const MEnt me = b.gm[m];
    if (!(me.tags & TAG_PRIMARY)) return;
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const World& w = b.w;
    const uint64_t reg = b.reg[m], cap = b.cand[m];
    const uint32_t A = me.slot;
    if (reg + cap > b.own_cap) {                      // region past the buffers: the host redoes the diff
        if (ln == 0) {
            atomicOr(&b.st->overflow, 1ull);
            b.cnt64[A] = 0;
        }
        return;
    }
    const SpaceP P = w.sp[me.space];
    const float d = P.d;
    const bool pn = me.x == me.x, po = me.ox == me.ox;
    const unsigned long long sA = w.stamp[A], soA = w.prev[A].ostamp;
    const Rects R = mover_rects(P, po, me.ox, me.oz, pn, me.x, me.z);
    uint32_t* out = b.own + reg;
    uint32_t n = 0, nl = 0;
    uint32_t c_old = 0, c_new = 0, c_band = 0, c_cli = 0;
    Flat f = flat_build<2>(P, R, w.gn_start, b.gm_start);
    for (uint32_t base = 0; base < f.total; base += 64u * DIFF_U) {
        uint32_t idx[DIFF_U], kd[DIFF_U];
        flat_map<DIFF_U, 2>(f, base, idx, kd);
        Cand cc[DIFF_U];
#pragma unroll
        for (int u = 0; u < DIFF_U; ++u) {
            cc[u].info = 0;
            cc[u].slot = A;                                    // invalid unless loaded below
            if (idx[u] != ~0u) {
                if (kd[u] == 0) {
                    const GEnt e = w.gn[idx[u]];
                    cc[u].x = cc[u].ox = e.x;
                    cc[u].z = cc[u].oz = e.z;
                    cc[u].slot = (e.meta & MOVER_BIT) ? A : e.slot;   // movers come from gm
                    cc[u].info = TAG_OLD | TAG_NEW | (e.meta & CLIENT_BIT ? CAND_CLIENT : 0u) | CAND_NONMOVER;
                } else {
                    const MEnt e = b.gm[idx[u]];
                    cc[u].x = e.x; cc[u].z = e.z; cc[u].ox = e.ox; cc[u].oz = e.oz;
                    cc[u].slot = e.slot;
                    cc[u].info = e.tags | (e.client ? CAND_CLIENT : 0u);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < DIFF_U; ++u) {
            if (base + 64u * u >= f.total) break;              // wave-uniform
            const Cand& e = cc[u];
            bool ev = false, lv = false;
            uint32_t key = 0;
            if (e.slot != A) {
                const bool nmv = (e.info & CAND_NONMOVER) != 0;
                // A's view: A's windows around B's old / new position
                const bool iao = in_win(me.ox, me.oz, d, e.ox, e.oz), ibo = in_win(e.ox, e.oz, d, me.ox, me.oz);
                const bool ian = in_win(me.x, me.z, d, e.x, e.z), ibn = in_win(e.x, e.z, d, me.x, me.z);
                bool ro = iao, rn = ian;
                if (iao != ibo || ian != ibn) {
                    const unsigned long long sb = w.stamp[e.slot];
                    const unsigned long long sbo = nmv ? sb : w.prev[e.slot].ostamp;
                    if (iao != ibo) { ro = resolve(iao, ibo, soA, sbo); ++c_band; }
                    if (ian != ibn) { rn = resolve(ian, ibn, sA, sb); ++c_band; }
                }
                const bool take = ((e.info & TAG_OLD) && ro) || ((e.info & TAG_NEW) && rn && !ro);
                if (take) {
                    c_old += ro; c_new += rn;
                    c_cli += rn && (e.info & CAND_CLIENT) != 0;
                    ev = ro != rn;
                    lv = ro;
                    key = (e.slot << 1) | (lv ? 1u : 0u);
                }
            }
            const uint64_t be = wave_ballot(ev), bl = wave_ballot(ev && lv);
            const uint32_t at = n + (uint32_t)popc64(be & lt);
            if (ev && at < cap) out[at] = key;
            n += (uint32_t)popc64(be);
            nl += (uint32_t)popc64(bl);
        }
    }
    // sort the own events by (target, kind)
    if (n > 1) {
        if (n <= 64) {
            wave_sync();
            uint32_t v = ln < (int)n ? out[ln] : 0xffffffffu;
            v = wave_sort64(v);
            if (ln < (int)n) out[ln] = v;
        } else if (n <= SORT_LDS) {
            uint32_t* L = lds + (threadIdx.x >> 6) * SORT_LDS;
            wave_sync();
            for (uint32_t i = ln; i < n; i += 64) L[i] = out[i];
            wave_sync();
            bitonic_inplace<64>(L, n, ln, [](uint32_t v) { return v; }, [] { wave_sync(); });
            for (uint32_t i = ln; i < n; i += 64) out[i] = L[i];
        } else if (ln == 0) {
            b.big[atomicAdd(&b.st->n_big, 1ull)] = (uint32_t)m;
        }
    }
    const uint32_t so = wave_sum<uint32_t>(c_old), sn = wave_sum<uint32_t>(c_new), sb = wave_sum<uint32_t>(c_band);
    const uint32_t scl = wave_sum<uint32_t>(c_cli);
    if (ln == 0) {
        b.cnt64[A] = (unsigned long long)(n - nl) | ((unsigned long long)nl << 32);
        if (pn) w.nbc[A] = ((unsigned long long)w.epoch << 32) | scl;
        shard_add(b.st, blockIdx.x, SH_AOLD, (unsigned long long)so | ((unsigned long long)sn << 32));
        shard_add(b.st, blockIdx.x, SH_BAND, sb);
    }
}

// block sort of a mover's own events too many for LDS
__global__ void __launch_bounds__(NT) k_big_own(TickBufs b) {
    const uint64_t nb = b.st->n_big;
    for (uint64_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const uint32_t m = b.big[k];
        const uint64_t c = b.cnt64[b.gm[m].slot];
        const uint32_t n = (uint32_t)(lo32(c) + hi32(c));
        bitonic_inplace<NT>(b.own + b.reg[m], n, (int)threadIdx.x, [](uint32_t v) { return v; },
                            [] { __syncthreads(); });
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// opless: the events of the op-less watchers, computed on the watcher side
// (no atomics, no scatter).  A wave takes 64 consecutive grid entries and
// groups its op-less watchers by grid row; for each group the movers (mover-
// grid entries) of the union of the watchers' search rectangles are staged in
// LDS sorted by slot, and every lane tests its watcher B against each of them
// in turn, so B's events come out in target order.  PASS 0 counts (packed
// enters | leaves << 32 into cnt64[B]), PASS 1 writes at the scanned offsets
// and clears the counter.  A group with more than OPL_CAP movers is handled in
// chunks; its watchers' segments are then re-sorted by the block sort.
constexpr uint32_t OPL_CAP = 256;

// ascending sort of one 64-bit key per lane across the wave (registers)
__device__ __forceinline__ uint64_t wave_sort64_u64(uint64_t v) {
    const int l = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t o = __shfl_xor(v, j, 64);
            const bool up = (l & k) == 0, lower = (l & j) == 0;
            const uint64_t mn = v < o ? v : o, mx = v < o ? o : v;
            v = (lower == up) ? mn : mx;
        }
    }
    return v;
}

template <int PASS>
__global__ void __launch_bounds__(64) k_opless(TickBufs b) {
    __shared__ __attribute__((aligned(16))) MEnt L[OPL_CAP];
    __shared__ uint64_t K[OPL_CAP];
    const World& w = b.w;
    const uint32_t np = w.gn_start[w.ncells];
    const uint32_t i0 = blockIdx.x * 64u;
    if (i0 >= np) return;
    const int ln = lane_id();
    // this lane's watcher
    const uint32_t gi = i0 + ln;
    GEnt e;
    e.x = e.z = 0.0f;
    e.slot = DEPARTED;
    e.meta = MOVER_BIT;
    if (gi < np) e = w.gn[gi];
    const bool valid = gi < np && !(e.meta & MOVER_BIT);
    uint32_t space = 0;
    if (valid) space = w.aoi[e.slot].meta & SPACE_MASK;
    const SpaceP P = w.sp[space];
    const uint32_t cell = e.meta & CELL_MASK;
    const uint32_t rowkey = valid ? cell - (cell - P.cell_base) % (uint32_t)P.W : 0xffffffffu;
    const Rect r = search_rect(P, e.x, e.z);
    unsigned long long sbv = 0;
    bool have_sb = false;
    uint32_t ne = 0, nl = 0;
    uint64_t off = 0;
    if (PASS == 1 && valid) off = b.off64[e.slot];
    bool chunked = false;
    uint64_t todo = wave_ballot(valid);
    while (todo) {
        // the group: lanes of the lowest remaining row
        const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)rowkey, __builtin_ctzll(todo));
        const bool mine = valid && rowkey == key;
        const uint64_t gmask = wave_ballot(mine);
        todo &= ~gmask;
        // the group's space and union rectangle
        const int lead = __builtin_ctzll(gmask);
        const uint32_t gsp = (uint32_t)__builtin_amdgcn_readlane((int)space, lead);
        const SpaceP G = w.sp[gsp];
        const float d = G.d;
        int x0 = mine ? r.x0 : INT_MAX, z0 = mine ? r.z0 : INT_MAX;
        int x1 = mine ? r.x1 : INT_MIN, z1 = mine ? r.z1 : INT_MIN;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            x0 = min(x0, __shfl_xor(x0, o, 64)); z0 = min(z0, __shfl_xor(z0, o, 64));
            x1 = max(x1, __shfl_xor(x1, o, 64)); z1 = max(z1, __shfl_xor(z1, o, 64));
        }
        Rects U;
        U.n = 1;
        U.r[0].x0 = x0; U.r[0].x1 = x1; U.r[0].z0 = z0; U.r[0].z1 = z1;
        Flat f = flat_build<1>(G, U, b.gm_start, nullptr);
        if (f.total > OPL_CAP) chunked = true;
        for (uint32_t cb = 0; cb < f.total; cb += OPL_CAP) {
            const uint32_t cn = min(OPL_CAP, f.total - cb);
            // the chunk's movers in slot order: registers for one lane-chunk,
            // else staged in LDS, sorted by (slot, index) and gathered back
            MEnt mv;
            mv.slot = 0xffffffffu;
            uint32_t nlc = 0;                              // lane-chunks of sorted movers
            if (cn <= 64) {
                uint32_t idx[1], kd[1];
                flat_map<1, 1>(f, cb, idx, kd);
                MEnt me;
                me.slot = 0xffffffffu;
                if (ln < (int)cn) me = b.gm[idx[0]];
                if (ln < (int)cn) L[ln] = me;
                const uint64_t k = ln < (int)cn ? (((uint64_t)me.slot << 32) | (uint32_t)ln) : ~0ull;
                const uint64_t sk = wave_sort64_u64(k);
                wave_sync();
                if (ln < (int)cn) mv = L[(uint32_t)sk];
                nlc = 1;
            } else {
                for (uint32_t j = 0; j < cn; j += 64) {
                    uint32_t idx[1], kd[1];
                    flat_map<1, 1>(f, cb + j, idx, kd);
                    if (j + ln < cn) {
                        const MEnt me = b.gm[idx[0]];
                        L[j + ln] = me;
                        K[j + ln] = ((uint64_t)me.slot << 32) | (j + ln);
                    }
                }
                wave_sync();
                bitonic_inplace<64>(K, cn, ln, [](uint64_t v) { return v; }, [] { wave_sync(); });
                nlc = (cn + 63) / 64;
            }
            for (uint32_t c = 0; c < nlc; ++c) {
                if (nlc > 1) {                             // gather the next 64 sorted movers into lanes
                    wave_sync();
                    mv.slot = 0xffffffffu;
                    if (c * 64 + ln < cn) mv = L[(uint32_t)K[c * 64 + ln]];
                }
                const uint32_t cnt = min(64u, cn - c * 64);
                // each mover broadcast to every lane of the group, in slot order
                for (uint32_t j = 0; j < cnt; ++j) {
                    const float mx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mv.x), (int)j));
                    const float mz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mv.z), (int)j));
                    const float mox = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mv.ox), (int)j));
                    const float moz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mv.oz), (int)j));
                    const uint32_t ms = (uint32_t)__builtin_amdgcn_readlane((int)mv.slot, (int)j);
                    const uint32_t mt = (uint32_t)__builtin_amdgcn_readlane((int)mv.tags, (int)j);
                    if (!mine) continue;
                    const bool iao = in_win(mox, moz, d, e.x, e.z), ibo = in_win(e.x, e.z, d, mox, moz);
                    const bool ian = in_win(mx, mz, d, e.x, e.z), ibn = in_win(e.x, e.z, d, mx, mz);
                    bool ro = iao, rn = ian;
                    if (iao != ibo || ian != ibn) {
                        if (!have_sb) { sbv = w.stamp[e.slot]; have_sb = true; }
                        if (iao != ibo) ro = resolve(iao, ibo, w.prev[ms].ostamp, sbv);
                        if (ian != ibn) rn = resolve(ian, ibn, w.stamp[ms], sbv);
                    }
                    const bool take = ((mt & TAG_OLD) && ro) || ((mt & TAG_NEW) && rn && !ro);
                    if (take && ro != rn) {
                        gw_event ev; ev.watcher = e.slot; ev.target = ms;
                        if (ro) {
                            if (PASS == 1) { uint64_t at = hi32(off) + nl; if (at < b.ev_cap) b.leave[at] = ev; }
                            ++nl;
                        } else {
                            if (PASS == 1) { uint64_t at = lo32(off) + ne; if (at < b.ev_cap) b.enter[at] = ev; }
                            ++ne;
                        }
                    }
                }
            }
            wave_sync();
        }
    }
    if (PASS == 0) {
        if (valid && (ne | nl)) b.cnt64[e.slot] = (unsigned long long)ne | ((unsigned long long)nl << 32);
    } else if (valid && (ne | nl)) {
        b.cnt64[e.slot] = 0;
        if (chunked && (ne > 1 || nl > 1)) b.bigseg[atomicAdd(&b.st->n_bigseg, 1ull)] = e.slot;   // rare
    }
}

// movers copy their sorted own events into the canonical arrays
__global__ void __launch_bounds__(NT) k_own_copy(TickBufs b) {
    const uint64_t m = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (m >= b.st->n_gm) return;
    const MEnt me = b.gm[m];
    if (!(me.tags & TAG_PRIMARY)) return;
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t A = me.slot;
    const uint64_t reg = b.reg[m], capm = b.cand[m];
    const uint64_t c = b.cnt64[A];
    const uint64_t off = b.off64[A];
    if (reg + capm > b.own_cap) return;               // overflowed region (k_mover): nothing was written
    const uint32_t n = (uint32_t)(lo32(c) + hi32(c));
    if (!n) return;
    const uint32_t* own = b.own + reg;
    uint32_t ie = 0, il = 0;
    for (uint32_t base = 0; base < n; base += 64) {
        const uint32_t j = base + ln;
        const bool v = j < n;
        const uint32_t key = v ? own[j] : 0u;
        const bool lv = v && (key & 1u), en = v && !(key & 1u);
        const uint64_t be = wave_ballot(en), bl = wave_ballot(lv);
        gw_event ev; ev.watcher = A; ev.target = key >> 1;
        if (en) { uint64_t at = lo32(off) + ie + popc64(be & lt); if (at < b.ev_cap) b.enter[at] = ev; }
        if (lv) { uint64_t at = hi32(off) + il + popc64(bl & lt); if (at < b.ev_cap) b.leave[at] = ev; }
        ie += (uint32_t)popc64(be);
        il += (uint32_t)popc64(bl);
    }
    if (ln == 0) b.cnt64[A] = 0;
}

// block sort of op-less segments assembled from several mover chunks (by target)
__global__ void __launch_bounds__(NT) k_big_seg(TickBufs b) {
    const uint64_t nb = b.st->n_bigseg;
    for (uint64_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const uint32_t B = b.bigseg[k];
        const uint64_t o0 = b.off64[B], o1 = b.off64[B + 1];
        auto key = [](const gw_event& e) { return e.target; };
        auto sy = [] { __syncthreads(); };
        const uint32_t ne = (uint32_t)(lo32(o1) - lo32(o0)), nl = (uint32_t)(hi32(o1) - hi32(o0));
        if (lo32(o0) + ne <= b.ev_cap) bitonic_inplace<NT>(b.enter + lo32(o0), ne, (int)threadIdx.x, key, sy);
        if (hi32(o0) + nl <= b.ev_cap) bitonic_inplace<NT>(b.leave + hi32(o0), nl, (int)threadIdx.x, key, sy);
        __syncthreads();
    }
}

void tick_diff(const TickBufs& b, hipStream_t s) {
    const uint64_t nmax = 2ull * b.m;
    switch (b.diff_u) {                    // GW_MOVER_WPB: waves per k_mover block
    case 2: hipLaunchKernelGGL((k_mover<2, 2>), dim3(nblk1(nmax, 2)), dim3(128), 0, s, b); break;
    case 4: hipLaunchKernelGGL((k_mover<2, 4>), dim3(nblk1(nmax, 4)), dim3(256), 0, s, b); break;
    default: hipLaunchKernelGGL((k_mover<2, 1>), dim3(nblk1(nmax, 1)), dim3(64), 0, s, b); break;
    }
    hipLaunchKernelGGL(k_big_own, dim3(64), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_opless<0>, dim3(nblk1(b.w.cap, 64)), dim3(64), 0, s, b);
}
void tick_events(const TickBufs& b, ScanCtx& sc, hipStream_t s) {
    const uint64_t nmax = 2ull * b.m;
    const uint32_t C = b.w.cap;
    scan_exclusive<uint64_t, uint64_t>((const uint64_t*)b.cnt64, b.off64, (uint64_t)C + 1, nullptr, sc,
                                       (uint64_t*)&b.st->ev_pk, s);
    hipLaunchKernelGGL(k_own_copy, dim3(nblk1(nmax, NWAVE)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_opless<1>, dim3(nblk1(C, 64)), dim3(64), 0, s, b);
    hipLaunchKernelGGL(k_big_seg, dim3(64), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// after the tick: per-op dedupe state of every op's slot back to -1 (thread
// i: op i); MOVER bits cleared at the movers' new grid entries (thread i:
// mover-grid entry i)
__global__ void __launch_bounds__(NT) k_tick_reset(TickBufs b) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i < b.m) {
        const uint32_t s = b.ops[i].slot;
        if (s < b.w.cap) {
            b.last_pos[s] = -1;
            b.last_aoi[s] = -1;
            b.last_leave[s] = -1;
        }
    }
    if (i < b.st->n_gm) {
        const MEnt e = b.gm[i];
        if (e.tags & TAG_NEW) b.w.gn[b.w.gidx[e.slot]].meta &= ~MOVER_BIT;
    }
}
void tick_reset(const TickBufs& b, hipStream_t s) {
    hipLaunchKernelGGL(k_tick_reset, dim3(nblk1(2ull * b.m, NT)), dim3(NT), 0, s, b);
}

}  // namespace gw
