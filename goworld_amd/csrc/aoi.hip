// aoi.hip — gfx950 kernels of one AOI tick.
//
// The relation of a pair is a pure function of the current positions and of
// the global stamps of the members' last AOI ops (gw_internal.hpp, DESIGN.md
// §2), so the tick keeps no neighbour lists.  For one tick:
//   ops      last-op dedupe per slot; movers save their pre-tick position and
//            stamp (PrevEnt) and take a new stamp
//   grid     stable radix sort of (cell, slot) -> current grid gn[] in (cell,
//            slot) order + cell starts; movers in grid order, then leavers
//   gm       mover grid: each mover at its old and its new cell (counting sort)
//   diff     one wave per mover scans non-movers of gn and the mover grid over
//            the cells of its old and new windows, evaluates the old and the
//            new relation of every candidate and emits own events, sorted
//   mirror   the relation is symmetric, so an own event (A,B) of a mover with
//            an op-less B is also B's event (B,A): the mover counts it into
//            B's packed counter (the returned value is its rank in B's
//            segment) and keeps (B, A, rank) for the scatter
//   events   scan of the per-watcher counts -> canonical offsets; movers copy
//            their sorted events and scatter the mirror ones; op-less segments
//            are insertion-sorted by one thread each (block sort when long)
// Outputs are placed by scans; the atomics are histogram/cursor updates, one
// counter increment per mirror event (spread over watchers), per-shard
// statistics and the rare big-segment lists.  No MFMA: compare and
// gather work bound by L2/HBM latency and bandwidth.
#include "dev_common.hpp"

namespace gw {

constexpr uint32_t SORT_LDS = 1024;     // own events sorted in a wave's LDS up to this many
constexpr uint32_t INS_MAX = 16;        // op-less segments insertion-sorted up to this many

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
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    if (op.slot >= b.w.cap || op.kind < GW_OP_ENTER || op.kind > GW_OP_SYNC) return;
    const uint32_t s = op.slot;
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
        a.seq = (int32_t)i;
        if (op.kind == GW_OP_LEAVE) a.meta &= ~PRESENT_BIT;
        else { a.x = op.x; a.z = op.z; a.meta |= PRESENT_BIT; }
        b.w.aoi[s] = a;
    }
}

void tick_ops(const TickBufs& b, hipStream_t s) {
    if (!b.m) return;
    hipLaunchKernelGGL(k_ops1, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_ops2, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_ops3, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// current grid: stable LSD radix sort of (cell, slot) pairs (absent slots get
// the sentinel key ncells and sort last), so gn[] is in (cell, slot) order and
// every output that follows grid order is deterministic
__global__ void __launch_bounds__(NT) k_grid_keys(TickBufs b) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s >= b.w.cap) return;
    const AoiEnt a = b.w.aoi[s];
    uint32_t key = b.w.ncells;
    if (a.meta & PRESENT_BIT) key = cell_of(b.w.sp[a.meta & SPACE_MASK], a.x, a.z);
    b.k0[s] = key;
    b.v0[s] = s;
}
__global__ void __launch_bounds__(NT) k_grid_fill(World w, const uint32_t* __restrict__ keys,
                                                  const uint32_t* __restrict__ slots, uint32_t* pflag) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= w.cap) return;
    const uint32_t key = keys[i];
    uint32_t mv = 0;
    if (key < w.ncells) {
        const uint32_t s = slots[i];
        const AoiEnt a = w.aoi[s];
        GEnt e;
        e.x = a.x; e.z = a.z; e.slot = s;
        mv = a.seq >= 0;
        e.meta = (uint32_t)w.gate[s] | (mv ? MOVER_BIT : 0u);
        w.gn[i] = e;
        w.gidx[s] = i;
    }
    if (pflag) pflag[i] = mv;
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

int tick_grid(const TickBufs& b, RadixTmp& rt, int key_bits, hipStream_t s) {
    const uint32_t C = b.w.cap;
    hipLaunchKernelGGL(k_grid_keys, dim3(nblk1(C, NT)), dim3(NT), 0, s, b);
    int r = radix_sort<uint32_t>(b.k0, b.v0, b.k1, b.v1, C, nullptr, 0, key_bits, rt, s);
    const uint32_t* keys = r ? b.k1 : b.k0;
    const uint32_t* slots = r ? b.v1 : b.v0;
    hipLaunchKernelGGL(k_grid_fill, dim3(nblk1(C, NT)), dim3(NT), 0, s, b.w, keys, slots, b.pflag);
    hipLaunchKernelGGL(k_grid_starts, dim3(nblk1((uint64_t)b.w.ncells + 1, NT)), dim3(NT), 0, s, b.w, keys, b.st);
    return r;
}

// ---------------------------------------------------------------------------
// movers: present movers in grid order (windows of neighbouring movers overlap
// in L2), then the leavers
__global__ void __launch_bounds__(NT) k_compact_grid_movers(TickBufs b) {
    uint64_t p = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (p >= b.st->n_present) return;
    if (b.pflag[p]) b.movers[b.pre[p]] = b.w.gn[p].slot;
}
__global__ void __launch_bounds__(NT) k_leaver_flags(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    bool f = op.kind == GW_OP_LEAVE && op.slot < b.w.cap && b.last_aoi[op.slot] == (int32_t)i;
    b.pflag[i] = f;
}
__global__ void __launch_bounds__(NT) k_compact_leavers(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    if (b.pflag[i]) b.movers[b.st->movers_present + b.pre[i]] = b.ops[i].slot;
    if (i == 0) b.st->n_movers = b.st->movers_present + b.st->leavers;
}
__global__ void k_set_nmov(DevStats* st) { st->n_movers = st->movers_present + st->leavers; }

// mover grid: the cells of a mover's old and new positions
__device__ __forceinline__ void mover_cells(const World& w, uint32_t A, uint32_t& co, uint32_t& cn) {
    const AoiEnt a = w.aoi[A];
    const PrevEnt p = w.prev[A];
    const SpaceP P = w.sp[a.meta & SPACE_MASK];
    co = cn = 0xffffffffu;
    if (p.ox == p.ox) co = cell_of(P, p.ox, p.oz);
    if (a.meta & PRESENT_BIT) cn = cell_of(P, a.x, a.z);
}
__global__ void __launch_bounds__(NT) k_gm_count(TickBufs b) {
    uint64_t m = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (m >= b.st->n_movers) return;
    uint32_t co, cn;
    mover_cells(b.w, b.movers[m], co, cn);
    if (co != 0xffffffffu) atomicAdd(&b.gm_cnt[co], 1u);
    if (cn != 0xffffffffu && cn != co) atomicAdd(&b.gm_cnt[cn], 1u);
}
__global__ void __launch_bounds__(NT) k_gm_scatter(TickBufs b) {
    uint64_t m = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (m >= b.st->n_movers) return;
    const uint32_t A = b.movers[m];
    uint32_t co, cn;
    mover_cells(b.w, A, co, cn);
    const AoiEnt a = b.w.aoi[A];
    const PrevEnt p = b.w.prev[A];
    MEnt e;
    const bool pn = (a.meta & PRESENT_BIT) != 0;
    e.x = pn ? a.x : qnan(); e.z = pn ? a.z : qnan();
    e.ox = p.ox; e.oz = p.oz;
    e.slot = A; e.gate = b.w.gate[A]; e.pad1 = 0;
    if (co != 0xffffffffu) {
        e.tags = TAG_OLD | (cn == co ? TAG_NEW : 0u);
        b.gm[atomicAdd(&b.gm_cnt[co], 1u)] = e;
    }
    if (cn != 0xffffffffu && cn != co) {
        e.tags = TAG_NEW;
        b.gm[atomicAdd(&b.gm_cnt[cn], 1u)] = e;
    }
}

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

// candidate bound of each mover (entries of gn and gm in its cells) -> the
// size of its own-event region
__global__ void __launch_bounds__(NT) k_bounds(TickBufs b) {
    uint64_t m = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (m >= b.st->n_movers) return;
    const uint32_t A = b.movers[m];
    const AoiEnt a = b.w.aoi[A];
    const PrevEnt p = b.w.prev[A];
    const SpaceP P = b.w.sp[a.meta & SPACE_MASK];
    const Rects R = mover_rects(P, p.ox == p.ox, p.ox, p.oz, (a.meta & PRESENT_BIT) != 0, a.x, a.z);
    uint64_t c = 0;
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
    b.cand[m] = c;
}

void tick_movers(const TickBufs& b, ScanCtx& sc, hipStream_t s) {
    const uint32_t C = b.w.cap, NC = b.w.ncells;
    scan_exclusive<uint32_t, uint64_t>(b.pflag, b.pre, C, (const uint64_t*)&b.st->n_present, sc,
                                       (uint64_t*)&b.st->movers_present, s);
    hipLaunchKernelGGL(k_compact_grid_movers, dim3(nblk1(C, NT)), dim3(NT), 0, s, b);
    if (b.m) {
        hipLaunchKernelGGL(k_leaver_flags, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
        scan_exclusive<uint32_t, uint64_t>(b.pflag, b.pre, b.m, nullptr, sc, (uint64_t*)&b.st->leavers, s);
        hipLaunchKernelGGL(k_compact_leavers, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    } else {
        hipLaunchKernelGGL(k_set_nmov, dim3(1), dim3(1), 0, s, b.st);
    }
    const uint64_t* nm = (const uint64_t*)&b.st->n_movers;
    (void)hipMemsetAsync(b.gm_cnt, 0, ((size_t)NC + 1) * 4, s);
    if (b.m) hipLaunchKernelGGL(k_gm_count, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    scan_exclusive<uint32_t, uint32_t>(b.gm_cnt, b.gm_start, (uint64_t)NC + 1, nullptr, sc, (uint32_t*)nullptr, s);
    (void)hipMemcpyAsync(b.gm_cnt, b.gm_start, ((size_t)NC + 1) * 4, hipMemcpyDeviceToDevice, s);
    if (b.m) {
        hipLaunchKernelGGL(k_gm_scatter, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
        hipLaunchKernelGGL(k_bounds, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
        scan_exclusive<uint64_t, uint64_t>(b.cand, b.reg, b.m, nm, sc, (uint64_t*)&b.st->cand_total, s);
    }
}

// ---------------------------------------------------------------------------
// diff: one wave per mover A.  For every candidate B in A's cells the old
// relation (pre-tick positions and stamps) and the new one are evaluated;
// r_old != r_new is an own event (A,B).  Non-movers come from gn (old = new
// position), movers from the mover grid, where B's entry at its old cell
// stands for the pair when r_old holds and its entry at the new cell when only
// r_new does, so each pair is taken once.  The row ranges of both grids are
// walked flattened (Flat), DIFF_U chunks of 64 candidates with their loads in
// flight together.  Events (B<<1 | leave) go to A's region and are sorted
// there: registers up to 64, LDS up to SORT_LDS, else a block sort later.
// The count of new neighbours with a client is kept for the next collect.
constexpr int DIFF_U = 2;

struct Cand {
    float x, z, ox, oz;
    uint32_t slot;
    uint32_t info;       // tags | gate << 8 | CAND_NONMOVER
};
constexpr uint32_t CAND_NONMOVER = 1u << 31;

__global__ void __launch_bounds__(NT) k_mover(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[NWAVE * SORT_LDS];
    const uint64_t nm = b.st->n_movers;
    const uint64_t m = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (m >= nm) return;
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const World& w = b.w;
    const uint32_t A = b.movers[m];
    const AoiEnt a = w.aoi[A];
    const PrevEnt p = w.prev[A];
    const SpaceP P = w.sp[a.meta & SPACE_MASK];
    const float d = P.d;
    const bool pn = (a.meta & PRESENT_BIT) != 0, po = p.ox == p.ox;
    const float nx = pn ? a.x : qnan(), nz = pn ? a.z : qnan();
    const unsigned long long sA = w.stamp[A], soA = p.ostamp;
    const Win wo = win_of(p.ox, p.oz, d), wn = win_of(nx, nz, d);
    const Rects R = mover_rects(P, po, p.ox, p.oz, pn, nx, nz);
    uint32_t* out = b.own + b.reg[m];
    uint64_t* mir = b.mir + b.reg[m];
    uint32_t* mrk = b.mir_rank + b.reg[m];
    const uint64_t cap = b.cand[m];
    uint32_t n = 0, nl = 0, nm_ = 0;
    uint32_t c_old = 0, c_new = 0, c_band = 0, c_cli = 0;
    Flat f = flat_build<2>(P, R, w.gn_start, b.gm_start);
    const uint32_t tested = f.total;
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
                    cc[u].info = TAG_OLD | TAG_NEW | ((e.meta & GATE_MASK) << 8) | CAND_NONMOVER;
                } else {
                    const MEnt e = b.gm[idx[u]];
                    cc[u].x = e.x; cc[u].z = e.z; cc[u].ox = e.ox; cc[u].oz = e.oz;
                    cc[u].slot = e.slot;
                    cc[u].info = e.tags | (e.gate << 8);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < DIFF_U; ++u) {
            if (base + 64u * u >= f.total) break;              // wave-uniform
            const Cand& e = cc[u];
            bool ev = false, lv = false, nmv = false;
            uint32_t key = 0;
            if (e.slot != A) {
                nmv = (e.info & CAND_NONMOVER) != 0;
                const bool iao = wo.has(e.ox, e.oz), ibo = in_win(e.ox, e.oz, d, p.ox, p.oz);
                const bool ian = wn.has(e.x, e.z), ibn = in_win(e.x, e.z, d, nx, nz);
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
                    c_cli += rn && (e.info & (GATE_MASK << 8)) != 0;
                    ev = ro != rn;
                    lv = ro;
                    key = (e.slot << 1) | (lv ? 1u : 0u);
                }
            }
            const bool mev = ev && nmv;
            // B has no op: (B,A) is B's event too; its rank in B's segment
            uint32_t rank = 0;
            if (mev) {
                const unsigned long long o = atomicAdd(&b.cnt64[e.slot], lv ? (1ull << 32) : 1ull);
                rank = lv ? (uint32_t)hi32(o) : (uint32_t)lo32(o);
            }
            const uint64_t be = wave_ballot(ev), bl = wave_ballot(ev && lv), bm = wave_ballot(mev);
            const uint32_t at = n + (uint32_t)popc64(be & lt);
            if (ev && at < cap) out[at] = key;
            const uint32_t atm = nm_ + (uint32_t)popc64(bm & lt);
            if (mev && atm < cap) {
                mir[atm] = ((uint64_t)e.slot << 32) | (A << 1) | (lv ? 1u : 0u);
                mrk[atm] = rank;
            }
            n += (uint32_t)popc64(be);
            nl += (uint32_t)popc64(bl);
            nm_ += (uint32_t)popc64(bm);
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
        if (n) b.cnt64[A] = (unsigned long long)(n - nl) | ((unsigned long long)nl << 32);
        b.mir_cnt[m] = nm_;
        if (pn) w.nbc[A] = ((unsigned long long)w.epoch << 32) | scl;
        shard_add(b.st, A, SH_PAIRS, tested);
        shard_add(b.st, A, SH_AOLD, so);
        shard_add(b.st, A, SH_ANEW, sn);
        shard_add(b.st, A, SH_BAND, sb);
    }
}

// block sort of a mover's own events too many for LDS
__global__ void __launch_bounds__(NT) k_big_own(TickBufs b) {
    const uint64_t nb = b.st->n_big;
    for (uint64_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const uint32_t m = b.big[k];
        const uint64_t c = b.cnt64[b.movers[m]];
        const uint32_t n = (uint32_t)(lo32(c) + hi32(c));
        bitonic_inplace<NT>(b.own + b.reg[m], n, (int)threadIdx.x, [](uint32_t v) { return v; },
                            [] { __syncthreads(); });
        __syncthreads();
    }
}

void tick_diff(const TickBufs& b, uint64_t n_movers, hipStream_t s) {
    if (!n_movers) return;
    hipLaunchKernelGGL(k_mover, dim3(nblk(n_movers, NWAVE)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_big_own, dim3(64), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------

// movers copy their sorted own events into the canonical arrays and scatter
// their mirror events to the op-less watchers' segments (offset + rank)
__global__ void __launch_bounds__(NT) k_own_copy(TickBufs b) {
    const uint64_t nmv = b.st->n_movers;
    const uint64_t m = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (m >= nmv) return;
    const int ln = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t A = b.movers[m];
    const uint64_t c = b.cnt64[A];
    const uint32_t n = (uint32_t)(lo32(c) + hi32(c));
    const uint64_t reg = b.reg[m];
    if (n) {
        const uint64_t off = b.off64[A];
        const uint32_t* own = b.own + reg;
        uint32_t ie = 0, il = 0;
        for (uint32_t base = 0; base < n; base += 64) {
            const uint32_t j = base + ln;
            const bool v = j < n;
            const uint32_t key = v ? own[j] : 0;
            const bool lv = v && (key & 1u), en = v && !(key & 1u);
            const uint64_t be = wave_ballot(en), bl = wave_ballot(lv);
            gw_event ev; ev.watcher = A; ev.target = key >> 1;
            if (en) { uint64_t at = lo32(off) + ie + popc64(be & lt); if (at < b.enter_cap) b.enter[at] = ev; }
            if (lv) { uint64_t at = hi32(off) + il + popc64(bl & lt); if (at < b.leave_cap) b.leave[at] = ev; }
            ie += (uint32_t)popc64(be);
            il += (uint32_t)popc64(bl);
        }
    }
    const uint32_t nmr = b.mir_cnt[m];
    for (uint32_t j = ln; j < nmr; j += 64) {
        const uint64_t v = b.mir[reg + j];
        const uint32_t W = (uint32_t)hi32(v), al = (uint32_t)lo32(v);
        const uint64_t off = b.off64[W];
        gw_event ev; ev.watcher = W; ev.target = al >> 1;
        if (al & 1u) { uint64_t at = hi32(off) + b.mir_rank[reg + j]; if (at < b.leave_cap) b.leave[at] = ev; }
        else { uint64_t at = lo32(off) + b.mir_rank[reg + j]; if (at < b.enter_cap) b.enter[at] = ev; }
    }
}

// op-less watchers: order their segments by target (the ranks came from
// atomics): insertion sort by one thread up to INS_MAX entries, else the block
// sort; every watcher's counter is cleared for the next tick
__device__ __forceinline__ void ins_sort(gw_event* a, uint32_t n) {
    for (uint32_t i = 1; i < n; ++i) {
        const gw_event x = a[i];
        uint32_t j = i;
        while (j > 0 && a[j - 1].target > x.target) { a[j] = a[j - 1]; --j; }
        a[j] = x;
    }
}
__global__ void __launch_bounds__(NT) k_seg_fix(TickBufs b) {
    const uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s >= b.w.cap) return;
    const uint64_t o0 = b.off64[s], o1 = b.off64[s + 1];
    if (o0 == o1) return;
    b.cnt64[s] = 0;
    const uint32_t ne = (uint32_t)(lo32(o1) - lo32(o0)), nl = (uint32_t)(hi32(o1) - hi32(o0));
    if (ne < 2 && nl < 2) return;
    if (b.w.aoi[s].seq >= 0) return;                 // a mover: its own events are sorted
    if (ne > INS_MAX || nl > INS_MAX) {
        b.big[atomicAdd(&b.st->n_big, 1ull)] = s;
        return;
    }
    ins_sort(b.enter + lo32(o0), ne);
    ins_sort(b.leave + hi32(o0), nl);
}

__global__ void k_n_big_mark(DevStats* st) { st->scratch = st->n_big; }

void tick_events(const TickBufs& b, uint64_t n_movers, ScanCtx& sc, hipStream_t s) {
    const uint32_t C = b.w.cap;
    scan_exclusive<uint64_t, uint64_t>((const uint64_t*)b.cnt64, b.off64, (uint64_t)C + 1, nullptr, sc,
                                       (uint64_t*)&b.st->ev_pk, s);
    if (n_movers) hipLaunchKernelGGL(k_own_copy, dim3(nblk(n_movers, NWAVE)), dim3(NT), 0, s, b);
    // big-own entries sit in b.big[0, n_big); op-less ones are appended after
    hipLaunchKernelGGL(k_n_big_mark, dim3(1), dim3(1), 0, s, b.st);
    hipLaunchKernelGGL(k_seg_fix, dim3(nblk1(C, NT)), dim3(NT), 0, s, b);
}

// block sort of op-less segments longer than INS_MAX (by target); they follow
// the big-own entries in b.big, from the index kept in st->scratch
__global__ void __launch_bounds__(NT) k_big_seg_dev(TickBufs b) {
    const uint64_t first = b.st->scratch, nb = b.st->n_big;
    for (uint64_t k = first + blockIdx.x; k < nb; k += gridDim.x) {
        const uint32_t B = b.big[k];
        const uint64_t o0 = b.off64[B], o1 = b.off64[B + 1];
        auto key = [](const gw_event& e) { return e.target; };
        auto sy = [] { __syncthreads(); };
        bitonic_inplace<NT>(b.enter + lo32(o0), (uint32_t)(lo32(o1) - lo32(o0)), (int)threadIdx.x, key, sy);
        bitonic_inplace<NT>(b.leave + hi32(o0), (uint32_t)(hi32(o1) - hi32(o0)), (int)threadIdx.x, key, sy);
        __syncthreads();
    }
}
void tick_sort_big_segments(const TickBufs& b, hipStream_t s) {
    hipLaunchKernelGGL(k_big_seg_dev, dim3(64), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) k_tick_reset(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    uint32_t s = b.ops[i].slot;
    if (s >= b.w.cap) return;
    b.last_pos[s] = -1;
    b.last_aoi[s] = -1;
    b.last_leave[s] = -1;
    b.w.aoi[s].seq = -1;
}
void tick_reset(const TickBufs& b, uint64_t n_movers, hipStream_t s) {
    (void)n_movers;
    tick_sort_big_segments(b, s);
    if (b.m) hipLaunchKernelGGL(k_tick_reset, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
}

__global__ void __launch_bounds__(NT) k_stats_reduce(DevStats* st) {
    __shared__ unsigned long long l[NWAVE];
    unsigned long long tot[SH_FIELDS];
    for (int f = 0; f < SH_FIELDS; ++f) {
        unsigned long long v = st->shard[threadIdx.x][f], tt;
        block_excl_scan<unsigned long long>(v, l, tt);
        tot[f] = tt;
    }
    if (threadIdx.x == 0) {
        st->pairs_tested = tot[SH_PAIRS];
        st->a_old = tot[SH_AOLD];
        st->a_new = tot[SH_ANEW];
        st->band = tot[SH_BAND];
    }
}
void stats_reduce(DevStats* st, hipStream_t s) {
    static_assert(STAT_SHARDS == NT, "one thread per shard");
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(NT), 0, s, st);
}

}  // namespace gw
