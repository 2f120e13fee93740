// kernels.hip — hand-written gfx950 kernels of the per-tick AOI + sync path.
//
// Semantics follow the batched parity contract: per tick, a pair
// (A,B) with at least one AOI op is related iff the member c with the larger
// last-op seq has the other inside its window [fl(c.x-d), fl(c.x+d)] x
// [fl(c.z-d), fl(c.z+d)] (go-aoi xzlist Mark bounds), both
// at final positions.  Window bounds are float32 round-to-nearest; the file is
// compiled with -ffp-contract=off and without fast-math.
//
// All kernels are HBM/latency-bound integer+compare work; no MFMA.
#include "gw_internal.hpp"
#include "prim.hpp"

namespace gw {

static inline uint32_t nblk(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }
static inline uint32_t nblk1(uint64_t n, uint32_t per) { uint32_t b = nblk(n, per); return b ? b : 1; }

__device__ __forceinline__ int cellc(float v, float o, float inv, int lim) {
    float f = floorf((v - o) * inv);           // monotone in v
    f = fminf(fmaxf(f, 0.0f), (float)(lim - 1));
    return (int)f;
}

// search range: every b with inWin_A(b) or inWin_b(A) lies inside
// [x-d-m, x+d+m] with m >= 8 ulp of |x|+d (covers the rounding of fl(b+-d)).
__device__ __forceinline__ void search_cells(const SpaceP& P, float x, float z, int& cx0, int& cx1,
                                             int& cz0, int& cz1) {
    float d = P.d;
    float mx = (fabsf(x) + d) * 1e-6f + 1e-30f;
    float mz = (fabsf(z) + d) * 1e-6f + 1e-30f;
    cx0 = cellc((x - d) - mx, P.x0, P.inv_cs, P.W);
    cx1 = cellc((x + d) + mx, P.x0, P.inv_cs, P.W);
    cz0 = cellc((z - d) - mz, P.z0, P.inv_cs, P.H);
    cz1 = cellc((z + d) + mz, P.z0, P.inv_cs, P.H);
}

__device__ __forceinline__ bool in_box(float lox, float hix, float loz, float hiz, float ox, float oz) {
    return ox >= lox && ox <= hix && oz >= loz && oz <= hiz;
}

// relation of A (mover, seqA) and B (seqB, position ox,oz) per the seq rule.
__device__ __forceinline__ bool relation(int seqA, float ax, float az, float lox, float hix, float loz,
                                         float hiz, int seqB, float bx, float bz, float d) {
    if (seqA > seqB) return in_box(lox, hix, loz, hiz, bx, bz);
    float lx = bx - d, hx = bx + d, lz = bz - d, hz = bz + d;
    return in_box(lx, hx, lz, hz, ax, az);
}

__device__ __forceinline__ bool bsearch_u32(const uint32_t* a, uint32_t n, uint32_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo < n && a[lo] == key;
}
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* a, uint32_t n, uint32_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t ev_key(uint32_t w, uint32_t t, uint32_t kind, int sb) {
    return ((uint64_t)w << (sb + 1)) | ((uint64_t)t << 1) | kind;   // kind 0 = enter, 1 = leave
}

// ---------------------------------------------------------------------------
// ops: last-op dedupe per slot (seq = index in the tick's op stream)
__global__ void __launch_bounds__(NT) k_ops1(const gw_op* __restrict__ ops, uint32_t m, uint32_t cap,
                                             int32_t* last_pos, int32_t* last_aoi, int32_t* last_leave,
                                             DevStats* st) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= m) return;
    gw_op op = ops[i];
    if (op.slot >= cap || op.kind < GW_OP_ENTER || op.kind > GW_OP_SYNC) {
        atomicAdd(&st->bad_ops, 1ull);
        return;
    }
    if (op.kind != GW_OP_LEAVE) atomicMax(&last_pos[op.slot], (int32_t)i);
    if (op.kind != GW_OP_SYNC) atomicMax(&last_aoi[op.slot], (int32_t)i);
    if (op.kind == GW_OP_LEAVE) atomicMax(&last_leave[op.slot], (int32_t)i);
}

// a Leave clears syncInfoFlag (the entity leaves this space's sync set)
__global__ void __launch_bounds__(NT) k_ops2(const gw_op* __restrict__ ops, uint32_t m, uint32_t cap,
                                             const int32_t* last_leave, uint32_t* flags) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= m) return;
    gw_op op = ops[i];
    if (op.slot >= cap || op.kind != GW_OP_LEAVE) return;
    if (last_leave[op.slot] == (int32_t)i) flags[op.slot] = 0;
}

__global__ void __launch_bounds__(NT) k_ops3(const gw_op* __restrict__ ops, uint32_t m, uint32_t cap,
                                             const int32_t* last_pos, const int32_t* last_aoi,
                                             const int32_t* last_leave, uint32_t* flags, float4* pos,
                                             AoiEnt* aoi, uint32_t* is_last) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= m) return;
    gw_op op = ops[i];
    uint32_t last = 0;
    if (op.slot < cap && op.kind >= GW_OP_ENTER && op.kind <= GW_OP_SYNC) {
        uint32_t s = op.slot;
        // syncInfoFlag |= bits of every call after the last Leave (Space.go:196,
        // Entity.go:1199-1204, 1286)
        if ((int32_t)i > last_leave[s] && op.sync_flags) atomicOr(&flags[s], (uint32_t)op.sync_flags);
        if (last_pos[s] == (int32_t)i) pos[s] = make_float4(op.x, op.y, op.z, op.yaw);
        if (last_aoi[s] == (int32_t)i) {
            AoiEnt a = aoi[s];
            a.seq = (int32_t)i;
            if (op.kind == GW_OP_LEAVE) a.meta &= ~PRESENT_BIT;
            else { a.x = op.x; a.z = op.z; a.meta |= PRESENT_BIT; }
            aoi[s] = a;
            last = 1;
        }
    }
    is_last[i] = last;
}

void launch_ops(const gw_op* ops, uint32_t m, uint32_t cap, int32_t* last_pos, int32_t* last_aoi,
                int32_t* last_leave, uint32_t* flags, float4* pos, AoiEnt* aoi, uint32_t* is_last,
                DevStats* st, hipStream_t s) {
    if (!m) return;
    hipLaunchKernelGGL(k_ops1, dim3(nblk(m, NT)), dim3(NT), 0, s, ops, m, cap, last_pos, last_aoi, last_leave, st);
    hipLaunchKernelGGL(k_ops2, dim3(nblk(m, NT)), dim3(NT), 0, s, ops, m, cap, last_leave, flags);
    hipLaunchKernelGGL(k_ops3, dim3(nblk(m, NT)), dim3(NT), 0, s, ops, m, cap, last_pos, last_aoi, last_leave,
                       flags, pos, aoi, is_last);
}

__global__ void __launch_bounds__(NT) k_compact_movers(const gw_op* __restrict__ ops, uint32_t m,
                                                       const uint32_t* is_last, const uint64_t* pre,
                                                       uint32_t* movers) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i < m && is_last[i]) movers[pre[i]] = ops[i].slot;
}
void launch_compact_movers(const gw_op* ops, uint32_t m, const uint32_t* is_last, const uint64_t* pre,
                           uint32_t* movers, hipStream_t s) {
    if (!m) return;
    hipLaunchKernelGGL(k_compact_movers, dim3(nblk(m, NT)), dim3(NT), 0, s, ops, m, is_last, pre, movers);
}

// ---------------------------------------------------------------------------
// uniform grid: cell key per slot (absent -> ncells, sorts last) + histogram
__global__ void __launch_bounds__(NT) k_cell_keys(const AoiEnt* __restrict__ aoi, const SpaceP* __restrict__ sp,
                                                  uint32_t cap, uint32_t ncells, uint32_t* keys, uint32_t* vals,
                                                  uint32_t* cell_cnt) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s >= cap) return;
    AoiEnt a = aoi[s];
    uint32_t key = ncells;
    if (a.meta & PRESENT_BIT) {
        SpaceP P = sp[a.meta & SPACE_MASK];
        int cx = cellc(a.x, P.x0, P.inv_cs, P.W);
        int cz = cellc(a.z, P.z0, P.inv_cs, P.H);
        key = P.cell_base + (uint32_t)cz * (uint32_t)P.W + (uint32_t)cx;
        atomicAdd(&cell_cnt[key], 1u);
    }
    keys[s] = key;
    vals[s] = s;
}
void launch_cell_keys(const AoiEnt* aoi, const SpaceP* sp, uint32_t cap, uint32_t ncells, uint32_t* keys,
                      uint32_t* vals, uint32_t* cell_cnt, hipStream_t s) {
    hipLaunchKernelGGL(k_cell_keys, dim3(nblk1(cap, NT)), dim3(NT), 0, s, aoi, sp, cap, ncells, keys, vals, cell_cnt);
}

__global__ void __launch_bounds__(NT) k_gather_sorted(const uint32_t* __restrict__ vals, const AoiEnt* __restrict__ aoi,
                                                      const uint32_t* n_present_dev, uint32_t cap, SortEnt* se,
                                                      DevStats* st) {
    uint32_t p = blockIdx.x * NT + threadIdx.x;
    if (p == 0) st->n_present = *n_present_dev;
    if (p >= cap || p >= *n_present_dev) return;
    uint32_t s = vals[p];
    AoiEnt a = aoi[s];
    SortEnt e;
    e.x = a.x; e.z = a.z; e.slot = s; e.seq = a.seq;
    se[p] = e;
}
void launch_gather_sorted(const uint32_t* vals, const AoiEnt* aoi, const uint32_t* n_present_dev, uint32_t cap,
                          SortEnt* se, DevStats* st, hipStream_t s) {
    hipLaunchKernelGGL(k_gather_sorted, dim3(nblk1(cap, NT)), dim3(NT), 0, s, vals, aoi, n_present_dev, cap, se, st);
}

// ---------------------------------------------------------------------------
// per-mover upper bound of emitted events: 2*(candidates + |old list|)
__global__ void __launch_bounds__(NT) k_bounds(const uint32_t* __restrict__ movers, const uint64_t* n_movers_dev,
                                               uint32_t m_max, const AoiEnt* __restrict__ aoi,
                                               const SpaceP* __restrict__ sp, const uint32_t* __restrict__ cell_start,
                                               const uint32_t* __restrict__ lst_cnt, DevStats* st) {
    uint64_t nm = load_n(m_max, n_movers_dev);
    uint64_t m = (uint64_t)blockIdx.x * NT + threadIdx.x;
    uint64_t bound = 0, ko = 0;
    if (m < nm) {
        uint32_t A = movers[m];
        AoiEnt a = aoi[A];
        ko = lst_cnt[A];
        uint64_t c = 0;
        if (a.meta & PRESENT_BIT) {
            SpaceP P = sp[a.meta & SPACE_MASK];
            int cx0, cx1, cz0, cz1;
            search_cells(P, a.x, a.z, cx0, cx1, cz0, cz1);
            for (int cz = cz0; cz <= cz1; ++cz) {
                uint32_t row = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
                c += cell_start[row + cx1 + 1] - cell_start[row + cx0];
            }
        }
        bound = 2 * (c + ko);
    }
    bound = wave_sum(bound);
    ko = wave_sum(ko);
    if (lane_id() == 0 && bound) {
        atomicAdd(&st->bound_total, (unsigned long long)bound);
        atomicAdd(&st->a_old, (unsigned long long)ko);
    }
}
void launch_bounds(const uint32_t* movers, const uint64_t* n_movers_dev, uint32_t m_max, const AoiEnt* aoi,
                   const SpaceP* sp, const uint32_t* cell_start, const uint32_t* lst_cnt, DevStats* st,
                   hipStream_t s) {
    if (!m_max) return;
    hipLaunchKernelGGL(k_bounds, dim3(nblk(m_max, NT)), dim3(NT), 0, s, movers, n_movers_dev, m_max, aoi, sp,
                       cell_start, lst_cnt, st);
}

// ---------------------------------------------------------------------------
// diff: one wave per mover A.
//   (i)  every grid candidate b in A's widened window: related(A,b) and
//        b not in old(A)  ->  enter(A,b) [+ enter(b,A) if b has no op]
//   (ii) every b in old(A): not related (or absent)  ->  leave(A,b) [+ mirror]
// Events are appended to a scratch buffer with one atomic per wave-iteration
// and canonicalised later by the radix sort.
__device__ __forceinline__ void emit2(bool e1, uint64_t k1, bool e2, uint64_t k2, uint64_t* ev, uint64_t cap,
                                      DevStats* st, uint64_t lt) {
    uint64_t b1 = wave_ballot(e1), b2 = wave_ballot(e2);
    uint32_t tot = (uint32_t)(popc64(b1) + popc64(b2));
    if (!tot) return;
    unsigned long long base = 0;
    if (lane_id() == 0) base = atomicAdd(&st->ev_count, (unsigned long long)tot);
    base = __shfl(base, 0, 64);
    if (base + tot > cap) {
        if (lane_id() == 0) atomicAdd(&st->ev_overflow, 1ull);
        return;
    }
    uint64_t p = base + (uint64_t)popc64(b1 & lt) + (uint64_t)popc64(b2 & lt);
    if (e1) ev[p++] = k1;
    if (e2) ev[p] = k2;
}

__global__ void __launch_bounds__(NT) k_diff(const uint32_t* __restrict__ movers, const uint64_t* n_movers_dev,
                                             uint32_t m_max, const AoiEnt* __restrict__ aoi,
                                             const SpaceP* __restrict__ sp, const uint32_t* __restrict__ cell_start,
                                             const SortEnt* __restrict__ se, const uint32_t* __restrict__ lst_off,
                                             const uint32_t* __restrict__ lst_cnt, const uint32_t* __restrict__ pool,
                                             uint64_t* ev, uint64_t ev_cap, int sb, DevStats* st) {
    const int ln = lane_id();
    uint64_t nm = load_n(m_max, n_movers_dev);
    uint64_t mi = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (mi >= nm) return;                                   // wave-uniform
    const uint64_t lt = lanemask_lt();
    const uint32_t A = movers[mi];
    const AoiEnt a = aoi[A];
    const bool presA = (a.meta & PRESENT_BIT) != 0;
    const SpaceP P = sp[a.meta & SPACE_MASK];
    const float d = P.d;
    const float lox = a.x - d, hix = a.x + d, loz = a.z - d, hiz = a.z + d;   // fl(x-d), fl(x+d)
    const uint32_t ko = lst_cnt[A];
    const uint32_t* old = pool + lst_off[A];
    const int seqA = a.seq;
    uint64_t tested = 0;
    if (presA) {
        int cx0, cx1, cz0, cz1;
        search_cells(P, a.x, a.z, cx0, cx1, cz0, cz1);
        for (int cz = cz0; cz <= cz1; ++cz) {
            uint32_t row = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
            uint32_t p0 = cell_start[row + cx0], p1 = cell_start[row + cx1 + 1];
            tested += p1 - p0;
            for (uint32_t base = p0; base < p1; base += 64) {
                uint32_t p = base + ln;
                bool ent = false, mir = false;
                uint32_t b = 0;
                if (p < p1) {
                    SortEnt e = se[p];
                    b = e.slot;
                    if (b != A && relation(seqA, a.x, a.z, lox, hix, loz, hiz, e.seq, e.x, e.z, d)) {
                        ent = !bsearch_u32(old, ko, b);
                        mir = ent && e.seq < 0;
                    }
                }
                emit2(ent, ev_key(A, b, 0, sb), mir, ev_key(b, A, 0, sb), ev, ev_cap, st, lt);
            }
        }
    }
    for (uint32_t base = 0; base < ko; base += 64) {
        uint32_t j = base + ln;
        bool lv = false, mir = false;
        uint32_t b = 0;
        if (j < ko) {
            b = old[j];
            AoiEnt eb = aoi[b];
            bool rel = presA && (eb.meta & PRESENT_BIT) &&
                       relation(seqA, a.x, a.z, lox, hix, loz, hiz, eb.seq, eb.x, eb.z, d);
            lv = !rel;
            mir = lv && eb.seq < 0;
        }
        emit2(lv, ev_key(A, b, 1, sb), mir, ev_key(b, A, 1, sb), ev, ev_cap, st, lt);
    }
    if (ln == 0 && tested) atomicAdd(&st->pairs_tested, (unsigned long long)tested);
}

void launch_diff(const uint32_t* movers, const uint64_t* n_movers_dev, uint32_t m_max, const AoiEnt* aoi,
                 const SpaceP* sp, const uint32_t* cell_start, const SortEnt* se, const uint32_t* lst_off,
                 const uint32_t* lst_cnt, const uint32_t* pool, uint64_t* ev, uint64_t ev_cap, int sb,
                 DevStats* st, hipStream_t s) {
    if (!m_max) return;
    hipLaunchKernelGGL(k_diff, dim3(nblk(m_max, NWAVE)), dim3(NT), 0, s, movers, n_movers_dev, m_max, aoi, sp,
                       cell_start, se, lst_off, lst_cnt, pool, ev, ev_cap, sb, st);
}

// ---------------------------------------------------------------------------
// sorted events -> packed flags (enter | segment-head<<32)
__global__ void __launch_bounds__(NT) k_ev_flags(const uint64_t* __restrict__ ev, const uint64_t* n_ev_dev,
                                                 uint64_t n_max, int sb, uint64_t* packed) {
    uint64_t n = load_n(n_max, n_ev_dev);
    uint64_t p = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (p >= n) return;
    uint64_t k = ev[p];
    uint64_t w = k >> (sb + 1);
    uint64_t head = (p == 0) || ((ev[p - 1] >> (sb + 1)) != w);
    packed[p] = (uint64_t)((k & 1) == 0) | (head << 32);
}
void launch_ev_flags(const uint64_t* ev, const uint64_t* n_ev_dev, uint64_t n_max, int sb, uint64_t* packed,
                     hipStream_t s) {
    if (!n_max) return;
    hipLaunchKernelGGL(k_ev_flags, dim3(nblk(n_max, NT)), dim3(NT), 0, s, ev, n_ev_dev, n_max, sb, packed);
}

__global__ void __launch_bounds__(NT) k_ev_split(const uint64_t* __restrict__ ev, const uint64_t* n_ev_dev,
                                                 uint64_t n_max, int sb, const uint64_t* __restrict__ pex,
                                                 gw_event* enter, gw_event* leave, uint32_t* seg_start,
                                                 int write_events) {
    uint64_t n = load_n(n_max, n_ev_dev);
    uint64_t p = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (p >= n) return;
    uint64_t k = ev[p];
    uint32_t w = (uint32_t)(k >> (sb + 1));
    uint32_t t = (uint32_t)((k >> 1) & ((1ull << sb) - 1));
    uint64_t x = pex[p];
    uint32_t er = (uint32_t)x, sr = (uint32_t)(x >> 32);
    bool is_enter = (k & 1) == 0;
    bool head = (p == 0) || ((ev[p - 1] >> (sb + 1)) != (uint64_t)w);
    if (write_events) {
        gw_event e; e.watcher = w; e.target = t;
        if (is_enter) enter[er] = e; else leave[p - er] = e;
    }
    if (head) seg_start[sr] = (uint32_t)p;
    if (p == n - 1) seg_start[sr + (head ? 1 : 0)] = (uint32_t)n;
}
void launch_ev_split(const uint64_t* ev, const uint64_t* n_ev_dev, uint64_t n_max, int sb, const uint64_t* pex,
                     gw_event* enter, gw_event* leave, uint32_t* seg_start, int write_events, hipStream_t s) {
    if (!n_max) return;
    hipLaunchKernelGGL(k_ev_split, dim3(nblk(n_max, NT)), dim3(NT), 0, s, ev, n_ev_dev, n_max, sb, pex, enter,
                       leave, seg_start, write_events);
}

// ---------------------------------------------------------------------------
// list update: one wave per watcher segment; new list = merge(old - leaves,
// enters) written to a freshly bump-allocated pool range.
__device__ __forceinline__ uint32_t ev_target(uint64_t k, int sb) {
    return (uint32_t)((k >> 1) & ((1ull << sb) - 1));
}

__global__ void __launch_bounds__(NT) k_list_update(const uint64_t* __restrict__ ev, const uint64_t* __restrict__ pex,
                                                    const uint32_t* __restrict__ seg_start,
                                                    const unsigned long long* ev_scan_total, uint64_t seg_max,
                                                    int sb, const AoiEnt* __restrict__ aoi, uint32_t* lst_off,
                                                    uint32_t* lst_cnt, const uint32_t* pool_old, uint32_t* pool_new,
                                                    uint64_t pool_cap, DevStats* st) {
    const int ln = lane_id();
    const unsigned long long tot = *ev_scan_total;
    const uint64_t nseg = tot >> 32;
    const uint32_t tot_enter = (uint32_t)tot;
    uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (k >= nseg || k >= seg_max) return;
    const uint32_t s = seg_start[k], e = seg_start[k + 1];
    const uint64_t n_ev = seg_start[nseg];
    const uint32_t W = (uint32_t)(ev[s] >> (sb + 1));
    const uint32_t ko = lst_cnt[W];
    const uint32_t* old = pool_old + lst_off[W];
    const uint32_t er_s = (uint32_t)pex[s];
    const uint32_t er_e = (e < n_ev) ? (uint32_t)pex[e] : tot_enter;
    const uint32_t ne = er_e - er_s, nl = (e - s) - ne;
    const uint32_t nn = ko - nl + ne;
    unsigned long long off = 0;
    if (ln == 0) off = atomicAdd(&st->pool_top, (unsigned long long)nn);
    off = __shfl(off, 0, 64);
    if (off + nn > pool_cap) {
        if (ln == 0) atomicAdd(&st->pool_overflow, 1ull);
        return;
    }
    uint32_t* out = pool_new + off;
    // kept old entries
    for (uint32_t j = ln; j < ko; j += 64) {
        uint32_t o = old[j];
        uint32_t lo = s, hi = e;                       // lower_bound over segment targets
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (ev_target(ev[mid], sb) < o) lo = mid + 1; else hi = mid;
        }
        if (lo < e && ev_target(ev[lo], sb) == o) continue;    // a leave of o
        uint32_t eb = ((lo < n_ev) ? (uint32_t)pex[lo] : tot_enter) - er_s;
        uint32_t lb = (lo - s) - eb;
        uint32_t idx = j - lb + eb;
        if (idx < nn) out[idx] = o;
    }
    // enters
    for (uint32_t q = s + ln; q < e; q += 64) {
        uint64_t key = ev[q];
        if (key & 1) continue;
        uint32_t t = ev_target(key, sb);
        uint32_t pos_old = lower_bound_u32(old, ko, t);
        uint32_t eb = (uint32_t)pex[q] - er_s;
        uint32_t lb = (q - s) - eb;
        uint32_t idx = pos_old - lb + eb;
        if (idx < nn) out[idx] = t;
    }
    if (ln == 0) {
        lst_off[W] = (uint32_t)off;
        lst_cnt[W] = nn;
        if (aoi[W].seq >= 0) atomicAdd(&st->a_new, (unsigned long long)nn);
        atomicAdd(&st->total_entries, (unsigned long long)((int64_t)ne - (int64_t)nl));
    }
}
void launch_list_update(const uint64_t* ev, const uint64_t* pex, const uint32_t* seg_start,
                        const unsigned long long* ev_scan_total, uint64_t seg_max, int sb, const AoiEnt* aoi,
                        uint32_t* lst_off, uint32_t* lst_cnt, const uint32_t* pool_old, uint32_t* pool_new,
                        uint64_t pool_cap, DevStats* st, hipStream_t s) {
    if (!seg_max) return;
    hipLaunchKernelGGL(k_list_update, dim3(nblk(seg_max, NWAVE)), dim3(NT), 0, s, ev, pex, seg_start,
                       ev_scan_total, seg_max, sb, aoi, lst_off, lst_cnt, pool_old, pool_new, pool_cap, st);
}

__global__ void __launch_bounds__(NT) k_tick_reset(const gw_op* __restrict__ ops, uint32_t m, uint32_t cap,
                                                   int32_t* last_pos, int32_t* last_aoi, int32_t* last_leave,
                                                   AoiEnt* aoi) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= m) return;
    uint32_t s = ops[i].slot;
    if (s >= cap) return;
    last_pos[s] = -1; last_aoi[s] = -1; last_leave[s] = -1;
    aoi[s].seq = -1;
}
void launch_tick_reset(const gw_op* ops, uint32_t m, uint32_t cap, int32_t* last_pos, int32_t* last_aoi,
                       int32_t* last_leave, AoiEnt* aoi, hipStream_t s) {
    if (!m) return;
    hipLaunchKernelGGL(k_tick_reset, dim3(nblk(m, NT)), dim3(NT), 0, s, ops, m, cap, last_pos, last_aoi,
                       last_leave, aoi);
}

// pool compaction: one wave per slot copies its list to the packed offset
__global__ void __launch_bounds__(NT) k_pool_compact(const uint32_t* __restrict__ lst_off,
                                                     const uint32_t* __restrict__ lst_cnt,
                                                     const uint64_t* __restrict__ new_off, uint32_t cap,
                                                     const uint32_t* __restrict__ pool_old, uint32_t* pool_new,
                                                     uint32_t* lst_off_out) {
    uint64_t s = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (s >= cap) return;
    uint32_t n = lst_cnt[s];
    const uint32_t* src = pool_old + lst_off[s];
    uint32_t* dst = pool_new + new_off[s];
    for (uint32_t j = lane_id(); j < n; j += 64) dst[j] = src[j];
    if (lane_id() == 0) lst_off_out[s] = (uint32_t)new_off[s];
}
void launch_pool_compact(const uint32_t* lst_off, const uint32_t* lst_cnt, const uint64_t* new_off, uint32_t cap,
                         const uint32_t* pool_old, uint32_t* pool_new, uint32_t* lst_off_out, hipStream_t s) {
    hipLaunchKernelGGL(k_pool_compact, dim3(nblk1(cap, NWAVE)), dim3(NT), 0, s, lst_off, lst_cnt, new_off, cap,
                       pool_old, pool_new, lst_off_out);
}

__global__ void __launch_bounds__(NT) k_set_clients(const uint32_t* slots, const uint16_t* gates, uint32_t n,
                                                    uint32_t cap, uint16_t* gate) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i < n && slots[i] < cap) gate[slots[i]] = gates[i];
}
void launch_set_clients(const uint32_t* slots, const uint16_t* gates, uint32_t n, uint32_t cap, uint16_t* gate,
                        hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_set_clients, dim3(nblk(n, NT)), dim3(NT), 0, s, slots, gates, n, cap, gate);
}

// ---------------------------------------------------------------------------
// CollectEntitySyncInfos (Entity.go:1221-1267)
__global__ void __launch_bounds__(NT) k_flag_mark(const uint32_t* __restrict__ flags, uint32_t cap, uint32_t* mark) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s < cap) mark[s] = flags[s] != 0;
}
void launch_flag_mark(const uint32_t* flags, uint32_t cap, uint32_t* mark, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_mark, dim3(nblk1(cap, NT)), dim3(NT), 0, s, flags, cap, mark);
}
__global__ void __launch_bounds__(NT) k_flag_compact(const uint32_t* __restrict__ mark, const uint64_t* __restrict__ pre,
                                                     uint32_t cap, uint32_t* flagged) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s < cap && mark[s]) flagged[pre[s]] = s;
}
void launch_flag_compact(const uint32_t* mark, const uint64_t* pre, uint32_t cap, uint32_t* flagged, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_compact, dim3(nblk1(cap, NT)), dim3(NT), 0, s, mark, pre, cap, flagged);
}

// records per flagged entity e: own (bit0 and e has a client) + one per
// neighbour n in e.InterestedBy with a client (bit1)
__global__ void __launch_bounds__(NT) k_sync_count(const uint32_t* __restrict__ flagged, const uint64_t* nf_dev,
                                                   uint32_t nf_max, const uint32_t* __restrict__ flags,
                                                   const AoiEnt* __restrict__ aoi, const uint16_t* __restrict__ gate,
                                                   const uint32_t* __restrict__ lst_off,
                                                   const uint32_t* __restrict__ lst_cnt,
                                                   const uint32_t* __restrict__ pool, uint32_t* cnt) {
    uint64_t nf = load_n(nf_max, nf_dev);
    uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (k >= nf) return;
    uint32_t e = flagged[k];
    uint32_t f = flags[e];
    uint32_t r = 0;
    if (aoi[e].meta & PRESENT_BIT) {
        if (f & GW_SIF_NEIGHBOR_CLIENTS) {
            uint32_t n = lst_cnt[e];
            const uint32_t* L = pool + lst_off[e];
            for (uint32_t j = lane_id(); j < n; j += 64) r += gate[L[j]] != 0;
            r = wave_sum(r);
        }
        if ((f & GW_SIF_OWN_CLIENT) && gate[e]) r += 1;
    }
    if (lane_id() == 0) cnt[k] = r;
}
void launch_sync_count(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, const uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const uint32_t* lst_off, const uint32_t* lst_cnt,
                       const uint32_t* pool, uint32_t* cnt, hipStream_t s) {
    if (!nf_max) return;
    hipLaunchKernelGGL(k_sync_count, dim3(nblk(nf_max, NWAVE)), dim3(NT), 0, s, flagged, nf_dev, nf_max, flags, aoi,
                       gate, lst_off, lst_cnt, pool, cnt);
}

// writes e's records in (entity, watcher) order; the own record sits at the
// rank of e among e's client-holding neighbours.  Clears the flag.
__global__ void __launch_bounds__(NT) k_sync_write(const uint32_t* __restrict__ flagged, const uint64_t* nf_dev,
                                                   uint32_t nf_max, uint32_t* flags, const AoiEnt* __restrict__ aoi,
                                                   const uint16_t* __restrict__ gate,
                                                   const uint32_t* __restrict__ lst_off,
                                                   const uint32_t* __restrict__ lst_cnt,
                                                   const uint32_t* __restrict__ pool, const float4* __restrict__ pos,
                                                   const uint64_t* __restrict__ rec_off, gw_sync_record* rec,
                                                   uint64_t rec_cap) {
    const int ln = lane_id();
    uint64_t nf = load_n(nf_max, nf_dev);
    uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (k >= nf) return;
    const uint64_t lt = lanemask_lt();
    uint32_t e = flagged[k];
    uint32_t f = flags[e];
    if (aoi[e].meta & PRESENT_BIT) {
        float4 p = pos[e];
        bool own = (f & GW_SIF_OWN_CLIENT) && gate[e];
        uint64_t base = rec_off[k];
        uint32_t run = 0, below = 0;
        if (f & GW_SIF_NEIGHBOR_CLIENTS) {
            uint32_t n = lst_cnt[e];
            const uint32_t* L = pool + lst_off[e];
            for (uint32_t j0 = 0; j0 < n; j0 += 64) {
                uint32_t j = j0 + ln;
                uint32_t w = 0;
                bool has = false;
                if (j < n) { w = L[j]; has = gate[w] != 0; }
                uint64_t bh = wave_ballot(has);
                uint64_t bl = wave_ballot(has && w < e);
                if (has) {
                    uint64_t idx = base + run + (uint64_t)popc64(bh & lt) + ((own && w > e) ? 1 : 0);
                    gw_sync_record r;
                    r.watcher = w; r.entity = e; r.x = p.x; r.y = p.y; r.z = p.z; r.yaw = p.w;
                    if (idx < rec_cap) rec[idx] = r;
                }
                run += (uint32_t)popc64(bh);
                below += (uint32_t)popc64(bl);
            }
        }
        if (own && ln == 0) {
            gw_sync_record r;
            r.watcher = e; r.entity = e; r.x = p.x; r.y = p.y; r.z = p.z; r.yaw = p.w;
            if (base + below < rec_cap) rec[base + below] = r;
        }
    }
    if (ln == 0) flags[e] = 0;
}
void launch_sync_write(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const uint32_t* lst_off, const uint32_t* lst_cnt,
                       const uint32_t* pool, const float4* pos, const uint64_t* rec_off, gw_sync_record* rec,
                       uint64_t rec_cap, hipStream_t s) {
    if (!nf_max) return;
    hipLaunchKernelGGL(k_sync_write, dim3(nblk(nf_max, NWAVE)), dim3(NT), 0, s, flagged, nf_dev, nf_max, flags, aoi,
                       gate, lst_off, lst_cnt, pool, pos, rec_off, rec, rec_cap);
}

// per-gate record histogram: LDS buckets for gates < 256, global atomics above
__global__ void __launch_bounds__(NT) k_gate_hist(const gw_sync_record* __restrict__ rec, const uint64_t* n_dev,
                                                  uint64_t n_max, const uint16_t* __restrict__ gate, uint32_t* hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    uint64_t n = load_n(n_max, n_dev);
    for (uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x; r < n; r += (uint64_t)gridDim.x * NT) {
        uint32_t g = gate[rec[r].watcher];
        if (g < 256) atomicAdd(&h[g], 1u); else atomicAdd(&hist[g], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
void launch_gate_hist(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* hist, hipStream_t s) {
    uint32_t nb = nblk1(n_max, NT * 16);
    if (nb > 2048) nb = 2048;
    hipLaunchKernelGGL(k_gate_hist, dim3(nb), dim3(NT), 0, s, rec, n_dev, n_max, gate, hist);
}
__global__ void __launch_bounds__(NT) k_gate_keys(const gw_sync_record* __restrict__ rec, const uint64_t* n_dev,
                                                  uint64_t n_max, const uint16_t* __restrict__ gate, uint32_t* keys,
                                                  uint32_t* vals) {
    uint64_t n = load_n(n_max, n_dev);
    uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r >= n) return;
    keys[r] = gate[rec[r].watcher];
    vals[r] = (uint32_t)r;
}
void launch_gate_keys(const gw_sync_record* rec, const uint64_t* n_dev, uint64_t n_max, const uint16_t* gate,
                      uint32_t* keys, uint32_t* vals, hipStream_t s) {
    if (!n_max) return;
    hipLaunchKernelGGL(k_gate_keys, dim3(nblk(n_max, NT)), dim3(NT), 0, s, rec, n_dev, n_max, gate, keys, vals);
}
__global__ void __launch_bounds__(NT) k_gather_records(const gw_sync_record* __restrict__ in,
                                                       const uint32_t* __restrict__ idx, const uint64_t* n_dev,
                                                       uint64_t n_max, gw_sync_record* out) {
    uint64_t n = load_n(n_max, n_dev);
    uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r < n) out[r] = in[idx[r]];
}
void launch_gather_records(const gw_sync_record* in, const uint32_t* idx, const uint64_t* n_dev, uint64_t n_max,
                           gw_sync_record* out, hipStream_t s) {
    if (!n_max) return;
    hipLaunchKernelGGL(k_gather_records, dim3(nblk(n_max, NT)), dim3(NT), 0, s, in, idx, n_dev, n_max, out);
}

__global__ void k_fill_u32(uint32_t* p, uint32_t v, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_fill_i32(int32_t* p, int32_t v, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i < n) p[i] = v;
}
void launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fill_u32, dim3(nblk(n, NT)), dim3(NT), 0, s, p, v, n);
}
void launch_fill_i32(int32_t* p, int32_t v, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fill_i32, dim3(nblk(n, NT)), dim3(NT), 0, s, p, v, n);
}

// ---------------------------------------------------------------------------
// primitive instantiations for the host code
uint64_t radix_tile() { return RS_TILE; }
uint64_t scan_tile() { return SCAN_TILE; }
void scan_u32_u32(const uint32_t* in, uint32_t* out, uint64_t n_max, const uint64_t* n_dev, uint32_t* tmp,
                  uint32_t* total, hipStream_t s) {
    scan_exclusive<uint32_t, uint32_t>(in, out, n_max, n_dev, tmp, total, s);
}
void scan_u32_u64(const uint32_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, uint64_t* tmp,
                  uint64_t* total, hipStream_t s) {
    scan_exclusive<uint32_t, uint64_t>(in, out, n_max, n_dev, tmp, total, s);
}
void scan_u64_u64(const uint64_t* in, uint64_t* out, uint64_t n_max, const uint64_t* n_dev, uint64_t* tmp,
                  uint64_t* total, hipStream_t s) {
    scan_exclusive<uint64_t, uint64_t>(in, out, n_max, n_dev, tmp, total, s);
}
int sort_u32_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n_max, const uint64_t* n_dev,
                 int lo_bit, int hi_bit, const RadixTmp& tmp, hipStream_t s) {
    return radix_sort<uint32_t>(k0, v0, k1, v1, n_max, n_dev, lo_bit, hi_bit, tmp, s);
}
int sort_u64(uint64_t* k0, uint64_t* k1, uint64_t n_max, const uint64_t* n_dev, int lo_bit, int hi_bit,
             const RadixTmp& tmp, hipStream_t s) {
    return radix_sort<uint64_t>(k0, nullptr, k1, nullptr, n_max, n_dev, lo_bit, hi_bit, tmp, s);
}

}  // namespace gw
