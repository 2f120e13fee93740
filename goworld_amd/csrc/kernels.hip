// kernels.hip — hand-written gfx950 kernels of the per-tick AOI + sync path.
//
// Semantics follow the batched parity contract: per tick, a pair
// (A,B) with at least one AOI op is related iff the member c with the larger
// last-op seq has the other inside its window [fl(c.x-d), fl(c.x+d)] x
// [fl(c.z-d), fl(c.z+d)] (go-aoi xzlist Mark bounds), both
// at final positions.  Window bounds are float32 round-to-nearest; the file is
// compiled with -ffp-contract=off and without fast-math.
//
// Pipeline of one tick (launchers at the bottom, orchestration in capi.cpp):
//   ops       last-op dedupe per slot, state update
//   grid      cell histogram -> scan -> atomic-cursor scatter into SortEnt[]
//   movers    movers in cell order (+ leavers), per-mover bounds and tiers
//   diff      one wave (tier S) / workgroup (tiers B, C) per mover: candidate
//             window scan, membership in the old sorted list, bitonic sort of
//             the enters in LDS, merge into the other half of the list; own
//             events come out sorted; mirror events for op-less neighbours
//   events    scan of per-watcher counts -> canonical offsets; mirror events
//             counting-sorted by watcher; segment sorts; op-less neighbours'
//             lists merged
// No single-address atomic sits on the hot path: outputs are placed by scans,
// the neighbour pool only bump-allocates when a list outgrows its capacity.
// All kernels are integer/compare work bound by HBM/L2 latency; no MFMA.
#include "gw_internal.hpp"
#include "prim.hpp"

namespace gw {

static inline uint32_t nblk(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }
static inline uint32_t nblk1(uint64_t n, uint32_t per) { uint32_t b = nblk(n, per); return b ? b : 1; }
static inline uint32_t gstride(uint64_t n, uint32_t per) {   // grid of a grid-stride loop
    uint32_t b = nblk1(n, per);
    return b > 4096 ? 4096 : b;
}

constexpr uint32_t TS_ECAP = 512, TS_OCAP = 512;       // tier S: one wave per mover
constexpr uint32_t TB_ECAP = 4096, TB_OCAP = 4096;     // tier B: one workgroup per mover
constexpr uint32_t SEG_SMALL = 512;                    // op-less watcher segments sorted by one wave

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

// relation of mover A (seqA >= 0) and B per the seq rule.
__device__ __forceinline__ bool relation(int seqA, float ax, float az, float lox, float hix, float loz,
                                         float hiz, int seqB, float bx, float bz, float d) {
    if (seqA > seqB) return in_box(lox, hix, loz, hiz, bx, bz);
    float lx = bx - d, hx = bx + d, lz = bz - d, hz = bz + d;
    return in_box(lx, hx, lz, hz, ax, az);
}

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* a, uint32_t n, uint32_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ bool contains_u32(const uint32_t* a, uint32_t n, uint32_t key) {
    uint32_t i = lower_bound_u32(a, n, key);
    return i < n && a[i] == key;
}
__device__ __forceinline__ uint32_t lower_bound_ev(const gw_event* a, uint32_t n, uint32_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (a[mid].target < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint32_t next_pow2(uint32_t v) {
    if (v <= 1) return 1;
    return 1u << (32 - __clz(v - 1));
}
// list offsets are in units of 16 entries (64 B): lists start on cache lines and
// a u32 offset addresses 2^36 entries
__device__ __forceinline__ uint32_t* lptr(uint32_t* pool, uint32_t off) { return pool + ((uint64_t)off << 4); }
__device__ __forceinline__ const uint32_t* lptr(const uint32_t* pool, uint32_t off) {
    return pool + ((uint64_t)off << 4);
}
__device__ __forceinline__ uint32_t round16(uint64_t v) {
    v = (v + 15) & ~15ull;
    return (uint32_t)(v > 0x7ffffff0ull ? 0x7ffffff0ull : v);
}
__device__ __forceinline__ uint64_t lo32(uint64_t v) { return v & 0xffffffffull; }
__device__ __forceinline__ uint64_t hi32(uint64_t v) { return v >> 32; }

// ---------------------------------------------------------------------------
// Group = the threads working on one item: one wave (TPM 64) or a workgroup
// (TPM 256).  Waves of a TPM-64 kernel never wait for each other.
template <int TPM>
struct Grp {
    uint32_t* sl;   // 16 words of LDS scratch (TPM 256 only)
    __device__ __forceinline__ int tid() const { return TPM == 64 ? lane_id() : (int)threadIdx.x; }
    __device__ __forceinline__ void sync() const {
        if constexpr (TPM == 64) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            __syncthreads();
        }
    }
    // exclusive prefixes of two flags over the group, in thread order
    __device__ __forceinline__ void excl2(bool f1, bool f2, uint32_t& p1, uint32_t& p2, uint32_t& t1,
                                          uint32_t& t2) const {
        uint64_t b1 = wave_ballot(f1), b2 = wave_ballot(f2);
        uint64_t lt = lanemask_lt();
        p1 = (uint32_t)popc64(b1 & lt);
        p2 = (uint32_t)popc64(b2 & lt);
        if constexpr (TPM == 64) {
            t1 = (uint32_t)popc64(b1);
            t2 = (uint32_t)popc64(b2);
        } else {
            int w = threadIdx.x >> 6;
            if (lane_id() == 0) sl[w] = (uint32_t)popc64(b1) | ((uint32_t)popc64(b2) << 16);
            __syncthreads();
            uint32_t a1 = 0, a2 = 0, s1 = 0, s2 = 0;
#pragma unroll
            for (int i = 0; i < NWAVE; ++i) {
                uint32_t v = sl[i];
                uint32_t c1 = v & 0xffffu, c2 = v >> 16;
                if (i < w) { a1 += c1; a2 += c2; }
                s1 += c1; s2 += c2;
            }
            __syncthreads();
            p1 += a1; p2 += a2; t1 = s1; t2 = s2;
        }
    }
    __device__ __forceinline__ uint32_t excl(uint32_t x, uint32_t& tot) const {
        if constexpr (TPM == 64) {
            uint32_t inc = wave_incl_scan(x);
            tot = __shfl(inc, 63, 64);
            return inc - x;
        } else {
            return block_excl_scan<uint32_t>(x, sl, tot);
        }
    }
    __device__ __forceinline__ unsigned long long bcast0(unsigned long long v) const {
        if constexpr (TPM == 64) {
            return __shfl(v, 0, 64);
        } else {
            unsigned long long* s64 = (unsigned long long*)(sl + 8);
            if (threadIdx.x == 0) *s64 = v;
            __syncthreads();
            unsigned long long r = *s64;
            __syncthreads();
            return r;
        }
    }
};

template <int TPM>
__device__ __forceinline__ void group_bitonic(uint32_t* E, uint32_t P2, const Grp<TPM>& G) {
    const int t = G.tid();
    for (uint32_t k = 2; k <= P2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < P2; i += TPM) {
                uint32_t ixj = i ^ j;
                if (ixj > i) {
                    uint32_t x = E[i], y = E[ixj];
                    bool up = (i & k) == 0;
                    if ((x > y) == up) { E[i] = y; E[ixj] = x; }
                }
            }
            G.sync();
        }
    }
}

// ascending bitonic sort of one value per lane across the wave (registers)
__device__ __forceinline__ uint32_t wave_sort64(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            uint32_t o = __shfl_xor(v, j, 64);
            bool up = (l & k) == 0;
            bool lower = (l & j) == 0;
            uint32_t mn = v < o ? v : o, mx = v < o ? o : v;
            v = (lower == up) ? mn : mx;
        }
    }
    return v;
}

__device__ __forceinline__ void shard_add(DevStats* st, uint32_t key, int field, unsigned long long v) {
    if (v) atomicAdd(&st->shard[key & (STAT_SHARDS - 1)][field], v);
}

// ---------------------------------------------------------------------------
// ops: last-op dedupe per slot (seq = index in the tick's op stream)
__global__ void __launch_bounds__(NT) k_ops1(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    if (op.slot >= b.cap || op.kind < GW_OP_ENTER || op.kind > GW_OP_SYNC) {
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
    if (op.slot >= b.cap || op.kind != GW_OP_LEAVE) return;
    if (b.last_leave[op.slot] == (int32_t)i) b.flags[op.slot] = 0;
}

__global__ void __launch_bounds__(NT) k_ops3(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    if (op.slot >= b.cap || op.kind < GW_OP_ENTER || op.kind > GW_OP_SYNC) return;
    uint32_t s = op.slot;
    // syncInfoFlag |= bits of every call after the last Leave (Space.go:196,
    // Entity.go:1199-1204, 1286)
    if ((int32_t)i > b.last_leave[s] && op.sync_flags) atomicOr(&b.flags[s], (uint32_t)op.sync_flags);
    if (b.last_pos[s] == (int32_t)i) b.pos[s] = make_float4(op.x, op.y, op.z, op.yaw);
    if (b.last_aoi[s] == (int32_t)i) {
        AoiEnt a = b.aoi[s];
        a.seq = (int32_t)i;
        if (op.kind == GW_OP_LEAVE) a.meta &= ~PRESENT_BIT;
        else { a.x = op.x; a.z = op.z; a.meta |= PRESENT_BIT; }
        b.aoi[s] = a;
        b.is_mover[s] = 1;
    }
}

void tick_ops(const TickBufs& b, hipStream_t s) {
    if (!b.m) return;
    hipLaunchKernelGGL(k_ops1, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_ops2, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_ops3, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// uniform grid: counting sort by cell (histogram, scan, atomic-cursor scatter).
// The order inside a cell is irrelevant downstream: every output is ordered by
// slot, never by candidate order.
__global__ void __launch_bounds__(NT) k_cell_count(TickBufs b) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s >= b.cap) return;
    AoiEnt a = b.aoi[s];
    uint32_t key = b.ncells;
    if (a.meta & PRESENT_BIT) {
        SpaceP P = b.sp[a.meta & SPACE_MASK];
        int cx = cellc(a.x, P.x0, P.inv_cs, P.W);
        int cz = cellc(a.z, P.z0, P.inv_cs, P.H);
        key = P.cell_base + (uint32_t)cz * (uint32_t)P.W + (uint32_t)cx;
        atomicAdd(&b.cell_cnt[key], 1u);
    }
    b.keys[s] = key;
}
__global__ void __launch_bounds__(NT) k_grid_prep(TickBufs b) {
    uint32_t c = blockIdx.x * NT + threadIdx.x;
    if (c < b.ncells) b.cursor[c] = b.cell_start[c];
    if (c == 0) b.st->n_present = b.cell_start[b.ncells];
}
__global__ void __launch_bounds__(NT) k_cell_scatter(TickBufs b) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s >= b.cap) return;
    uint32_t key = b.keys[s];
    if (key >= b.ncells) return;
    uint32_t p = atomicAdd(&b.cursor[key], 1u);
    AoiEnt a = b.aoi[s];
    SortEnt e;
    e.x = a.x; e.z = a.z; e.slot = s; e.seq = a.seq;
    b.se[p] = e;
    b.pflag[p] = a.seq >= 0;
}

void tick_grid(const TickBufs& b, uint64_t* scan_tmp64, uint32_t* scan_tmp32, hipStream_t s) {
    (void)scan_tmp64;
    (void)hipMemsetAsync(b.cell_cnt, 0, ((size_t)b.ncells + 1) * 4, s);
    hipLaunchKernelGGL(k_cell_count, dim3(nblk1(b.cap, NT)), dim3(NT), 0, s, b);
    scan_exclusive<uint32_t, uint32_t>(b.cell_cnt, b.cell_start, (uint64_t)b.ncells + 1, nullptr, scan_tmp32,
                                       nullptr, s);
    hipLaunchKernelGGL(k_grid_prep, dim3(nblk1(b.ncells, NT)), dim3(NT), 0, s, b);
    hipLaunchKernelGGL(k_cell_scatter, dim3(nblk1(b.cap, NT)), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// movers: the ones in the grid in cell order (L2 reuse of overlapping
// windows), then the leavers
__global__ void __launch_bounds__(NT) k_compact_cell_movers(TickBufs b) {
    uint64_t p = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (p >= b.st->n_present) return;
    if (b.pflag[p]) b.movers[b.pre[p]] = b.se[p].slot;
}
__global__ void __launch_bounds__(NT) k_leaver_flags(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    gw_op op = b.ops[i];
    bool f = op.kind == GW_OP_LEAVE && op.slot < b.cap && b.last_aoi[op.slot] == (int32_t)i;
    b.pflag[i] = f;
}
__global__ void __launch_bounds__(NT) k_compact_leavers(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    if (b.pflag[i]) b.movers[b.st->movers_present + b.pre[i]] = b.ops[i].slot;
}

void tick_movers(const TickBufs& b, uint64_t* scan_tmp64, hipStream_t s) {
    scan_exclusive<uint32_t, uint64_t>(b.pflag, b.pre, b.cap, (const uint64_t*)&b.st->n_present, scan_tmp64,
                                       (uint64_t*)&b.st->movers_present, s);
    hipLaunchKernelGGL(k_compact_cell_movers, dim3(nblk1(b.cap, NT)), dim3(NT), 0, s, b);
    if (b.m) {
        hipLaunchKernelGGL(k_leaver_flags, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
        scan_exclusive<uint32_t, uint64_t>(b.pflag, b.pre, b.m, nullptr, scan_tmp64, (uint64_t*)&b.st->leavers, s);
        hipLaunchKernelGGL(k_compact_leavers, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    }
}

// ---------------------------------------------------------------------------
// per-mover candidate count, old-list length and tier
__device__ __forceinline__ uint64_t n_movers_dev(const DevStats* st) { return st->movers_present + st->leavers; }

__global__ void __launch_bounds__(NT) k_bounds(TickBufs b) {
    uint64_t nm = n_movers_dev(b.st);
    uint64_t m = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (m >= nm) return;
    uint32_t A = b.movers[m];
    AoiEnt a = b.aoi[A];
    uint32_t ko = b.lst[A].cnt + b.log_cnt[A];     // >= the list size after its log is applied
    uint64_t c = 0;
    if (a.meta & PRESENT_BIT) {
        SpaceP P = b.sp[a.meta & SPACE_MASK];
        int cx0, cx1, cz0, cz1;
        search_cells(P, a.x, a.z, cx0, cx1, cz0, cz1);
        for (int cz = cz0; cz <= cz1; ++cz) {
            uint32_t row = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
            c += b.cell_start[row + cx1 + 1] - b.cell_start[row + cx0];
        }
    }
    uint32_t cand = (uint32_t)c;
    b.bpk[m] = (uint64_t)cand | ((uint64_t)ko << 32);
    bool ts = cand <= TS_ECAP && ko <= TS_OCAP;
    bool tb = !ts && cand <= TB_ECAP && ko <= TB_OCAP;
    b.tpk[m] = (uint64_t)ts | ((uint64_t)tb << 32);
    if (!ts && !tb) {                               // tier C: rare, atomics are fine
        unsigned long long i = atomicAdd(&b.st->n_tier_c, 1ull);
        b.list_c[i] = (uint32_t)m;
        uint64_t nw = (ko + 63) / 64;
        uint64_t words = next_pow2(cand ? cand : 1) + 2 * nw + nw + 4;
        words = (words + 3) & ~3ull;
        b.c_temp_off[m] = atomicAdd(&b.st->tier_c_temp, (unsigned long long)words);
    }
}
__global__ void __launch_bounds__(NT) k_tier_compact(TickBufs b) {
    uint64_t nm = n_movers_dev(b.st);
    uint64_t m = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (m >= nm) return;
    uint64_t t = b.tpk[m], p = b.tier_pre[m];
    if (t & 1) b.list_s[lo32(p)] = (uint32_t)m;
    if (t >> 32) b.list_b[hi32(p)] = (uint32_t)m;
}
__global__ void k_set_nm(DevStats* st) { st->scratch = st->movers_present + st->leavers; }

void tick_bounds(const TickBufs& b, uint64_t* scan_tmp64, hipStream_t s) {
    if (!b.m) return;
    hipLaunchKernelGGL(k_set_nm, dim3(1), dim3(1), 0, s, b.st);
    const uint64_t* nm = (const uint64_t*)&b.st->scratch;
    hipLaunchKernelGGL(k_bounds, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
    scan_exclusive<uint64_t, uint64_t>(b.bpk, b.reg_pk, b.m, nm, scan_tmp64, (uint64_t*)&b.st->bound_pk, s);
    scan_exclusive<uint64_t, uint64_t>(b.tpk, b.tier_pre, b.m, nm, scan_tmp64, (uint64_t*)&b.st->tier_pk, s);
    hipLaunchKernelGGL(k_tier_compact, dim3(nblk(b.m, NT)), dim3(NT), 0, s, b);
}

// ---------------------------------------------------------------------------
// delta logs: apply a slot's pending events to its sorted list (one wave)
struct ListCtx {
    LstMeta* lst;
    uint32_t* pool;
    uint64_t pool_cap;
    DevStats* st;
    uint32_t* log_cnt;
    uint32_t* logs;
};
__device__ __forceinline__ ListCtx list_ctx(const TickBufs& b) {
    ListCtx c;
    c.lst = b.lst; c.pool = b.pool; c.pool_cap = b.pool_cap; c.st = b.st; c.log_cnt = b.log_cnt; c.logs = b.logs;
    return c;
}

// destination of a list rewrite: the alternate half, or a new region of
// 2*ncap entries when the list outgrew its capacity (one lane allocates)
__device__ __forceinline__ bool list_dest(const ListCtx& c, const LstMeta& L, uint32_t nn, uint32_t key,
                                          uint32_t& dst_off, uint32_t& alt_off, uint32_t& ncap) {
    dst_off = L.alt; alt_off = L.cur; ncap = L.cap;
    if (nn <= L.cap) return true;
    ncap = round16((uint64_t)nn * 5 / 2 + 16);
    unsigned long long base = 0;
    if (lane_id() == 0) base = atomicAdd(&c.st->pool_top, 2ull * ncap);
    base = __shfl(base, 0, 64);
    if (base + 2ull * ncap > c.pool_cap) {
        if (lane_id() == 0) atomicAdd(&c.st->pool_overflow, 1ull);
        return false;
    }
    dst_off = (uint32_t)(base >> 4);
    alt_off = (uint32_t)((base + ncap) >> 4);
    if (lane_id() == 0) shard_add(c.st, key, SH_REALLOC, 1);
    return true;
}

// lbuf: 3*LOGCAP words of this wave's LDS
__device__ void wave_materialize(const ListCtx& c, uint32_t s, uint32_t* lbuf) {
    const int ln = lane_id();
    const uint32_t lc = c.log_cnt[s];
    if (lc == 0) return;
    const uint64_t lt = lanemask_lt();
    const uint32_t* lg = c.logs + (uint64_t)s * LOGCAP;
    const uint32_t P2 = next_pow2(lc);
    Grp<64> G;
    G.sl = nullptr;
    G.sync();
    for (uint32_t i = ln; i < P2; i += 64) lbuf[i] = i < lc ? lg[i] : 0xffffffffu;
    G.sync();
    group_bitonic<64>(lbuf, P2, G);
    // net effect per target: events of one pair alternate, so the majority
    // kind of its run decides (more enters -> add, more leaves -> remove)
    uint32_t* ADD = lbuf + LOGCAP;
    uint32_t* REM = lbuf + 2 * LOGCAP;
    uint32_t nadd = 0, nrem = 0;
    for (uint32_t base = 0; base < lc; base += 64) {
        const uint32_t i = base + ln;
        bool isadd = false, isrem = false;
        uint32_t t = 0;
        if (i < lc) {
            const uint32_t v = lbuf[i];
            t = v >> 1;
            if (i == 0 || (lbuf[i - 1] >> 1) != t) {
                int ne = 0, nl = 0;
                for (uint32_t j = i; j < lc && (lbuf[j] >> 1) == t; ++j) {
                    if (lbuf[j] & 1) ++nl; else ++ne;
                }
                isadd = ne > nl;
                isrem = nl > ne;
            }
        }
        const uint64_t b1 = wave_ballot(isadd), b2 = wave_ballot(isrem);
        if (isadd) ADD[nadd + popc64(b1 & lt)] = t;
        if (isrem) REM[nrem + popc64(b2 & lt)] = t;
        nadd += popc64(b1);
        nrem += popc64(b2);
    }
    G.sync();
    const LstMeta L = c.lst[s];
    const uint32_t ko = L.cnt;
    const uint32_t* __restrict__ old = lptr(c.pool, L.cur);
    const uint32_t nn = ko + nadd - nrem;
    uint32_t dst_off, alt_off, ncap;
    if (!list_dest(c, L, nn, s, dst_off, alt_off, ncap)) return;
    uint32_t* dst = lptr(c.pool, dst_off);
    for (uint32_t j = ln; j < ko; j += 64) {
        const uint32_t o = old[j];
        const uint32_t ir = lower_bound_u32(REM, nrem, o);
        if (ir < nrem && REM[ir] == o) continue;
        const uint32_t at = j - ir + lower_bound_u32(ADD, nadd, o);
        if (at < nn) dst[at] = o;
    }
    for (uint32_t q = ln; q < nadd; q += 64) {
        const uint32_t a = ADD[q];
        const uint32_t at = q + lower_bound_u32(old, ko, a) - lower_bound_u32(REM, nrem, a);
        if (at < nn) dst[at] = a;
    }
    if (ln == 0) {
        LstMeta n2;
        n2.cur = dst_off; n2.alt = alt_off; n2.cnt = nn; n2.cap = ncap;
        c.lst[s] = n2;
        c.log_cnt[s] = 0;
        shard_add(c.st, s, SH_MAT, 1);
    }
    G.sync();
}

// movers of tier C (global-scratch diff) materialise their logs first; tiers
// S and B apply them while staging the old list in LDS
__global__ void __launch_bounds__(NT) k_materialize_movers(TickBufs b, int all) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[NWAVE * 3 * LOGCAP];
    const uint64_t nc = all ? b.st->movers_present : b.st->n_tier_c;
    const ListCtx c = list_ctx(b);
    uint32_t* lbuf = lds + (threadIdx.x >> 6) * 3 * LOGCAP;
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    for (uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6); k < nc; k += stride)
        wave_materialize(c, b.movers[all ? k : b.list_c[k]], lbuf);
}
void tick_materialize_movers(const TickBufs& b, uint64_t n, bool all, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_materialize_movers, dim3(gstride(n, NWAVE)), dim3(NT), 0, s, b, (int)all);
}

__global__ void __launch_bounds__(NT) k_materialize_slots(ListCtx c, const uint32_t* __restrict__ slots,
                                                          const uint64_t* n_dev, uint64_t n_max) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[NWAVE * 3 * LOGCAP];
    const uint64_t n = load_n(n_max, n_dev);
    uint32_t* lbuf = lds + (threadIdx.x >> 6) * 3 * LOGCAP;
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    for (uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6); k < n; k += stride)
        wave_materialize(c, slots[k], lbuf);
}
void launch_materialize_slots(LstMeta* lst, uint32_t* pool, uint64_t pool_cap, DevStats* st, uint32_t* log_cnt,
                              uint32_t* logs, const uint32_t* slots, const uint64_t* n_dev, uint64_t n_max,
                              hipStream_t s) {
    if (!n_max) return;
    ListCtx c;
    c.lst = lst; c.pool = pool; c.pool_cap = pool_cap; c.st = st; c.log_cnt = log_cnt; c.logs = logs;
    hipLaunchKernelGGL(k_materialize_slots, dim3(gstride(n_max, NWAVE)), dim3(NT), 0, s, c, slots, n_dev, n_max);
}

// ---------------------------------------------------------------------------
// diff of one mover A by a group of TPM threads.
//   (i)   candidates b in A's widened window with related(A,b) and b not in
//         old(A) -> enters (buffer E), mirror enter (b,A) if b has no op
//   sort  E ascending (bitonic)
//   (ii)  old entries: related -> kept (bit in KM), else leave(A,b) [+mirror]
//   merge new = kept old U E into the alternate half (or a new region)
// Buffers E/KM/KP are LDS for tiers S/B and global scratch for tier C.
template <int TPM, uint32_t ECAP, uint32_t OCAP, bool GLOB>
__global__ void __launch_bounds__(NT, (TPM == 64 ? 6 : 4)) k_mover(TickBufs b, const uint32_t* __restrict__ list, int which) {
    constexpr uint32_t KW = GLOB ? 1 : (OCAP + 63) / 64;          // u64 words of kept mask
    static_assert(GLOB || ECAP >= 3 * LOGCAP, "the log is staged in E");
    constexpr uint32_t GWORDS = GLOB ? 4 : ((2 * KW + ECAP + OCAP + KW + 1 + 3) & ~3u);
    constexpr int GPB = NT / TPM;                                  // groups per block
    __shared__ __attribute__((aligned(16))) uint32_t lds[GPB * GWORDS + 16];
    const int gi = TPM == 64 ? (int)(threadIdx.x >> 6) : 0;
    Grp<TPM> G;
    G.sl = lds + GPB * GWORDS;
    const uint64_t nl = which == 0 ? lo32(b.st->tier_pk) : which == 1 ? hi32(b.st->tier_pk) : b.st->n_tier_c;
    const uint64_t li = (uint64_t)blockIdx.x * GPB + gi;
    if (li >= nl) return;                                          // group-uniform
    const int t = G.tid();
    const uint32_t m = list[li];
    const uint32_t A = b.movers[m];
    const AoiEnt a = b.aoi[A];
    const bool presA = (a.meta & PRESENT_BIT) != 0;
    const SpaceP P = b.sp[a.meta & SPACE_MASK];
    const float d = P.d;
    const float lox = a.x - d, hix = a.x + d, loz = a.z - d, hiz = a.z + d;   // fl(x-d), fl(x+d)
    const int seqA = a.seq;
    const LstMeta L = b.lst[A];
    uint32_t ko = L.cnt;
    const uint32_t* __restrict__ old_g = lptr(b.pool, L.cur);
    const uint64_t rp = b.reg_pk[m];
    const uint64_t reg = lo32(rp) + hi32(rp);
    uint32_t* own_l = b.own + reg;            // own leaves  [0, ko)
    uint32_t* own_e = b.own + reg + (uint32_t)hi32(b.bpk[m]);   // own enters [0, cand) after the leave bound
    uint64_t* mir = b.mir + reg;              // mirror events [0, cand + ko)
    uint64_t* KM;
    uint32_t *E, *KP;
    const uint32_t* old;
    if constexpr (GLOB) {
        uint32_t cand = (uint32_t)lo32(b.bpk[m]);
        uint32_t* base = b.c_temp + b.c_temp_off[m];
        uint32_t nw = (ko + 63) / 64;
        KM = (uint64_t*)base;
        E = base + 2 * nw;
        KP = E + next_pow2(cand ? cand : 1);
        old = old_g;
    } else {
        // the old list is staged in LDS: membership tests and merge ranks are
        // binary searches over it
        uint32_t* gb = lds + gi * GWORDS;
        KM = (uint64_t*)gb;
        E = gb + 2 * KW;
        uint32_t* OL = E + ECAP;
        KP = OL + OCAP;
        uint32_t* LG = E;                                        // 3*LOGCAP: log, adds, removes (E is free until (i))
        const uint32_t lc = b.log_cnt[A];
        if (lc == 0) {
            for (uint32_t j = t; j < ko; j += TPM) OL[j] = old_g[j];
        } else {
            // the mover's pending delta log is applied here (base list + net
            // adds - net removes -> OL); the materialised list is never written
            const uint32_t* lg = b.logs + (uint64_t)A * LOGCAP;
            const uint32_t LP2 = next_pow2(lc);
            for (uint32_t i = t; i < LP2; i += TPM) LG[i] = i < lc ? lg[i] : 0xffffffffu;
            G.sync();
            group_bitonic<TPM>(LG, LP2, G);
            uint32_t* ADD = LG + LOGCAP;
            uint32_t* REM = LG + 2 * LOGCAP;
            uint32_t nadd = 0, nrem = 0;
            for (uint32_t base = 0; base < lc; base += TPM) {
                const uint32_t i = base + t;
                bool isadd = false, isrem = false;
                uint32_t tg = 0;
                if (i < lc) {
                    tg = LG[i] >> 1;
                    if (i == 0 || (LG[i - 1] >> 1) != tg) {
                        int ne = 0, nl = 0;
                        for (uint32_t j = i; j < lc && (LG[j] >> 1) == tg; ++j) {
                            if (LG[j] & 1) ++nl; else ++ne;
                        }
                        isadd = ne > nl;
                        isrem = nl > ne;
                    }
                }
                uint32_t pa, pr, ta, tr;
                G.excl2(isadd, isrem, pa, pr, ta, tr);
                if (isadd) ADD[nadd + pa] = tg;
                if (isrem) REM[nrem + pr] = tg;
                nadd += ta;
                nrem += tr;
            }
            G.sync();
            const uint32_t kb0 = ko;
            ko = kb0 + nadd - nrem;
            for (uint32_t j = t; j < kb0; j += TPM) {
                const uint32_t o = old_g[j];
                const uint32_t ir = lower_bound_u32(REM, nrem, o);
                if (ir < nrem && REM[ir] == o) continue;
                const uint32_t at = j - ir + lower_bound_u32(ADD, nadd, o);
                if (at < ko) OL[at] = o;
            }
            for (uint32_t q = t; q < nadd; q += TPM) {
                const uint32_t av = ADD[q];
                const uint32_t at = q + lower_bound_u32(old_g, kb0, av) - lower_bound_u32(REM, nrem, av);
                if (at < ko) OL[at] = av;
            }
            if (t == 0) {
                b.log_cnt[A] = 0;
                shard_add(b.st, A, SH_MAT, 1);
            }
        }
        G.sync();
        old = OL;
    }
    uint32_t n_e = 0, n_mir = 0;
    uint64_t tested = 0;
    // (i) candidates
    if (presA) {
        int cx0, cx1, cz0, cz1;
        search_cells(P, a.x, a.z, cx0, cx1, cz0, cz1);
        for (int cz = cz0; cz <= cz1; ++cz) {
            const uint32_t row = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
            const uint32_t p0 = b.cell_start[row + cx0], p1 = b.cell_start[row + cx1 + 1];
            tested += p1 - p0;
            for (uint32_t base = p0; base < p1; base += TPM) {
                const uint32_t p = base + t;
                bool ent = false, mr = false;
                uint32_t bs = 0;
                if (p < p1) {
                    const SortEnt e = b.se[p];
                    bs = e.slot;
                    if (bs != A && relation(seqA, a.x, a.z, lox, hix, loz, hiz, e.seq, e.x, e.z, d)) {
                        ent = !contains_u32(old, ko, bs);
                        mr = ent && e.seq < 0;
                    }
                }
                uint32_t pe, pm, te, tm;
                G.excl2(ent, mr, pe, pm, te, tm);
                if (ent) E[n_e + pe] = bs;
                if (mr) {
                    mir[n_mir + pm] = ((uint64_t)bs << 32) | A;
                    atomicAdd(&b.cnt64[bs], 1ull);
                }
                n_e += te;
                n_mir += tm;
            }
        }
    }
    // sort the enters
    const uint32_t P2 = next_pow2(n_e);
    G.sync();
    for (uint32_t i = n_e + t; i < P2; i += TPM) E[i] = 0xffffffffu;
    G.sync();
    group_bitonic<TPM>(E, P2, G);
    for (uint32_t q = t; q < n_e; q += TPM) own_e[q] = E[q];
    // (ii) old entries: kept mask, own leaves (ascending), mirror leaves
    uint32_t n_l = 0;
    const uint32_t wv = TPM == 64 ? 0u : (threadIdx.x >> 6);
    for (uint32_t base = 0; base < ko; base += TPM) {
        const uint32_t j = base + t;
        bool kept = false, lv = false, mr = false;
        uint32_t bs = 0;
        if (j < ko) {
            bs = old[j];
            const AoiEnt eb = b.aoi[bs];
            bool rel = presA && (eb.meta & PRESENT_BIT) &&
                       relation(seqA, a.x, a.z, lox, hix, loz, hiz, eb.seq, eb.x, eb.z, d);
            kept = rel;
            lv = !rel;
            mr = lv && eb.seq < 0;
        }
        const uint64_t kb = wave_ballot(kept);
        if (lane_id() == 0 && base + 64u * wv < ko) KM[(base >> 6) + wv] = kb;
        uint32_t pl, pm, tl, tm;
        G.excl2(lv, mr, pl, pm, tl, tm);
        if (lv) own_l[n_l + pl] = bs;
        if (mr) {
            mir[n_mir + pm] = ((uint64_t)bs << 32) | 0x80000000ull | A;
            atomicAdd(&b.cnt64[bs], 1ull << 32);
        }
        n_l += tl;
        n_mir += tm;
    }
    G.sync();
    // KP: exclusive prefix of kept counts per 64-entry word
    const uint32_t nw = (ko + 63) / 64;
    {
        uint32_t run = 0;
        for (uint32_t base = 0; base < nw; base += TPM) {
            uint32_t w = base + t;
            uint32_t c = w < nw ? (uint32_t)popc64(KM[w]) : 0;
            uint32_t tot;
            uint32_t pre = G.excl(c, tot);
            if (w < nw) KP[w] = run + pre;
            run += tot;
        }
        if (t == 0) KP[nw] = run;
    }
    G.sync();
    const uint32_t n_kept = ko - n_l;
    const uint32_t nn = n_kept + n_e;
    uint32_t dst_off = L.alt, alt_off = L.cur, ncap = L.cap;
    bool ok = true;
    if (nn > L.cap) {                                        // outgrew: new region of 2*ncap
        ncap = round16((uint64_t)nn * 5 / 2 + 16);
        unsigned long long base = 0;
        if (t == 0) base = atomicAdd(&b.st->pool_top, 2ull * ncap);
        base = G.bcast0(base);
        if (base + 2ull * ncap > b.pool_cap) {
            ok = false;
            if (t == 0) atomicAdd(&b.st->pool_overflow, 1ull);
        }
        dst_off = (uint32_t)(base >> 4);
        alt_off = (uint32_t)((base + ncap) >> 4);
        if (t == 0) shard_add(b.st, m, SH_REALLOC, 1);
    }
    if (ok) {
        uint32_t* dst = lptr(b.pool, dst_off);
        for (uint32_t base = 0; base < ko; base += TPM) {
            const uint32_t j = base + t;
            if (j < ko) {
                const uint64_t w = KM[j >> 6];
                if ((w >> (j & 63)) & 1) {
                    const uint32_t o = old[j];
                    uint32_t pos = KP[j >> 6] + (uint32_t)popc64(w & ((1ull << (j & 63)) - 1)) +
                                   lower_bound_u32(E, n_e, o);
                    if (pos < nn) dst[pos] = o;
                }
            }
        }
        for (uint32_t q = t; q < n_e; q += TPM) {
            const uint32_t e = E[q];
            const uint32_t lb = lower_bound_u32(old, ko, e);
            const uint32_t kb = lb < ko ? KP[lb >> 6] + (uint32_t)popc64(KM[lb >> 6] & ((1ull << (lb & 63)) - 1))
                                        : n_kept;
            if (q + kb < nn) dst[q + kb] = e;
        }
    }
    if (t == 0) {
        if (ok) {
            LstMeta nl2;
            nl2.cur = dst_off; nl2.alt = alt_off; nl2.cnt = nn; nl2.cap = ncap;
            b.lst[A] = nl2;
        }
        b.cnt64[A] = (unsigned long long)n_e | ((unsigned long long)n_l << 32);
        b.mir_cnt[m] = n_mir;
        shard_add(b.st, m, SH_PAIRS, tested);
        shard_add(b.st, m, SH_AOLD, ko);
        shard_add(b.st, m, SH_ANEW, nn);
    }
}

void tick_diff(const TickBufs& b, uint64_t n_s, uint64_t n_b, uint64_t n_c, hipStream_t s) {
    if (n_s)
        hipLaunchKernelGGL((k_mover<64, TS_ECAP, TS_OCAP, false>), dim3(nblk(n_s, NWAVE)), dim3(NT), 0, s, b,
                           b.list_s, 0);
    if (n_b)
        hipLaunchKernelGGL((k_mover<256, TB_ECAP, TB_OCAP, false>), dim3((uint32_t)n_b), dim3(NT), 0, s, b,
                           b.list_b, 1);
    if (n_c)
        hipLaunchKernelGGL((k_mover<256, 0, 0, true>), dim3((uint32_t)n_c), dim3(NT), 0, s, b, b.list_c, 2);
}

// ---------------------------------------------------------------------------
// canonical events: offsets per watcher, affected op-less watchers
__global__ void __launch_bounds__(NT) k_affected_flags(TickBufs b) {
    uint32_t w = blockIdx.x * NT + threadIdx.x;
    if (w >= b.cap) return;
    uint64_t f = 0;
    if (!b.is_mover[w]) {
        uint64_t o0 = b.off64[w], o1 = b.off64[w + 1];
        if (o0 != o1) {
            uint64_t ne = lo32(o1) - lo32(o0), nlv = hi32(o1) - hi32(o0);
            bool big = ne > SEG_SMALL || nlv > SEG_SMALL;
            f = big ? (1ull << 32) : 1ull;
        }
    }
    b.pre[w] = f;
}
__global__ void __launch_bounds__(NT) k_affected_compact(TickBufs b) {
    uint32_t w = blockIdx.x * NT + threadIdx.x;
    if (w >= b.cap) return;
    uint64_t f = b.pre[w];
    if (!f) return;
    uint64_t p = b.fpre[w];
    if (f & 1) {
        b.affected[lo32(p)] = w;
    } else {
        uint64_t i = hi32(p);
        b.bigseg[i] = w;
        uint64_t o0 = b.off64[w], o1 = b.off64[w + 1];
        uint32_t ne = (uint32_t)(lo32(o1) - lo32(o0)), nlv = (uint32_t)(hi32(o1) - hi32(o0));
        unsigned long long words = next_pow2(ne) + next_pow2(nlv) + 4;
        unsigned long long off = atomicAdd(&b.st->bigseg_temp, words);
        if (off + words > b.bigseg_temp_cap) atomicAdd(&b.st->tmp_overflow, 1ull);
        b.bigseg_off[i] = off;
    }
}

void tick_events(const TickBufs& b, uint64_t n_movers, uint64_t* scan_tmp64, hipStream_t s) {
    (void)n_movers;
    // offsets: cnt64[cap] is always 0, so off64[cap] = totals
    scan_exclusive<uint64_t, uint64_t>((const uint64_t*)b.cnt64, b.off64, (uint64_t)b.cap + 1, nullptr, scan_tmp64,
                                       (uint64_t*)&b.st->ev_pk, s);
    hipLaunchKernelGGL(k_affected_flags, dim3(nblk1(b.cap, NT)), dim3(NT), 0, s, b);
    scan_exclusive<uint64_t, uint64_t>(b.pre, b.fpre, b.cap, nullptr, scan_tmp64, (uint64_t*)&b.st->n_affected, s);
    hipLaunchKernelGGL(k_affected_compact, dim3(nblk1(b.cap, NT)), dim3(NT), 0, s, b);
}

// one wave per mover: scatter its mirror events to their watchers' segments
// (order inside a segment fixed later by the segment sort), copy its own
// sorted events, reset its counter
__global__ void __launch_bounds__(NT) k_events_scatter(TickBufs b) {
    const uint64_t nm = n_movers_dev(b.st);
    const uint64_t m = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (m >= nm) return;
    const int ln = lane_id();
    const uint32_t A = b.movers[m];
    const uint64_t rp = b.reg_pk[m];
    const uint64_t reg = lo32(rp) + hi32(rp);
    const uint32_t ko = (uint32_t)hi32(b.bpk[m]);
    const uint32_t nmir = b.mir_cnt[m];
    const uint64_t* mir = b.mir + reg;
    for (uint32_t k = ln; k < nmir; k += 64) {
        const uint64_t e = mir[k];
        const uint32_t w = (uint32_t)(e >> 32);
        const uint32_t src = (uint32_t)(e & 0x7fffffffu);
        const bool lv = (e >> 31) & 1;
        const unsigned long long dec = lv ? (1ull << 32) : 1ull;
        const unsigned long long old = atomicAdd(&b.cnt64[w], (unsigned long long)(0ull - dec));
        const uint64_t off = b.off64[w];
        gw_event ev;
        ev.watcher = w;
        ev.target = src;
        if (lv) {
            const uint64_t at = hi32(off) + (hi32(old) - 1);
            if (at < b.leave_cap) b.leave[at] = ev;
        } else {
            const uint64_t at = lo32(off) + (lo32(old) - 1);
            if (at < b.enter_cap) b.enter[at] = ev;
        }
    }
    const uint64_t c = b.cnt64[A];
    const uint32_t ne = (uint32_t)lo32(c), nlv = (uint32_t)hi32(c);
    const uint64_t off = b.off64[A];
    for (uint32_t q = ln; q < ne; q += 64) {
        gw_event ev; ev.watcher = A; ev.target = b.own[reg + ko + q];
        if (lo32(off) + q < b.enter_cap) b.enter[lo32(off) + q] = ev;
    }
    for (uint32_t j = ln; j < nlv; j += 64) {
        gw_event ev; ev.watcher = A; ev.target = b.own[reg + j];
        if (hi32(off) + j < b.leave_cap) b.leave[hi32(off) + j] = ev;
    }
    if (ln == 0) b.cnt64[A] = 0;
}

// ---------------------------------------------------------------------------
// segment sorts of op-less watchers (their events arrive unordered)
__device__ __forceinline__ void wave_sort_segment(gw_event* seg, uint32_t n, uint32_t* lbuf) {
    const int ln = lane_id();
    if (n <= 1) return;
    if (n <= 64) {
        uint32_t v = ln < (int)n ? seg[ln].target : 0xffffffffu;
        v = wave_sort64(v);
        if (ln < (int)n) seg[ln].target = v;
        return;
    }
    const uint32_t P2 = next_pow2(n);
    Grp<64> G;
    G.sl = nullptr;
    G.sync();
    for (uint32_t i = ln; i < P2; i += 64) lbuf[i] = i < n ? seg[i].target : 0xffffffffu;
    G.sync();
    group_bitonic<64>(lbuf, P2, G);
    for (uint32_t i = ln; i < n; i += 64) seg[i].target = lbuf[i];
    G.sync();
}

__global__ void __launch_bounds__(NT) k_seg_sort_small(TickBufs b) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[NWAVE * SEG_SMALL];
    const uint64_t n = lo32(b.st->n_affected);
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    uint32_t* lbuf = lds + (threadIdx.x >> 6) * SEG_SMALL;
    for (uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6); k < n; k += stride) {
        const uint32_t w = b.affected[k];
        const uint64_t o0 = b.off64[w], o1 = b.off64[w + 1];
        wave_sort_segment(b.enter + lo32(o0), (uint32_t)(lo32(o1) - lo32(o0)), lbuf);
        wave_sort_segment(b.leave + hi32(o0), (uint32_t)(hi32(o1) - hi32(o0)), lbuf);
    }
}

__global__ void __launch_bounds__(NT) k_seg_sort_big(TickBufs b) {
    __shared__ uint32_t sl[16];
    Grp<256> G;
    G.sl = sl;
    const uint64_t n = hi32(b.st->n_affected);
    for (uint64_t k = blockIdx.x; k < n; k += gridDim.x) {
        const uint32_t w = b.bigseg[k];
        const uint64_t o0 = b.off64[w], o1 = b.off64[w + 1];
        uint32_t* tmp = b.bigseg_temp + b.bigseg_off[k];
        for (int part = 0; part < 2; ++part) {
            gw_event* seg = part == 0 ? b.enter + lo32(o0) : b.leave + hi32(o0);
            const uint32_t cnt = (uint32_t)(part == 0 ? lo32(o1) - lo32(o0) : hi32(o1) - hi32(o0));
            const uint32_t P2 = next_pow2(cnt);
            for (uint32_t i = threadIdx.x; i < P2; i += NT) tmp[i] = i < cnt ? seg[i].target : 0xffffffffu;
            __syncthreads();
            group_bitonic<256>(tmp, P2, G);
            for (uint32_t i = threadIdx.x; i < cnt; i += NT) seg[i].target = tmp[i];
            __syncthreads();
            tmp += P2;
        }
    }
}

// op-less watchers: append the tick's (sorted) events to the delta log; a
// watcher whose log would overflow is materialized first, and a burst larger
// than the whole log is merged straight into its list
__global__ void __launch_bounds__(NT, 6) k_nonmover_update(TickBufs b, int sort_small) {
    constexpr uint32_t WW = SEG_SMALL > 3 * LOGCAP ? SEG_SMALL : 3 * LOGCAP;
    __shared__ __attribute__((aligned(16))) uint32_t lds[NWAVE * WW];
    const uint64_t n_small = lo32(b.st->n_affected), n_big = hi32(b.st->n_affected);
    const uint64_t nlist = n_small + n_big;
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    const int ln = lane_id();
    const ListCtx c = list_ctx(b);
    uint32_t* lbuf = lds + (threadIdx.x >> 6) * WW;           // segment sort, then materialize
    uint32_t* sbuf = lbuf;
    for (uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6); k < nlist; k += stride) {
        const uint32_t w = k < n_small ? b.affected[k] : b.bigseg[k - n_small];
        const uint64_t o0 = b.off64[w], o1 = b.off64[w + 1];
        gw_event* E = b.enter + lo32(o0);
        gw_event* Lv = b.leave + hi32(o0);
        const uint32_t ne = (uint32_t)(lo32(o1) - lo32(o0)), nlv = (uint32_t)(hi32(o1) - hi32(o0));
        if (sort_small && k < n_small) {     // big segments were sorted by k_seg_sort_big
            wave_sort_segment(E, ne, sbuf);
            wave_sort_segment(Lv, nlv, sbuf);
        }
        const uint32_t n = ne + nlv;
        if (b.log_cnt[w] + n > LOGCAP) wave_materialize(c, w, lbuf);
        if (n <= LOGCAP) {
            const uint32_t lc = b.log_cnt[w];
            uint32_t* lg = b.logs + (uint64_t)w * LOGCAP + lc;
            for (uint32_t q = ln; q < ne; q += 64) lg[q] = E[q].target << 1;
            for (uint32_t q = ln; q < nlv; q += 64) lg[ne + q] = (Lv[q].target << 1) | 1u;
            if (ln == 0) {
                b.log_cnt[w] = lc + n;
                shard_add(b.st, w, SH_LOGAPP, 1);
            }
            continue;
        }
        // burst: log is empty now, merge the sorted segments into the list
        const LstMeta L = b.lst[w];
        const uint32_t ko = L.cnt;
        const uint32_t* __restrict__ old = lptr(b.pool, L.cur);
        const uint32_t nn = ko - nlv + ne;
        uint32_t dst_off, alt_off, ncap;
        if (!list_dest(c, L, nn, w, dst_off, alt_off, ncap)) continue;
        uint32_t* dst = lptr(b.pool, dst_off);
        for (uint32_t j = ln; j < ko; j += 64) {
            const uint32_t o = old[j];
            const uint32_t il = lower_bound_ev(Lv, nlv, o);
            if (il < nlv && Lv[il].target == o) continue;          // left
            const uint32_t at = j - il + lower_bound_ev(E, ne, o);
            if (at < nn) dst[at] = o;
        }
        for (uint32_t q = ln; q < ne; q += 64) {
            const uint32_t tg = E[q].target;
            const uint32_t at = q + lower_bound_u32(old, ko, tg) - lower_bound_ev(Lv, nlv, tg);
            if (at < nn) dst[at] = tg;
        }
        if (ln == 0) {
            LstMeta n2;
            n2.cur = dst_off; n2.alt = alt_off; n2.cnt = nn; n2.cap = ncap;
            b.lst[w] = n2;
            shard_add(b.st, w, SH_MERGE, 1);
        }
    }
}

void tick_nonmovers(const TickBufs& b, uint64_t n_affected_max, uint64_t n_big_max, uint64_t n_movers,
                    hipStream_t s, bool fuse_sort) {
    if (n_movers)
        hipLaunchKernelGGL(k_events_scatter, dim3(nblk(n_movers, NWAVE)), dim3(NT), 0, s, b);
    if (n_affected_max) {
        hipLaunchKernelGGL(k_seg_sort_big, dim3(gstride(n_big_max, 1) > 1024 ? 1024 : gstride(n_big_max, 1)),
                           dim3(NT), 0, s, b);
        if (!fuse_sort)
            hipLaunchKernelGGL(k_seg_sort_small, dim3(gstride(n_affected_max, NWAVE)), dim3(NT), 0, s, b);
        hipLaunchKernelGGL(k_nonmover_update, dim3(gstride(n_affected_max, NWAVE)), dim3(NT), 0, s, b,
                           (int)fuse_sort);
    }
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) k_tick_reset(TickBufs b) {
    uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= b.m) return;
    uint32_t s = b.ops[i].slot;
    if (s >= b.cap) return;
    b.last_pos[s] = -1;
    b.last_aoi[s] = -1;
    b.last_leave[s] = -1;
    b.aoi[s].seq = -1;
    b.is_mover[s] = 0;
}
void tick_reset(const TickBufs& b, uint64_t n_movers, hipStream_t s) {
    (void)n_movers;
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
        st->reallocs = tot[SH_REALLOC];
        st->materialized = tot[SH_MAT];
        st->log_appends = tot[SH_LOGAPP];
        st->seg_merges = tot[SH_MERGE];
    }
}
void stats_reduce(DevStats* st, hipStream_t s) {
    static_assert(STAT_SHARDS == NT, "one thread per shard");
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(NT), 0, s, st);
}

// pool compaction: one wave per slot copies its current list into a packed pool
__global__ void __launch_bounds__(NT) k_pool_compact(const LstMeta* __restrict__ lst_in,
                                                     const uint64_t* __restrict__ new_off, uint32_t cap,
                                                     const uint32_t* __restrict__ pool_old, uint32_t* pool_new,
                                                     LstMeta* lst_out) {
    uint64_t s = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (s >= cap) return;
    LstMeta L = lst_in[s];
    const uint32_t* src = lptr(pool_old, L.cur);
    uint32_t* dst = pool_new + new_off[s];
    for (uint32_t j = lane_id(); j < L.cnt; j += 64) dst[j] = src[j];
    if (lane_id() == 0) {
        LstMeta n;
        n.cur = (uint32_t)(new_off[s] >> 4);
        n.alt = (uint32_t)((new_off[s] + L.cap) >> 4);
        n.cnt = L.cnt;
        n.cap = L.cap;
        lst_out[s] = n;
    }
}
void launch_pool_compact(const LstMeta* lst_in, const uint64_t* new_off, uint32_t cap, const uint32_t* pool_old,
                         uint32_t* pool_new, LstMeta* lst_out, hipStream_t s) {
    hipLaunchKernelGGL(k_pool_compact, dim3(nblk1(cap, NWAVE)), dim3(NT), 0, s, lst_in, new_off, cap, pool_old,
                       pool_new, lst_out);
}
__global__ void __launch_bounds__(NT) k_cap2(const LstMeta* lst, uint32_t cap, uint32_t* out) {
    uint32_t s = blockIdx.x * NT + threadIdx.x;
    if (s < cap) out[s] = 2 * lst[s].cap;
}
void launch_cap2(const LstMeta* lst, uint32_t cap, uint32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_cap2, dim3(nblk1(cap, NT)), dim3(NT), 0, s, lst, cap, out);
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

// record bound per flagged entity e: own (bit0 and e has a client) + |list|
// (bit1).  Exact when every neighbour has a client (the usual case); the write
// kernel flags gaps and a compaction pass closes them.
__global__ void __launch_bounds__(NT) k_sync_count(const uint32_t* __restrict__ flagged, const uint64_t* nf_dev,
                                                   uint32_t nf_max, const uint32_t* __restrict__ flags,
                                                   const AoiEnt* __restrict__ aoi, const uint16_t* __restrict__ gate,
                                                   const LstMeta* __restrict__ lst,
                                                   const uint32_t* __restrict__ pool, uint32_t* cnt) {
    (void)pool;
    uint64_t nf = load_n(nf_max, nf_dev);
    uint64_t k = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (k >= nf) return;
    uint32_t e = flagged[k];
    uint32_t f = flags[e];
    uint32_t r = 0;
    if (aoi[e].meta & PRESENT_BIT) {
        if (f & GW_SIF_NEIGHBOR_CLIENTS) r += lst[e].cnt;
        if ((f & GW_SIF_OWN_CLIENT) && gate[e]) r += 1;
    }
    cnt[k] = r;
}
void launch_sync_count(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, const uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const LstMeta* lst, const uint32_t* pool,
                       uint32_t* cnt, hipStream_t s) {
    if (!nf_max) return;
    hipLaunchKernelGGL(k_sync_count, dim3(nblk(nf_max, NT)), dim3(NT), 0, s, flagged, nf_dev, nf_max, flags, aoi,
                       gate, lst, pool, cnt);
}

// writes e's records in (entity, watcher) order; the own record sits at the
// rank of e among e's client-holding neighbours.  Clears the flag.
__global__ void __launch_bounds__(NT) k_sync_write(const uint32_t* __restrict__ flagged, const uint64_t* nf_dev,
                                                   uint32_t nf_max, uint32_t* flags, const AoiEnt* __restrict__ aoi,
                                                   const uint16_t* __restrict__ gate,
                                                   const LstMeta* __restrict__ lst,
                                                   const uint32_t* __restrict__ pool, const float4* __restrict__ pos,
                                                   const uint64_t* __restrict__ rec_off, gw_sync_record* rec,
                                                   uint64_t rec_cap, uint32_t* act, DevStats* st) {
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
            LstMeta L = lst[e];
            const uint32_t* Ls = lptr(pool, L.cur);
            for (uint32_t j0 = 0; j0 < L.cnt; j0 += 64) {
                uint32_t j = j0 + ln;
                uint32_t w = 0;
                bool has = false;
                if (j < L.cnt) { w = Ls[j]; has = gate[w] != 0; }
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
        const uint32_t n_act = run + (own ? 1u : 0u);
        if (ln == 0) {
            act[k] = n_act;
            if (f & GW_SIF_NEIGHBOR_CLIENTS) {
                const uint32_t bound = lst[e].cnt + (own ? 1u : 0u);
                if (n_act != bound) atomicOr((unsigned int*)&st->scratch, 1u);   // gaps: compact
            }
        }
    } else if (ln == 0) {
        act[k] = 0;
    }
    if (ln == 0) flags[e] = 0;
}

// close the gaps left by neighbours without clients: copy each entity's
// records from its bound offset to its exact offset (into a second buffer)
__global__ void __launch_bounds__(NT) k_sync_compact(const uint64_t* nf_dev, uint32_t nf_max,
                                                     const uint64_t* __restrict__ rec_off,
                                                     const uint32_t* __restrict__ act,
                                                     const uint64_t* __restrict__ act_off,
                                                     const gw_sync_record* __restrict__ in, gw_sync_record* out) {
    uint64_t nf = load_n(nf_max, nf_dev);
    uint64_t k = (uint64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
    if (k >= nf) return;
    const uint32_t n = act[k];
    const gw_sync_record* src = in + rec_off[k];
    gw_sync_record* dst = out + act_off[k];
    for (uint32_t j = lane_id(); j < n; j += 64) dst[j] = src[j];
}
void launch_sync_compact(const uint64_t* nf_dev, uint32_t nf_max, const uint64_t* rec_off, const uint32_t* act,
                         const uint64_t* act_off, const gw_sync_record* in, gw_sync_record* out, hipStream_t s) {
    if (!nf_max) return;
    hipLaunchKernelGGL(k_sync_compact, dim3(nblk(nf_max, NWAVE)), dim3(NT), 0, s, nf_dev, nf_max, rec_off, act,
                       act_off, in, out);
}
void launch_sync_write(const uint32_t* flagged, const uint64_t* nf_dev, uint32_t nf_max, uint32_t* flags,
                       const AoiEnt* aoi, const uint16_t* gate, const LstMeta* lst, const uint32_t* pool,
                       const float4* pos, const uint64_t* rec_off, gw_sync_record* rec, uint64_t rec_cap,
                       uint32_t* act, DevStats* st, hipStream_t s) {
    if (!nf_max) return;
    hipLaunchKernelGGL(k_sync_write, dim3(nblk(nf_max, NWAVE)), dim3(NT), 0, s, flagged, nf_dev, nf_max, flags, aoi,
                       gate, lst, pool, pos, rec_off, rec, rec_cap, act, st);
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

}  // namespace gw
