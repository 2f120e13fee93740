// dev_common.hpp — device helpers shared by aoi.hip and sync.hip: cell
// search, window tests, the stamp-resolved pair relation, wave/block sorts.
//
// Window arithmetic follows go-aoi's XZList Mark bounds:
// B is inside A's window iff fl(A.x-d) <= B.x <= fl(A.x+d) and the same on z,
// in float32 round-to-nearest (files compiled with -ffp-contract=off).
#pragma once
#include "gw_internal.hpp"
#include "prim.hpp"

namespace gw {

static inline uint32_t nblk(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }
static inline uint32_t nblk1(uint64_t n, uint32_t per) { uint32_t b = nblk(n, per); return b ? b : 1; }
static inline uint32_t gstride(uint64_t n, uint32_t per) {   // grid of a grid-stride loop
    uint32_t b = nblk1(n, per);
    return b > 4096 ? 4096 : b;
}

__device__ __forceinline__ uint64_t lo32(uint64_t v) { return v & 0xffffffffull; }

// syncInfoFlag of slot s: 2 bits at flag_sh(s) of word flag_word(s) (the
// collect's compaction reads cap/16 words instead of a word per slot)
__device__ __forceinline__ uint32_t flag_word(uint32_t s) { return s >> 4; }
__device__ __forceinline__ uint32_t flag_sh(uint32_t s) { return (s & 15u) * 2u; }
__device__ __forceinline__ uint32_t flag_get(const uint32_t* f, uint32_t s) { return (f[flag_word(s)] >> flag_sh(s)) & 3u; }
__device__ __forceinline__ uint64_t hi32(uint64_t v) { return v >> 32; }
__device__ __forceinline__ float qnan() { return __builtin_nanf(""); }

__device__ __forceinline__ int cellc(float v, float o, float inv, int lim) {
    float f = floorf((v - o) * inv);           // monotone in v
    f = fminf(fmaxf(f, 0.0f), (float)(lim - 1));
    return (int)f;
}
__device__ __forceinline__ uint32_t cell_of(const SpaceP& P, float x, float z) {
    return P.cell_base + (uint32_t)cellc(z, P.z0, P.inv_cs, P.H) * (uint32_t)P.W +
           (uint32_t)cellc(x, P.x0, P.inv_cs, P.W);
}

// Cell rectangle (inclusive) holding every B with inWin_A(B) or inWin_B(A):
// both lie in [x-d-m, x+d+m] with m >= 8 ulp of |x|+d (the rounding of
// fl(B+-d)).  Cells are >= d wide, so a rectangle is at most 4x4 cells.
struct Rect {
    int x0, x1, z0, z1;
    __device__ bool empty() const { return x0 > x1; }
};
__device__ __forceinline__ Rect search_rect(const SpaceP& P, float x, float z) {
    const float d = P.d;
    const float mx = (fabsf(x) + d) * 1e-6f + 1e-30f;
    const float mz = (fabsf(z) + d) * 1e-6f + 1e-30f;
    Rect r;
    r.x0 = cellc((x - d) - mx, P.x0, P.inv_cs, P.W);
    r.x1 = cellc((x + d) + mx, P.x0, P.inv_cs, P.W);
    r.z0 = cellc((z - d) - mz, P.z0, P.inv_cs, P.H);
    r.z1 = cellc((z + d) + mz, P.z0, P.inv_cs, P.H);
    return r;
}
__device__ __forceinline__ Rect empty_rect() { Rect r; r.x0 = 1; r.x1 = 0; r.z0 = 1; r.z1 = 0; return r; }

// The cells a watcher scans: one or two rectangles (a mover's old and new
// windows, merged into their bounding box when they touch).
struct Rects {
    Rect r[2];
    int n;
};

// ---------------------------------------------------------------------------
// Flattened candidate ranges of one wave.  A grid row of a rectangle is one
// contiguous index range per grid (cells of a row are consecutive), so the
// candidates of a watcher are <= 2 rects x 10 rows x NK grids ranges.  Lane j
// holds range j (row j/NK, grid j%NK); the wave walks the concatenation in
// 64-lane chunks, so a sparse window (a few entities per row) fills one chunk
// instead of one mostly idle chunk per row.
struct Flat {
    uint32_t start, len, pre;   // per lane: range j = [start, start+len), exclusive prefix
    uint64_t live;              // uniform: non-empty ranges not consumed yet
    uint32_t total;             // uniform: candidates over all ranges
};

template <int NK>
__device__ __forceinline__ Flat flat_build(const SpaceP& P, const Rects& R, const uint32_t* __restrict__ s0,
                                           const uint32_t* __restrict__ s1) {
    const int ln = lane_id();
    const int row = NK == 2 ? (ln >> 1) : ln;
    const int kind = NK == 2 ? (ln & 1) : 0;
    const int nr0 = R.n > 0 ? R.r[0].z1 - R.r[0].z0 + 1 : 0;
    const int nr1 = R.n > 1 ? R.r[1].z1 - R.r[1].z0 + 1 : 0;
    uint32_t s = 0, l = 0;
    if (row < nr0 + nr1) {
        const bool first = row < nr0;
        const int x0 = first ? R.r[0].x0 : R.r[1].x0;
        const int x1 = first ? R.r[0].x1 : R.r[1].x1;
        const int cz = first ? R.r[0].z0 + row : R.r[1].z0 + (row - nr0);
        const uint32_t base = P.cell_base + (uint32_t)cz * (uint32_t)P.W;
        const uint32_t* st = kind ? s1 : s0;
        s = st[base + x0];
        l = st[base + x1 + 1] - s;
    }
    Flat f;
    const uint32_t inc = wave_incl_scan<uint32_t>(l);
    f.start = s;
    f.len = l;
    f.pre = inc - l;
    f.total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    f.live = wave_ballot(l != 0);
    return f;
}

// The same from ranges already gathered (lane j: range j = [s, s + l))
__device__ __forceinline__ Flat flat_from(uint32_t s, uint32_t l) {
    Flat f;
    const uint32_t inc = wave_incl_scan<uint32_t>(l);
    f.start = s;
    f.len = l;
    f.pre = inc - l;
    f.total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    f.live = wave_ballot(l != 0);
    return f;
}

// Maps the lane's candidates k = B + 64u + lane (u < U) to (grid, index);
// idx = ~0 past the end.  Each lane finds its range by a binary search over
// the ranges' exclusive prefixes (the largest range j with pre[j] <= k; empty
// ranges share their successor's prefix and lose the tie), log2(SPAN) shuffle
// steps per chunk instead of a serial walk over every live range with
// readlanes (a VALU cost per range that dominated the walk for short candidate
// lists).  SPAN: the ranges live in lanes [0, SPAN) (16 for the row ranges
// k_bounds hands to k_mover: two fewer dependent shuffles per chunk); the
// index is then one more shuffle, of start - pre (mod 2^32).
// The U chunks' searches run step by step together (their shuffles of one
// step in flight at once, one wait), and the first step, whose probe is the
// same lane for every lane, is a readlane: a chain of log2(SPAN) dependent
// shuffle rounds per U chunks instead of U * (log2(SPAN) + 1).
template <int U, int NK, int SPAN = 64>
__device__ __forceinline__ void flat_map(Flat& f, uint32_t B, uint32_t (&idx)[U], uint32_t (&kind)[U]) {
    const int ln = lane_id();
    const uint32_t off = f.start - f.pre;
    uint32_t k[U], lo[U];
    const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)f.pre, SPAN / 2);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        k[u] = B + 64u * u + (uint32_t)ln;
        lo[u] = p0 <= k[u] ? (uint32_t)(SPAN / 2) : 0u;
    }
#pragma unroll
    for (int step = SPAN / 4; step; step >>= 1) {
        uint32_t p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = lo[u] + (uint32_t)step;
            p[u] = (uint32_t)__shfl((int)f.pre, (int)(SPAN == 64 ? min(c, 63u) : c), 64);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = lo[u] + (uint32_t)step;
            if ((SPAN < 64 || c < 64u) && p[u] <= k[u]) lo[u] = c;
        }
    }
    uint32_t o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) o[u] = (uint32_t)__shfl((int)off, (int)lo[u], 64);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        idx[u] = k[u] < f.total ? o[u] + k[u] : ~0u;
        kind[u] = NK == 2 ? (lo[u] & 1u) : 0u;
    }
}

// The same by walking the live ranges with readlanes (cheaper in VALU when a
// chunk overlaps few ranges: the collect's long hotspot windows at config #3)
template <int U, int NK>
__device__ __forceinline__ void flat_map_walk(Flat& f, uint32_t B, uint32_t (&idx)[U], uint32_t (&kind)[U]) {
    const int ln = lane_id();
    const uint32_t end = B + 64u * U;
#pragma unroll
    for (int u = 0; u < U; ++u) { idx[u] = ~0u; kind[u] = 0; }
    uint64_t m = f.live;
    while (m) {
        const int j = __builtin_ctzll(m);
        const uint32_t sp = (uint32_t)__builtin_amdgcn_readlane((int)f.pre, j);
        if (sp >= end) break;
        const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((int)f.len, j);
        const uint32_t ss = (uint32_t)__builtin_amdgcn_readlane((int)f.start, j);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t r = B + 64u * u + (uint32_t)ln - sp;
            if (r < sl) { idx[u] = ss + r; kind[u] = NK == 2 ? (uint32_t)(j & 1) : 0u; }
        }
        if (sp + sl <= end) f.live &= ~(1ull << j);
        m &= m - 1;
    }
}

// (x, z) inside [lox, hix] x [loz, hiz], exactly: an IEEE difference keeps
// the sign of the exact one (ties give +0; f32 denormals are not flushed in
// these kernels), so lo <= x  <=>  lo - x <= 0, and the four comparisons
// become one: max(lox - x, x - hix, loz - z, z - hiz) <= 0.  One VALU chain
// and one compare instead of four compares ANDed as lane masks (scalar ALU
// work in every candidate chunk of the walks).  NaN: an absent entity has
// both coordinates NaN and an absent centre all four bounds, so every term is
// NaN, the max is NaN (maxnum drops a NaN only beside a number) and the test
// is false, as the four comparisons were.
__device__ __forceinline__ bool box_has(float lox, float hix, float loz, float hiz, float x, float z) {
    return fmaxf(fmaxf(lox - x, x - hix), fmaxf(loz - z, z - hiz)) <= 0.0f;
}

// Keep a wave-uniform value in a vector register: the walks are short of
// scalar registers (k_mover_c is capped at 80 for residency), and a spilled
// scalar is reloaded by a v_readlane in every chunk.  An empty asm with a
// VGPR constraint: no instruction.
__device__ __forceinline__ void in_vgpr(float& v) { asm volatile("" : "+v"(v)); }

// A's rounded window, computed once per watcher.  eps bounds the rounding
// band: B's own window test of A, fl(b -+ d) <= a <= ..., can disagree with
// A's test of B only where B lies within 2 max(ulp(a -+ d), ulp(b +- d)) of
// an edge of A's window (the two tests are one exact inequality, each side
// rounded once), i.e. within 2^-23 (|a| + d) per axis; eps is 8 times that
// (plus a floor for tiny coordinates), so outside eps of every edge the
// relation is A's test alone.  NaN centre: empty window, eps NaN (no band).
struct Win {
    float lox, hix, loz, hiz, eps;
    __device__ bool has(float x, float z) const { return box_has(lox, hix, loz, hiz, x, z); }
    // has(x, z), and whether (x, z) is within eps of an edge (where the
    // member with the later op decides the pair)
    __device__ __forceinline__ void to_vgprs() {
        in_vgpr(lox); in_vgpr(hix); in_vgpr(loz); in_vgpr(hiz); in_vgpr(eps);
    }
    __device__ __forceinline__ void test(float x, float z, bool& in, bool& near) const {
        const float t0 = lox - x, t1 = x - hix, t2 = loz - z, t3 = z - hiz;
        in = fmaxf(fmaxf(t0, t1), fmaxf(t2, t3)) <= 0.0f;
        near = fminf(fminf(fabsf(t0), fabsf(t1)), fminf(fabsf(t2), fabsf(t3))) <= eps;
    }
};
__device__ __forceinline__ Win win_of(float x, float z, float d) {
    Win w;
    w.lox = x - d; w.hix = x + d; w.loz = z - d; w.hiz = z + d;   // NaN centre -> empty window
    w.eps = (fabsf(x) + fabsf(z) + d) * 0x1p-20f + 0x1p-120f;
    return w;
}
// o inside c's window [fl(c-d), fl(c+d)]^2
__device__ __forceinline__ bool in_win(float cx, float cz, float d, float ox, float oz) {
    return box_has(cx - d, cx + d, cz - d, cz + d, ox, oz);
}

// related(A,B) from A's window test ia and B's window test ib: they agree
// outside the rounding band; inside it the member with the later last AOI op
// decides (XZList adjust() of that member was the last to touch the pair).
__device__ __forceinline__ bool resolve(bool ia, bool ib, unsigned long long sa, unsigned long long sb) {
    return sa > sb ? ia : ib;
}

__device__ __forceinline__ uint32_t next_pow2(uint32_t v) {
    if (v <= 1) return 1;
    return 1u << (32 - __clz(v - 1));
}

// Block copy of n 16-B items from HBM into LDS with 4 loads in flight per
// thread (a plain strided loop waits out one HBM round trip per item it copies)
template <int NTH>
__device__ __forceinline__ void lds_fill16(uint4* dst, const uint4* __restrict__ src, uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += 4 * NTH) {
        const uint32_t left = n - i;
        const uint4 r0 = src[i];
        const uint4 r1 = left > NTH ? src[i + NTH] : r0;
        const uint4 r2 = left > 2 * NTH ? src[i + 2 * NTH] : r0;
        const uint4 r3 = left > 3 * NTH ? src[i + 3 * NTH] : r0;
        dst[i] = r0;
        if (left > NTH) dst[i + NTH] = r1;
        if (left > 2 * NTH) dst[i + 2 * NTH] = r2;
        if (left > 3 * NTH) dst[i + 3 * NTH] = r3;
    }
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v of lane l ^ j.  j <= 8 stays inside a 16-lane row and runs on the DPP
// network (quad_perm for 1 and 2, row_shl / row_shr for 4 and 8: VALU moves);
// 16 and 32 cross rows and go through ds_bpermute.  j is a compile-time
// constant once the sorting network is unrolled.
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, int j) {
    const int x = (int)v;
    if (j == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    if (j == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    if (j == 4) {
        const int up = __builtin_amdgcn_update_dpp(0, x, 0x104, 0xf, 0xf, false);         // row_shl:4 (lane + 4)
        const int dn = __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);         // row_shr:4 (lane - 4)
        return (uint32_t)((lane_id() & 4) ? dn : up);
    }
    if (j == 8) {
        const int up = __builtin_amdgcn_update_dpp(0, x, 0x108, 0xf, 0xf, false);
        const int dn = __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
        return (uint32_t)((lane_id() & 8) ? dn : up);
    }
    return (uint32_t)__shfl_xor(x, j, 64);
}

// ascending bitonic sort of one value per lane across the wave (registers)
__device__ __forceinline__ uint32_t wave_sort64(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            uint32_t o = lane_xor(v, j);
            bool up = (l & k) == 0;
            bool lower = (l & j) == 0;
            uint32_t mn = v < o ? v : o, mx = v < o ? o : v;
            v = (lower == up) ? mn : mx;
        }
    }
    return v;
}

// the same for 64-bit keys
__device__ __forceinline__ uint64_t wave_sort64_u64(uint64_t v) {
    const int l = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t o = ((uint64_t)lane_xor((uint32_t)(v >> 32), j) << 32) | lane_xor((uint32_t)v, j);
            const bool up = (l & k) == 0;
            const bool lower = (l & j) == 0;
            const uint64_t mn = v < o ? v : o, mx = v < o ? o : v;
            v = (lower == up) ? mn : mx;
        }
    }
    return v;
}

// ascending bitonic sort of one value per lane inside each 32-lane half
__device__ __forceinline__ uint32_t half_sort32(uint32_t v) {
    const int l = lane_id() & 31;                     // both halves end ascending
#pragma unroll
    for (int k = 2; k <= 32; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint32_t o = lane_xor(v, j);
            const bool up = (l & k) == 0;
            const bool lower = (l & j) == 0;
            const uint32_t mn = v < o ? v : o, mx = v < o ? o : v;
            v = (lower == up) ? mn : mx;
        }
    }
    return v;
}

// In-place ascending sort of a[0, n) by a group of TPM threads with the
// all-ascending bitonic network (first step of each merge compares mirrored
// partners i ^ (k-1)).  Every exchange moves the smaller key to the lower
// index, so the virtual +inf padding past n never moves and n need not be a
// power of two.  `sync` orders the steps (wave barrier or __syncthreads).
template <int TPM, typename T, typename KeyF, typename SyncF>
__device__ __forceinline__ void bitonic_inplace(T* a, uint32_t n, int t, KeyF key, SyncF sync) {
    const uint32_t P2 = next_pow2(n);
    for (uint32_t k = 2; k <= P2; k <<= 1) {
        const uint32_t h = k >> 1;
        const int lh = __builtin_ctz(h);                 // powers of two: shifts, no integer division
        for (uint32_t i = t; i < (P2 >> 1); i += TPM) {
            const uint32_t lo = ((i >> lh) << (lh + 1)) | (i & (h - 1));
            const uint32_t hi = lo ^ (k - 1);
            if (hi < n) {
                T x = a[lo], y = a[hi];
                if (key(y) < key(x)) { a[lo] = y; a[hi] = x; }
            }
        }
        sync();
        for (uint32_t j = h >> 1; j > 0; j >>= 1) {
            const int lj = __builtin_ctz(j);
            for (uint32_t i = t; i < (P2 >> 1); i += TPM) {
                const uint32_t lo = ((i >> lj) << (lj + 1)) | (i & (j - 1));
                const uint32_t hi = lo + j;
                if (hi < n) {
                    T x = a[lo], y = a[hi];
                    if (key(y) < key(x)) { a[lo] = y; a[hi] = x; }
                }
            }
            sync();
        }
    }
}

__device__ __forceinline__ void shard_add(DevStats* st, uint32_t key, int field, unsigned long long v) {
    if (v) atomicAdd(&st->shard[key & (STAT_SHARDS - 1)][field], v);
}

}  // namespace gw
