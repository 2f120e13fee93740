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

// A's rounded window, computed once per watcher
struct Win {
    float lox, hix, loz, hiz;
    __device__ bool has(float x, float z) const { return x >= lox && x <= hix && z >= loz && z <= hiz; }
};
__device__ __forceinline__ Win win_of(float x, float z, float d) {
    Win w;
    w.lox = x - d; w.hix = x + d; w.loz = z - d; w.hiz = z + d;   // NaN centre -> empty window
    return w;
}
__device__ __forceinline__ bool in_win(float cx, float cz, float d, float ox, float oz) {
    return ox >= cx - d && ox <= cx + d && oz >= cz - d && oz <= cz + d;
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

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
        for (uint32_t i = t; i < (P2 >> 1); i += TPM) {
            const uint32_t lo = (i / h) * k + (i % h);
            const uint32_t hi = lo ^ (k - 1);
            if (hi < n) {
                T x = a[lo], y = a[hi];
                if (key(y) < key(x)) { a[lo] = y; a[hi] = x; }
            }
        }
        sync();
        for (uint32_t j = h >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < (P2 >> 1); i += TPM) {
                const uint32_t lo = (i / j) * (2 * j) + (i % j);
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
