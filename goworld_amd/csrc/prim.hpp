// prim.hpp — wave64 / LDS primitives for gfx950: wave scans, block scans,
// three-phase device exclusive scan, and a stable LSD radix sort whose
// per-block ranking uses wavefront ballots (match-any over the digit bits).
//
// Everything here is HBM-bound integer work: no MFMA.  Tiles are sized for
// 256-thread workgroups (4 waves of 64 lanes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "gw_internal.hpp"

namespace gw {

constexpr int NT = 256;          // threads per workgroup in every primitive
constexpr int NWAVE = NT / 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63u); }
__device__ __forceinline__ uint64_t lanemask_lt() {
    int l = lane_id();
    return l ? (~0ull >> (64 - l)) : 0ull;
}
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        T y = __shfl_up(x, off, 64);
        if (lane_id() >= off) x += y;
    }
    return x;
}

// 32-bit inclusive scan on the DPP network (VALU lane moves; the shuffle
// version above goes through ds_bpermute, an LDS round trip per step, which
// sits on the latency chain of every per-mover / per-entity walk): row_shr
// 1, 2, 4, 8 inside each 16-lane row, then row_bcast:15 into rows 1 and 3 and
// row_bcast:31 into rows 2 and 3 (GFX9 broadcast modes).  Lanes a DPP move
// does not write keep the identity 0.
template <>
__device__ __forceinline__ uint32_t wave_incl_scan<uint32_t>(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return (uint32_t)x;
}

// 64-bit version: each DPP step moves both halves, then one 64-bit add
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long x, int ctrl_sel) {
    const int lo = (int)(uint32_t)x, hi = (int)(uint32_t)(x >> 32);
    int a, b;
    switch (ctrl_sel) {
    case 0: a = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xf, 0xf, false); break;
    case 1: a = __builtin_amdgcn_update_dpp(0, lo, 0x112, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0, hi, 0x112, 0xf, 0xf, false); break;
    case 2: a = __builtin_amdgcn_update_dpp(0, lo, 0x114, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0, hi, 0x114, 0xf, 0xf, false); break;
    case 3: a = __builtin_amdgcn_update_dpp(0, lo, 0x118, 0xf, 0xf, false); b = __builtin_amdgcn_update_dpp(0, hi, 0x118, 0xf, 0xf, false); break;
    case 4: a = __builtin_amdgcn_update_dpp(0, lo, 0x142, 0xa, 0xf, false); b = __builtin_amdgcn_update_dpp(0, hi, 0x142, 0xa, 0xf, false); break;
    default: a = __builtin_amdgcn_update_dpp(0, lo, 0x143, 0xc, 0xf, false); b = __builtin_amdgcn_update_dpp(0, hi, 0x143, 0xc, 0xf, false); break;
    }
    return ((unsigned long long)(uint32_t)b << 32) | (uint32_t)a;
}
template <>
__device__ __forceinline__ unsigned long long wave_incl_scan<unsigned long long>(unsigned long long x) {
#pragma unroll
    for (int i = 0; i < 6; ++i) x += dpp_u64(x, i);
    return x;
}
template <>
__device__ __forceinline__ unsigned long wave_incl_scan<unsigned long>(unsigned long x) {
    return (unsigned long)wave_incl_scan<unsigned long long>((unsigned long long)x);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// exclusive scan of one value per thread over the workgroup; lds needs NWAVE
// elements.  Returns the exclusive prefix; total gets the workgroup sum.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T x, T* lds, T& total) {
    T inc = wave_incl_scan(x);
    int w = threadIdx.x >> 6;
    if (lane_id() == 63) lds[w] = inc;
    __syncthreads();
    T pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; ++i) {
        T v = lds[i];
        pre += (i < w) ? v : (T)0;
        tot += v;
    }
    __syncthreads();
    total = tot;
    return pre + inc - x;
}

// Exclusive scan of one tile of IPT * NT values held STRIPED (thread t holds
// elements j * NT + t, j < IPT: every load and store of the caller is
// coalesced).  Each row j is scanned by wave scans; the IPT * NWAVE row/wave
// partials (64 of them) are scanned once more by every wave, lane k holding
// partial k = j * NWAVE + w.  v[j] becomes the exclusive prefix of its element
// within the tile; total gets the tile sum.  lds: 64 elements.
template <typename T, int IPT>
__device__ __forceinline__ void tile_excl_scan_striped(T (&v)[IPT], T* lds, T& total) {
    constexpr int P = IPT * NWAVE;            // row/wave partials
    constexpr int Q = P / 64;                 // partials per lane
    static_assert(P % 64 == 0, "whole partials per lane");
    const int w = (int)(threadIdx.x >> 6), ln = lane_id();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {             // v[j] becomes the in-wave exclusive prefix
        const T inc = wave_incl_scan(v[j]);
        if (ln == 63) lds[j * NWAVE + w] = inc;
        v[j] = inc - v[j];
    }
    __syncthreads();
    // lane k holds partials k*Q .. k*Q+Q-1 (row-major: j * NWAVE + w)
    T q[Q], ls = 0;
#pragma unroll
    for (int k = 0; k < Q; ++k) {
        q[k] = ls;
        ls += lds[ln * Q + k];
    }
    const T li = wave_incl_scan(ls);
    total = __shfl(li, 63, 64);
    const T le = li - ls;
#pragma unroll
    for (int k = 0; k < Q; ++k) q[k] += le;      // exclusive prefix of each partial
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int idx = j * NWAVE + w;            // wave-uniform
        v[j] += __shfl(q[idx % Q], idx / Q, 64);
    }
    __syncthreads();
}

__device__ __forceinline__ uint64_t load_n(uint64_t n_max, const uint64_t* n_dev) {
    if (!n_dev) return n_max;
    uint64_t n = *n_dev;
    return n < n_max ? n : n_max;
}

// ---------------------------------------------------------------------------
// Device exclusive scan in ONE launch (decoupled look-back): out[i] =
// sum(in[0..i)), *total = sum(in[0..n)).  Tiles of 4096 elements take a
// ticket in dispatch order (a tile only waits on tiles that already run), post
// their aggregate, and wave 0 looks back over up to 64 predecessors at a time
// until it meets an inclusive prefix.  A tile publishes 4 status words: the
// aggregate and the inclusive prefix, each split into 32-bit halves; every
// word carries tag | flag | half in one 8-B agent-scope atomic (no separate
// payload, so no fence), and a reader takes the inclusive pair if both halves
// are posted, else the aggregate pair.  The per-call tag makes words of
// earlier scans read as "not posted", so the status array is never cleared.
constexpr int SCAN_IPT = 16;
constexpr int SCAN_TILE = NT * SCAN_IPT;
constexpr uint64_t SCAN_BIG = 1ull << 21;           // larger scans use 2 * SCAN_TILE tiles
constexpr int SCAN_SHIFT = 34;                       // tag above flag bit 33 and the 32-bit half
constexpr unsigned long long SCAN_POSTED = 1ull << 33;
constexpr uint32_t SCAN_TAG_MAX = (1u << 22) - 1;
constexpr int SCAN_WORDS = 4;                        // agg lo/hi, incl lo/hi

__device__ __forceinline__ unsigned long long scan_ld(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void scan_st(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename TO>
__device__ __forceinline__ void scan_post(unsigned long long* w, unsigned long long tg, TO v) {
    const unsigned long long x = (unsigned long long)v;
    scan_st(w, tg | SCAN_POSTED | (x & 0xffffffffull));
    scan_st(w + 1, tg | SCAN_POSTED | (x >> 32));
}

// Look-back of tile `tile` whose aggregate is tot, run by wave 0 (threads
// 0..63) of the block; returns the exclusive prefix of the tile (to every lane
// of wave 0) after posting the tile's inclusive prefix.
template <typename TO>
__device__ __forceinline__ TO scan_lookback(unsigned long long* __restrict__ status, uint32_t tile, uint32_t tag,
                                            TO tot) {
    const unsigned long long tg = (unsigned long long)tag << SCAN_SHIFT;
    unsigned long long* my = status + (uint64_t)tile * SCAN_WORDS;
    TO excl = 0;
    if (tile == 0) {
        if (threadIdx.x == 0) scan_post<TO>(my + 2, tg, tot);
        return excl;
    }
    if (threadIdx.x == 0) scan_post<TO>(my, tg, tot);
    const int ln = (int)threadIdx.x;
    int64_t j = (int64_t)tile - 1;
    while (true) {
        const int64_t q = j - ln;
        bool ready = true, incl = true;
        unsigned long long lo = 0, hi = 0;
        if (q >= 0) {
            const unsigned long long* w = status + (uint64_t)q * SCAN_WORDS;
            const unsigned long long il = scan_ld(w + 2), ih = scan_ld(w + 3);
            const bool ok = (il >> SCAN_SHIFT) == tag && (ih >> SCAN_SHIFT) == tag;
            if (ok) {
                lo = il; hi = ih;
            } else {
                incl = false;
                lo = scan_ld(w);
                hi = scan_ld(w + 1);
                ready = (lo >> SCAN_SHIFT) == tag && (hi >> SCAN_SHIFT) == tag;
            }
        }
        const uint64_t bi = wave_ballot(ready && incl);
        const uint64_t nr = wave_ballot(!ready);
        const int f = bi ? __builtin_ctzll(bi) : 64;
        const uint64_t need = f >= 63 ? ~0ull : ((2ull << f) - 1);  // lanes 0..f
        if (nr & need) continue;                                     // spin on the window
        const unsigned long long x = (lo & 0xffffffffull) | ((hi & 0xffffffffull) << 32);
        excl += wave_sum<TO>((ln <= f) ? (TO)x : (TO)0);
        if (f < 64) break;
        j -= 64;
    }
    if (threadIdx.x == 0) scan_post<TO>(my + 2, tg, excl + tot);
    return excl;
}

// Output hook of a scan (element index, exclusive prefix, element): work that
// needs the scanned offsets rides in the scan's store phase instead of a
// launch of its own.  active() is read once per thread.
struct ScanNoPost {
    __device__ bool active() const { return false; }
    template <typename T>
    __device__ void operator()(uint64_t, T, T) const {}
};

template <typename TI, typename TO, int IPT, class Post = ScanNoPost>
__global__ void __launch_bounds__(NT) k_scan1(const TI* in, TO* out, uint64_t n_max, const uint64_t* n_dev,
                                              unsigned long long* __restrict__ status,
                                              unsigned long long* __restrict__ ticket, unsigned long long tbase,
                                              uint32_t tag, TO* total, Post post) {
    __shared__ TO lds[IPT * NWAVE];
    __shared__ uint32_t s_tile;
    __shared__ TO s_prefix;
    // the device-side count is loaded under the ticket's round trip (not after
    // the barrier: one dependent load less on a chain of a few microseconds)
    const uint64_t n = load_n(n_max, n_dev);
    if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tbase);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t t0 = (uint64_t)tile * (IPT * NT);
    // tiles past a device-side count do nothing (no later tile waits on them)
    if (t0 >= n && tile > 0) return;
    TO v[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        v[j] = i < n ? (TO)in[i] : (TO)0;
    }
    const bool pa = post.active();
    TO x[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) x[j] = v[j];
    TO tot;
    tile_excl_scan_striped<TO, IPT>(v, lds, tot);
    if (threadIdx.x < 64) {
        const TO excl = scan_lookback<TO>(status, tile, tag, tot);
        if (threadIdx.x == 0) s_prefix = excl;
    }
    __syncthreads();
    const TO pre = s_prefix;
    if (out) {
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
            if (i < n) out[i] = pre + v[j];
        }
    }
    if (pa) {
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
            if (i < n) post(i, (TO)(pre + v[j]), x[j]);
        }
    }
    // the last tile holding data (tile 0 when n == 0) writes the total
    const uint64_t last = n ? (n - 1) / (IPT * NT) : 0;
    if (total && tile == last && threadIdx.x == 0) *total = pre + tot;
}

// host launcher; sc.status must hold SCAN_WORDS * ceil(n_max / SCAN_TILE) words
// Two u32 arrays of the same length scanned by one launch: element i packs
// a[i] | b[i] << 32 into a u64 (each sum stays below 2^32, so the halves never
// carry into each other), one look-back chain, the halves unpacked on store.
template <int IPT>
__global__ void __launch_bounds__(NT) k_scan_pair32(const uint32_t* a, const uint32_t* b, uint32_t* oa, uint32_t* ob,
                                                    uint64_t n, unsigned long long* __restrict__ status,
                                                    unsigned long long* __restrict__ ticket, unsigned long long tbase,
                                                    uint32_t tag, uint32_t* total_a, uint32_t* total_b) {
    __shared__ unsigned long long lds[IPT * NWAVE];
    __shared__ uint32_t s_tile;
    __shared__ unsigned long long s_prefix;
    if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(ticket, 1ull) - tbase);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t t0 = (uint64_t)tile * (IPT * NT);
    unsigned long long v[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        v[j] = i < n ? ((unsigned long long)a[i] | ((unsigned long long)b[i] << 32)) : 0ull;
    }
    unsigned long long tot;
    tile_excl_scan_striped<unsigned long long, IPT>(v, lds, tot);
    if (threadIdx.x < 64) {
        const unsigned long long excl = scan_lookback<unsigned long long>(status, tile, tag, tot);
        if (threadIdx.x == 0) s_prefix = excl;
    }
    __syncthreads();
    const unsigned long long pre = s_prefix;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = t0 + (uint64_t)j * NT + threadIdx.x;
        if (i < n) {
            const unsigned long long x = pre + v[j];
            oa[i] = (uint32_t)x;
            ob[i] = (uint32_t)(x >> 32);
        }
    }
    if (tile == gridDim.x - 1 && threadIdx.x == 0) {
        *total_a = (uint32_t)(pre + tot);
        *total_b = (uint32_t)((pre + tot) >> 32);
    }
}

inline void scan_pair32(const uint32_t* a, const uint32_t* b, uint32_t* oa, uint32_t* ob, uint64_t n, ScanCtx& sc,
                        uint32_t* total_a, uint32_t* total_b, hipStream_t st) {
    const uint64_t tile = SCAN_TILE;
    uint32_t nb = (uint32_t)((n + tile - 1) / tile);
    if (nb == 0) nb = 1;
    if (sc.tag >= SCAN_TAG_MAX) {
        (void)hipMemsetAsync(sc.status, 0, sc.max_tiles * SCAN_WORDS * 8, st);
        sc.tag = 0;
    }
    ++sc.tag;
    hipLaunchKernelGGL((k_scan_pair32<SCAN_IPT>), dim3(nb), dim3(NT), 0, st, a, b, oa, ob, n, sc.status, sc.ticket,
                       sc.tbase, sc.tag, total_a, total_b);
    sc.tbase += nb;
}

template <typename TI, typename TO, class Post = ScanNoPost>
inline void scan_exclusive(const TI* in, TO* out, uint64_t n_max, const uint64_t* n_dev, ScanCtx& sc,
                           TO* total_dev, hipStream_t st, Post post = Post{}) {
    // big scans take 8192-element tiles: half the tickets and look-back windows
    const bool big = n_max > SCAN_BIG;
    const uint64_t tile = big ? 2 * SCAN_TILE : SCAN_TILE;
    uint32_t nb = (uint32_t)((n_max + tile - 1) / tile);
    if (nb == 0) nb = 1;
    if (sc.tag >= SCAN_TAG_MAX) {   // tags exhausted: clear the status words once
        (void)hipMemsetAsync(sc.status, 0, sc.max_tiles * SCAN_WORDS * 8, st);
        sc.tag = 0;
    }
    ++sc.tag;
    if (big)
        hipLaunchKernelGGL((k_scan1<TI, TO, 2 * SCAN_IPT, Post>), dim3(nb), dim3(NT), 0, st, in, out, n_max, n_dev,
                           sc.status, sc.ticket, sc.tbase, sc.tag, total_dev, post);
    else
        hipLaunchKernelGGL((k_scan1<TI, TO, SCAN_IPT, Post>), dim3(nb), dim3(NT), 0, st, in, out, n_max, n_dev,
                           sc.status, sc.ticket, sc.tbase, sc.tag, total_dev, post);
    sc.tbase += nb;
}
inline uint64_t scan_tiles(uint64_t n_max) { return (n_max + SCAN_TILE - 1) / SCAN_TILE + 1; }

// ---------------------------------------------------------------------------
// Stable LSD radix sort, 8-bit digits.  Per pass: block digit histograms
// (LDS atomics), a device scan over the digit-major histogram table, then a
// stable scatter in which each wave ranks its 64 keys by match-any over the
// 8 digit bits (8 ballots) and the 4 waves combine counts through LDS.
constexpr int RS_IPT = 8;
constexpr int RS_TILE = NT * RS_IPT;
constexpr int RS_RADIX = 256;

template <typename K>
__global__ void __launch_bounds__(NT) k_rs_hist(const K* __restrict__ keys, uint64_t n_max,
                                                const uint64_t* n_dev, int shift,
                                                uint32_t* __restrict__ hist, uint32_t nblocks) {
    __shared__ uint32_t h[RS_RADIX];
    h[threadIdx.x] = 0;
    __syncthreads();
    uint64_t n = load_n(n_max, n_dev);
    uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll
    for (int j = 0; j < RS_IPT; ++j) {
        uint64_t i = base + (uint64_t)j * NT + threadIdx.x;
        if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

template <typename K, bool HAS_V>
__global__ void __launch_bounds__(NT) k_rs_scatter(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                   K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                   uint64_t n_max, const uint64_t* n_dev, int shift,
                                                   const uint32_t* __restrict__ offs, uint32_t nblocks) {
    __shared__ uint32_t run[RS_RADIX];
    __shared__ uint32_t wcnt[NWAVE][RS_RADIX];
    const int t = threadIdx.x, w = t >> 6;
    run[t] = offs[(uint64_t)t * nblocks + blockIdx.x];
    uint64_t n = load_n(n_max, n_dev);
    uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t lt = lanemask_lt();
    for (int j = 0; j < RS_IPT; ++j) {
#pragma unroll
        for (int k = 0; k < NWAVE; ++k) wcnt[k][t] = 0;
        __syncthreads();
        uint64_t i = base + (uint64_t)j * NT + t;
        bool valid = i < n;
        K key = valid ? kin[i] : (K)0;
        uint32_t dig = (uint32_t)(key >> shift) & 255u;
        uint64_t peers = wave_ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            bool bit = (dig >> b) & 1u;
            uint64_t bb = wave_ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        uint32_t rank = (uint32_t)popc64(peers & lt);
        if (valid && rank == 0) wcnt[w][dig] = (uint32_t)popc64(peers);
        __syncthreads();
        {   // thread t owns digit t: exclusive prefix over waves, advance run
            uint32_t r = run[t];
#pragma unroll
            for (int k = 0; k < NWAVE; ++k) { uint32_t c = wcnt[k][t]; wcnt[k][t] = r; r += c; }
            run[t] = r;
        }
        __syncthreads();
        if (valid) {
            uint32_t dst = wcnt[w][dig] + rank;
            if (dst >= n_max) dst = (uint32_t)(n_max - 1);   // never taken when offsets are consistent
            kout[dst] = key;
            if (HAS_V) vout[dst] = vin[i];
        }
        __syncthreads();
    }
}

inline uint64_t radix_blocks(uint64_t n_max) { return (n_max + RS_TILE - 1) / RS_TILE; }

// Sorts (k0,v0) by bits [lo_bit, hi_bit) using (k1,v1) as ping-pong.
// Returns 0 if the result is in (k0,v0), 1 if in (k1,v1).
template <typename K>
inline int radix_sort(K* k0, uint32_t* v0, K* k1, uint32_t* v1, uint64_t n_max, const uint64_t* n_dev,
                      int lo_bit, int hi_bit, RadixTmp& tmp, hipStream_t st) {
    uint32_t nb = (uint32_t)radix_blocks(n_max);
    if (nb == 0) return 0;
    int cur = 0;
    for (int shift = lo_bit; shift < hi_bit; shift += 8) {
        K* ki = cur ? k1 : k0; K* ko = cur ? k0 : k1;
        uint32_t* vi = cur ? v1 : v0; uint32_t* vo = cur ? v0 : v1;
        hipLaunchKernelGGL((k_rs_hist<K>), dim3(nb), dim3(NT), 0, st, ki, n_max, n_dev, shift, tmp.hist, nb);
        scan_exclusive<uint32_t, uint32_t>(tmp.hist, tmp.hist, (uint64_t)RS_RADIX * nb, nullptr, *tmp.sc,
                                           (uint32_t*)nullptr, st);
        if (v0)
            hipLaunchKernelGGL((k_rs_scatter<K, true>), dim3(nb), dim3(NT), 0, st, ki, vi, ko, vo, n_max,
                               n_dev, shift, tmp.hist, nb);
        else
            hipLaunchKernelGGL((k_rs_scatter<K, false>), dim3(nb), dim3(NT), 0, st, ki, nullptr, ko,
                               nullptr, n_max, n_dev, shift, tmp.hist, nb);
        cur ^= 1;
    }
    return cur;
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort of (u32 key, u32 value) pairs, ONE kernel per pass
// ("onesweep"), DB-bit digits (8: 10- and 11-bit digits measured slower, two
// passes of 214 us against three of 103 us over config #3's 14.7M fan-out
// pairs -- a wider digit's runs per tile are shorter write segments -- and
// were dropped): the digit counts of every pass are
// order-independent, so one upfront pass over the keys gives each pass's
// global digit bases; a pass then ranks its 4096-pair tile in LDS, publishes
// the tile's per-digit counts and gets the counts of all earlier tiles by a
// decoupled look-back per digit (a thread follows its digits back through the
// tiles' status words until an inclusive prefix; tiles take tickets in
// dispatch order, so every tile it waits on is running), and writes each
// digit's run of the tile contiguously from LDS.  Ranking is wave-private (no
// barrier inside the loop): wave w owns the tile's w-th eighth in input order
// and ranks each 64-key chunk by match-any over the DB digit bits (DB ballots)
// against a wave-private LDS histogram; the waves' counts are then
// prefix-summed per digit, so the order within a digit is the input order
// (stable).  The last pass may write gw_event {key & mask, value} instead of
// the two arrays.
constexpr int RS2_NT = 512;                          // 8 waves per tile: short serial ranking loops
constexpr int RS2_NW = RS2_NT / 64;
constexpr int RS2_TILE = 4096;
constexpr int RS2_WAVE_KEYS = RS2_TILE / RS2_NW;     // 512 per wave
constexpr int RS2_CHUNKS = RS2_WAVE_KEYS / 64;      // 8
constexpr int RS2_MAX_PASSES = 4;
constexpr int RS2_MAX_RADIX = 256;                  // DB = 8
constexpr int RS2_STATUS_PER_TILE = RS2_MAX_PASSES * RS2_MAX_RADIX;   // status words per tile
constexpr int RS2_GBLOCKS = 1024;                   // blocks of the upfront histogram (grid-stride)
constexpr uint32_t OS_AGG = 1u << 30, OS_INC = 2u << 30, OS_VAL = (1u << 30) - 1;
constexpr int OS_LB = 4;                             // predecessors a look-back step reads

template <int DB>
struct OsCfg {
    static constexpr int RD = 1 << DB;                                  // digits
    static constexpr int MAXP = RS2_MAX_PASSES;
    static constexpr int DPT = RD > RS2_NT ? RD / RS2_NT : 1;           // digits per pass thread
    static constexpr int DT = RD / DPT;                                 // pass threads owning digits
    static_assert(MAXP * RD <= RS2_STATUS_PER_TILE, "status words per tile");
};

// digit totals of every pass (wave-private LDS copies: the top digit of a key
// has few distinct values, so one shared copy would serialise its bins'
// atomics; grid-stride), added into the zeroed totals[p][d]
template <int DB, int KS = 1>   // KS: u32 words from one key to the next (2: packed pairs, key in the low word)
__global__ void __launch_bounds__(NT) k_os_hist(const uint32_t* __restrict__ keys, const uint64_t* n_dev,
                                                uint64_t n_max, int lo_bit, int passes, uint32_t* __restrict__ totals) {
    using C = OsCfg<DB>;
    __shared__ uint32_t h[NWAVE][C::MAXP][C::RD];
    const int w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < NWAVE * C::MAXP * C::RD; i += NT) (&h[0][0][0])[i] = 0;
    __syncthreads();
    const uint64_t n = load_n(n_max, n_dev);
    for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * NT) {
        const uint32_t k = keys[i * KS];
        for (int p = 0; p < passes; ++p) atomicAdd(&h[w][p][(k >> (lo_bit + DB * p)) & (C::RD - 1)], 1u);
    }
    __syncthreads();
    for (int p = 0; p < passes; ++p)
        for (int d = threadIdx.x; d < C::RD; d += NT) {
            uint32_t v = 0;
#pragma unroll
            for (int q = 0; q < NWAVE; ++q) v += h[q][p][d];
            if (v) atomicAdd(&totals[p * RS2_MAX_RADIX + d], v);
        }
}
// global digit bases per pass (block p): an exclusive scan over the digits,
// thread t owning digits [t*DPB, (t+1)*DPB)
template <int DB>
__global__ void __launch_bounds__(NT) k_os_bases(const uint32_t* __restrict__ totals, uint32_t* __restrict__ gbase) {
    using C = OsCfg<DB>;
    constexpr int DPB = C::RD / NT;
    __shared__ uint32_t red[NWAVE];
    const uint32_t p = blockIdx.x;
    uint32_t v[DPB], s = 0;
#pragma unroll
    for (int u = 0; u < DPB; ++u) {
        v[u] = totals[p * RS2_MAX_RADIX + threadIdx.x * DPB + u];
        s += v[u];
    }
    uint32_t all;
    uint32_t pre = block_excl_scan<uint32_t>(s, red, all);
#pragma unroll
    for (int u = 0; u < DPB; ++u) {
        gbase[p * RS2_MAX_RADIX + threadIdx.x * DPB + u] = pre;
        pre += v[u];
    }
}

__device__ __forceinline__ uint32_t os_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void os_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// P64: the pairs are packed u64 (value << 32 | key) in kin / kout (vin / vout unused): one
// 8-B load and one 8-B store per pair, a digit's run of a tile one contiguous segment
template <int DB, bool P64 = false>
__global__ void __launch_bounds__(RS2_NT) k_os_pass(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                    gw_event* __restrict__ aos, uint32_t aos_mask,
                                                    const uint64_t* n_dev, uint64_t n_max, int shift,
                                                    const uint32_t* __restrict__ gbase, uint32_t* __restrict__ status,
                                                    unsigned long long* __restrict__ ticket) {
    using C = OsCfg<DB>;
    constexpr uint32_t DM = C::RD - 1;
    // one 32-KB region: the waves' 16-bit digit counts while ranking, then the
    // tile's pairs in digit order (every position is in registers by then):
    // 40 KB of LDS at DB = 10, four tiles per CU
    __shared__ uint32_t region[2 * RS2_TILE];
    __shared__ uint32_t tstart[C::RD], gofs[C::RD], red[RS2_NW];
    __shared__ uint32_t s_tile;
    static_assert(RS2_NW * C::RD * 2 <= (int)sizeof(region), "wave counts fit the pair region");
    uint16_t(*whist)[C::RD] = reinterpret_cast<uint16_t(*)[C::RD]>(region);
    uint32_t* sk = region;
    uint32_t* sv = region + RS2_TILE;
    const int t = threadIdx.x, w = t >> 6, ln = lane_id();
    if (t == 0) s_tile = (uint32_t)atomicAdd(ticket, 1ull);
    for (int i = t; i < RS2_NW * C::RD / 2; i += RS2_NT) region[i] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t n = load_n(n_max, n_dev);
    const uint64_t base = (uint64_t)tile * RS2_TILE;
    if (base >= n) return;                                   // block-uniform; no later tile waits on it
    const uint64_t lt = lanemask_lt();
    uint32_t key[RS2_CHUNKS], val[RS2_CHUNKS], rk[RS2_CHUNKS];
    const uint64_t wbase = base + (uint64_t)w * RS2_WAVE_KEYS;
#pragma unroll
    for (int c = 0; c < RS2_CHUNKS; ++c) {                   // loads first: all in flight together
        const uint64_t i = wbase + (uint64_t)c * 64 + ln;
        if (P64) {
            const uint64_t x = i < n ? reinterpret_cast<const uint64_t*>(kin)[i] : 0ull;
            key[c] = (uint32_t)x;
            val[c] = (uint32_t)(x >> 32);
        } else {
            key[c] = i < n ? kin[i] : 0u;
            val[c] = i < n ? vin[i] : 0u;
        }
    }
    uint16_t* hw = whist[w];
#pragma unroll
    for (int c = 0; c < RS2_CHUNKS; ++c) {
        const uint64_t i = wbase + (uint64_t)c * 64 + ln;
        const bool valid = i < n;
        const uint32_t d = (key[c] >> shift) & DM;
        uint64_t peers = wave_ballot(valid);
#pragma unroll
        for (int b = 0; b < DB; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = wave_ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t r = (uint32_t)popc64(peers & lt);
        const uint32_t old = valid ? hw[d] : 0u;             // same-digit lanes read the same count
        __builtin_amdgcn_wave_barrier();
        if (valid && r == 0) hw[d] = (uint16_t)(old + (uint32_t)popc64(peers));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        rk[c] = valid ? old + r : 0xffffffffu;
    }
    __syncthreads();
    // thread t < DT owns digits [t*DPT, (t+1)*DPT): prefix over the waves, the
    // tile's global offset per digit by a look-back over earlier tiles, then
    // the tile's digit starts by a scan over the digits
    uint32_t run[C::DPT], tsum = 0;
    if (t < C::DT) {
#pragma unroll
        for (int u = 0; u < C::DPT; ++u) {
            const uint32_t d = (uint32_t)t * C::DPT + u;
            uint32_t r = 0;
#pragma unroll
            for (int k = 0; k < RS2_NW; ++k) { const uint32_t v = whist[k][d]; whist[k][d] = (uint16_t)r; r += v; }
            run[u] = r;
            tsum += r;
            os_st(status + (uint64_t)tile * C::RD + d, (tile == 0 ? OS_INC : OS_AGG) | r);
        }
#pragma unroll
        for (int u = 0; u < C::DPT; ++u) {
            // the look-back reads OS_LB predecessors per step (their loads in
            // flight together) and consumes them nearest first, up to the first
            // inclusive prefix or the first word not posted yet (re-read from
            // there): a walk over many aggregate-only tiles is OS_LB times shorter
            const uint32_t d = (uint32_t)t * C::DPT + u;
            uint32_t excl = 0;
            int64_t j = (int64_t)tile - 1;
            while (j >= 0) {
                uint32_t v[OS_LB];
#pragma unroll
                for (int q = 0; q < OS_LB; ++q)
                    v[q] = j - q >= 0 ? os_ld(status + (uint64_t)(j - q) * C::RD + d) : OS_INC;
                bool done = false;
                int used = 0;
#pragma unroll
                for (int q = 0; q < OS_LB; ++q) {
                    if (done || used < q || !(v[q] & (OS_AGG | OS_INC))) continue;
                    excl += v[q] & OS_VAL;
                    ++used;
                    done = (v[q] & OS_INC) != 0;
                }
                if (done) break;
                j -= used;
            }
            if (tile) os_st(status + (uint64_t)tile * C::RD + d, OS_INC | (excl + run[u]));
            gofs[d] = gbase[d] + excl;
        }
    }
    const uint32_t inc = wave_incl_scan<uint32_t>(t < C::DT ? tsum : 0u);
    if (ln == 63) red[w] = inc;
    __syncthreads();
    if (t < C::DT) {
        uint32_t pre = 0;
#pragma unroll
        for (int k = 0; k < RS2_NW; ++k) pre += (k < w) ? red[k] : 0u;
        pre += inc - tsum;
#pragma unroll
        for (int u = 0; u < C::DPT; ++u) {
            tstart[t * C::DPT + u] = pre;
            pre += run[u];
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < RS2_CHUNKS; ++c) {                   // positions to registers: the counts' region
        if (rk[c] == 0xffffffffu) continue;                  // becomes the pair buffer below
        const uint32_t d = (key[c] >> shift) & DM;
        rk[c] += tstart[d] + hw[d];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < RS2_CHUNKS; ++c) {
        if (rk[c] == 0xffffffffu) continue;
        sk[rk[c]] = key[c];
        sv[rk[c]] = val[c];
    }
    __syncthreads();
    const uint32_t tn = (uint32_t)min<uint64_t>((uint64_t)RS2_TILE, n - base);
    for (uint32_t i = t; i < tn; i += RS2_NT) {              // each digit's run of the tile is contiguous
        const uint32_t k = sk[i], v = sv[i];
        const uint32_t d = (k >> shift) & DM;
        const uint32_t dst = gofs[d] + (i - tstart[d]);
        if (P64) {
            reinterpret_cast<uint64_t*>(kout)[dst] = ((uint64_t)v << 32) | k;
        } else if (aos) {
            gw_event e;
            e.watcher = k & aos_mask;
            e.target = v;
            aos[dst] = e;
        } else {
            kout[dst] = k;
            vout[dst] = v;
        }
    }
}

inline uint64_t radix2_tiles(uint64_t n_max) { return (n_max + RS2_TILE - 1) / RS2_TILE; }
// scratch words radix_sort2 needs for n_max pairs: tickets (8 words), digit
// totals and bases ([MAX_PASSES][MAX_RADIX] each), status ([tiles][<= 4096])
inline uint64_t radix2_scratch_words(uint64_t n_max) {
    return 8 + 2ull * RS2_MAX_PASSES * RS2_MAX_RADIX + (uint64_t)RS2_STATUS_PER_TILE * radix2_tiles(n_max);
}

template <int DB, bool P64 = false>
inline int radix_sort2_db(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n_max,
                          const uint64_t* n_dev, int lo_bit, int passes, uint32_t* scratch, hipStream_t st,
                          gw_event* aos, uint32_t aos_mask) {
    using C = OsCfg<DB>;
    const uint64_t nt = radix2_tiles(n_max);
    unsigned long long* tickets = (unsigned long long*)scratch;                 // [MAX_PASSES]
    uint32_t* totals = scratch + 8;                                             // [MAX_PASSES][MAX_RADIX]
    uint32_t* status = totals + RS2_MAX_PASSES * RS2_MAX_RADIX;                 // [passes][tiles][RD]
    uint32_t* gbase = status + (uint64_t)RS2_STATUS_PER_TILE * nt;              // [MAX_PASSES][MAX_RADIX]
    // tickets, totals and the status words of the passes used start at zero
    (void)hipMemsetAsync(scratch, 0, 32 + (uint64_t)RS2_MAX_PASSES * RS2_MAX_RADIX * 4 +
                                         (uint64_t)passes * C::RD * nt * 4, st);
    hipLaunchKernelGGL((k_os_hist<DB, P64 ? 2 : 1>), dim3(RS2_GBLOCKS), dim3(NT), 0, st, k0, n_dev, n_max, lo_bit,
                       passes, totals);
    hipLaunchKernelGGL(k_os_bases<DB>, dim3(passes), dim3(NT), 0, st, totals, gbase);
    int cur = 0;
    for (int p = 0; p < passes; ++p) {
        const bool last = p == passes - 1;
        uint32_t* ki = cur ? k1 : k0; uint32_t* ko = cur ? k0 : k1;
        uint32_t* vi = cur ? v1 : v0; uint32_t* vo = cur ? v0 : v1;
        hipLaunchKernelGGL((k_os_pass<DB, P64>), dim3((uint32_t)nt), dim3(RS2_NT), 0, st, ki, vi, ko, vo,
                           last ? aos : nullptr, aos_mask, n_dev, n_max, lo_bit + DB * p,
                           gbase + p * RS2_MAX_RADIX, status + (uint64_t)p * C::RD * nt, tickets + p);
        cur ^= 1;
    }
    return cur;
}

// Sorts (k0,v0) by bits [lo_bit, hi_bit) (at most 32 bits) with (k1,v1) as
// ping-pong; scratch holds radix2_scratch_words(n_max) u32 (no clearing
// needed by the caller).  Digit width: 8 bits.  With aos, the last pass
// writes gw_event {key & aos_mask, value} there (and the return value is
// meaningless).  Returns 0 if the result is in (k0,v0), 1 if in (k1,v1).
inline int radix_sort2(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint64_t n_max, const uint64_t* n_dev,
                       int lo_bit, int hi_bit, uint32_t* scratch, hipStream_t st,
                       gw_event* aos = nullptr, uint32_t aos_mask = 0xffffffffu) {
    const uint64_t nt = radix2_tiles(n_max);
    if (nt == 0 || hi_bit <= lo_bit) return 0;
    const int bits = hi_bit - lo_bit;
    return radix_sort2_db<8>(k0, v0, k1, v1, n_max, n_dev, lo_bit, (bits + 7) / 8, scratch, st, aos, aos_mask);
}

// The same for packed pairs (u64: value << 32 | key) in p0 with p1 as ping-pong.
// Returns 0 if the result is in p0, 1 if in p1.
inline int radix_sort2_p64(uint64_t* p0, uint64_t* p1, uint64_t n_max, const uint64_t* n_dev, int lo_bit, int hi_bit,
                           uint32_t* scratch, hipStream_t st) {
    const uint64_t nt = radix2_tiles(n_max);
    if (nt == 0 || hi_bit <= lo_bit) return 0;
    const int bits = hi_bit - lo_bit;
    uint32_t* a = reinterpret_cast<uint32_t*>(p0);
    uint32_t* b = reinterpret_cast<uint32_t*>(p1);
    return radix_sort2_db<8, true>(a, nullptr, b, nullptr, n_max, n_dev, lo_bit, (bits + 7) / 8, scratch, st,
                                   nullptr, 0);
}

}  // namespace gw
