// prim.hpp — wave64 / LDS primitives for gfx950: wave scans, block scans,
// three-phase device exclusive scan, and a stable LSD radix sort whose
// per-block ranking uses wavefront ballots (match-any over the digit bits).
//
// Everything here is HBM-bound integer work: no MFMA.  Tiles are sized for
// 256-thread workgroups (4 waves of 64 lanes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

__device__ __forceinline__ uint64_t load_n(uint64_t n_max, const uint64_t* n_dev) {
    if (!n_dev) return n_max;
    uint64_t n = *n_dev;
    return n < n_max ? n : n_max;
}

// ---------------------------------------------------------------------------
// Device exclusive scan: out[i] = sum(in[0..i)), *total = sum(in[0..n)).
// Phase 1 reduces 4096-element tiles, phase 2 scans the tile sums in one
// workgroup, phase 3 rescans each tile with its carry.
constexpr int SCAN_IPT = 16;
constexpr int SCAN_TILE = NT * SCAN_IPT;

template <typename TI, typename TO>
__global__ void __launch_bounds__(NT) k_scan_reduce(const TI* __restrict__ in, uint64_t n_max,
                                                    const uint64_t* n_dev, TO* __restrict__ partial) {
    __shared__ TO lds[NWAVE];
    uint64_t n = load_n(n_max, n_dev);
    uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    TO s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_IPT; ++j) {
        uint64_t i = base + (uint64_t)j * NT + threadIdx.x;
        if (i < n) s += (TO)in[i];
    }
    TO tot;
    block_excl_scan<TO>(s, lds, tot);
    if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

template <typename TO>
__global__ void __launch_bounds__(NT) k_scan_partials(TO* __restrict__ partial, uint32_t nb, TO* total_out) {
    __shared__ TO lds[NWAVE];
    TO carry = 0;
    for (uint32_t base = 0; base < nb; base += NT * 4) {
        TO v[4];
        TO s = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t i = base + threadIdx.x * 4 + j;
            v[j] = i < nb ? partial[i] : (TO)0;
            s += v[j];
        }
        TO tot;
        TO pre = block_excl_scan<TO>(s, lds, tot);
        TO run = carry + pre;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t i = base + threadIdx.x * 4 + j;
            if (i < nb) partial[i] = run;
            run += v[j];
        }
        carry += tot;
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

template <typename TI, typename TO>
__global__ void __launch_bounds__(NT) k_scan_down(const TI* __restrict__ in, TO* __restrict__ out,
                                                  uint64_t n_max, const uint64_t* n_dev,
                                                  const TO* __restrict__ partial) {
    __shared__ TO lds[NWAVE];
    uint64_t n = load_n(n_max, n_dev);
    uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_IPT;
    TO v[SCAN_IPT];
    TO s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_IPT; ++j) {
        uint64_t i = base + j;
        v[j] = i < n ? (TO)in[i] : (TO)0;
        s += v[j];
    }
    TO tot;
    TO run = block_excl_scan<TO>(s, lds, tot) + partial[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SCAN_IPT; ++j) {
        uint64_t i = base + j;
        if (i < n) out[i] = run;
        run += v[j];
    }
}

// host launcher: tmp must hold ceil(n_max/SCAN_TILE) elements of TO.
template <typename TI, typename TO>
inline void scan_exclusive(const TI* in, TO* out, uint64_t n_max, const uint64_t* n_dev,
                           TO* tmp, TO* total_dev, hipStream_t st) {
    uint32_t nb = (uint32_t)((n_max + SCAN_TILE - 1) / SCAN_TILE);
    if (nb == 0) nb = 1;
    hipLaunchKernelGGL((k_scan_reduce<TI, TO>), dim3(nb), dim3(NT), 0, st, in, n_max, n_dev, tmp);
    hipLaunchKernelGGL((k_scan_partials<TO>), dim3(1), dim3(NT), 0, st, tmp, nb, total_dev);
    if (out)
        hipLaunchKernelGGL((k_scan_down<TI, TO>), dim3(nb), dim3(NT), 0, st, in, out, n_max, n_dev, tmp);
}
inline uint64_t scan_tmp_elems(uint64_t n_max) { return (n_max + SCAN_TILE - 1) / SCAN_TILE + 1; }

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
                      int lo_bit, int hi_bit, const RadixTmp& tmp, hipStream_t st) {
    uint32_t nb = (uint32_t)radix_blocks(n_max);
    if (nb == 0) return 0;
    int cur = 0;
    for (int shift = lo_bit; shift < hi_bit; shift += 8) {
        K* ki = cur ? k1 : k0; K* ko = cur ? k0 : k1;
        uint32_t* vi = cur ? v1 : v0; uint32_t* vo = cur ? v0 : v1;
        hipLaunchKernelGGL((k_rs_hist<K>), dim3(nb), dim3(NT), 0, st, ki, n_max, n_dev, shift, tmp.hist, nb);
        scan_exclusive<uint32_t, uint32_t>(tmp.hist, tmp.hist, (uint64_t)RS_RADIX * nb, nullptr,
                                           tmp.scan_tmp, tmp.scan_total, st);
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

}  // namespace gw
