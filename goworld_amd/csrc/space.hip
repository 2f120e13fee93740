// space.hip — slot-range maintenance for the space lifecycle (capi.cpp
// gw_space_create / gw_space_grow / gw_space_destroy).
//
// The reference creates and destroys spaces at run time (goworld.go:52-60
// CreateSpaceLocally / CreateSpaceAnywhere -> SpaceManager.putSpace,
// Space.OnDestroy -> SpaceManager.delSpace, engine/entity/SpaceManager.go:
// 21-27, Space.go:143-151) and a space grows without bound (Space.enter,
// Space.go:179-217).  Here a space owns a contiguous range of slot-indexed
// state; growing it past the slots behind it moves the range, and a destroyed
// space's range is cleared and handed out again.  Three one-thread-per-slot
// passes, HBM-bound copies (a few hundred bytes per slot), run only on those
// calls, never per tick.
#include "dev_common.hpp"

namespace gw {

namespace {

// state of slot src + i -> slot dst + i.  The destination range is clear (all
// zero flags), so its sync bits are set with an OR; the source is cleared by
// k_slots_clear afterwards (same stream).
__global__ void __launch_bounds__(NT) k_slots_move(World w, OpLast* __restrict__ ol, uint4* __restrict__ eid,
                                                    uint4* __restrict__ cid, uint32_t src, uint32_t dst, uint32_t n) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = src + i, d = dst + i;
    w.rec[d] = w.rec[s];               // (its grid offset is rebuilt with the grid)
    w.gate[d] = w.gate[s];
    w.nbc[d] = 0;                      // cached neighbour counts are recomputed (the epoch moves on)
    ol[d] = ol[s];
    eid[d] = eid[s];
    cid[d] = cid[s];
    const uint32_t f = flag_get(w.flags, s);
    if (f) atomicOr(&w.flags[flag_word(d)], f << flag_sh(d));
}

// slots base + i: absent, in space `meta`, no flags, no client, no ids
__global__ void __launch_bounds__(NT) k_slots_clear(World w, OpLast* __restrict__ ol, uint4* __restrict__ eid,
                                                     uint4* __restrict__ cid, uint32_t base, uint32_t n,
                                                     uint32_t meta) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = base + i;
    AoiEnt a;
    a.x = 0.f;
    a.z = 0.f;
    a.seq = -1;
    a.meta = meta;
    w.rec[s].a = a;
    PrevEnt p;
    p.ox = 0.f;
    p.oz = 0.f;
    p.ostamp = 0ull;
    w.rec[s].pv = p;
    w.rec[s].stamp = 0ull;
    w.rec[s].p = make_float4(0.f, 0.f, 0.f, 0.f);
    w.gate[s] = 0;
    w.rec[s].gate = 0;
    w.nbc[s] = 0ull;
    OpLast z{};
    ol[s] = z;
    eid[s] = make_uint4(0u, 0u, 0u, 0u);
    cid[s] = make_uint4(0u, 0u, 0u, 0u);
    if (flag_get(w.flags, s)) atomicAnd(&w.flags[flag_word(s)], ~(3u << flag_sh(s)));
}

// entities present in [base, base + n): one add per wave
__global__ void __launch_bounds__(NT) k_count_present(const SlotRec* __restrict__ rec, uint32_t base, uint32_t n,
                                                       unsigned long long* out) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    const bool p = i < n && (rec[base + i].a.meta & PRESENT_BIT) != 0;
    const uint64_t bm = wave_ballot(p);
    if (lane_id() == 0 && bm) atomicAdd(out, (unsigned long long)popc64(bm));
}

}  // namespace

void launch_slots_move(const World& w, OpLast* ol, uint4* eid, uint4* cid, uint32_t src, uint32_t dst, uint32_t n,
                       hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_slots_move, dim3(nblk(n, NT)), dim3(NT), 0, s, w, ol, eid, cid, src, dst, n);
}

void launch_slots_clear(const World& w, OpLast* ol, uint4* eid, uint4* cid, uint32_t base, uint32_t n,
                        uint32_t meta, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_slots_clear, dim3(nblk(n, NT)), dim3(NT), 0, s, w, ol, eid, cid, base, n, meta);
}

void launch_count_present(const SlotRec* rec, uint32_t base, uint32_t n, unsigned long long* out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_count_present, dim3(nblk(n, NT)), dim3(NT), 0, s, rec, base, n, out);
}

}  // namespace gw
