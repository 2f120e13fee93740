// halo.hip — owner-side routing of a decomposed world (gw_route_halo).
//
// A strip process forwards, for each entity its ops touched this tick, the
// net effect those ops have on a neighbour's copy (goworld_amd/dworld.py
// module doc).  The entity state before the tick IS the
// routing state: AoiEnt (x, present), flags (sync flags pending since the
// last collect).  Three light passes over the owned ops, O(ops), no host sync:
//   r1  last AOI op / last payload op / last Leave per slot (u64 atomicMax
//       into the session-tagged OpLast words, exactly k_ops1 of the tick,
//       which reuses them); the ops' stamps in the world path
//   r2  the fix-up of r1's plain stores where a slot has several ops; r1
//       also keeps, per sync bit, the last non-Leave op setting it (r3 compares
//       it with the last Leave clearing the bit: a Leave's sync_flags is the
//       mask of bits it keeps, as in the tick)
//   r3  the entity's last op writes up to 3 rows per destination, entities
//       placed by one counter add per block and destination
//   r4  (fixed-size buffers only) zero (NOP) rows past the entities placed
// Nothing is reset afterwards: the words age out with their session tag.  The
// placement counters are zeroed by r1 of the next call.  Integer/byte work
// bound by the latency of the per-slot gathers; no LDS or MFMA.
#include "dev_common.hpp"

namespace gw {

namespace {

constexpr uint32_t ROWS = 3;

__device__ __forceinline__ bool op_valid(const gw_op& op, uint32_t cap) {
    return op.kind >= GW_OP_ENTER && op.kind <= GW_OP_SYNC && op.slot < cap;
}

__global__ void __launch_bounds__(NT) k_route1(const gw_op* __restrict__ ops, uint32_t n, uint32_t cap,
                                                OpLast* ol, uint32_t tag, HaloStats* hs,
                                                unsigned long long* stamps_out, unsigned long long stamp_base,
                                                HaloFar F) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i == 0) hs->cnt[0] = hs->cnt[1] = hs->far_n = hs->long_n = 0;   // placement counters of this call
    if (F.cnt && i < F.nranks + FAR_EXTRA) F.cnt[i] = 0;
    if (i >= n) return;
    if (stamps_out) stamps_out[i] = stamp_base + i;
    const gw_op op = ops[i];
    if (op.kind == GW_OP_NOP) return;
    if (!op_valid(op, cap)) {
        atomicAdd(&hs->bad_ops, 1ull);
        return;
    }
    // plain stores of the tagged index (as k_ops1): the fix-up in k_route2
    // takes the maximum only where a slot has several ops (device-scope
    // atomics run memory-side: one per word and op cost the pass its latency)
    const unsigned long long v = ol_put(tag, i);
    OpLast& o = ol[op.slot];
    if (op.kind != GW_OP_LEAVE) {
        o.pos = v;
        for (int c = 0; c < 2; ++c)                  // the last op setting bit c (rb[c], compared with clr[c])
            if ((op.sync_flags >> c) & 1) o.rb[c] = v;
    }
    if (op.kind != GW_OP_SYNC) o.aoi = v;
    if (op.kind == GW_OP_LEAVE) {
        o.leave = v;
        for (int c = 0; c < 2; ++c)
            if (!((op.sync_flags >> c) & 1)) o.clr[c] = v;
    }
}

// the fix-up: an op whose index is above the stored one takes the maximum
// (only where a slot had several ops this call)
__global__ void __launch_bounds__(NT) k_route2(const gw_op* __restrict__ ops, uint32_t n, uint32_t cap,
                                                OpLast* ol, uint32_t tag) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const gw_op op = ops[i];
    if (op.kind == GW_OP_NOP || !op_valid(op, cap)) return;
    const unsigned long long v = ol_put(tag, i);
    OpLast& w = ol[op.slot];
    const OpLast o = w;
    const int32_t me = (int32_t)i;
    if (op.kind != GW_OP_LEAVE) {
        if (ol_get(o.pos, tag) < me) atomicMax(&w.pos, v);
        for (int c = 0; c < 2; ++c)
            if (((op.sync_flags >> c) & 1) && ol_get(o.rb[c], tag) < me) atomicMax(&w.rb[c], v);
    }
    if (op.kind != GW_OP_SYNC && ol_get(o.aoi, tag) < me) atomicMax(&w.aoi, v);
    if (op.kind == GW_OP_LEAVE) {
        if (ol_get(o.leave, tag) < me) atomicMax(&w.leave, v);
        for (int c = 0; c < 2; ++c)
            if (!((op.sync_flags >> c) & 1) && ol_get(o.clr[c], tag) < me) atomicMax(&w.clr[c], v);
    }
}

__device__ __forceinline__ gw_op mk_op(uint8_t kind, uint8_t flags, uint32_t slot, const gw_op* payload,
                                       uint16_t res = 0) {
    gw_op o;
    o.kind = kind;
    o.sync_flags = flags;
    o.reserved = res;
    o.slot = slot;
    if (payload) {
        o.x = payload->x; o.y = payload->y; o.z = payload->z; o.yaw = payload->yaw;
    } else {
        o.x = o.y = o.z = o.yaw = 0.f;
    }
    return o;
}

__device__ __forceinline__ void put_row(gw_halo_row* r, const gw_op& o, unsigned long long stamp) {
    r->op = o;
    r->stamp = stamp;
}

// the three rows of an entity for a destination holding [lo, hi): LEAVE
// (left and re-entered inside the tick) / the net AOI change / SYNC
struct RowKinds {
    uint8_t k0, k1, k2;
};
__device__ __forceinline__ RowKinds row_kinds(bool was, bool now, int32_t la, int32_t ll, int32_t lp, uint32_t f) {
    RowKinds k{GW_OP_NOP, GW_OP_NOP, GW_OP_NOP};
    if (la >= 0) {
        if (ll >= 0 && was && now) k.k0 = GW_OP_LEAVE;
        if (now && (!was || ll >= 0)) k.k1 = GW_OP_ENTER;
        else if (was && now) k.k1 = GW_OP_MOVED;
        else if (was) k.k1 = GW_OP_LEAVE;
    }
    if (now && (f != 0 || lp > la)) k.k2 = GW_OP_SYNC;
    return k;
}

__device__ __forceinline__ void put_triple(gw_halo_row* r, const RowKinds& k, uint32_t s, const gw_op& oa,
                                           const gw_op& op_pos, uint32_t f, uint16_t res,
                                           const unsigned long long* stamps, int32_t ll, int32_t la, uint32_t i) {
    const gw_op nop = mk_op(GW_OP_NOP, 0, 0, nullptr);
    put_row(r + 0, k.k0 ? mk_op(k.k0, 0, s, nullptr, res) : nop, k.k0 ? stamps[ll] : 0ull);
    put_row(r + 1, k.k1 ? mk_op(k.k1, 0, s, &oa, res) : nop, k.k1 ? stamps[la] : 0ull);
    put_row(r + 2, k.k2 ? mk_op(k.k2, (uint8_t)f, s, &op_pos) : nop, k.k2 ? stamps[i] : 0ull);
}

// a far triple (long moves only: rare, one atomic each)
__device__ __forceinline__ void put_far(const HaloFar& F, HaloStats* hs, uint32_t q, const RowKinds& k, uint32_t s,
                                        const gw_op& oa, const gw_op& op_pos, uint32_t f,
                                        const unsigned long long* stamps, int32_t ll, int32_t la, uint32_t i) {
    atomicAdd(&F.cnt[q], 1u);                        // counted even past the buffer: the exchange sizes
    const uint32_t t = atomicAdd(&hs->far_n, 1u);
    if (t >= F.cap) return;                          // the host grows the buffer and routes again
    put_triple(F.rows + (size_t)t * ROWS, k, s, oa, op_pos, f, RES_LONG, stamps, ll, la, i);
    F.dest[t] = q;
}

// Entities are placed in a destination's buffer by one counter add per block
// and destination (the waves' ballots summed in LDS): one add per wave put a
// few thousand adds on each of two words per call, which serialise
// memory-side (a 16M world's 8-strip rank, 200k ops: route 74 -> 57 us with
// 1024-thread blocks).  Small calls keep 256-thread blocks (a 1M world's
// 8-strip rank, 12.5k ops: 1024-thread blocks cost it 4 us).
template <uint32_t RNT>
__global__ void __launch_bounds__(RNT) k_route3(const gw_op* __restrict__ ops, const unsigned long long* __restrict__ stamps,
                                                uint32_t n, World w, const OpLast* __restrict__ ol, uint32_t tag,
                                                float max_step, HaloDsts D, HaloStats* hs, HaloFar F) {
    constexpr uint32_t RNW = RNT / 64;
    __shared__ uint32_t s_cnt[2][RNW];
    __shared__ uint32_t s_base[2];
    const uint32_t i = blockIdx.x * RNT + threadIdx.x;
    // every lane reaches the wave-aggregated appends below
    bool rep = false;
    uint32_t s = 0;
    int32_t la = -1, ll = -1, lp = -1;
    if (i < n) {
        const gw_op op = ops[i];
        if (op_valid(op, w.cap)) {
            s = op.slot;
            la = ol_get(ol[s].aoi, tag);
            ll = ol_get(ol[s].leave, tag);
            lp = ol_get(ol[s].pos, tag);
            rep = (int32_t)i == max(lp, ll);          // the entity's last op
        }
    }
    bool old_p = false, new_p = false, lng = false;
    float old_x = 0.f, new_x = 0.f;
    uint32_t f = 0;
    gw_op oa{}, op_pos{};
    if (rep) {
        const AoiEnt a = w.rec[s].a;
        old_p = (a.meta & PRESENT_BIT) != 0;
        old_x = a.x;
        new_p = old_p;
        new_x = old_x;
        if (la >= 0) {
            oa = ops[la];
            new_p = oa.kind != GW_OP_LEAVE;
            if (new_p) new_x = oa.x;
            // a long move (a teleport: Entity.SetPosition has no step bound,
            // Entity.go:1185-1187): routed to every rank holding either end
            lng = old_p && new_p && fabsf(new_x - old_x) > max_step;
            if (lng) atomicAdd(&hs->long_moves, 1ull);
        }
        if (lp >= 0) op_pos = ops[lp];
        // syncInfoFlag after the tick's ops (k_ops3 / k_place): old bits a Leave
        // did not clear, OR'd with the bits set since the Leave that cleared them
        uint32_t keep = 0, rbits = 0;
        for (int c = 0; c < 2; ++c) {
            const int32_t lc = ol_get(ol[s].clr[c], tag);
            if (lc < 0) keep |= 1u << c;
            if (ol_get(ol[s].rb[c], tag) > lc) rbits |= 1u << c;   // bit c set after the last Leave clearing it
        }
        f = ((flag_get(w.flags, s) & keep) | rbits) & SIF_ROUTED;
    }
    const uint16_t res = lng ? RES_LONG : 0;
    const uint32_t wv = threadIdx.x >> 6;
    RowKinds k[2];
    bool emit[2];
    uint64_t bm[2];
#pragma unroll
    for (uint32_t d = 0; d < 2; ++d) {
        k[d] = RowKinds{GW_OP_NOP, GW_OP_NOP, GW_OP_NOP};
        emit[d] = false;
        if (d < D.n && rep) {
            const HaloDst& dst = D.d[d];
            const bool was = old_p && old_x >= dst.x_lo && old_x < dst.x_hi;
            const bool now = new_p && new_x >= dst.x_lo && new_x < dst.x_hi;
            k[d] = row_kinds(was, now, la, ll, lp, f);
            emit[d] = (k[d].k0 | k[d].k1 | k[d].k2) != 0;
        }
        bm[d] = wave_ballot(emit[d]);
        if (lane_id() == 0) s_cnt[d][wv] = (uint32_t)popc64(bm[d]);
    }
    __syncthreads();
    if (threadIdx.x < D.n) {
        const uint32_t d = threadIdx.x;
        uint32_t tot = 0;
        for (uint32_t q = 0; q < RNW; ++q) tot += s_cnt[d][q];
        uint32_t base = 0;
        if (tot) {
            base = atomicAdd(&hs->cnt[d], tot);
            // the same count by side in the all-gathered vector (>= 3 ranks: it
            // replaces the neighbours' count round); one destination = the
            // outer rank's only neighbour
            if (F.cnt) atomicAdd(&F.cnt[F.nranks + 2 + (D.n == 2 ? d : (F.self == 0 ? 1u : 0u))], tot);
        }
        s_base[d] = base;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t d = 0; d < 2; ++d) {
        if (!emit[d]) continue;
        uint32_t e = s_base[d] + (uint32_t)popc64(bm[d] & lanemask_lt());
        for (uint32_t q = 0; q < wv; ++q) e += s_cnt[d][q];
        const HaloDst& dst = D.d[d];
        if (e >= dst.cap) {
            atomicAdd(&hs->overflow, 1ull);
            continue;
        }
        put_triple(dst.rows + (size_t)e * ROWS, k[d], s, oa, op_pos, f, res, stamps, ll, la, i);
    }
    if (lng && F.longs) {
        // the long-mover list (group teleports): state before and after the
        // tick, for the owner of every other long mover's new position
        atomicAdd(&F.cnt[F.nranks], 1u);
        const uint32_t t = atomicAdd(&hs->long_n, 1u);
        if (t < F.long_cap) {                         // else the host grows the list and routes again
            gw_long_move L;
            L.slot = s;
            L.reserved[0] = L.reserved[1] = L.reserved[2] = 0;
            L.old_x = old_x;
            L.old_z = w.rec[s].a.z;
            L.new_x = oa.x;
            L.new_z = oa.z;
            L.old_stamp = w.rec[s].stamp;             // the pre-tick state: the tick has not run
            L.new_stamp = stamps[la];
            F.longs[t] = L;
        }
    }
    if (lng && F.rows) {
        // every other rank (not this one, not a neighbour) holding either end
        for (uint32_t q = 0; q < F.nranks; ++q) {
            if (q + 1 >= F.self && q <= F.self + 1) continue;   // self and the neighbours
            const float lo = F.ext[2 * q], hi = F.ext[2 * q + 1];
            const bool was = old_x >= lo && old_x < hi, now = new_x >= lo && new_x < hi;
            if (!(was || now)) continue;
            put_far(F, hs, q, row_kinds(was, now, la, ll, lp, f), s, oa, op_pos, f, stamps, ll, la, i);
        }
        // this rank's own copy, if the entity left its held range: a LEAVE
        // (keep-mask 0) after the tick's own ops, so no copy stays outside
        const float lo = F.ext[2 * F.self], hi = F.ext[2 * F.self + 1];
        if (!(new_x >= lo && new_x < hi)) {
            RowKinds k{GW_OP_NOP, GW_OP_LEAVE, GW_OP_NOP};
            put_far(F, hs, F.self, k, s, oa, op_pos, 0, stamps, ll, la, i);
        }
    }
}

// zero (NOP) rows past the entities placed (fixed-size exchanges), so no
// memset of the buffers is needed; thread i: row i of each buffer
__global__ void __launch_bounds__(NT) k_route4(HaloDsts D, const HaloStats* __restrict__ hs) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    for (uint32_t d = 0; d < D.n; ++d) {
        const uint64_t used = (uint64_t)min(hs->cnt[d], D.d[d].cap) * ROWS;
        if (i >= used && i < (uint64_t)D.d[d].cap * ROWS) put_row(D.d[d].rows + i, mk_op(GW_OP_NOP, 0, 0, nullptr), 0ull);
    }
}

__global__ void __launch_bounds__(NT) k_split_rows(const gw_halo_row* __restrict__ rows, uint32_t n,
                                                    gw_op* __restrict__ ops, unsigned long long* __restrict__ stamps) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    ops[i] = rows[i].op;
    stamps[i] = rows[i].stamp;
}

// the tick's device segments (ops with or without stamps, halo rows) into
// one op stream by one launch (a copy per segment was a blit launch each:
// ~3.5 us apiece per world tick)
__global__ void __launch_bounds__(NT) k_gather_segs(SegTable t, gw_op* __restrict__ ops,
                                                    unsigned long long* __restrict__ stamps) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= t.total) return;
    uint32_t k = 0;
    while (k + 1 < t.n && i >= t.seg[k + 1].off) ++k;
    const SegTable::Seg& g = t.seg[k];
    const uint32_t j = i - g.off;
    if (g.rows) {
        const gw_halo_row r = g.rows[j];
        ops[i] = r.op;
        if (stamps) stamps[i] = r.stamp;
    } else {
        ops[i] = g.ops[j];
        if (stamps) stamps[i] = g.stamps[j];
    }
}

}  // namespace

void launch_gather_segs(const SegTable& t, gw_op* ops, unsigned long long* stamps, hipStream_t s) {
    if (t.total) hipLaunchKernelGGL(k_gather_segs, dim3(nblk1(t.total, NT)), dim3(NT), 0, s, t, ops, stamps);
}

void launch_route_halo(const World& w, const gw_op* ops, const unsigned long long* stamps, uint32_t n,
                       float max_step, const HaloDsts& D, OpLast* ol, uint32_t ol_tag, HaloStats* hs, hipStream_t s,
                       bool pad, unsigned long long* stamps_out, unsigned long long stamp_base, const HaloFar* far) {
    HaloFar F{};
    if (far) F = *far;
    const uint32_t nb = nblk1(std::max<uint32_t>(n, F.nranks + FAR_EXTRA), NT);
    uint64_t rows = 0;                                   // NOP padding up to the capacity (fixed-size exchanges)
    if (pad)
        for (uint32_t d = 0; d < D.n; ++d) rows = std::max<uint64_t>(rows, (uint64_t)D.d[d].cap * ROWS);
    hipLaunchKernelGGL(k_route1, dim3(nb), dim3(NT), 0, s, ops, n, w.cap, ol, ol_tag, hs, stamps_out, stamp_base, F);
    hipLaunchKernelGGL(k_route2, dim3(nb), dim3(NT), 0, s, ops, n, w.cap, ol, ol_tag);
    if (n >= 65536)
        hipLaunchKernelGGL(k_route3<1024>, dim3(nblk1(n, 1024)), dim3(1024), 0, s, ops, stamps, n, w, ol, ol_tag,
                           max_step, D, hs, F);
    else
        hipLaunchKernelGGL(k_route3<NT>, dim3(nblk1(std::max<uint32_t>(n, 1u), NT)), dim3(NT), 0, s, ops, stamps, n, w,
                           ol, ol_tag, max_step, D, hs, F);
    if (rows) hipLaunchKernelGGL(k_route4, dim3(nblk1(rows, NT)), dim3(NT), 0, s, D, hs);
}

__global__ void __launch_bounds__(NT) k_far_partition(const gw_halo_row* __restrict__ rows,
                                                       const uint32_t* __restrict__ dest, uint32_t n,
                                                       const uint32_t* __restrict__ off, uint32_t* cursor,
                                                       uint32_t nranks, gw_halo_row* __restrict__ out) {
    const uint32_t t = blockIdx.x * NT + threadIdx.x;
    if (t >= n) return;
    const uint32_t q = dest[t];
    if (q >= nranks) return;
    const uint32_t at = off[q] + atomicAdd(&cursor[q], 1u);
    for (uint32_t j = 0; j < ROWS; ++j) out[(size_t)at * ROWS + j] = rows[(size_t)t * ROWS + j];
}
__global__ void k_zero_u32(uint32_t* p, uint32_t n) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i < n) p[i] = 0;
}
void launch_far_partition(const gw_halo_row* rows, const uint32_t* dest, uint32_t n, const uint32_t* off,
                          uint32_t* cursor, uint32_t nranks, gw_halo_row* out, hipStream_t s) {
    hipLaunchKernelGGL(k_zero_u32, dim3(nblk1(nranks, NT)), dim3(NT), 0, s, cursor, nranks);
    if (n) hipLaunchKernelGGL(k_far_partition, dim3(nblk(n, NT)), dim3(NT), 0, s, rows, dest, n, off, cursor, nranks, out);
}

__global__ void __launch_bounds__(NT) k_iota_u64(unsigned long long* p, unsigned long long base, uint32_t n) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i < n) p[i] = base + i;
}
void launch_iota_u64(unsigned long long* p, unsigned long long base, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_iota_u64, dim3(nblk(n, NT)), dim3(NT), 0, s, p, base, n);
}

// loopback all-reduce (xport.cpp): out[i] = sum / max over the R gathered copies in[r * n + i]
__global__ void __launch_bounds__(NT) k_reduce_u64(const unsigned long long* __restrict__ in,
                                                    unsigned long long* __restrict__ out, uint32_t n, uint32_t R,
                                                    bool mx) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    unsigned long long v = in[i];
    for (uint32_t r = 1; r < R; ++r) {
        const unsigned long long x = in[(size_t)r * n + i];
        v = mx ? (x > v ? x : v) : v + x;
    }
    out[i] = v;
}
void launch_reduce_u64(const unsigned long long* in, unsigned long long* out, uint32_t n, uint32_t R, bool mx,
                       hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_reduce_u64, dim3(nblk(n, NT)), dim3(NT), 0, s, in, out, n, R, mx);
}

void launch_split_rows(const gw_halo_row* rows, uint32_t n, gw_op* ops, unsigned long long* stamps,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_split_rows, dim3(nblk1(n, NT)), dim3(NT), 0, s, rows, n, ops, stamps);
}

}  // namespace gw
