// world.cpp — RCCL communicator of a context and the decomposed world
// (include/gpuaoi.h gw_comm_* / gw_world_*).
//
// The reference keeps a space inside one game process (engine/entity/
// SpaceManager.go:11-31); splitting one huge space into X-strips over GPUs is
// new capability.  go-aoi's relation is a pure function of the two positions
// and of which member made the later AOI call, so a strip needs no neighbour
// lists from its neighbours, only the state of the entities near its borders:
// the owner of an entity forwards the net effect of its ops of the tick as
// halo rows (gw_route_halo, halo.hip) and every rank orders all ops by global
// stamps.  Per tick on every rank, all on the context's stream:
//   stamps (iota) -> route into send buffers sized for the worst case (n
//   entities per side, so they cannot overflow) -> RCCL exchange of the two
//   row counts -> one host sync -> RCCL exchange of exactly the used rows ->
//   the tick's op stream = owned ops (stamped) + both neighbours' rows.
// Point-to-point with <= 2 peers per rank (one xGMI link each); the volumes are
// small (a few thousand entities x 96 B per border), so the exact-size second
// round costs a host round trip but never sends padding.
#include <cmath>
#include <cstring>

#include "ctx.hpp"

using namespace gw;
using namespace gw::host;

namespace {

constexpr uint64_t STAMP_STRIDE = 1ull << 26;   // stamp = 1 + (tick * ranks + rank) * 2^26 + op index
constexpr uint32_t ROWS = 3;                    // rows per routed entity (gw_route_halo)

#define NCCLCHK(expr)                                                                            \
    do {                                                                                         \
        ncclResult_t _r = (expr);                                                                \
        if (_r != ncclSuccess)                                                                   \
            return set_err(c, GW_EDEVICE, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r), \
                           __FILE__, __LINE__);                                                  \
    } while (0)

// dworld.Strips geometry, in double like the Python statement, rounded to float32 where the device compares
double strip_lo(const gw_world_geom& g, int r) { return r == 0 ? -INFINITY : (double)g.x0 + r * (double)g.strip_w; }
double strip_hi(const gw_world_geom& g, int r) {
    return r == (int)g.ranks - 1 ? INFINITY : (double)g.x0 + (r + 1) * (double)g.strip_w;
}
// smallest float32 >= v (x >= lo <=> x >= that float32 for float32 x); +-3e38 for the open ends
float f32_ceil(double v, int side) {
    if (!std::isfinite(v)) return side < 0 ? -3.0e38f : 3.0e38f;
    float f = (float)v;
    if ((double)f < v) f = std::nextafterf(f, INFINITY);
    return f;
}

// the routing launch of one world tick (both paths): neighbour rows into the
// send buffers, far triples (long moves) into the far buffer
int route_launch(gw_ctx* c, const gw_op* ops, uint32_t n, const HaloDsts& D, uint32_t tag, unsigned long long base) {
    WorldHost& W = c->wd;
    HaloFar F{};
    if (W.far_cap) {
        F.rows = P<gw_halo_row>(W.far_rows);
        F.dest = P<uint32_t>(W.far_dest);
        F.cap = W.far_cap;
    }
    F.cnt = P<uint32_t>(W.far_cnt);
    F.ext = P<float>(W.ext);
    F.nranks = W.g.ranks;
    F.self = W.g.rank;
    if (!W.long_cap) {                                // the long-mover list (group teleports)
        if (int rc = ensure(c, W.longs, 256 * sizeof(gw_long_move))) return rc;
        W.long_cap = 256;
    }
    F.longs = P<gw_long_move>(W.longs);
    F.long_cap = W.long_cap;
    // without a far buffer the long moves are still counted (F.rows null:
    // nothing placed); a rank of 1 or 2 strips has no far destination, but the
    // owner's own copy may still need its LEAVE row
    if (!F.rows) {
        if (int rc = ensure(c, W.far_rows, 1024 * ROWS * sizeof(gw_halo_row))) return rc;
        if (int rc = ensure(c, W.far_dest, 1024 * 4)) return rc;
        W.far_cap = 1024;
        F.rows = P<gw_halo_row>(W.far_rows);
        F.dest = P<uint32_t>(W.far_dest);
        F.cap = W.far_cap;
    }
    launch_route_halo(world_of(c), ops, P<unsigned long long>(W.stamps), n, W.g.max_step, D, c->ol, tag, c->halo,
                      c->st, /*pad=*/false, P<unsigned long long>(W.stamps), base, &F);   // stamps by r1
    HIPCHK(hipGetLastError());
    return 0;
}

// words of the routing's counts in WorldHost::pub_h: HaloStats first, then
// the 4 received counts (rows from left / right, long movers from left / right)
constexpr size_t pub_off_cnt() { return (sizeof(HaloStats) + 3) / 4; }
constexpr size_t RCNT = 4;

// the routing's counts (HaloStats, the far / long counts, and with rcnt the
// received counts, with far_mat the all-gathered count vectors) into pub_h by
// one kernel, the host sync, then into hs / the vectors
int read_route_counts(gw_ctx* c, HaloStats& hs, uint32_t* rcnt, bool far_mat) {
    WorldHost& W = c->wd;
    const uint32_t R = W.g.ranks, R1 = R + FAR_EXTRA;
    const size_t o_cnt = pub_off_cnt(), o_far = o_cnt + RCNT, o_mat = o_far + R1;
    PubSeg segs[4];
    int n = 0;
    segs[n++] = PubSeg{(const uint32_t*)c->halo, W.pub_d, (uint32_t)o_cnt};
    segs[n++] = PubSeg{P<uint32_t>(W.far_cnt), W.pub_d + o_far, R1};
    if (rcnt) segs[n++] = PubSeg{P<uint32_t>(W.cnt), W.pub_d + o_cnt, (uint32_t)RCNT};
    if (far_mat) segs[n++] = PubSeg{P<uint32_t>(W.far_mat), W.pub_d + o_mat, R * R1};
    publish_words(segs, n, c->st);
    HIPCHK(hipStreamSynchronize(c->st));
    memcpy(&hs, W.pub_h, sizeof hs);
    memcpy(W.far_cnt_h.data(), W.pub_h + o_far, (size_t)R1 * 4);
    if (rcnt) memcpy(rcnt, W.pub_h + o_cnt, RCNT * 4);
    if (far_mat) memcpy(W.far_mat_h.data(), W.pub_h + o_mat, (size_t)R * R1 * 4);
    return 0;
}

// after the routing's host sync (hs, cnt read back): a far buffer too small
// is grown and the routing rerun (idempotent: same session, same stamps,
// same counts); then the far triples are grouped by destination
int far_settle(gw_ctx* c, const gw_op* ops, uint32_t n, const HaloDsts& D, uint32_t tag, unsigned long long base,
               HaloStats& hs) {
    WorldHost& W = c->wd;
    int rc;
    if (hs.far_n > W.far_cap || hs.long_n > W.long_cap) {
        if (hs.far_n > W.far_cap) {
            const uint32_t cap = hs.far_n + hs.far_n / 2 + 64;
            if ((rc = ensure(c, W.far_rows, (size_t)cap * ROWS * sizeof(gw_halo_row))) ||
                (rc = ensure(c, W.far_dest, (size_t)cap * 4)))
                return rc;
            W.far_cap = cap;
        }
        if (hs.long_n > W.long_cap) {
            const uint32_t cap = hs.long_n + hs.long_n / 2 + 64;
            if ((rc = ensure(c, W.longs, (size_t)cap * sizeof(gw_long_move)))) return rc;
            W.long_cap = cap;
        }
        // the rerun places the same rows again; the accumulating counters
        // (overflow, conflicts, bad ops, long moves) must not count them twice
        unsigned long long keep[4] = {hs.overflow, hs.conflicts, hs.bad_ops, hs.long_moves};
        if ((rc = route_launch(c, ops, n, D, tag, base))) return rc;
        HIPCHK(hipMemcpyAsync(c->halo, keep, sizeof keep, hipMemcpyHostToDevice, c->st));
        HIPCHK(hipMemcpyAsync(&hs, c->halo, sizeof hs, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        if (hs.far_n > W.far_cap || hs.long_n > W.long_cap)
            return set_err(c, GW_ENOMEM, "far halo rows / long-mover list overflowed twice");
    }
    W.own_nlong = hs.long_n;
    uint32_t acc = 0;
    for (uint32_t q = 0; q < W.g.ranks; ++q) {
        W.far_off_h[q] = acc;
        acc += W.far_cnt_h[q];
    }
    if (acc != hs.far_n) return set_err(c, GW_EDEVICE, "far halo counts disagree (%u vs %u)", acc, hs.far_n);
    if (!acc) return 0;
    if ((rc = ensure(c, W.far_sorted, (size_t)acc * ROWS * sizeof(gw_halo_row)))) return rc;
    HIPCHK(hipMemcpyAsync(W.far_off.p, W.far_off_h.data(), (size_t)W.g.ranks * 4, hipMemcpyHostToDevice, c->st));
    launch_far_partition(P<gw_halo_row>(W.far_rows), P<uint32_t>(W.far_dest), acc, P<uint32_t>(W.far_off),
                         P<uint32_t>(W.far_cursor), W.g.ranks, P<gw_halo_row>(W.far_sorted), c->st);
    HIPCHK(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

int gw_comm_unique_id(void* id) {
    if (!id) return GW_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return GW_EDEVICE;
    memcpy(id, &u, sizeof u);
    return 0;
}

int gw_comm_init(gw_ctx* c, const void* id, int nranks, int rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return GW_EINVAL;
    if (xp_on(c)) return set_err(c, GW_ESTATE, "communicator already initialised");
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    NCCLCHK(ncclCommInitRank(&c->comm, nranks, u, rank));
    c->c_nranks = nranks;
    c->c_rank = rank;
    return 0;
}

int gw_comm_info(gw_ctx* c, int* nranks, int* rank) {
    if (!c) return GW_EINVAL;
    if (nranks) *nranks = xp_on(c) ? c->c_nranks : 0;
    if (rank) *rank = xp_on(c) ? c->c_rank : 0;
    return 0;
}

int gw_comm_exchange(gw_ctx* c, const gw_xfer* x, uint32_t n) {
    if (!c || (n && !x)) return GW_EINVAL;
    if (!xp_on(c)) return set_err(c, GW_ESTATE, "no communicator (gw_comm_init)");
    for (uint32_t i = 0; i < n; ++i)
        if (x[i].peer < 0 || x[i].peer >= c->c_nranks || (x[i].send_bytes && !x[i].send) ||
            (x[i].recv_bytes && !x[i].recv))
            return set_err(c, GW_EINVAL, "bad transfer %u", i);
    int rc;
    if ((rc = xp_group_start(c))) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        if (x[i].send_bytes) (void)xp_send(c, x[i].send, x[i].send_bytes, x[i].peer);
        if (x[i].recv_bytes) (void)xp_recv(c, x[i].recv, x[i].recv_bytes, x[i].peer);
    }
    return xp_group_end(c);
}

int gw_comm_allreduce_u64(gw_ctx* c, uint64_t* dev, uint32_t n, int op) {
    if (!c || (n && !dev) || (op != GW_RED_SUM && op != GW_RED_MAX)) return GW_EINVAL;
    if (!xp_on(c)) return set_err(c, GW_ESTATE, "no communicator (gw_comm_init)");
    return xp_allreduce_u64(c, (unsigned long long*)dev, n, op);
}

int gw_world_create(gw_ctx* c, const gw_world_geom* g, uint32_t capacity, const float* bounds, uint32_t* space_id) {
    if (!c || !g) return GW_EINVAL;
    if (c->wd.on) return set_err(c, GW_ESTATE, "the context already holds a world strip");
    if (g->ranks < 1 || g->rank >= g->ranks || !(g->strip_w > 0) || !(g->aoi_dist > 0) || !(g->max_step >= 0) ||
        !std::isfinite(g->x0))
        return set_err(c, GW_EINVAL, "bad world geometry");
    WorldHost& W = c->wd;
    W.g = *g;
    W.h = (double)g->aoi_dist + 2.0 * g->max_step + 1.0 +
          1e-5 * (std::fabs((double)g->x0) + g->ranks * (double)g->strip_w);
    if (g->ranks > 2 && !(g->strip_w > W.h + g->max_step))
        return set_err(c, GW_EINVAL, "strip width %g must exceed halo %g + max_step %g", g->strip_w, W.h,
                       g->max_step);
    const int r = (int)g->rank;
    for (int side = 0; side < 2; ++side) {
        const int nb = side == 0 ? r - 1 : r + 1;
        W.nb[side] = (nb >= 0 && nb < (int)g->ranks) ? nb : -1;
        if (W.nb[side] >= 0) {
            W.ext_lo[side] = (float)(strip_lo(*g, nb) - W.h);
            W.ext_hi[side] = (float)(strip_hi(*g, nb) + W.h);
        }
    }
    W.ext_h.assign(2 * (size_t)g->ranks, 0.f);
    for (uint32_t q = 0; q < g->ranks; ++q) {
        W.ext_h[2 * q] = (float)(strip_lo(*g, (int)q) - W.h);
        W.ext_h[2 * q + 1] = (float)(strip_hi(*g, (int)q) + W.h);
    }
    // the world's buffers first: a failure leaves no space behind (a retry
    // must find the context empty, the strip's space at slot base 0)
    int rc2;
    if ((rc2 = ensure(c, W.ext, W.ext_h.size() * 4)) ||
        (rc2 = ensure(c, W.far_cnt, ((size_t)g->ranks + FAR_EXTRA) * 4)) ||
        (rc2 = ensure(c, W.far_off, (size_t)g->ranks * 4)) || (rc2 = ensure(c, W.far_cursor, (size_t)g->ranks * 4)) ||
        (rc2 = ensure(c, W.far_mat, (size_t)g->ranks * (g->ranks + FAR_EXTRA) * 4)))
        return rc2;
    HIPCHK(hipMemcpyAsync(W.ext.p, W.ext_h.data(), W.ext_h.size() * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (W.pub_h) (void)hipHostFree(W.pub_h);
    W.pub_h = W.pub_d = nullptr;
    const size_t pub_words = pub_off_cnt() + RCNT + (g->ranks + FAR_EXTRA) + (size_t)g->ranks * (g->ranks + FAR_EXTRA);
    if (hipHostMalloc((void**)&W.pub_h, pub_words * 4, hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&W.pub_d, W.pub_h, 0) != hipSuccess)
        return set_err(c, GW_ENOMEM, "world count buffer");
    uint32_t sid = 0, base = 0;
    if (int rc = gw_space_create(c, g->aoi_dist, capacity, bounds, &sid, &base)) return rc;
    if (base != 0) {
        (void)gw_space_destroy(c, sid);
        return set_err(c, GW_ESTATE, "a world strip must be the context's first space (slot = id)");
    }
    if (int rc = gw_space_set_ownership(c, sid, f32_ceil(strip_lo(*g, r), -1), f32_ceil(strip_hi(*g, r), 1))) {
        std::string keep = c->err;
        (void)gw_space_destroy(c, sid);
        c->err = keep;
        return rc;
    }
    W.far_cnt_h.assign(g->ranks + FAR_EXTRA, 0);
    W.far_off_h.assign(g->ranks, 0);
    W.far_mat_h.assign((size_t)g->ranks * (g->ranks + FAR_EXTRA), 0);
    W.own_nlong = 0;
    W.tick_longs = nullptr;
    W.tick_nlong = 0;
    W.far_cap = 0;
    W.sid = sid & SID_MASK;
    W.tick = 0;
    W.on = true;
    if (space_id) *space_id = sid;
    return 0;
}

int gw_world_route(gw_ctx* c, const gw_op* ops, uint32_t n, const gw_halo_row* send[2], uint32_t send_rows[2]) {
    if (!c || (n && !ops)) return GW_EINVAL;
    WorldHost& W = c->wd;
    if (!W.on) return set_err(c, GW_ESTATE, "no world strip (gw_world_create)");
    if (W.routed) return set_err(c, GW_ESTATE, "tick already routed: gw_world_submit first");
    if (W.ol_pre) return set_err(c, GW_ESTATE, "the last routed world tick was not ticked (gw_tick first)");
    if ((uint64_t)n >= STAMP_STRIDE) return set_err(c, GW_ERANGE, "too many ops in one tick for the stamp layout");
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    int rc;
    const uint64_t cap_ent = std::max<uint64_t>(n, 1);   // an entity is routed at most once per side
    if ((rc = ensure(c, W.stamps, (size_t)cap_ent * 8)) || (rc = ensure(c, W.cnt, 64))) return rc;
    HaloDsts D{};
    for (int side = 0; side < 2; ++side) {
        if (W.nb[side] < 0) continue;
        if ((rc = ensure(c, W.send[side], (size_t)cap_ent * ROWS * sizeof(gw_halo_row)))) return rc;
        D.d[D.n++] = HaloDst{W.ext_lo[side], W.ext_hi[side], P<gw_halo_row>(W.send[side]), (uint32_t)cap_ent};
    }
    const unsigned long long base = 1 + (W.tick * W.g.ranks + W.g.rank) * STAMP_STRIDE;
    uint32_t tag = 0;
    if ((rc = next_ol_tag(c, &tag))) return rc;      // the tick reuses this session (gw_world_submit)
    if ((rc = route_launch(c, ops, n, D, tag, base))) return rc;
    W.kept = n;
    W.kept_tag = tag;
    HaloStats hs{};
    if ((rc = read_route_counts(c, hs, nullptr, false))) return rc;
    if ((rc = far_settle(c, ops, n, D, tag, base, hs))) return rc;
    uint32_t k = 0;
    for (int side = 0; side < 2; ++side) {
        W.send_cnt[side] = 0;
        if (W.nb[side] < 0) continue;
        W.send_cnt[side] = std::min<uint32_t>(hs.cnt[k++], (uint32_t)cap_ent);
    }
    W.ops = ops;
    W.n_ops = n;
    W.routed = true;
    for (int side = 0; side < 2; ++side) {
        if (send) send[side] = W.nb[side] >= 0 ? P<gw_halo_row>(W.send[side]) : nullptr;
        if (send_rows) send_rows[side] = W.send_cnt[side] * ROWS;
    }
    return 0;
}

int gw_world_submit(gw_ctx* c, const gw_halo_row* const recv[2], const uint32_t recv_rows[2]) {
    if (!c) return GW_EINVAL;
    WorldHost& W = c->wd;
    if (!W.routed) return set_err(c, GW_ESTATE, "gw_world_route first");
    // everything is checked before anything is queued: a failed submit leaves
    // the routed tick in place (the caller may retry with the right rows)
    for (int side = 0; side < 2; ++side) {
        const uint32_t nr = recv_rows ? recv_rows[side] : 0;
        if (nr && (!recv || !recv[side])) return set_err(c, GW_EINVAL, "rows from side %d missing", side);
        if (nr && W.nb[side] < 0) return set_err(c, GW_EINVAL, "rows from side %d, which has no neighbour", side);
        if (nr % ROWS) return set_err(c, GW_EINVAL, "side %d: %u rows, not whole entities", side, nr);
    }
    if (!c->segs.empty()) return set_err(c, GW_ESTATE, "ops queued outside the world tick: gw_tick first");
    W.routed = false;
    ++W.tick;
    const size_t nseg = c->segs.size();
    int rc = gw_submit_device_stamped(c, W.ops, (const uint64_t*)W.stamps.p, W.n_ops);
    for (int side = 0; side < 2 && !rc; ++side) {
        const uint32_t nr = recv_rows ? recv_rows[side] : 0;
        if (nr) rc = gw_submit_device_rows(c, recv[side], nr);
    }
    if (rc) {                                         // nothing of this tick stays queued
        c->segs.resize(nseg);
        W.kept = 0;                                   // (the session's words age out)
        W.ol_pre = 0;
        return rc;
    }
    W.ol_pre = W.kept;                   // the tick's stream starts with the routed ops (gw_tick checks)
    W.kept = 0;
    W.submitted = true;                  // far rows may join until gw_tick
    return 0;
}

int gw_world_step(gw_ctx* c, const gw_op* ops, uint32_t n) {
    if (!c) return GW_EINVAL;
    WorldHost& W = c->wd;
    if (!W.on) return set_err(c, GW_ESTATE, "no world strip (gw_world_create)");
    if (W.ol_pre) return set_err(c, GW_ESTATE, "the last routed world tick was not ticked (gw_tick first)");
    if (W.routed) return set_err(c, GW_ESTATE, "tick already routed: gw_world_submit first");
    const bool any_nb = W.nb[0] >= 0 || W.nb[1] >= 0;
    if (any_nb && (!xp_on(c) || c->c_nranks != (int)W.g.ranks || c->c_rank != (int)W.g.rank))
        return set_err(c, GW_ESTATE, "world of %u ranks needs a matching communicator (gw_comm_init)", W.g.ranks);
    if ((uint64_t)n >= STAMP_STRIDE) return set_err(c, GW_ERANGE, "too many ops in one tick for the stamp layout");
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    int rc;
    const uint64_t cap_ent = std::max<uint64_t>(n, 1);
    if ((rc = ensure(c, W.stamps, (size_t)cap_ent * 8)) || (rc = ensure(c, W.cnt, 64))) return rc;
    HaloDsts D{};
    for (int side = 0; side < 2; ++side) {
        if (W.nb[side] < 0) continue;
        if ((rc = ensure(c, W.send[side], (size_t)cap_ent * ROWS * sizeof(gw_halo_row)))) return rc;
        D.d[D.n++] = HaloDst{W.ext_lo[side], W.ext_hi[side], P<gw_halo_row>(W.send[side]), (uint32_t)cap_ent};
    }
    const unsigned long long base = 1 + (W.tick * W.g.ranks + W.g.rank) * STAMP_STRIDE;
    if (!D.n) launch_iota_u64(P<unsigned long long>(W.stamps), base, n, c->st);
    uint32_t tag = 0;
    if (D.n) {                                        // a one-strip world has nobody to route to
        if ((rc = next_ol_tag(c, &tag))) return rc;  // the tick reuses this session (gw_world_submit)
        if ((rc = route_launch(c, ops, n, D, tag, base))) return rc;
        W.kept = n;
        W.kept_tag = tag;
    }
    HIPCHK(hipGetLastError());
    const uint32_t R = W.g.ranks, me = W.g.rank, R1 = R + FAR_EXTRA;
    const bool far_round = R >= 3;                    // ranks that are not neighbours exist
    uint32_t rcnt[2] = {0, 0};
    uint32_t far_in = 0;                              // triples received from far ranks
    uint32_t n_long = 0;                              // long movers of all ranks (group teleports)
    if (any_nb) {
        // round 1, the counts.  Two ranks: the entity count (u32) and the
        // long-mover count both ways (HaloStats.cnt[k] is the k-th destination
        // of D, i.e. left first when both exist).  More: ONE all-gather of every
        // rank's count vector (far triples per rank, long movers, entities to
        // its left / right neighbour) instead of a neighbour round and an
        // all-gather
        uint32_t k = 0;
        if (!far_round) {
            uint32_t* dcnt = P<uint32_t>(W.cnt);     // [0..1] rows from left / right, [2..3] long movers
            if ((rc = xp_group_start(c))) return rc;
            for (int side = 0; side < 2; ++side) {
                if (W.nb[side] < 0) continue;
                (void)xp_send(c, &c->halo->cnt[k++], 4, W.nb[side]);
                (void)xp_recv(c, dcnt + side, 4, W.nb[side]);
                (void)xp_send(c, P<uint32_t>(W.far_cnt) + R, 4, W.nb[side]);
                (void)xp_recv(c, dcnt + 2 + side, 4, W.nb[side]);
            }
            if ((rc = xp_group_end(c))) return rc;
        } else if ((rc = xp_allgather(c, W.far_cnt.p, W.far_mat.p, (size_t)R1 * 4))) {
            return rc;
        }
        uint32_t h[RCNT] = {0, 0, 0, 0};
        HaloStats hs{};
        if ((rc = read_route_counts(c, hs, far_round ? nullptr : h, far_round))) return rc;
        if (far_round) {                             // the neighbours' entity counts towards this rank
            if (me > 0) h[0] = W.far_mat_h[(size_t)(me - 1) * R1 + R + 3];    // left neighbour's "to the right"
            if (me + 1 < R) h[1] = W.far_mat_h[(size_t)(me + 1) * R1 + R + 2];   // right neighbour's "to the left"
        }
        if ((rc = far_settle(c, ops, n, D, tag, base, hs))) return rc;
        k = 0;
        for (int side = 0; side < 2; ++side) {
            W.send_cnt[side] = 0;
            if (W.nb[side] < 0) continue;
            W.send_cnt[side] = std::min<uint32_t>(hs.cnt[k++], (uint32_t)cap_ent);
            rcnt[side] = h[side];
            if ((rc = ensure(c, W.recv[side], (size_t)std::max<uint32_t>(rcnt[side], 1) * ROWS * sizeof(gw_halo_row))))
                return rc;
        }
        if (far_round) {
            for (uint32_t p = 0; p < R; ++p)
                if (p != me) far_in += W.far_mat_h[(size_t)p * R1 + me];
            if (far_in && (rc = ensure(c, W.far_recv, (size_t)far_in * ROWS * sizeof(gw_halo_row)))) return rc;
        }
        // every rank's long-mover list into long_all, in rank order
        auto nlong = [&](uint32_t p) -> uint32_t {
            if (p == me) return W.own_nlong;
            if (far_round) return W.far_mat_h[(size_t)p * R1 + R];
            return h[2 + (p < me ? 0 : 1)];
        };
        for (uint32_t p = 0; p < R; ++p) n_long += nlong(p);
        if (n_long) {
            if ((rc = ensure(c, W.long_all, (size_t)n_long * sizeof(gw_long_move)))) return rc;
            size_t off = 0;
            for (uint32_t p = 0; p < me; ++p) off += nlong(p);
            if (W.own_nlong)
                HIPCHK(hipMemcpyAsync(P<gw_long_move>(W.long_all) + off, W.longs.p, (size_t)W.own_nlong *
                                      sizeof(gw_long_move), hipMemcpyDeviceToDevice, c->st));
        }
        // round 2: exactly the used rows (neighbours), and the far triples
        if ((rc = xp_group_start(c))) return rc;
        for (int side = 0; side < 2; ++side) {
            if (W.nb[side] < 0) continue;
            if (W.send_cnt[side])
                (void)xp_send(c, W.send[side].p, (size_t)W.send_cnt[side] * ROWS * sizeof(gw_halo_row), W.nb[side]);
            if (rcnt[side])
                (void)xp_recv(c, W.recv[side].p, (size_t)rcnt[side] * ROWS * sizeof(gw_halo_row), W.nb[side]);
        }
        if (n_long) {                                 // the long lists: everyone's to everyone
            size_t off = 0;
            for (uint32_t p = 0; p < R; ++p) {
                const uint32_t np_ = nlong(p);
                if (p != me && (far_round || p + 1 == me || p == me + 1)) {
                    if (W.own_nlong) (void)xp_send(c, W.longs.p, (size_t)W.own_nlong * sizeof(gw_long_move), (int)p);
                    if (np_)
                        (void)xp_recv(c, P<gw_long_move>(W.long_all) + off, (size_t)np_ * sizeof(gw_long_move), (int)p);
                }
                off += np_;
            }
        }
        if (far_round) {
            size_t roff = 0;
            for (uint32_t p = 0; p < R; ++p) {
                if (p == me) continue;
                const uint32_t out = W.far_cnt_h[p], in = W.far_mat_h[(size_t)p * R1 + me];
                if (out)
                    (void)xp_send(c, P<gw_halo_row>(W.far_sorted) + (size_t)W.far_off_h[p] * ROWS,
                                  (size_t)out * ROWS * sizeof(gw_halo_row), (int)p);
                if (in)
                    (void)xp_recv(c, P<gw_halo_row>(W.far_recv) + roff * ROWS, (size_t)in * ROWS * sizeof(gw_halo_row),
                                  (int)p);
                roff += in;
            }
        }
        if ((rc = xp_group_end(c))) return rc;
    }
    W.ops = ops;
    W.n_ops = n;
    W.routed = true;
    const gw_halo_row* recv[2] = {P<gw_halo_row>(W.recv[0]), P<gw_halo_row>(W.recv[1])};
    const uint32_t rrows[2] = {rcnt[0] * ROWS, rcnt[1] * ROWS};
    if ((rc = gw_world_submit(c, recv, rrows))) return rc;
    // this rank's own LEAVE rows (long movers that left its range), then the far rows received
    const uint32_t self_n = any_nb ? W.far_cnt_h[me] : 0;
    if (self_n && (rc = gw_submit_device_rows(c, P<gw_halo_row>(W.far_sorted) + (size_t)W.far_off_h[me] * ROWS,
                                              self_n * ROWS)))
        return rc;
    if (far_in && (rc = gw_submit_device_rows(c, P<gw_halo_row>(W.far_recv), far_in * ROWS))) return rc;
    W.tick_longs = n_long ? P<gw_long_move>(W.long_all) : nullptr;
    W.tick_nlong = n_long;
    return 0;
}

int gw_world_stage_ops(gw_ctx* c, const gw_op* ops, uint32_t n, const gw_op** dev_ops) {
    if (!c || !dev_ops || (n && !ops)) return GW_EINVAL;
    *dev_ops = nullptr;
    WorldHost& W = c->wd;
    if (!W.on) return set_err(c, GW_ESTATE, "no world strip (gw_world_create)");
    if (W.routed || W.ol_pre || W.submitted)      // the staged ops of a queued tick are still to be read
        return set_err(c, GW_ESTATE, "a world tick is pending (gw_world_submit / gw_tick first)");
    if ((uint64_t)n >= STAMP_STRIDE) return set_err(c, GW_ERANGE, "too many ops in one tick for the stamp layout");
    // what the host can check without the entity state (the owner's presence
    // is on the device): kind, slot inside the world's id range, finite x/z
    const uint32_t cap = c->spaces[W.sid].cap;
    for (uint32_t i = 0; i < n; ++i) {
        const gw_op& o = ops[i];
        if (o.kind < GW_OP_ENTER || o.kind > GW_OP_SYNC || o.reserved)
            return set_err(c, GW_EINVAL, "op %u: bad kind %u / reserved %u", i, o.kind, o.reserved);
        if (o.slot >= cap) return set_err(c, GW_ERANGE, "op %u: entity %u outside the world (%u ids)", i, o.slot, cap);
        if ((o.kind == GW_OP_ENTER || o.kind == GW_OP_MOVED) && !(std::isfinite(o.x) && std::isfinite(o.z)))
            return set_err(c, GW_EINVAL, "op %u: non-finite coordinates", i);
    }
    (void)hipSetDevice(c->dev);
    if (!W.staged) HIPCHK(hipEventCreateWithFlags(&W.staged, hipEventDisableTiming));
    HIPCHK(hipEventSynchronize(W.staged));           // the last upload has left the pinned buffer
    const size_t bytes = (size_t)std::max<uint32_t>(n, 1) * sizeof(gw_op);
    int rc;
    if ((rc = ensure_host(c, W.hstage, bytes)) || (rc = ensure(c, W.dstage, bytes))) return rc;
    if (n) {
        memcpy(W.hstage.p, ops, (size_t)n * sizeof(gw_op));
        HIPCHK(hipMemcpyAsync(W.dstage.p, W.hstage.p, (size_t)n * sizeof(gw_op), hipMemcpyHostToDevice, c->st));
    }
    HIPCHK(hipEventRecord(W.staged, c->st));
    *dev_ops = P<gw_op>(W.dstage);
    return 0;
}

int gw_world_step_host(gw_ctx* c, const gw_op* ops, uint32_t n) {
    const gw_op* dev = nullptr;
    if (int rc = gw_world_stage_ops(c, ops, n, &dev)) return rc;
    return gw_world_step(c, dev, n);
}

int gw_world_far(gw_ctx* c, const gw_halo_row** rows, const uint32_t** counts) {
    if (!c) return GW_EINVAL;
    WorldHost& W = c->wd;
    if (!W.on) return set_err(c, GW_ESTATE, "no world strip (gw_world_create)");
    if (rows) *rows = W.far_sorted.p ? P<gw_halo_row>(W.far_sorted) : nullptr;
    if (counts) *counts = W.far_cnt_h.data();
    return 0;
}

int gw_world_submit_far(gw_ctx* c, const gw_halo_row* rows, uint32_t n_rows) {
    if (!c || (n_rows && !rows)) return GW_EINVAL;
    WorldHost& W = c->wd;
    if (!W.on) return set_err(c, GW_ESTATE, "no world strip (gw_world_create)");
    if (W.routed || !W.submitted) return set_err(c, GW_ESTATE, "gw_world_submit first (far rows join its tick)");
    if (n_rows % ROWS) return set_err(c, GW_EINVAL, "%u rows: not whole entities", n_rows);
    return gw_submit_device_rows(c, rows, n_rows);
}

int gw_world_longs(gw_ctx* c, const gw_long_move** rows, uint32_t* n) {
    if (!c) return GW_EINVAL;
    WorldHost& W = c->wd;
    if (!W.on) return set_err(c, GW_ESTATE, "no world strip (gw_world_create)");
    if (rows) *rows = W.own_nlong ? P<gw_long_move>(W.longs) : nullptr;
    if (n) *n = W.own_nlong;
    return 0;
}

int gw_world_submit_longs(gw_ctx* c, const gw_long_move* rows, uint32_t n) {
    if (!c || (n && !rows)) return GW_EINVAL;
    WorldHost& W = c->wd;
    if (!W.on) return set_err(c, GW_ESTATE, "no world strip (gw_world_create)");
    if (W.routed || !W.submitted) return set_err(c, GW_ESTATE, "gw_world_submit first (the lists join its tick)");
    W.tick_longs = n ? rows : nullptr;
    W.tick_nlong = n;
    return 0;
}

int gw_world_status(gw_ctx* c, uint64_t* overflow, uint64_t* conflicts, uint64_t* bad_ops) {
    if (!c) return GW_EINVAL;
    if (int rs = settle(c)) return rs;
    (void)hipSetDevice(c->dev);
    if (c->wd.conflicts_acc) {                       // the ticks' conflicts (DevStats, counted per attempt)
        HaloStats h0{};
        HIPCHK(hipMemcpyAsync(&h0, c->halo, sizeof h0, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        h0.conflicts += c->wd.conflicts_acc;
        c->wd.conflicts_acc = 0;
        HIPCHK(hipMemcpyAsync(c->halo, &h0, sizeof h0, hipMemcpyHostToDevice, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
    }
    if (xp_on(c) && c->c_nranks > 1) {                // the three counters are the first three u64 of HaloStats
        if (int rc = xp_allreduce_u64(c, (unsigned long long*)c->halo, 3, GW_RED_SUM)) return rc;
    }
    HaloStats h{};
    HIPCHK(hipMemcpyAsync(&h, c->halo, sizeof h, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemsetAsync(c->halo, 0, sizeof h, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (overflow) *overflow = h.overflow;
    if (conflicts) *conflicts = h.conflicts;
    if (bad_ops) *bad_ops = h.bad_ops;
    return 0;
}

}  // extern "C"
