// xport.cpp — the transport of a context's data-path collectives
// (include/gpuaoi.h gw_comm_*; the decomposed world's exchange, world.cpp).
//
// Two transports behind one set of calls, both ordered on the context's
// stream and both with NCCL's point-to-point semantics (sends and receives of
// one group are matched per peer pair in issue order, counts must agree):
//   * RCCL (gw_comm_init): one process per GPU, xGMI;
//   * loopback (gw_comm_init_local): R contexts of ONE process, each driven by
//     its own host thread (the way R processes would drive them), bytes moved
//     by hipMemcpyAsync between the contexts' buffers.  It runs the world's
//     exact call sequence (count round, host read, far all-gather, exact-size
//     rows) with R ranks on one device, so that sequence is exercised before
//     any multi-GPU run (tests/test_gpu_loopback.py).
// Loopback group end, per rank: post every send (pointer, bytes and an event
// recorded on the sender's stream after the data was produced), then for each
// receive take the matching post, make the own stream wait on its event, copy,
// and hand back an event after the copy; finally make the own stream wait on
// the receivers' events of its own sends, so the send buffers are not reused
// before they were read (ncclSend completes when the peer has the data).
// Posts are made before any wait, so matched groups cannot deadlock; a rank
// whose peer never posts fails after GW_LOOPBACK_TIMEOUT_S (default 120 s)
// and marks the group broken, so its peers fail fast instead of hanging.
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>

#include "ctx.hpp"

using namespace gw;
using namespace gw::host;

namespace gw {
namespace host {

struct LocalGroup {
    int R = 0;
    int refs = 0;
    bool broken = false;
    std::mutex mu;
    std::condition_variable cv;
    struct Post {
        const void* p;
        size_t bytes;
        hipEvent_t ready;
    };
    std::vector<std::deque<Post>> posts;        // [src * R + dst] sends not yet received
    std::vector<std::deque<hipEvent_t>> done;   // [src * R + dst] receivers' copy-done events
    double timeout_s = 120.0;
};

namespace {

#define NCCLX(expr)                                                                              \
    do {                                                                                         \
        ncclResult_t _r = (expr);                                                                \
        if (_r != ncclSuccess)                                                                   \
            return set_err(c, GW_EDEVICE, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r), \
                           __FILE__, __LINE__);                                                  \
    } while (0)

int broken(gw_ctx* c, LocalGroup* G, const char* what) {
    {
        std::lock_guard<std::mutex> lk(G->mu);
        G->broken = true;
    }
    G->cv.notify_all();
    return set_err(c, GW_EDEVICE, "loopback group: %s", what);
}

// A HIP failure inside a loopback group end breaks the group (its flag set and
// the peers woken) before returning, so the peers fail at once instead of
// waiting out GW_LOOPBACK_TIMEOUT_S for posts or copies that never come
#define LGCHK(expr)                                                                              \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess) {                                                                  \
            char _m[256];                                                                        \
            snprintf(_m, sizeof _m, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
            return broken(c, G, _m);                                                             \
        }                                                                                        \
    } while (0)

int local_group_end(gw_ctx* c) {
    LocalGroup* G = c->lgrp;
    const int R = G->R, me = c->c_rank;
    std::vector<P2P> pend;
    pend.swap(c->xp_pend);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(G->timeout_s);
    for (const P2P& x : pend) {                      // 1. every send is posted before any wait
        if (!x.send) continue;
        hipEvent_t ev = nullptr;
        LGCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (hipError_t e = hipEventRecord(ev, c->st)) {
            (void)hipEventDestroy(ev);
            LGCHK(e);
        }
        std::lock_guard<std::mutex> lk(G->mu);
        G->posts[(size_t)me * R + x.peer].push_back(LocalGroup::Post{x.p, x.bytes, ev});
    }
    G->cv.notify_all();
    for (const P2P& x : pend) {                      // 2. receives, in issue order per peer
        if (x.send) continue;
        LocalGroup::Post po{};
        {
            std::unique_lock<std::mutex> lk(G->mu);
            auto& q = G->posts[(size_t)x.peer * R + me];
            if (!G->cv.wait_until(lk, deadline, [&] { return G->broken || !q.empty(); }))
                return lk.unlock(), broken(c, G, "a peer never sent (timeout)");
            if (G->broken && q.empty()) return set_err(c, GW_EDEVICE, "loopback group broken by a peer");
            po = q.front();
            q.pop_front();
        }
        if (po.bytes != x.bytes) {
            (void)hipEventDestroy(po.ready);
            char msg[128];
            snprintf(msg, sizeof msg, "rank %d sent %zu bytes, rank %d receives %zu", x.peer, po.bytes, me, x.bytes);
            return broken(c, G, msg);
        }
        const hipError_t we = hipStreamWaitEvent(c->st, po.ready, 0);
        (void)hipEventDestroy(po.ready);           // released once the recorded work completes (or on error)
        LGCHK(we);
        if (x.bytes) LGCHK(hipMemcpyAsync(x.p, po.p, x.bytes, hipMemcpyDeviceToDevice, c->st));
        hipEvent_t dn = nullptr;
        LGCHK(hipEventCreateWithFlags(&dn, hipEventDisableTiming));
        if (hipError_t e = hipEventRecord(dn, c->st)) {
            (void)hipEventDestroy(dn);
            LGCHK(e);
        }
        {
            std::lock_guard<std::mutex> lk(G->mu);
            G->done[(size_t)x.peer * R + me].push_back(dn);
        }
        G->cv.notify_all();
    }
    for (const P2P& x : pend) {                      // 3. a send completes when its receiver has copied
        if (!x.send) continue;
        hipEvent_t dn = nullptr;
        {
            std::unique_lock<std::mutex> lk(G->mu);
            auto& q = G->done[(size_t)me * R + x.peer];
            if (!G->cv.wait_until(lk, deadline, [&] { return G->broken || !q.empty(); }))
                return lk.unlock(), broken(c, G, "a peer never received (timeout)");
            if (G->broken && q.empty()) return set_err(c, GW_EDEVICE, "loopback group broken by a peer");
            dn = q.front();
            q.pop_front();
        }
        LGCHK(hipStreamWaitEvent(c->st, dn, 0));
        (void)hipEventDestroy(dn);
    }
    return 0;
}

}  // namespace

bool xp_on(const gw_ctx* c) { return c->comm || c->lgrp; }

int xp_group_start(gw_ctx* c) {
    if (!xp_on(c)) return set_err(c, GW_ESTATE, "no communicator (gw_comm_init / gw_comm_init_local)");
    if (c->xp_open) return set_err(c, GW_ESTATE, "transport group already open");
    c->xp_open = true;
    c->xp_pend.clear();
    return 0;
}

int xp_send(gw_ctx* c, const void* p, size_t bytes, int peer) {
    if (!c->xp_open || peer < 0 || peer >= c->c_nranks) return set_err(c, GW_EINVAL, "bad send to %d", peer);
    c->xp_pend.push_back(P2P{true, const_cast<void*>(p), bytes, peer});
    return 0;
}

int xp_recv(gw_ctx* c, void* p, size_t bytes, int peer) {
    if (!c->xp_open || peer < 0 || peer >= c->c_nranks) return set_err(c, GW_EINVAL, "bad receive from %d", peer);
    c->xp_pend.push_back(P2P{false, p, bytes, peer});
    return 0;
}

int xp_group_end(gw_ctx* c) {
    if (!c->xp_open) return set_err(c, GW_ESTATE, "no transport group open");
    c->xp_open = false;
    (void)hipSetDevice(c->dev);
    if (c->lgrp) return local_group_end(c);
    std::vector<P2P> pend;
    pend.swap(c->xp_pend);
    NCCLX(ncclGroupStart());
    for (const P2P& x : pend) {
        ncclResult_t r = x.send ? ncclSend(x.p, x.bytes, ncclUint8, x.peer, c->comm, c->st)
                                : ncclRecv(x.p, x.bytes, ncclUint8, x.peer, c->comm, c->st);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            NCCLX(r);
        }
    }
    NCCLX(ncclGroupEnd());
    return 0;
}

void xp_abort(gw_ctx* c) {
    c->xp_open = false;
    c->xp_pend.clear();
}

int xp_allgather(gw_ctx* c, const void* send, void* recv, size_t bytes) {
    if (!xp_on(c)) return set_err(c, GW_ESTATE, "no communicator");
    (void)hipSetDevice(c->dev);
    if (c->comm) {
        NCCLX(ncclAllGather(send, recv, bytes, ncclUint8, c->comm, c->st));
        return 0;
    }
    int rc;
    if ((rc = xp_group_start(c))) return rc;
    for (int p = 0; p < c->c_nranks; ++p) {
        (void)xp_send(c, send, bytes, p);
        (void)xp_recv(c, (char*)recv + (size_t)p * bytes, bytes, p);
    }
    return xp_group_end(c);
}

int xp_allreduce_u64(gw_ctx* c, unsigned long long* dev, uint32_t n, int op) {
    if (!xp_on(c)) return set_err(c, GW_ESTATE, "no communicator");
    if (!n) return 0;
    (void)hipSetDevice(c->dev);
    if (c->comm) {
        NCCLX(ncclAllReduce(dev, dev, n, ncclUint64, op == GW_RED_SUM ? ncclSum : ncclMax, c->comm, c->st));
        return 0;
    }
    // loopback: every rank gathers every rank's words, then reduces them in place
    int rc;
    const size_t bytes = (size_t)n * 8;
    if ((rc = ensure(c, c->xp_tmp, bytes * (c->c_nranks + 1)))) return rc;
    char* tmp = (char*)c->xp_tmp.p;
    // a private copy of the input: the peers read it while this rank overwrites dev
    HIPCHK(hipMemcpyAsync(tmp + bytes * c->c_nranks, dev, bytes, hipMemcpyDeviceToDevice, c->st));
    if ((rc = xp_allgather(c, tmp + bytes * c->c_nranks, tmp, bytes))) return rc;
    launch_reduce_u64((const unsigned long long*)tmp, dev, n, (uint32_t)c->c_nranks, op == GW_RED_MAX, c->st);
    HIPCHK(hipGetLastError());
    return 0;
}

void xp_release(gw_ctx* c) {
    if (c->comm) {
        (void)ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    if (LocalGroup* G = c->lgrp) {
        c->lgrp = nullptr;
        bool last;
        {
            std::lock_guard<std::mutex> lk(G->mu);
            last = --G->refs == 0;
            if (!last) G->broken = true;            // a peer still waiting must not hang on this rank
            if (last) {                            // events of groups a broken peer left unmatched
                for (auto& q : G->posts)
                    for (auto& p : q) (void)hipEventDestroy(p.ready);
                for (auto& q : G->done)
                    for (hipEvent_t e : q) (void)hipEventDestroy(e);
            }
        }
        G->cv.notify_all();
        if (last) delete G;
    }
    if (c->xp_tmp.p) {
        (void)hipFree(c->xp_tmp.p);
        c->xp_tmp = DevBuf{};
    }
}

}  // namespace host
}  // namespace gw

extern "C" {

int gw_comm_init_local(gw_ctx* const* ctxs, int nranks) {
    if (!ctxs || nranks < 1) return GW_EINVAL;
    for (int r = 0; r < nranks; ++r) {
        if (!ctxs[r]) return GW_EINVAL;
        for (int q = 0; q < r; ++q)
            if (ctxs[q] == ctxs[r]) return set_err(ctxs[r], GW_EINVAL, "context listed twice");
        if (xp_on(ctxs[r])) return set_err(ctxs[r], GW_ESTATE, "communicator already initialised");
    }
    for (int r = 0; r < nranks; ++r)
        if (int rs = settle(ctxs[r])) return rs;
    LocalGroup* G = new LocalGroup();
    G->R = nranks;
    G->refs = nranks;
    G->posts.resize((size_t)nranks * nranks);
    G->done.resize((size_t)nranks * nranks);
    if (const char* e = getenv("GW_LOOPBACK_TIMEOUT_S")) G->timeout_s = std::max(1.0, atof(e));
    for (int r = 0; r < nranks; ++r) {
        ctxs[r]->lgrp = G;
        ctxs[r]->c_nranks = nranks;
        ctxs[r]->c_rank = r;
    }
    return 0;
}

}  // extern "C"
