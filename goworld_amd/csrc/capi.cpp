// capi.cpp — C ABI of include/gpuaoi.h on one HIP device.
//
// Host orchestration of the per-tick pipeline (kernels in kernels.hip):
//   ops -> grid (counting sort by cell) -> movers in cell order + leavers ->
//   per-mover bounds and tiers [the one mid-tick host sync: size the event
//   regions, reserve pool space] -> diff (tiers S/B/C) -> per-watcher offsets
//   -> mirror scatter + own copy -> segment sorts -> op-less watchers' merges
//   -> reset.
// No torch, no CPU fallback: every compute step is a HIP kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gw_internal.hpp"

using namespace gw;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct SpaceHost {
    float d;
    uint32_t cap, base;
    SpaceP p;
    bool alive;
};

struct OpSeg {            // submission order of a tick: host or device segment
    bool host;
    const gw_op* dev;
    uint32_t n;
    size_t host_off;
};

struct Stage {
    const char* name;
    hipEvent_t a, b;
    uint64_t bytes;
};

}  // namespace

struct gw_ctx {
    int dev = 0;
    int ab = 1;           // GW_AB: kernel-variant switches for A/B timing (bit0 materialize movers
                          // in a separate pass, bit1 separate small-segment sort); same results
    hipStream_t st = nullptr;
    std::string err;

    std::vector<SpaceHost> spaces;
    uint32_t total_slots = 0, slot_cap = 0, total_cells = 0;
    uint16_t max_gate = 0;

    // persistent device state (slot-indexed)
    AoiEnt* aoi = nullptr;
    float4* pos = nullptr;
    uint32_t* flags = nullptr;
    uint16_t* gate = nullptr;
    LstMeta* lst = nullptr;
    uint8_t* is_mover = nullptr;
    unsigned long long* cnt64 = nullptr;     // [slot_cap + 1], zero between ticks
    uint32_t* log_cnt = nullptr;             // [slot_cap] pending delta-log entries
    uint32_t* logs = nullptr;                // [slot_cap * LOGCAP]
    int32_t *last_pos = nullptr, *last_aoi = nullptr, *last_leave = nullptr;
    SpaceP* sp_dev = nullptr;
    uint32_t sp_cap = 0;
    uint32_t* pool = nullptr;
    uint64_t pool_cap = 0;
    uint64_t h_pool_top = 0, h_total_entries = 0, h_live_caps = 0;

    DevStats* stats = nullptr;     // device
    DevStats* hstats = nullptr;    // pinned host

    // tick scratch
    DevBuf ops_buf, keys, cell_cnt, cell_start, cursor, se, pflag, pre, fpre;
    DevBuf movers, bpk, tpk, reg_pk, tier_pre, list_s, list_b, list_c, c_temp_off, c_temp, own, mir, mir_cnt;
    DevBuf off64, enter_d, leave_d, affected, bigseg, bigseg_off, bigseg_temp;
    DevBuf scan_tmp64, scan_tmp32, rs_hist, rs_scan_tmp;
    // sync scratch
    DevBuf flag_mark, flag_pre, flagged, rec_cnt, rec_off, rec0, rec1, gate_hist, gk0, gv0, gk1, gv1, rec_act, act_off;
    uint32_t* scal32 = nullptr;    // small device scalars

    // host mirror for validation of host-submitted ops
    std::vector<uint8_t> present_h;
    std::vector<int32_t> space_of_h;   // slot -> space id (-1 none)
    bool validate = true;

    // pending ops
    std::vector<gw_op> pend_host;
    std::vector<OpSeg> segs;

    // outputs
    DevBuf h_enter, h_leave, h_rec;   // pinned host
    std::vector<uint64_t> gate_off;

    // profiling
    bool prof = false;
    std::vector<Stage> stages;
    size_t nstage = 0;
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;
    gw_stage_times last_times{};
};

namespace {

int set_err(gw_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIPCHK(expr)                                                                             \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return set_err(c, GW_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                           __FILE__, __LINE__);                                                  \
    } while (0)

// (re)allocate scratch without preserving contents; callers only grow buffers
// at points where the stream is idle (after a host sync)
int ensure(gw_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return 0;
    size_t nb = std::max(bytes, b.cap + b.cap / 2);
    nb = (nb + 255) & ~(size_t)255;
    if (b.p) HIPCHK(hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    if (hipMalloc(&b.p, nb) != hipSuccess) {
        b.p = nullptr;
        (void)hipGetLastError();
        return set_err(c, GW_ENOMEM, "hipMalloc(%zu) failed", nb);
    }
    b.cap = nb;
    return 0;
}

int ensure_host(gw_ctx* c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return 0;
    size_t nb = std::max(bytes, b.cap + b.cap / 2);
    if (b.p) HIPCHK(hipHostFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    if (hipHostMalloc(&b.p, nb, hipHostMallocDefault) != hipSuccess) {
        b.p = nullptr;
        (void)hipGetLastError();
        return set_err(c, GW_ENOMEM, "hipHostMalloc(%zu) failed", nb);
    }
    b.cap = nb;
    return 0;
}

template <typename T>
int grow_preserve(gw_ctx* c, T*& p, size_t old_n, size_t new_n) {
    T* q = nullptr;
    if (hipMalloc(&q, new_n * sizeof(T)) != hipSuccess) {
        (void)hipGetLastError();
        return set_err(c, GW_ENOMEM, "hipMalloc(%zu) failed", new_n * sizeof(T));
    }
    if (p && old_n) HIPCHK(hipMemcpyAsync(q, p, old_n * sizeof(T), hipMemcpyDeviceToDevice, c->st));
    if (p) {
        HIPCHK(hipStreamSynchronize(c->st));
        HIPCHK(hipFree(p));
    }
    p = q;
    return 0;
}

template <typename T>
T* P(DevBuf& b) { return (T*)b.p; }

int ceil_log2(uint64_t v) {   // bits needed to represent values in [0, v)
    int b = 1;
    while (b < 63 && (1ull << b) < v) ++b;
    return b;
}

// ---- profiling ------------------------------------------------------------
void prof_begin(gw_ctx* c, const char* name) {
    if (!c->prof) return;
    if (c->nstage >= c->stages.size()) {
        Stage s{};
        (void)hipEventCreate(&s.a);
        (void)hipEventCreate(&s.b);
        c->stages.push_back(s);
    }
    Stage& s = c->stages[c->nstage];
    s.name = name;
    s.bytes = 0;
    (void)hipEventRecord(s.a, c->st);
}
size_t prof_end(gw_ctx* c, uint64_t bytes) {
    if (!c->prof) return 0;
    Stage& s = c->stages[c->nstage];
    s.bytes = bytes;
    (void)hipEventRecord(s.b, c->st);
    size_t idx = c->nstage;
    if (c->nstage + 1 < GW_MAX_STAGES) c->nstage++;
    return idx;
}
void prof_set_bytes(gw_ctx* c, size_t idx, uint64_t bytes) {
    if (c->prof && idx < c->stages.size()) c->stages[idx].bytes = bytes;
}
void prof_collect(gw_ctx* c) {
    gw_stage_times& t = c->last_times;
    t.n = 0;
    if (!c->prof) return;
    for (size_t i = 0; i < c->nstage && i < GW_MAX_STAGES; ++i) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->stages[i].a, c->stages[i].b);
        t.name[t.n] = c->stages[i].name;
        t.us[t.n] = ms * 1000.0;
        t.bytes_alg[t.n] = c->stages[i].bytes;
        t.n++;
    }
}

int radix_tmp(gw_ctx* c, uint64_t n_max, RadixTmp& rt) {
    uint64_t nb = (n_max + radix_tile() - 1) / radix_tile();
    if (!nb) nb = 1;
    uint64_t hn = 256 * nb;
    int rc;
    if ((rc = ensure(c, c->rs_hist, hn * 4))) return rc;
    if ((rc = ensure(c, c->rs_scan_tmp, ((hn + scan_tile() - 1) / scan_tile() + 2) * 4))) return rc;
    rt.hist = P<uint32_t>(c->rs_hist);
    rt.scan_tmp = P<uint32_t>(c->rs_scan_tmp);
    rt.scan_total = c->scal32;
    return 0;
}

int ensure_scan64(gw_ctx* c, uint64_t n) {
    return ensure(c, c->scan_tmp64, ((n + scan_tile() - 1) / scan_tile() + 2) * 8);
}
int ensure_scan32(gw_ctx* c, uint64_t n) {
    return ensure(c, c->scan_tmp32, ((n + scan_tile() - 1) / scan_tile() + 2) * 4);
}

// grow slot-indexed state to hold new_total slots, initialising the new range
int grow_slots(gw_ctx* c, uint32_t new_total) {
    if (new_total <= c->slot_cap) return 0;
    uint32_t nc = std::max<uint32_t>(new_total, c->slot_cap + c->slot_cap / 2);
    uint32_t oc = c->slot_cap;
    int rc;
    if ((rc = grow_preserve(c, c->aoi, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->pos, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->flags, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->gate, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->lst, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->is_mover, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->cnt64, oc ? oc + 1 : 0, (size_t)nc + 1))) return rc;
    if ((rc = grow_preserve(c, c->last_pos, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->last_aoi, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->last_leave, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->log_cnt, oc, nc))) return rc;
    if ((rc = grow_preserve(c, c->logs, (size_t)oc * LOGCAP, (size_t)nc * LOGCAP))) return rc;
    size_t n = nc - oc;
    HIPCHK(hipMemsetAsync(c->log_cnt + oc, 0, n * 4, c->st));
    HIPCHK(hipMemsetAsync(c->aoi + oc, 0, n * sizeof(AoiEnt), c->st));
    HIPCHK(hipMemsetAsync(c->pos + oc, 0, n * sizeof(float4), c->st));
    HIPCHK(hipMemsetAsync(c->flags + oc, 0, n * 4, c->st));
    HIPCHK(hipMemsetAsync(c->gate + oc, 0, n * 2, c->st));
    HIPCHK(hipMemsetAsync(c->lst + oc, 0, n * sizeof(LstMeta), c->st));
    HIPCHK(hipMemsetAsync(c->is_mover + oc, 0, n, c->st));
    HIPCHK(hipMemsetAsync(c->cnt64 + oc, 0, (n + 1) * 8, c->st));
    launch_fill_i32(c->last_pos + oc, -1, n, c->st);
    launch_fill_i32(c->last_aoi + oc, -1, n, c->st);
    launch_fill_i32(c->last_leave + oc, -1, n, c->st);
    HIPCHK(hipStreamSynchronize(c->st));
    c->slot_cap = nc;
    c->present_h.resize(nc, 0);
    c->space_of_h.resize(nc, -1);
    return 0;
}

// write seq=-1 and space id for a new space's slots (AoiEnt.meta)
int init_space_slots(gw_ctx* c, uint32_t base, uint32_t cap, uint32_t sid) {
    std::vector<AoiEnt> h(cap);
    for (uint32_t i = 0; i < cap; ++i) { h[i].x = 0; h[i].z = 0; h[i].seq = -1; h[i].meta = sid; }
    HIPCHK(hipMemcpyAsync(c->aoi + base, h.data(), cap * sizeof(AoiEnt), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int upload_spaces(gw_ctx* c) {
    uint32_t n = (uint32_t)c->spaces.size();
    if (n > c->sp_cap) {
        uint32_t nc = std::max<uint32_t>(n, c->sp_cap * 2 + 16);
        if (c->sp_dev) HIPCHK(hipFree(c->sp_dev));
        c->sp_dev = nullptr;
        if (hipMalloc(&c->sp_dev, nc * sizeof(SpaceP)) != hipSuccess) return set_err(c, GW_ENOMEM, "hipMalloc spaces");
        c->sp_cap = nc;
    }
    std::vector<SpaceP> h(n);
    for (uint32_t i = 0; i < n; ++i) h[i] = c->spaces[i].p;
    HIPCHK(hipMemcpyAsync(c->sp_dev, h.data(), n * sizeof(SpaceP), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int read_stats(gw_ctx* c) {
    HIPCHK(hipMemcpyAsync(c->hstats, c->stats, offsetof(DevStats, shard), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// Guarantee `reserve` free entries past the pool top; when the pool cannot
// hold them, compact every slot's current list (capacities kept) into a new
// pool sized for the live capacities plus twice the reserve.
int pool_reserve(gw_ctx* c, uint64_t reserve) {
    if (c->pool && c->h_pool_top + reserve <= c->pool_cap) return 0;
    int rc;
    uint64_t live = 0;
    if (c->pool && c->total_slots) {
        // (sized by total_slots: gw_tick already holds buffers at least this big)
        if ((rc = ensure(c, c->pflag, (size_t)c->total_slots * 4))) return rc;
        if ((rc = ensure(c, c->pre, (size_t)c->total_slots * 8))) return rc;
        if ((rc = ensure_scan64(c, (uint64_t)c->total_slots + 1))) return rc;
        launch_cap2(c->lst, c->total_slots, P<uint32_t>(c->pflag), c->st);
        scan_u32_u64(P<uint32_t>(c->pflag), P<uint64_t>(c->pre), c->total_slots, nullptr, P<uint64_t>(c->scan_tmp64),
                     (uint64_t*)&c->stats->scratch, c->st);
        HIPCHK(hipMemcpyAsync(&live, &c->stats->scratch, 8, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
    }
    uint64_t ncap = (2 * (live + reserve) + (1u << 20) + 15) & ~15ull;
    if (ncap >= (1ull << 36)) return set_err(c, GW_ENOMEM, "neighbour pool exceeds 2^36 entries");
    uint32_t* np = nullptr;
    if (hipMalloc(&np, ncap * 4) != hipSuccess) {
        (void)hipGetLastError();
        return set_err(c, GW_ENOMEM, "pool hipMalloc(%llu entries) failed", (unsigned long long)ncap);
    }
    if (c->pool && c->total_slots) {
        launch_pool_compact(c->lst, P<uint64_t>(c->pre), c->total_slots, c->pool, np, c->lst, c->st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(c->st));
    }
    if (c->pool) HIPCHK(hipFree(c->pool));
    c->pool = np;
    c->pool_cap = ncap;
    c->h_pool_top = live;
    c->h_live_caps = live;
    return 0;
}

int validate_ops(gw_ctx* c, const gw_op* ops, uint32_t n) {
    // all-or-nothing: replay against the host presence mirror, undo on error
    std::vector<std::pair<uint32_t, uint8_t>> undo;
    int rc = 0;
    for (uint32_t i = 0; i < n && !rc; ++i) {
        const gw_op& o = ops[i];
        if (o.slot >= c->total_slots || c->space_of_h[o.slot] < 0 ||
            !c->spaces[(size_t)c->space_of_h[o.slot]].alive) {
            rc = set_err(c, GW_ERANGE, "op %u: slot %u not in a live space", i, o.slot);
            break;
        }
        bool pres = c->present_h[o.slot] != 0;
        switch (o.kind) {
        case GW_OP_ENTER:
            if (pres) rc = set_err(c, GW_ESTATE, "op %u: Enter of slot %u already in the space", i, o.slot);
            break;
        case GW_OP_MOVED:
        case GW_OP_LEAVE:
        case GW_OP_SYNC:
            if (!pres) rc = set_err(c, GW_ESTATE, "op %u: kind %u on slot %u not in the space", i, o.kind, o.slot);
            break;
        default:
            rc = set_err(c, GW_EINVAL, "op %u: bad kind %u", i, o.kind);
        }
        if (rc) break;
        if ((o.kind == GW_OP_ENTER || o.kind == GW_OP_MOVED) && !(std::isfinite(o.x) && std::isfinite(o.z)))
            rc = set_err(c, GW_EINVAL, "op %u: non-finite coordinates", i);
        if (rc) break;
        if (o.kind == GW_OP_ENTER || o.kind == GW_OP_LEAVE) {
            undo.push_back({o.slot, c->present_h[o.slot]});
            c->present_h[o.slot] = o.kind == GW_OP_ENTER;
        }
    }
    if (rc)
        for (auto it = undo.rbegin(); it != undo.rend(); ++it) c->present_h[it->first] = it->second;
    return rc;
}

void reset_stats_host(gw_ctx* c) {
    memset(c->hstats, 0, sizeof(DevStats));
    c->hstats->pool_top = c->h_pool_top;
}

}  // namespace

// =========================================================================
extern "C" {

int gw_abi_version(void) { return GW_ABI_VERSION; }

const char* gw_last_error(const gw_ctx* c) { return c ? c->err.c_str() : "null context"; }

int gw_init(int device_id, gw_ctx** out) {
    if (!out) return GW_EINVAL;
    *out = nullptr;
    gw_ctx* c = new gw_ctx();
    c->dev = device_id;
    if (const char* e = getenv("GW_AB")) c->ab = atoi(e);
    int rc = 0;
    do {
        if (hipSetDevice(device_id) != hipSuccess) { rc = set_err(c, GW_EDEVICE, "hipSetDevice(%d) failed", device_id); break; }
        if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) { rc = set_err(c, GW_EDEVICE, "stream"); break; }
        if (hipMalloc(&c->stats, sizeof(DevStats)) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "stats"); break; }
        if (hipHostMalloc((void**)&c->hstats, sizeof(DevStats), hipHostMallocDefault) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "hstats"); break; }
        if (hipMalloc(&c->scal32, 64) != hipSuccess) { rc = set_err(c, GW_ENOMEM, "scal"); break; }
        memset(c->hstats, 0, sizeof(DevStats));
        (void)hipMemset(c->stats, 0, sizeof(DevStats));
        (void)hipEventCreate(&c->ev_t0);
        (void)hipEventCreate(&c->ev_t1);
    } while (0);
    if (rc) {
        (void)hipGetLastError();
        gw_shutdown(c);
        return rc;
    }
    *out = c;
    return 0;
}

void gw_shutdown(gw_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->dev);
    if (c->st) (void)hipStreamSynchronize(c->st);
    DevBuf* bufs[] = {&c->ops_buf, &c->keys, &c->cell_cnt, &c->cell_start, &c->cursor, &c->se, &c->pflag, &c->pre,
                      &c->fpre, &c->movers, &c->bpk, &c->tpk, &c->reg_pk, &c->tier_pre, &c->list_s, &c->list_b,
                      &c->list_c, &c->c_temp_off, &c->c_temp, &c->own, &c->mir, &c->mir_cnt, &c->off64,
                      &c->enter_d, &c->leave_d, &c->affected, &c->bigseg, &c->bigseg_off, &c->bigseg_temp,
                      &c->scan_tmp64, &c->scan_tmp32, &c->rs_hist, &c->rs_scan_tmp, &c->flag_mark, &c->flag_pre,
                      &c->flagged, &c->rec_cnt, &c->rec_off, &c->rec0, &c->rec1, &c->gate_hist, &c->gk0, &c->gv0,
                      &c->gk1, &c->gv1, &c->rec_act, &c->act_off};
    for (DevBuf* b : bufs) if (b->p) (void)hipFree(b->p);
    DevBuf* hb[] = {&c->h_enter, &c->h_leave, &c->h_rec};
    for (DevBuf* b : hb) if (b->p) (void)hipHostFree(b->p);
    void* ps[] = {c->aoi, c->pos, c->flags, c->gate, c->lst, c->is_mover, c->cnt64, c->last_pos, c->last_aoi,
                  c->last_leave, c->log_cnt, c->logs, c->sp_dev, c->pool, c->stats, c->scal32};
    for (void* p : ps) if (p) (void)hipFree(p);
    if (c->hstats) (void)hipHostFree(c->hstats);
    for (auto& s : c->stages) { (void)hipEventDestroy(s.a); (void)hipEventDestroy(s.b); }
    if (c->ev_t0) (void)hipEventDestroy(c->ev_t0);
    if (c->ev_t1) (void)hipEventDestroy(c->ev_t1);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

int gw_space_create(gw_ctx* c, float aoi_dist, uint32_t capacity, const float* bounds, uint32_t* space_id,
                    uint32_t* slot_base) {
    if (!c) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    if (!(aoi_dist > 0) || !std::isfinite(aoi_dist))
        return set_err(c, GW_EINVAL, "defaultAOIDistance <= 0");          // Space.go:92-94
    if (capacity == 0) return set_err(c, GW_EINVAL, "capacity must be > 0");
    if ((uint64_t)c->total_slots + capacity >= (1ull << 31)) return set_err(c, GW_ERANGE, "too many slots");
    float b[4] = {-1000.f, -1000.f, 1000.f, 1000.f};                       // Space.GetSpaceRange, Space.go:52-54
    if (bounds) for (int i = 0; i < 4; ++i) b[i] = bounds[i];
    if (!(b[2] > b[0]) || !(b[3] > b[1]) || !std::isfinite(b[0]) || !std::isfinite(b[1]) || !std::isfinite(b[2]) ||
        !std::isfinite(b[3]))
        return set_err(c, GW_EINVAL, "bad bounds");
    // square cells of side >= d; at most 8192 cells per axis
    double ex = (double)b[2] - b[0], ez = (double)b[3] - b[1];
    double cs = std::max((double)aoi_dist, std::max(ex, ez) / 8192.0);
    SpaceHost s{};
    s.d = aoi_dist;
    s.cap = capacity;
    s.base = c->total_slots;
    s.alive = true;
    s.p.d = aoi_dist;
    s.p.x0 = b[0];
    s.p.z0 = b[1];
    s.p.inv_cs = (float)(1.0 / cs);
    s.p.W = std::max(1, (int)std::ceil(ex / cs));
    s.p.H = std::max(1, (int)std::ceil(ez / cs));
    s.p.cell_base = c->total_cells;
    s.p.alive = 1;
    uint64_t ncells = (uint64_t)s.p.W * (uint64_t)s.p.H;
    if ((uint64_t)c->total_cells + ncells + 1 >= (1ull << 31)) return set_err(c, GW_ERANGE, "too many grid cells");
    int rc;
    if ((rc = grow_slots(c, c->total_slots + capacity))) return rc;
    uint32_t sid = (uint32_t)c->spaces.size();
    if ((rc = init_space_slots(c, s.base, capacity, sid))) return rc;
    c->spaces.push_back(s);
    c->total_slots += capacity;
    c->total_cells += (uint32_t)ncells;
    for (uint32_t i = 0; i < capacity; ++i) c->space_of_h[s.base + i] = (int32_t)sid;
    if ((rc = upload_spaces(c))) return rc;
    if (space_id) *space_id = sid;
    if (slot_base) *slot_base = s.base;
    return 0;
}

int gw_space_destroy(gw_ctx* c, uint32_t sid) {
    if (!c) return GW_EINVAL;
    if (sid >= c->spaces.size() || !c->spaces[sid].alive) return set_err(c, GW_ERANGE, "no space %u", sid);
    SpaceHost& s = c->spaces[sid];
    if (c->validate) {
        for (uint32_t i = 0; i < s.cap; ++i)
            if (c->present_h[s.base + i]) return set_err(c, GW_ESTATE, "space %u not empty", sid);
    }
    s.alive = false;
    s.p.alive = 0;
    return upload_spaces(c);
}

int gw_submit(gw_ctx* c, const gw_op* ops, uint32_t n) {
    if (!c || (!ops && n)) return GW_EINVAL;
    if (!n) return 0;
    if (c->validate) {
        int rc = validate_ops(c, ops, n);
        if (rc) return rc;
    }
    OpSeg sg{true, nullptr, n, c->pend_host.size()};
    c->pend_host.insert(c->pend_host.end(), ops, ops + n);
    c->segs.push_back(sg);
    return 0;
}

int gw_submit_device(gw_ctx* c, const gw_op* dev_ops, uint32_t n) {
    if (!c || (!dev_ops && n)) return GW_EINVAL;
    if (!n) return 0;
    c->validate = false;   // device-resident ops are trusted; the host mirror is no longer exact
    c->segs.push_back(OpSeg{false, dev_ops, n, 0});
    return 0;
}

int gw_set_clients(gw_ctx* c, const uint32_t* slots, const uint16_t* gates, uint32_t n) {
    if (!c || (n && (!slots || !gates))) return GW_EINVAL;
    if (!n) return 0;
    (void)hipSetDevice(c->dev);
    for (uint32_t i = 0; i < n; ++i) {
        if (slots[i] >= c->total_slots) return set_err(c, GW_ERANGE, "slot %u out of range", slots[i]);
        c->max_gate = std::max(c->max_gate, gates[i]);
    }
    int rc;
    if ((rc = ensure(c, c->gk0, (size_t)n * 4))) return rc;
    if ((rc = ensure(c, c->gv0, (size_t)n * 2))) return rc;
    HIPCHK(hipMemcpyAsync(c->gk0.p, slots, (size_t)n * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(c->gv0.p, gates, (size_t)n * 2, hipMemcpyHostToDevice, c->st));
    launch_set_clients(P<uint32_t>(c->gk0), (const uint16_t*)c->gv0.p, n, c->total_slots, c->gate, c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int gw_tick(gw_ctx* c, uint32_t flags, gw_tick_out* out) {
    if (!c || !out) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    memset(out, 0, sizeof *out);
    c->nstage = 0;
    uint64_t M64 = 0;
    for (auto& s : c->segs) M64 += s.n;
    if (M64 >= (1ull << 31)) return set_err(c, GW_ERANGE, "too many ops in one tick");
    const uint32_t M = (uint32_t)M64;
    const uint32_t C = c->total_slots;
    int rc;
    HIPCHK(hipEventRecord(c->ev_t0, c->st));
    if (M == 0 || C == 0) {
        c->segs.clear();
        c->pend_host.clear();
        return 0;
    }
    // ---- the tick's op stream, in submission order -----------------------
    const gw_op* ops = nullptr;
    if (c->segs.size() == 1 && !c->segs[0].host) {
        ops = c->segs[0].dev;
    } else {
        if ((rc = ensure(c, c->ops_buf, (size_t)M * sizeof(gw_op)))) return rc;
        size_t off = 0;
        for (auto& s : c->segs) {
            if (s.host)
                HIPCHK(hipMemcpyAsync(P<gw_op>(c->ops_buf) + off, c->pend_host.data() + s.host_off,
                                      (size_t)s.n * sizeof(gw_op), hipMemcpyHostToDevice, c->st));
            else
                HIPCHK(hipMemcpyAsync(P<gw_op>(c->ops_buf) + off, s.dev, (size_t)s.n * sizeof(gw_op),
                                      hipMemcpyDeviceToDevice, c->st));
            off += s.n;
        }
        ops = P<gw_op>(c->ops_buf);
    }
    const uint32_t NC = c->total_cells;
    const uint64_t CM = std::max<uint64_t>(C, M);
    // ---- buffers whose size is known before the tick ----------------------
    if ((rc = ensure(c, c->keys, (size_t)C * 4)) || (rc = ensure(c, c->cell_cnt, ((size_t)NC + 1) * 4)) ||
        (rc = ensure(c, c->cell_start, ((size_t)NC + 2) * 4)) || (rc = ensure(c, c->cursor, ((size_t)NC + 1) * 4)) ||
        (rc = ensure(c, c->se, (size_t)C * sizeof(SortEnt))) || (rc = ensure(c, c->pflag, CM * 4)) ||
        (rc = ensure(c, c->pre, CM * 8)) || (rc = ensure(c, c->fpre, (size_t)C * 8)) ||
        (rc = ensure(c, c->movers, (size_t)M * 4)) || (rc = ensure(c, c->bpk, (size_t)M * 8)) ||
        (rc = ensure(c, c->tpk, (size_t)M * 8)) || (rc = ensure(c, c->reg_pk, (size_t)M * 8)) ||
        (rc = ensure(c, c->tier_pre, (size_t)M * 8)) || (rc = ensure(c, c->list_s, (size_t)M * 4)) ||
        (rc = ensure(c, c->list_b, (size_t)M * 4)) || (rc = ensure(c, c->list_c, (size_t)M * 4)) ||
        (rc = ensure(c, c->c_temp_off, (size_t)M * 8)) || (rc = ensure(c, c->mir_cnt, (size_t)M * 4)) ||
        (rc = ensure(c, c->off64, ((size_t)C + 2) * 8)) || (rc = ensure(c, c->affected, (size_t)C * 4)) ||
        (rc = ensure(c, c->bigseg, (size_t)C * 4)) || (rc = ensure(c, c->bigseg_off, (size_t)C * 8)) ||
        (rc = ensure_scan64(c, CM + 1)) || (rc = ensure_scan32(c, (uint64_t)NC + 1)))
        return rc;
    if (!c->pool && (rc = pool_reserve(c, 1u << 20))) return rc;
    reset_stats_host(c);
    HIPCHK(hipMemcpyAsync(c->stats, c->hstats, sizeof(DevStats), hipMemcpyHostToDevice, c->st));
    DevStats* st = c->stats;

    TickBufs b{};
    b.ops = ops; b.m = M; b.cap = C; b.ncells = NC;
    b.last_pos = c->last_pos; b.last_aoi = c->last_aoi; b.last_leave = c->last_leave;
    b.flags = c->flags; b.pos = c->pos; b.aoi = c->aoi; b.is_mover = c->is_mover; b.lst = c->lst; b.sp = c->sp_dev;
    b.log_cnt = c->log_cnt; b.logs = c->logs;
    b.pool = c->pool; b.pool_cap = c->pool_cap; b.st = st;
    b.keys = P<uint32_t>(c->keys); b.cell_cnt = P<uint32_t>(c->cell_cnt); b.cell_start = P<uint32_t>(c->cell_start);
    b.cursor = P<uint32_t>(c->cursor); b.se = P<SortEnt>(c->se); b.pflag = P<uint32_t>(c->pflag);
    b.pre = P<uint64_t>(c->pre); b.fpre = P<uint64_t>(c->fpre);
    b.movers = P<uint32_t>(c->movers); b.bpk = P<uint64_t>(c->bpk); b.tpk = P<uint64_t>(c->tpk);
    b.reg_pk = P<uint64_t>(c->reg_pk); b.tier_pre = P<uint64_t>(c->tier_pre); b.list_s = P<uint32_t>(c->list_s);
    b.list_b = P<uint32_t>(c->list_b); b.list_c = P<uint32_t>(c->list_c); b.c_temp_off = P<uint64_t>(c->c_temp_off);
    b.mir_cnt = P<uint32_t>(c->mir_cnt); b.cnt64 = c->cnt64; b.off64 = P<uint64_t>(c->off64);
    b.affected = P<uint32_t>(c->affected); b.bigseg = P<uint32_t>(c->bigseg); b.bigseg_off = P<uint64_t>(c->bigseg_off);
    b.write_events = (flags & GW_TICK_NO_EVENTS) ? 0 : 1;

    uint64_t* stmp = P<uint64_t>(c->scan_tmp64);
    prof_begin(c, "ops");
    tick_ops(b, c->st);
    prof_end(c, (uint64_t)M * 24);
    prof_begin(c, "grid");
    tick_grid(b, stmp, P<uint32_t>(c->scan_tmp32), c->st);
    size_t s_grid = prof_end(c, 0);
    prof_begin(c, "movers");
    tick_movers(b, stmp, c->st);
    tick_bounds(b, stmp, c->st);
    size_t s_movers = prof_end(c, 0);
    HIPCHK(hipGetLastError());
    // ---- the one mid-tick host sync ---------------------------------------
    if ((rc = read_stats(c))) return rc;
    DevStats hs0 = *c->hstats;
    if (hs0.bad_ops) return set_err(c, GW_EINVAL, "%llu ops with bad slot/kind", hs0.bad_ops);
    const uint64_t n_mov = hs0.movers_present + hs0.leavers;
    const uint64_t sum_cand = hs0.bound_pk & 0xffffffffull, sum_old = hs0.bound_pk >> 32;
    const uint64_t n_s = hs0.tier_pk & 0xffffffffull, n_b = hs0.tier_pk >> 32, n_c = hs0.n_tier_c;
    const uint64_t region = std::max<uint64_t>(sum_cand + sum_old, 1);
    if (sum_cand >= (1ull << 32) - 1 || sum_old >= (1ull << 32) - 1)
        return set_err(c, GW_ERANGE, "tick too large: %llu candidates", (unsigned long long)sum_cand);
    if ((rc = ensure(c, c->own, region * 4)) || (rc = ensure(c, c->mir, region * 8)) ||
        (rc = ensure(c, c->enter_d, std::max<uint64_t>(2 * sum_cand, 1) * sizeof(gw_event))) ||
        (rc = ensure(c, c->leave_d, std::max<uint64_t>(2 * sum_old, 1) * sizeof(gw_event))) ||
        (rc = ensure(c, c->c_temp, std::max<uint64_t>(hs0.tier_c_temp, 4) * 4)) ||
        (rc = ensure(c, c->bigseg_temp, std::max<uint64_t>(4 * (sum_cand + sum_old) + 64, 64) * 4)))
        return rc;
    // worst-case reallocation of one tick (every list that outgrows its
    // capacity moves to a region of 2 * 2.5 * size): movers' materialization
    // (<= old + log), movers' new lists (<= cand), op-less watchers' bursts
    // (<= old + enters) and log materializations (<= old + LOGCAP each)
    const uint64_t n_aff_bound = std::min<uint64_t>(C, sum_cand + sum_old);
    const uint64_t reserve = 5 * (3 * sum_cand + sum_old + 2 * c->h_total_entries) +
                             (5 * LOGCAP + 64) * n_aff_bound + 64 * ((uint64_t)C + n_mov) + (1u << 16);
    uint64_t top_before = c->h_pool_top;
    if ((rc = pool_reserve(c, reserve))) return rc;
    if (c->h_pool_top != top_before) {   // compaction moved the lists
        c->hstats->pool_top = c->h_pool_top;
        HIPCHK(hipMemcpyAsync(&st->pool_top, &c->hstats->pool_top, 8, hipMemcpyHostToDevice, c->st));
    }
    b.pool = c->pool; b.pool_cap = c->pool_cap;
    b.own = P<uint32_t>(c->own); b.mir = P<uint64_t>(c->mir);
    b.enter = P<gw_event>(c->enter_d); b.leave = P<gw_event>(c->leave_d);
    b.enter_cap = std::max<uint64_t>(2 * sum_cand, 1); b.leave_cap = std::max<uint64_t>(2 * sum_old, 1);
    b.c_temp = P<uint32_t>(c->c_temp); b.c_temp_cap = std::max<uint64_t>(hs0.tier_c_temp, 4);
    b.bigseg_temp = P<uint32_t>(c->bigseg_temp); b.bigseg_temp_cap = c->bigseg_temp.cap / 4;

    // ---- movers' delta logs, then the diff -----------------------------------
    prof_begin(c, "materialize");
    if (c->ab & 1) tick_materialize_movers(b, hs0.movers_present, true, c->st);
    else tick_materialize_movers(b, n_c, false, c->st);
    prof_end(c, 0);
    prof_begin(c, "diff");
    tick_diff(b, n_s, n_b, n_c, c->st);
    size_t s_diff = prof_end(c, 0);
    prof_begin(c, "events");
    tick_events(b, n_mov, stmp, c->st);
    const uint64_t aff_max = std::min<uint64_t>(C, sum_cand + sum_old);
    tick_nonmovers(b, aff_max, aff_max, n_mov, c->st, !(c->ab & 2));
    size_t s_events = prof_end(c, 0);
    prof_begin(c, "reset");
    tick_reset(b, n_mov, c->st);
    stats_reduce(st, c->st);
    prof_end(c, (uint64_t)M * 40);
    HIPCHK(hipEventRecord(c->ev_t1, c->st));
    HIPCHK(hipGetLastError());
    if ((rc = read_stats(c))) return rc;
    DevStats& hs = *c->hstats;
    c->segs.clear();
    c->pend_host.clear();
    if (hs.pool_overflow) return set_err(c, GW_EDEVICE, "internal: neighbour pool overflow");
    if (hs.tmp_overflow) return set_err(c, GW_EDEVICE, "internal: segment scratch overflow");
    const uint64_t n_enter = hs.ev_pk & 0xffffffffull, n_leave = hs.ev_pk >> 32;
    c->h_pool_top = hs.pool_top;
    c->h_total_entries = c->h_total_entries + n_enter - n_leave;   // every list changes by its enters - leaves
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev_t0, c->ev_t1);
    out->device_us = ms * 1000.0;
    out->ops = M;
    out->movers = n_mov;
    out->pairs_tested = hs.pairs_tested;
    out->nbr_old = hs.a_old;
    out->nbr_new = hs.a_new;
    out->enter_dev = (flags & GW_TICK_NO_EVENTS) ? nullptr : P<gw_event>(c->enter_d);
    out->leave_dev = (flags & GW_TICK_NO_EVENTS) ? nullptr : P<gw_event>(c->leave_d);
    out->n_enter = n_enter;
    out->n_leave = n_leave;
    // SURVEY 8(d) algorithmic bytes of the AOI part (records are counted by gw_sync_collect)
    const uint64_t n_evt = n_enter + n_leave;
    out->bytes_alg = 20ull * n_mov + 8ull * hs.n_present + 4ull * (hs.a_old + hs.a_new) + 8ull * n_evt;
    if (c->prof) {
        prof_set_bytes(c, s_grid, 16ull * C + 16ull * hs.n_present + 8ull * NC);
        prof_set_bytes(c, s_movers, 8ull * hs.n_present + 40ull * n_mov);
        // diff: candidates (16 B) + old lists read twice (4 B) + neighbour state gathered (16 B per old
        // entry) + new lists (4 B) + own and mirror events (12 B per directed event)
        prof_set_bytes(c, s_diff, 16ull * hs.pairs_tested + 24ull * hs.a_old + 4ull * hs.a_new + 12ull * n_evt);
        prof_set_bytes(c, s_events, 16ull * (C + 1) + 24ull * n_evt);
        prof_collect(c);
    }
    if ((flags & GW_TICK_COPY_TO_HOST) && !(flags & GW_TICK_NO_EVENTS)) {
        if ((rc = ensure_host(c, c->h_enter, std::max<uint64_t>(n_enter, 1) * sizeof(gw_event)))) return rc;
        if ((rc = ensure_host(c, c->h_leave, std::max<uint64_t>(n_leave, 1) * sizeof(gw_event)))) return rc;
        if (n_enter) HIPCHK(hipMemcpyAsync(c->h_enter.p, c->enter_d.p, n_enter * sizeof(gw_event), hipMemcpyDeviceToHost, c->st));
        if (n_leave) HIPCHK(hipMemcpyAsync(c->h_leave.p, c->leave_d.p, n_leave * sizeof(gw_event), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        out->enter = (const gw_event*)c->h_enter.p;
        out->leave = (const gw_event*)c->h_leave.p;
    }
    return 0;
}

int gw_sync_collect(gw_ctx* c, uint32_t flags, gw_sync_out* out) {
    if (!c || !out) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    memset(out, 0, sizeof *out);
    c->nstage = 0;
    const uint32_t C = c->total_slots;
    int rc;
    HIPCHK(hipEventRecord(c->ev_t0, c->st));
    const uint32_t G = (uint32_t)c->max_gate + 1;
    c->gate_off.assign((size_t)G + 1, 0);
    if (C == 0 || !c->pool) {
        out->gate_off = c->gate_off.data();
        out->n_gates = G;
        return 0;
    }
    // flagged entities with pending logs are materialized before reading lists
    if ((rc = pool_reserve(c, 5 * c->h_total_entries + (5 * LOGCAP + 64) * (uint64_t)C + (1u << 16)))) return rc;
    reset_stats_host(c);
    HIPCHK(hipMemcpyAsync(c->stats, c->hstats, sizeof(DevStats), hipMemcpyHostToDevice, c->st));
    DevStats* st = c->stats;
    const uint64_t rec_bound = (uint64_t)C + c->h_total_entries;
    if ((rc = ensure(c, c->flag_mark, (size_t)C * 4)) || (rc = ensure(c, c->flag_pre, (size_t)C * 8)) ||
        (rc = ensure(c, c->flagged, (size_t)C * 4)) || (rc = ensure(c, c->rec_cnt, (size_t)C * 4)) ||
        (rc = ensure(c, c->rec_off, (size_t)C * 8)) || (rc = ensure(c, c->rec_act, (size_t)C * 4)) ||
        (rc = ensure(c, c->act_off, (size_t)C * 8)) ||
        (rc = ensure(c, c->rec0, (size_t)std::max<uint64_t>(rec_bound, 1) * sizeof(gw_sync_record))) ||
        (rc = ensure_scan64(c, C)))
        return rc;
    prof_begin(c, "sync_flagged");
    launch_flag_mark(c->flags, C, P<uint32_t>(c->flag_mark), c->st);
    scan_u32_u64(P<uint32_t>(c->flag_mark), P<uint64_t>(c->flag_pre), C, nullptr, P<uint64_t>(c->scan_tmp64),
                 (uint64_t*)&st->flagged, c->st);
    launch_flag_compact(P<uint32_t>(c->flag_mark), P<uint64_t>(c->flag_pre), C, P<uint32_t>(c->flagged), c->st);
    prof_end(c, (uint64_t)C * 4 * 4);
    const uint64_t* nf = (const uint64_t*)&st->flagged;
    prof_begin(c, "sync_materialize");
    launch_materialize_slots(c->lst, c->pool, c->pool_cap, st, c->log_cnt, c->logs, P<uint32_t>(c->flagged), nf, C,
                             c->st);
    prof_end(c, 0);
    prof_begin(c, "sync_count");
    launch_sync_count(P<uint32_t>(c->flagged), nf, C, c->flags, c->aoi, c->gate, c->lst, c->pool,
                      P<uint32_t>(c->rec_cnt), c->st);
    scan_u32_u64(P<uint32_t>(c->rec_cnt), P<uint64_t>(c->rec_off), C, nf, P<uint64_t>(c->scan_tmp64),
                 (uint64_t*)&st->rec_total, c->st);
    size_t s_count = prof_end(c, 0);
    prof_begin(c, "sync_write");
    launch_sync_write(P<uint32_t>(c->flagged), nf, C, c->flags, c->aoi, c->gate, c->lst, c->pool, c->pos,
                      P<uint64_t>(c->rec_off), P<gw_sync_record>(c->rec0), c->rec0.cap / sizeof(gw_sync_record),
                      P<uint32_t>(c->rec_act), st, c->st);
    size_t s_write = prof_end(c, 0);
    HIPCHK(hipGetLastError());
    if ((rc = read_stats(c))) return rc;
    uint64_t R = c->hstats->rec_total;         // the bound; exact unless gaps were flagged
    const uint64_t NF = c->hstats->flagged;
    if (R > rec_bound) return set_err(c, GW_EDEVICE, "internal: record bound exceeded");
    if (c->hstats->pool_overflow) return set_err(c, GW_ENOMEM, "internal: neighbour pool overflow");
    c->h_pool_top = c->hstats->pool_top;
    gw_sync_record* recs = P<gw_sync_record>(c->rec0);
    if (c->hstats->scratch & 1) {            // some neighbours have no client: compact
        prof_begin(c, "sync_compact");
        if ((rc = ensure(c, c->rec1, std::max<uint64_t>(R, 1) * sizeof(gw_sync_record)))) return rc;
        scan_u32_u64(P<uint32_t>(c->rec_act), P<uint64_t>(c->act_off), C, nf, P<uint64_t>(c->scan_tmp64),
                     (uint64_t*)&st->rec_total, c->st);
        launch_sync_compact(nf, C, P<uint64_t>(c->rec_off), P<uint32_t>(c->rec_act), P<uint64_t>(c->act_off), recs,
                            P<gw_sync_record>(c->rec1), c->st);
        prof_end(c, 48 * R);
        if ((rc = read_stats(c))) return rc;
        R = c->hstats->rec_total;
        std::swap(c->rec0, c->rec1);
        recs = P<gw_sync_record>(c->rec0);
    }
    // ---- per-gate grouping (stable, keeps (entity, watcher) order) -------
    if (R && G > 2) {
        prof_begin(c, "sync_gates");
        if ((rc = ensure(c, c->gate_hist, (size_t)65536 * 4))) return rc;
        HIPCHK(hipMemsetAsync(c->gate_hist.p, 0, (size_t)G * 4, c->st));
        launch_gate_hist(recs, nullptr, R, c->gate, P<uint32_t>(c->gate_hist), c->st);
        std::vector<uint32_t> h(G);
        HIPCHK(hipMemcpyAsync(h.data(), c->gate_hist.p, (size_t)G * 4, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        uint32_t nonzero = 0;
        for (uint32_t g = 0; g < G; ++g) nonzero += h[g] != 0;
        uint64_t acc = 0;
        for (uint32_t g = 0; g < G; ++g) { c->gate_off[g] = acc; acc += h[g]; }
        c->gate_off[G] = acc;
        if (nonzero > 1) {
            if ((rc = ensure(c, c->gk0, R * 4)) || (rc = ensure(c, c->gv0, R * 4)) || (rc = ensure(c, c->gk1, R * 4)) ||
                (rc = ensure(c, c->gv1, R * 4)) || (rc = ensure(c, c->rec1, R * sizeof(gw_sync_record))))
                return rc;
            RadixTmp rt;
            if ((rc = radix_tmp(c, R, rt))) return rc;
            launch_gate_keys(recs, nullptr, R, c->gate, P<uint32_t>(c->gk0), P<uint32_t>(c->gv0), c->st);
            int gw = sort_u32_u32(P<uint32_t>(c->gk0), P<uint32_t>(c->gv0), P<uint32_t>(c->gk1), P<uint32_t>(c->gv1), R,
                                  nullptr, 0, ceil_log2(G), rt, c->st);
            launch_gather_records(recs, gw ? P<uint32_t>(c->gv1) : P<uint32_t>(c->gv0), nullptr, R,
                                  P<gw_sync_record>(c->rec1), c->st);
            std::swap(c->rec0, c->rec1);
            recs = P<gw_sync_record>(c->rec0);
        }
        prof_end(c, R * (24 * 2 + 8 * 4));
    } else {
        // at most one gate id in use: every record belongs to the last gate
        for (uint32_t g = 0; g <= G; ++g) c->gate_off[g] = (g == G) ? R : 0;
    }
    HIPCHK(hipEventRecord(c->ev_t1, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev_t0, c->ev_t1);
    out->device_us = ms * 1000.0;
    out->n_rec = R;
    out->flagged = NF;
    out->rec_dev = recs;
    out->gate_off = c->gate_off.data();
    out->n_gates = G;
    out->bytes_alg = 24ull * R;
    if (c->prof) {
        prof_set_bytes(c, s_count, NF * 32);
        prof_set_bytes(c, s_write, 4ull * R + 24ull * R + NF * 24);
        prof_collect(c);
    }
    if (flags & GW_SYNC_COPY_TO_HOST) {
        if ((rc = ensure_host(c, c->h_rec, std::max<uint64_t>(R, 1) * sizeof(gw_sync_record)))) return rc;
        if (R) HIPCHK(hipMemcpyAsync(c->h_rec.p, recs, R * sizeof(gw_sync_record), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        out->rec = (const gw_sync_record*)c->h_rec.p;
    }
    return 0;
}

int gw_neighbors(gw_ctx* c, uint32_t slot, uint32_t* buf, uint32_t cap, uint32_t* n) {
    if (!c || !n) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    if (slot >= c->total_slots) return set_err(c, GW_ERANGE, "slot %u out of range", slot);
    LstMeta L{};
    uint32_t lc = 0;
    HIPCHK(hipMemcpyAsync(&L, c->lst + slot, sizeof L, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemcpyAsync(&lc, c->log_cnt + slot, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    std::vector<uint32_t> base(L.cnt), lg(lc);
    if (L.cnt)
        HIPCHK(hipMemcpyAsync(base.data(), c->pool + ((uint64_t)L.cur << 4), (size_t)L.cnt * 4,
                              hipMemcpyDeviceToHost, c->st));
    if (lc) HIPCHK(hipMemcpyAsync(lg.data(), c->logs + (uint64_t)slot * LOGCAP, (size_t)lc * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (lc) {   // net effect of the delta log: majority kind per target
        std::sort(lg.begin(), lg.end());
        std::vector<uint32_t> add, rem;
        for (size_t i = 0; i < lg.size();) {
            size_t j = i;
            int ne = 0, nl = 0;
            while (j < lg.size() && (lg[j] >> 1) == (lg[i] >> 1)) { if (lg[j] & 1) ++nl; else ++ne; ++j; }
            if (ne > nl) add.push_back(lg[i] >> 1);
            if (nl > ne) rem.push_back(lg[i] >> 1);
            i = j;
        }
        std::vector<uint32_t> out;
        out.reserve(base.size() + add.size());
        size_t ia = 0;
        for (uint32_t v : base) {
            while (ia < add.size() && add[ia] < v) out.push_back(add[ia++]);
            if (!std::binary_search(rem.begin(), rem.end(), v)) out.push_back(v);
        }
        while (ia < add.size()) out.push_back(add[ia++]);
        base.swap(out);
    }
    *n = (uint32_t)base.size();
    uint32_t k = std::min<uint32_t>((uint32_t)base.size(), cap);
    if (buf && k) memcpy(buf, base.data(), (size_t)k * 4);
    return 0;
}

int gw_total_neighbors(gw_ctx* c, uint64_t* out) {
    if (!c || !out) return GW_EINVAL;
    *out = c->h_total_entries;
    return 0;
}

int gw_set_profiling(gw_ctx* c, int enable) {
    if (!c) return GW_EINVAL;
    c->prof = enable != 0;
    return 0;
}

int gw_get_stage_times(gw_ctx* c, gw_stage_times* out) {
    if (!c || !out) return GW_EINVAL;
    *out = c->last_times;
    return 0;
}

int gw_device_alloc(gw_ctx* c, size_t bytes, void** p) {
    if (!c || !p) return GW_EINVAL;
    (void)hipSetDevice(c->dev);
    if (hipMalloc(p, bytes ? bytes : 16) != hipSuccess) {
        (void)hipGetLastError();
        return set_err(c, GW_ENOMEM, "hipMalloc(%zu)", bytes);
    }
    return 0;
}
int gw_device_free(gw_ctx* c, void* p) {
    if (!c) return GW_EINVAL;
    if (p) HIPCHK(hipFree(p));
    return 0;
}
int gw_memcpy_h2d(gw_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return GW_EINVAL;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}
int gw_memcpy_d2h(gw_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return GW_EINVAL;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}
int gw_synchronize(gw_ctx* c) {
    if (!c) return GW_EINVAL;
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

}  // extern "C"
